// Error reporting + ABI version of libposeu.so.
#include "posu_common.h"

namespace posu {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return POSU_ERR_HIP;
  }
  return POSU_OK;
}

}  // namespace posu

extern "C" const char* posu_last_error(void) { return posu::g_last_error.c_str(); }

extern "C" int posu_abi_version(void) { return 16; }
