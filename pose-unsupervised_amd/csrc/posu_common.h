// Internal helpers shared by the libposeu.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/posu.h"

namespace posu {

// thread-local error message behind posu_last_error()
void set_error(const std::string& msg);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Records a launch failure (if any) and converts it to a status code.
int check_launch(const char* what);

#define POSU_REQUIRE(cond, msg)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::posu::set_error(std::string(msg));      \
      return POSU_ERR_ARG;                      \
    }                                           \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// IEEE binary16 storage type (POSU_F16); distinct from the bf16 storage type uint16_t
// so the kernels' per-dtype traits can tell them apart.
struct f16_t {
  uint16_t bits;
};

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
// round-to-nearest-even via the hardware conversion (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, h);
}

// wave64 reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

}  // namespace posu
