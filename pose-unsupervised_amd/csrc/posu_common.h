// Internal helpers shared by the libposeu.so translation units (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
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

// Split-fp16 storage type (POSU_F16X3): each value a (hi, lo) pair of fp16, [hi 32 | lo 32] per
// 32-channel block (include/posu.h).  Its own type so the conv kernel's traits select the
// three-MFMA products and the pair epilogue.
struct f16s_t {
  uint16_t bits;
};

// physical element offset of logical channel c's hi half in a split pixel (lo: + 32)
__host__ __device__ __forceinline__ int split_ch(int c) { return ((c >> 5) << 6) + (c & 31); }

// v -> (hi, lo): hi = fp16(v), lo = fp16(v - hi) (v - hi is exact in f32)
__device__ __forceinline__ void split8(const float* v, uint4& hi, uint4& lo) {
  f16x8 h, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = static_cast<_Float16>(v[i]);
    l[i] = static_cast<_Float16>(v[i] - static_cast<float>(h[i]));
  }
  hi = __builtin_bit_cast(uint4, h);
  lo = __builtin_bit_cast(uint4, l);
}
// (hi, lo) -> hi + lo in f32 (exact: the pair spans at most 22 significant bits)
__device__ __forceinline__ void join8(const uint4& hi, const uint4& lo, float* v) {
  const f16x8 h = __builtin_bit_cast(f16x8, hi), l = __builtin_bit_cast(f16x8, lo);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(h[i]) + static_cast<float>(l[i]);
}

__device__ __forceinline__ float bf2f(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
// round-to-nearest-even via the hardware conversion (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 h = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, h);
}

// two f32 -> packed bf16x2 (round to nearest even, as f2bf): ONE v_cvt_pk_bf16_f32, where
// two f2bf calls cost two conversions and an OR
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f2bf2(float lo, float hi) {
  const f32x2v v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
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

// 16-byte streaming (non-temporal) store: activations written once and read by the
// next layer from beyond L2 anyway, so their lines should not evict operands from L2
__device__ __forceinline__ void st16_nt(void* p, const uint4& v) {
  typedef unsigned int u4 __attribute__((ext_vector_type(4)));
  const u4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<u4*>(p));
}

// log2 of a power of two, -1 otherwise
inline int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return ((1 << l) == v) ? l : -1;
}

// 16-byte chunk of a storage type <-> E floats (E = 16 / sizeof(T))
template <typename T>
struct Vec;
template <>
struct Vec<uint16_t> {
  static constexpr int E = 8;
  static __device__ __forceinline__ void unpack(const uint4& u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint4 pack(const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = f2bf2(v[2 * i], v[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <>
struct Vec<f16_t> {
  static constexpr int E = 8;
  static __device__ __forceinline__ void unpack(const uint4& u, float* v) {
    const f16x8 h = __builtin_bit_cast(f16x8, u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(h[i]);
  }
  static __device__ __forceinline__ uint4 pack(const float* v) {
    f16x8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = static_cast<_Float16>(v[i]);
    return __builtin_bit_cast(uint4, h);
  }
};
template <>
struct Vec<float> {
  static constexpr int E = 4;
  static __device__ __forceinline__ void unpack(const uint4& u, float* v) {
    v[0] = __uint_as_float(u.x);
    v[1] = __uint_as_float(u.y);
    v[2] = __uint_as_float(u.z);
    v[3] = __uint_as_float(u.w);
  }
  static __device__ __forceinline__ uint4 pack(const float* v) {
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                      __float_as_uint(v[3]));
  }
};

// storage-type dispatch: fn(T{}) for the dtype code, false if unsupported
template <typename Fn>
bool with_storage(int dtype, Fn&& fn) {
  switch (dtype) {
    case POSU_BF16: fn(uint16_t{}); return true;
    case POSU_F16: fn(f16_t{}); return true;
    case POSU_F32: fn(float{}); return true;
    default: return false;
  }
}

}  // namespace posu
