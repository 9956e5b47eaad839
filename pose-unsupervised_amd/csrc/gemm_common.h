// MFMA operand traits and LDS-DMA helpers shared by the implicit-GEMM convolution
// (conv_igemm.hip) and the fused Bottleneck (bottleneck.hip) kernels.  gfx950 only.
#pragma once
#include "posu_common.h"

namespace posu {
namespace {

template <typename T>
struct Op;

template <>
struct Op<uint16_t> {  // bf16
  static constexpr int E = 8;
  static constexpr bool SPLIT = false;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void load_vals(const uint4& u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint4 store_vals(const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = f2bf2(v[2 * i], v[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

template <>
struct Op<f16_t> {  // IEEE fp16
  static constexpr int E = 8;
  static constexpr bool SPLIT = false;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc,
                                                 0, 0, 0);
  }
  static __device__ __forceinline__ void load_vals(const uint4& u, float* v) {
    const f16x8 h = __builtin_bit_cast(f16x8, u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = static_cast<float>(h[i]);
  }
  static __device__ __forceinline__ uint4 store_vals(const float* v) {
    f16x8 h;
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = static_cast<_Float16>(v[i]);
    return __builtin_bit_cast(uint4, h);
  }
};

// split fp16 (POSU_F16X3): the operands are fp16 halves of (hi, lo) pairs; a K-tile of 64 halves
// holds 32 logical k as [hi 32 | lo 32], i.e. its two MFMA k-steps are the hi and the lo halves of
// the same k, and the kernels issue hi.hi + lo(w).hi(x) + hi(w).lo(x) per K-tile (SPLIT).
template <>
struct Op<f16s_t> {
  static constexpr int E = 8;
  static constexpr bool SPLIT = true;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    Op<f16_t>::mma(acc, a, b);
  }
  static __device__ __forceinline__ void load_vals(const uint4& u, float* v) { Op<f16_t>::load_vals(u, v); }
  static __device__ __forceinline__ uint4 store_vals(const float* v) { return Op<f16_t>::store_vals(v); }
};

template <>
struct Op<float> {
  static constexpr int E = 4;
  static constexpr bool SPLIT = false;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void load_vals(const uint4& u, float* v) {
    v[0] = __uint_as_float(u.x);
    v[1] = __uint_as_float(u.y);
    v[2] = __uint_as_float(u.z);
    v[3] = __uint_as_float(u.w);
  }
  static __device__ __forceinline__ uint4 store_vals(const float* v) {
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                      __float_as_uint(v[3]));
  }
};

// v = v * s + b and v += r over 8 values.  PK: as four packed f32 FMAs / adds (v_pk_fma_f32, two
// fused multiply-adds per instruction, the same rounding as v_fma_f32); else one scalar
// instruction per value.  Measured in round 4 (profiles/r04/pk_epilogue_ab_r4l.txt): packed
// helps the layer1 identity Bottleneck (150.7 vs 154.3 us) and costs elsewhere (the network
// 2.518 vs 2.499 ms with every epilogue packed: the even-aligned register pairs they need add
// moves and pressure), so only that kernel uses it.
template <bool PK>
__device__ __forceinline__ void affine8(float* v, const float* s, const float* b) {
  if constexpr (!PK) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] * s[e] + b[e];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x2v x = {v[2 * i], v[2 * i + 1]};
      const f32x2v ss = {s[2 * i], s[2 * i + 1]}, bb = {b[2 * i], b[2 * i + 1]};
      x = __builtin_elementwise_fma(x, ss, bb);
      v[2 * i] = x.x;
      v[2 * i + 1] = x.y;
    }
  }
}
template <bool PK>
__device__ __forceinline__ void add8(float* v, const float* r) {
  if constexpr (!PK) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += r[e];
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x2v x = {v[2 * i], v[2 * i + 1]};
      const f32x2v rr = {r[2 * i], r[2 * i + 1]};
      x = x + rr;
      v[2 * i] = x.x;
      v[2 * i + 1] = x.y;
    }
  }
}

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

constexpr int kOOB = 0x7ffffff0;  // buffer offset past num_records: the load returns zeros
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Buffer resource descriptor (base, num_records = bytes, raw dword format) built from
// wave-uniform values, kept in SGPRs.
__device__ __forceinline__ u32x4 make_srd(const void* base, int bytes) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  u32x4 r;
  r.x = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(p));
  r.y = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(p >> 32));
  r.z = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(bytes));
  r.w = 0x00020000u;
  return r;
}

// One 16-B-per-lane LDS-DMA: buffer_load_dwordx4 ... lds writes lane l's 16 bytes to
// LDS address lds + 16*l (wave-uniform `lds` in M0); offsets past num_records load 0.
// Issued from inline asm so hipcc neither waits for it before unrelated ds_reads of
// the other ring slots nor drains it early: the kernel retires it itself with a
// counted s_waitcnt vmcnt(N) before the barrier that precedes the reads.
__device__ __forceinline__ void dma16(u32x4 srd, int voff, unsigned lds) {
  // the operands are wave-uniform; readfirstlane lets the compiler prove it (a no-op on
  // values already in SGPRs)
  srd.x = __builtin_amdgcn_readfirstlane(srd.x);
  srd.y = __builtin_amdgcn_readfirstlane(srd.y);
  srd.z = __builtin_amdgcn_readfirstlane(srd.z);
  srd.w = __builtin_amdgcn_readfirstlane(srd.w);
  lds = __builtin_amdgcn_readfirstlane(lds);
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(lds)
      : "memory");
}

// workgroup barrier that also publishes this wave's LDS writes and retires its LDS reads
// (lgkmcnt(0) first); LDS-DMA and global loads stay in flight across it -- unlike
// __syncthreads(), whose fence waits for them too
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// wait until at most N of this wave's vector-memory ops are outstanding
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// s_waitcnt vmcnt(n) for a runtime (wave-uniform) n in 0..63
__device__ __forceinline__ void vm_wait_dyn(int n) {
  switch (n) {
    case 0: vm_wait<0>(); break;
    case 1: vm_wait<1>(); break;
    case 2: vm_wait<2>(); break;
    case 3: vm_wait<3>(); break;
    case 4: vm_wait<4>(); break;
    case 5: vm_wait<5>(); break;
    case 6: vm_wait<6>(); break;
    case 7: vm_wait<7>(); break;
    case 8: vm_wait<8>(); break;
    case 9: vm_wait<9>(); break;
    case 10: vm_wait<10>(); break;
    case 11: vm_wait<11>(); break;
    case 12: vm_wait<12>(); break;
    case 13: vm_wait<13>(); break;
    case 14: vm_wait<14>(); break;
    case 15: vm_wait<15>(); break;
    case 16: vm_wait<16>(); break;
    case 17: vm_wait<17>(); break;
    case 18: vm_wait<18>(); break;
    case 19: vm_wait<19>(); break;
    case 20: vm_wait<20>(); break;
    case 21: vm_wait<21>(); break;
    case 22: vm_wait<22>(); break;
    case 23: vm_wait<23>(); break;
    case 24: vm_wait<24>(); break;
    case 25: vm_wait<25>(); break;
    case 26: vm_wait<26>(); break;
    case 27: vm_wait<27>(); break;
    case 28: vm_wait<28>(); break;
    case 29: vm_wait<29>(); break;
    case 30: vm_wait<30>(); break;
    case 31: vm_wait<31>(); break;
    case 32: vm_wait<32>(); break;
    case 33: vm_wait<33>(); break;
    case 34: vm_wait<34>(); break;
    case 35: vm_wait<35>(); break;
    case 36: vm_wait<36>(); break;
    case 37: vm_wait<37>(); break;
    case 38: vm_wait<38>(); break;
    case 39: vm_wait<39>(); break;
    case 40: vm_wait<40>(); break;
    case 41: vm_wait<41>(); break;
    case 42: vm_wait<42>(); break;
    case 43: vm_wait<43>(); break;
    case 44: vm_wait<44>(); break;
    case 45: vm_wait<45>(); break;
    case 46: vm_wait<46>(); break;
    case 47: vm_wait<47>(); break;
    case 48: vm_wait<48>(); break;
    case 49: vm_wait<49>(); break;
    case 50: vm_wait<50>(); break;
    case 51: vm_wait<51>(); break;
    case 52: vm_wait<52>(); break;
    case 53: vm_wait<53>(); break;
    case 54: vm_wait<54>(); break;
    case 55: vm_wait<55>(); break;
    case 56: vm_wait<56>(); break;
    case 57: vm_wait<57>(); break;
    case 58: vm_wait<58>(); break;
    case 59: vm_wait<59>(); break;
    case 60: vm_wait<60>(); break;
    case 61: vm_wait<61>(); break;
    case 62: vm_wait<62>(); break;
    case 63: vm_wait<63>(); break;
    default: vm_wait<0>(); break;
  }
}

// ---- weight warm-up (round 5; conv_igemm.hip explains the measurement).  In the network a launch's
// weights come from HBM, and every workgroup walks its weights in the same order, so all of them
// miss on the same lines at once, step after step.  Workgroups 0 .. nwarm-1 instead each load one
// dword of distinct 64-B segments of the whole tensor at their start (kWarmLoads per lane), so
// every line is requested once, together, up front; warm_use() consumes the values (an empty asm)
// after the launch's first operand loads are issued.  Loads only: nothing is stored, no result
// depends on it.
#ifndef POSU_WARM
#define POSU_WARM 1
#endif
#ifndef POSU_WARM_MIN_KB
#define POSU_WARM_MIN_KB 64
#endif
constexpr long long kWarmMinBytes = POSU_WARM_MIN_KB * 1024LL;   // smaller weight tensors are not warmed
constexpr int kWarmWG = 512;                   // workgroups that take part (about one round of a grid)
constexpr int kWarmLoads = 4;                  // segments per lane at most

// the warm-up's workgroup count for a weight tensor of `bytes` (0: none)
inline int warm_wgs(long long bytes) { return POSU_WARM && bytes >= kWarmMinBytes ? kWarmWG : 0; }

__device__ __forceinline__ void warm_issue(unsigned (&v)[kWarmLoads], const void* w, long long nseg, int nwarm,
                                           int threads) {
#pragma unroll
  for (int k = 0; k < kWarmLoads; ++k) v[k] = 0;
  const int bid = blockIdx.x;
  nwarm = min(nwarm, static_cast<int>(gridDim.x));
  if (bid < nwarm) {
    const unsigned* __restrict__ w32 = reinterpret_cast<const unsigned*>(w);
    const long long s0 = static_cast<long long>(bid) * threads + threadIdx.x;
    const long long st = static_cast<long long>(nwarm) * threads;
#pragma unroll
    for (int k = 0; k < kWarmLoads; ++k)
      if (s0 + k * st < nseg) v[k] = w32[16 * (s0 + k * st)];
  }
}

__device__ __forceinline__ void warm_use(const unsigned (&v)[kWarmLoads]) {
  unsigned a = 0;
#pragma unroll
  for (int k = 0; k < kWarmLoads; ++k) a ^= v[k];
  asm volatile("" ::"v"(a));
}

}  // namespace
}  // namespace posu
