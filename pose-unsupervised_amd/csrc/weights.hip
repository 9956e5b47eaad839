// Batched weight packing for the training step: every conv / deconv / head weight of the
// network, from its fp32 PyTorch layout into the layouts the MFMA kernels read, in ONE launch
// per step (lib/posu/packing.py restates each mode in torch: pack_conv_weight,
// pack_conv_dgrad_weight, pack_deconv4x4_weight).  Replaces ~110 per-layer packs of 3-6 torch
// ops each (zero fill, permute/flip copies, dtype casts) that the training plan ran per step
// (reference: the parameters the optimizer updates in place, pose_resnet.py:234-247 init,
// train.py Adam).
//
// The job table (posu_pack_job[], device memory) is built once per parameter set; each job owns
// a contiguous range of blocks, a block finds its job by binary search over block_start.
// HBM-bound: 4 B read + 2 B written per packed element.  Every block stages its source
// region in LDS with coalesced reads (a conv row is contiguous; the dgrad / deconv modes
// transpose (co, ci) tiles) and writes whole 16-B groups of 8 consecutive packed elements.
#include "posu_common.h"
#include "../../include/posu.h"

namespace posu {
namespace {

constexpr int kThreads = 256, kPerThread = 8;
constexpr int kLdsFloats = 8448;  // 33 KB of source staging per block

template <typename T>
__device__ __forceinline__ T cvt(float v);
template <>
__device__ __forceinline__ uint16_t cvt<uint16_t>(float v) { return f2bf(v); }
template <>
__device__ __forceinline__ f16_t cvt<f16_t>(float v) {
  return f16_t{__builtin_bit_cast(uint16_t, static_cast<_Float16>(v))};
}
template <>
__device__ __forceinline__ float cvt<float>(float v) { return v; }

// 8 consecutive packed elements -> one 16-B (two for f32) store
template <typename T>
__device__ __forceinline__ void store8(T* dst, const float* v) {
  if constexpr (sizeof(T) == 4) {
    reinterpret_cast<float4*>(dst)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(dst)[1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint16_t lo = __builtin_bit_cast(uint16_t, cvt<T>(v[2 * i]));
      const uint16_t hi = __builtin_bit_cast(uint16_t, cvt<T>(v[2 * i + 1]));
      w[i] = static_cast<uint32_t>(lo) | (static_cast<uint32_t>(hi) << 16);
    }
    *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// ---- block decomposition per mode (host and device agree through these helpers)
// CONV: R whole destination rows per block, their source rows staged contiguously in LDS.
// DGRAD: a tile of kDgCi destination rows (ci) x 64 output channels (co), all taps.
// DECONV: a tile of kDcCo destination rows (co) x 64 input channels (ci), all 16 taps.
// GENERIC (a CONV row larger than the staging buffer): per-element gathers.
constexpr int kTileC = 64, kDcCo = 8;
__host__ __device__ inline int conv_rows_per_block(int cin, int ntap) {
  const int per = cin * ntap;
  int r = kLdsFloats / (per + 1);
  return r < 1 ? 0 : (r > 16 ? 16 : r);
}
__host__ __device__ inline int dgrad_ci_per_block(int ntap) {
  int c = kLdsFloats / (kTileC * ntap + kTileC);
  return c < 1 ? 0 : (c > 8 ? 8 : c);
}
__host__ __device__ inline long long ceil_div(long long a, long long b) { return (a + b - 1) / b; }

// element-wise gathers (any shape): the fallback for jobs the tiled paths do not cover
__host__ __device__ inline bool tiled(int mode, int cin, int ntap, int pitch) {
  if (mode == POSU_PACK_CONV) return conv_rows_per_block(cin, ntap) > 0;
  if (mode == POSU_PACK_DGRAD) return dgrad_ci_per_block(ntap) > 0 && pitch % 8 == 0;
  return (ntap == 16 || ntap == 9) && cin % 8 == 0;
}

template <typename T>
__device__ void pack_generic(const posu_pack_job& j, long long b) {
  const long long per_cls = static_cast<long long>(j.rows) * j.kpad;
  const long long n = per_cls * (j.mode == POSU_PACK_DECONV ? 4 : 1);
  const long long e0 = (b * kThreads) * kPerThread + threadIdx.x;
  T* __restrict__ dst = reinterpret_cast<T*>(j.dst);
  const float* __restrict__ src = j.src;
  const int ntap = j.kh * j.kw;
  for (int i = 0; i < kPerThread; ++i) {
    const long long e = e0 + static_cast<long long>(i) * kThreads;
    if (e >= n) break;
    float v = 0.f;
    if (j.mode == POSU_PACK_CONV) {
      const int row = static_cast<int>(e / j.kpad), k = static_cast<int>(e - static_cast<long long>(row) * j.kpad);
      const int tap = k / j.pitch, ci = k - tap * j.pitch;
      if (row < j.cout && tap < ntap && ci < j.cin) v = src[(static_cast<long long>(row) * j.cin + ci) * ntap + tap];
    } else if (j.mode == POSU_PACK_DGRAD) {
      const int row = static_cast<int>(e / j.kpad), k = static_cast<int>(e - static_cast<long long>(row) * j.kpad);
      const int tap = k / j.pitch, co = k - tap * j.pitch;
      if (row < j.cin && tap < ntap && co < j.cout)
        v = src[(static_cast<long long>(co) * j.cin + row) * ntap + (ntap - 1 - tap)];
    } else {
      const int c = static_cast<int>(e / per_cls);
      const long long r = e - c * per_cls;
      const int row = static_cast<int>(r / j.kpad), k = static_cast<int>(r - static_cast<long long>(row) * j.kpad);
      const int t = k / j.cin, ci = k - t * j.cin;
      if (row < j.cout && t < 4) {
        const int py = c >> 1, px = c & 1, ty = t >> 1, tx = t & 1;
        const int kh = 3 - py - 2 * ty, kw = 3 - px - 2 * tx;  // kh / kw = 3 of a 3x3 source: a zero tap
        if (kh < j.kh && kw < j.kw)
          v = src[((static_cast<long long>(ci) * j.cout + row) * j.kh + kh) * j.kw + kw];
      }
    }
    dst[e] = cvt<T>(v);
  }
}

// LDS staging: lds[dst(i)] = src[srcoff(i)] for i < n, 8 loads in flight per thread
template <typename SrcOff, typename DstOff>
__device__ __forceinline__ void stage(float* lds, const float* __restrict__ src, int n, SrcOff so, DstOff dof) {
  for (int base = threadIdx.x; base < n; base += kThreads * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * kThreads;
      v[u] = i < n ? src[so(i)] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = base + u * kThreads;
      if (i < n) lds[dof(i)] = v[u];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void pack_weights_kernel(const posu_pack_job* __restrict__ jobs, int njobs) {
  __shared__ float lds[kLdsFloats];
  int lo = 0, hi = njobs - 1;  // last job with block_start <= blockIdx.x
  const long long bid = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].block_start <= bid) lo = mid;
    else hi = mid - 1;
  }
  const posu_pack_job j = jobs[lo];
  const long long b = bid - j.block_start;
  const int tid = threadIdx.x;
  const int ntap = j.kh * j.kw;
  const float* __restrict__ src = j.src;
  T* __restrict__ dst = reinterpret_cast<T*>(j.dst);
  const int kq = j.kpad / 8;  // 8-element store groups per destination row

  if (!tiled(j.mode, j.cin, ntap, j.pitch)) {
    pack_generic<T>(j, b);
    return;
  }
  if (j.mode == POSU_PACK_CONV) {
    // out[row = co][k = tap * pitch + ci] = w[co][ci][tap]: rows r0 .. r0+R-1
    const int R = conv_rows_per_block(j.cin, ntap);
    const int per = j.cin * ntap;
    const int r0 = static_cast<int>(b) * R;
    const int rs = max(0, min(R, j.cout - r0));  // rows that have a source
    const float* __restrict__ s0 = src + static_cast<long long>(r0) * per;
    stage(lds, s0, rs * per, [](int i) { return static_cast<long long>(i); }, [](int i) { return i; });
    __syncthreads();
    const int rr = min(R, j.rows - r0);
    for (int g = tid; g < rr * kq; g += kThreads) {
      const int r = g / kq, k0 = (g - r * kq) * 8;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e, tap = k / j.pitch, ci = k - tap * j.pitch;
        v[e] = (r < rs && tap < ntap && ci < j.cin) ? lds[r * per + ci * ntap + tap] : 0.f;
      }
      store8(dst + static_cast<long long>(r0 + r) * j.kpad + k0, v);
    }
  } else if (j.mode == POSU_PACK_DGRAD) {
    // out[row = ci][k = tap * pitch + co] = w[co][ci][ntap-1-tap]: ci c0 .. c0+CI-1, co o0 .. o0+63
    const int CI = dgrad_ci_per_block(ntap);
    const int cot = static_cast<int>(ceil_div(j.pitch, kTileC));
    const int c0 = static_cast<int>(b / cot) * CI, o0 = static_cast<int>(b % cot) * kTileC;
    const int str = CI * ntap + 1;  // LDS row (one co) stride, padded against bank conflicts
    const int cin_n = max(0, min(CI, j.cin - c0)), co_n = max(0, min(kTileC, j.cout - o0));
    const int run = cin_n * ntap;   // contiguous source floats per co
    if (run > 0) {
      const float* __restrict__ s0 = src + (static_cast<long long>(o0) * j.cin + c0) * ntap;
      const long long cs = static_cast<long long>(j.cin) * ntap;  // source stride between co
      stage(lds, s0, co_n * run, [=](int i) { return (i / run) * cs + i % run; },
            [=](int i) { return (i / run) * str + i % run; });
    }
    __syncthreads();
    const int rr = min(CI, j.rows - c0);
    // groups of 8 co: (ci, tap, co group)
    for (int g = tid; g < rr * ntap * (kTileC / 8); g += kThreads) {
      const int og = g % (kTileC / 8), t = (g / (kTileC / 8)) % ntap, c = g / ((kTileC / 8) * ntap);
      const int co = o0 + 8 * og;
      if (co >= j.pitch) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int o = 8 * og + e;
        v[e] = (c < cin_n && o < co_n && co + e < j.pitch) ? lds[o * str + c * ntap + (ntap - 1 - t)] : 0.f;
      }
      store8(dst + static_cast<long long>(c0 + c) * j.kpad + t * j.pitch + co, v);
    }
    if (o0 == 0) {  // the rows' K tail past ntap * pitch
      const int k1 = ntap * j.pitch;
      const int tail = (j.kpad - k1) / 8;
      const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int g = tid; g < rr * tail; g += kThreads) {
        const int c = g / tail, k0 = k1 + (g - c * tail) * 8;
        store8(dst + static_cast<long long>(c0 + c) * j.kpad + k0, z);
      }
    }
  } else {
    // deconv class c = py*2+px: out[c][row = co][k = (ty*2+tx) * cin + ci] = w[ci][co][3-py-2ty][3-px-2tx];
    // a 3x3 source (round 5: the data gradient of a 3x3 / s2 / p1 conv is this transposed conv with the
    // kernel zero-padded to 4x4) reads its taps kh, kw < 3 and zeros at index 3
    const int KK = ntap;  // 16 or 9 source taps per (ci, co)
    const int cit = static_cast<int>(ceil_div(j.cin, kTileC));
    const int o0 = static_cast<int>(b / cit) * kDcCo, i0 = static_cast<int>(b % cit) * kTileC;
    const int str = kDcCo * KK + 1;
    const int ci_n = max(0, min(kTileC, j.cin - i0)), co_n = max(0, min(kDcCo, j.cout - o0));
    const int run = co_n * KK;
    if (run > 0) {
      const float* __restrict__ s0 = src + (static_cast<long long>(i0) * j.cout + o0) * KK;
      const long long cs = static_cast<long long>(j.cout) * KK;  // source stride between ci
      stage(lds, s0, ci_n * run, [=](int i) { return (i / run) * cs + i % run; },
            [=](int i) { return (i / run) * str + i % run; });
    }
    __syncthreads();
    const long long per_cls = static_cast<long long>(j.rows) * j.kpad;
    const int rr = min(kDcCo, j.rows - o0);
    // groups of 8 ci: (class, co, t, ci group)
    for (int g = tid; g < 4 * rr * 4 * (kTileC / 8); g += kThreads) {
      const int ig = g % (kTileC / 8), t = (g / (kTileC / 8)) % 4, o = (g / (4 * (kTileC / 8))) % rr,
                cls = g / (4 * (kTileC / 8) * rr);
      const int ci = i0 + 8 * ig;
      if (ci >= j.cin) continue;
      const int py = cls >> 1, px = cls & 1, ty = t >> 1, tx = t & 1;
      const int kh = 3 - py - 2 * ty, kw = 3 - px - 2 * tx;
      const bool tv = kh < j.kh && kw < j.kw;
      const int tap = tv ? kh * j.kw + kw : 0;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = 8 * ig + e;
        v[e] = (tv && o < co_n && c < ci_n) ? lds[c * str + o * KK + tap] : 0.f;
      }
      store8(dst + cls * per_cls + static_cast<long long>(o0 + o) * j.kpad + t * j.cin + ci, v);
    }
    if (i0 == 0) {  // K tail past 4 * cin, every class
      const int k1 = 4 * j.cin, tail = (j.kpad - k1) / 8;
      const float z[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int g = tid; g < 4 * rr * tail; g += kThreads) {
        const int cls = g / (rr * tail), rem = g - cls * rr * tail, o = rem / tail, k0 = k1 + (rem - o * tail) * 8;
        store8(dst + cls * per_cls + static_cast<long long>(o0 + o) * j.kpad + k0, z);
      }
    }
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" long long posu_pack_job_blocks(int mode, int cout, int cin, int kh, int kw, int pitch, int rows,
                                         int kpad) {
  if (rows <= 0 || kpad <= 0 || kpad % 8 || cout <= 0 || cin <= 0 || kh <= 0 || kw <= 0 || pitch <= 0) return -1;
  if (mode != POSU_PACK_CONV && mode != POSU_PACK_DGRAD && mode != POSU_PACK_DECONV) return -1;
  if (mode == POSU_PACK_DECONV && !(kh == kw && (kh == 4 || kh == 3))) return -1;
  const int ntap = kh * kw;
  if (!tiled(mode, cin, ntap, pitch))
    return ceil_div(static_cast<long long>(rows) * kpad * (mode == POSU_PACK_DECONV ? 4 : 1),
                    static_cast<long long>(kThreads) * kPerThread);
  if (mode == POSU_PACK_CONV) return ceil_div(rows, conv_rows_per_block(cin, ntap));
  if (mode == POSU_PACK_DGRAD) return ceil_div(rows, dgrad_ci_per_block(ntap)) * ceil_div(pitch, kTileC);
  return ceil_div(rows, kDcCo) * ceil_div(cin, kTileC);
}

extern "C" int posu_pack_weights(int dtype, const posu_pack_job* jobs, int njobs, long long total_blocks,
                                 void* stream) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16 || dtype == POSU_F32,
               "posu_pack_weights: dtype must be F32, BF16 or F16");
  POSU_REQUIRE(jobs && njobs > 0, "posu_pack_weights: empty job table");
  POSU_REQUIRE(total_blocks > 0 && total_blocks < (1LL << 31), "posu_pack_weights: block count out of range");
  hipStream_t s = as_stream(stream);
  const dim3 grid(static_cast<unsigned>(total_blocks)), block(kThreads);
  if (dtype == POSU_BF16) hipLaunchKernelGGL(pack_weights_kernel<uint16_t>, grid, block, 0, s, jobs, njobs);
  else if (dtype == POSU_F16) hipLaunchKernelGGL(pack_weights_kernel<f16_t>, grid, block, 0, s, jobs, njobs);
  else hipLaunchKernelGGL(pack_weights_kernel<float>, grid, block, 0, s, jobs, njobs);
  return check_launch("posu_pack_weights");
}
