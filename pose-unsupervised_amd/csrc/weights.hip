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
// HBM-bound: 4 B read + 2 B written per packed element (the source reads of the flipped /
// transposed modes are gathers, served from L2: every layer's weight is <= 8 MB).
#include "posu_common.h"
#include "../../include/posu.h"

namespace posu {
namespace {

constexpr int kThreads = 256, kPerThread = 8;

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

template <typename T>
__global__ __launch_bounds__(kThreads) void pack_weights_kernel(const posu_pack_job* __restrict__ jobs, int njobs) {
  int lo = 0, hi = njobs - 1;  // last job with block_start <= blockIdx.x
  const long long b = blockIdx.x;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].block_start <= b) lo = mid;
    else hi = mid - 1;
  }
  const posu_pack_job j = jobs[lo];
  const long long per_cls = static_cast<long long>(j.rows) * j.kpad;
  const long long n = per_cls * (j.mode == POSU_PACK_DECONV ? 4 : 1);
  const long long e0 = ((b - j.block_start) * kThreads) * kPerThread + threadIdx.x;
  T* __restrict__ dst = reinterpret_cast<T*>(j.dst);
  const float* __restrict__ src = j.src;
  const int ntap = j.kh * j.kw;
#pragma unroll
  for (int i = 0; i < kPerThread; ++i) {
    const long long e = e0 + static_cast<long long>(i) * kThreads;
    if (e >= n) break;
    float v = 0.f;
    if (j.mode == POSU_PACK_CONV) {
      // out[row = co][k = tap * pitch + ci] = w[co][ci][kh][kw]
      const int row = static_cast<int>(e / j.kpad), k = static_cast<int>(e - static_cast<long long>(row) * j.kpad);
      const int tap = k / j.pitch, ci = k - tap * j.pitch;
      if (row < j.cout && tap < ntap && ci < j.cin) v = src[(static_cast<long long>(row) * j.cin + ci) * ntap + tap];
    } else if (j.mode == POSU_PACK_DGRAD) {
      // out[row = ci][k = tap * pitch + co] = w[co][ci][KH-1-th][KW-1-tw]
      const int row = static_cast<int>(e / j.kpad), k = static_cast<int>(e - static_cast<long long>(row) * j.kpad);
      const int tap = k / j.pitch, co = k - tap * j.pitch;
      if (row < j.cin && tap < ntap && co < j.cout)
        v = src[(static_cast<long long>(co) * j.cin + row) * ntap + (ntap - 1 - tap)];
    } else {
      // deconv class c = py*2+px: out[c][row = co][k = (ty*2+tx) * cin + ci] = w[ci][co][3-py-2ty][3-px-2tx]
      const int c = static_cast<int>(e / per_cls);
      const long long r = e - c * per_cls;
      const int row = static_cast<int>(r / j.kpad), k = static_cast<int>(r - static_cast<long long>(row) * j.kpad);
      const int t = k / j.cin, ci = k - t * j.cin;
      if (row < j.cout && t < 4) {
        const int py = c >> 1, px = c & 1, ty = t >> 1, tx = t & 1;
        v = src[((static_cast<long long>(ci) * j.cout + row) * 4 + (3 - py - 2 * ty)) * 4 + (3 - px - 2 * tx)];
      }
    }
    dst[e] = cvt<T>(v);
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" long long posu_pack_job_blocks(int mode, int rows, int kpad) {
  const long long n = static_cast<long long>(rows) * kpad * (mode == POSU_PACK_DECONV ? 4 : 1);
  const long long per_block = static_cast<long long>(kThreads) * kPerThread;
  return (n + per_block - 1) / per_block;
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
