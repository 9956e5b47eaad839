// Adam update of the training step (BASELINE configs[3]; the reference's optimizer is
// torch.optim.Adam, utils/utils.py:79-83, stepped by core/function.py:366) over every parameter
// tensor of the network in a few launches: per element
//   g' = g (+ weight_decay * p)
//   m  = beta1 m + (1 - beta1) g'
//   v  = beta2 v + (1 - beta2) g'^2
//   p  = p - step_size * m / (sqrt(v) / sqrt(bc2) + eps),   step_size = lr / bc1,
//   bc1 = 1 - beta1^t, bc2 = 1 - beta2^t (the host computes both in double),
// the order of torch's Adam, in f32 (torch's kernels carry some of the products in double: the
// results agree within f32 rounding, not bit for bit).  HBM-bound: 28 B per element (p, g, m, v
// read; p, m, v written).  torch's fused multi-tensor Adam splits the step into launches of at
// most 320 chunks (~1.3 blocks per CU, 3.1 TB/s on the benched step); here every launch takes up
// to kAdamTensors tensors by value (kernel arguments, nothing to stage in device memory), one
// 2048-element chunk per block, a block finding its tensor by a scan of the launch's block
// offsets.
#include <cmath>

#include "posu_common.h"
#include "../../include/posu.h"

namespace posu {
namespace {

constexpr int kAdamTensors = 64;   // 64 x 40 B tensor records + offsets + scalars: 3.1 KB of kernel arguments (< 4 KB)
constexpr int kAdamThreads = 256, kAdamVec = 2;   // 2 float4 per thread: 2048 elements per block
constexpr int kAdamChunk = kAdamThreads * 4 * kAdamVec;

struct AdamLaunch {
  posu_adam_tensor t[kAdamTensors];
  long long blk0[kAdamTensors + 1];   // first block of tensor i; blk0[nt] = the launch's blocks
  int nt;
  float step_size, inv_bc2s, beta1, beta2, omb1, omb2, eps, wd;
};

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamLaunch& a) {
  if (a.wd != 0.f) g += a.wd * p;
  m = a.beta1 * m + a.omb1 * g;
  v = a.beta2 * v + a.omb2 * g * g;
  const float denom = sqrtf(v) * a.inv_bc2s + a.eps;
  p -= a.step_size * m / denom;
}

__global__ __launch_bounds__(kAdamThreads) void adam_kernel(const AdamLaunch a) {
  const long long b = blockIdx.x;
  int ti = 0;
  while (ti + 1 < a.nt && a.blk0[ti + 1] <= b) ++ti;   // uniform scan over <= 64 offsets
  const posu_adam_tensor& t = a.t[ti];
  const long long e0 = (b - a.blk0[ti]) * kAdamChunk;
  const long long e1 = min(t.n, e0 + kAdamChunk);
  const bool vec = ((reinterpret_cast<size_t>(t.p) | reinterpret_cast<size_t>(t.g) | reinterpret_cast<size_t>(t.m) |
                     reinterpret_cast<size_t>(t.v)) & 15) == 0;
  if (vec && e1 - e0 == kAdamChunk) {
    float4 p4[kAdamVec], g4[kAdamVec], m4[kAdamVec], v4[kAdamVec];
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
      const long long i = e0 / 4 + u * kAdamThreads + threadIdx.x;
      p4[u] = reinterpret_cast<const float4*>(t.p)[i];
      g4[u] = reinterpret_cast<const float4*>(t.g)[i];
      m4[u] = reinterpret_cast<const float4*>(t.m)[i];
      v4[u] = reinterpret_cast<const float4*>(t.v)[i];
    }
#pragma unroll
    for (int u = 0; u < kAdamVec; ++u) {
      adam_one(p4[u].x, g4[u].x, m4[u].x, v4[u].x, a);
      adam_one(p4[u].y, g4[u].y, m4[u].y, v4[u].y, a);
      adam_one(p4[u].z, g4[u].z, m4[u].z, v4[u].z, a);
      adam_one(p4[u].w, g4[u].w, m4[u].w, v4[u].w, a);
      const long long i = e0 / 4 + u * kAdamThreads + threadIdx.x;
      reinterpret_cast<float4*>(t.p)[i] = p4[u];
      reinterpret_cast<float4*>(t.m)[i] = m4[u];
      reinterpret_cast<float4*>(t.v)[i] = v4[u];
    }
    return;
  }
  for (long long i = e0 + threadIdx.x; i < e1; i += kAdamThreads) {   // ragged / unaligned tail
    float p = t.p[i], m = t.m[i], v = t.v[i];
    adam_one(p, t.g[i], m, v, a);
    t.p[i] = p;
    t.m[i] = m;
    t.v[i] = v;
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_adam_step(const posu_adam_tensor* tensors, int ntensors, double lr, double beta1, double beta2,
                              double eps, double weight_decay, long long step, void* stream) {
  POSU_REQUIRE(ntensors >= 0 && (ntensors == 0 || tensors), "posu_adam_step: null tensor table");
  POSU_REQUIRE(step >= 1, "posu_adam_step: step counts from 1");
  POSU_REQUIRE(lr >= 0.0 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0,
               "posu_adam_step: bad hyper-parameters");
  for (int i = 0; i < ntensors; ++i)
    POSU_REQUIRE(tensors[i].n >= 0 && (tensors[i].n == 0 || (tensors[i].p && tensors[i].g && tensors[i].m &&
                                                               tensors[i].v)),
                 "posu_adam_step: tensor " + std::to_string(i) + " has a null pointer");
  const double bc1 = 1.0 - std::pow(beta1, static_cast<double>(step));
  const double bc2 = 1.0 - std::pow(beta2, static_cast<double>(step));
  AdamLaunch a{};
  a.step_size = static_cast<float>(lr / bc1);
  a.inv_bc2s = static_cast<float>(1.0 / std::sqrt(bc2));
  a.beta1 = static_cast<float>(beta1);
  a.beta2 = static_cast<float>(beta2);
  a.omb1 = static_cast<float>(1.0 - beta1);
  a.omb2 = static_cast<float>(1.0 - beta2);
  a.eps = static_cast<float>(eps);
  a.wd = static_cast<float>(weight_decay);
  hipStream_t s = as_stream(stream);
  int i = 0;
  while (i < ntensors) {
    a.nt = 0;
    long long blocks = 0;
    for (; i < ntensors && a.nt < kAdamTensors; ++i) {
      if (tensors[i].n == 0) continue;
      a.t[a.nt] = tensors[i];
      a.blk0[a.nt] = blocks;
      blocks += (tensors[i].n + kAdamChunk - 1) / kAdamChunk;
      ++a.nt;
    }
    a.blk0[a.nt] = blocks;
    if (a.nt == 0) break;
    POSU_REQUIRE(blocks < (1LL << 31), "posu_adam_step: too many blocks in one launch");
    hipLaunchKernelGGL(adam_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kAdamThreads), 0, s, a);
    if (int st = check_launch("posu_adam_step")) return st;
  }
  return POSU_OK;
}
