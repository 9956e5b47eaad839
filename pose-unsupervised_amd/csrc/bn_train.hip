// Training-mode BatchNorm2d on NHWC activations (BASELINE configs[3] training step):
// batch statistics per segment (the reference runs the backbone once per camera view,
// multiview_pose_resnet.py:74-78, so every view has its own statistics; here the views
// are stacked along the batch as `nseg` segments of `Pseg` pixels and one launch
// serves all of them), the normalise + residual + ReLU epilogue, the matching
// backward, the bias-gradient channel sum and the stem max-pool backward.
//
// Reductions are deterministic: per-block partial sums in f64 written to a workspace,
// then a data-independent order (lanes over blocks, then the lanes in order) per channel.  Running statistics
// follow torch.nn.BatchNorm2d: biased variance for normalisation, unbiased variance in
// running_var, running = (1 - momentum) * running + momentum * batch, updated once per
// segment in segment (= view) order like the reference's four backbone calls.
#include <initializer_list>

#include "posu_common.h"

namespace posu {
namespace {

// pixels in flight per thread in the partial passes (the sums do not depend on them: each thread
// adds its pixels in order).  The launches are ~256 blocks of 4 waves, one wave per SIMD, so the
// loads in flight per wave set the bandwidth (round 6: 4 / 8 -> 16)
#ifndef POSU_BN_U1
#define POSU_BN_U1 4    // the backward partial pass (z, gy and the mask per pixel)
#endif
#ifndef POSU_BN_U0
#define POSU_BN_U0 8    // the forward statistics (z per pixel)
#endif
#ifndef POSU_BN_NBT
#define POSU_BN_NBT 256  // partial-sum blocks per launch (target)
#endif
#ifndef POSU_BN_RED1
#define POSU_BN_RED1 0   // 1: the block reduction through one [256][E] f64 array, sums then squares
#endif
#ifndef POSU_BN_FIN2
#define POSU_BN_FIN2 1  // the second finalize form (block per 16 channels, lane sums met in LDS)
#endif
#ifndef POSU_POOL_BWD2
#define POSU_POOL_BWD2 1  // the max-pool backward's second form (a thread per 2x2 input block)
#endif
#ifndef POSU_BN_SEGU
#define POSU_BN_SEGU 4  // chunks in flight per thread in the segment-major apply passes
#endif

constexpr int kMaxNB = 256;  // partial-sum blocks per segment

struct RedShape {
  int CPR, CB, PL, CG, NB, PPB;
};

RedShape red_shape(int Pseg, int C, int E, int nseg) {
  RedShape r;
  r.CPR = C / E;
  r.CB = std::min(r.CPR, 64);  // one wave of channel chunks per pixel row: wide layers get more blocks
  r.PL = 256 / r.CB;
  r.CG = (r.CPR + r.CB - 1) / r.CB;
  // <= 64 partial blocks per view of 4 (one load round per finalize lane); per training step
  // measured 128 / 256 / 512 / 1024 total blocks: 22.61 / 21.93 / 22.09 / 22.43 ms
  int nb = std::max(1, POSU_BN_NBT / (r.CG * nseg));
  nb = std::min(nb, kMaxNB);
  nb = std::min(nb, std::max(1, Pseg / r.PL));
  // f64 partials of wide, short layers (layer4: 2048 channels x 2048 pixels per view) stay
  // below 1/8 of the input they reduce: at least 64 pixels per block
  nb = std::min(nb, std::max(1, Pseg / 64));
  r.NB = nb;
  r.PPB = (Pseg + nb - 1) / nb;
  return r;
}

// 16 B at p + off when `ok`, else zeros; a byte of m at i when `ok`, else 0.  Loaded from a valid
// address (`alt` when not ok) and selected by value: a select between *p and a local zero becomes
// a select of addresses, which puts the zero in scratch (the f16 / f32 kernels had 32 B of it)
template <typename T>
__device__ __forceinline__ uint4 ld16_if(bool ok, const T* p, const T* alt, size_t off) {
  const uint4 v = *reinterpret_cast<const uint4*>((ok ? p : alt) + off);
  return ok ? v : make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ unsigned ld8_if(bool ok, const uint8_t* m, const void* alt, size_t i) {
  const unsigned v = (ok ? m : static_cast<const uint8_t*>(alt))[i];
  return ok ? v : 0u;
}

// MODE 0: (sum (z - K), sum (z - K)^2) -- forward statistics / channel sums; K = the
//         segment's first pixel when kout is non-null (shifted sums: a channel whose
//         mean is large against its spread keeps its variance in the f32 partials),
//         else 0.  Block 0 of each segment stores K to kout [nseg][C].
// MODE 1: (sum g', sum g' * xhat)     -- backward, g' = gy * [y > 0]: the ReLU mask from the
//         forward's bit mask (ym, one byte per 16-B chunk, bn_apply_mask), from y, or recomputed
//         from z (msc / msh); none of them: no ReLU
template <typename T, int MODE>
__global__ __launch_bounds__(256) void bn_partial_kernel(const T* __restrict__ z, const T* __restrict__ gy,
                                                         const T* __restrict__ y, const float* __restrict__ msc,
                                                         const float* __restrict__ msh,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, int Pseg, int C,
                                                         RedShape rs, double* __restrict__ part,
                                                         float* __restrict__ kout, const uint8_t* __restrict__ ym) {
  constexpr int E = Vec<T>::E;
  __shared__ double red[POSU_BN_RED1 ? 1 : 2][256][E];
  const int tid = threadIdx.x;
  const int pl = tid / rs.CB, cb = tid - pl * rs.CB;
  const int ch = blockIdx.y * rs.CB + cb;
  const int seg = blockIdx.z, blk = blockIdx.x;
  const bool active = ch < rs.CPR;
  float a[E], b[E], mu[E], rd[E], ks[E], kh[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    a[e] = 0.f;
    b[e] = 0.f;
    mu[e] = 0.f;
    rd[e] = 0.f;
    ks[e] = 0.f;
    kh[e] = 0.f;
  }
  if (MODE == 1 && active) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      mu[e] = mean[seg * C + ch * E + e];
      rd[e] = rstd[seg * C + ch * E + e];
      if (msc) {
        ks[e] = msc[seg * C + ch * E + e];
        kh[e] = msh[seg * C + ch * E + e];
      }
    }
  }
  float kv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) kv[e] = 0.f;
  if (MODE == 0 && kout && active) {
    Vec<T>::unpack(*reinterpret_cast<const uint4*>(z + static_cast<size_t>(seg) * Pseg * C + ch * E), kv);
    if (blk == 0 && pl == 0) {
#pragma unroll
      for (int e = 0; e < E; ++e) kout[seg * C + ch * E + e] = kv[e];
    }
  }
  if (active) {
    const int pbeg = blk * rs.PPB, pend = min(Pseg, pbeg + rs.PPB);
    const size_t sbase = static_cast<size_t>(seg) * Pseg * C + ch * E;
    // one pixel's contribution, accumulated in pixel order (the sums do not depend on U)
    auto acc = [&](const uint4& zq, const uint4& gq, const uint4& yq, unsigned mq) {
      float v[E];
      Vec<T>::unpack(zq, v);
      if constexpr (MODE == 0) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float d = v[e] - kv[e];
          a[e] += d;
          b[e] += d * d;
        }
      } else {
        float gv[E];
        Vec<T>::unpack(gq, gv);
        if (ym) {
#pragma unroll
          for (int e = 0; e < E; ++e) gv[e] = (mq >> e) & 1u ? gv[e] : 0.f;
        } else if (y) {
          float yv[E];
          Vec<T>::unpack(yq, yv);
#pragma unroll
          for (int e = 0; e < E; ++e) gv[e] = yv[e] > 0.f ? gv[e] : 0.f;
        } else if (msc) {  // ReLU mask recomputed from z (no residual): y > 0 <=> z*scale+shift > 0
#pragma unroll
          for (int e = 0; e < E; ++e) gv[e] = v[e] * ks[e] + kh[e] > 0.f ? gv[e] : 0.f;
        }
#pragma unroll
        for (int e = 0; e < E; ++e) {
          a[e] += gv[e];
          b[e] += gv[e] * ((v[e] - mu[e]) * rd[e]);
        }
      }
    };
    // U pixels per step with all their loads issued first (memory-level parallelism); the ReLU
    // source's loads behind wave-uniform branches (a y or mask load only when that is the source)
    constexpr int U = MODE == 0 ? POSU_BN_U0 : POSU_BN_U1;
    const uint4 zero = make_uint4(0, 0, 0, 0);
    const bool use_y = MODE == 1 && y && !ym, use_m = MODE == 1 && ym;
    int p = pbeg + pl;
    for (; p + (U - 1) * rs.PL < pend; p += U * rs.PL) {
      uint4 zq[U], gq[U], yq[U];
      unsigned mq[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t off = sbase + static_cast<size_t>(p + u * rs.PL) * C;
        zq[u] = *reinterpret_cast<const uint4*>(z + off);
        gq[u] = MODE == 1 ? *reinterpret_cast<const uint4*>(gy + off) : zero;
        yq[u] = zero;
        mq[u] = 0u;
      }
      if (use_y) {
#pragma unroll
        for (int u = 0; u < U; ++u) yq[u] = *reinterpret_cast<const uint4*>(y + sbase + static_cast<size_t>(p + u * rs.PL) * C);
      } else if (use_m) {
#pragma unroll
        for (int u = 0; u < U; ++u) mq[u] = ym[(sbase + static_cast<size_t>(p + u * rs.PL) * C) / E];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc(zq[u], gq[u], yq[u], mq[u]);
    }
    for (; p < pend; p += rs.PL) {
      const size_t off = sbase + static_cast<size_t>(p) * C;
      acc(*reinterpret_cast<const uint4*>(z + off), MODE == 1 ? *reinterpret_cast<const uint4*>(gy + off) : zero,
          ld16_if(MODE == 1 && y && !ym, y, z, off), ld8_if(MODE == 1 && ym, ym, z, off / E));
    }
  }
  double* dst = part + (static_cast<size_t>(seg) * rs.NB + blk) * 2 * C;
  if constexpr (POSU_BN_RED1) {
    // the same tree, one quantity at a time through a 16 KB array (the partial pass shares CUs
    // with the weight-gradient kernels' 128 KB of LDS in the backward)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
#pragma unroll
      for (int e = 0; e < E; ++e) red[0][tid][e] = k ? b[e] : a[e];
      __syncthreads();
      for (int s = rs.PL / 2; s > 0; s >>= 1) {
        if (pl < s) {
          const int o = tid + s * rs.CB;
#pragma unroll
          for (int e = 0; e < E; ++e) red[0][tid][e] += red[0][o][e];
        }
        __syncthreads();
      }
      if (pl == 0 && active) {
#pragma unroll
        for (int e = 0; e < E; ++e) dst[k * C + ch * E + e] = red[0][tid][e];
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < E; ++e) {
    red[0][tid][e] = a[e];
    red[POSU_BN_RED1 ? 0 : 1][tid][e] = b[e];
  }
  __syncthreads();
  for (int s = rs.PL / 2; s > 0; s >>= 1) {
    if (pl < s) {
      const int o = tid + s * rs.CB;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        red[0][tid][e] += red[0][o][e];
        red[POSU_BN_RED1 ? 0 : 1][tid][e] += red[POSU_BN_RED1 ? 0 : 1][o][e];
      }
    }
    __syncthreads();
  }
  if (pl == 0 && active) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      dst[ch * E + e] = red[0][tid][e];
      dst[C + ch * E + e] = red[POSU_BN_RED1 ? 0 : 1][tid][e];
    }
  }
}

// ---- finalize: one block per FCH channels, FLN lanes sum the partial blocks of up to
// FSEG segments at once (every load of the pass in flight together: the partials are a few
// hundred KiB, so this pass is latency-bound), then a fixed xor butterfly across the lanes
// (round 2 combined the lanes serially through LDS in one thread: ~12 us per launch).
constexpr int FCH = 8, FLN = 32, FSEG = 4;

// thread t of a finalize block: channel blockIdx.x * FCH + t / FLN, lane t % FLN; the FLN lanes
// of a channel are one half-wave.  Each lane sums the partial blocks ln, ln + FLN, .. of up to
// FSEG segments (all loads in flight together), then a fixed xor butterfly over the half-wave;
// lane 0's sums are the result (its association order does not depend on the data)
__device__ __forceinline__ void reduce_segs(const double* __restrict__ part, int seg0, int ns, int NB, int C, int c,
                                            bool valid, int ln, double* s, double* q) {
  double a[FSEG], b[FSEG];
#pragma unroll
  for (int k = 0; k < FSEG; ++k) a[k] = b[k] = 0.0;
  if (valid) {
    const double* base = part + static_cast<size_t>(seg0) * NB * 2 * C + c;
#pragma unroll 4
    for (int blk = ln; blk < NB; blk += FLN) {
#pragma unroll
      for (int k = 0; k < FSEG; ++k)
        if (k < ns) {
          const double* p = base + (static_cast<size_t>(k) * NB + blk) * 2 * C;
          a[k] += p[0];
          b[k] += p[C];
        }
    }
  }
#pragma unroll
  for (int off = FLN / 2; off > 0; off >>= 1)
#pragma unroll
    for (int k = 0; k < FSEG; ++k) {
      a[k] += __shfl_xor(a[k], off, FLN);
      b[k] += __shfl_xor(b[k], off, FLN);
    }
#pragma unroll
  for (int k = 0; k < FSEG; ++k) {
    s[k] = a[k];
    q[k] = b[k];
  }
}

__global__ __launch_bounds__(256) void bn_stats_finalize_kernel(const double* __restrict__ part, int nseg, int NB,
                                                                int Pseg, int C, const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, float eps,
                                                                float momentum, const float* __restrict__ kshift,
                                                                float* __restrict__ running_mean,
                                                                float* __restrict__ running_var,
                                                                float* __restrict__ mean, float* __restrict__ rstd,
                                                                float* __restrict__ scale,
                                                                float* __restrict__ shift) {
  const int cl = threadIdx.x / FLN, ln = threadIdx.x % FLN;
  const int c = blockIdx.x * FCH + cl;
  const bool valid = c < C;
  const double n = static_cast<double>(Pseg);
  // the per-channel parameters first: their loads overlap the partials' (one round trip, not
  // one per segment behind the running-statistics stores)
  const int cc = valid ? c : 0;
  const float gm = gamma ? gamma[cc] : 1.f, bt = beta ? beta[cc] : 0.f;
  float rm = running_mean ? running_mean[cc] : 0.f, rv = running_var ? running_var[cc] : 0.f;
  for (int seg0 = 0; seg0 < nseg; seg0 += FSEG) {
    const int ns = min(FSEG, nseg - seg0);
    float ks[FSEG];
#pragma unroll
    for (int k = 0; k < FSEG; ++k) ks[k] = k < ns ? kshift[(seg0 + k) * C + cc] : 0.f;
    double sums[FSEG], sqs[FSEG];
    reduce_segs(part, seg0, ns, NB, C, c, valid, ln, sums, sqs);
    if (ln != 0 || !valid) continue;
    for (int k = 0; k < ns; ++k) {  // in segment order: running stats compose like V calls
      const int seg = seg0 + k;
      const double sum = sums[k], sq = sqs[k];  // shifted by K = kshift[seg][c]
      const double dm = sum / n;
      const double mu = static_cast<double>(ks[k]) + dm;
      const double var = fmax(sq / n - dm * dm, 0.0);
      const double r = 1.0 / sqrt(var + static_cast<double>(eps));
      mean[seg * C + c] = static_cast<float>(mu);
      rstd[seg * C + c] = static_cast<float>(r);
      scale[seg * C + c] = static_cast<float>(gm * r);
      shift[seg * C + c] = static_cast<float>(bt - mu * gm * r);
      rm = (1.f - momentum) * rm + momentum * static_cast<float>(mu);
      rv = (1.f - momentum) * rv + momentum * static_cast<float>(Pseg > 1 ? var * n / (n - 1.0) : var);
    }
  }
  if (ln == 0 && valid) {
    if (running_mean) running_mean[c] = rm;
    if (running_var) running_var[c] = rv;
  }
}

// y = act(z * scale[seg] + shift[seg] (+ res)), one thread per 16-B chunk; mask (optional, ReLU
// only): one byte per chunk, bit e = [y_e > 0] -- the backward's ReLU mask at 1/16 of y's bytes
template <typename T>
__device__ __forceinline__ uint8_t pos_bits(const float* v) {
  unsigned m = 0;
#pragma unroll
  for (int e = 0; e < Vec<T>::E; ++e) m |= (v[e] > 0.f ? 1u : 0u) << e;
  return static_cast<uint8_t>(m);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ z, int Pseg, int C,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const T* __restrict__ res,
                                                       int relu, T* __restrict__ y, long long total,
                                                       uint8_t* __restrict__ mask) {
  constexpr int E = Vec<T>::E;
  const int CPR = C / E;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const long long pix = i / CPR;
    const int c0 = static_cast<int>(i - pix * CPR) * E;
    const int seg = static_cast<int>(pix / Pseg);
    float v[E];
    Vec<T>::unpack(*reinterpret_cast<const uint4*>(z + i * E), v);
    float r[E];
    if (res) Vec<T>::unpack(*reinterpret_cast<const uint4*>(res + i * E), r);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float t = v[e] * scale[seg * C + c0 + e] + shift[seg * C + c0 + e];
      if (res) t += r[e];
      v[e] = relu ? fmaxf(t, 0.f) : t;
    }
    const uint4 o = Vec<T>::pack(v);
    *reinterpret_cast<uint4*>(y + i * E) = o;
    if (mask) {
      Vec<T>::unpack(o, v);   // the stored (rounded) values: the mask the backward would read from y
      mask[i] = pos_bits<T>(v);
    }
  }
}

// Segment-major variants (C / E divides 256): blockIdx.y = segment, a thread's channel
// chunk never changes (the grid stride is a multiple of 256), so the per-channel
// parameters live in registers; U chunks per step with their loads issued first.
// Same arithmetic per element as the kernels above.
constexpr int kSegU = POSU_BN_SEGU;

// E consecutive per-channel f32 parameters as 16-B loads (E = 4 or 8; every parameter
// row starts at a multiple of 8 channels of a 16-B aligned allocation)
template <int E>
__device__ __forceinline__ void ldparams(const float* __restrict__ p, float* v) {
#pragma unroll
  for (int i = 0; i < E / 4; ++i) {
    const float4 q = reinterpret_cast<const float4*>(p)[i];
    v[4 * i] = q.x;
    v[4 * i + 1] = q.y;
    v[4 * i + 2] = q.z;
    v[4 * i + 3] = q.w;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_seg_kernel(const T* __restrict__ z, int Pseg, int C,
                                                           const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const T* __restrict__ res, int relu, T* __restrict__ y,
                                                           uint8_t* __restrict__ mask) {
  constexpr int E = Vec<T>::E, U = kSegU;
  const int CPR = C / E, seg = blockIdx.y;
  const int c0 = (threadIdx.x % CPR) * E;
  float sc[E], sh[E];
  ldparams<E>(scale + seg * C + c0, sc);
  ldparams<E>(shift + seg * C + c0, sh);
  const int n = Pseg * CPR, stride = gridDim.x * 256;
  const T* __restrict__ zs = z + static_cast<size_t>(seg) * Pseg * C;
  const T* __restrict__ rs = res ? res + static_cast<size_t>(seg) * Pseg * C : nullptr;
  T* __restrict__ ys = y + static_cast<size_t>(seg) * Pseg * C;
  uint8_t* __restrict__ ms = mask ? mask + static_cast<size_t>(seg) * Pseg * CPR : nullptr;
  auto one = [&](int i, const uint4& zq, const uint4& rq) {
    float v[E], r[E];
    Vec<T>::unpack(zq, v);
    if (rs) Vec<T>::unpack(rq, r);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float t = v[e] * sc[e] + sh[e];
      if (rs) t += r[e];
      v[e] = relu ? fmaxf(t, 0.f) : t;
    }
    const uint4 o = Vec<T>::pack(v);
    *reinterpret_cast<uint4*>(ys + static_cast<size_t>(i) * E) = o;
    if (ms) {
      Vec<T>::unpack(o, v);
      ms[i] = pos_bits<T>(v);
    }
  };
  int i = blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    uint4 zq[U], rq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      zq[u] = *reinterpret_cast<const uint4*>(zs + static_cast<size_t>(i + u * stride) * E);
      rq[u] = ld16_if(rs != nullptr, rs, zs, static_cast<size_t>(i + u * stride) * E);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(i + u * stride, zq[u], rq[u]);
  }
  for (; i < n; i += stride)
    one(i, *reinterpret_cast<const uint4*>(zs + static_cast<size_t>(i) * E),
        ld16_if(rs != nullptr, rs, zs, static_cast<size_t>(i) * E));
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_seg_kernel(const T* __restrict__ gy, const T* __restrict__ y,
                                                               const float* __restrict__ msc,
                                                               const float* __restrict__ msh,
                                                               const T* __restrict__ z, int Pseg, int C,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ coef, T* __restrict__ dz,
                                                               T* __restrict__ gres, const uint8_t* __restrict__ ym) {
  constexpr int E = Vec<T>::E, U = kSegU;
  const int CPR = C / E, seg = blockIdx.y;
  const int c0 = (threadIdx.x % CPR) * E;
  float mu[E], rd[E], k1[E], mg[E], mgx[E], ks[E], kh[E];
  ldparams<E>(mean + seg * C + c0, mu);
  ldparams<E>(rstd + seg * C + c0, rd);
  ldparams<E>(coef + (seg * 3 + 0) * C + c0, k1);
  ldparams<E>(coef + (seg * 3 + 1) * C + c0, mg);
  ldparams<E>(coef + (seg * 3 + 2) * C + c0, mgx);
  if (msc) {
    ldparams<E>(msc + seg * C + c0, ks);
    ldparams<E>(msh + seg * C + c0, kh);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e) ks[e] = kh[e] = 0.f;
  }
  const int n = Pseg * CPR, stride = gridDim.x * 256;
  const size_t sb = static_cast<size_t>(seg) * Pseg * C;
  auto one = [&](int i, const uint4& gq, const uint4& zq, const uint4& yq, unsigned mq) {
    const size_t off = sb + static_cast<size_t>(i) * E;
    float g[E], v[E];
    Vec<T>::unpack(gq, g);
    Vec<T>::unpack(zq, v);
    if (ym) {
#pragma unroll
      for (int e = 0; e < E; ++e) g[e] = (mq >> e) & 1u ? g[e] : 0.f;
    } else if (y) {
      float yv[E];
      Vec<T>::unpack(yq, yv);
#pragma unroll
      for (int e = 0; e < E; ++e) g[e] = yv[e] > 0.f ? g[e] : 0.f;
    } else if (msc) {
#pragma unroll
      for (int e = 0; e < E; ++e) g[e] = v[e] * ks[e] + kh[e] > 0.f ? g[e] : 0.f;
    }
    if (gres) *reinterpret_cast<uint4*>(gres + off) = Vec<T>::pack(g);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float xh = (v[e] - mu[e]) * rd[e];
      v[e] = k1[e] * (g[e] - mg[e] - xh * mgx[e]);
    }
    *reinterpret_cast<uint4*>(dz + off) = Vec<T>::pack(v);
  };
  int i = blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    uint4 gq[U], zq[U], yq[U];
    unsigned mq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = sb + static_cast<size_t>(i + u * stride) * E;
      gq[u] = *reinterpret_cast<const uint4*>(gy + off);
      zq[u] = *reinterpret_cast<const uint4*>(z + off);
      yq[u] = ld16_if(y && !ym, y, z, off);
      mq[u] = ld8_if(ym != nullptr, ym, z, off / E);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(i + u * stride, gq[u], zq[u], yq[u], mq[u]);
  }
  for (; i < n; i += stride) {
    const size_t off = sb + static_cast<size_t>(i) * E;
    one(i, *reinterpret_cast<const uint4*>(gy + off), *reinterpret_cast<const uint4*>(z + off),
        ld16_if(y && !ym, y, z, off), ld8_if(ym != nullptr, ym, z, off / E));
  }
}

// blocks per segment of a segment-major launch: at least 16 chunks per thread (the
// per-channel parameters are loaded once per thread), at most about 1024 blocks in all
inline int seg_blocks(int Pseg, int C, int E, int nseg) {
  const long long chunks = static_cast<long long>(Pseg) * (C / E);
  const long long need = (chunks + 256LL * 16 - 1) / (256LL * 16);
  const long long cap = std::max(1, 1024 / nseg);
  return static_cast<int>(std::max(1LL, std::min(need, cap)));
}

inline bool aligned16(const void* p) { return (reinterpret_cast<size_t>(p) & 15) == 0; }

inline bool seg_major(int C, int E, int nseg, int Pseg, std::initializer_list<const void*> params) {
  for (const void* p : params)
    if (p && !aligned16(p)) return false;
  const int cpr = C / E;
  // the loops index chunks in int: i + (U - 1) * stride and i + U * stride must stay below
  // 2^31 for the largest i < Pseg * cpr (stride <= 1024 blocks * 256 threads)
  const long long n = static_cast<long long>(Pseg) * cpr;
  return cpr > 0 && 256 % cpr == 0 && nseg <= 65535 && n + static_cast<long long>(kSegU) * 1024 * 256 < (1LL << 31);
}

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const double* __restrict__ part, int nseg, int NB,
                                                              int Pseg, int C, const float* __restrict__ gamma,
                                                              const float* __restrict__ rstd,
                                                              float* __restrict__ coef, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta) {
  const int cl = threadIdx.x / FLN, ln = threadIdx.x % FLN;
  const int c = blockIdx.x * FCH + cl;
  const bool valid = c < C;
  const double n = static_cast<double>(Pseg);
  const int cc = valid ? c : 0;
  const float gm = gamma ? gamma[cc] : 1.f;
  double tg = 0.0, tgx = 0.0;
  for (int seg0 = 0; seg0 < nseg; seg0 += FSEG) {
    const int ns = min(FSEG, nseg - seg0);
    float rs[FSEG];  // loaded beside the partials
#pragma unroll
    for (int k = 0; k < FSEG; ++k) rs[k] = k < ns ? rstd[(seg0 + k) * C + cc] : 0.f;
    double sgs[FSEG], sgxs[FSEG];
    reduce_segs(part, seg0, ns, NB, C, c, valid, ln, sgs, sgxs);
    if (ln != 0 || !valid) continue;
    for (int k = 0; k < ns; ++k) {
      const int seg = seg0 + k;
      const double sg = sgs[k], sgx = sgxs[k];
      tg += sg;
      tgx += sgx;
      coef[(seg * 3 + 0) * C + c] = gm * rs[k];
      coef[(seg * 3 + 1) * C + c] = static_cast<float>(sg / n);
      coef[(seg * 3 + 2) * C + c] = static_cast<float>(sgx / n);
    }
  }
  if (ln == 0 && valid) {
    if (dgamma) dgamma[c] = static_cast<float>(tgx);
    if (dbeta) dbeta[c] = static_cast<float>(tg);
  }
}

// dz = gamma*rstd * (g' - mean(g') - xhat * mean(g' xhat)), g' = gy * [y > 0];
// gres (optional) = g', the gradient of the residual branch
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ gy, const T* __restrict__ y,
                                                           const float* __restrict__ msc,
                                                           const float* __restrict__ msh,
                                                           const T* __restrict__ z, int Pseg, int C,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           const float* __restrict__ coef, T* __restrict__ dz,
                                                           T* __restrict__ gres, long long total,
                                                           const uint8_t* __restrict__ ym) {
  constexpr int E = Vec<T>::E;
  const int CPR = C / E;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const long long pix = i / CPR;
    const int c0 = static_cast<int>(i - pix * CPR) * E;
    const int seg = static_cast<int>(pix / Pseg);
    float g[E], v[E];
    Vec<T>::unpack(*reinterpret_cast<const uint4*>(gy + i * E), g);
    Vec<T>::unpack(*reinterpret_cast<const uint4*>(z + i * E), v);
    if (ym) {
      const unsigned mq = ym[i];
#pragma unroll
      for (int e = 0; e < E; ++e) g[e] = (mq >> e) & 1u ? g[e] : 0.f;
    } else if (y) {
      float yv[E];
      Vec<T>::unpack(*reinterpret_cast<const uint4*>(y + i * E), yv);
#pragma unroll
      for (int e = 0; e < E; ++e) g[e] = yv[e] > 0.f ? g[e] : 0.f;
    } else if (msc) {
#pragma unroll
      for (int e = 0; e < E; ++e) g[e] = v[e] * msc[seg * C + c0 + e] + msh[seg * C + c0 + e] > 0.f ? g[e] : 0.f;
    }
    if (gres) *reinterpret_cast<uint4*>(gres + i * E) = Vec<T>::pack(g);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int c = c0 + e;
      const float xh = (v[e] - mean[seg * C + c]) * rstd[seg * C + c];
      const float k1 = coef[(seg * 3 + 0) * C + c], mg = coef[(seg * 3 + 1) * C + c],
                  mgx = coef[(seg * 3 + 2) * C + c];
      v[e] = k1 * (g[e] - mg - xh * mgx);
    }
    *reinterpret_cast<uint4*>(dz + i * E) = Vec<T>::pack(v);
  }
}

__global__ __launch_bounds__(256) void channel_sum_finalize_kernel(const double* __restrict__ part, int NB, int C,
                                                                   float* __restrict__ out) {
  const int cl = threadIdx.x / FLN, ln = threadIdx.x % FLN;
  const int c = blockIdx.x * FCH + cl;
  double s[FSEG], q[FSEG];
  reduce_segs(part, 0, 1, NB, C, c, c < C, ln, s, q);
  if (ln == 0 && c < C) out[c] = static_cast<float>(s[0]);
}

// ---- finalize, second form (POSU_BN_FIN2, the default): the passes above took 12 us per launch
// in the training step (112 launches, 1.3 ms of the main stream) for a few hundred KiB of
// partials: half-waves of one channel gather 32 scattered lines per load, under per-segment
// branches.  Here a block serves FC2 consecutive channels: lane ln of channel cl sums the partial
// blocks ln, ln + FL2, .. (FIT2 of them per pass, for up to FSEG segments: every load of a pass
// issued before the first add), a wave's loads covering 4 blocks x 16 channels = 4 lines of
// 128 B; the FL2 lane sums meet in LDS and thread (k, cl) of wave 0 adds them in lane order (a
// fixed association), then does segment k's arithmetic -- the segments in parallel, not one
// lane's serial chain.
constexpr int FC2 = 16, FL2 = 16, FIT2 = 4;
constexpr int kFinLds = 2 * FSEG * FL2 * FC2;  // doubles

// returns, in thread t < FSEG * FC2 (segment seg0 + t / FC2, channel c0 + t % FC2), the sums
// over the partial blocks; zeros elsewhere.  Every thread of the block calls it.
__device__ __forceinline__ void reduce_partials(const double* __restrict__ part, int seg0, int ns, int NB, int C,
                                                int c0, double* __restrict__ lds, double& s, double& q) {
  const int t = threadIdx.x, cl = t % FC2, ln = t / FC2;
  const int c = c0 + cl;
  const bool cv = c < C;
  double a[FSEG], b[FSEG];
#pragma unroll
  for (int k = 0; k < FSEG; ++k) a[k] = b[k] = 0.0;
  for (int base = 0; base < NB; base += FL2 * FIT2) {
    double va[FSEG][FIT2], vb[FSEG][FIT2];
#pragma unroll
    for (int k = 0; k < FSEG; ++k)
#pragma unroll
      for (int j = 0; j < FIT2; ++j) {
        const int blk = base + ln + FL2 * j;
        const bool ok = cv && k < ns && blk < NB;
        // a valid address either way, the value selected (no select of a load against a zero)
        const double* p = part + (ok ? static_cast<size_t>((seg0 + k) * NB + blk) * 2 * C + c : 0);
        const double x = p[0], y = p[ok ? C : 0];
        va[k][j] = ok ? x : 0.0;
        vb[k][j] = ok ? y : 0.0;
      }
#pragma unroll
    for (int k = 0; k < FSEG; ++k)
#pragma unroll
      for (int j = 0; j < FIT2; ++j) {
        a[k] += va[k][j];
        b[k] += vb[k][j];
      }
  }
#pragma unroll
  for (int k = 0; k < FSEG; ++k) {
    lds[((0 * FSEG + k) * FL2 + ln) * FC2 + cl] = a[k];
    lds[((1 * FSEG + k) * FL2 + ln) * FC2 + cl] = b[k];
  }
  __syncthreads();
  s = q = 0.0;
  if (t < FSEG * FC2) {
    const int k = t / FC2;
#pragma unroll
    for (int l = 0; l < FL2; ++l) {
      s += lds[((0 * FSEG + k) * FL2 + l) * FC2 + cl];
      q += lds[((1 * FSEG + k) * FL2 + l) * FC2 + cl];
    }
  }
  __syncthreads();  // lds is reused by the next call
}

__global__ __launch_bounds__(256) void bn_stats_finalize2_kernel(const double* __restrict__ part, int nseg, int NB,
                                                                 int Pseg, int C, const float* __restrict__ gamma,
                                                                 const float* __restrict__ beta, float eps,
                                                                 float momentum, const float* __restrict__ kshift,
                                                                 float* __restrict__ running_mean,
                                                                 float* __restrict__ running_var,
                                                                 float* __restrict__ mean, float* __restrict__ rstd,
                                                                 float* __restrict__ scale,
                                                                 float* __restrict__ shift) {
  __shared__ double lds[kFinLds];
  __shared__ float mus[FSEG][FC2], vus[FSEG][FC2];
  const int t = threadIdx.x, k = t / FC2, cl = t % FC2;
  const int c0 = blockIdx.x * FC2, c = c0 + cl;
  const bool mine = t < FSEG * FC2 && c < C;  // thread (segment k, channel c) of wave 0
  const double n = static_cast<double>(Pseg);
  const int cc = c < C ? c : 0;
  const float gm = gamma ? gamma[cc] : 1.f, bt = beta ? beta[cc] : 0.f;
  float rm = 0.f, rv = 0.f;
  if (t < FC2 && c < C) {
    rm = running_mean ? running_mean[c] : 0.f;
    rv = running_var ? running_var[c] : 0.f;
  }
  for (int seg0 = 0; seg0 < nseg; seg0 += FSEG) {
    const int ns = min(FSEG, nseg - seg0);
    const bool act = mine && k < ns;
    const int seg = seg0 + (act ? k : 0);
    const float ks = kshift[seg * C + cc];  // issued beside the partials
    double sum, sq;
    reduce_partials(part, seg0, ns, NB, C, c0, lds, sum, sq);
    if (act) {
      const double dm = sum / n;  // shifted by K = kshift[seg][c]
      const double mu = static_cast<double>(ks) + dm;
      const double var = fmax(sq / n - dm * dm, 0.0);
      const double r = 1.0 / sqrt(var + static_cast<double>(eps));
      mean[seg * C + c] = static_cast<float>(mu);
      rstd[seg * C + c] = static_cast<float>(r);
      scale[seg * C + c] = static_cast<float>(gm * r);
      shift[seg * C + c] = static_cast<float>(bt - mu * gm * r);
      mus[k][cl] = static_cast<float>(mu);
      vus[k][cl] = static_cast<float>(Pseg > 1 ? var * n / (n - 1.0) : var);
    }
    __syncthreads();
    if (t < FC2 && c < C)
      for (int j = 0; j < ns; ++j) {  // in segment order: running stats compose like V calls
        rm = (1.f - momentum) * rm + momentum * mus[j][t];
        rv = (1.f - momentum) * rv + momentum * vus[j][t];
      }
    __syncthreads();
  }
  if (t < FC2 && c < C) {
    if (running_mean) running_mean[c] = rm;
    if (running_var) running_var[c] = rv;
  }
}

__global__ __launch_bounds__(256) void bn_bwd_finalize2_kernel(const double* __restrict__ part, int nseg, int NB,
                                                               int Pseg, int C, const float* __restrict__ gamma,
                                                               const float* __restrict__ rstd,
                                                               float* __restrict__ coef, float* __restrict__ dgamma,
                                                               float* __restrict__ dbeta) {
  __shared__ double lds[kFinLds];
  __shared__ double sgs[FSEG][FC2], sgxs[FSEG][FC2];
  const int t = threadIdx.x, k = t / FC2, cl = t % FC2;
  const int c0 = blockIdx.x * FC2, c = c0 + cl;
  const bool mine = t < FSEG * FC2 && c < C;
  const double n = static_cast<double>(Pseg);
  const int cc = c < C ? c : 0;
  const float gm = gamma ? gamma[cc] : 1.f;
  double tg = 0.0, tgx = 0.0;
  for (int seg0 = 0; seg0 < nseg; seg0 += FSEG) {
    const int ns = min(FSEG, nseg - seg0);
    const bool act = mine && k < ns;
    const int seg = seg0 + (act ? k : 0);
    const float rs = rstd[seg * C + cc];
    double sg, sgx;
    reduce_partials(part, seg0, ns, NB, C, c0, lds, sg, sgx);
    if (act) {
      coef[(seg * 3 + 0) * C + c] = gm * rs;
      coef[(seg * 3 + 1) * C + c] = static_cast<float>(sg / n);
      coef[(seg * 3 + 2) * C + c] = static_cast<float>(sgx / n);
      sgs[k][cl] = sg;
      sgxs[k][cl] = sgx;
    }
    __syncthreads();
    if (t < FC2 && c < C)
      for (int j = 0; j < ns; ++j) {  // segment order
        tg += sgs[j][t];
        tgx += sgxs[j][t];
      }
    __syncthreads();
  }
  if (t < FC2 && c < C) {
    if (dgamma) dgamma[c] = static_cast<float>(tgx);
    if (dbeta) dbeta[c] = static_cast<float>(tg);
  }
}

__global__ __launch_bounds__(256) void channel_sum_finalize2_kernel(const double* __restrict__ part, int NB, int C,
                                                                    float* __restrict__ out) {
  __shared__ double lds[kFinLds];
  const int t = threadIdx.x, c = blockIdx.x * FC2 + t % FC2;
  double s, q;
  reduce_partials(part, 0, 1, NB, C, blockIdx.x * FC2, lds, s, q);
  if (t < FC2 && c < C) out[c] = static_cast<float>(s);
}

// ---- max-pool 3x3 / s2 / p1 backward (PyTorch's tie rule: the first maximum in
// window scan order, pool.h max_pool2d `val > maxval || isnan(val)`).
// pass 1: argmax tap (0..8) per output element; pass 2: every input element gathers
// the gradients of the (at most 2 x 2) windows whose argmax it is -- no atomics.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_argmax_kernel(const T* __restrict__ x, int N, int H, int W, int C,
                                                             int Ho, int Wo, uint8_t* __restrict__ idx) {
  constexpr int E = Vec<T>::E;
  const int chunks = C / E;
  const long long total = static_cast<long long>(N) * Ho * Wo * chunks;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const int ox = static_cast<int>(pix % Wo);
    const long long t = pix / Wo;
    const int oy = static_cast<int>(t % Ho);
    const long long n = t / Ho;
    float m[E];
    int am[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      m[e] = 0.f;
      am[e] = -1;
    }
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap - 3 * dy;
      const int iy = oy * 2 - 1 + dy, ix = ox * 2 - 1 + dx;
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
      float v[E];
      Vec<T>::unpack(*reinterpret_cast<const uint4*>(x + ((n * H + iy) * W + ix) * C + ch * E), v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const bool take = am[e] < 0 || v[e] > m[e] || v[e] != v[e];
        m[e] = take ? v[e] : m[e];
        am[e] = take ? tap : am[e];
      }
    }
    uint8_t* dst = idx + pix * C + ch * E;
#pragma unroll
    for (int e = 0; e < E; ++e) dst[e] = static_cast<uint8_t>(am[e]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const uint8_t* __restrict__ idx, const T* __restrict__ gy,
                                                          int N, int H, int W, int C, int Ho, int Wo,
                                                          T* __restrict__ gx) {
  constexpr int E = Vec<T>::E;
  const int chunks = C / E;
  const long long total = static_cast<long long>(N) * H * W * chunks;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const int ix = static_cast<int>(pix % W);
    const long long t = pix / W;
    const int iy = static_cast<int>(t % H);
    const long long n = t / H;
    float acc[E];
#pragma unroll
    for (int e = 0; e < E; ++e) acc[e] = 0.f;
    // windows oy with 2*oy - 1 <= iy <= 2*oy + 1, in increasing (oy, ox) order
    const int oy0 = max(0, (iy - 1) / 2), oy1 = min(Ho - 1, (iy + 1) / 2);
    const int ox0 = max(0, (ix - 1) / 2), ox1 = min(Wo - 1, (ix + 1) / 2);
    for (int oy = oy0; oy <= oy1; ++oy) {
      const int dy = iy - (oy * 2 - 1);
      if (dy < 0 || dy > 2) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int dx = ix - (ox * 2 - 1);
        if (dx < 0 || dx > 2) continue;
        const long long o = ((n * Ho + oy) * Wo + ox) * C + ch * E;
        float g[E];
        Vec<T>::unpack(*reinterpret_cast<const uint4*>(gy + o), g);
        const unsigned tap = dy * 3 + dx;
        // the chunk's E taps in one 4- / 8-byte load (o is a multiple of E)
        unsigned long long tv;
        if constexpr (E == 8) tv = *reinterpret_cast<const unsigned long long*>(idx + o);
        else tv = *reinterpret_cast<const unsigned*>(idx + o);
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (((tv >> (8 * e)) & 0xffu) == tap) acc[e] += g[e];
      }
    }
    *reinterpret_cast<uint4*>(gx + pix * C + ch * E) = Vec<T>::pack(acc);
  }
}

// second form (POSU_POOL_BWD2, the default): a thread per 2x2 input block (rows 2a, 2a+1, columns
// 2b, 2b+1) and 16-B channel chunk.  Input row 2a lies in window row a only (tap row 1), row 2a+1 in
// window rows a (tap row 2) and a+1 (tap row 0), and likewise for columns, so the block's four
// outputs need exactly the windows (a | a+1) x (b | b+1): four gradient / tap loads per four
// stores, no data-dependent loop and 32-bit index math (the first form loaded 2.25 windows per
// input chunk with 64-bit divisions: 193 us for the training stem's 268 MB at 128 frames).  The
// windows are added in increasing (oy, ox) order, as in the first form: the same sums.
template <typename T>
__global__ __launch_bounds__(256) void maxpool_bwd2_kernel(const uint8_t* __restrict__ idx, const T* __restrict__ gy,
                                                           int N, int H, int W, int C, int Ho, int Wo,
                                                           T* __restrict__ gx) {
  constexpr int E = Vec<T>::E;
  const int chunks = C / E, Hq = (H + 1) / 2, Wq = (W + 1) / 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * Hq * Wq * chunks) return;
  const int ch = i % chunks;
  int q = i / chunks;
  const int b = q % Wq;
  q /= Wq;
  const int a = q % Hq, n = q / Hq;
  float g[2][2][E];
  unsigned long long tv[2][2];
#pragma unroll
  for (int wy = 0; wy < 2; ++wy)
#pragma unroll
    for (int wx = 0; wx < 2; ++wx) {
      const bool ok = a + wy < Ho && b + wx < Wo;
      // a valid address either way, the value selected (an absent window matches no tap)
      const size_t o = ok ? ((static_cast<size_t>(n) * Ho + a + wy) * Wo + b + wx) * C + ch * E : 0;
      const uint4 gq = *reinterpret_cast<const uint4*>(gy + o);
      unsigned long long t;
      if constexpr (E == 8) t = *reinterpret_cast<const unsigned long long*>(idx + o);
      else t = *reinterpret_cast<const unsigned*>(idx + o);
      Vec<T>::unpack(ok ? gq : make_uint4(0, 0, 0, 0), g[wy][wx]);
      tv[wy][wx] = ok ? t : ~0ull;
    }
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int iy = 2 * a + r, ix = 2 * b + c;
      if (iy >= H || ix >= W) continue;
      float acc[E];
#pragma unroll
      for (int e = 0; e < E; ++e) acc[e] = 0.f;
#pragma unroll
      for (int wy = 0; wy < 2; ++wy) {
        if (r == 0 && wy == 1) continue;   // even row: window row a only (tap row 1)
        const unsigned ty = r == 0 ? 1u : (wy == 0 ? 2u : 0u);
#pragma unroll
        for (int wx = 0; wx < 2; ++wx) {
          if (c == 0 && wx == 1) continue;
          const unsigned tap = ty * 3 + (c == 0 ? 1u : (wx == 0 ? 2u : 0u));
#pragma unroll
          for (int e = 0; e < E; ++e)
            if (((tv[wy][wx] >> (8 * e)) & 0xffu) == tap) acc[e] += g[wy][wx][e];
        }
      }
      *reinterpret_cast<uint4*>(gx + ((static_cast<size_t>(n) * H + iy) * W + ix) * C + ch * E) = Vec<T>::pack(acc);
    }
}

// Training stem (round 5): a = relu(z * scale[seg] + shift[seg]) rounded to the dtype, its 3x3 /
// s2 / p1 max-pool (maxpool_kernel's fmaxf over the window) and the argmax tap per output element
// (maxpool_argmax_kernel's rule: the first maximum in window scan order, NaN taken) in one pass
// over z, without writing a: the backward takes the taps (maxpool_bwd_kernel) and its ReLU mask
// from z.  Replaces bn_apply + maxpool + the backward's argmax pass (1.17 GB -> 0.37 GB per step
// at the training stem's 128 x 128 x 128 x 64).
template <typename T>
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(const T* __restrict__ z, int N, int nimg, int H, int W,
                                                              int C, int Ho, int Wo, const float* __restrict__ scale,
                                                              const float* __restrict__ shift, T* __restrict__ y,
                                                              uint8_t* __restrict__ idx) {
  constexpr int E = Vec<T>::E;
  const int chunks = C / E;
  const long long total = static_cast<long long>(N) * Ho * Wo * chunks;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const int ox = static_cast<int>(pix % Wo);
    const long long t = pix / Wo;
    const int oy = static_cast<int>(t % Ho);
    const long long n = t / Ho;
    const int seg = static_cast<int>(n / nimg);
    float sc[E], sh[E], m[E], bm[E];
    int am[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      sc[e] = scale[seg * C + ch * E + e];
      sh[e] = shift[seg * C + ch * E + e];
      m[e] = -INFINITY;
      bm[e] = 0.f;
      am[e] = -1;
    }
    for (int tap = 0; tap < 9; ++tap) {
      const int dy = tap / 3, dx = tap - 3 * dy;
      const int iy = oy * 2 - 1 + dy, ix = ox * 2 - 1 + dx;
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
      float v[E];
      Vec<T>::unpack(*reinterpret_cast<const uint4*>(z + ((n * H + iy) * W + ix) * C + ch * E), v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float tv = v[e] * sc[e] + sh[e];   // bn_apply's expression
        v[e] = fmaxf(tv, 0.f);
      }
      Vec<T>::unpack(Vec<T>::pack(v), v);        // rounded like the stored activation
#pragma unroll
      for (int e = 0; e < E; ++e) {
        m[e] = fmaxf(m[e], v[e]);
        const bool take = am[e] < 0 || v[e] > bm[e] || v[e] != v[e];
        bm[e] = take ? v[e] : bm[e];
        am[e] = take ? tap : am[e];
      }
    }
    *reinterpret_cast<uint4*>(y + pix * C + ch * E) = Vec<T>::pack(m);
    uint8_t* dst = idx + pix * C + ch * E;
#pragma unroll
    for (int e = 0; e < E; ++e) dst[e] = static_cast<uint8_t>(am[e]);
  }
}

inline int grid_for(long long total) {
  long long g = (total + 255) / 256;
  return static_cast<int>(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

int chunk_elems(int dtype) { return dtype == POSU_F32 ? 4 : 8; }

// the block reduction pairs pixel lanes in powers of two
bool reducible(int C, int dtype) {
  const int cpr = C / chunk_elems(dtype);
  return cpr >= 256 ? cpr % 256 == 0 : ilog2(cpr) >= 0;
}

template <typename T>
void pool_bwd_launch(const uint8_t* idx, const T* gy, int N, int H, int W, int C, int Ho, int Wo, T* gx,
                     hipStream_t s) {
  const long long quads = static_cast<long long>(N) * ((H + 1) / 2) * ((W + 1) / 2) * (C / Vec<T>::E);
  if (POSU_POOL_BWD2 && quads < (1LL << 31) - 256) {
    hipLaunchKernelGGL(maxpool_bwd2_kernel<T>, dim3(static_cast<unsigned>((quads + 255) / 256)), dim3(256), 0, s, idx,
                       gy, N, H, W, C, Ho, Wo, gx);
    return;
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel<T>, dim3(grid_for(static_cast<long long>(N) * H * W * C / Vec<T>::E)),
                     dim3(256), 0, s, idx, gy, N, H, W, C, Ho, Wo, gx);
}

long long partial_bytes(int nseg, int C) { return static_cast<long long>(nseg) * kMaxNB * 2 * C * 8; }

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" long long posu_bn_workspace(int nseg, int C) {
  return partial_bytes(nseg, C) + static_cast<long long>(nseg) * 3 * C * 4;
}

extern "C" int posu_bn_train_fwd(int dtype, const void* z, int nseg, int Pseg, int C, const float* gamma,
                                 const float* beta, float eps, float momentum, float* running_mean,
                                 float* running_var, float* mean, float* rstd, float* scale, float* shift,
                                 void* workspace, long long workspace_bytes, void* stream) {
  POSU_REQUIRE(z && mean && rstd && scale && shift && workspace, "posu_bn_train_fwd: null pointer");
  POSU_REQUIRE(nseg > 0 && Pseg > 0 && C > 0 && C % chunk_elems(dtype) == 0 && reducible(C, dtype),
               "posu_bn_train_fwd: bad shape (C / chunk must be a power of two or a multiple of 256)");
  POSU_REQUIRE(workspace_bytes >= posu_bn_workspace(nseg, C), "posu_bn_train_fwd: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  // the per-segment shifts K live where the backward keeps its coefficients
  float* kshift = reinterpret_cast<float*>(static_cast<char*>(workspace) + partial_bytes(nseg, C));
  const RedShape rs = red_shape(Pseg, C, chunk_elems(dtype), nseg);
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((bn_partial_kernel<T, 0>), dim3(rs.NB, rs.CG, nseg), dim3(256), 0, s,
                       static_cast<const T*>(z), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, Pseg, C, rs, part,
                       kshift, nullptr);
  });
  POSU_REQUIRE(ok, "posu_bn_train_fwd: unsupported dtype");
  if (POSU_BN_FIN2)
    hipLaunchKernelGGL(bn_stats_finalize2_kernel, dim3((C + FC2 - 1) / FC2), dim3(256), 0, s, part, nseg, rs.NB, Pseg,
                       C, gamma, beta, eps, momentum, kshift, running_mean, running_var, mean, rstd, scale, shift);
  else
    hipLaunchKernelGGL(bn_stats_finalize_kernel, dim3((C + FCH - 1) / FCH), dim3(256), 0, s, part, nseg, rs.NB, Pseg,
                       C, gamma, beta, eps, momentum, kshift, running_mean, running_var, mean, rstd, scale, shift);
  return check_launch("posu_bn_train_fwd");
}

namespace {
int bn_apply_impl(const char* name, int dtype, const void* z, int nseg, int Pseg, int C, const float* scale,
                  const float* shift, const void* residual, int relu, void* y, void* mask, void* stream) {
  const std::string what = name;
  POSU_REQUIRE(z && scale && shift && y, what + ": null pointer");
  POSU_REQUIRE(nseg > 0 && Pseg > 0 && C > 0 && C % chunk_elems(dtype) == 0, what + ": bad shape");
  hipStream_t s = as_stream(stream);
  const long long total = static_cast<long long>(nseg) * Pseg * C / chunk_elems(dtype);
  const int E = chunk_elems(dtype);
  uint8_t* mk = static_cast<uint8_t*>(mask);
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    if (seg_major(C, E, nseg, Pseg, {scale, shift})) {
      hipLaunchKernelGGL(bn_apply_seg_kernel<T>, dim3(seg_blocks(Pseg, C, E, nseg), nseg), dim3(256), 0, s,
                         static_cast<const T*>(z), Pseg, C, scale, shift, static_cast<const T*>(residual), relu,
                         static_cast<T*>(y), mk);
      return;
    }
    hipLaunchKernelGGL(bn_apply_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, static_cast<const T*>(z), Pseg,
                       C, scale, shift, static_cast<const T*>(residual), relu, static_cast<T*>(y), total, mk);
  });
  POSU_REQUIRE(ok, what + ": unsupported dtype");
  return check_launch(name);
}

int bn_bwd_impl(const char* name, int dtype, const void* gy, const void* y, const void* ymask,
                const float* relu_scale, const float* relu_shift, const void* z, int nseg, int Pseg, int C,
                const float* mean, const float* rstd, const float* gamma, float* dgamma, float* dbeta, void* dz,
                void* gres, void* workspace, long long workspace_bytes, void* stream) {
  const std::string what = name;
  POSU_REQUIRE(gy && z && mean && rstd && dz && workspace, what + ": null pointer");
  POSU_REQUIRE(nseg > 0 && Pseg > 0 && C > 0 && C % chunk_elems(dtype) == 0 && reducible(C, dtype),
               what + ": bad shape (C / chunk must be a power of two or a multiple of 256)");
  POSU_REQUIRE(workspace_bytes >= posu_bn_workspace(nseg, C), what + ": workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  float* coef = reinterpret_cast<float*>(static_cast<char*>(workspace) + partial_bytes(nseg, C));
  const RedShape rs = red_shape(Pseg, C, chunk_elems(dtype), nseg);
  const long long total = static_cast<long long>(nseg) * Pseg * C / chunk_elems(dtype);
  const uint8_t* ym = static_cast<const uint8_t*>(ymask);
  bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((bn_partial_kernel<T, 1>), dim3(rs.NB, rs.CG, nseg), dim3(256), 0, s,
                       static_cast<const T*>(z), static_cast<const T*>(gy), static_cast<const T*>(y), relu_scale,
                       relu_shift, mean, rstd, Pseg, C, rs, part, nullptr, ym);
  });
  POSU_REQUIRE(ok, what + ": unsupported dtype");
  if (POSU_BN_FIN2)
    hipLaunchKernelGGL(bn_bwd_finalize2_kernel, dim3((C + FC2 - 1) / FC2), dim3(256), 0, s, part, nseg, rs.NB, Pseg, C,
                       gamma, rstd, coef, dgamma, dbeta);
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + FCH - 1) / FCH), dim3(256), 0, s, part, nseg, rs.NB, Pseg, C,
                       gamma, rstd, coef, dgamma, dbeta);
  with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    const int E = chunk_elems(dtype);
    if (seg_major(C, E, nseg, Pseg, {mean, rstd, coef, relu_scale, relu_shift})) {
      hipLaunchKernelGGL(bn_bwd_apply_seg_kernel<T>, dim3(seg_blocks(Pseg, C, E, nseg), nseg), dim3(256), 0, s,
                         static_cast<const T*>(gy), static_cast<const T*>(y), relu_scale, relu_shift,
                         static_cast<const T*>(z), Pseg, C, mean, rstd, coef, static_cast<T*>(dz),
                         static_cast<T*>(gres), ym);
      return;
    }
    hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, static_cast<const T*>(gy),
                       static_cast<const T*>(y), relu_scale, relu_shift, static_cast<const T*>(z), Pseg, C, mean, rstd, coef,
                       static_cast<T*>(dz), static_cast<T*>(gres), total, ym);
  });
  return check_launch(name);
}
}  // namespace

extern "C" int posu_bn_apply(int dtype, const void* z, int nseg, int Pseg, int C, const float* scale,
                             const float* shift, const void* residual, int relu, void* y, void* stream) {
  return bn_apply_impl("posu_bn_apply", dtype, z, nseg, Pseg, C, scale, shift, residual, relu, y, nullptr, stream);
}

extern "C" int posu_bn_apply_mask(int dtype, const void* z, int nseg, int Pseg, int C, const float* scale,
                                  const float* shift, const void* residual, void* y, void* mask, void* stream) {
  POSU_REQUIRE(mask, "posu_bn_apply_mask: null pointer (mask)");
  POSU_REQUIRE(mask != y && mask != z && mask != residual, "posu_bn_apply_mask: the mask must not alias a tensor");
  return bn_apply_impl("posu_bn_apply_mask", dtype, z, nseg, Pseg, C, scale, shift, residual, 1, y, mask, stream);
}

extern "C" int posu_bn_train_bwd(int dtype, const void* gy, const void* y, const float* relu_scale,
                                 const float* relu_shift, const void* z, int nseg, int Pseg, int C,
                                 const float* mean, const float* rstd, const float* gamma, float* dgamma,
                                 float* dbeta, void* dz, void* gres, void* workspace, long long workspace_bytes,
                                 void* stream) {
  return bn_bwd_impl("posu_bn_train_bwd", dtype, gy, y, nullptr, relu_scale, relu_shift, z, nseg, Pseg, C, mean,
                     rstd, gamma, dgamma, dbeta, dz, gres, workspace, workspace_bytes, stream);
}

extern "C" int posu_bn_train_bwd_mask(int dtype, const void* gy, const void* mask, const void* z, int nseg, int Pseg,
                                      int C, const float* mean, const float* rstd, const float* gamma, float* dgamma,
                                      float* dbeta, void* dz, void* gres, void* workspace, long long workspace_bytes,
                                      void* stream) {
  POSU_REQUIRE(mask, "posu_bn_train_bwd_mask: null pointer (mask)");
  return bn_bwd_impl("posu_bn_train_bwd_mask", dtype, gy, nullptr, mask, nullptr, nullptr, z, nseg, Pseg, C, mean,
                     rstd, gamma, dgamma, dbeta, dz, gres, workspace, workspace_bytes, stream);
}

extern "C" int posu_channel_sum(int dtype, const void* x, int P, int C, float* out, void* workspace,
                                long long workspace_bytes, void* stream) {
  POSU_REQUIRE(x && out && workspace, "posu_channel_sum: null pointer");
  POSU_REQUIRE(P > 0 && C > 0 && C % chunk_elems(dtype) == 0 && reducible(C, dtype),
               "posu_channel_sum: bad shape (C / chunk must be a power of two or a multiple of 256)");
  POSU_REQUIRE(workspace_bytes >= posu_bn_workspace(1, C), "posu_channel_sum: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  const RedShape rs = red_shape(P, C, chunk_elems(dtype), 1);
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL((bn_partial_kernel<T, 0>), dim3(rs.NB, rs.CG, 1), dim3(256), 0, s, static_cast<const T*>(x),
                       nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, P, C, rs, part, nullptr, nullptr);
  });
  POSU_REQUIRE(ok, "posu_channel_sum: unsupported dtype");
  if (POSU_BN_FIN2)
    hipLaunchKernelGGL(channel_sum_finalize2_kernel, dim3((C + FC2 - 1) / FC2), dim3(256), 0, s, part, rs.NB, C, out);
  else
    hipLaunchKernelGGL(channel_sum_finalize_kernel, dim3((C + FCH - 1) / FCH), dim3(256), 0, s, part, rs.NB, C, out);
  return check_launch("posu_channel_sum");
}

extern "C" long long posu_maxpool3x3s2_bwd_workspace(int N, int H, int W, int C) {
  const long long Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  return N * Ho * Wo * C;
}

extern "C" int posu_maxpool3x3s2_bwd(int dtype, const void* x, int N, int H, int W, int C, const void* gy, void* gx,
                                     void* workspace, long long workspace_bytes, void* stream) {
  POSU_REQUIRE(x && gy && gx && workspace, "posu_maxpool3x3s2_bwd: null pointer");
  POSU_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % chunk_elems(dtype) == 0, "posu_maxpool3x3s2_bwd: bad shape");
  POSU_REQUIRE(workspace_bytes >= posu_maxpool3x3s2_bwd_workspace(N, H, W, C),
               "posu_maxpool3x3s2_bwd: workspace too small");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipStream_t s = as_stream(stream);
  uint8_t* idx = static_cast<uint8_t*>(workspace);
  const int E = chunk_elems(dtype);
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(maxpool_argmax_kernel<T>, dim3(grid_for(static_cast<long long>(N) * Ho * Wo * C / E)),
                       dim3(256), 0, s, static_cast<const T*>(x), N, H, W, C, Ho, Wo, idx);
    pool_bwd_launch<T>(idx, static_cast<const T*>(gy), N, H, W, C, Ho, Wo, static_cast<T*>(gx), s);
  });
  POSU_REQUIRE(ok, "posu_maxpool3x3s2_bwd: unsupported dtype");
  return check_launch("posu_maxpool3x3s2_bwd");
}

extern "C" int posu_bn_relu_maxpool3x3s2_fwd(int dtype, const void* z, int nseg, int N, int H, int W, int C,
                                             const float* scale, const float* shift, void* y, void* idx,
                                             void* stream) {
  POSU_REQUIRE(z && scale && shift && y && idx, "posu_bn_relu_maxpool3x3s2_fwd: null pointer");
  POSU_REQUIRE(nseg > 0 && N > 0 && N % nseg == 0 && H > 0 && W > 0 && C > 0 && C % chunk_elems(dtype) == 0,
               "posu_bn_relu_maxpool3x3s2_fwd: bad shape (N a multiple of nseg, C of the 16-B chunk)");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipStream_t s = as_stream(stream);
  const int E = chunk_elems(dtype);
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(bn_relu_maxpool_kernel<T>, dim3(grid_for(static_cast<long long>(N) * Ho * Wo * C / E)),
                       dim3(256), 0, s, static_cast<const T*>(z), N, N / nseg, H, W, C, Ho, Wo, scale, shift,
                       static_cast<T*>(y), static_cast<uint8_t*>(idx));
  });
  POSU_REQUIRE(ok, "posu_bn_relu_maxpool3x3s2_fwd: unsupported dtype");
  return check_launch("posu_bn_relu_maxpool3x3s2_fwd");
}

extern "C" int posu_maxpool3x3s2_bwd_idx(int dtype, const void* idx, const void* gy, int N, int H, int W, int C,
                                         void* gx, void* stream) {
  POSU_REQUIRE(idx && gy && gx, "posu_maxpool3x3s2_bwd_idx: null pointer");
  POSU_REQUIRE((reinterpret_cast<size_t>(idx) & 7) == 0, "posu_maxpool3x3s2_bwd_idx: idx must be 8-byte aligned");
  POSU_REQUIRE(N > 0 && H > 0 && W > 0 && C > 0 && C % chunk_elems(dtype) == 0, "posu_maxpool3x3s2_bwd_idx: bad shape");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipStream_t s = as_stream(stream);
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    pool_bwd_launch<T>(static_cast<const uint8_t*>(idx), static_cast<const T*>(gy), N, H, W, C, Ho, Wo,
                       static_cast<T*>(gx), s);
  });
  POSU_REQUIRE(ok, "posu_maxpool3x3s2_bwd_idx: unsupported dtype");
  return check_launch("posu_maxpool3x3s2_bwd_idx");
}
