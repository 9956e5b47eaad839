// Heatmap -> joint coordinate kernels.  One wave64 per (sample, joint) map; the
// map is streamed once with float4 loads and reduced in registers + wave shuffles
// (no MFMA: this is an HBM/latency-bound reduction, 16 KiB per 64x64 map).
//
//   soft-argmax fwd : online softmax (running max / rescaled sums) of beta*h,
//                     x = sum p*col, y = sum p*row, then the crop affine
//                     (generate_integral_preds_2d_th + transform_back_th,
//                     lib/utils/transforms.py:149-198)
//   soft-argmax bwd : dh = beta p ((col-x) gx + (row-y) gy)
//   argmax          : get_max_preds + get_final_preds post-process + transform_preds
//                     (lib/core/inference.py:19-75)
#include "posu_common.h"

namespace posu {
namespace {

__device__ __forceinline__ void online_add(float t, float col, float row, float& m, float& s, float& sx,
                                           float& sy) {
  if (t > m) {
    const float sc = __expf(m - t);
    s *= sc;
    sx *= sc;
    sy *= sc;
    m = t;
  }
  const float e = __expf(t - m);
  s += e;
  sx += e * col;
  sy += e * row;
}

// one 64-lane block per map (round 5: was four maps per 256-thread block -- NJ / 4 blocks, half the
// CUs idle at the training step's 512 maps; the per-map arithmetic is unchanged)
__global__ __launch_bounds__(64) void softargmax_fwd_kernel(const float* __restrict__ hm, int NJ, int J, int H,
                                                            int W, float beta, const float* __restrict__ aff,
                                                            float* __restrict__ out, float* __restrict__ stats) {
  const int map = blockIdx.x;
  const int lane = threadIdx.x;
  if (map >= NJ) return;
  const int HW = H * W;
  const float* h = hm + static_cast<size_t>(map) * HW;
  float m = -INFINITY, s = 0.f, sx = 0.f, sy = 0.f;
  if ((HW & 3) == 0 && (W & 3) == 0) {
    const float4* h4 = reinterpret_cast<const float4*>(h);
    for (int i = lane; i < HW / 4; i += 64) {
      const float4 v = h4[i];
      const int idx = i * 4;
      const int row = idx / W, col = idx - row * W;
      online_add(beta * v.x, col + 0.f, row, m, s, sx, sy);
      online_add(beta * v.y, col + 1.f, row, m, s, sx, sy);
      online_add(beta * v.z, col + 2.f, row, m, s, sx, sy);
      online_add(beta * v.w, col + 3.f, row, m, s, sx, sy);
    }
  } else {
    for (int i = lane; i < HW; i += 64) {
      const int row = i / W, col = i - row * W;
      online_add(beta * h[i], col, row, m, s, sx, sy);
    }
  }
  // combine lanes: rescale each lane's sums to the wave max
  const float M = wave_max(m);
  const float sc = (m == -INFINITY) ? 0.f : __expf(m - M);
  s = wave_sum(s * sc);
  sx = wave_sum(sx * sc);
  sy = wave_sum(sy * sc);
  if (lane == 0) {
    const float x = sx / s, y = sy / s;
    float ox = x, oy = y;
    if (aff) {
      const float* T = aff + static_cast<size_t>(map / J) * 6;
      ox = x * T[0] + y * T[1] + T[2];
      oy = x * T[3] + y * T[4] + T[5];
    }
    out[2 * map] = ox;
    out[2 * map + 1] = oy;
    if (stats) {
      stats[4 * map] = M;
      stats[4 * map + 1] = s;
      stats[4 * map + 2] = x;
      stats[4 * map + 3] = y;
    }
  }
}

__global__ __launch_bounds__(64) void softargmax_bwd_kernel(const float* __restrict__ hm,
                                                            const float* __restrict__ stats, int NJ, int J,
                                                            int H, int W, float beta,
                                                            const float* __restrict__ aff,
                                                            const float* __restrict__ gout,
                                                            float* __restrict__ ghm) {
  const int map = blockIdx.x;
  const int lane = threadIdx.x;
  if (map >= NJ) return;
  const int HW = H * W;
  const float M = stats[4 * map], inv_s = 1.f / stats[4 * map + 1];
  const float x = stats[4 * map + 2], y = stats[4 * map + 3];
  float gx = gout[2 * map], gy = gout[2 * map + 1];
  if (aff) {  // chain through [x, y, 1] @ T^T
    const float* T = aff + static_cast<size_t>(map / J) * 6;
    const float ax = gx * T[0] + gy * T[3];
    const float ay = gx * T[1] + gy * T[4];
    gx = ax;
    gy = ay;
  }
  const float* h = hm + static_cast<size_t>(map) * HW;
  float* gh = ghm + static_cast<size_t>(map) * HW;
  auto one = [&](float hv, int row, int col) {
    const float p = __expf(beta * hv - M) * inv_s;
    return beta * p * ((col - x) * gx + (row - y) * gy);
  };
  // 16-B loads / stores (the same per-element arithmetic) when both maps are 16-B aligned: a view with
  // a storage offset that is not a multiple of 4 floats takes the scalar loop
  if ((HW & 3) == 0 && (W & 3) == 0 && ((reinterpret_cast<size_t>(h) | reinterpret_cast<size_t>(gh)) & 15) == 0) {
    const float4* h4 = reinterpret_cast<const float4*>(h);
    float4* g4 = reinterpret_cast<float4*>(gh);
#pragma unroll 4
    for (int i = lane; i < HW / 4; i += 64) {
      const float4 v = h4[i];
      const int row = (i * 4) / W, col = i * 4 - row * W;
      g4[i] = make_float4(one(v.x, row, col), one(v.y, row, col + 1), one(v.z, row, col + 2), one(v.w, row, col + 3));
    }
    return;
  }
  for (int i = lane; i < HW; i += 64) {
    const int row = i / W, col = i - row * W;
    gh[i] = one(h[i], row, col);
  }
}

__global__ __launch_bounds__(256) void argmax_kernel(const float* __restrict__ hm, int NJ, int J, int H, int W,
                                                     int post, const double* __restrict__ aff,
                                                     float* __restrict__ preds, float* __restrict__ maxvals) {
  const int map = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (map >= NJ) return;
  const int HW = H * W;
  const float* h = hm + static_cast<size_t>(map) * HW;
  float best = -INFINITY;
  int bidx = 0x7fffffff;
  for (int i = lane; i < HW; i += 64) {
    const float v = h[i];
    if (v > best) {  // strict: the first (smallest) index of a tie within the lane
      best = v;
      bidx = i;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bidx, o, 64);
    if (ov > best || (ov == best && oi < bidx)) {
      best = ov;
      bidx = oi;
    }
  }
  if (lane == 0) {
    if (bidx == 0x7fffffff) bidx = 0;  // all -inf / NaN map
    float px = static_cast<float>(bidx % W);
    float py = floorf(static_cast<float>(bidx) / W);
    if (!(best > 0.f)) {
      px = 0.f;
      py = 0.f;
    }
    if (post) {
      const int ix = static_cast<int>(floorf(px + 0.5f)), iy = static_cast<int>(floorf(py + 0.5f));
      if (1 < ix && ix < W - 1 && 1 < iy && iy < H - 1) {
        const float dx = h[iy * W + ix + 1] - h[iy * W + ix - 1];
        const float dy = h[(iy + 1) * W + ix] - h[(iy - 1) * W + ix];
        px += (dx > 0.f ? 0.25f : (dx < 0.f ? -0.25f : 0.f));
        py += (dy > 0.f ? 0.25f : (dy < 0.f ? -0.25f : 0.f));
      }
    }
    float ox = px, oy = py;
    if (aff) {
      const double* T = aff + static_cast<size_t>(map / J) * 6;
      ox = static_cast<float>(static_cast<double>(px) * T[0] + static_cast<double>(py) * T[1] + T[2]);
      oy = static_cast<float>(static_cast<double>(px) * T[3] + static_cast<double>(py) * T[4] + T[5]);
    }
    preds[2 * map] = ox;
    preds[2 * map + 1] = oy;
    maxvals[map] = best;
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_softargmax2d_fwd(const float* hm, int N, int J, int H, int W, float beta, const float* affine,
                                     float* out, float* stats, void* stream) {
  POSU_REQUIRE(hm && out, "posu_softargmax2d_fwd: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0 && H > 0 && W > 0, "posu_softargmax2d_fwd: bad shape");
  if (N == 0) return POSU_OK;
  const int NJ = N * J;
  hipLaunchKernelGGL(softargmax_fwd_kernel, dim3(NJ), dim3(64), 0, as_stream(stream), hm, NJ, J, H, W,
                     beta, affine, out, stats);
  return check_launch("posu_softargmax2d_fwd");
}

extern "C" int posu_softargmax2d_bwd(const float* hm, const float* stats, int N, int J, int H, int W, float beta,
                                     const float* affine, const float* gout, float* ghm, void* stream) {
  POSU_REQUIRE(hm && stats && gout && ghm, "posu_softargmax2d_bwd: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0 && H > 0 && W > 0, "posu_softargmax2d_bwd: bad shape");
  if (N == 0) return POSU_OK;
  const int NJ = N * J;
  hipLaunchKernelGGL(softargmax_bwd_kernel, dim3(NJ), dim3(64), 0, as_stream(stream), hm, stats, NJ,
                     J, H, W, beta, affine, gout, ghm);
  return check_launch("posu_softargmax2d_bwd");
}

extern "C" int posu_argmax2d_fwd(const float* hm, int N, int J, int H, int W, int post_process,
                                 const double* affine, float* preds, float* maxvals, void* stream) {
  POSU_REQUIRE(hm && preds && maxvals, "posu_argmax2d_fwd: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0 && H > 0 && W > 0, "posu_argmax2d_fwd: bad shape");
  if (N == 0) return POSU_OK;
  const int NJ = N * J;
  hipLaunchKernelGGL(argmax_kernel, dim3((NJ + 3) / 4), dim3(256), 0, as_stream(stream), hm, NJ, J, H, W,
                     post_process, affine, preds, maxvals);
  return check_launch("posu_argmax2d_fwd");
}

// ------------------------------------------------------------ JointsMSELoss
namespace posu {
namespace {

// one 64-lane block per heatmap: 16-B loads, four independent partial sums per lane (a fixed
// association: lane l adds elements 4l.., chunk j into sum j % 4), then the wave sum.  (Round 2 ran
// a wave per map at four maps per block with 4-B loads: 128 blocks, 28 us per call for 32 x 16
// maps of 64 x 64 -- latency-bound on half the CUs.)
__global__ __launch_bounds__(64) void mse_partial_kernel(const float* __restrict__ pred,
                                                         const float* __restrict__ gt,
                                                         const float* __restrict__ w, int NJ, int HW,
                                                         float* __restrict__ ws) {
  const int map = blockIdx.x;
  const int lane = threadIdx.x;
  const float* p = pred + static_cast<size_t>(map) * HW;
  const float* t = gt + static_cast<size_t>(map) * HW;
  const float wt = w ? w[map] : 1.f;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if ((HW & 3) == 0 && ((reinterpret_cast<size_t>(p) | reinterpret_cast<size_t>(t)) & 15) == 0) {
    const int n4 = HW >> 2;
#pragma unroll 4
    for (int j = lane; j < n4; j += 64) {
      const float4 a = reinterpret_cast<const float4*>(p)[j], b = reinterpret_cast<const float4*>(t)[j];
      const float d0 = a.x * wt - b.x * wt, d1 = a.y * wt - b.y * wt, d2 = a.z * wt - b.z * wt,
                  d3 = a.w * wt - b.w * wt;
      acc[(j >> 6) & 3] += (d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3);
    }
  } else {
    for (int i = lane; i < HW; i += 64) {
      const float d = p[i] * wt - t[i] * wt;
      acc[(i >> 6) & 3] += d * d;
    }
  }
  const float s = wave_sum((acc[0] + acc[1]) + (acc[2] + acc[3]));
  if (lane == 0) ws[map] = s;
}

__global__ __launch_bounds__(256) void mse_final_kernel(const float* __restrict__ ws, int NJ, float denom,
                                                        float* __restrict__ loss) {
  __shared__ float part[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < NJ; i += 256) acc += ws[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) loss[0] = ((part[0] + part[1]) + (part[2] + part[3])) / denom;
}

__global__ __launch_bounds__(256) void mse_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ gt,
                                                      const float* __restrict__ w, int NJ, int HW,
                                                      const float* __restrict__ gloss, float denom,
                                                      float* __restrict__ gpred) {
  const long long total = static_cast<long long>(NJ) * HW;
  const float g = 2.f * gloss[0] / denom;
  if (total < (1LL << 31)) {   // 32-bit index math (the map of element i: an unsigned 32-bit division)
    const unsigned tot = static_cast<unsigned>(total), hw = static_cast<unsigned>(HW);
    for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < tot; i += gridDim.x * 256u) {
      const float wt = w ? w[i / hw] : 1.f;
      gpred[i] = g * wt * (pred[i] * wt - gt[i] * wt);
    }
    return;
  }
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int map = static_cast<int>(i / HW);
    const float wt = w ? w[map] : 1.f;
    gpred[i] = g * wt * (pred[i] * wt - gt[i] * wt);
  }
}

}  // namespace
}  // namespace posu

extern "C" int posu_joints_mse_fwd(const float* pred, const float* gt, const float* w, int N, int J, int HW,
                                   float* ws, float* loss, void* stream) {
  POSU_REQUIRE(pred && gt && ws && loss, "posu_joints_mse_fwd: null pointer");
  POSU_REQUIRE(N > 0 && J > 0 && HW > 0, "posu_joints_mse_fwd: bad shape");
  const int NJ = N * J;
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(mse_partial_kernel, dim3(NJ), dim3(64), 0, s, pred, gt, w, NJ, HW, ws);
  hipLaunchKernelGGL(mse_final_kernel, dim3(1), dim3(256), 0, s, ws, NJ,
                     static_cast<float>(static_cast<long long>(N) * HW), loss);
  return check_launch("posu_joints_mse_fwd");
}

extern "C" int posu_joints_mse_bwd(const float* pred, const float* gt, const float* w, int N, int J, int HW,
                                   const float* gloss, float* gpred, void* stream) {
  POSU_REQUIRE(pred && gt && gloss && gpred, "posu_joints_mse_bwd: null pointer");
  POSU_REQUIRE(N > 0 && J > 0 && HW > 0, "posu_joints_mse_bwd: bad shape");
  const long long total = static_cast<long long>(N) * J * HW;
  long long grid = (total + 255) / 256;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(mse_bwd_kernel, dim3(static_cast<int>(grid)), dim3(256), 0, as_stream(stream), pred, gt, w,
                     N * J, HW, gloss, static_cast<float>(static_cast<long long>(N) * HW), gpred);
  return check_launch("posu_joints_mse_bwd");
}

// ---------------------------------------------------------------- flip test
namespace posu {
namespace {

// out[n][j][y][x] = (avg ? 0.5 * (hm[n][j][y][x] + F) : F),
// F = hf[n][perm[j]][y][W-1-xs], xs = shift ? max(x-1, 0) : x
// (flip_back_th transforms.py:33-47 + SHIFT_HEATMAP function.py:579-582 + the average
// of function.py:583), one thread per heatmap element.
__global__ __launch_bounds__(256) void flip_back_kernel(const float* __restrict__ hf, const int* __restrict__ perm,
                                                        const float* __restrict__ hm, int N, int J, int H, int W,
                                                        int shift, float* __restrict__ out) {
  const long long total = static_cast<long long>(N) * J * H * W;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int x = static_cast<int>(i % W);
    const long long r = i / W;
    const int y = static_cast<int>(r % H);
    const long long nj = r / H;
    const int j = static_cast<int>(nj % J);
    const long long n = nj / J;
    const int xs = shift ? (x > 0 ? x - 1 : 0) : x;
    const int js = perm ? perm[j] : j;
    const float f = hf[((n * J + js) * H + y) * W + (W - 1 - xs)];
    out[i] = hm ? 0.5f * (hm[i] + f) : f;
  }
}

}  // namespace
}  // namespace posu

extern "C" int posu_flip_back(const float* hm_flipped, const int* perm, const float* hm, int N, int J, int H, int W,
                              int shift, float* out, void* stream) {
  POSU_REQUIRE(hm_flipped && out, "posu_flip_back: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0 && H > 0 && W > 0, "posu_flip_back: bad shape");
  POSU_REQUIRE(out != hm_flipped, "posu_flip_back: out must not alias the flipped heatmaps");
  if (N == 0) return POSU_OK;
  const long long total = static_cast<long long>(N) * J * H * W;
  const long long blocks = std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(flip_back_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, as_stream(stream),
                     hm_flipped, perm, hm, N, J, H, W, shift, out);
  return check_launch("posu_flip_back");
}
