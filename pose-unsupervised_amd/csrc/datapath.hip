// Data-path kernels around the network:
//   gaussian targets : JointsDatasetCompatible.generate_heatmap
//                      (lib/dataset/joints_dataset_compatible.py:215-253) for a whole batch,
//                      one thread per target pixel;
//   integral decode  : the sum-normalised integral coordinates of
//                      run/test/test_integral.py:63-70, one wave per map;
//   crop warp        : JointsDatasetCompatible.__getitem__'s cv2.warpAffine (INTER_LINEAR,
//                      lib/dataset/joints_dataset_compatible.py:161-164) for a whole batch,
//                      optionally fused with ToTensor + Normalize, one thread per output pixel.
#include "posu_common.h"

namespace posu {
namespace {

// target[n][j][y][x] = g(x - ul_x, y - ul_y) inside the (2*3sigma+1)^2 patch around
// mu = int(joint / stride + 0.5) when the joint is visible and the patch touches the
// map; weight[n][j] = vis (0 when the patch lies outside the map, or for samples whose
// weights the caller zeroes: H36M without pseudo labels, joints_dataset_compatible.py
// :250-251).  g is evaluated in f32 as numpy does.
__global__ __launch_bounds__(256) void gaussian_targets_kernel(const float* __restrict__ joints,
                                                               const float* __restrict__ vis, int N, int J,
                                                               double stride_x, double stride_y, int hw, int hh,
                                                               double sigma, const unsigned char* __restrict__ zero_w,
                                                               float* __restrict__ target, float* __restrict__ weight) {
  const long long total = static_cast<long long>(N) * J * hh * hw;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int x = static_cast<int>(i % hw);
    const long long r = i / hw;
    const int y = static_cast<int>(r % hh);
    const long long nj = r / hh;
    const int n = static_cast<int>(nj / J);
    const double tmp = sigma * 3.0;
    // Python int(): truncation toward zero
    const int mu_x = static_cast<int>(trunc(static_cast<double>(joints[nj * 2]) / stride_x + 0.5));
    const int mu_y = static_cast<int>(trunc(static_cast<double>(joints[nj * 2 + 1]) / stride_y + 0.5));
    const int ul_x = static_cast<int>(trunc(mu_x - tmp)), ul_y = static_cast<int>(trunc(mu_y - tmp));
    const int br_x = static_cast<int>(trunc(mu_x + tmp + 1.0)), br_y = static_cast<int>(trunc(mu_y + tmp + 1.0));
    const bool outside = ul_x >= hw || ul_y >= hh || br_x < 0 || br_y < 0;
    const float v = outside ? 0.f : vis[nj];
    if (x == 0 && y == 0) weight[nj] = (zero_w && zero_w[n]) ? 0.f : v;
    float t = 0.f;
    if (v > 0.5f && x >= ul_x && x < br_x && y >= ul_y && y < br_y) {
      const double size = 2.0 * tmp + 1.0;
      const float c0 = static_cast<float>(floor(size / 2.0));  // x0 = y0 = size // 2
      const float dx = static_cast<float>(x - ul_x) - c0, dy = static_cast<float>(y - ul_y) - c0;
      const float den = static_cast<float>(2.0 * sigma * sigma);
      t = expf(-(dx * dx + dy * dy) / den);
    }
    target[i] = t;
  }
}

// coords[n][j] = (sum_x x * sum_y h, sum_y y * sum_x h) / sum h   (f32, as numpy does
// on the f32 h5 heatmaps; summation order differs)
__global__ __launch_bounds__(256) void integral_kernel(const float* __restrict__ hm, int NJ, int H, int W,
                                                       float* __restrict__ out) {
  const int map = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (map >= NJ) return;
  const float* h = hm + static_cast<size_t>(map) * H * W;
  float s = 0.f, sx = 0.f, sy = 0.f;
  for (int i = lane; i < H * W; i += 64) {
    const int row = i / W, col = i - row * W;
    const float v = h[i];
    s += v;
    sx += v * col;
    sy += v * row;
  }
  s = wave_sum(s);
  sx = wave_sum(sx);
  sy = wave_sum(sy);
  if (lane == 0) {
    out[2 * map] = sx / s;
    out[2 * map + 1] = sy / s;
  }
}

// OpenCV 3.4's warpAffine (imgwarp.cpp: WarpAffineInvoker + remapBilinear, 8-bit) restated:
// the src -> dst matrix inverted in double; source coordinates in 1/1024-px fixed point
// (cvRound = round half to even) with the row term and the column term rounded separately,
// reduced to 1/32 px; the 4 taps weighted by the exact-integer bilinear table (sum 32768);
// (sum + 2^14) >> 15.  Border: constant 0 -- a pixel whose 2x2 footprint misses the image is 0,
// a partly covered one takes 0 for the missing taps.  No FMA contraction anywhere: every
// double is rounded like OpenCV's separate multiplies and adds.
#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void crop_warp_kernel(const unsigned char* __restrict__ src,
                                                        const long long* __restrict__ src_off,
                                                        const int* __restrict__ src_hw, int C,
                                                        const double* __restrict__ Mall, int N, int dh, int dw,
                                                        int mode, const float* __restrict__ mean,
                                                        const float* __restrict__ stdv, void* __restrict__ out) {
  const long long total = static_cast<long long>(N) * dh * dw;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int x = static_cast<int>(i % dw);
    const long long r = i / dw;
    const int y = static_cast<int>(r % dh);
    const int n = static_cast<int>(r / dh);
    const double* Mi = Mall + 6 * n;
    double m0 = Mi[0], m1 = Mi[1], m2 = Mi[2], m3 = Mi[3], m4 = Mi[4], m5 = Mi[5];
    double D = m0 * m4 - m1 * m3;
    D = D != 0.0 ? 1.0 / D : 0.0;
    const double a11 = m4 * D, a22 = m0 * D;
    m0 = a11;
    m1 *= -D;
    m3 *= -D;
    m4 = a22;
    const double b1 = -m0 * m2 - m1 * m5;
    const double b2 = -m3 * m2 - m4 * m5;
    m2 = b1;
    m5 = b2;
    const int adelta = static_cast<int>(rint(m0 * x * 1024.0));
    const int bdelta = static_cast<int>(rint(m3 * x * 1024.0));
    const int X0 = static_cast<int>(rint((m1 * y + m2) * 1024.0)) + 16;
    const int Y0 = static_cast<int>(rint((m4 * y + m5) * 1024.0)) + 16;
    const int X = (X0 + adelta) >> 5, Y = (Y0 + bdelta) >> 5;
    const int sx = min(max(X >> 5, -32768), 32767), sy = min(max(Y >> 5, -32768), 32767);
    const int fx = X & 31, fy = Y & 31;
    const int w[4] = {(32 - fy) * (32 - fx) * 32, (32 - fy) * fx * 32, fy * (32 - fx) * 32, fy * fx * 32};
    const int H = src_hw[2 * n], W = src_hw[2 * n + 1];
    const unsigned char* S = src + src_off[n];
    const bool outside = sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0;
    for (int c = 0; c < C; ++c) {
      int v = 0;
      if (!outside) {
        int acc = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int tx = sx + (k & 1), ty = sy + (k >> 1);
          if (tx >= 0 && tx < W && ty >= 0 && ty < H)
            acc += static_cast<int>(S[(static_cast<long long>(ty) * W + tx) * C + c]) * w[k];
        }
        v = (acc + (1 << 14)) >> 15;
        v = v < 0 ? 0 : (v > 255 ? 255 : v);
      }
      if (mode == 0) {
        static_cast<unsigned char*>(out)[(r * dw + x) * C + c] = static_cast<unsigned char>(v);
      } else {
        const float t = static_cast<float>(v) / 255.f;
        static_cast<float*>(out)[((static_cast<long long>(n) * C + c) * dh + y) * dw + x] = (t - mean[c]) / stdv[c];
      }
    }
  }
}
#pragma clang fp contract(on)

inline int grid_for(long long total) {
  long long g = (total + 255) / 256;
  return static_cast<int>(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_gaussian_targets(const float* joints, const float* vis, int N, int J, int image_w, int image_h,
                                     int hm_w, int hm_h, double sigma, const unsigned char* zero_weight,
                                     float* target, float* weight, void* stream) {
  POSU_REQUIRE(joints && vis && target && weight, "posu_gaussian_targets: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0 && image_w > 0 && image_h > 0 && hm_w > 0 && hm_h > 0 && sigma > 0,
               "posu_gaussian_targets: bad shape");
  if (N == 0) return POSU_OK;
  const long long total = static_cast<long long>(N) * J * hm_h * hm_w;
  hipLaunchKernelGGL(gaussian_targets_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), joints, vis, N,
                     J, static_cast<double>(image_w) / hm_w, static_cast<double>(image_h) / hm_h, hm_w, hm_h, sigma,
                     zero_weight, target, weight);
  return check_launch("posu_gaussian_targets");
}

extern "C" int posu_integral2d_fwd(const float* hm, int N, int J, int H, int W, float* out, void* stream) {
  POSU_REQUIRE(hm && out, "posu_integral2d_fwd: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0 && H > 0 && W > 0, "posu_integral2d_fwd: bad shape");
  const int NJ = N * J;
  if (NJ == 0) return POSU_OK;
  hipLaunchKernelGGL(integral_kernel, dim3((NJ + 3) / 4), dim3(256), 0, as_stream(stream), hm, NJ, H, W, out);
  return check_launch("posu_integral2d_fwd");
}

extern "C" int posu_crop_warp(const unsigned char* src, const long long* src_off, const int* src_hw, int C,
                              const double* M, int N, int dh, int dw, int mode, const float* mean, const float* std,
                              void* out, void* stream) {
  POSU_REQUIRE(src && src_off && src_hw && M && out, "posu_crop_warp: null pointer");
  POSU_REQUIRE(N >= 0 && C > 0 && C <= 4 && dh > 0 && dw > 0, "posu_crop_warp: bad shape");
  POSU_REQUIRE(mode == 0 || mode == 1, "posu_crop_warp: mode must be 0 (uint8 HWC) or 1 (normalised f32 NCHW)");
  POSU_REQUIRE(mode == 0 || (mean && std), "posu_crop_warp: mode 1 needs mean and std");
  if (N == 0) return POSU_OK;
  const long long total = static_cast<long long>(N) * dh * dw;
  hipLaunchKernelGGL(crop_warp_kernel, dim3(grid_for(total)), dim3(256), 0, as_stream(stream), src, src_off, src_hw,
                     C, M, N, dh, dw, mode, mean, std, out);
  return check_launch("posu_crop_warp");
}
