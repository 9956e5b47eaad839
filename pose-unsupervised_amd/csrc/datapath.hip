// Data-path kernels around the network:
//   gaussian targets : JointsDatasetCompatible.generate_heatmap
//                      (lib/dataset/joints_dataset_compatible.py:215-253) for a whole batch,
//                      one thread per target pixel;
//   integral decode  : the sum-normalised integral coordinates of
//                      run/test/test_integral.py:63-70, one wave per map.
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
