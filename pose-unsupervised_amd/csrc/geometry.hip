// Multi-view geometry kernels: epipolar (fundamental-matrix) loss forward/backward
// and fp64 DLT triangulation.  Latency-bound, tiny working sets: no MFMA, no LDS
// tiling beyond the block reductions.
//
// Epipolar loss (FundamentalLoss.__call__, lib/core/loss.py:101-133): residual of
// ordered view pair p = (i, j) (itertools.permutations order, loss.py:123) at joint k
// of sample b is |x~_j^T F_{subj(b), i, j} x~_i| (loss.py:128), weighted by
// w_i * w_j when target weights are given (loss.py:129-130), summed and divided by
// N * P * J (loss.py:132).  One 256-thread block does the whole reduction in a fixed
// order, so the value is deterministic (no atomics).
//
// Triangulation (triangulate_poses -> pymvg MultiCameraSystem.find3d,
// lib/multiviews/triangulate.py:43-99): one thread per (group, joint); OpenCV-model
// fixed-point undistortion (5 iterations) of each visible view's pixel, two DLT rows
// per view, and the right singular vector of the smallest singular value from a
// one-sided (Hestenes) Jacobi SVD in fp64.
#include "posu_common.h"

namespace posu {
namespace {

__device__ __forceinline__ void pair_of(int p, int V, int& i, int& j) {
  // permutations(range(V), 2): i major, j over the remaining views ascending
  i = p / (V - 1);
  const int r = p - i * (V - 1);
  j = r < i ? r : r + 1;
}

// signed epipolar residual x~_j^T F x~_i  (row vector h_j times F, dotted with h_i)
__device__ __forceinline__ float epi_residual(const float* F, float xi, float yi, float xj, float yj) {
  const float a0 = xj * F[0] + yj * F[3] + F[6];
  const float a1 = xj * F[1] + yj * F[4] + F[7];
  const float a2 = xj * F[2] + yj * F[5] + F[8];
  return a0 * xi + a1 * yi + a2;
}

__global__ __launch_bounds__(256) void epipolar_fwd_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ F,
                                                           const int* __restrict__ subj, int V, int N, int J,
                                                           float* __restrict__ loss, float* __restrict__ resid) {
  const int P = V * (V - 1);
  const int total = N * P * J;
  float acc = 0.f;
  for (int t = threadIdx.x; t < total; t += 256) {
    const int k = t % J;
    const int bp = t / J;
    const int p = bp % P, b = bp / P;
    int i, j;
    pair_of(p, V, i, j);
    const float* xi = x + (static_cast<size_t>(i) * N + b) * J * 2 + 2 * k;
    const float* xj = x + (static_cast<size_t>(j) * N + b) * J * 2 + 2 * k;
    const float* Fm = F + (static_cast<size_t>(subj[b]) * P + p) * 9;
    float r = fabsf(epi_residual(Fm, xi[0], xi[1], xj[0], xj[1]));
    if (w) r *= w[(static_cast<size_t>(j) * N + b) * J + k] * w[(static_cast<size_t>(i) * N + b) * J + k];
    if (resid) resid[t] = r;
    acc += r;
  }
  __shared__ float part[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float s = (part[0] + part[1]) + (part[2] + part[3]);
    loss[0] = s / static_cast<float>(static_cast<long long>(N) * P * J);
  }
}

// one thread per (view v, sample b, joint k): sums d|r|/dx over the 2(V-1) pairs
// in which view v takes part (as i with F^T h_j, as j with F h_i)
__global__ __launch_bounds__(256) void epipolar_bwd_kernel(const float* __restrict__ x,
                                                           const float* __restrict__ w,
                                                           const float* __restrict__ F,
                                                           const int* __restrict__ subj, int V, int N, int J,
                                                           const float* __restrict__ gloss,
                                                           float* __restrict__ gx) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int total = V * N * J;
  if (t >= total) return;
  const int k = t % J;
  const int vb = t / J;
  const int b = vb % N, v = vb / N;
  const int P = V * (V - 1);
  const float g = gloss[0] / static_cast<float>(static_cast<long long>(N) * P * J);
  float dx = 0.f, dy = 0.f;
  for (int p = 0; p < P; ++p) {
    int i, j;
    pair_of(p, V, i, j);
    if (i != v && j != v) continue;
    const float* Fm = F + (static_cast<size_t>(subj[b]) * P + p) * 9;
    const float* xi = x + (static_cast<size_t>(i) * N + b) * J * 2 + 2 * k;
    const float* xj = x + (static_cast<size_t>(j) * N + b) * J * 2 + 2 * k;
    const float r = epi_residual(Fm, xi[0], xi[1], xj[0], xj[1]);
    float sg = r > 0.f ? g : (r < 0.f ? -g : 0.f);
    if (w) sg *= w[(static_cast<size_t>(j) * N + b) * J + k] * w[(static_cast<size_t>(i) * N + b) * J + k];
    if (i == v) {  // d/dx_i (h_j^T F h_i) = F^T h_j
      dx += sg * (xj[0] * Fm[0] + xj[1] * Fm[3] + Fm[6]);
      dy += sg * (xj[0] * Fm[1] + xj[1] * Fm[4] + Fm[7]);
    } else {  // d/dx_j = F h_i
      dx += sg * (Fm[0] * xi[0] + Fm[1] * xi[1] + Fm[2]);
      dy += sg * (Fm[3] * xi[0] + Fm[4] * xi[1] + Fm[5]);
    }
  }
  gx[2 * t] = dx;
  gx[2 * t + 1] = dy;
}

constexpr int kMaxViews = 16;

// pymvg CameraModel.undistort (OpenCV fixed point, 5 iterations); returns the input
// unchanged when every coefficient is zero, as pymvg does
__device__ __forceinline__ void undistort_px(const double* c, double& u, double& v) {
  const double fx = c[0], fy = c[1], cx = c[2], cy = c[3];
  const double k1 = c[4], k2 = c[5], p1 = c[6], p2 = c[7], k3 = c[8];
  if (fabs(k1) + fabs(k2) + fabs(p1) + fabs(p2) + fabs(k3) == 0.0) return;
  const double xd = (u - cx) / fx, yd = (v - cy) / fy;
  double xx = xd, yy = yd;
#pragma unroll
  for (int it = 0; it < 5; ++it) {
    const double r2 = xx * xx + yy * yy;
    const double icdist = 1.0 / (1.0 + ((k3 * r2 + k2) * r2 + k1) * r2);
    const double dX = 2.0 * p1 * xx * yy + p2 * (r2 + 2.0 * xx * xx);
    const double dY = p1 * (r2 + 2.0 * yy * yy) + 2.0 * p2 * xx * yy;
    xx = (xd - dX) * icdist;
    yy = (yd - dY) * icdist;
  }
  u = xx * fx + cx;
  v = yy * fy + cy;
}

// Smallest right singular vector of A (one-sided Jacobi), dehomogenised: the DLT
// point of pymvg MultiCameraSystem.find3d (svd -> vt[-1, :3] / vt[-1, 3]).
template <int ROWS>
__device__ __forceinline__ void dlt_point(double (&A)[ROWS][4], double* out) {
  // rotate column pairs of A until mutually orthogonal; Vm accumulates the rotations
  double Vm[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
  for (int sweep = 0; sweep < 30; ++sweep) {
    bool rotated = false;
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
          alpha += A[r][p] * A[r][p];
          beta += A[r][q] * A[r][q];
          gamma += A[r][p] * A[r][q];
        }
        if (gamma != 0.0 && fabs(gamma) > 1e-15 * sqrt(alpha * beta)) {
          rotated = true;
          const double zeta = (beta - alpha) / (2.0 * gamma);
          const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
          const double cs = 1.0 / sqrt(1.0 + tt * tt), sn = cs * tt;
#pragma unroll
          for (int r = 0; r < ROWS; ++r) {
            const double ap = A[r][p], aq = A[r][q];
            A[r][p] = cs * ap - sn * aq;
            A[r][q] = sn * ap + cs * aq;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const double vp = Vm[r][p], vq = Vm[r][q];
            Vm[r][p] = cs * vp - sn * vq;
            Vm[r][q] = sn * vp + cs * vq;
          }
        }
      }
    }
    if (!rotated) break;
  }
  double nrm[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    nrm[c] = 0;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) nrm[c] += A[r][c] * A[r][c];
  }
  double v0 = Vm[0][0], v1 = Vm[1][0], v2 = Vm[2][0], v3 = Vm[3][0], bn = nrm[0];
#pragma unroll
  for (int c = 1; c < 4; ++c) {
    if (nrm[c] < bn) {
      bn = nrm[c];
      v0 = Vm[0][c];
      v1 = Vm[1][c];
      v2 = Vm[2][c];
      v3 = Vm[3][c];
    }
  }
  out[0] = v0 / v3;
  out[1] = v1 / v3;
  out[2] = v2 / v3;
}

// R (4 x 4 upper triangular) <- the R factor of [R; a]: Givens rotations fold the row a into R, so
// A^T A = R^T R over every row folded so far and R has A's right singular vectors and values (an
// orthogonal transformation of the rows; nothing is squared).  Up to 4 + 4 doubles live per row
// instead of the whole 2V x 4 matrix.
__device__ __forceinline__ void givens_fold(double (&R)[4][4], double (&a)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (a[c] == 0.0) continue;
    const double r = hypot(R[c][c], a[c]);
    const double cs = R[c][c] / r, sn = a[c] / r;
#pragma unroll
    for (int j = c; j < 4; ++j) {
      const double t = R[c][j];
      R[c][j] = cs * t + sn * a[j];
      a[j] = cs * a[j] - sn * t;
    }
  }
}

// Rows of invisible views are zero: a zero row adds nothing to A^T A, so the right
// singular vectors of the remaining rows are unchanged.  ROWS is a compile-time
// bound, so A lives in registers (no scratch) for the 4-view case; above 4 views the rows are
// folded into a 4 x 4 R factor as they are formed (givens_fold: A = 32 x 4 doubles spilled 32 VGPRs).
template <int VMAX>
__global__ __launch_bounds__(64) void triangulate_kernel(const double* __restrict__ Mall,
                                                         const double* __restrict__ intr,
                                                         const void* __restrict__ xyv, int xy_dtype, int sg,
                                                         int sv, const unsigned char* __restrict__ vis, int G, int V,
                                                         int J, int undistort, double* __restrict__ X) {
  constexpr bool FOLD = VMAX > 4;
  constexpr int ROWS = FOLD ? 4 : 2 * VMAX;
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= G * J) return;
  const int g = t / J, k = t - g * J;
  double A[ROWS][4];
  if constexpr (FOLD) {
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int c = 0; c < 4; ++c) A[r][c] = 0.0;
  }
  int nvis = 0;
#pragma unroll
  for (int v = 0; v < VMAX; ++v) {
    const size_t gv = static_cast<size_t>(g) * V + (v < V ? v : 0);
    const bool on = v < V && (!vis || vis[gv * J + k]);
    double u = 0.0, vv = 0.0;
    if (on) {
      const size_t xoff = static_cast<size_t>(g) * sg + static_cast<size_t>(v) * sv + 2 * k;
      if (xy_dtype == POSU_F64) {
        u = static_cast<const double*>(xyv)[xoff];
        vv = static_cast<const double*>(xyv)[xoff + 1];
      } else {
        u = static_cast<const float*>(xyv)[xoff];
        vv = static_cast<const float*>(xyv)[xoff + 1];
      }
      if (undistort) undistort_px(intr + gv * 9, u, vv);
      ++nvis;
    }
    const double* M = Mall + gv * 12;
    if constexpr (FOLD) {
      if (on) {
        double a0[4], a1[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          a0[c] = u * M[8 + c] - M[c];
          a1[c] = vv * M[8 + c] - M[4 + c];
        }
        givens_fold(A, a0);
        givens_fold(A, a1);
      }
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        A[2 * v][c] = on ? u * M[8 + c] - M[c] : 0.0;
        A[2 * v + 1][c] = on ? vv * M[8 + c] - M[4 + c] : 0.0;
      }
    }
  }
  double* out = X + static_cast<size_t>(t) * 3;
  if (nvis < 2) {  // fewer than two views: the reference leaves zeros (triangulate.py:95-96)
    out[0] = out[1] = out[2] = 0.0;
    return;
  }
  dlt_point<ROWS>(A, out);
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_epipolar_loss_fwd(const float* x, const float* w, const float* F, const int* subj, int V, int N,
                                      int J, int S, float* loss, float* resid, void* stream) {
  POSU_REQUIRE(x && F && subj && loss, "posu_epipolar_loss_fwd: null pointer");
  POSU_REQUIRE(V >= 2 && N >= 0 && J > 0 && S > 0, "posu_epipolar_loss_fwd: bad shape");
  if (N == 0) {
    set_error("posu_epipolar_loss_fwd: empty batch (the reference divides by zero)");
    return POSU_ERR_ARG;
  }
  hipLaunchKernelGGL(epipolar_fwd_kernel, dim3(1), dim3(256), 0, as_stream(stream), x, w, F, subj, V, N, J, loss,
                     resid);
  return check_launch("posu_epipolar_loss_fwd");
}

extern "C" int posu_epipolar_loss_bwd(const float* x, const float* w, const float* F, const int* subj, int V, int N,
                                      int J, int S, const float* gloss, float* gx, void* stream) {
  POSU_REQUIRE(x && F && subj && gloss && gx, "posu_epipolar_loss_bwd: null pointer");
  POSU_REQUIRE(V >= 2 && N > 0 && J > 0 && S > 0, "posu_epipolar_loss_bwd: bad shape");
  const int total = V * N * J;
  hipLaunchKernelGGL(epipolar_bwd_kernel, dim3((total + 255) / 256), dim3(256), 0, as_stream(stream), x, w, F,
                     subj, V, N, J, gloss, gx);
  return check_launch("posu_epipolar_loss_bwd");
}

extern "C" int posu_triangulate_dlt(const double* M, const double* intr, const void* xy, int xy_dtype,
                                    int xy_stride_g, int xy_stride_v, const unsigned char* vis, int G, int V,
                                    int J, int undistort, double* X, void* stream) {
  POSU_REQUIRE(M && intr && xy && X, "posu_triangulate_dlt: null pointer");
  POSU_REQUIRE(G >= 0 && V >= 1 && V <= kMaxViews && J > 0, "posu_triangulate_dlt: bad shape (V <= 16)");
  POSU_REQUIRE(xy_dtype == POSU_F32 || xy_dtype == POSU_F64, "posu_triangulate_dlt: xy dtype must be F32 or F64");
  POSU_REQUIRE(xy_stride_g >= 0 && xy_stride_v >= 0, "posu_triangulate_dlt: negative xy stride");
  if (G == 0) return POSU_OK;
  const int total = G * J;
  if (V <= 4)
    hipLaunchKernelGGL(triangulate_kernel<4>, dim3((total + 63) / 64), dim3(64), 0, as_stream(stream), M, intr, xy,
                       xy_dtype, xy_stride_g, xy_stride_v, vis, G, V, J, undistort, X);
  else
    hipLaunchKernelGGL(triangulate_kernel<kMaxViews>, dim3((total + 63) / 64), dim3(64), 0, as_stream(stream), M,
                       intr, xy, xy_dtype, xy_stride_g, xy_stride_v, vis, G, V, J, undistort, X);
  return check_launch("posu_triangulate_dlt");
}

// ------------------------------------------------------- per-sample 2-D affine
namespace posu {
namespace {

__global__ __launch_bounds__(256) void affine_kernel(const float* __restrict__ pts, const float* __restrict__ T,
                                                     int N, int J, int transpose, float* __restrict__ out) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= N * J) return;
  const float* A = T + static_cast<size_t>(t / J) * 6;
  const float x = pts[2 * t], y = pts[2 * t + 1];
  if (!transpose) {
    out[2 * t] = x * A[0] + y * A[1] + A[2];
    out[2 * t + 1] = x * A[3] + y * A[4] + A[5];
  } else {
    out[2 * t] = x * A[0] + y * A[3];
    out[2 * t + 1] = x * A[1] + y * A[4];
  }
}

}  // namespace
}  // namespace posu

extern "C" int posu_affine2d_apply(const float* pts, const float* T, int N, int J, int transpose, float* out,
                                   void* stream) {
  POSU_REQUIRE(pts && T && out, "posu_affine2d_apply: null pointer");
  POSU_REQUIRE(N >= 0 && J > 0, "posu_affine2d_apply: bad shape");
  if (N == 0) return POSU_OK;
  hipLaunchKernelGGL(affine_kernel, dim3((N * J + 255) / 256), dim3(256), 0, as_stream(stream), pts, T, N, J,
                     transpose, out);
  return check_launch("posu_affine2d_apply");
}

// ------------------------------------------- pseudo-label RANSAC / reprojection
// multiviews/triangulate.py:102-213 (ransac, reproject_poses) for V <= 4 views: one
// thread per (group, joint).  The per-view camera is (M = K[R|t], intr) as for
// posu_triangulate_dlt; find2d is pymvg's CameraModel.project_3d_to_pixel with the
// OpenCV plumb-bob distortion of intr (zero coefficients = pinhole).
namespace posu {
namespace {

constexpr int kPairViews = 4;

__device__ __forceinline__ void project_px(const double* M, const double* c, const double* X, double& u, double& v) {
  const double fx = c[0], fy = c[1], cx = c[2], cy = c[3];
  const double k1 = c[4], k2 = c[5], p1 = c[6], p2 = c[7], k3 = c[8];
  // [R|t] = K^-1 M (zero-skew K)
  double P[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) P[r] = M[4 * r] * X[0] + M[4 * r + 1] * X[1] + M[4 * r + 2] * X[2] + M[4 * r + 3];
  const double zc = P[2];
  const double yc = (P[1] - cy * P[2]) / fy;
  const double xc = (P[0] - cx * P[2]) / fx;
  const double x = xc / zc, y = yc / zc;
  const double r2 = x * x + y * y;
  const double radial = 1.0 + ((k3 * r2 + k2) * r2 + k1) * r2;
  const double xd = x * radial + 2.0 * p1 * x * y + p2 * (r2 + 2.0 * x * x);
  const double yd = y * radial + p1 * (r2 + 2.0 * y * y) + 2.0 * p2 * x * y;
  u = fx * xd + cx;
  v = fy * yd + cy;
}

struct ViewPts {
  double raw[kPairViews][2];  // predictions as given (reprojection errors are measured on these)
  double und[kPairViews][2];  // undistorted (the DLT rows)
  bool on[kPairViews];
  int nvis;
};

__device__ __forceinline__ void load_views(const double* Mall, const double* intr, const double* xy,
                                           const unsigned char* vis, int g, int k, int V, int J, int undistort,
                                           ViewPts& p) {
  p.nvis = 0;
#pragma unroll
  for (int v = 0; v < kPairViews; ++v) {
    const size_t gv = static_cast<size_t>(g) * V + (v < V ? v : 0);
    p.on[v] = v < V && (!vis || vis[gv * J + k]);
    const double* q = xy + (gv * J + k) * 2;
    p.raw[v][0] = v < V ? q[0] : 0.0;
    p.raw[v][1] = v < V ? q[1] : 0.0;
    double u = p.raw[v][0], w = p.raw[v][1];
    if (p.on[v] && undistort) undistort_px(intr + gv * 9, u, w);
    p.und[v][0] = u;
    p.und[v][1] = w;
    if (p.on[v]) ++p.nvis;
  }
}

__global__ __launch_bounds__(64) void ransac_kernel(const double* __restrict__ Mall, const double* __restrict__ intr,
                                                    const double* __restrict__ xy, const unsigned char* __restrict__ vis,
                                                    int G, int V, int J, int undistort, double thre, int min_inliers,
                                                    unsigned char* __restrict__ res_vis) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= G * J) return;
  const int g = t / J, k = t - g * J;
  ViewPts p;
  load_views(Mall, intr, xy, vis, g, k, V, J, undistort, p);
  int best_mask = 0, best_n = 0;
  double best_err = 10000.0;
  if (p.nvis >= 2) {
    // itertools.combinations over the visible views, in view order (loops unrolled: the view
    // indices are compile-time, so p's arrays stay in registers -- a run-time index put them in
    // 144 B of scratch)
#pragma unroll
    for (int a = 0; a < kPairViews; ++a) {
#pragma unroll
      for (int b = a + 1; b < kPairViews; ++b) {
        if (!p.on[a] || !p.on[b]) continue;
        double A[4][4];
        const int pv[2] = {a, b};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          const double* M = Mall + (static_cast<size_t>(g) * V + pv[r]) * 12;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            A[2 * r][c] = p.und[pv[r]][0] * M[8 + c] - M[c];
            A[2 * r + 1][c] = p.und[pv[r]][1] * M[8 + c] - M[4 + c];
          }
        }
        double X[3];
        dlt_point<4>(A, X);
        int mask = 0, n = 0;
        double err = 0.0;
#pragma unroll
        for (int v = 0; v < kPairViews; ++v) {
          if (v >= V) break;
          const size_t gv = static_cast<size_t>(g) * V + v;
          double u, w;
          project_px(Mall + gv * 12, intr + gv * 9, X, u, w);
          const double du = u - p.raw[v][0], dv = w - p.raw[v][1];
          const double e = sqrt(du * du + dv * dv);
          if (e < thre) {
            mask |= 1 << v;
            ++n;
            err += e;
          }
        }
        if (n < min_inliers) continue;
        err /= n;
        if (n > best_n || (n == best_n && err < best_err)) {
          best_n = n;
          best_mask = mask;
          best_err = err;
        }
      }
    }
  }
  for (int v = 0; v < V; ++v) res_vis[(static_cast<size_t>(g) * V + v) * J + k] = (best_mask >> v) & 1;
}

__global__ __launch_bounds__(64) void reproject_kernel(const double* __restrict__ Mall, const double* __restrict__ intr,
                                                       const double* __restrict__ xy,
                                                       const unsigned char* __restrict__ vis, int G, int V, int J,
                                                       int undistort, double* __restrict__ proj,
                                                       unsigned char* __restrict__ res_vis) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= G * J) return;
  const int g = t / J, k = t - g * J;
  ViewPts p;
  load_views(Mall, intr, xy, vis, g, k, V, J, undistort, p);
  const bool ok = p.nvis >= 2;
  double X[3] = {0.0, 0.0, 0.0};
  if (ok) {
    double A[2 * kPairViews][4];
#pragma unroll
    for (int v = 0; v < kPairViews; ++v) {
      const double* M = Mall + (static_cast<size_t>(g) * V + (v < V ? v : 0)) * 12;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        A[2 * v][c] = p.on[v] ? p.und[v][0] * M[8 + c] - M[c] : 0.0;
        A[2 * v + 1][c] = p.on[v] ? p.und[v][1] * M[8 + c] - M[4 + c] : 0.0;
      }
    }
    dlt_point<2 * kPairViews>(A, X);
  }
  for (int v = 0; v < V; ++v) {
    const size_t gv = static_cast<size_t>(g) * V + v;
    double u = 0.0, w = 0.0;
    if (ok) project_px(Mall + gv * 12, intr + gv * 9, X, u, w);
    proj[(gv * J + k) * 2] = u;
    proj[(gv * J + k) * 2 + 1] = w;
    res_vis[gv * J + k] = ok ? 1 : 0;
  }
}

}  // namespace
}  // namespace posu

extern "C" int posu_ransac_inliers(const double* M, const double* intr, const double* xy, const unsigned char* vis,
                                   int G, int V, int J, int undistort, double reproj_thre, int min_inliers,
                                   unsigned char* res_vis, void* stream) {
  POSU_REQUIRE(M && intr && xy && res_vis, "posu_ransac_inliers: null pointer");
  POSU_REQUIRE(G >= 0 && V >= 2 && V <= kPairViews && J > 0, "posu_ransac_inliers: bad shape (2 <= V <= 4)");
  POSU_REQUIRE(min_inliers >= 1, "posu_ransac_inliers: min_inliers >= 1 (the reference divides by the inlier count)");
  if (G == 0) return POSU_OK;
  hipLaunchKernelGGL(ransac_kernel, dim3((G * J + 63) / 64), dim3(64), 0, as_stream(stream), M, intr, xy, vis, G, V,
                     J, undistort, reproj_thre, min_inliers, res_vis);
  return check_launch("posu_ransac_inliers");
}

extern "C" int posu_reproject(const double* M, const double* intr, const double* xy, const unsigned char* vis, int G,
                              int V, int J, int undistort, double* proj, unsigned char* res_vis, void* stream) {
  POSU_REQUIRE(M && intr && xy && proj && res_vis, "posu_reproject: null pointer");
  POSU_REQUIRE(G >= 0 && V >= 2 && V <= kPairViews && J > 0, "posu_reproject: bad shape (2 <= V <= 4)");
  if (G == 0) return POSU_OK;
  hipLaunchKernelGGL(reproject_kernel, dim3((G * J + 63) / 64), dim3(64), 0, as_stream(stream), M, intr, xy, vis, G,
                     V, J, undistort, proj, res_vis);
  return check_launch("posu_reproject");
}
