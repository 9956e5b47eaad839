// HBM-bound layout kernels around the conv stack: NCHW f32 -> NHWC packing of the
// input crops, NHWC -> NCHW f32 unpacking of returned feature maps, and the stem
// max-pool.  One 16-byte channel chunk per thread, vectorised loads/stores.
#include "posu_common.h"

namespace posu {
namespace {

// one thread per (pixel, 16-B output chunk)
template <typename T>
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ x, int N, int C, int H, int W,
                                                   T* __restrict__ y, int Cpad, int hflip) {
  constexpr int E = Vec<T>::E;
  const int chunks = Cpad / E;
  const long long total = static_cast<long long>(N) * H * W * chunks;
  const long long HW = static_cast<long long>(H) * W;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const long long n = pix / HW;
    long long p = pix - n * HW;
    if (hflip) {  // torch.flip(x, dims=[3]) (function.py:569) folded into the pack
      const long long row = p / W;
      p = row * W + (W - 1 - (p - row * W));
    }
    float v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int c = ch * E + e;
      v[e] = c < C ? x[(n * C + c) * HW + p] : 0.f;
    }
    *reinterpret_cast<uint4*>(y + pix * Cpad + ch * E) = Vec<T>::pack(v);
  }
}

// space-to-depth 2x2 pack for the stem: y[n][y][x][(dy*2+dx)*C + c] = x[n][c][2y+dy][2x+dx]
// (one thread per output pixel and 16-B chunk)
template <typename T>
__global__ __launch_bounds__(256) void pack_s2d_kernel(const float* __restrict__ x, int N, int C, int H, int W,
                                                       T* __restrict__ y, int Cpad, int hflip) {
  constexpr int E = Vec<T>::E;
  const int chunks = Cpad / E;
  const int Hs = H / 2, Ws = W / 2;
  const long long total = static_cast<long long>(N) * Hs * Ws * chunks;
  const long long HW = static_cast<long long>(H) * W;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const int xs = static_cast<int>(pix % Ws);
    const long long t = pix / Ws;
    const int ys = static_cast<int>(t % Hs);
    const long long n = t / Hs;
    float v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int cc = ch * E + e;
      const int sub = cc / C, c = cc - sub * C;
      const int col = 2 * xs + (sub & 1);
      v[e] = sub < 4 ? x[(n * C + c) * HW + static_cast<long long>(2 * ys + (sub >> 1)) * W + (hflip ? W - 1 - col : col)]
                     : 0.f;
    }
    *reinterpret_cast<uint4*>(y + pix * Cpad + ch * E) = Vec<T>::pack(v);
  }
}

// rows of the cross-view aggregation GEMM: dst[m][o*HW + q] = src[o][m][q]
// (src f32 view-major [V][M][HW], e.g. V views of [N, J, H, W] heatmaps with M = N*J)
template <typename T>
__global__ __launch_bounds__(256) void pack_view_rows_kernel(const float* __restrict__ src, int V, int M, int HW,
                                                             T* __restrict__ dst) {
  constexpr int E = Vec<T>::E;
  const int cpv = HW / E;  // chunks per view
  const long long total = static_cast<long long>(M) * V * cpv;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % cpv);
    const long long r = i / cpv;
    const int o = static_cast<int>(r % V);
    const long long m = r / V;
    const float* s = src + (static_cast<long long>(o) * M + m) * HW + ch * E;
    float v[E];
#pragma unroll
    for (int e = 0; e < E; e += 4) {
      const float4 t = *reinterpret_cast<const float4*>(s + e);
      v[e] = t.x;
      v[e + 1] = t.y;
      v[e + 2] = t.z;
      v[e + 3] = t.w;
    }
    *reinterpret_cast<uint4*>(dst + i * E) = Vec<T>::pack(v);
  }
}

// one thread per (pixel, 16-B input chunk); writes E channel planes
template <typename T>
__global__ __launch_bounds__(256) void unpack_kernel(const T* __restrict__ x, int N, int H, int W, int C,
                                                     float* __restrict__ y) {
  constexpr int E = Vec<T>::E;
  const int chunks = C / E;
  const long long HW = static_cast<long long>(H) * W;
  const long long total = N * HW * chunks;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    // pixel-fastest thread order so the NCHW stores coalesce
    const long long p = i % HW;
    const long long rest = i / HW;
    const int ch = static_cast<int>(rest % chunks);
    const long long n = rest / chunks;
    float v[E];
    Vec<T>::unpack(*reinterpret_cast<const uint4*>(x + (n * HW + p) * C + ch * E), v);
#pragma unroll
    for (int e = 0; e < E; ++e) y[(n * C + ch * E + e) * HW + p] = v[e];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void maxpool_kernel(const T* __restrict__ x, int N, int H, int W, int C,
                                                      T* __restrict__ y, int Ho, int Wo) {
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
#pragma unroll
    for (int e = 0; e < E; ++e) m[e] = -INFINITY;
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = oy * 2 - 1 + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int ix = ox * 2 - 1 + dx;
        if (ix < 0 || ix >= W) continue;
        float v[E];
        Vec<T>::unpack(*reinterpret_cast<const uint4*>(x + ((n * H + iy) * W + ix) * C + ch * E), v);
#pragma unroll
        for (int e = 0; e < E; ++e) m[e] = fmaxf(m[e], v[e]);
      }
    }
    *reinterpret_cast<uint4*>(y + pix * C + ch * E) = Vec<T>::pack(m);
  }
}

// ---- split fp16 (POSU_F16X3) layouts: logical channel c's hi at split_ch(c), its lo 32 later;
// one thread per (pixel, 8-channel logical chunk), a 16-B store to each half.
// s2d == 0: NCHW f32 -> NHWC [N, H, W, 2 Cpad]; s2d == 1: the space-to-depth pack (channel
// (dy*2+dx)*C + c) [N, H/2, W/2, 2 Cpad].
__global__ __launch_bounds__(256) void pack_split_kernel(const float* __restrict__ x, int N, int C, int H, int W,
                                                         uint16_t* __restrict__ y, int Cpad, int hflip, int s2d) {
  const int chunks = Cpad / 8;
  const int Ho = s2d ? H / 2 : H, Wo = s2d ? W / 2 : W;
  const long long total = static_cast<long long>(N) * Ho * Wo * chunks;
  const long long HW = static_cast<long long>(H) * W;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const int xo = static_cast<int>(pix % Wo);
    const long long t = pix / Wo;
    const int yo = static_cast<int>(t % Ho);
    const long long n = t / Ho;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int cc = ch * 8 + e;
      int c = cc, row = yo, col = xo;
      bool ok = cc < C;
      if (s2d) {
        const int sub = cc / C;
        c = cc - sub * C;
        row = 2 * yo + (sub >> 1);
        col = 2 * xo + (sub & 1);
        ok = sub < 4;
      }
      v[e] = ok ? x[(n * C + c) * HW + static_cast<long long>(row) * W + (hflip ? W - 1 - col : col)] : 0.f;
    }
    uint4 hi, lo;
    split8(v, hi, lo);
    uint16_t* d = y + pix * (2 * Cpad) + split_ch(ch * 8);
    *reinterpret_cast<uint4*>(d) = hi;
    *reinterpret_cast<uint4*>(d + 32) = lo;
  }
}

// MaxPool2d(3, 2, 1) over split pairs: the max of the f32 values hi + lo, stored re-split (the
// winner's own pair: the split of hi + lo reproduces (hi, lo))
__global__ __launch_bounds__(256) void maxpool_split_kernel(const uint16_t* __restrict__ x, int N, int H, int W,
                                                            int C, uint16_t* __restrict__ y, int Ho, int Wo) {
  const int chunks = C / 8;
  const long long total = static_cast<long long>(N) * Ho * Wo * chunks;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const int ch = static_cast<int>(i % chunks);
    const long long pix = i / chunks;
    const int ox = static_cast<int>(pix % Wo);
    const long long t = pix / Wo;
    const int oy = static_cast<int>(t % Ho);
    const long long n = t / Ho;
    const int co = split_ch(ch * 8);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
    for (int dy = 0; dy < 3; ++dy) {
      const int iy = oy * 2 - 1 + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int ix = ox * 2 - 1 + dx;
        if (ix < 0 || ix >= W) continue;
        const uint16_t* s = x + ((n * H + iy) * W + ix) * (2LL * C) + co;
        float v[8];
        join8(*reinterpret_cast<const uint4*>(s), *reinterpret_cast<const uint4*>(s + 32), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], v[e]);
      }
    }
    uint4 hi, lo;
    split8(m, hi, lo);
    uint16_t* d = y + pix * (2LL * C) + co;
    *reinterpret_cast<uint4*>(d) = hi;
    *reinterpret_cast<uint4*>(d + 32) = lo;
  }
}

// split NHWC [N, H, W, 2C] -> NCHW f32 (hi + lo)
__global__ __launch_bounds__(256) void unpack_split_kernel(const uint16_t* __restrict__ x, int N, int H, int W,
                                                           int C, float* __restrict__ y) {
  const int chunks = C / 8;
  const long long HW = static_cast<long long>(H) * W;
  const long long total = N * HW * chunks;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += static_cast<long long>(gridDim.x) * 256) {
    const long long p = i % HW;
    const long long rest = i / HW;
    const int ch = static_cast<int>(rest % chunks);
    const long long n = rest / chunks;
    const uint16_t* s = x + (n * HW + p) * (2LL * C) + split_ch(ch * 8);
    float v[8];
    join8(*reinterpret_cast<const uint4*>(s), *reinterpret_cast<const uint4*>(s + 32), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) y[(n * C + ch * 8 + e) * HW + p] = v[e];
  }
}

inline int grid_for(long long total) {
  long long g = (total + 255) / 256;
  return static_cast<int>(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

int chunk_elems(int dtype) { return dtype == POSU_F32 ? 4 : 8; }

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_pack_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W, void* y, int Cpad,
                                      int hflip, void* stream) {
  POSU_REQUIRE(x && y, "posu_pack_nchw_to_nhwc: null pointer");
  POSU_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0 && Cpad >= C, "posu_pack_nchw_to_nhwc: bad shape");
  POSU_REQUIRE(Cpad % chunk_elems(dtype) == 0, "posu_pack_nchw_to_nhwc: Cpad is not a whole number of 16-B chunks");
  hipStream_t s = as_stream(stream);
  const long long pix = static_cast<long long>(N) * H * W;
  if (dtype == POSU_F16X3) {
    POSU_REQUIRE(Cpad % 32 == 0, "posu_pack_nchw_to_nhwc: split fp16 needs Cpad % 32 == 0");
    hipLaunchKernelGGL(pack_split_kernel, dim3(grid_for(pix * Cpad / 8)), dim3(256), 0, s, x, N, C, H, W,
                       static_cast<uint16_t*>(y), Cpad, hflip, 0);
    return check_launch("posu_pack_nchw_to_nhwc");
  }
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(pack_kernel<T>, dim3(grid_for(pix * Cpad / Vec<T>::E)), dim3(256), 0, s, x, N, C, H, W,
                       static_cast<T*>(y), Cpad, hflip);
  });
  POSU_REQUIRE(ok, "posu_pack_nchw_to_nhwc: unsupported dtype");
  return check_launch("posu_pack_nchw_to_nhwc");
}

extern "C" int posu_pack_s2d_nchw(int dtype, const float* x, int N, int C, int H, int W, void* y, int Cpad,
                                  int hflip, void* stream) {
  POSU_REQUIRE(x && y, "posu_pack_s2d_nchw: null pointer");
  POSU_REQUIRE(N > 0 && C > 0 && H > 1 && W > 1 && H % 2 == 0 && W % 2 == 0 && 4 * C <= Cpad,
               "posu_pack_s2d_nchw: bad shape (H, W even, 4C <= Cpad)");
  POSU_REQUIRE(Cpad % chunk_elems(dtype) == 0, "posu_pack_s2d_nchw: Cpad is not a whole number of 16-B chunks");
  hipStream_t s = as_stream(stream);
  const long long pix = static_cast<long long>(N) * (H / 2) * (W / 2);
  if (dtype == POSU_F16X3) {
    POSU_REQUIRE(Cpad % 32 == 0, "posu_pack_s2d_nchw: split fp16 needs Cpad % 32 == 0");
    hipLaunchKernelGGL(pack_split_kernel, dim3(grid_for(pix * Cpad / 8)), dim3(256), 0, s, x, N, C, H, W,
                       static_cast<uint16_t*>(y), Cpad, hflip, 1);
    return check_launch("posu_pack_s2d_nchw");
  }
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(pack_s2d_kernel<T>, dim3(grid_for(pix * Cpad / Vec<T>::E)), dim3(256), 0, s, x, N, C, H, W,
                       static_cast<T*>(y), Cpad, hflip);
  });
  POSU_REQUIRE(ok, "posu_pack_s2d_nchw: unsupported dtype");
  return check_launch("posu_pack_s2d_nchw");
}

extern "C" int posu_nhwc_to_nchw_f32(int dtype, const void* x, int N, int H, int W, int C, float* y,
                                     void* stream) {
  POSU_REQUIRE(x && y, "posu_nhwc_to_nchw_f32: null pointer");
  POSU_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0, "posu_nhwc_to_nchw_f32: bad shape");
  POSU_REQUIRE(C % chunk_elems(dtype) == 0, "posu_nhwc_to_nchw_f32: C is not a whole number of 16-B chunks");
  hipStream_t s = as_stream(stream);
  const long long el = static_cast<long long>(N) * H * W * C;
  if (dtype == POSU_F16X3) {
    POSU_REQUIRE(C % 32 == 0, "posu_nhwc_to_nchw_f32: split fp16 needs C % 32 == 0");
    hipLaunchKernelGGL(unpack_split_kernel, dim3(grid_for(el / 8)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       N, H, W, C, y);
    return check_launch("posu_nhwc_to_nchw_f32");
  }
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(unpack_kernel<T>, dim3(grid_for(el / Vec<T>::E)), dim3(256), 0, s, static_cast<const T*>(x),
                       N, H, W, C, y);
  });
  POSU_REQUIRE(ok, "posu_nhwc_to_nchw_f32: unsupported dtype");
  return check_launch("posu_nhwc_to_nchw_f32");
}

extern "C" int posu_maxpool3x3s2_fwd(int dtype, const void* x, int N, int H, int W, int C, void* y,
                                     void* stream) {
  POSU_REQUIRE(x && y, "posu_maxpool3x3s2_fwd: null pointer");
  POSU_REQUIRE(N > 0 && C > 0 && H > 0 && W > 0, "posu_maxpool3x3s2_fwd: bad shape");
  POSU_REQUIRE(C % chunk_elems(dtype) == 0, "posu_maxpool3x3s2_fwd: C is not a whole number of 16-B chunks");
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  hipStream_t s = as_stream(stream);
  const long long el = static_cast<long long>(N) * Ho * Wo * C;
  if (dtype == POSU_F16X3) {
    POSU_REQUIRE(C % 32 == 0, "posu_maxpool3x3s2_fwd: split fp16 needs C % 32 == 0");
    hipLaunchKernelGGL(maxpool_split_kernel, dim3(grid_for(el / 8)), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       N, H, W, C, static_cast<uint16_t*>(y), Ho, Wo);
    return check_launch("posu_maxpool3x3s2_fwd");
  }
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(maxpool_kernel<T>, dim3(grid_for(el / Vec<T>::E)), dim3(256), 0, s, static_cast<const T*>(x),
                       N, H, W, C, static_cast<T*>(y), Ho, Wo);
  });
  POSU_REQUIRE(ok, "posu_maxpool3x3s2_fwd: unsupported dtype");
  return check_launch("posu_maxpool3x3s2_fwd");
}

extern "C" int posu_pack_view_rows(int dtype, const float* src, int V, int M, int HW, void* dst, void* stream) {
  POSU_REQUIRE(src && dst, "posu_pack_view_rows: null pointer");
  POSU_REQUIRE(V > 0 && M > 0 && HW > 0 && HW % chunk_elems(dtype) == 0 && HW % 4 == 0,
               "posu_pack_view_rows: bad shape (HW a multiple of the 16-B chunk)");
  hipStream_t s = as_stream(stream);
  const long long total = static_cast<long long>(M) * V * (HW / chunk_elems(dtype));
  const bool ok = with_storage(dtype, [&](auto tag) {
    using T = decltype(tag);
    hipLaunchKernelGGL(pack_view_rows_kernel<T>, dim3(grid_for(total)), dim3(256), 0, s, src, V, M, HW,
                       static_cast<T*>(dst));
  });
  POSU_REQUIRE(ok, "posu_pack_view_rows: unsupported dtype");
  return check_launch("posu_pack_view_rows");
}
