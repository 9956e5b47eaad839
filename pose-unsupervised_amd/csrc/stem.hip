// Fused PoseResNet stem: input pack + conv1 (7x7 / s2 / p3, 3 -> 64) + bn1 + ReLU +
// maxpool (3x3 / s2 / p1) in one launch (lib/models/pose_resnet.py:111-115, 192-195).
//
// The layer-by-layer path writes the 128x128x64 stem output (268 MB per 128 frames at
// 256x256) and reads it back 1.5x through the max-pool; here a block owns two pool rows
// of one image and keeps everything on chip:
//
//   1. the input window (15 input rows x W+8 columns) is read once from the caller's NCHW
//      f32 tensor, rounded to the compute dtype and staged in LDS as [row][col][4 ch]
//      (3 channels + a zero channel: 8 bytes per pixel, so one ds_read_b128 = 2 pixels
//      x 4 channels = 8 consecutive K of the MFMA operand); the flip test's mirror is
//      folded into the column index;
//   2. the 5 stem rows under the two pool rows (2 p0 - 1 .. 2 p0 + 3) are an implicit GEMM
//      M = 5 x W/2 pixels, N = 64, K = 7 kernel rows x 8 taps x 4 ch = 224 (tap 7 and the
//      4th channel carry zero weights) on v_mfma_f32_16x16x32_{bf16,f16}: one k-step per
//      kernel row, lane group q = tap pair (2q, 2q+1); wave w owns a 16-column band;
//   3. BN scale/shift + ReLU in registers, the 3-row vertical max in-lane, the 3-column
//      horizontal max with lane shuffles (the one column a wave's band borrows from its
//      left neighbour goes through LDS), 8-byte NHWC stores of the pooled pixels.
//
// Pool padding (-inf in MaxPool2d) and ReLU >= 0 make "ignore" and "0" the same, so rows /
// columns outside the stem image enter the max as 0.  The stem values are rounded to the
// compute dtype before the max exactly like the two-launch path (rounding is monotonic).
#include "posu_common.h"

namespace posu {
namespace {

constexpr int kStemK = 224;       // 7 kernel rows x 8 taps x 4 channels
constexpr int kStemPitch = 232;   // weight row pitch in LDS (elements): conflict-free B reads
constexpr int kWinRows = 15;      // input rows under two pool rows
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <typename T>
struct StemOp;
template <>
struct StemOp<uint16_t> {
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                  0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    return f2bf2(a, b);
  }
  static __device__ __forceinline__ float round(float a) { return bf2f(f2bf(a)); }
};
template <>
struct StemOp<f16_t> {
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc, 0,
                                                 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack2(float a, float b) {
    const _Float16 ha = static_cast<_Float16>(a), hb = static_cast<_Float16>(b);
    return static_cast<uint32_t>(__builtin_bit_cast(uint16_t, ha)) |
           (static_cast<uint32_t>(__builtin_bit_cast(uint16_t, hb)) << 16);
  }
  static __device__ __forceinline__ float round(float a) { return static_cast<float>(static_cast<_Float16>(a)); }
};

// NW waves; wave w owns stem columns 16w .. 16w + 15 (one m-tile column group) of the 5
// stem rows -> 5 m-tiles x 4 n-tiles (64 channels) of accumulators.
template <typename T, int NW>
__global__ __launch_bounds__(NW * 64) void stem_pool_kernel(const float* __restrict__ x, int N, int H, int W,
                                                            int hflip, const T* __restrict__ w,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, T* __restrict__ y) {
  using O = StemOp<T>;
  constexpr int NT = NW * 64;
  constexpr int WP = NW * 32 + 8;            // window columns: input cols -3 .. W + 4
  constexpr int WIN_BYTES = kWinRows * WP * 8;
  constexpr int W_BYTES = 64 * kStemPitch * 2;
  __shared__ __attribute__((aligned(16))) char smem[WIN_BYTES + W_BYTES + NW * 2 * 64 * 4];
  char* win = smem;
  char* wl = smem + WIN_BYTES;
  float* edge = reinterpret_cast<float*>(smem + WIN_BYTES + W_BYTES);  // [wave][pool row][64 ch]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int Hp = H / 4, Wp = W / 4;
  const int pairs = Hp / 2;
  const int n = blockIdx.x / pairs, p0 = 2 * (blockIdx.x - n * pairs);  // pool rows p0, p0 + 1
  const int r0 = 4 * p0 - 5;                                           // first window input row

  // ---- global -> registers first (the block's loads all in flight at once), then LDS
  constexpr int WCH = 64 * (kStemK / 8);                 // 16-B weight chunks
  constexpr int WIT = (WCH + NT - 1) / NT;
  u32x4 wv[WIT];
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int i = min(tid + it * NT, WCH - 1);  // clamped: duplicate chunks store the same bytes
    wv[it] = *reinterpret_cast<const u32x4*>(w + i * 8);
  }
  // input window pixel (r, c) = input (r0 + r, c - 3), 3 channels + 0, read as 16-B groups
  // of 4 input columns (4 gk - 4 .. 4 gk - 1) per plane: window columns 4 gk - 1 .. 4 gk + 2
  const size_t plane = static_cast<size_t>(H) * W;
  const float* __restrict__ xn = x + static_cast<size_t>(n) * 3 * plane;
  constexpr int GPR = NW * 8 + 2;                          // groups per window row (W / 4 + 2)
  constexpr int XG = (kWinRows * GPR + NT - 1) / NT;       // groups per thread
  float4 xv[XG][3];
#pragma unroll
  for (int it = 0; it < XG; ++it) {
    const int i = tid + it * NT;
    const int r = i / GPR, gk = i - r * GPR;
    const int iy = r0 + r, c0 = 4 * (gk - 1);
#pragma unroll
    for (int p = 0; p < 3; ++p) xv[it][p] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < kWinRows * GPR && static_cast<unsigned>(iy) < static_cast<unsigned>(H) &&
        static_cast<unsigned>(c0) < static_cast<unsigned>(W)) {
      const size_t o = static_cast<size_t>(iy) * W + (hflip ? W - 4 - c0 : c0);
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        float4 v = *reinterpret_cast<const float4*>(xn + p * plane + o);
        if (hflip) v = make_float4(v.w, v.z, v.y, v.x);
        xv[it][p] = v;
      }
    }
  }
#pragma unroll
  for (int it = 0; it < WIT; ++it) {
    const int i = min(tid + it * NT, WCH - 1);
    const int co = i / (kStemK / 8), ck = i - co * (kStemK / 8);
    *reinterpret_cast<u32x4*>(wl + (co * kStemPitch + ck * 8) * 2) = wv[it];
  }
#pragma unroll
  for (int it = 0; it < XG; ++it) {
    const int i = tid + it * NT;
    if (i >= kWinRows * GPR) continue;
    const int r = i / GPR, gk = i - r * GPR;
    const float a0[4] = {xv[it][0].x, xv[it][0].y, xv[it][0].z, xv[it][0].w};
    const float a1[4] = {xv[it][1].x, xv[it][1].y, xv[it][1].z, xv[it][1].w};
    const float a2[4] = {xv[it][2].x, xv[it][2].y, xv[it][2].z, xv[it][2].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int wc = 4 * gk - 1 + e;
      if (wc >= 0 && wc < WP)
        *reinterpret_cast<uint2*>(win + (r * WP + wc) * 8) = make_uint2(O::pack2(a0[e], a1[e]), O::pack2(a2[e], 0.f));
    }
  }
  __syncthreads();

  // ---- stem GEMM: m-tile rl = local stem row, pixel column sc = 16 wid + r16
  f32x4 acc[5][4];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int sc = 16 * wid + r16;
#pragma unroll 1
  for (int kh = 0; kh < 7; ++kh) {
    uint4 bfr[4], af[5];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = *reinterpret_cast<const uint4*>(wl + ((16 * j + r16) * kStemPitch + kh * 32 + 8 * q) * 2);
    // window row 2 rl + kh, window column 2 sc + 2 q (= input col 2 sc - 3 + 2 q)
#pragma unroll
    for (int rl = 0; rl < 5; ++rl)
      af[rl] = *reinterpret_cast<const uint4*>(win + ((2 * rl + kh) * WP + 2 * sc + 2 * q) * 8);
#pragma unroll
    for (int rl = 0; rl < 5; ++rl)
#pragma unroll
      for (int j = 0; j < 4; ++j) O::mma(acc[rl][j], bfr[j], af[rl]);
  }

  // ---- BN + ReLU (+ rounding to T), vertical max over local stem rows 2p .. 2p + 2
  const bool row0_valid = p0 > 0;  // local stem row 0 = stem row 2 p0 - 1
  float vm[2][4][4];               // [pool row][n-tile][ch]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = 16 * j + 4 * q + e;
      const float s_ = scale[co], b_ = shift[co];
      float v[5];
#pragma unroll
      for (int rl = 0; rl < 5; ++rl) v[rl] = O::round(fmaxf(acc[rl][j][e] * s_ + b_, 0.f));
      if (!row0_valid) v[0] = 0.f;
      vm[0][j][e] = fmaxf(fmaxf(v[0], v[1]), v[2]);
      vm[1][j][e] = fmaxf(fmaxf(v[2], v[3]), v[4]);
    }
  // the band's last column (r16 = 15) is the next wave's left neighbour
  if (r16 == 15) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) edge[(wid * 2 + p) * 64 + 16 * j + 4 * q + e] = vm[p][j][e];
  }
  __syncthreads();

  // ---- horizontal max: pool col pc <- stem cols 2 pc - 1, 2 pc, 2 pc + 1 (even lanes)
  T* __restrict__ yn = y + static_cast<size_t>(n) * Hp * Wp * 64;
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float self = vm[p][j][e];
        const float right = __shfl_down(self, 1, 16);  // column sc + 1 (r16 even < 15)
        float left = __shfl_up(self, 1, 16);           // column sc - 1
        if (r16 == 0) left = wid > 0 ? edge[((wid - 1) * 2 + p) * 64 + 16 * j + 4 * q + e] : 0.f;
        o[e] = fmaxf(fmaxf(left, self), right);
      }
      if ((r16 & 1) == 0) {
        const int pc = 8 * wid + (r16 >> 1);
        T* dst = yn + (static_cast<size_t>(p0 + p) * Wp + pc) * 64 + 16 * j + 4 * q;
        *reinterpret_cast<uint2*>(dst) = make_uint2(O::pack2(o[0], o[1]), O::pack2(o[2], o[3]));
      }
    }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_stem_pool_fwd(int dtype, const float* x, int N, int H, int W, int hflip, const void* w,
                                  const float* scale, const float* shift, void* y, void* stream) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, "posu_stem_pool_fwd: dtype must be BF16 or F16");
  POSU_REQUIRE(x && w && scale && shift && y, "posu_stem_pool_fwd: null pointer");
  POSU_REQUIRE(N > 0 && H > 0 && H % 8 == 0 && (W == 256 || W == 384),
               "posu_stem_pool_fwd: needs H % 8 == 0 and W in {256, 384}");
  POSU_REQUIRE(static_cast<long long>(N) * 3 * H * W < (1LL << 40), "posu_stem_pool_fwd: input too large");
  hipStream_t s = as_stream(stream);
  const int blocks = N * (H / 8);
  if (dtype == POSU_BF16) {
    if (W == 256)
      hipLaunchKernelGGL((stem_pool_kernel<uint16_t, 8>), dim3(blocks), dim3(512), 0, s, x, N, H, W, hflip,
                         static_cast<const uint16_t*>(w), scale, shift, static_cast<uint16_t*>(y));
    else
      hipLaunchKernelGGL((stem_pool_kernel<uint16_t, 12>), dim3(blocks), dim3(768), 0, s, x, N, H, W, hflip,
                         static_cast<const uint16_t*>(w), scale, shift, static_cast<uint16_t*>(y));
  } else {
    if (W == 256)
      hipLaunchKernelGGL((stem_pool_kernel<f16_t, 8>), dim3(blocks), dim3(512), 0, s, x, N, H, W, hflip,
                         static_cast<const f16_t*>(w), scale, shift, static_cast<f16_t*>(y));
    else
      hipLaunchKernelGGL((stem_pool_kernel<f16_t, 12>), dim3(blocks), dim3(768), 0, s, x, N, H, W, hflip,
                         static_cast<const f16_t*>(w), scale, shift, static_cast<f16_t*>(y));
  }
  return check_launch("posu_stem_pool_fwd");
}
