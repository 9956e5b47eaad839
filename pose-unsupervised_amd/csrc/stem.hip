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
#include <string>
#include <type_traits>

#include "posu_common.h"

namespace posu {
namespace {

constexpr int kStemK = 224;       // 7 kernel rows x 8 taps x 4 channels
constexpr int kStemPitch = 232;   // weight row pitch in LDS (elements): conflict-free B reads
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
};

// The views of one forward (the caller's NCHW f32 tensors, each [Nv, 3, H, W]) in one launch.
constexpr int kMaxViews = 8;
struct StemViews {
  const float* x[kMaxViews];
};

// timing ablations (tools/stem_micro.py only; wrong results when non-zero): 1 no MFMAs, 2 no input
// loads, 4 no output stores
#ifndef POSU_STEM_ABLATE
#define POSU_STEM_ABLATE 0
#endif
// input prefetch depth of the eight-wave kernel (items ahead): 2 measured equal to 1
// (profiles/r04/stem_micro_r4g.txt), so 1
#ifndef POSU_STEM_PFD
#define POSU_STEM_PFD 1
#endif
constexpr int kStemAbl = POSU_STEM_ABLATE;

// NW waves; wave w owns stem columns 16w .. 16w + 15 (one m-tile column group).  A block walks a
// strip of consecutive pool-row pairs of one image (item k = pool rows 2k, 2k+1 = stem rows
// 4k-1 .. 4k+3):
//   * the input rows live in a 16-row LDS ring (slot = input row & 15, [col][4 ch] as above);
//     item k reads input rows 8k-3 .. 8k+9, of which 8k+2 .. 8k+9 are new: they are loaded into
//     registers while item k-1 computes and written to the ring behind it;
//   * stem row 4k-1 (the first row of pool row 2k's window) is item k-1's last stem row, carried
//     in registers: an item computes 4 stem rows (the strip's first item 5), not 5.
// SPL (round 5, the split-fp16 dtype POSU_F16X3, T = f16_t): the input window is staged twice, as
// its fp16 hi and lo halves (two rings), the weights likewise ([hi 64][224] then [lo 64][224] in
// w), every kernel row issues w_hi.x_hi + w_lo.x_hi + w_hi.x_lo, and the pooled outputs are stored
// as (hi, lo) pairs in the split layout (128 halves per pixel).  Eight waves (W = 256) only: the
// twelve-wave rings do not fit twice.
// RAW (round 5, the training step's stem, lib/models/pose_resnet.py:192): the raw convolution
// [N, H/2, W/2, 64] (no BN / ReLU / pool: the batch statistics need it), from the parameter's own
// f32 [64][3][7][7] weights (re-laid out into LDS by every block: no per-step pack); every item
// computes its 4 stem rows and stores them (8-byte NHWC stores).
template <typename T, int NW, bool SPL = false, bool RAW = false>
__global__ __launch_bounds__(NW * 64, 1) void stem_pool_kernel(StemViews xs, int Nv, int N, int H, int W, int hflip,
                                                               int strips, const void* __restrict__ wv_,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ shift, T* __restrict__ y) {
  using O = StemOp<T>;
  constexpr int NT = NW * 64;
  constexpr int WP = NW * 32 + 8;            // window columns: input cols -3 .. W + 4
  constexpr int RB = WP * 8;                 // bytes per ring row
  constexpr int RING = 16;
  constexpr int W_BYTES = 64 * kStemPitch * 2;
  constexpr int NS = SPL ? 2 : 1;            // halves staged (hi [, lo])
  constexpr int CPX = SPL ? 128 : 64;        // stored elements per output pixel
  static_assert(!SPL || (NW == 8 && std::is_same<T, f16_t>::value), "split stem: fp16 halves, eight waves");
  static_assert(!RAW || (!SPL && NW == 8), "raw stem: one dtype, eight waves");
  const T* __restrict__ w = static_cast<const T*>(wv_);
  __shared__ __attribute__((aligned(16))) char smem[NS * (RING * RB + W_BYTES) + NW * 2 * 64 * 4 + 2 * 64 * 4];
  char* win = smem;
  char* winl = smem + RING * RB;              // SPL: the lo ring
  char* wl = smem + NS * RING * RB;
  char* wll = wl + W_BYTES;                   // SPL: the lo weights
  float* edge = reinterpret_cast<float*>(smem + NS * (RING * RB + W_BYTES));  // [wave][pool row][64 ch]
  float* bn = edge + NW * 2 * 64;                                             // scale [64], shift [64]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int Hp = H / 4, Wp = W / 4;
  const int pairs = Hp / 2, per = pairs / strips;
  const int n = blockIdx.x / strips;
  const int k0 = (blockIdx.x - n * strips) * per, k1 = k0 + per;
  const float* __restrict__ xn = xs.x[n / Nv] + static_cast<size_t>(n % Nv) * 3 * H * W;
  const size_t plane = static_cast<size_t>(H) * W;

  // ---- weights and BN -> LDS (once per block)
  if constexpr (RAW) {
    // w = f32 [64 co][3 ci][7 kh][7 kw] -> LDS [co][kh * 32 + kw * 4 + ci] (tap 7 and ci 3 zero)
    const float* __restrict__ wf = static_cast<const float*>(wv_);
    for (int i = tid; i < 64 * kStemK / 2; i += NT) {
      const int co = i / (kStemK / 2), k0 = 2 * (i - co * (kStemK / 2));
      float v[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int k = k0 + u, kh = k >> 5, kw = (k >> 2) & 7, ci = k & 3;
        v[u] = (kw < 7 && ci < 3) ? wf[((co * 3 + ci) * 7 + kh) * 7 + kw] : 0.f;
      }
      *reinterpret_cast<uint32_t*>(wl + (co * kStemPitch + k0) * 2) = O::pack2(v[0], v[1]);
    }
  } else {
  if (tid < 64) {
    bn[tid] = fabsf(scale[tid]);   // |s|: the sign is in the staged weights
    bn[64 + tid] = shift[tid];
  }
  {
    constexpr int WCH = 64 * (kStemK / 8);
#pragma unroll
    for (int it = 0; it < (NS * WCH + NT - 1) / NT; ++it) {
      const int i = tid + it * NT;
      if (i < NS * WCH) {
        const int h = i / WCH, ii = i - h * WCH;   // h = 1: the lo plane (SPL)
        const int co = ii / (kStemK / 8), ck = ii - co * (kStemK / 8);
        // the sign of the channel's BN scale folded into its weights (negation is exact, in the
        // MFMA sums too): the accumulators are sgn(s) * conv, which the pool maximises directly
        const unsigned sg = __float_as_uint(scale[co]) & 0x80000000u ? 0x80008000u : 0u;
        u32x4 wv = *reinterpret_cast<const u32x4*>(w + i * 8);
        wv ^= sg;
        *reinterpret_cast<u32x4*>((h ? wll : wl) + (co * kStemPitch + ck * 8) * 2) = wv;
      }
    }
  }
  }

  // input rows -> registers: row i0 + r (r < NR), group gk = 4 input columns 4 (gk - 1) .. + 3 of
  // each plane (window columns 4 gk - 1 .. 4 gk + 2)
  constexpr int GPR = NW * 8 + 2;
  constexpr int XG8 = (8 * GPR + NT - 1) / NT;
  auto load_rows = [&](int i0, auto nr, float4 (*xv)[3]) __attribute__((always_inline)) {
    constexpr int NR = decltype(nr)::value, XG = (NR * GPR + NT - 1) / NT;
#pragma unroll
    for (int it = 0; it < XG; ++it) {
      const int i = tid + it * NT;
      const int r = i / GPR, gk = i - r * GPR;
      const int iy = i0 + r, c0 = 4 * (gk - 1);
#pragma unroll
      for (int p = 0; p < 3; ++p) xv[it][p] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (kStemAbl & 2) {
        xv[it][0] = make_float4(iy, c0, 1.f, 0.5f);
        continue;
      }
      if (i < NR * GPR && static_cast<unsigned>(iy) < static_cast<unsigned>(H) &&
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
  };
  auto store_rows = [&](int i0, auto nr, float4 (*xv)[3]) __attribute__((always_inline)) {
    constexpr int NR = decltype(nr)::value, XG = (NR * GPR + NT - 1) / NT;
#pragma unroll
    for (int it = 0; it < XG; ++it) {
      const int i = tid + it * NT;
      if (i >= NR * GPR) continue;
      const int r = i / GPR, gk = i - r * GPR;
      char* row = win + ((i0 + r) & (RING - 1)) * RB;
      const float a0[4] = {xv[it][0].x, xv[it][0].y, xv[it][0].z, xv[it][0].w};
      const float a1[4] = {xv[it][1].x, xv[it][1].y, xv[it][1].z, xv[it][1].w};
      const float a2[4] = {xv[it][2].x, xv[it][2].y, xv[it][2].z, xv[it][2].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int wc = 4 * gk - 1 + e;
        if (wc >= 0 && wc < WP) {
          *reinterpret_cast<uint2*>(row + wc * 8) = make_uint2(O::pack2(a0[e], a1[e]), O::pack2(a2[e], 0.f));
          if constexpr (SPL) {   // lo = fp16(v - hi) (exact difference in f32)
            const float l0 = a0[e] - static_cast<float>(static_cast<_Float16>(a0[e]));
            const float l1 = a1[e] - static_cast<float>(static_cast<_Float16>(a1[e]));
            const float l2 = a2[e] - static_cast<float>(static_cast<_Float16>(a2[e]));
            *reinterpret_cast<uint2*>(row - win + winl + wc * 8) = make_uint2(O::pack2(l0, l1), O::pack2(l2, 0.f));
          }
        }
      }
    }
  };

  const int sc = 16 * wid + r16;
  // Pool first, BN after: with t = sgn(s) * conv (the sign-folded weights' accumulator),
  // relu(s conv + b) = relu(fma(|s|, t, b)) is non-decreasing in t, and so is its rounding to the
  // compute dtype, so the max-pool of the rounded stem values equals that function of the max-pool
  // of t -- bit for bit the two-launch result, with the BN / ReLU / rounding done once per pooled
  // value instead of once per stem value.  Pool padding: -inf in t (the max of the rest is >= 0
  // after the ReLU either way).
  // stem rows r0 .. r0 + M - 1 (m-tile rl = stem row r0 + rl; pixel column sc), folded straight
  // into the two pool rows' vertical maxima of t (rows outside the image: -inf):
  // M = 5: rows 4k-1 .. 4k+3; M = 4: rows 4k .. 4k+3 with row 4k-1 = carry.  carry <- row 4k+3.
  // (channel 16 j + 4 q + e)
  auto stem_rows = [&](int r0, auto mrows, float (*carry)[4], float (*vm)[4][4]) __attribute__((always_inline)) {
    constexpr int M = decltype(mrows)::value;
    f32x4 acc[M][4];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // window row of (m-tile rl, kernel row kh): 2 (r0 + rl) - 3 + kh = 2 r0 - 3 + rho, rho = 2 rl + kh;
    // column 2 sc + 2 q (= input col 2 sc - 3 + 2 q)
    auto rd = [&](int rho) {
      return *reinterpret_cast<const uint4*>(win + ((2 * r0 - 3 + rho) & (RING - 1)) * RB + (2 * sc + 2 * q) * 8);
    };
    auto rdl = [&](int rho) {   // SPL: the lo ring
      return *reinterpret_cast<const uint4*>(winl + ((2 * r0 - 3 + rho) & (RING - 1)) * RB + (2 * sc + 2 * q) * 8);
    };
    auto bload = [&](int kh, uint4 (&bfr)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(wl + ((16 * j + r16) * kStemPitch + kh * 32 + 8 * q) * 2);
    };
    auto bloadl = [&](int kh, uint4 (&bfr)[4]) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(wll + ((16 * j + r16) * kStemPitch + kh * 32 + 8 * q) * 2);
    };
    auto mmas = [&](const uint4 (&bfr)[4], const uint4 (&af)[M]) {
#pragma unroll
      for (int rl = 0; rl < M; ++rl)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (kStemAbl & 1) acc[rl][j][0] += __uint_as_float(bfr[j].x ^ af[rl].y);
          else O::mma(acc[rl][j], bfr[j], af[rl]);
        }
    };
    if constexpr (SPL) {
      // w_hi.x_hi + w_lo.x_hi + w_hi.x_lo per kernel row; the rolling sets of the plain kernel for
      // both halves of the window
      uint4 ev[M], od[M], evl[M], odl[M], bfr[4], bfl[4];
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        uint4 (&set)[M] = (kh & 1) ? od : ev;
        uint4 (&setl)[M] = (kh & 1) ? odl : evl;
        bload(kh, bfr);
        bloadl(kh, bfl);
        if (kh < 2) {
#pragma unroll
          for (int rl = 0; rl < M; ++rl) {
            set[rl] = rd(kh + 2 * rl);
            setl[rl] = rdl(kh + 2 * rl);
          }
        } else {
#pragma unroll
          for (int rl = 0; rl + 1 < M; ++rl) {
            set[rl] = set[rl + 1];
            setl[rl] = setl[rl + 1];
          }
          set[M - 1] = rd(kh + 2 * (M - 1));
          setl[M - 1] = rdl(kh + 2 * (M - 1));
        }
        mmas(bfr, set);
        mmas(bfl, set);
        mmas(bfr, setl);
      }
    } else if constexpr (NW <= 8) {
      // kernel rows of one parity read the same window rows shifted by one m-tile: two rolling
      // sets (even / odd kh) load 2 M + 5 distinct rows instead of 7 M
      uint4 ev[M], od[M], bfr[4];
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        uint4 (&set)[M] = (kh & 1) ? od : ev;
        bload(kh, bfr);
        if (kh < 2) {
#pragma unroll
          for (int rl = 0; rl < M; ++rl) set[rl] = rd(kh + 2 * rl);
        } else {
#pragma unroll
          for (int rl = 0; rl + 1 < M; ++rl) set[rl] = set[rl + 1];
          set[M - 1] = rd(kh + 2 * (M - 1));
        }
        mmas(bfr, set);
      }
    } else {  // twelve waves: fewer registers in flight
#pragma unroll 1
      for (int kh = 0; kh < 7; ++kh) {
        uint4 bfr[4];
        bload(kh, bfr);
#pragma unroll
        for (int rl = 0; rl < M; ++rl) {
          const uint4 af = rd(kh + 2 * rl);
#pragma unroll
          for (int j = 0; j < 4; ++j) O::mma(acc[rl][j], bfr[j], af);
        }
      }
    }
    if constexpr (RAW) {
      // stem row r0 + rl, column sc, channels 16 j + 4 q .. + 3 (every row of an item is inside
      // the image: items start at stem row 4 k)
      T* __restrict__ zr = y + (static_cast<size_t>(n) * (H / 2) + r0) * (W / 2) * 64 + sc * 64 + 4 * q;
#pragma unroll
      for (int rl = 0; rl < M; ++rl)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint2 u = make_uint2(O::pack2(acc[rl][j][0], acc[rl][j][1]), O::pack2(acc[rl][j][2], acc[rl][j][3]));
          if (kStemAbl & 4) asm volatile("" ::"v"(u.x), "v"(u.y));
          else *reinterpret_cast<uint2*>(zr + static_cast<size_t>(rl) * (W / 2) * 64 + 16 * j) = u;
        }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v[M];
#pragma unroll
        for (int rl = 0; rl < M; ++rl)   // (only the strip's first item, M = 5, reaches above the image)
          v[rl] = (M == 4 || r0 + rl >= 0) ? acc[rl][j][e] : -INFINITY;
        const float first = M == 5 ? v[0] : carry[j][e];
        const float* u = v + (M == 5 ? 1 : 0);   // stem rows 4k .. 4k+3
        vm[0][j][e] = fmaxf(fmaxf(first, u[0]), u[1]);
        vm[1][j][e] = fmaxf(fmaxf(u[1], u[2]), u[3]);
        carry[j][e] = u[3];
      }
  };

  T* __restrict__ yn = y + static_cast<size_t>(n) * Hp * Wp * CPX;
  // pool rows 2k, 2k+1 from their vertical maxima: horizontal max with DPP row shifts (a wave's
  // left neighbour column through LDS), then BN + ReLU + rounding, 8-byte NHWC stores
  auto pool = [&](int k, const float (*vm)[4][4]) __attribute__((always_inline)) {
    if (r16 == 15) {
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *reinterpret_cast<float4*>(edge + (wid * 2 + p) * 64 + 16 * j + 4 * q) =
              make_float4(vm[p][j][0], vm[p][j][1], vm[p][j][2], vm[p][j][3]);
    }
    __syncthreads();
    // the left neighbour wave's last column, read by every lane (16-B reads, no divergent branch)
    // and taken by the r16 = 0 lanes; wave 0's left is the pool padding
    const int wl = wid > 0 ? wid - 1 : 0;
    const bool first_col = r16 == 0, pad_left = wid == 0;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float4 s4 = *reinterpret_cast<const float4*>(bn + 16 * j + 4 * q);
        const float4 b4 = *reinterpret_cast<const float4*>(bn + 64 + 16 * j + 4 * q);
        const float sv[4] = {s4.x, s4.y, s4.z, s4.w}, bv[4] = {b4.x, b4.y, b4.z, b4.w};
        const float4 l4 = *reinterpret_cast<const float4*>(edge + (wl * 2 + p) * 64 + 16 * j + 4 * q);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float self = vm[p][j][e];
          // DPP row shifts inside the 16-lane rows (= the wave's 16 columns): column sc + 1
          // (used by even r16 < 15 only) and column sc - 1 (r16 = 0 takes the neighbour's edge)
          const float right = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(self), 0x101, 0xf, 0xf, true));
          float left = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(self), 0x111, 0xf, 0xf, true));
          if (first_col) left = pad_left ? -INFINITY : lv[e];
          o[e] = fmaxf(fmaf(sv[e], fmaxf(fmaxf(left, self), right), bv[e]), 0.f);
        }
        if ((r16 & 1) == 0) {
          const int pc = 8 * wid + (r16 >> 1);
          const int c0 = 16 * j + 4 * q;
          T* dst = yn + (static_cast<size_t>(2 * k + p) * Wp + pc) * CPX + (SPL ? split_ch(c0) : c0);
          const uint2 u = make_uint2(O::pack2(o[0], o[1]), O::pack2(o[2], o[3]));
          if (kStemAbl & 4) {
            asm volatile("" ::"v"(u.x), "v"(u.y));
          } else {
            *reinterpret_cast<uint2*>(dst) = u;
            if constexpr (SPL) {
              float l[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) l[e] = o[e] - static_cast<float>(static_cast<_Float16>(o[e]));
              *reinterpret_cast<uint2*>(dst + 32) = make_uint2(O::pack2(l[0], l[1]), O::pack2(l[2], l[3]));
            }
          }
        }
      }
  };

  // ---- the strip's first item: input rows 8 k0 - 5 .. 8 k0 + 9, stem rows 4 k0 - 1 .. 4 k0 + 3
  using I4 = std::integral_constant<int, 4>;
  using I5 = std::integral_constant<int, 5>;
  using I8 = std::integral_constant<int, 8>;
  float carry[4][4], vm[2][4][4];
  // PF: the following items' new input rows are loaded into registers while this item computes
  // (PFD items ahead, one register set each), and stem row 4k-1 is carried (eight waves); twelve
  // waves per block (W = 384) have no registers left for either: rows loaded in turn, every item
  // computes its 5 stem rows
  constexpr bool PF = NW <= 8;
  constexpr int PFD = PF ? POSU_STEM_PFD : 1;
  static_assert(PFD == 1 || PFD == 2, "prefetch depth 1 or 2");
  float4 xv[PFD][XG8][3];
  // (16 rows 8 k0 - 5 .. 8 k0 + 10: two 8-row loads through the prefetch registers; the last row
  // is not read by this item and is rewritten before item k0 + 1 reads it)
  load_rows(8 * k0 - 5, I8{}, xv[0]);
  store_rows(8 * k0 - 5, I8{}, xv[0]);
  load_rows(8 * k0 + 3, I8{}, xv[0]);
  store_rows(8 * k0 + 3, I8{}, xv[0]);
  __syncthreads();
  if constexpr (RAW) stem_rows(4 * k0, I4{}, carry, vm);
  else stem_rows(4 * k0 - 1, I5{}, carry, vm);
  // item k0 + d's new rows into set d % PFD, during item k0's pool
  if constexpr (PF) {
    if (k0 + 1 < k1) load_rows(8 * k0 + 10, I8{}, xv[PFD - 1]);
    if (PFD == 2 && k0 + 2 < k1) load_rows(8 * k0 + 18, I8{}, xv[0]);
  }
  if constexpr (RAW) __syncthreads();   // item k0 + 1's ring writes follow every wave's reads
  else pool(k0, vm);
  // item k: its rows are in set S = (k - k0) % PFD (a compile-time index: a register set picked
  // at run time would live in scratch); once stored, the set takes item k + PFD's
  auto item = [&](int k, auto sidx) __attribute__((always_inline)) {
    constexpr int S = decltype(sidx)::value;
    if (!PF) load_rows(8 * k + 2, I8{}, xv[S]);
    // every wave is past item k-1's window reads -- they precede the barrier in item k-1's pool --
    // so its dead rows take item k's without another barrier (item k-1's edge reads after that
    // barrier touch only the edge slots, which the next write reaches past the barrier below)
    store_rows(8 * k + 2, I8{}, xv[S]);
    __syncthreads();
    if (PF && k + PFD < k1) load_rows(8 * (k + PFD) + 2, I8{}, xv[S]);
    if constexpr (PF) stem_rows(4 * k, I4{}, carry, vm);
    else stem_rows(4 * k - 1, I5{}, carry, vm);
    if constexpr (RAW) {
      // the next item's ring writes wait for every wave's window reads (the pool's barrier does
      // this in the pooled kernel)
      __syncthreads();
    } else {
      pool(k, vm);
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, PFD - 1>;
  int k = k0 + 1;
  if constexpr (PFD == 2) {
    for (; k + 1 < k1; k += 2) {   // two items per trip
      item(k, S1{});
      item(k + 1, S0{});
    }
  }
  for (; k < k1; ++k) item(k, S1{});   // PFD 2: at most one item left, its rows in set 1
}


// ---- the training stem's weight gradient (round 5; lib/models/pose_resnet.py:192 under autograd):
//   dW[co][ci][kh][kw] = sum over (n, oy, ox) of dz[n][oy][ox][co] * x[n][ci][2 oy - 3 + kh][2 ox - 3 + kw]
// as MFMAs over the pixels (K) of one stem row at a time: D[co][f] with f = kw * 4 + ci (kw < 8,
// ci < 4: tap 7 and channel 3 are dropped by the reduction).  A block walks a strip of stem rows
// of one image; wave w = kernel row kh.  Per stem row:
//   * dz row [128 px][64 co] in LDS (16-B chunks XOR-swizzled by pixel: conflict-free transposed
//     reads), A = dz^T by ds_read_b64_tr_b16 (4 pixel rows x 16 channels per 16-lane group);
//   * the input window as the inference stem stages it ([input row][col + 3][3 ch + 0] bf16 in a
//     16-row ring, read straight from the caller's NCHW f32 views): the im2col row of pixel px at
//     kernel row kh is the 64 contiguous bytes at 16 px of ring row 2 oy - 3 + kh, so B = X is a
//     transposed read with a 16-B row stride;
//   * the next row's dz and its two new input rows are loaded into registers while this row's
//     MFMAs run, then written to the other dz buffer / free ring slots (one barrier per row).
// Each block writes its partial [7 kh][32 f][64 co] f32; posu_stem_wgrad sums the partials in block
// order (deterministic) into the parameter's [64][3][7][7] layout.
typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int kWgThreads = 448;          // 7 waves
constexpr int kWgRing = 16;
constexpr int kWgCols = 264;             // window columns: input cols -3 .. 260
constexpr int kWgRB = kWgCols * 8;
constexpr int kWgDz = 128 * 128;         // one dz row: 128 px x 64 ch x 2 B
constexpr int kWgGroups = 66;            // 4-column input groups per row
constexpr int kWgPart = 7 * 32 * 64;     // floats per block partial

__device__ __forceinline__ int wg_sw(int px) { return (((px >> 1) & 1) << 1) | (((px >> 3) & 1) << 2); }

__device__ __forceinline__ uint4 tr_pair(const char* p0, const char* p1) {
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1));
  const uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
  return make_uint4(u0.x, u0.y, u1.x, u1.y);
}

template <typename T>
__global__ __launch_bounds__(kWgThreads, 2) void stem_wgrad_kernel(StemViews xs, int Nv, int H, int strips,
                                                                   const T* __restrict__ dz, float* __restrict__ part) {
  using O = StemOp<T>;
  constexpr int W = 256, Wo = 128;
  __shared__ __attribute__((aligned(16))) char smem[kWgRing * kWgRB + 2 * kWgDz];
  char* ring = smem;
  char* dzb = smem + kWgRing * kWgRB;
  const int tid = threadIdx.x, lane = tid & 63, kh = tid >> 6;
  const int q = lane >> 4, a = (lane >> 2) & 3, p = lane & 3;
  const int Ho = H / 2, rows = Ho / strips;
  const int n = blockIdx.x / strips;
  const int ya = (blockIdx.x - n * strips) * rows, yb = ya + rows;
  const float* __restrict__ xn = xs.x[n / Nv] + static_cast<size_t>(n % Nv) * 3 * H * W;
  const size_t plane = static_cast<size_t>(H) * W;
  const T* __restrict__ dzn = dz + static_cast<size_t>(n) * Ho * Wo * 64;

  // input rows iy0 .. iy0 + nr - 1 -> registers (item i: row i / 66, group i % 66 = input cols
  // 4 (g - 1) .. + 3 of each plane) and -> ring slots (window cols 4 g - 1 .. 4 g + 2)
  auto load_x = [&](int iy0, int nr, int it, float4 (&xv)[3]) {
    const int i = tid + it * kWgThreads;
    const int r = i / kWgGroups, g = i - r * kWgGroups;
    const int iy = iy0 + r, c0 = 4 * (g - 1);
    // a load from a valid address (the image's first pixels when outside) and a value select: a
    // conditional load into zeros made the compiler keep the zeros in scratch
    const bool ok = i < nr * kWgGroups && static_cast<unsigned>(iy) < static_cast<unsigned>(H) &&
                    static_cast<unsigned>(c0) < static_cast<unsigned>(W);
    const size_t o = ok ? static_cast<size_t>(iy) * W + c0 : 0;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
      const float4 v = *reinterpret_cast<const float4*>(xn + pl * plane + o);
      xv[pl] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  auto store_x = [&](int iy0, int nr, int it, const float4 (&xv)[3]) {
    const int i = tid + it * kWgThreads;
    if (i >= nr * kWgGroups) return;
    const int r = i / kWgGroups, g = i - r * kWgGroups;
    char* row = ring + ((iy0 + r) & (kWgRing - 1)) * kWgRB;
    // (components by compile-time index: arrays of them went to scratch)
    auto cmp = [](const float4& v, int e) { return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w; };
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int wc = 4 * g - 1 + e;
      if (wc >= 0 && wc < kWgCols)
        *reinterpret_cast<uint2*>(row + wc * 8) =
            make_uint2(O::pack2(cmp(xv[0], e), cmp(xv[1], e)), O::pack2(cmp(xv[2], e), 0.f));
    }
  };
  // dz row oy: 1024 16-B chunks, chunk i = pixel i / 8, channels 8 (i % 8) ..
  auto load_dz = [&](int oy, uint4 (&dv)[3]) {
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int i = tid + it * kWgThreads;
      dv[it] = i < 1024 ? *reinterpret_cast<const uint4*>(dzn + (static_cast<size_t>(oy) * Wo) * 64 + i * 8)
                        : make_uint4(0, 0, 0, 0);
    }
  };
  auto store_dz = [&](int buf, const uint4 (&dv)[3]) {
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int i = tid + it * kWgThreads;
      if (i < 1024) {
        const int px = i >> 3, c = i & 7;
        *reinterpret_cast<uint4*>(dzb + buf * kWgDz + px * 128 + ((c ^ wg_sw(px)) << 4)) = dv[it];
      }
    }
  };

  {  // prologue: input rows 2 ya - 3 .. 2 ya + 3, dz row ya
    float4 xv[3];
#pragma unroll
    for (int it = 0; it < (7 * kWgGroups + kWgThreads - 1) / kWgThreads; ++it) {
      load_x(2 * ya - 3, 7, it, xv);
      store_x(2 * ya - 3, 7, it, xv);
    }
    uint4 dv[3];
    load_dz(ya, dv);
    store_dz(0, dv);
  }
  __syncthreads();

  f32x4 acc[4][2];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) acc[mt][hf] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int oy = ya; oy < yb; ++oy) {
    const bool more = oy + 1 < yb;
    float4 xv[3];
    uint4 dv[3];
    if (more) {   // two new input rows (132 items: threads 0 .. 131) and the next dz row
      load_x(2 * oy + 4, 2, 0, xv);
      load_dz(oy + 1, dv);
    }
    const char* dzr = dzb + (oy & 1) * kWgDz;
    const char* xr = ring + ((2 * oy - 3 + kh) & (kWgRing - 1)) * kWgRB;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // pixel rows of this lane's two 4-row blocks: 32 s + 8 q + 4 t + a
      const int px0 = 32 * s + 8 * q + a, px1 = px0 + 4;
      uint4 af[4], bf[2];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) {
        const int chunk = 2 * mt + (p >> 1), within = (p & 1) * 8;
        af[mt] = tr_pair(dzr + px0 * 128 + ((chunk ^ wg_sw(px0)) << 4) + within,
                         dzr + px1 * 128 + ((chunk ^ wg_sw(px1)) << 4) + within);
      }
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
        bf[hf] = tr_pair(xr + 16 * px0 + 32 * hf + 8 * p, xr + 16 * px1 + 32 * hf + 8 * p);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          if (kStemAbl & 1) acc[mt][hf][0] += __uint_as_float(af[mt].x ^ bf[hf].y);
          else O::mma(acc[mt][hf], af[mt], bf[hf]);
        }
    }
    if (more) {
      store_x(2 * oy + 4, 2, 0, xv);
      store_dz((oy + 1) & 1, dv);
    }
    __syncthreads();
  }
  // partial [kh][f][co]: lane (col f = 16 hf + (lane & 15), rows co = 16 mt + 4 q + r)
  float* dst = part + static_cast<size_t>(blockIdx.x) * kWgPart + kh * 32 * 64;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
      *reinterpret_cast<float4*>(dst + (16 * hf + (lane & 15)) * 64 + 16 * mt + 4 * q) =
          make_float4(acc[mt][hf][0], acc[mt][hf][1], acc[mt][hf][2], acc[mt][hf][3]);
}

// dw[co][ci][kh][kw] (the parameter's layout) = sum over the blocks' partials in a fixed order: a
// 256-thread block owns 16 consecutive co of one (kh, kw, ci); lane sl of an output sums blocks
// sl, sl + 16, .. (loads in flight together), then the 16 lanes combine in lane order via LDS
constexpr int kWrLanes = 16;
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nblocks,
                                                                 float* __restrict__ dw) {
  __shared__ float red[kWrLanes][17];
  const int c = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int rest = blockIdx.x >> 2, co = (blockIdx.x & 3) * 16 + c;   // rest = (kh * 7 + kw) * 3 + ci
  const int ci = rest % 3, tap = rest / 3, kh = tap / 7, kw = tap - 7 * kh;
  const float* p = part + (kh * 32 + kw * 4 + ci) * 64 + co;
  float s = 0.f;
#pragma unroll 4
  for (int b = sl; b < nblocks; b += kWrLanes) s += p[static_cast<size_t>(b) * kWgPart];
  red[sl][c] = s;
  __syncthreads();
  if (threadIdx.x < 16) {
    float t = 0.f;
#pragma unroll
    for (int l = 0; l < kWrLanes; ++l) t += red[l][threadIdx.x];
    dw[((co * 3 + ci) * 7 + kh) * 7 + kw] = t;
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

namespace {
int stem_launch(int dtype, const float* const* views, int nviews, int Nv, int H, int W, int hflip, const void* w,
                const float* scale, const float* shift, void* y, void* stream, const char* what) {
  const std::string wh(what);
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16 || dtype == POSU_F16X3, wh + ": dtype must be BF16, F16 or F16X3");
  POSU_REQUIRE(dtype != POSU_F16X3 || W == 256, wh + ": the split-fp16 stem is built for W = 256");
  POSU_REQUIRE(views && nviews >= 1 && nviews <= kMaxViews, wh + ": 1 .. 8 views");
  for (int v = 0; v < nviews; ++v) POSU_REQUIRE(views[v], wh + ": null view pointer");
  POSU_REQUIRE(w && scale && shift && y, wh + ": null pointer");
  POSU_REQUIRE(Nv > 0 && H > 0 && H % 8 == 0 && (W == 256 || W == 384),
               wh + ": needs H % 8 == 0 and W in {256, 384}");
  POSU_REQUIRE(static_cast<long long>(Nv) * 3 * H * W < (1LL << 40), wh + ": input too large");
  StemViews xs{};
  for (int v = 0; v < nviews; ++v) xs.x[v] = views[v];
  const int N = Nv * nviews, pairs = H / 8;
  // strips per image: about one block per CU (a strip of `pairs / strips` consecutive items)
  int strips = 1;
  while (N * strips * 2 <= 256 && pairs % (strips * 2) == 0) strips *= 2;
  hipStream_t s = as_stream(stream);
  const dim3 grid(static_cast<unsigned>(N * strips));
  if (dtype == POSU_F16X3) {
    hipLaunchKernelGGL((stem_pool_kernel<f16_t, 8, true>), grid, dim3(512), 0, s, xs, Nv, N, H, W, hflip, strips,
                       static_cast<const f16_t*>(w), scale, shift, static_cast<f16_t*>(y));
  } else if (dtype == POSU_BF16) {
    if (W == 256)
      hipLaunchKernelGGL((stem_pool_kernel<uint16_t, 8>), grid, dim3(512), 0, s, xs, Nv, N, H, W, hflip, strips,
                         static_cast<const uint16_t*>(w), scale, shift, static_cast<uint16_t*>(y));
    else
      hipLaunchKernelGGL((stem_pool_kernel<uint16_t, 12>), grid, dim3(768), 0, s, xs, Nv, N, H, W, hflip, strips,
                         static_cast<const uint16_t*>(w), scale, shift, static_cast<uint16_t*>(y));
  } else {
    if (W == 256)
      hipLaunchKernelGGL((stem_pool_kernel<f16_t, 8>), grid, dim3(512), 0, s, xs, Nv, N, H, W, hflip, strips,
                         static_cast<const f16_t*>(w), scale, shift, static_cast<f16_t*>(y));
    else
      hipLaunchKernelGGL((stem_pool_kernel<f16_t, 12>), grid, dim3(768), 0, s, xs, Nv, N, H, W, hflip, strips,
                         static_cast<const f16_t*>(w), scale, shift, static_cast<f16_t*>(y));
  }
  return check_launch(what);
}
}  // namespace

extern "C" int posu_stem_pool_fwd(int dtype, const float* x, int N, int H, int W, int hflip, const void* w,
                                  const float* scale, const float* shift, void* y, void* stream) {
  return stem_launch(dtype, &x, 1, N, H, W, hflip, w, scale, shift, y, stream, "posu_stem_pool_fwd");
}

// The same over the views of one forward in one launch: views[v] = [Nv, 3, H, W] f32 (host array
// of device pointers), y = the views' pooled outputs stacked view-major [nviews * Nv, H/4, W/4, 64].
extern "C" int posu_stem_pool_views_fwd(int dtype, const float* const* views, int nviews, int Nv, int H, int W,
                                        int hflip, const void* w, const float* scale, const float* shift, void* y,
                                        void* stream) {
  return stem_launch(dtype, views, nviews, Nv, H, W, hflip, w, scale, shift, y, stream, "posu_stem_pool_views_fwd");
}

// ---- training stem (round 5, ABI 14)
namespace {
int stem_train_views(const char* what, int dtype, const float* const* views, int nviews, int Nv, int H, int W,
                     StemViews& xs) {
  const std::string wh(what);
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, wh + ": dtype must be BF16 or F16");
  POSU_REQUIRE(views && nviews >= 1 && nviews <= kMaxViews, wh + ": 1 .. 8 views");
  for (int v = 0; v < nviews; ++v) POSU_REQUIRE(views[v], wh + ": null view pointer");
  POSU_REQUIRE(Nv > 0 && H > 0 && H % 8 == 0 && W == 256, wh + ": built for W = 256 and H % 8 == 0");
  POSU_REQUIRE(static_cast<long long>(Nv) * 3 * H * W < (1LL << 40), wh + ": input too large");
  for (int v = 0; v < nviews; ++v) {
    POSU_REQUIRE((reinterpret_cast<size_t>(views[v]) & 15) == 0, wh + ": views must be 16-byte aligned");
    xs.x[v] = views[v];
  }
  return 0;
}

int wgrad_strips(int N, int H) {
  int strips = 1;   // about two blocks per CU
  while (N * strips * 2 <= 512 && (H / 2) % (strips * 2) == 0 && (H / 2) / (strips * 2) >= 8) strips *= 2;
  return strips;
}
}  // namespace

extern "C" int posu_stem_conv_views_fwd(int dtype, const float* const* views, int nviews, int Nv, int H, int W,
                                        const float* w, void* z, void* stream) {
  StemViews xs{};
  const int rc = stem_train_views("posu_stem_conv_views_fwd", dtype, views, nviews, Nv, H, W, xs);
  if (rc) return rc;
  POSU_REQUIRE(w && z, "posu_stem_conv_views_fwd: null pointer");
  const int N = Nv * nviews, pairs = H / 8;
  int strips = 1;
  while (N * strips * 2 <= 256 && pairs % (strips * 2) == 0) strips *= 2;
  hipStream_t s = as_stream(stream);
  const dim3 grid(static_cast<unsigned>(N * strips));
  if (dtype == POSU_BF16)
    hipLaunchKernelGGL((stem_pool_kernel<uint16_t, 8, false, true>), grid, dim3(512), 0, s, xs, Nv, N, H, W, 0, strips,
                       static_cast<const void*>(w), nullptr, nullptr, static_cast<uint16_t*>(z));
  else
    hipLaunchKernelGGL((stem_pool_kernel<f16_t, 8, false, true>), grid, dim3(512), 0, s, xs, Nv, N, H, W, 0, strips,
                       static_cast<const void*>(w), nullptr, nullptr, static_cast<f16_t*>(z));
  return check_launch("posu_stem_conv_views_fwd");
}

extern "C" long long posu_stem_wgrad_workspace(int N, int H, int W) {
  if (N <= 0 || H <= 0 || H % 8 != 0 || W != 256) return -1;
  return static_cast<long long>(N) * wgrad_strips(N, H) * kWgPart * 4;
}

extern "C" int posu_stem_wgrad_views(int dtype, const float* const* views, int nviews, int Nv, int H, int W,
                                     const void* dz, float* dw, void* workspace, long long workspace_bytes,
                                     void* stream) {
  StemViews xs{};
  const int rc = stem_train_views("posu_stem_wgrad_views", dtype, views, nviews, Nv, H, W, xs);
  if (rc) return rc;
  POSU_REQUIRE(dz && dw && workspace, "posu_stem_wgrad_views: null pointer");
  POSU_REQUIRE((reinterpret_cast<size_t>(dz) & 15) == 0 && (reinterpret_cast<size_t>(workspace) & 15) == 0,
               "posu_stem_wgrad_views: dz / workspace must be 16-byte aligned");
  const int N = Nv * nviews, strips = wgrad_strips(N, H);
  POSU_REQUIRE(workspace_bytes >= posu_stem_wgrad_workspace(N, H, W), "posu_stem_wgrad_views: workspace too small");
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  const dim3 grid(static_cast<unsigned>(N * strips));
  if (dtype == POSU_BF16)
    hipLaunchKernelGGL(stem_wgrad_kernel<uint16_t>, grid, dim3(kWgThreads), 0, s, xs, Nv, H, strips,
                       static_cast<const uint16_t*>(dz), part);
  else
    hipLaunchKernelGGL(stem_wgrad_kernel<f16_t>, grid, dim3(kWgThreads), 0, s, xs, Nv, H, strips,
                       static_cast<const f16_t*>(dz), part);
  hipLaunchKernelGGL(stem_wgrad_reduce_kernel, dim3(147 * 4), dim3(256), 0, s, part, N * strips, dw);
  return check_launch("posu_stem_wgrad_views");
}
