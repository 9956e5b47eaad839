// Weight gradient of an NHWC convolution on CDNA4 MFMA (training path, BASELINE configs[3]).
//
//   dW[m][k] = sum_p  G[p][m] * X_window[p][k]
//     p: pixels of the convolution's output grid (n, oy, ox), the reduction axis
//     m: output channels (G = dL/dy, NHWC, channels contiguous)
//     k: (kh, kw, ci) taps of the input window over X (NHWC), the forward's K order
//
// Both operands arrive pixel-major (channels contiguous), i.e. with the reduction axis
// OUTER, which is the transpose of what an MFMA operand register wants (8 consecutive
// k-values per lane).  Tiles are therefore staged into LDS exactly as they lie in
// memory -- [BP pixels][BM channels] and [BP pixels][BN taps], one LDS-DMA
// (buffer_load ... lds) per 16-byte chunk, window taps outside the image read as zeros
// -- and the fragments are read back with gfx950's transposing LDS read
// ds_read_b64_tr_b16 (a 4-row x 16-column block per 16-lane group, delivered column-
// major), two per 16x16x32 operand.  fp32 (the parity mode) reads single dwords for
// v_mfma_f32_16x16x4_f32 instead.  The 16-byte chunk index of every LDS row is XOR-
// swizzled by row (on the DMA source side) so both kinds of read are conflict-free.
//
// The pixel axis is split over blockIdx (split-K): every block writes an f32 partial
// [split][Mpad][Npad]; posu_wgrad_reduce sums the splits in a fixed order
// (deterministic) and scatters into the parameter's own layout.
//
// ConvTranspose2d(4, s2, p1) weight gradients use the same kernel: the transposed
// convolution's input x plays G (its pixel grid is the reduction axis) and its output
// gradient dy plays X under a 4x4 / stride-2 / pad-1 window, which yields
// dW[ci][co][ky][kx] directly in the ConvTranspose2d layout.
#include "posu_common.h"

namespace posu {
namespace {

struct FastDiv {  // q = (umulhi(p, m) + p) >> s  for 0 <= p < 2^31
  unsigned m;
  int s;
};

FastDiv make_fastdiv(int d) {
  FastDiv f;
  int s = 0;
  while ((1LL << s) < d) ++s;
  f.s = s;
  f.m = static_cast<unsigned>(((1ULL << 32) * ((1ULL << s) - static_cast<unsigned long long>(d))) / d + 1);
  return f;
}

__device__ __forceinline__ int fdiv(int p, FastDiv f) {
  return static_cast<int>((__umulhi(static_cast<unsigned>(p), f.m) + static_cast<unsigned>(p)) >> f.s);
}

struct WgradGeom {
  const void* g;  // [P][M] output gradient
  const void* x;  // [N][H][W][C] convolution input
  float* part;    // [splits][Mpad][Npad]
  int N, H, W, C, logC;
  int Ho, Wo, P, M, K;
  int KH, KW, stride, pad;
  int Mpad, Npad, mtiles, ntiles, splits, pps;
  FastDiv div_hw, div_w;
};

constexpr int kOOB = 0x7ffffff0;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 make_srd(const void* base, int bytes) {
  const unsigned long long p = reinterpret_cast<unsigned long long>(base);
  u32x4 r;
  r.x = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(p));
  r.y = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(p >> 32));
  r.z = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(bytes));
  r.w = 0x00020000u;
  return r;
}

__device__ __forceinline__ void dma16(u32x4 srd, int voff, unsigned lds) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(srd), "s"(lds)
      : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// s_waitcnt vmcnt(n), n wave-uniform in {0, D, 2D, ..} up to 3D (the ring's younger stages)
template <int D>
__device__ __forceinline__ void vm_wait_stages(int stages) {
  if (stages >= 3) vm_wait<3 * D>();
  else if (stages == 2) vm_wait<2 * D>();
  else if (stages == 1) vm_wait<D>();
  else vm_wait<0>();
}

// workgroup barrier that retires this wave's LDS reads (lgkmcnt(0)) and leaves the ring's
// younger LDS-DMA stages in flight (__syncthreads() would wait for them too)
__device__ __forceinline__ void wg_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS ring slots of the weight-gradient kernel (S - 1 pixel stages in flight).  Measured on the
// R50 training shapes (tools/wgrad_micro.py, profiles/r03/wgrad_slots_r3h.txt): S = 2 1644 us,
// S = 3 2047 us, S = 4 1944 us summed -- the 3x3 layers lose 50-90 % with deeper rings, the
// 1x1 ones gain up to 20 %; S = 2 kept
#ifndef POSU_WG_SLOTS
#define POSU_WG_SLOTS 2
#endif
constexpr int kWgSlots = POSU_WG_SLOTS;
// pixel-stage groups per block (round 5): KG groups of four waves take alternate pixel stages,
// each through its own S-slot ring, and add their f32 tiles in LDS at the end -- twice the waves
// issuing MFMAs and DMAs per CU at the same partial traffic (one partial tile per block)
#ifndef POSU_WG_KG
#define POSU_WG_KG 2
#endif
constexpr int kWgKG = POSU_WG_KG;
// pixels per LDS stage of the 2-byte kernels (A/B knob)
#ifndef POSU_WG_BP2
#define POSU_WG_BP2 64
#endif

// chunk swizzle of LDS row `row` for rows of CG 16-byte chunks (see the header)
template <int ES, int CG>
__device__ __forceinline__ int swz_row(int row) {
  if constexpr (ES == 4) return (row & 1) << 2;
  else if constexpr (CG == 8) return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;
  else return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
}

// one MFMA operand fragment (16 rows of the tile's column axis x one k-step of pixels)
template <typename T>
struct WOp;

template <>
struct WOp<uint16_t> {
  static constexpr int KSTEP = 32;  // pixels per MFMA
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                  0, 0, 0);
  }
};
template <>
struct WOp<f16_t> {
  static constexpr int KSTEP = 32;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), acc,
                                                 0, 0, 0);
  }
};
template <>
struct WOp<float> {
  static constexpr int KSTEP = 4;
  static __device__ __forceinline__ void mma(f32x4& acc, float a, float b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
};

// 16-bit operand: lane l takes column c0 + (l & 15) of pixel rows ks + 8*(l >> 4) .. +7
template <int ROWB, int CG>
__device__ __forceinline__ uint4 frag_tr16(const char* tile, int ks, int c0, int lane) {
  const int gq = lane >> 4, a = (lane >> 2) & 3, b = lane & 3;
  const int col = c0 + 4 * b;  // 16-bit element column
  const int chunk = col >> 3, within = (col & 7) * 2;
  const int r0 = ks + 8 * gq + a, r1 = r0 + 4;
  const char* p0 = tile + r0 * ROWB + ((chunk ^ swz_row<2, CG>(r0)) << 4) + within;
  const char* p1 = tile + r1 * ROWB + ((chunk ^ swz_row<2, CG>(r1)) << 4) + within;
  const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p0));
  const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p1));
  const uint2 u0 = __builtin_bit_cast(uint2, v0), u1 = __builtin_bit_cast(uint2, v1);
  return make_uint4(u0.x, u0.y, u1.x, u1.y);
}

// f32 operand: lane l takes column c0 + (l & 15) of pixel row ks + (l >> 4)
template <int ROWB, int CG>
__device__ __forceinline__ float frag_f32(const char* tile, int ks, int c0, int lane) {
  const int r = ks + (lane >> 4), col = c0 + (lane & 15);
  const int chunk = col >> 2;
  return *reinterpret_cast<const float*>(tile + r * ROWB + ((chunk ^ swz_row<4, CG>(r)) << 4) + (col & 3) * 4);
}

// BM x BN tile of dW, 4 waves in a 2 x 2 grid, BP pixels per LDS stage, S-slot ring; KG such
// groups take pixel stages kg, kg + KG, .. (lockstep: one workgroup barrier per round)
template <typename T, int BM, int BN, int S, int KG>
__global__ __launch_bounds__(256 * KG) void conv_wgrad_kernel(WgradGeom g) {
  constexpr int ES = static_cast<int>(sizeof(T));
  constexpr int E = 16 / ES;
  constexpr int BP = ES == 2 ? POSU_WG_BP2 : 32;
  constexpr int RG = BM * ES, RX = BN * ES;  // LDS row bytes
  constexpr int CGG = RG / 16, CGX = RX / 16;
  constexpr int G_BYTES = BP * RG, STAGE = BP * (RG + RX);
  constexpr int DG = G_BYTES / 4096, DX = BP * RX / 4096;  // DMAs per thread per stage
  constexpr int WTM = BM / 2, WTN = BN / 2, TM = WTM / 16, TN = WTN / 16;
  constexpr int KSTEP = WOp<T>::KSTEP;
  static_assert(DG >= 1 && DX >= 1 && DG * 4096 == G_BYTES && DX * 4096 == BP * RX, "tile / DMA split");
  static_assert(S >= 2 && S <= 4 && (DG + DX) * (S - 2) < 64, "vmcnt range");
  static_assert(KG == 1 || KG * S * STAGE >= 4 * BM * BN, "the groups' tiles fit in the rings");
  __shared__ __attribute__((aligned(16))) char smem[KG * S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int kg = __builtin_amdgcn_readfirstlane(tid >> 8), wid = (tid >> 6) & 3;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware order: consecutive tile ids on one XCD (its L2 holds the shared G rows)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = wg % g.ntiles;
  const int rest = wg / g.ntiles;
  const int mt = rest % g.mtiles;
  const int split = rest / g.mtiles;
  const int m0 = mt * BM, n0 = nt * BN;
  const int pbeg = split * g.pps;
  const int pend = min(g.P, pbeg + g.pps);

  const u32x4 grs = make_srd(g.g, g.P * g.M * ES);
  const u32x4 xrs = make_srd(g.x, g.N * g.H * g.W * g.C * ES);
  // this group's ring
  char* const ring = smem + kg * S * STAGE;
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)ring));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));

  // per-thread DMA slots: G slot d covers tile bytes (4d + wid) KiB + 16 lane
  int grow[DG], gcol[DG];
#pragma unroll
  for (int d = 0; d < DG; ++d) {
    const int byte = (4 * d + wid) * 1024 + 16 * lane;
    const int row = byte / RG, pc = (byte % RG) / 16;
    grow[d] = row;
    const int col = m0 + ((pc ^ swz_row<ES, CGG>(row)) * E);
    gcol[d] = col < g.M ? col : -1;
  }
  int xrow[DX], xkh[DX], xkw[DX], xci[DX];
#pragma unroll
  for (int d = 0; d < DX; ++d) {
    const int byte = (4 * d + wid) * 1024 + 16 * lane;
    const int row = byte / RX, pc = (byte % RX) / 16;
    xrow[d] = row;
    const int k = n0 + (pc ^ swz_row<ES, CGX>(row)) * E;
    if (k < g.K) {
      const int tap = k >> g.logC;
      xkh[d] = tap / g.KW;
      xkw[d] = tap - xkh[d] * g.KW;
      xci[d] = k & (g.C - 1);
    } else {
      xkh[d] = -(1 << 28);  // never inside the image
      xkw[d] = 0;
      xci[d] = 0;
    }
  }

  const int nst_all = (pend - pbeg + BP - 1) / BP;
  // this group's stages: kg, kg + KG, ..; local stage i is global stage kg + KG i
  const int nst = nst_all > kg ? (nst_all - kg + KG - 1) / KG : 0;
  const int rounds = (nst_all + KG - 1) / KG;

#define POSU_WG_DMA(ST, BUF)                                                                        \
  {                                                                                                 \
    const int pb = pbeg + (kg + KG * (ST)) * BP;                                                    \
    const unsigned Gs_ = lds0 + (BUF) * STAGE + wid_u * 1024;                                       \
    const unsigned Xs_ = lds0 + (BUF) * STAGE + G_BYTES + wid_u * 1024;                             \
    _Pragma("unroll") for (int d = 0; d < DG; ++d) {                                                \
      const int p = pb + grow[d];                                                                   \
      const int off = (p < pend && gcol[d] >= 0) ? (p * g.M + gcol[d]) * ES : kOOB;                 \
      dma16(grs, off, Gs_ + d * 4096);                                                              \
    }                                                                                               \
    _Pragma("unroll") for (int d = 0; d < DX; ++d) {                                                \
      const int p = pb + xrow[d];                                                                   \
      int off = kOOB;                                                                               \
      if (p < pend) {                                                                               \
        const int n = fdiv(p, g.div_hw), rem = p - n * g.Ho * g.Wo;                                 \
        const int oy = fdiv(rem, g.div_w), ox = rem - oy * g.Wo;                                    \
        const int hi = oy * g.stride - g.pad + xkh[d], wi = ox * g.stride - g.pad + xkw[d];         \
        if (static_cast<unsigned>(hi) < static_cast<unsigned>(g.H) &&                               \
            static_cast<unsigned>(wi) < static_cast<unsigned>(g.W))                                 \
          off = (((n * g.H + hi) * g.W + wi) * g.C + xci[d]) * ES;                                  \
      }                                                                                             \
      dma16(xrs, off, Xs_ + d * 4096);                                                              \
    }                                                                                               \
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // S-slot ring: stages st+1 .. st+S-2 stay in flight while stage st is consumed; the
  // barrier publishes stage st and frees slot (st - 1) % S for stage st + S - 1
  for (int s0 = 0; s0 < S - 1 && s0 < nst; ++s0) POSU_WG_DMA(s0, s0);
  for (int st = 0; st < rounds; ++st) {
    // a group with no stage left this round still joins the round's barrier
    if (st < nst) vm_wait_stages<DG + DX>(min(S - 2, nst - 1 - st));
    wg_barrier();
    if (st >= nst) continue;
    if (st + S - 1 < nst) POSU_WG_DMA(st + S - 1, (st + S - 1) % S);
    const char* Gs = ring + (st % S) * STAGE;
    const char* Xs = Gs + G_BYTES;
#pragma unroll
    for (int ks = 0; ks < BP; ks += KSTEP) {
      if constexpr (ES == 2) {
        uint4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_tr16<RG, CGG>(Gs, ks, wm * WTM + i * 16, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag_tr16<RX, CGX>(Xs, ks, wn * WTN + j * 16, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) WOp<T>::mma(acc[i][j], bfr[j], af[i]);  // D[n][m]
      } else {
        float af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_f32<RG, CGG>(Gs, ks, wm * WTM + i * 16, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag_f32<RX, CGX>(Xs, ks, wn * WTN + j * 16, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) WOp<T>::mma(acc[i][j], bfr[j], af[i]);
      }
    }
  }
#undef POSU_WG_DMA

  if constexpr (KG > 1) {
    // groups 1 .. KG-1 hand their tiles to group 0 through the (now idle) rings, lane-major per
    // wave (16-B per lane and fragment); group 0 adds them in group order
    wg_barrier();
    float4* xch = reinterpret_cast<float4*>(smem);
    if (kg > 0) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          xch[(((kg - 1) * 4 + wid) * TM * TN + i * TN + j) * 64 + lane] =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    wg_barrier();
    if (kg > 0) return;
#pragma unroll
    for (int h = 1; h < KG; ++h)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const float4 v = xch[(((h - 1) * 4 + wid) * TM * TN + i * TN + j) * 64 + lane];
          acc[i][j][0] += v.x;
          acc[i][j][1] += v.y;
          acc[i][j][2] += v.z;
          acc[i][j][3] += v.w;
        }
  }
  // lane holds dW[m0 + .. + (lane & 15)][n .. n+3]: one 16-B store per fragment
  float* out = g.part + static_cast<size_t>(split) * g.Mpad * g.Npad;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int m = m0 + wm * WTM + i * 16 + (lane & 15);
      const int n = n0 + wn * WTN + j * 16 + 4 * (lane >> 4);
      *reinterpret_cast<float4*>(out + static_cast<size_t>(m) * g.Npad + n) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
}

// dW (parameter layout [M][Creal][KH][KW], f32) = sum over splits, in split order.  One thread per
// float4 column (m, k .. k+3) of the partial tiles: its `splits` loads in flight together (the
// partials were just written: the pass is latency-bound), summed in split order, scattered into
// the parameter layout.  (Round 4's kernel spread a row's 64 columns over 16 split lanes per
// block -- M * K / 64 blocks, 37 k for layer4's 3x3 -- and took 1.2 ms per training step in all.)
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int splits, int Mpad,
                                                           int Npad, int M, int K, int C, int Creal, int KH, int KW,
                                                           float* __restrict__ out) {
  const int kq = K / 4;
  const long long t = blockIdx.x * 256LL + threadIdx.x;
  if (t >= static_cast<long long>(M) * kq) return;
  const int m = static_cast<int>(t / kq), k = 4 * static_cast<int>(t - static_cast<long long>(m) * kq);
  const size_t stride = static_cast<size_t>(Mpad) * Npad;
  const float* src = part + static_cast<size_t>(m) * Npad + k;
  float4 a = *reinterpret_cast<const float4*>(src);
#pragma unroll 8
  for (int sp = 1; sp < splits; ++sp) {
    const float4 v = *reinterpret_cast<const float4*>(src + sp * stride);
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  }
  const float r[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int kk = k + e, tap = kk / C, ci = kk - tap * C;
    if (ci < Creal) {
      const int kh = tap / KW, kw = tap - kh * KW;
      out[((static_cast<size_t>(m) * Creal + ci) * KH + kh) * KW + kw] = r[e];
    }
  }
}

// blocks per weight-gradient launch (tiles x pixel splits): one per CU.  Every block writes an
// f32 partial tile, so more blocks cost partial traffic (2 x 67 MB at 1024 blocks); measured
// per training step (weight gradients on the side stream): 128 blocks 23.06 ms, 192 22.21,
// 256 21.97, 384 22.03, 512 22.12, 1024 22.76, 2048 23.69
#ifndef POSU_WG_BLOCKS
#define POSU_WG_BLOCKS 128
#endif
constexpr int kWgradBlocks = POSU_WG_BLOCKS;

template <typename T, int BM, int BN>
void launch_wgrad(WgradGeom& g, hipStream_t s) {
  constexpr int ES = static_cast<int>(sizeof(T));
  constexpr int BP = ES == 2 ? POSU_WG_BP2 : 32;
  g.mtiles = (g.M + BM - 1) / BM;
  g.ntiles = (g.K + BN - 1) / BN;
  g.Mpad = g.mtiles * BM;
  g.Npad = g.ntiles * BN;
  const int tiles = g.mtiles * g.ntiles;
  const int pst = (g.P + BP - 1) / BP;
  int splits = (kWgradBlocks + tiles - 1) / tiles;
  splits = std::max(1, std::min(splits, pst));
  const int stages_per_split = (pst + splits - 1) / splits;
  g.pps = stages_per_split * BP;
  g.splits = (g.P + g.pps - 1) / g.pps;
  hipLaunchKernelGGL((conv_wgrad_kernel<T, BM, BN, kWgSlots, kWgKG>), dim3(tiles * g.splits), dim3(256 * kWgKG), 0, s,
                     g);
}

template <typename T>
void launch_wgrad_t(WgradGeom& g, hipStream_t s) {
  if (g.M <= 64) launch_wgrad<T, 64, 128>(g, s);
  else launch_wgrad<T, 128, 128>(g, s);
}

int wgrad_part_floats(int dtype, int M, int K, int P) {
  (void)dtype;
  (void)P;
  const int BM = M <= 64 ? 64 : 128;
  const long long mp = static_cast<long long>((M + BM - 1) / BM) * BM;
  const long long np = static_cast<long long>((K + 127) / 128) * 128;
  // splits <= ceil(kWgradBlocks / tiles) + 1: the partial buffer bound below is what the
  // launcher can use
  const long long tiles = (mp / BM) * (np / 128);
  const long long splits = (kWgradBlocks + tiles - 1) / tiles + 1;
  const long long n = splits * mp * np;
  return n > (1LL << 31) - 1 ? -1 : static_cast<int>(n);
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" long long posu_conv2d_wgrad_workspace(int dtype, int N, int H, int W, int C, int Cout, int KH, int KW,
                                                 int stride, int pad) {
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  const int n = wgrad_part_floats(dtype, Cout, KH * KW * C, N * Ho * Wo);
  return n < 0 ? -1 : static_cast<long long>(n) * 4;
}

extern "C" int posu_conv2d_wgrad(int dtype, const void* dy, const void* x, int N, int H, int W, int C, int Creal,
                                 int Cout, int KH, int KW, int stride, int pad, float* dw, void* workspace,
                                 long long workspace_bytes, void* stream) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16 || dtype == POSU_F32,
               "posu_conv2d_wgrad: dtype must be F32, BF16 or F16");
  POSU_REQUIRE(dy && x && dw && workspace, "posu_conv2d_wgrad: null pointer");
  POSU_REQUIRE(N > 0 && H > 0 && W > 0 && Cout > 0 && KH > 0 && KW > 0 && stride > 0 && pad >= 0,
               "posu_conv2d_wgrad: bad shape");
  POSU_REQUIRE(C >= 8 && ilog2(C) >= 0 && Creal > 0 && Creal <= C, "posu_conv2d_wgrad: C must be a power of two >= 8");
  const int ES = dtype == POSU_F32 ? 4 : 2;
  POSU_REQUIRE(Cout % (16 / ES) == 0, "posu_conv2d_wgrad: Cout must be a multiple of 16 bytes");
  WgradGeom g{};
  g.g = dy;
  g.x = x;
  g.part = static_cast<float*>(workspace);
  g.N = N;
  g.H = H;
  g.W = W;
  g.C = C;
  g.logC = ilog2(C);
  g.Ho = (H + 2 * pad - KH) / stride + 1;
  g.Wo = (W + 2 * pad - KW) / stride + 1;
  POSU_REQUIRE(g.Ho > 0 && g.Wo > 0, "posu_conv2d_wgrad: empty output grid");
  g.P = N * g.Ho * g.Wo;
  g.M = Cout;
  g.K = KH * KW * C;
  g.KH = KH;
  g.KW = KW;
  g.stride = stride;
  g.pad = pad;
  g.div_hw = make_fastdiv(g.Ho * g.Wo);
  g.div_w = make_fastdiv(g.Wo);
  POSU_REQUIRE(static_cast<long long>(g.P) * Cout * ES < (1LL << 31) - 256 &&
                   static_cast<long long>(N) * H * W * C * ES < (1LL << 31) - 256,
               "posu_conv2d_wgrad: operands exceed the 2 GiB buffer-descriptor range");
  const long long need = posu_conv2d_wgrad_workspace(dtype, N, H, W, C, Cout, KH, KW, stride, pad);
  POSU_REQUIRE(need > 0 && workspace_bytes >= need, "posu_conv2d_wgrad: workspace too small");
  hipStream_t s = as_stream(stream);
  if (dtype == POSU_BF16) launch_wgrad_t<uint16_t>(g, s);
  else if (dtype == POSU_F16) launch_wgrad_t<f16_t>(g, s);
  else launch_wgrad_t<float>(g, s);
  if (int st = check_launch("posu_conv2d_wgrad")) return st;
  const long long cols = static_cast<long long>(Cout) * (g.K / 4);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(static_cast<unsigned>((cols + 255) / 256)), dim3(256), 0, s, g.part,
                     g.splits, g.Mpad, g.Npad, Cout, g.K, C, Creal, KH, KW, dw);
  return check_launch("posu_conv2d_wgrad");
}
