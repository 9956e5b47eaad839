// Implicit-GEMM convolution on CDNA4 MFMA, NHWC activations.
//
// GEMM view of one launch:  rows m = output pixels (n, oy, ox) of the launch grid,
//                           cols   = output channels,
//                           k      = (kh, kw, ci) taps of the input window.
// A[m][k] is gathered on the fly from the NHWC input (16-byte channel chunks,
// out-of-window taps read as zeros through a buffer descriptor), B[k][co] is the
// packed weight [CoutPad][Kpad] (K contiguous, zero padded).
//
// Block tile BM x BN (BM in {64, 128}, BN in {64, 128}), K-tile of 128 bytes per row
// (64 bf16 / 32 f32), 256 threads = 4 waves in a 2x2 grid, each wave owning a
// (BM/2) x (BN/2) accumulator tile made of 16x16 MFMA tiles:
//   bf16: v_mfma_f32_16x16x32_bf16 (one 16-B chunk per lane = one MFMA k-step)
//   f32 : v_mfma_f32_16x16x4_f32   (one 16-B chunk per lane = four MFMA k-steps;
//         the k order inside a chunk is permuted identically for A and B, which
//         leaves the sum unchanged)
// Pipeline: global->register prefetch of K-tile t+1 while the MFMAs of tile t run
// out of LDS buffer t&1; the registers are written to the other LDS buffer after
// the MFMAs; one barrier per K-tile.  LDS rows are 128 B with the 16-B chunk index
// XOR-swizzled by (row>>1)&7, which makes the 16-lane ds_read_b128 groups of the
// fragment reads conflict-free.
//
// DUAL variant (Bottleneck tail with a downsample branch, pose_resnet.py:90-99,
// 136-141): two 1x1 sources share one accumulator,
//   y = act( [W3*s3 | Wd*sd] . [conv2_out(m) ; block_in(n, oy*s, ox*s)] + (b3 + bd) ),
// so the downsample output is never written to / re-read from HBM.
//
// Epilogue: residual chunks are prefetched into registers first; the accumulators
// (+BN scale/shift) are staged through LDS as an f32 tile, then written as 16-byte
// NHWC chunks with residual add + ReLU, or as NCHW f32 heatmaps (+bias) for the
// final 1x1 layer (pose_resnet.py:126-132).
//
// ConvTranspose2d(4, s2, p1) runs as 4 sub-pixel 2x2 stride-1 convolutions, one per
// output parity class (py, px) = blockIdx.z: output (2*qy+py, 2*qx+px) reads inputs
// qy + py - 1 + ty, qx + px - 1 + tx with the deconv tap (3-py-2ty, 3-px-2tx);
// the Python layer packs those taps per class.
#include <type_traits>

#include "gemm_common.h"

namespace posu {
namespace {

struct ConvGeom {
  const void* x;
  const void* x2;  // DUAL: second 1x1 source
  const void* w;
  const float* scale;
  const float* shift;
  const void* res;
  void* y;
  int N, H, W, C, logC;
  int H2, W2, C2, stride2, K1;  // DUAL: source-2 geometry, K offset where it starts
  int Ho, Wo, M;                // launch grid: rows = N*Ho*Wo
  int Cout, CoutPad, K, Kpad;
  int KH, KW, stride, pad_h, pad_w;
  int relu;
  int up;            // 1: the input is read as its zero-upsampled image u[2i] = x[i], u[odd] = 0
                     //    (data gradient of a stride-2 convolution as a stride-1 one)
  int deconv;        // blockIdx.z = parity class
  int ostride;       // > 1: output pixel (oy, ox) is written at (ostride oy, ostride ox) of out_H x out_W
                     //      (data gradient of a 1x1 / stride-2 convolution, accumulated in place)
  int out_H, out_W;  // output tensor spatial dims
  int mode;          // 0: NHWC out (dtype), 1: NCHW f32 out, 2: f32 rows blocked by vblk columns
  int vblk;          // mode 2: out[(co / vblk)][m][co % vblk] (view-major heatmaps of a GEMM)
  // fused 1x1 head (mode 0, Cout == 256): hm[n][j][pix] = bias[j] + sum_c hw[j][c] relu(out[c])
  const void* hw;    // packed head weight [>= 16 rows][hkp] (dtype)
  const void* hw_lo;  // NULL, or the head weight's rounding residual (w - hw, rounded, same layout):
                      // the split-precision head (hi + lo operands on both sides, three MFMAs)
  const float* hbias;
  float* hm;
  int J, hkp;
  int mtiles, ntiles;
  int warm;          // > 0: workgroups 0 .. warm-1 touch the weights at their start (kernel comment)
  long long wseg;    // the weight tensor's 64-B segments (all parity classes)
};

// Weight warm-up (round 5, gemm_common.h warm_issue): layer4's 3x3 ran 59.4 us with its weights
// coming from HBM against 49.7 us with them re-read beforehand (tools/tile_micro.py --flush --touch,
// profiles/r05/tile_cold_touch_r5v.txt); with the warm-up the network ran 2.355-2.363 vs
// 2.405-2.413 ms (profiles/r05/weight_warmup_ab_r5y.txt).  (A side-stream prefetch launch inside
// the captured graph lost: its launches serialised with the network's, prefetch_ab_r5x.txt.)

template <int BM, int BN, int S>
constexpr int ring_bytes() {
  return S * (BM + BN) * 128;
}
// rows per epilogue pass: the f32 [rows][BN+4] staging tile must fit in the ring
template <int BM, int BN, int S>
constexpr int pass_rows() {
  return (BM * (BN + 4) * 4 <= ring_bytes<BM, BN, S>())         ? BM
         : ((BM / 2) * (BN + 4) * 4 <= ring_bytes<BM, BN, S>()) ? BM / 2
                                                                 : BM / 4;
}

// residual-add launches with at most this many K-tiles load their residual before the
// operand fetch (direct epilogue), so its HBM latency overlaps the main loop
constexpr int kEarlyNK = 8;

// BM x BN tile, NW waves (NT = 64*NW threads) in a WGM x (NW/WGM) grid, S-slot ring.
// SG: eight-wave tiles with waves 4-7 staggered by half a K-tile (two-slot ring).
// HD: the instance that carries the fused 1x1 head in its epilogue (256x256 eight-wave tiles
// only).  Its registers (head accumulators and weight fragments) made the 256x256 instance
// spill 36 VGPRs to scratch in every launch until round 4, head or not; the plain instances
// no longer hold that code (228 VGPRs, no scratch).
// KS (round 5): eight waves as two K groups of four -- the K-tiles come in pairs (two LDS sub-slots
// per ring slot), group g multiplies K-tile 2t + g of every pair over the WHOLE BM x BN tile, and
// the two partial sums meet in LDS at the end (each group adds the other's half of the m-tiles and
// stores that half).  Per wave 64 x 64 (TM = TN = 4) instead of the 64 x 32 of the eight-wave
// 128 x 128 tile: half the LDS fragment reads per MFMA, for grids of few tiles (layer4's M = 8192
// convs: 256 tiles of 128 x 128, one per CU).  The K order differs from the other tiles (the even
// and the odd K-tiles summed apart, then added), so KS results are not bit-identical to them.
template <typename T, int BM, int BN, int NW, int WGM, int S, bool DUAL, bool SG = false, bool HD = false,
          bool KS = false>
__global__ __launch_bounds__(NW * 64) void conv_igemm_kernel(ConvGeom g) {
  using O = Op<T>;
  constexpr int NT = NW * 64;
  constexpr int E = O::E;
  constexpr int ES = static_cast<int>(sizeof(T));
  // split fp16: K-tiles of [hi 32 | lo 32] halves, three MFMAs per K-tile and fragment pair;
  // outputs / residuals are (hi, lo) pairs, ocs halves per output pixel
  constexpr bool SPL = O::SPLIT;
  // (round 6: the split dtype staggers too -- the lagging waves hold a K-tile's third product, hi(w).lo(x))
  constexpr int BK = 8 * E;                   // 128-byte LDS rows
  static_assert(!KS || (NW == 8 && S == 2 && !SG && !HD && E == 8), "K groups: eight waves, two slots of pairs");
  constexpr int NWG = KS ? NW / 2 : NW;       // waves per K group
  constexpr int SL = KS ? 2 * S : S;          // LDS K-tile slots (KS: a pair per ring slot)
  constexpr int WGN = NWG / WGM;              // wave grid WGM x WGN (of a K group)
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int ROWS = NW * 8;                // LDS rows filled per DMA round (1 KiB per wave)
  constexpr int RA = BM / ROWS, RB = BN / ROWS;
  constexpr int ND = RA + RB;                 // DMA instructions per thread per K-tile
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int PR = pass_rows<BM, BN, SL>();
  constexpr bool PRELOAD = TM + TN <= 8;  // both k-steps' fragments fit the VGPR budget
  static_assert(S >= 1 && S <= 4, "1..4 stages");
  static_assert(ND * (S - 2) < 64, "vmcnt range");
  static_assert(PR * (BN + 4) * 4 <= ring_bytes<BM, BN, SL>(), "epilogue staging must fit in the ring");
  static_assert(RA * ROWS == BM && RB * ROWS == BN, "tile rows must be a multiple of 8 * waves");
  __shared__ __attribute__((aligned(16))) char smem[ring_bytes<BM, BN, SL>()];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int grp = KS ? wid / NWG : 0, wl = KS ? wid % NWG : wid;   // K group, wave in the group
  const int wm = wl / WGN, wn = wl % WGN;
  const int r16 = lane & 15, q = lane >> 4;
  // tile row of the wave's m-tile i / tile column of its n-tile j
  auto rowA = [&](int i) { return wm * WTM + i * 16; };
  auto colB = [&](int j) { return wn * WTN + j * 16; };

  // XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a
  // contiguous run of tiles so neighbouring tiles (same A rows) share its L2.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  // tile id -> (m-tile, [deconv parity class,] n-tile), n fastest; the 4 parity
  // classes of one m-tile are adjacent so their overlapping input windows are read
  // from the same XCD's L2 instead of once per class from HBM
  const int nt = wg % g.ntiles;
  const int rest = wg / g.ntiles;
  const int mt = g.deconv ? rest >> 2 : rest;
  const int m0 = mt * BM, n0 = nt * BN;

  int pad_h = g.pad_h, pad_w = g.pad_w, oy_off = 0, ox_off = 0, osc = g.ostride > 1 ? g.ostride : 1;
  const T* __restrict__ wp = reinterpret_cast<const T*>(g.w);
  if (g.deconv) {
    const int cls = rest & 3, py = cls >> 1, px = cls & 1;
    pad_h = 1 - py;
    pad_w = 1 - px;
    oy_off = py;
    ox_off = px;
    osc = 2;
    wp += static_cast<size_t>(cls) * g.CoutPad * g.Kpad;
  }
  const T* __restrict__ xp = reinterpret_cast<const T*>(g.x);
  const u32x4 xrs = make_srd(xp, g.N * g.H * g.W * g.C * ES);
  const u32x4 wrs = make_srd(wp, g.CoutPad * g.Kpad * ES);
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));

  // ---- LDS-DMA staging.  One buffer_load_dwordx4 ... lds per wave writes 1 KiB =
  // 8 LDS rows x 8 chunks, lane l at byte 16*l: row (tid >> 3) + ROWS*i, physical
  // chunk tid & 7.  The XOR swizzle of the fragment reads is applied on the SOURCE:
  // that lane fetches logical chunk cL = (tid & 7) ^ ((row >> 1) & 7), which is the
  // same for every i because ROWS*i does not touch bits 1..3 of the row.
  const int cL = (tid & 7) ^ ((tid >> 4) & 7);
  auto drow = [&](int i) { return (tid >> 3) + ROWS * i; };
  const int HoWo = g.Ho * g.Wo;
  const int ocs = SPL ? 2 * g.Cout : g.Cout;  // elements per output pixel
  int hb[RA], wb[RA], nb[RA];   // generic window gather
  int o1[RA], o2[RA];           // DUAL: byte offsets of the two 1x1 sources
  u32x4 x2rs = xrs;
  if constexpr (DUAL) x2rs = make_srd(g.x2, g.N * g.H2 * g.W2 * g.C2 * ES);
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int m = m0 + drow(i);
    if (m < g.M) {
      const int n = m / HoWo, rem = m - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      hb[i] = oy * g.stride - pad_h;
      wb[i] = ox * g.stride - pad_w;
      nb[i] = n * g.H * g.W * g.C;
      if constexpr (DUAL) {
        o1[i] = (m * g.C + cL * E) * ES;
        o2[i] = (((n * g.H2 + oy * g.stride2) * g.W2 + ox * g.stride2) * g.C2 + cL * E) * ES;
      }
    } else {
      hb[i] = -(1 << 28);
      wb[i] = 0;
      nb[i] = 0;
      if constexpr (DUAL) {
        o1[i] = kOOB;
        o2[i] = kOOB;
      }
    }
  }
  // K-tile -> (kh, kw, ci) of this thread's chunk.  Three regimes:
  //  tap_uniform: C % BK == 0, one tap per K-tile (all 3x3 / 1x1 / deconv layers);
  //  row_uniform: KW*C == BK, one kernel row per K-tile (space-to-depth stem);
  //  generic    : per-chunk tap decode (C = 8 direct stem, f32 stem).
  const bool tap_uniform = (g.C % BK) == 0;
  const bool fast_gather = tap_uniform && g.up == 0;
  const bool row_fast = !tap_uniform && g.KW * g.C == BK && g.up == 0;
  int rbase[RA];   // row_fast: window row origin + this lane's (kw, ci) column
  bool wok[RA];
  {
    const int kwl = (cL * E) >> g.logC, cil = (cL * E) & (g.C - 1);
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      wok[i] = static_cast<unsigned>(wb[i] + kwl) < static_cast<unsigned>(g.W);
      rbase[i] = static_cast<int>(static_cast<unsigned>(nb[i]) +
                                  (static_cast<unsigned>(hb[i]) * g.W + static_cast<unsigned>(wb[i] + kwl)) * g.C +
                                  cil);
    }
  }
  int pbase[RA];  // element offset of row i's window origin + this lane's channel chunk
#pragma unroll
  for (int i = 0; i < RA; ++i)  // unsigned: rows past M carry a huge negative hb (never dereferenced)
    pbase[i] = static_cast<int>(static_cast<unsigned>(nb[i]) +
                                (static_cast<unsigned>(hb[i]) * g.W + static_cast<unsigned>(wb[i])) * g.C + cL * E);
  const bool row_uniform = !tap_uniform && g.KW * g.C == BK;
  const int kw_row = (cL * E) >> g.logC, ci_row = (cL * E) & (g.C - 1);
  const int nk = g.Kpad / BK;
  const int wbrow = (n0 + (tid >> 3)) * g.Kpad + cL * E;  // weight row offset (elements) for i = 0

  // global -> LDS (async DMA) for K-tile KT into ring slot BUF: exactly ND dma16 per thread
#define POSU_DMA_TILE(KT, BUF)                                                                      \
  {                                                                                                 \
    const int kbase = (KT) * BK;                                                                    \
    const unsigned As_ = lds0 + (BUF) * STAGE + wid_u * 1024;                                       \
    const unsigned Bs_ = As_ + A_BYTES;                                                             \
    if constexpr (DUAL) {                                                                           \
      const bool first = kbase < g.K1;                                                              \
      _Pragma("unroll") for (int i = 0; i < RA; ++i) {                                              \
        const int o = first ? o1[i] : o2[i];                                                        \
        const int off = o == kOOB ? kOOB : o + (first ? kbase : kbase - g.K1) * ES;                 \
        dma16(first ? xrs : x2rs, off, As_ + i * NW * 1024);                                        \
      }                                                                                             \
    } else {                                                                                        \
      int kh, kw, ci;                                                                               \
      bool kvalid = true;                                                                           \
      if (fast_gather) {                                                                            \
        /* one tap per K-tile, no zero-upsampling: row base + a wave-uniform tap offset */          \
        const int tap = kbase >> g.logC;                                                            \
        const int th = tap / g.KW, tw = tap - th * g.KW;                                            \
        const int toff = (th * g.W + tw) * g.C + (kbase & (g.C - 1));                               \
        _Pragma("unroll") for (int i = 0; i < RA; ++i) {                                            \
          const bool ok = static_cast<unsigned>(hb[i] + th) < static_cast<unsigned>(g.H) &&         \
                          static_cast<unsigned>(wb[i] + tw) < static_cast<unsigned>(g.W);           \
          const int off = ok ? (pbase[i] + toff) * ES : kOOB;                                       \
          dma16(xrs, off, As_ + i * NW * 1024);                                                     \
        }                                                                                           \
      } else if (row_fast) {                                                                        \
        /* one kernel row per K-tile (space-to-depth stem): lane column fixed per row */            \
        const int roff = (KT) * g.W * g.C;                                                          \
        _Pragma("unroll") for (int i = 0; i < RA; ++i) {                                            \
          const bool ok = wok[i] && static_cast<unsigned>(hb[i] + (KT)) < static_cast<unsigned>(g.H); \
          const int off = ok ? (rbase[i] + roff) * ES : kOOB;                                       \
          dma16(xrs, off, As_ + i * NW * 1024);                                                     \
        }                                                                                           \
      } else {                                                                                      \
      if (tap_uniform) {                                                                            \
        const int tap = kbase >> g.logC;                                                            \
        kh = tap / g.KW;                                                                            \
        kw = tap - kh * g.KW;                                                                       \
        ci = (kbase & (g.C - 1)) + cL * E;                                                          \
      } else if (row_uniform) {                                                                     \
        kh = (KT);                                                                                  \
        kw = kw_row;                                                                                \
        ci = ci_row;                                                                                \
      } else {                                                                                      \
        const int k = kbase + cL * E;                                                               \
        const int tap = k >> g.logC;                                                                \
        kh = tap / g.KW;                                                                            \
        kw = tap - kh * g.KW;                                                                       \
        ci = k & (g.C - 1);                                                                         \
        kvalid = k < g.K;                                                                           \
      }                                                                                             \
      _Pragma("unroll") for (int i = 0; i < RA; ++i) {                                              \
        const int hl = hb[i] + kh, wl = wb[i] + kw;                                                 \
        const int hi = hl >> g.up, wi = wl >> g.up;                                                 \
        const bool ok = kvalid && ((hl | wl) & g.up) == 0 &&                                        \
                        static_cast<unsigned>(hi) < static_cast<unsigned>(g.H) &&                   \
                        static_cast<unsigned>(wi) < static_cast<unsigned>(g.W);                     \
        const int off = ok ? (nb[i] + (hi * g.W + wi) * g.C + ci) * ES : kOOB;                      \
        dma16(xrs, off, As_ + i * NW * 1024);                                                       \
      }                                                                                             \
      }                                                                                             \
    }                                                                                               \
    _Pragma("unroll") for (int i = 0; i < RB; ++i)                                                  \
      dma16(wrs, (wbrow + ROWS * i * g.Kpad + kbase) * ES, Bs_ + i * NW * 1024);                    \
  }
  // MFMAs over one LDS K-tile.  Operands are swapped (A = weights, B = pixels), so a
  // lane's accumulator holds 4 consecutive output channels of one pixel, staged into
  // LDS with one 16-B write.
#define POSU_COMPUTE(BUF)                                                                           \
  {                                                                                                 \
    const char* As_ = smem + (BUF) * STAGE;                                                         \
    const char* Bs_ = As_ + A_BYTES;                                                                \
    if constexpr (SPL) {                                                                            \
      /* k-step 0 = the hi halves, k-step 1 = the lo halves of the same 32 k: w.x as */             \
      /* hi.hi + lo(w).hi(x) + hi(w).lo(x); at most TM + 2 TN fragments live */                     \
      uint4 x0[TM], w0[TN];                                                                         \
      _Pragma("unroll") for (int j = 0; j < TN; ++j)                                                \
        w0[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, q));             \
      _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                \
        x0[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, q));             \
      _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                \
        _Pragma("unroll") for (int j = 0; j < TN; ++j) O::mma(acc[i][j], w0[j], x0[i]);             \
      {                                                                                             \
        uint4 w1[TN];                                                                               \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                              \
          w1[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, 4 + q));       \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          _Pragma("unroll") for (int j = 0; j < TN; ++j) O::mma(acc[i][j], w1[j], x0[i]);           \
      }                                                                                             \
      {                                                                                             \
        uint4 x1[TM];                                                                               \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          x1[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, 4 + q));       \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          _Pragma("unroll") for (int j = 0; j < TN; ++j) O::mma(acc[i][j], w0[j], x1[i]);           \
      }                                                                                             \
    } else if constexpr (PRELOAD) {                                                                 \
      /* both k-steps' fragments first: the MFMAs then run back to back while the */                \
      /* second half's reads land, instead of stalling on them mid-tile */                          \
      uint4 af[2][TM], bfr[2][TN];                                                                  \
      _Pragma("unroll") for (int cb = 0; cb < 2; ++cb) {                                            \
        const int c = 4 * cb + q;                                                                   \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                              \
          bfr[cb][j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, c));      \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          af[cb][i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, c));       \
      }                                                                                             \
      _Pragma("unroll") for (int cb = 0; cb < 2; ++cb)                                              \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          _Pragma("unroll") for (int j = 0; j < TN; ++j) O::mma(acc[i][j], bfr[cb][j], af[cb][i]);  \
    } else {                                                                                        \
      _Pragma("unroll") for (int cb = 0; cb < 2; ++cb) {                                            \
        const int c = 4 * cb + q;                                                                   \
        uint4 af[TM], bfr[TN];                                                                      \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          af[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, c));           \
        _Pragma("unroll") for (int j = 0; j < TN; ++j)                                              \
          bfr[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, c));          \
        _Pragma("unroll") for (int i = 0; i < TM; ++i)                                              \
          _Pragma("unroll") for (int j = 0; j < TN; ++j) O::mma(acc[i][j], bfr[j], af[i]);          \
      }                                                                                             \
    }                                                                                               \
  }

  // acc[i][j]: rows = channels of n-tile j (16 per MFMA tile), cols = pixels of m-tile i;
  // lane holds channels 4q..4q+3 of pixel r16
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Early residual prefetch (short-K Bottleneck tails): the residual chunks, in the direct
  // epilogue's lane layout, are loaded before the first operand DMA, so their HBM latency
  // overlaps the operand fetch instead of following the main loop.
  constexpr bool EARLY = E == 8 && TN % 2 == 0 && TM * TN <= 16 && !SPL && !KS;
  constexpr int ETM = EARLY ? TM : 1, ETP = EARLY ? TN / 2 : 1;
  const bool early = EARLY && g.res && g.mode == 0 && !g.hm && nk <= kEarlyNK;
  uint4 rve[ETM][ETP];
  auto out_pix = [&](int i, bool& mok) -> size_t {  // element offset of the pixel of row i
    const int m = m0 + rowA(i) + r16;
    mok = m < g.M;
    const int mm = mok ? m : 0;
    const int n = mm / HoWo, rem = mm - n * HoWo;
    const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
    return (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * ocs;
  };
  if constexpr (EARLY) {
    if (early) {
      const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
#pragma unroll
      for (int i = 0; i < ETM; ++i) {
        bool mok;
        const size_t pix = out_pix(i, mok);
#pragma unroll
        for (int jp = 0; jp < ETP; ++jp) {
          const int co = n0 + colB(2 * jp + (q & 1)) + 8 * (q >> 1);
          rve[i][jp] = make_uint4(0, 0, 0, 0);
          if (mok && co < g.Cout) rve[i][jp] = *reinterpret_cast<const uint4*>(rp + pix + co);
        }
      }
    }
  }

  // weight warm-up: this workgroup's segments requested now, consumed right after the first
  // K-tile DMAs are issued
  unsigned wv[kWarmLoads];
  warm_issue(wv, g.w, g.wseg, g.warm, NT);
  auto warm_done = [&] { warm_use(wv); };

  // S-slot ring, DMA running S-1 K-tiles ahead; per K-tile one counted vmcnt (the
  // K-tile being consumed has landed, up to S-2 younger tiles stay in flight) and one
  // barrier (makes the DMA visible to every wave and retires the slot the next DMA
  // overwrites, which every wave finished reading in the previous iteration)
  if constexpr (KS) {
    // K-tile pairs: pair t in slots 2 (t & 1) and 2 (t & 1) + 1, DMA'd by all eight waves one pair
    // ahead; group g multiplies the pair's K-tile 2t + g (a missing last odd K-tile is skipped)
    const int np = (nk + 1) / 2;
    POSU_DMA_TILE(0, 0);
    if (1 < nk) POSU_DMA_TILE(1, 1);
    warm_done();
    for (int t = 0; t < np; ++t) {
      vm_wait<0>();
      __syncthreads();
      if (t + 1 < np) {
        const int b = 2 * ((t + 1) & 1);
        POSU_DMA_TILE(2 * t + 2, b);
        if (2 * t + 3 < nk) POSU_DMA_TILE(2 * t + 3, b + 1);
      }
      if (2 * t + grp < nk) POSU_COMPUTE(2 * (t & 1) + grp);
    }
    // the two groups' partial sums: group 0 keeps m-tiles 0 .. TM/2 - 1, group 1 the rest; each hands
    // the other its half through LDS (f32, lane-major) and adds the half it keeps (a + b == b + a)
    __syncthreads();  // every wave is done reading the ring
    constexpr int HT = TM / 2, PER = HT * TN * 64;   // f32x4 per wave's hand-off
    f32x4* xch = reinterpret_cast<f32x4*>(smem);
    auto give = [&](auto g0) {
      constexpr bool G0 = decltype(g0)::value;
#pragma unroll
      for (int i = 0; i < HT; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) xch[(G0 ? 0 : NWG) * PER + wl * PER + (i * TN + j) * 64 + lane] = acc[G0 ? HT + i : i][j];
    };
    auto take = [&](auto g0) {
      constexpr bool G0 = decltype(g0)::value;
#pragma unroll
      for (int i = 0; i < HT; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[G0 ? i : HT + i][j] += xch[(G0 ? NWG : 0) * PER + wl * PER + (i * TN + j) * 64 + lane];
    };
    if (grp == 0) give(std::true_type{});
    else give(std::false_type{});
    __syncthreads();
    if (grp == 0) take(std::true_type{});
    else take(std::false_type{});
  } else if constexpr (SG) {
    // Stagger (two-slot ring, one barrier per K-tile): waves 4-7 run half a K-tile behind
    // waves 0-3 -- they keep the second k-step's fragments of K-tile t in registers and
    // issue its MFMAs after the next barrier, while waves 0-3 wait for their first
    // fragment reads; every read still happens before the barrier that frees its slot.
    static_assert(S == 2 && NW == 8, "stagger: eight waves, two slots");
    const bool lag = wid_u >= 4;
    uint4 hA[TM], hB[TN];
    auto read = [&](const char* As_, const char* Bs_, int cb, uint4 (&a)[TM], uint4 (&b)[TN]) {
      const int c = 4 * cb + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, c));
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, c));
    };
    auto mma = [&](const uint4 (&a)[TM], const uint4 (&b)[TN]) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) O::mma(acc[i][j], b[j], a[i]);
    };
    // timing ablations (tools/igemm_ablations.sh; results wrong): POSU_IG_ABLATE bit 1 no
    // MFMA, 2 no vmcnt wait, 4 no operand DMA, 8 no LDS fragment reads
#ifndef POSU_IG_ABLATE
#define POSU_IG_ABLATE 0
#endif
    constexpr int ABL = POSU_IG_ABLATE;
    auto mmx = [&](const uint4 (&a)[TM], const uint4 (&b)[TN]) {
      if constexpr (ABL & 1) {
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][0][0] += __builtin_bit_cast(float, a[i].x ^ b[i % TN].y);
      } else {
        mma(a, b);
      }
    };
    auto rdx = [&](const char* As_, const char* Bs_, int cb, uint4 (&a)[TM], uint4 (&b)[TN]) {
      if constexpr (ABL & 8) {
#pragma unroll
        for (int i = 0; i < TM; ++i) a[i] = make_uint4(cb, i, 0, 0);
#pragma unroll
        for (int j = 0; j < TN; ++j) b[j] = make_uint4(j, cb, 0, 0);
      } else {
        read(As_, Bs_, cb, a, b);
      }
    };
    if constexpr (!(ABL & 4)) POSU_DMA_TILE(0, 0);
    warm_done();
    if (lag) __builtin_amdgcn_s_setprio(1);  // the lagging half wins issue arbitration (-2..-7 %)
    if constexpr (SPL) {
      // split fp16 (round 6): a K-tile's products are hi.hi and lo(w).hi(x) over the hi pixel
      // fragments, then hi(w).lo(x); the lagging waves keep the last one's operands (the lo pixel and
      // the hi weight fragments) and issue it after the next barrier, before the next K-tile's hi.hi
      // -- per accumulator the plain loop's sequence, so the results are bit-identical to it
      for (int kt = 0; kt < nk; ++kt) {
        vm_wait<0>();
        __syncthreads();
        if (kt + 1 < nk) POSU_DMA_TILE(kt + 1, (kt + 1) & 1);
        const char* As_ = smem + (kt & 1) * STAGE;
        const char* Bs_ = As_ + A_BYTES;
        if (lag && kt > 0) mma(hA, hB);
        uint4 af[TM], bfr[TN];
        read(As_, Bs_, 0, af, bfr);
        mma(af, bfr);
        {
          uint4 bl[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) bl[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, 4 + q));
          mma(af, bl);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) hA[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, 4 + q));
#pragma unroll
        for (int j = 0; j < TN; ++j) hB[j] = bfr[j];
        if (!lag) mma(hA, hB);
      }
    } else {
    for (int kt = 0; kt < nk; ++kt) {
      if constexpr (!(ABL & 2)) vm_wait<0>();
      __syncthreads();
      if constexpr (!(ABL & 4))
        if (kt + 1 < nk) POSU_DMA_TILE(kt + 1, (kt + 1) & 1);
      const char* As_ = smem + (kt & 1) * STAGE;
      const char* Bs_ = As_ + A_BYTES;
      uint4 af[TM], bfr[TN];
      if (lag && kt > 0) mmx(hA, hB);
      rdx(As_, Bs_, 0, af, bfr);
      mmx(af, bfr);
      rdx(As_, Bs_, 1, hA, hB);
      if (!lag) mmx(hA, hB);
    }
    }
    if (lag) mmx(hA, hB);
    if constexpr (ABL & 2) vm_wait<0>();
    __builtin_amdgcn_s_setprio(0);
  } else if constexpr (S == 1) {
    // single slot (short-K layers): a quarter of the LDS of a 2-slot ring, so more
    // blocks share a CU and one block's epilogue overlaps another's operand fetch
    for (int kt = 0; kt < nk; ++kt) {
      if (kt > 0) __syncthreads();  // every wave is done reading the slot
      POSU_DMA_TILE(kt, 0);
      if (kt == 0) warm_done();
      vm_wait<0>();
      __syncthreads();
      POSU_COMPUTE(0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < S - 1; ++s)
      if (s < nk) POSU_DMA_TILE(s, s);
    warm_done();
    for (int kt = 0; kt < nk; ++kt) {
      const int ahead = min(S - 2, nk - 1 - kt);  // younger K-tiles in flight
      if (S >= 4 && ahead >= 2) vm_wait<ND * (S >= 4 ? 2 : 0)>();
      else if (S >= 3 && ahead >= 1) vm_wait<ND * (S >= 3 ? 1 : 0)>();
      else vm_wait<0>();
      __syncthreads();
      if (kt + S - 1 < nk) POSU_DMA_TILE(kt + S - 1, (kt + S - 1) % S);
      POSU_COMPUTE(kt % S);
    }
  }
#undef POSU_DMA_TILE
#undef POSU_COMPUTE

  // ---- direct epilogue (NHWC outputs): each lane stores its 4
  // consecutive channels of one pixel straight from the accumulators (BN, residual,
  // ReLU applied in registers) -- no LDS round trip, no barriers
  // 256x256 tiles also carry the fused 1x1 head (pose_resnet.py:126-132, 203): each
  // wave's rounded outputs are already MFMA B fragments (8 consecutive channels of one
  // pixel per lane), so its partial heatmaps over its 64 channels are 2 MFMAs per m-tile;
  // the four column waves' partials are summed in LDS in a fixed order.
  constexpr bool HEAD256 = HD && BM == 256 && BN == 256 && NW == 8 && WGM == 2 && E == 8;
  static_assert(!HD || HEAD256, "the fused head runs on the 2-byte 256x256 eight-wave tile");
  if constexpr (SG && (POSU_IG_ABLATE & 16)) {  // timing ablation: no epilogue (results wrong)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }
  if constexpr (HEAD256) {  // the HD instance: launched only with g.hm set, no other epilogue
    T* __restrict__ yp = reinterpret_cast<T*>(g.y);
    const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
    constexpr int TP = TN / 2;
    {
        // fused head: pair jp outer, m-tile inner -- one pair's BN parameters and head fragments
        // are live at a time and each accumulator pair dies once consumed (the 256x256 head
        // instance spilled 38 VGPRs with m-tile outer); every hacc[i] still receives its MFMAs in
        // the same order (pair 0's, then pair 1's), so the heatmaps are unchanged
        const bool split = SPL || g.hw_lo != nullptr;  // the split dtype's head is always split
        const T* __restrict__ hwp = reinterpret_cast<const T*>(g.hw);
        const T* __restrict__ hwq = reinterpret_cast<const T*>(split ? g.hw_lo : g.hw);
        f32x4 hacc[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) hacc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const bool need_pix = yp != nullptr || rp != nullptr;
#pragma unroll
        for (int jp = 0; jp < TP; ++jp) {
          // 8 consecutive channels cp .. cp + 7 of this lane (all inside Cout or all past it)
          const int cp = n0 + colB(2 * jp + (q & 1)) + 8 * (q >> 1);
          const bool in = cp < g.Cout;
          const float4 one = make_float4(1.f, 1.f, 1.f, 1.f), zero = make_float4(0.f, 0.f, 0.f, 0.f);
          const float4 s0 = in && g.scale ? *reinterpret_cast<const float4*>(g.scale + cp) : one;
          const float4 s1 = in && g.scale ? *reinterpret_cast<const float4*>(g.scale + cp + 4) : one;
          const float4 h0 = in && g.shift ? *reinterpret_cast<const float4*>(g.shift + cp) : zero;
          const float4 h1 = in && g.shift ? *reinterpret_cast<const float4*>(g.shift + cp + 4) : zero;
          const float sc8[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sh8[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
          // joint r16's weights over this lane's 8 channels
          const size_t o = static_cast<size_t>(r16) * g.hkp + cp;
          const uint4 hw = *reinterpret_cast<const uint4*>(hwp + o);
          const uint4 hl = *reinterpret_cast<const uint4*>(hwq + o);
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int m = m0 + rowA(i) + r16;
            const bool mok = m < g.M;
            size_t pix = 0;
            if (need_pix) {
              const int mm = mok ? m : 0;
              const int n = mm / HoWo, rem = mm - n * HoWo;
              const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
              pix = (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * ocs;
            }
            float v[8], r[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][e]),
                                                               __float_as_uint(acc[i][2 * jp + 1][e]), false, false);
              v[e] = __uint_as_float(sw[0]);
              v[4 + e] = __uint_as_float(sw[1]);
            }
            if constexpr (SPL) {
              uint4 rh = make_uint4(0, 0, 0, 0), rl = rh;
              if (rp && mok && in) {
                rh = *reinterpret_cast<const uint4*>(rp + pix + split_ch(cp));
                rl = *reinterpret_cast<const uint4*>(rp + pix + split_ch(cp) + 32);
              }
              join8(rh, rl, r);
            } else {
              uint4 rv = make_uint4(0, 0, 0, 0);
              if (rp && mok && in) rv = *reinterpret_cast<const uint4*>(rp + pix + cp);
              O::load_vals(rv, r);
            }
            affine8<false>(v, sc8, sh8);
            if (rp) add8<false>(v, r);
            if (g.relu) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
            }
            const uint4 pk = O::store_vals(v);
            O::mma(hacc[i], hw, pk);  // rows = joints, cols = pixels
            uint4 pl = make_uint4(0, 0, 0, 0);
            if (split) {
              // the deconv output's rounding residual v - round(v) (exact in f32) rounded again: the
              // head sees v to 2 x the dtype's mantissa, its weights likewise (hi.hi + lo.hi + hi.lo)
              float vr[8], vl[8];
              O::load_vals(pk, vr);
#pragma unroll
              for (int e = 0; e < 8; ++e) vl[e] = v[e] - vr[e];
              pl = O::store_vals(vl);
              O::mma(hacc[i], hl, pk);
              O::mma(hacc[i], hw, pl);
            }
            if constexpr (SPL) {
              if (yp && mok) {
                *reinterpret_cast<uint4*>(yp + pix + split_ch(cp)) = pk;
                *reinterpret_cast<uint4*>(yp + pix + split_ch(cp) + 32) = pl;
              }
            } else {
              if (yp && mok) *reinterpret_cast<uint4*>(yp + pix + cp) = pk;
            }
          }
        }
        if constexpr (SG && (POSU_IG_ABLATE & 32)) {  // timing ablation: no head reduction / stores
#pragma unroll
          for (int i = 0; i < TM; ++i) asm volatile("" ::"v"(hacc[i]));
          return;
        }
        __syncthreads();  // the ring is no longer read: partial heatmaps [wn][joint][256 px]
        float* Hs = reinterpret_cast<float*>(smem);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) Hs[(wn * 16 + 4 * q + e) * BM + rowA(i) + r16] = hacc[i][e];
        __syncthreads();
        const int HWo = g.out_H * g.out_W;
        for (int idx = tid; idx < g.J * BM; idx += NT) {
          const int j = idx / BM, pl = idx - j * BM;
          const int m = m0 + pl;
          if (m >= g.M) continue;
          float sum = g.hbias ? g.hbias[j] : 0.f;
#pragma unroll
          for (int w4 = 0; w4 < 4; ++w4) sum += Hs[(w4 * 16 + j) * BM + pl];
          const int n = m / HoWo, rem = m - n * HoWo;
          const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
          g.hm[(static_cast<size_t>(n) * g.J + j) * HWo + (oy * osc + oy_off) * g.out_W + ox * osc + ox_off] = sum;
        }
        return;
      }
  } else if (E == 8 && TN % 2 == 0 && g.mode == 0 && !g.hm) {
    // 2-byte outputs: v_permlane16_swap pairs the n-tiles (j, j+1) so that every lane
    // holds 8 consecutive channels (16-B stores, half the store instructions):
    // lane (r16, q) gets n-tile j + (q & 1), channels 8 * (q >> 1) .. + 7 of pixel r16
    T* __restrict__ yp = reinterpret_cast<T*>(g.y);
    const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
    constexpr int TP = TN / 2;
    int cop[TP];
    float sc[TP][8], sh[TP][8];
#pragma unroll
    for (int jp = 0; jp < TP; ++jp) {
      // 8 consecutive channels, all inside Cout or all past it (Cout is a multiple of 8): two
      // 16-B loads per parameter instead of eight 4-B ones
      cop[jp] = n0 + colB(2 * jp + (q & 1)) + 8 * (q >> 1);
      const bool in = cop[jp] < g.Cout;
      const float4 one = make_float4(1.f, 1.f, 1.f, 1.f), zero = make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 s0 = in && g.scale ? *reinterpret_cast<const float4*>(g.scale + cop[jp]) : one;
      const float4 s1 = in && g.scale ? *reinterpret_cast<const float4*>(g.scale + cop[jp] + 4) : one;
      const float4 h0 = in && g.shift ? *reinterpret_cast<const float4*>(g.shift + cop[jp]) : zero;
      const float4 h1 = in && g.shift ? *reinterpret_cast<const float4*>(g.shift + cop[jp] + 4) : zero;
      sc[jp][0] = s0.x; sc[jp][1] = s0.y; sc[jp][2] = s0.z; sc[jp][3] = s0.w;
      sc[jp][4] = s1.x; sc[jp][5] = s1.y; sc[jp][6] = s1.z; sc[jp][7] = s1.w;
      sh[jp][0] = h0.x; sh[jp][1] = h0.y; sh[jp][2] = h0.z; sh[jp][3] = h0.w;
      sh[jp][4] = h1.x; sh[jp][5] = h1.y; sh[jp][6] = h1.z; sh[jp][7] = h1.w;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      if (KS && (i < TM / 2) != (grp == 0)) continue;   // (wave-uniform) the other group's half
      const int m = m0 + rowA(i) + r16;
      const bool mok = m < g.M;
      const int mm = mok ? m : 0;
      const int n = mm / HoWo, rem = mm - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      const size_t pix =
          (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * ocs;
      uint4 rv[TP], rl[TP];
#pragma unroll
      for (int jp = 0; jp < TP; ++jp) {
        rv[jp] = make_uint4(0, 0, 0, 0);
        rl[jp] = rv[jp];
        if constexpr (SPL) {
          if (rp && mok && cop[jp] < g.Cout) {
            rv[jp] = *reinterpret_cast<const uint4*>(rp + pix + split_ch(cop[jp]));
            rl[jp] = *reinterpret_cast<const uint4*>(rp + pix + split_ch(cop[jp]) + 32);
          }
          continue;
        }
        if constexpr (EARLY) {
          if (early) {
            rv[jp] = rve[i][jp];
            continue;
          }
        }
        if (rp && mok && cop[jp] < g.Cout) rv[jp] = *reinterpret_cast<const uint4*>(rp + pix + cop[jp]);
      }
#pragma unroll
      for (int jp = 0; jp < TP; ++jp) {
        float v[8], r[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][e]),
                                                           __float_as_uint(acc[i][2 * jp + 1][e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
        if constexpr (SPL) {
          join8(rv[jp], rl[jp], r);
        } else {
          O::load_vals(rv[jp], r);
        }
        affine8<false>(v, sc[jp], sh[jp]);
        if (rp) add8<false>(v, r);
        if (g.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if constexpr (SPL) {
          if (mok && cop[jp] < g.Cout) {
            uint4 h, l;
            split8(v, h, l);
            *reinterpret_cast<uint4*>(yp + pix + split_ch(cop[jp])) = h;
            *reinterpret_cast<uint4*>(yp + pix + split_ch(cop[jp]) + 32) = l;
          }
        } else {
          if (mok && cop[jp] < g.Cout) *reinterpret_cast<uint4*>(yp + pix + cop[jp]) = O::store_vals(v);
        }
      }
    }
  } else if (!SPL && g.mode == 0 && !g.hm) {
    T* __restrict__ yp = reinterpret_cast<T*>(g.y);
    const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
    float sc[TN][4], sh[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = n0 + colB(j) + q * 4 + e;
        sc[j][e] = (co < g.Cout && g.scale) ? g.scale[co] : 1.f;
        sh[j][e] = (co < g.Cout && g.shift) ? g.shift[co] : 0.f;
      }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + rowA(i) + r16;
      const bool mok = m < g.M;
      const int mm = mok ? m : 0;
      const int n = mm / HoWo, rem = mm - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      const size_t pix =
          (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * g.Cout;
      uint4 rv[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = n0 + colB(j) + q * 4;
        rv[j] = make_uint4(0, 0, 0, 0);
        if (rp && mok && co < g.Cout) {
          if constexpr (E == 4) {
            rv[j] = *reinterpret_cast<const uint4*>(rp + pix + co);
          } else {
            const uint2 r2 = *reinterpret_cast<const uint2*>(rp + pix + co);
            rv[j] = make_uint4(r2.x, r2.y, 0, 0);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int co = n0 + colB(j) + q * 4;
        if (!mok || co >= g.Cout) continue;
        float r[E], v[E];
        O::load_vals(rv[j], r);
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] * sc[j][e] + sh[j][e];
          if (rp) v[e] += r[e];
          if (g.relu) v[e] = fmaxf(v[e], 0.f);
        }
        const uint4 pk = O::store_vals(v);
        if constexpr (E == 4) {
          *reinterpret_cast<uint4*>(yp + pix + co) = pk;
        } else {
          *reinterpret_cast<uint2*>(yp + pix + co) = make_uint2(pk.x, pk.y);
        }
      }
    }
  } else {
  // ---- epilogue through LDS, PR rows per pass: the accumulators (BN applied) are
  // staged as an f32 [pixel][channel] tile, then written as whole 16-B NHWC chunks
  // with residual add + ReLU (mode 0), as NCHW f32 planes (mode 1), or fed to the
  // fused 1x1 head (g.hm, single pass)
  constexpr int LD = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
  constexpr int CPR = BN / E;            // output chunks per tile row
  constexpr int ITER = PR * CPR / NT;    // chunks per thread per pass
  static_assert(ITER * NT == PR * CPR, "epilogue chunk split");
  const bool mode0 = !SPL && g.mode == 0 && !g.hm;  // (split NHWC outputs take the direct epilogue)
  const bool relu_at_stage = g.relu && !mode0;  // mode 0: ReLU after the residual add
  float sc[TN][4], sh[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = n0 + colB(j) + q * 4 + e;
      sc[j][e] = (co < g.Cout && g.scale) ? g.scale[co] : 1.f;
      sh[j][e] = (co < g.Cout && g.shift) ? g.shift[co] : 0.f;
    }
#pragma unroll
  for (int p = 0; p < BM / PR; ++p) {
    // residual chunks of this pass first (their latency overlaps the staging)
    const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
    size_t off[ITER];
    bool ok[ITER];
    uint4 rv[ITER];
    if (mode0) {
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        const int idx = tid + it * NT;
        const int row = idx / CPR, cc = idx - row * CPR;
        const int m = m0 + p * PR + row, co = n0 + cc * E;
        ok[it] = m < g.M && co < g.Cout;
        const int mm = ok[it] ? m : 0;
        const int n = mm / HoWo, rem = mm - n * HoWo;
        const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
        off[it] = (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * g.Cout +
                  (ok[it] ? co : 0);
        rv[it] = make_uint4(0, 0, 0, 0);
        if (rp && ok[it]) rv[it] = *reinterpret_cast<const uint4*>(rp + off[it]);
      }
    }
    __syncthreads();  // the ring (or the previous pass) is no longer read
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = rowA(i) + r16 - p * PR;
      if (rowA(i) / PR != p) continue;  // wave-uniform
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int colb = colB(j) + q * 4;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[i][j][e] * sc[j][e] + sh[j][e];
          if (relu_at_stage) v[e] = fmaxf(v[e], 0.f);
        }
        *reinterpret_cast<float4*>(Cs + row * LD + colb) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    __syncthreads();
    if (mode0) {
      T* __restrict__ yp = reinterpret_cast<T*>(g.y);
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        if (!ok[it]) continue;
        const int idx = tid + it * NT;
        const int row = idx / CPR, cc = idx - row * CPR;
        float v[E];
#pragma unroll
        for (int e = 0; e < E; e += 4) {
          const float4 t4 = *reinterpret_cast<const float4*>(Cs + row * LD + cc * E + e);
          v[e] = t4.x;
          v[e + 1] = t4.y;
          v[e + 2] = t4.z;
          v[e + 3] = t4.w;
        }
        if (rp) {
          float r[E];
          O::load_vals(rv[it], r);
#pragma unroll
          for (int e = 0; e < E; ++e) v[e] += r[e];
        }
        if (g.relu) {
#pragma unroll
          for (int e = 0; e < E; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        *reinterpret_cast<uint4*>(yp + off[it]) = O::store_vals(v);
      }
    } else if (g.mode == 2) {
      // f32 GEMM rows, column blocks of vblk stored as separate [M][vblk] planes
      float* __restrict__ yp = reinterpret_cast<float*>(g.y);
      for (int idx = tid; idx < PR * CPR; idx += NT) {
        const int row = idx / CPR, cc = idx - row * CPR;
        const int m = m0 + p * PR + row, co = n0 + cc * E;
        if (m >= g.M || co >= g.Cout) continue;
        const int blk = co / g.vblk, cin = co - blk * g.vblk;
        float* dst = yp + (static_cast<size_t>(blk) * g.M + m) * g.vblk + cin;
#pragma unroll
        for (int e = 0; e < E; e += 4)
          *reinterpret_cast<float4*>(dst + e) = *reinterpret_cast<const float4*>(Cs + row * LD + cc * E + e);
      }
    } else if (!g.hm) {
      // NCHW f32 (heatmap head): consecutive threads walk pixels of one channel
      float* __restrict__ yp = reinterpret_cast<float*>(g.y);
      const int ncol = min(BN, g.Cout - n0);
      for (int idx = tid; idx < PR * ncol; idx += NT) {
        const int col = idx / PR, row = idx - col * PR;
        const int m = m0 + p * PR + row;
        if (m >= g.M) continue;
        const int n = m / HoWo, pixo = m - n * HoWo;
        yp[(static_cast<size_t>(n) * g.Cout + n0 + col) * HoWo + pixo] = Cs[row * LD + col];
      }
    } else if constexpr (!SPL && BN == 256 && BM == 64 && PR == BM && NW == 4) {
      // optional store of the deconv output f (NHWC), values rounded to T in place so
      // the head sees exactly what a separate head launch would read
      T* __restrict__ yp = reinterpret_cast<T*>(g.y);
      for (int idx = tid; idx < BM * CPR; idx += NT) {
        const int row = idx / CPR, cc = idx - row * CPR;
        const int m = m0 + row;
        float v[E];
#pragma unroll
        for (int e = 0; e < E; e += 4) {
          const float4 t4 = *reinterpret_cast<const float4*>(Cs + row * LD + cc * E + e);
          v[e] = t4.x;
          v[e + 1] = t4.y;
          v[e + 2] = t4.z;
          v[e + 3] = t4.w;
        }
        const uint4 packed = O::store_vals(v);
        float vr[E];
        O::load_vals(packed, vr);
#pragma unroll
        for (int e = 0; e < E; e += 4)
          *reinterpret_cast<float4*>(Cs + row * LD + cc * E + e) = make_float4(vr[e], vr[e + 1], vr[e + 2], vr[e + 3]);
        if (yp && m < g.M) {
          const int n = m / HoWo, rem = m - n * HoWo;
          const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
          const size_t off2 =
              (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * g.Cout +
              cc * E;
          *reinterpret_cast<uint4*>(yp + off2) = packed;
        }
      }
      __syncthreads();
      // final_layer (pose_resnet.py:126-132, 203) on the tile in LDS: wave w takes
      // pixel rows 16w..16w+15, one 16x16 MFMA tile = 16 joints, K = Cout
      f32x4 hacc = f32x4{0.f, 0.f, 0.f, 0.f};
      const T* __restrict__ hwp = reinterpret_cast<const T*>(g.hw);
      const int hrow = wid * 16 + r16;
      for (int kc = 0; kc < g.Cout / (4 * E); ++kc) {
        const int c = 4 * kc + q;
        float av[E];
#pragma unroll
        for (int e = 0; e < E; e += 4) {
          const float4 t4 = *reinterpret_cast<const float4*>(Cs + hrow * LD + c * E + e);
          av[e] = t4.x;
          av[e + 1] = t4.y;
          av[e + 2] = t4.z;
          av[e + 3] = t4.w;
        }
        const uint4 a = O::store_vals(av);
        const uint4 b = *reinterpret_cast<const uint4*>(hwp + static_cast<size_t>(r16) * g.hkp + c * E);
        O::mma(hacc, a, b);  // rows = pixels, cols = joints
      }
      const int joint = r16;
      if (joint < g.J) {
        const float bj = g.hbias ? g.hbias[joint] : 0.f;
        const int HWo = g.out_H * g.out_W;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + wid * 16 + q * 4 + e;
          if (m < g.M) {
            const int n = m / HoWo, rem = m - n * HoWo;
            const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
            const int pixo = (oy * osc + oy_off) * g.out_W + ox * osc + ox_off;
            g.hm[(static_cast<size_t>(n) * g.J + joint) * HWo + pixo] = hacc[e] + bj;
          }
        }
      }
    }
  }
  }  // LDS epilogue

}

// ---------------------------------------------------------------------------------
// Persistent variant (2-byte dtypes, direct NHWC epilogue).  The grid is the resident
// block count; each block walks a run of tiles (every XCD owns a contiguous slice of the
// tile order, so its concurrently running tiles still share operand rows in its L2) as ONE
// flattened stream of K-tiles through an S-slot LDS-DMA ring: the DMA of the next tile's
// first K-tiles is already in flight while the current tile's epilogue stores drain, and
// the stores never block the stream -- every epilogue issues exactly NST buffer stores per
// thread (out-of-range rows go to an offset past num_records), so each wait is a counted
// vmcnt that retires the K-tile being consumed and nothing younger.
template <typename T, int BM, int BN, int NW, int WGM, int S, bool DUAL>
__global__ __launch_bounds__(NW * 64) void conv_persist_kernel(ConvGeom g) {
  using O = Op<T>;

  constexpr int E = O::E;
  constexpr int ES = static_cast<int>(sizeof(T));
  constexpr int BK = 8 * E;
  constexpr int WGN = NW / WGM;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int ROWS = NW * 8;
  constexpr int RA = BM / ROWS, RB = BN / ROWS;
  constexpr int ND = RA + RB;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int TP = TN / 2;
  constexpr int NST = TM * TP;  // 16-B stores per thread per tile
  constexpr bool PRELOAD = TM + TN <= 8;
  static_assert(E == 8 && TN % 2 == 0, "persistent variant: 2-byte dtypes, paired n-tiles");
  static_assert(S == 2 || S == 3, "2 or 3 ring slots");
  static_assert(ND * (S - 2) + 2 * NST < 64, "vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[ring_bytes<BM, BN, S>()];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int r16 = lane & 15, q = lane >> 4;
  const int HoWo = g.Ho * g.Wo;

  // ---- this block's tiles: XCD xcd = blockIdx & 7 owns tiles [cstart, cstart + clen);
  // its nslot blocks take them round robin
  const int ntile = g.mtiles * g.ntiles * (g.deconv ? 4 : 1);
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = gridDim.x >> 3;
  const int qq = ntile >> 3, rr = ntile & 7;
  const int cstart = xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq;
  const int clen = qq + (xcd < rr ? 1 : 0);
  const int ntl = slot < clen ? (clen - slot + nslot - 1) / nslot : 0;
  const int nk = g.Kpad / BK;
  const int total = ntl * nk;
  if (total == 0) return;

  auto decode = [&](int k, int& mt, int& cls, int& nt) {
    const int w = cstart + slot + k * nslot;
    nt = w % g.ntiles;
    const int rest = w / g.ntiles;
    mt = g.deconv ? rest >> 2 : rest;
    cls = g.deconv ? rest & 3 : 0;
  };

  const u32x4 xrs = make_srd(g.x, g.N * g.H * g.W * g.C * ES);
  u32x4 x2rs = xrs;
  if constexpr (DUAL) x2rs = make_srd(g.x2, g.N * g.H2 * g.W2 * g.C2 * ES);
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));
  const int cL = (tid & 7) ^ ((tid >> 4) & 7);
  const bool tap_uniform = (g.C % BK) == 0;
  const bool fast_gather = tap_uniform && g.up == 0;
  const bool row_fast = !tap_uniform && g.KW * g.C == BK && g.up == 0;
  const int kwl = (cL * E) >> g.logC, cil = (cL * E) & (g.C - 1);

  // ---- load side: geometry of the tile whose K-tiles the DMA is fetching
  int l_tile = -1;
  u32x4 wrs = make_srd(g.w, 16);
  int wbrow = 0;
  int hb[RA], wb[RA], nb[RA], pbase[RA], rbase[RA], o1[RA], o2[RA];
  bool wok[RA];
  auto setup_load = [&](int k) {
    int mt, cls, nt;
    decode(k, mt, cls, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    int pad_h = g.pad_h, pad_w = g.pad_w;
    const T* wp = reinterpret_cast<const T*>(g.w);
    if (g.deconv) {
      pad_h = 1 - (cls >> 1);
      pad_w = 1 - (cls & 1);
      wp += static_cast<size_t>(cls) * g.CoutPad * g.Kpad;
    }
    wrs = make_srd(wp, g.CoutPad * g.Kpad * ES);
    wbrow = (n0 + (tid >> 3)) * g.Kpad + cL * E;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int m = m0 + (tid >> 3) + ROWS * i;
      if (m < g.M) {
        const int n = m / HoWo, rem = m - n * HoWo;
        const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
        hb[i] = oy * g.stride - pad_h;
        wb[i] = ox * g.stride - pad_w;
        nb[i] = n * g.H * g.W * g.C;
        if constexpr (DUAL) {
          o1[i] = (m * g.C + cL * E) * ES;
          o2[i] = (((n * g.H2 + oy * g.stride2) * g.W2 + ox * g.stride2) * g.C2 + cL * E) * ES;
        }
      } else {
        hb[i] = -(1 << 28);
        wb[i] = 0;
        nb[i] = 0;
        if constexpr (DUAL) {
          o1[i] = kOOB;
          o2[i] = kOOB;
        }
      }
      wok[i] = static_cast<unsigned>(wb[i] + kwl) < static_cast<unsigned>(g.W);
      rbase[i] = static_cast<int>(static_cast<unsigned>(nb[i]) +
                                  (static_cast<unsigned>(hb[i]) * g.W + static_cast<unsigned>(wb[i] + kwl)) * g.C +
                                  cil);
      pbase[i] = static_cast<int>(static_cast<unsigned>(nb[i]) +
                                  (static_cast<unsigned>(hb[i]) * g.W + static_cast<unsigned>(wb[i])) * g.C + cL * E);
    }
  };
  // DMA of stream K-tile sq into ring slot sq % S: exactly ND dma16 per thread
  // DMA of stream K-tile sq into ring slot sq % S: exactly ND dma16 per thread.  The
  // source offsets are computed first (dma_prep), the instructions issued by dma_issue(d)
  // -- all at once, or (eight-wave tiles) interleaved with the previous K-tile's MFMAs.
  int doff[ND];
  unsigned dAs = 0;
  bool dsec = false;
  auto dma_prep = [&](int sq) {
    const int k = sq / nk, kt = sq - k * nk;
    if (k != l_tile) {
      setup_load(k);
      l_tile = k;
    }
    const int kbase = kt * BK;
    dAs = __builtin_amdgcn_readfirstlane(lds0 + (sq % S) * STAGE + wid_u * 1024);
    if constexpr (DUAL) {
      const bool first = kbase < g.K1;
      dsec = __builtin_amdgcn_readfirstlane(first ? 0 : 1) != 0;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const int o = first ? o1[i] : o2[i];
        doff[i] = o == kOOB ? kOOB : o + (first ? kbase : kbase - g.K1) * ES;
      }
    } else if (fast_gather) {
      const int tap = kbase >> g.logC;
      const int th = tap / g.KW, tw = tap - th * g.KW;
      const int toff = (th * g.W + tw) * g.C + (kbase & (g.C - 1));
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const bool ok = static_cast<unsigned>(hb[i] + th) < static_cast<unsigned>(g.H) &&
                        static_cast<unsigned>(wb[i] + tw) < static_cast<unsigned>(g.W);
        doff[i] = ok ? (pbase[i] + toff) * ES : kOOB;
      }
    } else if (row_fast) {
      const int roff = kt * g.W * g.C;
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const bool ok = wok[i] && static_cast<unsigned>(hb[i] + kt) < static_cast<unsigned>(g.H);
        doff[i] = ok ? (rbase[i] + roff) * ES : kOOB;
      }
    } else {
      int kh, kw, ci;
      bool kvalid = true;
      if (tap_uniform) {
        const int tap = kbase >> g.logC;
        kh = tap / g.KW;
        kw = tap - kh * g.KW;
        ci = (kbase & (g.C - 1)) + cL * E;
      } else {
        const int kk = kbase + cL * E;
        const int tap = kk >> g.logC;
        kh = tap / g.KW;
        kw = tap - kh * g.KW;
        ci = kk & (g.C - 1);
        kvalid = kk < g.K;
      }
#pragma unroll
      for (int i = 0; i < RA; ++i) {
        const int hl = hb[i] + kh, wl = wb[i] + kw;
        const int hi = hl >> g.up, wi = wl >> g.up;
        const bool ok = kvalid && ((hl | wl) & g.up) == 0 && static_cast<unsigned>(hi) < static_cast<unsigned>(g.H) &&
                        static_cast<unsigned>(wi) < static_cast<unsigned>(g.W);
        doff[i] = ok ? (nb[i] + (hi * g.W + wi) * g.C + ci) * ES : kOOB;
      }
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) doff[RA + i] = (wbrow + ROWS * i * g.Kpad + kbase) * ES;
  };
  auto dma_issue = [&](int d) {  // d compile-time after unrolling
    if (d < RA) {
      if (DUAL && dsec) dma16(x2rs, doff[d], dAs + d * NW * 1024);
      else dma16(xrs, doff[d], dAs + d * NW * 1024);
    } else {
      dma16(wrs, doff[d], dAs + A_BYTES + (d - RA) * NW * 1024);
    }
  };
  auto dma_ktile = [&](int sq) {
    dma_prep(sq);
#pragma unroll
    for (int d = 0; d < ND; ++d) dma_issue(d);
  };
  constexpr bool IL = NW == 8;  // interleave the next K-tile's DMAs with the MFMAs
  constexpr int IL_STEP = 4;    // one DMA after every IL_STEP MFMAs
  static_assert(!IL || ND * IL_STEP <= 2 * TM * TN, "interleave slots");
  auto mma_il = [&](int f, bool more, f32x4& a, const uint4& b, const uint4& x) {
    O::mma(a, b, x);
    if constexpr (IL) {
      if (f % IL_STEP == IL_STEP - 1 && f / IL_STEP < ND && more) {
        __builtin_amdgcn_sched_barrier(0);
        dma_issue(f / IL_STEP);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  f32x4 acc[TM][TN];
  auto zero_acc = [&] {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto compute = [&](int slot_, bool more) {
    const char* As_ = smem + slot_ * STAGE;
    const char* Bs_ = As_ + A_BYTES;
    if constexpr (PRELOAD) {
      uint4 af[2][TM], bfr[2][TN];
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c = 4 * cb + q;
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[cb][j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, c));
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[cb][i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, c));
      }
#pragma unroll
      for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mma_il((cb * TM + i) * TN + j, more, acc[i][j], bfr[cb][j], af[cb][i]);
    } else {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c = 4 * cb + q;
        uint4 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, c));
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, c));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mma_il((cb * TM + i) * TN + j, more, acc[i][j], bfr[j], af[i]);
      }
    }
  };
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
      g.y, 0, g.N * g.out_H * g.out_W * g.Cout * ES, 0x00020000);
  const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
  // Small tiles load the residual with counted (inline-asm) loads issued before the last
  // K-tile's wait, so the epilogue waits only for them -- not for the DMA issued after.
  constexpr bool ARES = TM * TP <= 8;
  constexpr int NR = ARES ? TM * TP : 0;
  const u32x4 rrs = make_srd(g.res ? g.res : g.y, g.N * g.out_H * g.out_W * g.Cout * ES);
  u32x4 rres[ARES ? TM : 1][ARES ? TP : 1];
  auto res_issue = [&](int k) {
    int mt, cls, nt;
    decode(k, mt, cls, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    const int osc = g.deconv ? 2 : (g.ostride > 1 ? g.ostride : 1), oy_off = g.deconv ? cls >> 1 : 0,
              ox_off = g.deconv ? cls & 1 : 0;
    asm volatile("s_nop 4" ::: "memory");
#pragma unroll
    for (int i = 0; i < (ARES ? TM : 1); ++i) {
      const int m = m0 + wm * WTM + i * 16 + r16;
      const bool mok = m < g.M;
      const int mm = mok ? m : 0;
      const int n = mm / HoWo, rem = mm - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      const int pix = ((n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * g.Cout;
#pragma unroll
      for (int jp = 0; jp < (ARES ? TP : 1); ++jp) {
        const int co = n0 + wn * WTN + (2 * jp + (q & 1)) * 16 + 8 * (q >> 1);
        const int off = (mok && co < g.Cout) ? (pix + co) * ES : kOOB;
        asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(rres[i][jp]) : "v"(off), "s"(rrs) : "memory");
      }
    }
  };
  const bool ares = ARES && g.res != nullptr;
  // epilogue of stream tile k: BN, residual, ReLU in registers; NST 16-B buffer stores
  auto epilogue = [&](int k) {
    int mt, cls, nt;
    decode(k, mt, cls, nt);
    const int m0 = mt * BM, n0 = nt * BN;
    const int osc = g.deconv ? 2 : (g.ostride > 1 ? g.ostride : 1), oy_off = g.deconv ? cls >> 1 : 0,
              ox_off = g.deconv ? cls & 1 : 0;
    int cop[TP];
    float sc[TP][8], sh[TP][8];
#pragma unroll
    for (int jp = 0; jp < TP; ++jp) {
      cop[jp] = n0 + wn * WTN + (2 * jp + (q & 1)) * 16 + 8 * (q >> 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = cop[jp] + e;
        sc[jp][e] = (co < g.Cout && g.scale) ? g.scale[co] : 1.f;
        sh[jp][e] = (co < g.Cout && g.shift) ? g.shift[co] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WTM + i * 16 + r16;
      const bool mok = m < g.M;
      const int mm = mok ? m : 0;
      const int n = mm / HoWo, rem = mm - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      const int pix = ((n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * g.Cout;
      uint4 rv[TP];
#pragma unroll
      for (int jp = 0; jp < TP; ++jp) {
        rv[jp] = make_uint4(0, 0, 0, 0);
        if constexpr (ARES) {
          if (ares) {
            rv[jp] = make_uint4(rres[i][jp].x, rres[i][jp].y, rres[i][jp].z, rres[i][jp].w);
            continue;
          }
        }
        if (rp && mok && cop[jp] < g.Cout) rv[jp] = *reinterpret_cast<const uint4*>(rp + pix + cop[jp]);
      }
#pragma unroll
      for (int jp = 0; jp < TP; ++jp) {
        float v[8], r[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][e]),
                                                           __float_as_uint(acc[i][2 * jp + 1][e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
        O::load_vals(rv[jp], r);
        affine8<false>(v, sc[jp], sh[jp]);
        if (rp) add8<false>(v, r);
        if (g.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        const uint4 pk = O::store_vals(v);
        const u32x4 pv = {pk.x, pk.y, pk.z, pk.w};
        const int voff = (mok && cop[jp] < g.Cout) ? (pix + cop[jp]) * ES : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(pv, yrs, voff, 0, 0);
      }
    }
  };
  auto barrier = [] {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  zero_acc();
  unsigned wv[kWarmLoads];   // weight warm-up (gemm_common.h), consumed after the first DMAs
  warm_issue(wv, g.w, g.wseg, g.warm, NW * 64);
#pragma unroll
  for (int sq = 0; sq < S - 1; ++sq)
    if (sq < total) dma_ktile(sq);
  warm_use(wv);
  for (int sq = 0; sq < total; ++sq) {
    const bool tile_end = (sq + 1) % nk == 0;
    if (ares && tile_end) res_issue(sq / nk);
    // retire K-tile sq: younger = the DMA groups of sq+1 .. sq+S-2, the stores of the
    // epilogues run since sq's DMA was issued (iterations sq-S+1 .. sq-1) and the
    // residual loads just issued
    const int a = min(S - 2, total - 1 - sq);
    int e = 0;
#pragma unroll
    for (int d = 1; d < S; ++d) e += (sq - d >= 0 && (sq - d + 1) % nk == 0) ? 1 : 0;
    vm_wait_dyn(ND * a + NST * e + ((ares && tile_end) ? NR : 0));
    barrier();
    const bool more = sq + S - 1 < total;
    if (IL) {
      if (more) dma_prep(sq + S - 1);
    } else if (more) {
      dma_ktile(sq + S - 1);
    }
    compute(sq % S, more);
    if (tile_end) {
      if constexpr (ARES) {
        if (ares) {  // the residual has landed once only this iteration's DMA group is younger
          if (more) vm_wait<ND>();
          else vm_wait<0>();
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int jp = 0; jp < TP; ++jp) asm volatile("" : "+v"(rres[i][jp]));
        }
      }
      epilogue(sq / nk);
      zero_acc();
    }
  }
}

int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

template <typename T, int BM, int BN, int NW, int WGM, bool DUAL>
void launch_persist(const ConvGeom& g, int ntile, hipStream_t s) {
  // four-wave tiles keep two slots (several blocks per CU hide each other's latencies);
  // eight-wave tiles take a third slot where it fits
  constexpr int S = (NW == 8 && ring_bytes<BM, BN, 3>() <= 160 * 1024) ? 3 : 2;
  static const int occ = [] {
    int b = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, conv_persist_kernel<T, BM, BN, NW, WGM, S, DUAL>, NW * 64,
                                                     0) != hipSuccess || b < 1)
      b = 1;
    return b;
  }();
  int grid = std::min(ntile, cu_count() * occ);
  grid = std::max(8, grid & ~7);  // whole XCD rounds (blockIdx & 7 = XCD slice)
  hipLaunchKernelGGL((conv_persist_kernel<T, BM, BN, NW, WGM, S, DUAL>), dim3(grid), dim3(NW * 64), 0, s, g);
}

template <typename T, int BM, int BN, int NW, int WGM, bool DUAL>
void launch_cfg(const ConvGeom& g, int blocks, int stages, hipStream_t s) {
  if constexpr (NW == 4) {
    if (stages == 1) {
      hipLaunchKernelGGL((conv_igemm_kernel<T, BM, BN, NW, WGM, 1, DUAL>), dim3(blocks), dim3(NW * 64), 0, s, g);
      return;
    }
  }
  if constexpr (ring_bytes<BM, BN, 3>() <= 160 * 1024) {
    if (stages >= 3) {
      hipLaunchKernelGGL((conv_igemm_kernel<T, BM, BN, NW, WGM, 3, DUAL>), dim3(blocks), dim3(NW * 64), 0, s, g);
      return;
    }
  }
  hipLaunchKernelGGL((conv_igemm_kernel<T, BM, BN, NW, WGM, 2, DUAL>), dim3(blocks), dim3(NW * 64), 0, s, g);
}


// Tile configurations (the `tile` argument of the conv entry points): cfg + 8 * variant,
//   cfg 0: 256x64, 1: 128x64, 2: 64x64, 3: 128x128, 4: 64x128 (four waves),
//       5: 256x256, 6: 256x128 (eight waves);
//   variant 1: single-slot LDS ring (cfg 0-4; short-K layers: more blocks per CU),
//   variant 2: three-slot ring (cfg != 5),
//   +32 (2-byte dtypes): the persistent K-tile stream (conv_persist_kernel);
//   23 / 31 (2-byte dtypes): 256x256 / 256x128 with waves 4-7 staggered by half a K-tile
//   (also what the heuristic runs for those shapes);
//   7 / 15 (2-byte dtypes, round 4): 128x128 with eight waves, staggered, as 2x4 waves of
//   64x32 / 4x2 waves of 32x64 (M = 8192-pixel layers: 256 tiles of 128x128 give every CU one
//   block, and eight waves two per SIMD);
//   -1: the built-in heuristic.
bool tile_ok(int tile) {
  if (tile == -1 || tile == 23 || tile == 31 || tile == 7 || tile == 15 || tile == 39 || tile == 47 || tile == 55)
    return true;
  if (tile < 0 || tile >= 64) return false;
  const int c = tile & 7, v = (tile >> 3) & 3;
  return c <= 6 && v <= 2 && !(v == 1 && c > 4) && !(v == 2 && c == 5);
}

#ifndef POSU_SPLIT_SG_HEAD
#define POSU_SPLIT_SG_HEAD 0   // (the staggered split 256x256 head instance spills 23 VGPRs)
#endif
template <typename T, bool DUAL>
int launch(ConvGeom g, int nclass, hipStream_t s, const char* what, int tile) {
  // the split dtype runs the plain (unstaggered, non-persistent) loops: its K-tiles pair two
  // k-steps, which the half-K-tile stagger would cut apart
  constexpr bool SPL = Op<T>::SPLIT;
  constexpr bool FAST2 = sizeof(T) == 2 && !SPL;
  {
    const long long wbytes = static_cast<long long>(g.CoutPad) * g.Kpad * static_cast<long long>(sizeof(T)) * nclass;
    g.warm = warm_wgs(wbytes);
    g.wseg = wbytes / 64;
  }
  if constexpr (sizeof(T) == 2 && !DUAL) {  // fused head on the eight-wave 256x256 tile, direct epilogue
    if (g.hm && g.CoutPad == 256) {
      g.ntiles = 1;
      g.mtiles = (g.M + 255) / 256;
      if constexpr (SPL) {
        // (round 6: the staggered loop in split fp16 too, POSU_SPLIT_SG_HEAD; bit-identical either way)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 256, 256, 8, 2, 2, DUAL, POSU_SPLIT_SG_HEAD != 0, true>),
                           dim3(g.mtiles * nclass), dim3(512), 0, s, g);
      } else {
        // staggered two-slot loop (waves 4-7 half a K-tile behind; bit-exact with tile 5)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 256, 256, 8, 2, 2, DUAL, true, true>), dim3(g.mtiles * nclass),
                           dim3(512), 0, s, g);
      }
      return check_launch(what);
    }
  }
  if (g.hm) {  // fused head (f32): one 64x256 block owns all 256 output channels, head from LDS
    g.ntiles = 1;
    g.mtiles = (g.M + 63) / 64;
    hipLaunchKernelGGL((conv_igemm_kernel<T, 64, 256, 4, 1, 2, DUAL>), dim3(g.mtiles * nclass), dim3(256), 0, s, g);
    return check_launch(what);
  }
  // heuristic: 64-channel layers take 256 x 64 tiles (four waves stacked along M, 64 x 64
  // each); wider layers 256 x 256 with eight 128 x 64 waves when the grid still gives
  // every CU a block, else 128 x 128; grids that would not give every CU two blocks drop
  // to 64-row tiles.
  auto blocks = [&](int bm, int bn) {
    return static_cast<long long>((g.M + bm - 1) / bm) * (g.CoutPad / bn) * nclass;
  };
  int cfg;
  if (g.CoutPad % 128 != 0) {
    cfg = blocks(256, 64) >= 1024 ? 0 : (blocks(128, 64) >= 512 ? 1 : 2);
  } else if (g.CoutPad % 256 == 0 && blocks(256, 256) >= 256) {
    cfg = 5;
  } else {  // 128-channel layers: 256 x 128 measured slower than 128 x 128 (layer2 c1/c2, R50@256)
    cfg = blocks(128, 128) >= 512 ? 3 : 4;
  }
  int st = 2;
  bool sg = false, persist = false;
  bool wg4 = false;  // tile 15: the 4 x 2 wave grid of the 128x128 eight-wave tile
  bool ks = false;   // tile 39: the 128x128 tile with two K groups of four waves
  bool w8 = false;   // SPL: tiles 7 / 15 as the unstaggered eight-wave 128x128 tile
  if (tile == 39) {
    if (sizeof(T) == 2 && g.CoutPad % 128 == 0 && g.mode == 0 && !g.hm) {
      cfg = 3;
      ks = true;
    }
  } else if (tile == 23 || tile == 31) {
    const int c = tile == 23 ? 5 : 6;
    // (split fp16: 31 only -- its staggered 256x256 instance spills 56 VGPRs)
    if ((FAST2 || (SPL && c == 6)) && g.CoutPad % (c == 5 ? 256 : 128) == 0) {
      cfg = c;
      sg = true;
    }
  } else if (tile == 7 || tile == 15) {
    if (sizeof(T) == 2 && g.CoutPad % 128 == 0) {
      cfg = 7;
      sg = FAST2;
      w8 = SPL;
      wg4 = tile == 15;
    }
  } else if (tile == 47 || tile == 55) {   // split fp16: the staggered 128x128 eight-wave tiles (round 6)
    if (SPL && g.CoutPad % 128 == 0) {
      cfg = 7;
      sg = true;
      wg4 = tile == 55;
    }
  } else if (tile >= 0) {
    const int c = tile & 7, v = (tile >> 3) & 3;
    const bool wide_ok = g.CoutPad % 128 == 0 && (c != 5 || g.CoutPad % 256 == 0);
    if (c <= 2 || wide_ok) {
      cfg = c;
      st = v == 1 ? (c <= 4 ? 1 : 2) : v == 2 ? 3 : 2;
      // persistent K-tile stream: 2-byte dtypes, direct NHWC epilogue, outputs addressable
      // by a 32-bit buffer offset
      persist = (tile & 32) != 0 && FAST2 && g.mode == 0 &&
                static_cast<long long>(g.N) * g.out_H * g.out_W * g.Cout * sizeof(T) < (1LL << 31) - 256;
    }
  } else if (FAST2 && (cfg == 5 || cfg == 6)) {
    sg = true;  // untuned eight-wave launches take the staggered loop (bit-exact with the plain one)
  }
  static const int kBM[] = {256, 128, 64, 128, 64, 256, 256, 128};
  static const int kBN[] = {64, 64, 64, 128, 128, 256, 128, 128};
  g.ntiles = g.CoutPad / kBN[cfg];
  g.mtiles = (g.M + kBM[cfg] - 1) / kBM[cfg];
  const int nb = g.mtiles * g.ntiles * nclass;
  if constexpr (SPL) {   // the split dtype's eight-wave 128x128 tiles: two K groups (39) or one (7 / 15)
    if (ks) {
      hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 2, 2, DUAL, false, false, true>), dim3(nb), dim3(512), 0,
                         s, g);
      return check_launch(what);
    }
    if (w8) {
      if (wg4)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 4, 2, DUAL>), dim3(nb), dim3(512), 0, s, g);
      else
        hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 2, 2, DUAL>), dim3(nb), dim3(512), 0, s, g);
      return check_launch(what);
    }
    if (sg) {   // round 6: the staggered eight-wave tiles in split fp16: 256x128 (31), 128x128 (47 / 55)
      if (cfg == 7 && wg4)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 4, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      else if (cfg == 7)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 2, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      else
        hipLaunchKernelGGL((conv_igemm_kernel<T, 256, 128, 8, 4, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      return check_launch(what);
    }
  }
  if constexpr (FAST2) {
    if (persist) {
      switch (cfg) {
        // (no persistent 256x64 instance: dynamic indexing of its store registers put 960 B per lane
        // in scratch; tile 32 runs the plain 256x64 tile)
        case 0: launch_cfg<T, 256, 64, 4, 4, DUAL>(g, nb, st, s); break;
        case 1: launch_persist<T, 128, 64, 4, 2, DUAL>(g, nb, s); break;
        case 2: launch_persist<T, 64, 64, 4, 2, DUAL>(g, nb, s); break;
        case 3: launch_persist<T, 128, 128, 4, 2, DUAL>(g, nb, s); break;
        case 4: launch_persist<T, 64, 128, 4, 2, DUAL>(g, nb, s); break;
        case 5: launch_persist<T, 256, 256, 8, 2, DUAL>(g, nb, s); break;
        default: launch_persist<T, 256, 128, 8, 4, DUAL>(g, nb, s); break;
      }
      return check_launch(what);
    }
    if (ks) {
      hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 2, 2, DUAL, false, false, true>), dim3(nb), dim3(512), 0,
                         s, g);
      return check_launch(what);
    }
    if (sg) {
      if (cfg == 5)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 256, 256, 8, 2, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      else if (cfg == 7 && wg4)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 4, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      else if (cfg == 7)
        hipLaunchKernelGGL((conv_igemm_kernel<T, 128, 128, 8, 2, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      else
        hipLaunchKernelGGL((conv_igemm_kernel<T, 256, 128, 8, 4, 2, DUAL, true>), dim3(nb), dim3(512), 0, s, g);
      return check_launch(what);
    }
  }
  switch (cfg) {
    case 0: launch_cfg<T, 256, 64, 4, 4, DUAL>(g, nb, st, s); break;
    case 1: launch_cfg<T, 128, 64, 4, 2, DUAL>(g, nb, st, s); break;
    case 2: launch_cfg<T, 64, 64, 4, 2, DUAL>(g, nb, st, s); break;
    case 3: launch_cfg<T, 128, 128, 4, 2, DUAL>(g, nb, st, s); break;
    case 4: launch_cfg<T, 64, 128, 4, 2, DUAL>(g, nb, st, s); break;
    case 5: launch_cfg<T, 256, 256, 8, 2, DUAL>(g, nb, 2, s); break;
    default: launch_cfg<T, 256, 128, 8, 4, DUAL>(g, nb, st == 3 ? 3 : 2, s); break;
  }
  return check_launch(what);
}

template <bool DUAL>
int dispatch(int dtype, ConvGeom& g, int nclass, void* stream, const char* what, int tile = -1) {
  hipStream_t s = as_stream(stream);
  if (dtype == POSU_BF16) return launch<uint16_t, DUAL>(g, nclass, s, what, tile);
  if (dtype == POSU_F32) return launch<float, DUAL>(g, nclass, s, what, tile);
  if (dtype == POSU_F16) return launch<f16_t, DUAL>(g, nclass, s, what, tile);
  if (dtype == POSU_F16X3) return launch<f16s_t, DUAL>(g, nclass, s, what, tile);
  set_error(std::string(what) + ": unsupported dtype");
  return POSU_ERR_ARG;
}

// the direct epilogue reads the per-channel BN parameters as 16-B vectors
bool params_aligned(const float* scale, const float* shift) {
  return (reinterpret_cast<size_t>(scale) & 15) == 0 && (reinterpret_cast<size_t>(shift) & 15) == 0;
}

int bk_of(int dtype) { return dtype == POSU_F32 ? 32 : 64; }
int esz_of(int dtype) { return dtype == POSU_F32 ? 4 : 2; }
// stored elements per logical channel (the split dtype keeps a (hi, lo) pair)
int cm_of(int dtype) { return dtype == POSU_F16X3 ? 2 : 1; }

int common_checks(int dtype, const void* x, const void* w, const void* y, int N, int H, int W, int C,
                  int Cout, const char* what) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F32 || dtype == POSU_F16 || dtype == POSU_F16X3,
               std::string(what) + ": dtype must be F32, BF16, F16 or F16X3");
  POSU_REQUIRE(x && w && y, std::string(what) + ": null pointer");
  POSU_REQUIRE(N > 0 && H > 0 && W > 0 && Cout > 0, std::string(what) + ": empty shape");
  POSU_REQUIRE(C >= 8 && ilog2(C) >= 0, std::string(what) + ": C must be a power of two >= 8");
  POSU_REQUIRE(dtype != POSU_F16X3 || (C % 32 == 0 && Cout % 32 == 0),
               std::string(what) + ": split fp16 needs C and Cout multiples of 32");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * cm_of(dtype) * esz_of(dtype) < (1LL << 31) - 256,
               std::string(what) + ": input exceeds the 2 GiB buffer-descriptor range");
  return POSU_OK;
}

ConvGeom base_geom(const void* x, int N, int H, int W, int C, const void* w, int Cout, int dtype) {
  ConvGeom g{};
  g.x = x;
  g.w = w;
  g.N = N;
  g.H = H;
  g.W = W;
  g.C = C * cm_of(dtype);  // stored channels (the GEMM's K per tap)
  g.logC = ilog2(g.C);
  g.Cout = Cout;
  g.CoutPad = round_up(Cout, 64);
  g.stride = 1;
  g.KH = g.KW = 1;
  return g;
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_conv_bk(int dtype) { return bk_of(dtype); }

extern "C" int posu_conv2d_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w, int Cout,
                               int KH, int KW, int stride, int pad, const float* scale, const float* shift,
                               const void* residual, int relu, void* y, int Ho, int Wo, int tile, void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_conv2d_fwd")) return st;
  POSU_REQUIRE(tile_ok(tile), "posu_conv2d_fwd: tile must be -1 (auto), cfg + 8 * variant (+ 32), 7, 15, 23 or 31");
  const int E = 16 / esz_of(dtype);
  POSU_REQUIRE(Cout % E == 0, "posu_conv2d_fwd: Cout must be a multiple of 16 bytes");
  POSU_REQUIRE(KH > 0 && KW > 0 && stride > 0 && pad >= 0, "posu_conv2d_fwd: bad window");
  POSU_REQUIRE(Ho > 0 && Wo > 0 && Ho <= (H + 2 * pad - KH) / stride + 1 && Wo <= (W + 2 * pad - KW) / stride + 1,
               "posu_conv2d_fwd: Ho/Wo larger than the window allows");
  POSU_REQUIRE(static_cast<long long>(N) * Ho * Wo * Cout * cm_of(dtype) < (1LL << 31),
               "posu_conv2d_fwd: output too large");
  POSU_REQUIRE(params_aligned(scale, shift), "posu_conv2d_fwd: scale / shift must be 16-byte aligned");
  ConvGeom g = base_geom(x, N, H, W, C, w, Cout, dtype);
  g.scale = scale;
  g.shift = shift;
  g.res = residual;
  g.y = y;
  g.Ho = Ho;
  g.Wo = Wo;
  g.M = N * Ho * Wo;
  g.K = KH * KW * g.C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = KH;
  g.KW = KW;
  g.stride = stride;
  g.pad_h = pad;
  g.pad_w = pad;
  g.relu = relu;
  g.out_H = Ho;
  g.out_W = Wo;
  return dispatch<false>(dtype, g, 1, stream, "posu_conv2d_fwd", tile);
}

extern "C" int posu_conv1x1_dual_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* x2, int H2,
                                     int W2, int C2, int stride2, const void* w, int Cout, const float* scale,
                                     const float* shift, int relu, void* y, int tile, void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_conv1x1_dual_fwd")) return st;
  POSU_REQUIRE(tile_ok(tile), "posu_conv1x1_dual_fwd: tile must be -1 (auto), cfg + 8 * variant (+ 32), 7, 15, 23 or 31");
  if (int st = common_checks(dtype, x2, w, y, N, H2, W2, C2, Cout, "posu_conv1x1_dual_fwd")) return st;
  const int BK = bk_of(dtype);
  POSU_REQUIRE(C % BK == 0 && C2 % BK == 0, "posu_conv1x1_dual_fwd: C and C2 must be multiples of the K-tile");
  POSU_REQUIRE(stride2 > 0 && (H - 1) * stride2 < H2 && (W - 1) * stride2 < W2,
               "posu_conv1x1_dual_fwd: source-2 grid too small for the output grid");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * Cout * cm_of(dtype) < (1LL << 31),
               "posu_conv1x1_dual_fwd: output too large");
  POSU_REQUIRE(params_aligned(scale, shift), "posu_conv1x1_dual_fwd: scale / shift must be 16-byte aligned");
  ConvGeom g = base_geom(x, N, H, W, C, w, Cout, dtype);
  g.x2 = x2;
  g.H2 = H2;
  g.W2 = W2;
  g.C2 = C2 * cm_of(dtype);
  g.stride2 = stride2;
  g.K1 = g.C;
  g.scale = scale;
  g.shift = shift;
  g.y = y;
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.K = g.C + g.C2;
  g.Kpad = g.C + g.C2;
  g.relu = relu;
  g.out_H = H;
  g.out_W = W;
  return dispatch<true>(dtype, g, 1, stream, "posu_conv1x1_dual_fwd", tile);
}

extern "C" int posu_deconv4x4s2_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w,
                                    int Cout, const float* scale, const float* shift, int relu, void* y, int tile,
                                    void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_deconv4x4s2_fwd")) return st;
  POSU_REQUIRE(tile_ok(tile), "posu_deconv4x4s2_fwd: tile must be -1 (auto), cfg + 8 * variant (+ 32), 7, 15, 23 or 31");
  const int E = 16 / esz_of(dtype);
  POSU_REQUIRE(Cout % E == 0, "posu_deconv4x4s2_fwd: Cout must be a multiple of 16 bytes");
  POSU_REQUIRE(static_cast<long long>(N) * 4 * H * W * Cout * cm_of(dtype) < (1LL << 31),
               "posu_deconv4x4s2_fwd: output too large");
  POSU_REQUIRE(params_aligned(scale, shift), "posu_deconv4x4s2_fwd: scale / shift must be 16-byte aligned");
  ConvGeom g = base_geom(x, N, H, W, C, w, Cout, dtype);
  g.scale = scale;
  g.shift = shift;
  g.y = y;
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.K = 4 * g.C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = 2;
  g.KW = 2;
  g.relu = relu;
  g.deconv = 1;
  g.out_H = 2 * H;
  g.out_W = 2 * W;
  return dispatch<false>(dtype, g, 4, stream, "posu_deconv4x4s2_fwd", tile);
}

extern "C" int posu_deconv4x4s2_head_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w,
                                         int Cout, const float* scale, const float* shift, void* y, const void* hw,
                                         const void* hw_lo, int J, const float* hbias, float* hm, void* stream) {
  if (int st = common_checks(dtype, x, w, hm, N, H, W, C, Cout, "posu_deconv4x4s2_head_fwd")) return st;
  POSU_REQUIRE(hw && Cout == 256 && J > 0 && J <= 16,
               "posu_deconv4x4s2_head_fwd: needs Cout == 256, 0 < J <= 16 and head weights");
  POSU_REQUIRE(dtype != POSU_F16X3 || hw_lo, "posu_deconv4x4s2_head_fwd: split fp16 needs hw_lo");
  POSU_REQUIRE(((reinterpret_cast<size_t>(hw) | reinterpret_cast<size_t>(hw_lo)) & 15) == 0,
               "posu_deconv4x4s2_head_fwd: hw / hw_lo must be 16-byte aligned");
  POSU_REQUIRE(params_aligned(scale, shift), "posu_deconv4x4s2_head_fwd: scale / shift must be 16-byte aligned");
  ConvGeom g = base_geom(x, N, H, W, C, w, Cout, dtype);
  g.scale = scale;
  g.shift = shift;
  g.y = y;
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.K = 4 * g.C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = 2;
  g.KW = 2;
  g.relu = 1;
  g.deconv = 1;
  g.out_H = 2 * H;
  g.out_W = 2 * W;
  g.hw = hw;
  g.hw_lo = (dtype == POSU_BF16 || dtype == POSU_F16 || dtype == POSU_F16X3) ? hw_lo : nullptr;  // f32: exact
  g.hbias = hbias;
  g.hm = hm;
  g.J = J;
  g.hkp = round_up(Cout, bk_of(dtype));
  return dispatch<false>(dtype, g, 4, stream, "posu_deconv4x4s2_head_fwd");
}

extern "C" int posu_head1x1_nchw_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w,
                                     int Cout, const float* bias, float* y, void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_head1x1_nchw_fwd")) return st;
  ConvGeom g = base_geom(x, N, H, W, C, w, Cout, dtype);
  g.shift = bias;
  g.y = y;
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.K = g.C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.out_H = H;
  g.out_W = W;
  g.mode = 1;
  return dispatch<false>(dtype, g, 1, stream, "posu_head1x1_nchw_fwd");
}

// Data gradient of a KHxKW / stride / pad convolution x[N,H,W,Cin] -> y[N,Ho,Wo,Cout]:
// dx = conv(dy, W flipped and transposed, pad K-1-pad) over dy, read as its
// zero-upsampled image when stride == 2 (g.up), so strided layers run through the same
// MFMA kernel as the forward.  `residual` (optional, [N,H,W,Cin]) is added in the
// epilogue: the identity-branch gradient of a residual block.
extern "C" int posu_conv2d_dgrad_tile(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, const void* wt,
                                      int Cin, int KH, int KW, int stride, int pad, const void* residual, void* dx,
                                      int H, int W, int tile, void* stream);

extern "C" int posu_conv2d_dgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, const void* wt,
                                 int Cin, int KH, int KW, int stride, int pad, const void* residual, void* dx, int H,
                                 int W, void* stream) {
  return posu_conv2d_dgrad_tile(dtype, dy, N, Ho, Wo, Cout, wt, Cin, KH, KW, stride, pad, residual, dx, H, W, -1,
                                stream);
}

extern "C" int posu_conv2d_dgrad_tile(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, const void* wt,
                                      int Cin, int KH, int KW, int stride, int pad, const void* residual, void* dx,
                                      int H, int W, int tile, void* stream) {
  POSU_REQUIRE(dtype != POSU_F16X3, "posu_conv2d_dgrad: the split dtype is inference-only");
  POSU_REQUIRE(tile_ok(tile), "posu_conv2d_dgrad: unknown tile configuration");
  if (int st = common_checks(dtype, dy, wt, dx, N, Ho, Wo, Cout, Cin, "posu_conv2d_dgrad")) return st;
  POSU_REQUIRE(Cin % (16 / esz_of(dtype)) == 0, "posu_conv2d_dgrad: Cin must be a multiple of 16 bytes");
  POSU_REQUIRE(stride == 1 || stride == 2, "posu_conv2d_dgrad: stride 1 or 2");
  POSU_REQUIRE(KH > 0 && KW > 0 && pad >= 0 && pad < KH && pad < KW, "posu_conv2d_dgrad: bad window");
  POSU_REQUIRE(H > 0 && W > 0 && Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1,
               "posu_conv2d_dgrad: H/W do not produce Ho/Wo under this window");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * Cin < (1LL << 31), "posu_conv2d_dgrad: output too large");
  ConvGeom g = base_geom(dy, N, Ho, Wo, Cout, wt, Cin, dtype);
  g.res = residual;
  g.y = dx;
  if (KH == 1 && KW == 1 && pad == 0 && stride == 2 && residual == dx) {
    // 1x1 / stride 2, accumulated in place: dx[2i][2j] += dy[i][j] W^T, the other pixels keep
    // the residual -- a GEMM over dy's pixels instead of the zero-upsampled grid (4x fewer MACs)
    g.Ho = Ho;
    g.Wo = Wo;
    g.M = N * Ho * Wo;
    g.K = Cout;
    g.Kpad = round_up(g.K, bk_of(dtype));
    g.KH = 1;
    g.KW = 1;
    g.stride = 1;
    g.pad_h = 0;
    g.pad_w = 0;
    g.up = 0;
    g.out_H = H;
    g.out_W = W;
    g.ostride = 2;
    return dispatch<false>(dtype, g, 1, stream, "posu_conv2d_dgrad", tile);
  }
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.K = KH * KW * Cout;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = KH;
  g.KW = KW;
  g.stride = 1;
  g.pad_h = KH - 1 - pad;
  g.pad_w = KW - 1 - pad;
  g.up = stride == 2 ? 1 : 0;
  g.out_H = H;
  g.out_W = W;
  return dispatch<false>(dtype, g, 1, stream, "posu_conv2d_dgrad", tile);
}

// Plain GEMM on the conv kernel (1x1 window over M "pixels" of K channels):
//   out[blk][m][j] = sum_k x[m][k] * wt[blk * vblk + j][k]   (f32, blk = column / vblk)
// x: [M][K] dtype, K % 64 == 0 and a power of two; wt: packed [round_up(Ncol, 64)][K]
// dtype.  Used by the cross-view Aggregation (ChannelWiseFC, multiview_pose_resnet.py
// :16-58): the V(V-1) per-pair [HW x HW] matrices are one block matrix, so all target
// views come out of one launch, view-major.
extern "C" int posu_gemm_rows_f32(int dtype, const void* x, int M, int K, const void* wt, int Ncol, int vblk,
                                  float* out, void* stream) {
  POSU_REQUIRE(dtype != POSU_F16X3, "posu_gemm_rows_f32: the split dtype is not supported");
  if (int st = common_checks(dtype, x, wt, out, M, 1, 1, K, Ncol, "posu_gemm_rows_f32")) return st;
  POSU_REQUIRE(K % bk_of(dtype) == 0, "posu_gemm_rows_f32: K must be a multiple of the K-tile");
  POSU_REQUIRE(vblk > 0 && vblk % 8 == 0 && Ncol % vblk == 0, "posu_gemm_rows_f32: vblk must divide Ncol (x8)");
  ConvGeom g = base_geom(x, M, 1, 1, K, wt, Ncol, dtype);
  g.y = out;
  g.Ho = 1;
  g.Wo = 1;
  g.M = M;
  g.K = K;
  g.Kpad = K;
  g.out_H = 1;
  g.out_W = 1;
  g.mode = 2;
  g.vblk = vblk;
  return dispatch<false>(dtype, g, 1, stream, "posu_gemm_rows_f32");
}
