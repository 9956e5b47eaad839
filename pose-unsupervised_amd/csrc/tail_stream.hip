// Tail of an identity Bottleneck (lib/models/pose_resnet.py:79-99, eval mode, BN folded) of
// PoseResNet at 256x256 with the weights streamed straight into registers, for layer2
// (W = 32, planes 128, C = 512) and layer3 (W = 16, planes 256, C = 1024):
//
//     y = relu( bn3(conv3( relu(bn2(conv2_3x3(t1))) )) + x ),   t1 = conv1's output
//
// Why (the round-2 LDS-ring versions, removed in round 4, streamed the weights through a
// two-slot 32 KB LDS ring): so one 32 KB stage is in flight per CU and every
// stage pays a full L2 round trip -- layer3's 52 stages x ~1.5 us = its 80 us (profiles/r02).
// Here the LDS holds only activations; each wave loads its own weight fragments from L2 into
// VGPRs kD k-steps ahead of their use (one contiguous 2 KB per k-step and wave, prepacked by
// packing.pack_tail_stream), so 8 waves x kD x 2 KB are in flight and no barrier sits in the
// weight stream.
//
// One workgroup (8 waves, one per CU) owns 8 image rows (128 px at W = 16, 256 px at W = 32).
// Wave w: pixel group pg = w / NCQ (128 px = 8 m-tiles each, NPG = 8 / NCQ groups), channel
// group cq = w % NCQ (32 output channels = 2 n-tiles of conv2, and of each conv3 chunk of
// 32 NCQ channels).  The pixel operands come from LDS (8 x 1 KB ds_reads per 16 MFMAs).
//   LDS: the t1 window (rows y0-1 .. y0+8, columns -1 .. W, zero padding; staged once by
//        LDS-DMA), BN2; after conv2: t2 [8 W px][P ch] and BN3 over the window.
//   weight stream of a wave: conv2 tap t, channel step c (p = KT t + c, KT = P / 32: the conv
//        kernel's tap-major K order -- bit-identical accumulators), then conv3 chunk nc,
//        channel step c (p = 9 KT + KT nc + c).
// MFMA operands swapped (A = weights, B = pixels): lane (r16, q) accumulates channels
// 4q .. 4q+3 of pixel r16; v_permlane16_swap pairs the 2 n-tiles into 8 consecutive channels.
#include <cstddef>
#include <type_traits>

#include "gemm_common.h"

namespace posu {
namespace {

struct TailSGeom {
  const void* t1;
  const void* x;
  void* y;
  const uint4* wst;  // [8 / NPG channel groups][steps][2 n-tiles][64 lanes] x 16 B
  const float* s2;
  const float* b2;
  const float* s3;
  const float* b3;
  int N, H;
  // NEXT (chained tails): the next identity block's conv1 + BN1 + ReLU computed from this
  // block's output y while it is produced (t1n = relu(y conv1n * s1n + b1n), [N][H][W][P])
  const float* s1n;
  const float* b1n;
  void* t1n;
  long long wseg;  // the weight stream's 64-B segments (warm-up, gemm_common.h)
  int warm;        // warm-up workgroups (0: none)
};

// timing ablations (tools/tail_ablations.sh; never set in the product build, wrong results):
//   1 no MFMAs, 2 no weight loads in the loop, 4 no pixel-fragment LDS reads, 8 no conv3
//   residual loads / y stores, 16 no window DMA, 32 no y stores, 64 no residual loads
#ifndef POSU_TS_ABLATE
#define POSU_TS_ABLATE 0
#endif
constexpr int kAbl = POSU_TS_ABLATE;
// cache-policy bits of the residual loads / y stores (A/B knobs; 0 = default)
#ifndef POSU_TS_LD_AUX
#define POSU_TS_LD_AUX 0
#endif
#ifndef POSU_TS_ST_AUX
#define POSU_TS_ST_AUX 0
#endif

#ifndef POSU_TS_KD
#define POSU_TS_KD 4
#endif
// NEXT (chained) variant: weight prefetch depth and pixel-fragment register sets (0: the default
// below).  Until round 4 the second accumulator set left no room for the plain tail's 4-deep stream
// and two fragment sets (profiles/r03/chain_r3s.txt: layer2 kD 1 / one set, layer3 kD 2 / two sets,
// the latter spilling 34 VGPRs); round 5's 32-bit buffer addressing freed the registers.
#ifndef POSU_TS_KD_NEXT
#define POSU_TS_KD_NEXT 0  // 0: per layer, as measured
#endif
#ifndef POSU_TS_NB_NEXT
#define POSU_TS_NB_NEXT 0
#endif

__device__ __forceinline__ void ld8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <int W, int P, int C, int ROWS, int NW, bool NEXT = false, int MT = 8, int CM = 1, bool DOWN = false,
          int NX = 1>
struct TailCfg {
  static constexpr int kRows = ROWS;               // image rows per workgroup
  static constexpr int kNW = NW;                   // waves per workgroup
  static constexpr int kMT = MT;                   // m-tiles (16 px) per wave
  static constexpr int kPx = kRows * W;            // tile pixels
  static constexpr int kNPG = kPx / (16 * MT);     // pixel groups of 16 MT px
  static constexpr int kNCQ = NW / kNPG;           // channel groups of 32
  static constexpr int kCM = CM;                   // stored halves per logical channel (2: split fp16 pairs)
  static constexpr int kRowB = P * 2 * CM;         // LDS bytes per pixel (bf16 / fp16 / split pairs)
  static constexpr int kWinCols = W + 2;
  static constexpr int kWinPix = (kRows + 2) * kWinCols;
  static constexpr int kBN2 = kWinPix * kRowB;     // s2 b2 f32 behind the window
  static constexpr int kLds = kBN2 + 2 * P * 4;
  static constexpr int kS3 = kPx * kRowB;          // s3 b3 f32 behind t2 (over the window)
  static constexpr int kKT = CM * P / 32;          // k-steps per tap / per conv3 chunk (split: hi, lo per 32 ch)
  static constexpr int kChunk = 32 * kNCQ;         // conv3 output channels per chunk
  static constexpr int kNC = C / kChunk;           // conv3 chunks
  // stream blocks per conv3 chunk (+ DOWN: the downsample's K slice over x; + NEXT: the next conv1's)
  // (NX: the next conv1's output channels in units of P -- 2 when it opens the next layer, round 6)
  static constexpr int kBlk3 = 1 + DOWN + NEXT * NX;
  static constexpr int kSteps = 9 * kKT + kNC * kKT * kBlk3;
  static constexpr int kYC = kS3 + 2 * C * 4;      // NEXT: the y chunk [kPx][P] behind BN3
  static constexpr int kLdsN = NEXT && kYC + kPx * kRowB > kLds ? kYC + kPx * kRowB : kLds;
  // DOWN: the tile's block-input pixels (the downsample's B operand, P channels) behind everything
  // else, staged by LDS-DMA at the start beside the window
  static constexpr int kX0 = kLdsN;
  static constexpr int kLdsAll = DOWN ? kX0 + kPx * kRowB : kLdsN;
  // weight prefetch depth (k-steps); NEXT keeps a second accumulator set live, so its stream
  // runs POSU_TS_KD_NEXT deep
  // (W = 24: nine m-tiles per wave, one fragment set and a two-deep stream -- 256 VGPRs, no
  // spills; no chained W = 24 variant: its second accumulator set does not fit)
  // (round 5: with x / y / t1n behind buffer descriptors the chained variants fit the plain tail's
  // 4-deep stream and two fragment sets without spills -- network 2.3529 / 2.3514 vs 2.3991 / 2.3966
  // ms with round 4's 1-deep / one set (layer2) and 2-deep / two sets (layer3), profiles/r05)
  // (round 6: the chained W = 24 tail runs 2-row tiles, three m-tiles per wave: the plain tail's depths)
  static constexpr int kDW = W == 24 && MT >= 6 ? 2 : !NEXT ? POSU_TS_KD : POSU_TS_KD_NEXT ? POSU_TS_KD_NEXT : 4;
  static constexpr int kNB = W == 24 && MT >= 6 ? 1 : !NEXT ? 2 : POSU_TS_NB_NEXT ? POSU_TS_NB_NEXT : 2;
  static constexpr int kD = kDW < kKT ? kDW : kKT;
  // swizzle keys stay inside a pixel row: 16 chunks or more take (column & 15), the 8-chunk rows of
  // 64-channel 2-byte images (layer1 at 384x384) (column & 7)
  static constexpr int kKM = kRowB / 16 >= 16 ? 15 : kRowB / 16 - 1;
  static_assert(kNPG * kNCQ == NW && kNPG >= 1 && kPx % (16 * MT) == 0 && (16 * MT) % W == 0,
                "every wave: 16 MT px (whole image rows) x 32 channels");
  // W = 24 (R152@384's layer3, round 5): m-tiles straddle image rows -- m-tile i = 3 m + c holds
  // tile pixels 48 m + 16 c .. (rows 2 m, 2 m + 1), three lane-address classes c
  static_assert(W % 16 == 0 || (W == 24 && MT % 3 == 0 && kNPG == 1), "W a multiple of 16, or 24 in 3-m-tile periods");
  static_assert(kS3 + 2 * C * 4 <= kBN2, "t2 and BN3 fit over the window");
  static_assert(kLdsAll <= 160 * 1024, "LDS");
  static_assert(!NEXT || kChunk == P, "the next conv1 takes one y chunk per K slice of P channels");
  static_assert(kKT % kD == 0, "the ring slot of a k-step is static inside a block");
  static_assert(CM == 1 || (kD % 2 == 0 && kNB == 2 && W % 16 == 0), "split pairs: even stream depth, two fragment sets");
};

// P-channel LDS row of pixel `pix`, 16-B chunk `chunk`: the chunk index XOR `key` = the pixel's
// column (in its LDS image) & 15.  Keyed by the column rather than the pixel index, the key of
// an m-tile's lane is the same for every m-tile of a wave, so a k-step's fragment addresses are
// four per-block base registers plus compile-time offsets (no address arithmetic in the loop).
template <int RowB>
__device__ __forceinline__ int swzp(int pix, int key, int chunk) { return pix * RowB + ((chunk ^ key) << 4); }

// swizzle key of the t1 window's pixel (window row wr, column wc): the column & 15 for W a multiple
// of 16; for W = 24 the column plus 8 on odd rows, so the 16 lanes of an m-tile that straddles two
// image rows (columns 16 .. 23 of one, 0 .. 7 of the next) still hit 16 distinct chunk slots
template <int W>
__device__ __forceinline__ int wkey(int wr, int wc) {
  return W % 16 == 0 ? (wc & 15) : ((wc + 8 * (wr & 1)) & 15);
}

// waves per CU the four-m-tile variant is compiled for (A/B builds: 8 gives it 256 registers)
#ifndef POSU_TS_MT4_WAVES
#define POSU_TS_MT4_WAVES 12
#endif
// DOWN (round 6, layer1's first block in split fp16): the Bottleneck with a stride-1 1x1 downsample
// (pose_resnet.py:136-141) -- no residual; each conv3 chunk also runs the downsample over the block
// input x (P channels, staged in LDS) into the same accumulators, [w3*s3 | wd*sd] with shift = b3 + bd
// (posu_conv1x1_dual_fwd's K order: bit-identical to it)
// NX = 2 (round 6, split fp16): the next conv1 has 2 P outputs -- the first block of the NEXT layer
// (layer2 / 3 / 4 block 0's conv1, C -> 2 P at this map size) -- so the last identity block of a layer
// chains it too: two accumulator sets, each over the same y chunk image
template <typename T, int W, int P, int C, int ROWS, int NW, bool NEXT = false, int MT = 8, bool DOWN = false,
          int NX = 1>
__global__ __launch_bounds__(NW * 64, (DOWN && Op<T>::SPLIT ? 4 : W == 24 && MT == 6 ? 32 : Op<T>::SPLIT || MT == 8 || W == 48 || W == 96 || NX == 2 ? 8 : POSU_TS_MT4_WAVES) / NW) void tail_stream_kernel(TailSGeom g) {
  using O = Op<T>;
  // split fp16 (POSU_F16X3, round 6): every pixel row holds [hi 32 | lo 32] per 32 channels, i.e. the
  // kernel is the same GEMM over twice the K, whose k-step pairs (2c, 2c + 1) -- the hi and the lo
  // halves of the same 32 channels, in the weight stream too -- are multiplied as hi.hi +
  // lo(w).hi(x) + hi(w).lo(x) (the conv kernel's order per accumulator: bit-identical to it); the
  // epilogues join residual pairs and split their outputs
  constexpr bool SPL = O::SPLIT;
  constexpr int CM = SPL ? 2 : 1;
  using K = TailCfg<W, P, C, ROWS, NW, NEXT, MT, CM, DOWN, NX>;
  constexpr int kRows = ROWS, kThreads = NW * 64;
  constexpr int ES = 2, kD = K::kD;
  __shared__ __attribute__((aligned(16))) char smem[K::kLdsAll];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int wu = __builtin_amdgcn_readfirstlane(wid);
  const int pg = wu / K::kNCQ, cq = wu - pg * K::kNCQ;
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const int H = g.H;
  const int tiles_per_img = H / kRows;
  const int n = blockIdx.x / tiles_per_img;
  const int y0 = (blockIdx.x - n * tiles_per_img) * kRows;
  float* bn2 = reinterpret_cast<float*>(smem + K::kBN2);
  for (int c = tid; c < P; c += kThreads) {
    bn2[c] = g.s2[c];
    bn2[P + c] = g.b2[c];
  }

  // ---- the t1 window: 1 KB wave-instructions (1024 / kRowB pixels each), instruction m by wave m & 7
  {
    constexpr int kPixPerInst = 1024 / K::kRowB, kInst = K::kWinPix / kPixPerInst;
    static_assert(K::kWinPix % kPixPerInst == 0, "whole instructions");
    constexpr int kChunks = K::kRowB / 16;
    const u32x4 t1s = make_srd(g.t1, g.N * H * W * P * CM * ES);
    const int sub = lane / kChunks, pc = lane % kChunks;
#pragma unroll
    for (int k = 0; k < (kInst + NW - 1) / NW; ++k) {
      const int m = wid + NW * k;
      if (m < kInst && !(kAbl & 16)) {  // wave-uniform
        const int pix = kPixPerInst * m + sub;
        const int wr = pix / K::kWinCols, wc = pix - wr * K::kWinCols;
        const int yy = y0 + wr - 1, xx = wc - 1;
        const int lc = pc ^ (wkey<W>(wr, wc) & K::kKM);
        const bool ok = static_cast<unsigned>(yy) < static_cast<unsigned>(H) && static_cast<unsigned>(xx) < W;
        dma16(t1s, ok ? (((n * H + yy) * W + xx) * P * CM + 8 * lc) * ES : kOOB, lds0 + static_cast<unsigned>(m) * 1024u);
      }
    }
    if constexpr (DOWN) {
      // the block input's tile pixels (x: [N][H][W][P], the rows y0 .. y0 + kRows - 1 contiguous),
      // pixel p's chunks keyed by its column & 15 (the t2 image's layout)
      constexpr int kXInst = K::kPx / kPixPerInst;
      static_assert(K::kPx % kPixPerInst == 0, "whole instructions");
      const u32x4 xs = make_srd(g.x, g.N * H * W * P * CM * ES);
#pragma unroll
      for (int k = 0; k < (kXInst + NW - 1) / NW; ++k) {
        const int m = wid + NW * k;
        if (m < kXInst) {
          const int pix = kPixPerInst * m + sub;
          const int lc = pc ^ ((pix % W) & K::kKM);
          dma16(xs, ((n * H + y0) * W * P * CM + pix * P * CM + 8 * lc) * ES,
                lds0 + static_cast<unsigned>(K::kX0 + m * 1024));
        }
      }
    }
  }

  // ---- the weight stream: fragment j (n-tile 2 cq + j of the step's output group) of k-step p,
  // one contiguous 2 KB per k-step and wave (prefetches past the end reload the last k-step)
  const char* wst = reinterpret_cast<const char*>(g.wst) + cq * (K::kSteps * 2 * 1024);  // wave-uniform
  const int wlane = lane * 16;
  auto frag = [&](int p, int j) -> const uint4* {
    return reinterpret_cast<const uint4*>(wst + (min(p, K::kSteps - 1) * 2 + j) * 1024 + wlane);
  };
  uint4 wa[kD][2];
#pragma unroll
  for (int d = 0; d < kD; ++d) {
    wa[d][0] = *frag(d, 0);
    wa[d][1] = *frag(d, 1);
  }
  unsigned wv[kWarmLoads];   // the stream's warm-up (gemm_common.h): every line requested up front
  warm_issue(wv, g.wst, g.wseg, g.warm, kThreads);
  vm_wait<0>();  // the window (LDS-DMA) and the first fragments
  warm_use(wv);
  lds_barrier();

  f32x4 acc[MT][2];   // [m-tile i: tile pixels 16 MT pg + 16 i ..][n-tile j]
  f32x4 acc1[NX][MT][2];  // NEXT: the next conv1's accumulators over the whole chunk loop
  auto zero = [&](f32x4 (&a)[MT][2]) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) a[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // the pair of n-tiles -> this lane's 8 consecutive channels cpair .. cpair + 7 of pixel r16
  auto pair = [&](const f32x4 (&a)[MT][2], int i, float* v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[i][0][e]), __float_as_uint(a[i][1][e]),
                                                       false, false);
      v[e] = __uint_as_float(sw[0]);
      v[4 + e] = __uint_as_float(sw[1]);
    }
  };
  const int cpair = 16 * (q & 1) + 8 * (q >> 1);
  constexpr bool kLateRes = NEXT || (W == 24 && MT == 6);   // residual loads after a chunk's MFMAs
  // relu(v * sc + sh (+ r)) over this lane's 8 values; the multiply-add as an explicit fma, the conv
  // epilogue's contraction: left to the compiler, the split variants' epilogues were vectorised into
  // v_mul + v_pk_add (two roundings) and differed from the conv launches in the last f32 bit
  auto bn_relu = [&](float* v, const float* sc, const float* sh, const float* r) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(__builtin_fmaf(v[e], sc[e], sh[e]) + (r ? r[e] : 0.f), 0.f);
  };
  // m-tile i's tile pixel (row-major in the tile) for this lane
  auto tpix = [&](int i) { return 16 * MT * pg + 16 * i + r16; };
  // one block of kKT k-steps (one conv2 tap, or one conv3 output chunk over t2's P channels):
  // k-step d reads, for m-tile i, the pixel lpix + coff(i) (coff compile-time) of an LDS image
  // with `cols` pixels per row at 16-B chunk 4 d + q, swizzled by the lane's key (column & 15).
  // The pixel fragments of k-step d + 1 are read while k-step d's MFMAs run (two register
  // sets); the scheduling barriers keep the compiler from hoisting more of them.
  // chunk (4 d + q) ^ key = 4 ((d & 3) ^ (key >> 2)) + 16 (d >> 2) + (q ^ (key & 3)): four base
  // pointers per (lane pixel, key), the k-step's 16 B at kb[d & 3] + (d >> 2) * 256
  auto bases = [&](const char* (&kb)[4], int base, int lpix, int key) {
    key &= K::kKM;
    const char* lb = smem + base + lpix * K::kRowB + ((q ^ (key & 3)) << 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) kb[k] = lb + ((k ^ (key >> 2)) << 6);
  };
  auto block = [&](f32x4 (&acc)[MT][2], int blk, int base, int lpix, int key, auto coff) {
    constexpr int NB = K::kNB;  // pixel-fragment register sets
    uint4 b[NB][MT];
    const char* kb[4];
    bases(kb, base, lpix, key);
    // W = 24 window reads (conv2, coff = nullptr_t): m-tile i = 3 m + c reads from its class's
    // bases at + 2 m window rows
    const char* kc[3][4];
    constexpr bool W24 = W % 16 != 0 && std::is_same<decltype(coff), std::nullptr_t>::value;
    if constexpr (W24) {
      const int dy = lpix, dx = key;   // (the W = 24 window call passes the tap here)
      const int bb = r16 >= 8;
      const int ro[3] = {0, bb, 1}, co[3] = {r16, 16 + r16 - 24 * bb, 8 + r16};
#pragma unroll
      for (int c = 0; c < 3; ++c)
        bases(kc[c], base, (ro[c] + dy) * K::kWinCols + co[c] + dx, wkey<W>(ro[c] + dy, co[c] + dx));
    }
    auto rd = [&](int i, int d) -> uint4 {
      if (kAbl & 4) return make_uint4(i, d, lane, blk);
      if constexpr (W24)
        return *reinterpret_cast<const uint4*>(kc[i % 3][d & 3] + (i / 3) * 2 * K::kWinCols * K::kRowB + (d >> 2) * 256);
      else
        return *reinterpret_cast<const uint4*>(kb[d & 3] + coff(i) * K::kRowB + (d >> 2) * 256);
    };
#pragma unroll
    for (int i = 0; i < MT; ++i) b[0][i] = rd(i, 0);
#pragma unroll
    for (int d = 0; d < K::kKT; ++d) {
      if (NB == 2 && d + 1 < K::kKT) {
#pragma unroll
        for (int i = 0; i < MT; ++i) b[(d + 1) % NB][i] = rd(i, d + 1);
      }
      const int s = d % kD;
      if constexpr (SPL) {
        // the hi step (d even) issues both uses of its pixel fragments, hi.hi then lo(w).hi(x) (the
        // lo weights of step d + 1 are in their slot already), the lo step hi(w).lo(x); then the slot
        // used for the last time is refilled: the lo weights' after the hi step, the hi weights'
        // after the lo step (a slot keeps its k-steps mod kD)
        const int s2 = (d & 1) ? s - 1 : s + 1;
        if ((d & 1) == 0) {
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) O::mma(acc[i][j], wa[s][j], b[d % NB][i]);
        }
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) O::mma(acc[i][j], wa[s2][j], b[d % NB][i]);
        const int p = K::kKT * blk + ((d & 1) ? d - 1 : d + 1) + kD;
        if (!(kAbl & 2)) {
          wa[s2][0] = *frag(p, 0);
          wa[s2][1] = *frag(p, 1);
        }
      } else {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            if (kAbl & 1) acc[i][j][0] += __uint_as_float(wa[s][j].x ^ b[d % NB][i].y);
            else O::mma(acc[i][j], wa[s][j], b[d % NB][i]);
          }
          // one set: m-tile i's fragment of the next k-step once its MFMAs are issued
          if (NB == 1 && d + 1 < K::kKT) b[0][i] = rd(i, d + 1);
        }
        const int p = K::kKT * blk + d + kD;
        if (!(kAbl & 2)) {
          wa[s][0] = *frag(p, 0);
          wa[s][1] = *frag(p, 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- conv2: 9 taps x kKT channel steps over the window
  zero(acc);
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    const int dy = t / 3, dx = t - 3 * (t / 3);
    if constexpr (W % 16 != 0) {
      block(acc, t, 0, dy, dx, nullptr);   // W = 24: per-class lane addresses (one pixel group)
    } else {
      // window pixel of m-tile i: tile row (16 MT pg + 16 i) / W + dy, column (16 i) % W + r16 + dx
      block(acc, t, 0, ((16 * MT / W) * pg + dy) * K::kWinCols + r16 + dx, wkey<W>(0, r16 + dx),
            [&](int i) { return (16 * i / W) * K::kWinCols + (16 * i) % W; });
    }
  }
  const T* xg = reinterpret_cast<const T*>(g.x) + static_cast<size_t>(n * H + y0) * W * C * CM;
  T* yg = reinterpret_cast<T*>(g.y) + static_cast<size_t>(n * H + y0) * W * C * CM;
  // the tile's x / y (/ t1n) through buffer descriptors: a lane's 32-bit byte offset plus
  // compile-time per-m-tile / per-chunk steps, instead of a 64-bit address per m-tile (the
  // chained layer3 tail spilled such addresses: 34 VGPRs, round 4); stores keep soffset 0 (the
  // store-data hazard)
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(xg), 0, K::kPx * C * CM * ES, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(yg, 0, K::kPx * C * CM * ES, 0x00020000);
  // m-tile 0, chunk 0 (split: the hi half; the lo half 32 elements = 64 B further)
  const int lane_xy = ((16 * MT * pg + r16) * C * CM + (SPL ? split_ch(32 * cq + cpair) : 32 * cq + cpair)) * ES;
  auto xy_off = [&](int i, int nc) { return lane_xy + (16 * i * C + K::kChunk * nc) * CM * ES; };
  // conv3 chunk nc's residual in the epilogue's lane layout (rl: the split pairs' lo halves)
  auto res_load = [&](int nc, uint4 (&rv)[MT], uint4 (&rl)[MT]) {
    const int c0 = K::kChunk * nc + 32 * cq + cpair;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      if (kAbl & 72) {
        rv[i] = make_uint4(i, c0, 0, 0);
        rl[i] = rv[i];
      } else {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(xrs, xy_off(i, nc), 0, POSU_TS_LD_AUX);
        rv[i] = make_uint4(v[0], v[1], v[2], v[3]);
        if constexpr (SPL) {
          const auto l = __builtin_amdgcn_raw_buffer_load_b128(xrs, xy_off(i, nc) + 64, 0, POSU_TS_LD_AUX);
          rl[i] = make_uint4(l[0], l[1], l[2], l[3]);
        }
      }
    }
  };
  // 16-B store of the 8 values of this lane (split: the hi and the lo halves, 64 B apart)
  auto st8 = [&](__amdgpu_buffer_rsrc_t rs, int off, const float* v) {
    if constexpr (SPL) {
      uint4 h, l;
      split8(v, h, l);
      __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned){h.x, h.y, h.z, h.w}, rs,
                                             off, 0, POSU_TS_ST_AUX);
      __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned){l.x, l.y, l.z, l.w}, rs,
                                             off + 64, 0, POSU_TS_ST_AUX);
    } else {
      const uint4 o = O::store_vals(v);
      __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned){o.x, o.y, o.z, o.w}, rs,
                                             off, 0, POSU_TS_ST_AUX);
    }
  };
  // the same 8 values into an LDS image of P-channel rows (t2, the NEXT y chunk): chunk c8 (the
  // logical 8-channel chunk in the row), split: hi and lo chunks
  auto lds8 = [&](int base, int pix, int c8, const float* v) {
    if constexpr (SPL) {
      uint4 h, l;
      split8(v, h, l);
      const int ch = split_ch(8 * c8) >> 3;
      *reinterpret_cast<uint4*>(smem + base + swzp<K::kRowB>(pix, r16 & K::kKM, ch)) = h;
      *reinterpret_cast<uint4*>(smem + base + swzp<K::kRowB>(pix, r16 & K::kKM, ch + 4)) = l;
    } else {
      *reinterpret_cast<uint4*>(smem + base + swzp<K::kRowB>(pix, r16 & K::kKM, c8)) = O::store_vals(v);
    }
  };
  // BN2 + ReLU -> t2 over the window (every wave is done reading it first), BN3 beside it
  lds_barrier();
  {
    float* b3l = reinterpret_cast<float*>(smem + K::kS3);
    for (int c = tid; c < C; c += kThreads) {
      b3l[c] = g.s3[c];
      b3l[C + c] = g.b3[c];
    }
    const int c0 = 32 * cq + cpair;
    float sc[8], sh[8];
    ld8(bn2 + c0, sc);
    ld8(bn2 + P + c0, sh);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8];
      pair(acc, i, v);
      bn_relu(v, sc, sh, nullptr);
      lds8(0, tpix(i), c0 >> 3, v);
    }
  }
  lds_barrier();

  // ---- conv3: output chunk nc (kChunk channels; this wave's 32), kKT channel steps over t2
  const float* b3l = reinterpret_cast<const float*>(smem + K::kS3);
  auto chunk = [&](int nc, uint4 (&rv)[MT], uint4 (&rl)[MT]) {
    const int c0 = K::kChunk * nc + 32 * cq + cpair;
    zero(acc);
    block(acc, 9 + K::kBlk3 * nc, 0, 16 * MT * pg + r16, r16, [&](int i) { return 16 * i; });
    // DOWN: the downsample's K slice over the block input into the same accumulators
    if constexpr (DOWN) block(acc, 9 + K::kBlk3 * nc + 1, K::kX0, 16 * MT * pg + r16, r16, [&](int i) { return 16 * i; });
    // NEXT: the residual after the MFMAs (the next conv1's accumulators take its registers; so do
    // the W = 24 4-row tiles' 128-register budget)
    if constexpr (kLateRes && !DOWN) res_load(nc, rv, rl);
    float sc[8], sh[8];
    ld8(b3l + c0, sc);
    ld8(b3l + C + c0, sh);
    if constexpr (NEXT) {
      if (nc > 0) lds_barrier();  // every wave is done reading the previous y chunk
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8], r[8];
      pair(acc, i, v);
      if constexpr (DOWN) {
        bn_relu(v, sc, sh, nullptr);   // no residual: the downsample is in the accumulators
      } else {
        if constexpr (SPL) join8(rv[i], rl[i], r);
        else O::load_vals(rv[i], r);
        bn_relu(v, sc, sh, r);
      }
      if (kAbl & 40) asm volatile("" ::"v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
      else st8(yrs, xy_off(i, nc), v);
      // NEXT: the chunk's y, laid out like t2 ([pixel][P] rows, column-keyed swizzle)
      if constexpr (NEXT) lds8(K::kYC, tpix(i), (32 * cq + cpair) >> 3, v);
    }
    if constexpr (NEXT) {
      // the next block's conv1 over this K slice (y channels kChunk nc ..): same k order as a
      // conv launch over y, so t1n is bit-identical to it
      lds_barrier();
#pragma unroll
      for (int h = 0; h < NX; ++h)
        block(acc1[h], 9 + K::kBlk3 * nc + 1 + DOWN + h, K::kYC, 16 * MT * pg + r16, r16, [&](int i) { return 16 * i; });
    }
  };
  // unrolled: hipcc's wait counts at a loop head merge both paths and made every chunk's first
  // weight wait also wait for the previous chunk's y stores (layer2 tail 90.7 -> 86.7 us)
  if constexpr (NEXT) {
#pragma unroll
    for (int h = 0; h < NX; ++h) zero(acc1[h]);
  }
#pragma unroll
  for (int nc = 0; nc < K::kNC; ++nc) {
    // the chunk's residual, kKT k-steps ahead of its epilogue (the weight fragments consumed
    // meanwhile were loaded before it: the in-order vmcnt does not hold them back)
    uint4 rv[MT], rl[MT];
    if constexpr (!kLateRes && !DOWN) res_load(nc, rv, rl);
    chunk(nc, rv, rl);
  }
  if constexpr (NEXT) {
    // t1n = relu(conv1n * s1n + b1n) [.., NX P], this lane's 8 channels (of each half) of each m-tile's pixel
    constexpr int PN = NX * P;
    T* tg = reinterpret_cast<T*>(g.t1n) + static_cast<size_t>(n * H + y0) * W * PN * CM;
    const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(tg, 0, K::kPx * PN * CM * ES, 0x00020000);
#pragma unroll
    for (int h = 0; h < NX; ++h) {
      const int c0 = h * P + 32 * cq + cpair;
      float sc[8], sh[8];
      ld8(g.s1n + c0, sc);
      ld8(g.b1n + c0, sh);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float v[8];
        pair(acc1[h], i, v);
        bn_relu(v, sc, sh, nullptr);
        st8(trs, (tpix(i) * PN * CM + (SPL ? split_ch(c0) : c0)) * ES, v);
      }
    }
  }
}

// split fp16 instances (round 6): layer1 (W = 64, planes 64: 2 rows x 64 px, four waves as 2 pixel x 2
// channel groups), layer2 (2 rows x 32 px, four waves), layer3 (4 rows x 16 px, eight waves) -- the
// pairs double the t1 window, so the tiles are the bf16 ones' small variants (68 / 69 / 110 KB of LDS)
template <int W, int P, int C, int ROWS, int NW, bool NEXT, int MT, bool DOWN = false, int NX = 1>
void launch_tail_split(const TailSGeom& g, hipStream_t s) {
  hipLaunchKernelGGL((tail_stream_kernel<f16s_t, W, P, C, ROWS, NW, NEXT, MT, DOWN, NX>),
                     dim3(static_cast<unsigned>(g.N * (g.H / ROWS))), dim3(NW * 64), 0, s, g);
}

template <int W, int P, int C, int ROWS, int NW, bool NEXT = false, int MT = 8, bool DOWN = false, int NX = 1>
void launch_tail(int dtype, const TailSGeom& g, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>(g.N * (g.H / ROWS)));
  if (dtype == POSU_BF16)
    hipLaunchKernelGGL((tail_stream_kernel<uint16_t, W, P, C, ROWS, NW, NEXT, MT, DOWN, NX>), grid, dim3(NW * 64), 0, s,
                       g);
  else
    hipLaunchKernelGGL((tail_stream_kernel<f16_t, W, P, C, ROWS, NW, NEXT, MT, DOWN, NX>), grid, dim3(NW * 64), 0, s, g);
}

// layer3 at W = 24 (R152@384): the plain tail's rows per tile -- 6 (144 px, 9 m-tiles per wave, one
// workgroup per CU) or 4 (96 px, 6 m-tiles per wave, 80 KB of LDS: two workgroups per CU, 128 registers
// with the residual loaded after a chunk's MFMAs; measured slower: configs[4] 7.10 vs 6.71 ms, call r6s)
#ifndef POSU_TS_L3W_ROWS
#define POSU_TS_L3W_ROWS 6
#endif
// layer3's 4-row tiles below this many 8-row workgroups (A/B builds: 0 never, a large value always)
#ifndef POSU_TS_L3_SMALL_GRID
#define POSU_TS_L3_SMALL_GRID 256
#endif
// tiles: layer3 8 rows x 16 px with 8 waves (one workgroup per CU, 256 at batch 128); layer2
// 4 rows x 32 px with 4 waves, two workgroups per CU, so one's conv3 epilogue (residual loads,
// y stores) overlaps the other's MFMAs
#ifndef POSU_TS_L2_ROWS
#define POSU_TS_L2_ROWS 4
#endif
// layer2 m-tiles per wave: 8 (4-row tiles of 128 px, 4 waves) or 4 (2-row tiles of 64 px, 4 waves,
// up to three workgroups per CU)
#ifndef POSU_TS_L2_MT
#define POSU_TS_L2_MT 8
#endif
constexpr int kL2MT = POSU_TS_L2_MT;
constexpr int kL2Rows = POSU_TS_L2_ROWS * kL2MT / 8, kL2Waves = POSU_TS_L2_ROWS;

}  // namespace
}  // namespace posu

using namespace posu;

namespace {
int tail_stream_impl(const char* name, int dtype, const void* t1, const void* x, int N, int H, int W, int C, int P,
                     const void* wstream, long long wstream_bytes, const float* s2, const float* b2,
                     const float* s3, const float* b3, void* y, const float* s1n, const float* b1n, void* t1n,
                     void* stream, bool down = false, int nx = 1) {
  const std::string what = name;
  const bool next = t1n != nullptr;
  const bool spl = dtype == POSU_F16X3;
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16 || spl, what + ": dtype must be BF16, F16 or F16X3");
  POSU_REQUIRE(t1 && x && wstream && s2 && b2 && s3 && b3 && y, what + ": null pointer");
  POSU_REQUIRE(x != y && t1 != y, what + ": the output must not alias an input");
  POSU_REQUIRE(!next || (s1n && b1n && t1n != y && t1n != x && t1n != t1),
               what + ": the next conv1 needs its BN and an output that aliases no other operand");
  const bool l3 = W == 16 && C == 1024 && P == 256, l2 = W == 32 && C == 512 && P == 128;
  const bool l3w = W == 24 && C == 1024 && P == 256;   // layer3 at 384x384 (R152 configs[4])
  const bool l2w = W == 48 && C == 512 && P == 128;    // layer2 at 384x384
  const bool l1 = W == 64 && C == 256 && P == 64;      // layer1 at 256x256 (the split dtype only)
  const bool l1w = W == 96 && C == 256 && P == 64;     // layer1 at 384x384 (R152 configs[4]; bf16 / fp16)
  POSU_REQUIRE(l2 || l3 || l3w || l2w || (spl && l1) || (!spl && l1w),
               what + ": built for layer2 (W = 32 or 48, C = 512, planes = 128) and layer3 (W = 16 or 24, C = 1024, "
                      "planes = 256) of PoseResNet at 256x256 / 384x384, layer1 at 384x384 (W = 96, C = 256, planes "
                      "64; BF16 / F16) and (split fp16) layer1 at 256x256 (W = 64)");
  POSU_REQUIRE(!spl || !(l3w || l2w), what + ": the split dtype runs the 256x256 tails (W = 64, 32, 16)");
  POSU_REQUIRE(!down || (spl && l1) || (!spl && l1w),
               what + ": built for layer1's first Bottleneck (x 64 -> y 256 channels, planes 64) at W = 64 in split "
                      "fp16 and at W = 96 in BF16 / F16");
  const int cm = spl ? 2 : 1;   // stored halves per logical channel
  POSU_REQUIRE(nx == 1 || (nx == 2 && next && !down && (l2 || l3 || (spl && l1))),
               what + ": a next conv1 of 2 P outputs is chained by the 256x256 identity tails only (layer1: split)");
  {
    // the stream the selected variant reads: NCQ channel groups x (9 KT conv2 + NC KT conv3 [+ NC KT
    // next conv1]) k-steps x 2 n-tiles x 1 KB (packing.pack_tail_stream); split: KT = 2 P / 32
    const long long kt = cm * P / 32, nc = C / P;
    const long long need = (P / 32) * (9 * kt + (1 + down + (next ? nx : 0)) * nc * kt) * 2 * 64 * 8 * 2;
    POSU_REQUIRE(wstream_bytes == need, what + ": wstream holds " + std::to_string(wstream_bytes) + " bytes, the " +
                                            (next ? "chained" : "plain") + " tail reads " + std::to_string(need));
  }
  // (W = 24 chained: 2-row tiles, round 6; the plain W = 24 tail keeps 6-row tiles)
  // layer3 at W = 16: 8-row tiles (128 px, 8 m-tiles per wave) while they give every CU a
  // workgroup, else 4-row tiles (64 px, 4 m-tiles per wave): at batch 64 (BASELINE configs[1]) the
  // 8-row grid left half the CUs idle (128 workgroups)
  const bool l3h = l3 && N > 0 && H % 4 == 0 && static_cast<long long>(N) * (H / 8) < POSU_TS_L3_SMALL_GRID;
  // (nx = 2, bf16 / fp16: the 4-m-tile variants -- layer2 2-row, layer3 4-row tiles -- whose second
  // accumulator set fits twice)
  const int rows = spl ? (l3 ? 4 : 2) : nx == 2 ? (l3 ? 4 : 2) : l3 ? (l3h ? 4 : 8) : l3w ? (next ? 2 : POSU_TS_L3W_ROWS) :
                   (l2w || l1w) ? 2 : kL2Rows;
  POSU_REQUIRE(N > 0 && H > 0 && H % rows == 0,
               what + ": H must be a positive multiple of " + std::to_string(rows) + " (the tile rows)");
  POSU_REQUIRE(!down || x != t1n, what + ": t1n must not alias x");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * 2 * cm < (1LL << 31) - 256,
               what + ": activation exceeds the 2 GiB addressing range");
  for (const void* p : {t1, x, static_cast<const void*>(y), wstream, static_cast<const void*>(s3),
                        static_cast<const void*>(b3), next ? t1n : t1, static_cast<const void*>(next ? s1n : s3),
                        static_cast<const void*>(next ? b1n : b3)})
    POSU_REQUIRE((reinterpret_cast<size_t>(p) & 15) == 0, what + ": pointers must be 16-byte aligned");
  TailSGeom g{};
  g.t1 = t1;
  g.x = x;
  g.y = y;
  g.wst = static_cast<const uint4*>(wstream);
  g.s2 = s2;
  g.b2 = b2;
  g.s3 = s3;
  g.b3 = b3;
  g.N = N;
  g.H = H;
  g.s1n = s1n;
  g.b1n = b1n;
  g.t1n = t1n;
  g.wseg = wstream_bytes / 64;
  g.warm = warm_wgs(wstream_bytes);
  hipStream_t s = as_stream(stream);
  if (spl && down) {
    if (next) launch_tail_split<64, 64, 256, 2, 4, true, 4, true>(g, s);
    else launch_tail_split<64, 64, 256, 2, 4, false, 4, true>(g, s);
  } else if (spl && nx == 2) {
    if (l1) launch_tail_split<64, 64, 256, 2, 4, true, 4, false, 2>(g, s);
    else if (l2) launch_tail_split<32, 128, 512, 2, 4, true, 4, false, 2>(g, s);
    else launch_tail_split<16, 256, 1024, 4, 8, true, 4, false, 2>(g, s);
  } else if (spl) {
    if (l1) {
      if (next) launch_tail_split<64, 64, 256, 2, 4, true, 4>(g, s);
      else launch_tail_split<64, 64, 256, 2, 4, false, 4>(g, s);
    } else if (l2) {
      if (next) launch_tail_split<32, 128, 512, 2, 4, true, 4>(g, s);
      else launch_tail_split<32, 128, 512, 2, 4, false, 4>(g, s);
    } else {
      if (next) launch_tail_split<16, 256, 1024, 4, 8, true, 4>(g, s);
      else launch_tail_split<16, 256, 1024, 4, 8, false, 4>(g, s);
    }
  } else if (nx == 2) {   // a layer's last tail chaining the next layer's first conv1 (2 P outputs)
    if (l3) launch_tail<16, 256, 1024, 4, 8, true, 4, false, 2>(dtype, g, s);
    else launch_tail<32, 128, 512, 2, 4, true, 4, false, 2>(dtype, g, s);
  } else if (l1w) {   // 2 rows x 96 px = 192 px, 6 m-tiles per wave (one image row), 4 waves
    if (down) {
      if (next) launch_tail<96, 64, 256, 2, 4, true, 6, true>(dtype, g, s);
      else launch_tail<96, 64, 256, 2, 4, false, 6, true>(dtype, g, s);
    } else {
      if (next) launch_tail<96, 64, 256, 2, 4, true, 6>(dtype, g, s);
      else launch_tail<96, 64, 256, 2, 4, false, 6>(dtype, g, s);
    }
  } else if (l3h) {
    if (next) launch_tail<16, 256, 1024, 4, 8, true, 4>(dtype, g, s);
    else launch_tail<16, 256, 1024, 4, 8, false, 4>(dtype, g, s);
  } else if (l3) {
    if (next) launch_tail<16, 256, 1024, 8, 8, true>(dtype, g, s);
    else launch_tail<16, 256, 1024, 8, 8>(dtype, g, s);
  } else if (l3w) {   // 6 rows x 24 px = 144 px, 9 m-tiles per wave (chained: 2 rows x 24 px, 3 m-tiles)
    if (next) launch_tail<24, 256, 1024, 2, 8, true, 3>(dtype, g, s);
    else launch_tail<24, 256, 1024, POSU_TS_L3W_ROWS, 8, false, POSU_TS_L3W_ROWS * 3 / 2>(dtype, g, s);
  } else if (l2w) {   // 2 rows x 48 px = 96 px, 6 m-tiles per wave, 4 waves
    if (next) launch_tail<48, 128, 512, 2, 4, true, 6>(dtype, g, s);
    else launch_tail<48, 128, 512, 2, 4, false, 6>(dtype, g, s);
  } else {
    if (next) launch_tail<32, 128, 512, kL2Rows, kL2Waves, true, kL2MT>(dtype, g, s);
    else launch_tail<32, 128, 512, kL2Rows, kL2Waves, false, kL2MT>(dtype, g, s);
  }
  return check_launch(name);
}
}  // namespace

extern "C" int posu_bottleneck_tail_stream_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                               int P, const void* wstream, long long wstream_bytes,
                                               const float* s2, const float* b2, const float* s3, const float* b3,
                                               void* y, void* stream) {
  return tail_stream_impl("posu_bottleneck_tail_stream_fwd", dtype, t1, x, N, H, W, C, P, wstream, wstream_bytes, s2,
                          b2, s3, b3, y, nullptr, nullptr, nullptr, stream);
}

// Chained identity Bottlenecks: the tail above, and the NEXT identity block's conv1 (+ BN1 +
// ReLU) over this block's output y while its chunks are produced -- t1n, which the next
// block's tail takes instead of a conv1 launch over y.  wstream = packing.pack_tail_stream
// (conv2, conv3, next conv1).
extern "C" int posu_bottleneck_tail_stream_next_fwd(int dtype, const void* t1, const void* x, int N, int H, int W,
                                                    int C, int P, const void* wstream, long long wstream_bytes,
                                                    const float* s2, const float* b2, const float* s3,
                                                    const float* b3, void* y, const float* s1n, const float* b1n,
                                                    void* t1n, void* stream) {
  if (!t1n) {
    set_error("posu_bottleneck_tail_stream_next_fwd: null pointer (t1n)");
    return POSU_ERR_ARG;
  }
  return tail_stream_impl("posu_bottleneck_tail_stream_next_fwd", dtype, t1, x, N, H, W, C, P, wstream,
                          wstream_bytes, s2, b2, s3, b3, y, s1n, b1n, t1n, stream);
}

// Layer1's first Bottleneck (split fp16, round 6): conv2 + [conv3 | downsample] dual GEMM + ReLU in one
// launch (the downsample over the block input x [N, H, 64, P] staged in LDS), optionally chained with
// the next block's conv1 (t1n != nullptr).  s3 / b3: the dual GEMM's scale / shift (b3 + bd);
// wstream = packing.pack_down_tail_stream(conv2 pack, dual pack[, next conv1 pack]).
extern "C" int posu_bottleneck_down_tail_stream_fwd(int dtype, const void* t1, const void* x, int N, int H, int W,
                                                    int C, int P, const void* wstream, long long wstream_bytes,
                                                    const float* s2, const float* b2, const float* s3,
                                                    const float* b3, void* y, const float* s1n, const float* b1n,
                                                    void* t1n, void* stream) {
  return tail_stream_impl("posu_bottleneck_down_tail_stream_fwd", dtype, t1, x, N, H, W, C, P, wstream, wstream_bytes,
                          s2, b2, s3, b3, y, s1n, b1n, t1n, stream, true);
}

// The last identity block of a layer chained with the NEXT layer's first conv1 (1x1, C -> Pn = 2 P at this
// map size; the strided block's conv2 / dual GEMM follow as their own launches), split fp16 only (round 6):
// t1n [N, H, W, Pn] (logical), s1n / b1n [Pn]; wstream = packing.pack_tail_stream(conv2, conv3, next conv1
// pack [Pn][C']).  Pn = P is posu_bottleneck_tail_stream_next_fwd.
extern "C" int posu_bottleneck_tail_stream_chain_fwd(int dtype, const void* t1, const void* x, int N, int H, int W,
                                                     int C, int P, int Pn, const void* wstream,
                                                     long long wstream_bytes, const float* s2, const float* b2,
                                                     const float* s3, const float* b3, void* y, const float* s1n,
                                                     const float* b1n, void* t1n, void* stream) {
  if (!t1n || P <= 0 || (Pn != P && Pn != 2 * P)) {
    set_error("posu_bottleneck_tail_stream_chain_fwd: t1n must be given and Pn must be P or 2 P");
    return POSU_ERR_ARG;
  }
  return tail_stream_impl("posu_bottleneck_tail_stream_chain_fwd", dtype, t1, x, N, H, W, C, P, wstream, wstream_bytes,
                          s2, b2, s3, b3, y, s1n, b1n, t1n, stream, false, Pn / P);
}
