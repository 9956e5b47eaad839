// Fused Bottleneck block (lib/models/pose_resnet.py:61-99, eval mode, BN folded):
//
//     y = relu( bn3(conv3( relu(bn2(conv2_3x3( relu(bn1(conv1(x))) ))) )) + x )
//
// for the identity-residual blocks of layer1 (x [N, H, 64, 256], planes 64) in ONE
// launch that reads x from HBM exactly once and writes y once: per block 2 x 268 MB at
// batch 128, against 1.07 GB for three separate convolutions (whose two 64-channel
// intermediates and the residual re-read make up the rest).
//
// Streaming structure.  One workgroup (8 waves = 2 per SIMD, 1 per CU: 155 KiB of LDS) walks
// down a strip of output rows of one image, one row (64 pixels) per step.  Waves w and w+4
// are a pair on pixels 16 (w & 3) .. +15; h = w >> 2 picks the channel half a wave owns:
//   conv1    t1 row y+1 = relu(bn1(x row y+1 . w1)), split over K: wave h multiplies its
//            128 input channels (x fragments straight from HBM into VGPRs, prefetched two
//            rows ahead; its half of w1 held in VGPRs for the whole strip) into all 64
//            outputs, hands the partner's two n-tiles over in LDS (f32) and finishes its
//            own two (sum of the halves in the order half 0 + half 1, BN1, ReLU) into a
//            3-row LDS ring [row][66 px][64 ch] (rows outside the image are zeros =
//            conv2's padding), so every conv1 row is computed once.
//   conv2    3x3 over ring rows y-1, y, y+1 (x-padding = two zero columns of the ring), output n-tiles
//            2h, 2h+1, w2 [9][64][64] resident in LDS; BN2 + ReLU stay in registers,
//            rounded: the two n-tiles ARE conv3's B fragment of k-step h (lane (p, q) holds
//            channels 4q..4q+3 of each, a permuted channel order in which conv3's weights are
//            packed).  The pair swaps these fragments through LDS (1 KiB per wave).
//   conv3    output channels 128 h .. +127, w3 [256][64] resident in LDS; BN3 + residual +
//            ReLU.  The residual is x row y in the registers conv1 consumed one step
//            earlier: conv1's K order is permuted so that lane q's x fragment of k-step s is
//            exactly the 8 channels its conv3 epilogue adds for output pair s, and the K half
//            of conv1 is the channel half of conv3.  The row's 16-B NHWC stores are issued
//            during the NEXT row's step, spread over its phases (see flush()).
// Per row and wave: 16 + 36 + 16 MFMAs against 64 KB of HBM traffic per CU.  An image is
// split into S strips (S * N ~ the CU count); a strip recomputes the one conv1 row above it.
// Measured (tools/bottleneck_micro.py, 128 x 64 x 64 x 256 bf16): 148 us against 300 us for
// the three unfused launches and 102 us for a plain 268 MB copy; without any HBM traffic
// (timing ablations, POSU_BNECK_ABLATE) the loop itself takes 116 us -- VALU-heavy
// epilogues (BN, ReLU, residual, packing) and three barriers per row.
//
// K order: conv2 sums its K in the unfused kernel's order (tap-major, channel-minor);
// conv1 and conv3 sum their channels in permuted orders (f32 rounding differences only).
#include "gemm_common.h"

namespace posu {
namespace {

struct BottleGeom {
  const void* x;
  void* y;
  const void* w1;  // [64][256], K permuted (bottleneck_conv1_order)
  const float* s1;
  const float* b1;
  const void* w2;  // [64][576], k = (kh * 3 + kw) * 64 + ci
  const float* s2;
  const float* b2;
  const void* w3;  // [256][64], K permuted (bottleneck_conv3_order); DOWN: [256][128] =
                   // [w3 * s3 permuted | wd * sd], the dual tail's folded weights
  const float* s3;  // DOWN: unused
  const float* b3;  // DOWN: b3 + bd
  int N, H;
  int strips;      // strips per image
  int rows;        // rows per strip (H / strips)
};

// timing ablations for tools/bottleneck_micro.py only (wrong results when non-zero): 1 no conv2
// MFMAs, 2 no conv3 MFMAs, 4 no output stores, 8 no barriers, 16 no conv1 MFMAs, 32 no x loads;
// 64 / 128: non-temporal stores / loads (correct results)
#ifndef POSU_BNECK_ABLATE
#define POSU_BNECK_ABLATE 0
#endif
constexpr int kAbl = POSU_BNECK_ABLATE;


constexpr int kP = 64, kW = 64, kC = 256;
constexpr int kW2 = 0;                  // w2: 9 taps x [64 co][128 B]                73728 B
constexpr int kW3 = 73728;              // w3: [256 co][128 B]                         32768 B
constexpr int kT1 = 106496;             // t1 ring: 3 x [66 px][128 B] (px -1, 64 zero)  25344 B
constexpr int kSlot = 66 * 128;
constexpr int kBN = kT1 + 3 * kSlot;    // s1 b1 s2 b2 (64 each), s3 b3 (256 each) f32   3072 B
constexpr int kXP = kBN + 3072;         // conv1 partial sums: 8 waves x [64 lanes][8 f32] 16384 B
constexpr int kXT = kXP + 16384;        // t2 exchange: 8 waves x [64 lanes][16 B]       8192 B
constexpr int kLds = kXT + 8192;        // 159488
static_assert(kLds <= 160 * 1024, "LDS");

__device__ __forceinline__ void raw_barrier() {
  if (kAbl & 8) return;
  lds_barrier();
}

__device__ __forceinline__ void ld8(const float* p, float* v) {  // 8 f32 from LDS
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// DOWN: the first block of layer1 (x [N, H, 64, 64], a downsample branch instead of the
// identity): conv1 split over N (K = 64, no partial hand-off), the downsample's MFMAs from the
// x fragments of row y join conv3's accumulators, weights [w3*s3 | wd*sd] (wd in VGPRs).
template <typename T, bool DOWN>
__global__ __launch_bounds__(512, 1) void bottleneck64_kernel(BottleGeom g) {
  using O = Op<T>;
  constexpr int ES = static_cast<int>(sizeof(T));
  static_assert(ES == 2, "bf16 / f16 activations");
  constexpr int kCi = DOWN ? 64 : kC;        // block input channels
  constexpr int NF = DOWN ? 2 : 4;           // x fragments per lane and row
  constexpr int kW3K = DOWN ? 2 * kP : kP;   // row length of the packed conv3 weight
  __shared__ __attribute__((aligned(16))) char smem[kLds];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int pg = wid & 3, h = wid >> 2;            // pixel group, channel half
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));

  const int n = blockIdx.x / g.strips;
  const int ya = (blockIdx.x - n * g.strips) * g.rows, yb = ya + g.rows;
  const int H = g.H;
  const int px = 16 * pg + r16;                    // this lane's pixel column
  // channel offset of lane q in a 32-channel k-step of conv1 (and of the conv3 epilogue)
  const int cq = 16 * (q & 1) + 8 * (q >> 1);
  const float* bn = reinterpret_cast<const float*>(smem + kBN);
  // this wave's / the partner wave's (same pixels, other half) exchange slots
  float* xp_mine = reinterpret_cast<float*>(smem + kXP + (2 * pg + h) * 2048 + lane * 32);
  const float* xp_part = reinterpret_cast<const float*>(smem + kXP + (2 * pg + 1 - h) * 2048 + lane * 32);
  uint4* xt_mine = reinterpret_cast<uint4*>(smem + kXT + (2 * pg + h) * 1024 + lane * 16);
  const uint4* xt_part = reinterpret_cast<const uint4*>(smem + kXT + (2 * pg + 1 - h) * 1024 + lane * 16);

  // ---- prologue: w2 / w3 -> LDS (LDS-DMA, swizzled rows), BN params -> LDS, w1 -> VGPRs
  {
    const u32x4 w2s = make_srd(g.w2, kP * 9 * kP * ES);
    const u32x4 w3s = make_srd(g.w3, kC * kW3K * ES);
    const int cL = (tid & 7) ^ ((tid >> 4) & 7), drow = tid >> 3;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      dma16(w2s, (drow * (9 * kP) + t * kP + cL * 8) * ES, lds0 + kW2 + t * 8192 + wid_u * 1024);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dma16(w3s, ((drow + 64 * i) * kW3K + cL * 8) * ES, lds0 + kW3 + i * 8192 + wid_u * 1024);
    float* bw = reinterpret_cast<float*>(smem + kBN);
    if (tid < 64) {
      bw[tid] = g.s1[tid];
      bw[64 + tid] = g.b1[tid];
      bw[128 + tid] = g.s2[tid];
      bw[192 + tid] = g.b2[tid];
    }
    if (tid < 256) {
      bw[256 + tid] = DOWN ? 1.f : g.s3[tid];
      bw[512 + tid] = g.b3[tid];
    }
    // conv2's x-padding: ring columns px = -1 and px = 64 (rows 0 and 65 of each slot) stay zero
    if (tid < 48) {
      const int sl = tid >> 4, side = (tid >> 3) & 1, ch = tid & 7;
      *reinterpret_cast<uint4*>(smem + kT1 + sl * kSlot + side * 65 * 128 + ch * 16) = make_uint4(0, 0, 0, 0);
    }
  }
  // [k-step 4h + s][jj]: n-tile (jj + 2h) & 3 -- this wave's own two n-tiles first, then the
  // partner's -- rows 16 j + r16, permuted K columns 32 s + 8 q .. + 7
  // DOWN: [k-step s][jj] = n-tile 2h + jj over the whole K = 64 (natural channel order)
  uint4 w1f[4][4];
  {
    const T* w1 = reinterpret_cast<const T*>(g.w1);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if constexpr (DOWN) {
          if (s < 2 && j < 2) w1f[s][j] = *reinterpret_cast<const uint4*>(w1 + (16 * (2 * h + j) + r16) * kCi + 32 * s + 8 * q);
        } else {
          w1f[s][j] = *reinterpret_cast<const uint4*>(w1 + (16 * ((j + 2 * h) & 3) + r16) * kC + 32 * (4 * h + s) + 8 * q);
        }
      }
  }
  // DOWN: the downsample's weights wd * sd, rows 128 h + 64 qh + 16 j + r16 (this wave's
  // output channels), natural K columns 64 + 32 s + 8 q .. + 7 of the packed [256][128]
  uint4 wdf[2][2][4];
  if constexpr (DOWN) {
    const T* w3 = reinterpret_cast<const T*>(g.w3);
#pragma unroll
    for (int qh = 0; qh < 2; ++qh)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          wdf[qh][s][j] = *reinterpret_cast<const uint4*>(w3 + (128 * h + 64 * qh + 16 * j + r16) * kW3K + kP + 32 * s + 8 * q);
  }

  // x row r -> this lane's 4 fragments of this wave's channel half (k-steps 4h .. 4h+3).
  // Always 4 loads: rows outside [0, min(yb, H-1)] re-read a row of the strip instead (an L2
  // hit; the values are not used).  A load under a branch would make the compiler's vmcnt
  // bookkeeping assume the shorter path at the join and wait for the prefetch it just issued.
  // x / y through buffer descriptors: the row offset is wave-uniform (soffset, an SGPR) and
  // the lane's offset a loop constant, so the loop holds no 64-bit addresses in VGPRs
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(g.x), 0, g.N * H * kW * kCi * ES, 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(g.y, 0, g.N * H * kW * kC * ES, 0x00020000);
  const int lane_off = (px * kC + 128 * h + cq) * ES;   // y (and identity x): + 64 B per k-step
  const int lane_offx = DOWN ? (px * kCi + 8 * q) * ES : lane_off;
  constexpr int kRowBytes = kW * kC * ES, kRowBytesX = kW * kCi * ES;
  const int rmax = (yb < H - 1 ? yb : H - 1);
  auto load_row = [&](int r, uint4(&f)[4]) {
    const int rr = r < 0 ? 0 : (r > rmax ? rmax : r);
    const int roff = __builtin_amdgcn_readfirstlane((n * H + rr) * kRowBytesX);
    if (kAbl & 32) {
#pragma unroll
      for (int s = 0; s < NF; ++s) f[s] = make_uint4(rr, s, lane, 1);
      return;
    }
#pragma unroll
    for (int s = 0; s < NF; ++s) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(xrs, lane_offx + 64 * s, roff, (kAbl & 128) ? 2 : 0);
      f[s] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  // conv1 of x row r over this wave's channel half, all 64 outputs; the partner's two n-tiles
  // go to the exchange slot, this wave's two stay in acc
  // (DOWN: this wave's two n-tiles over the whole K, nothing handed over)
  auto conv1_part = [&](int r, const uint4(&f)[4], f32x4(&acc)[2]) {
    f32x4 a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (DOWN) {
      if (r >= 0 && r < H) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j) O::mma(a[j], w1f[s][j], f[s]);
      }
      acc[0] = a[0];
      acc[1] = a[1];
      return;
    }
    if (r >= 0 && r < H) {
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (kAbl & 16) a[j][0] += __uint_as_float(f[s].x ^ w1f[s][j].y);
          else O::mma(a[j], w1f[s][j], f[s]);
        }
    }
    *reinterpret_cast<f32x4*>(xp_mine) = a[2];
    *reinterpret_cast<f32x4*>(xp_mine + 4) = a[3];
    acc[0] = a[0];
    acc[1] = a[1];
  };
  // full sums of n-tiles 2h, 2h+1 (half 0 + half 1), BN1 + ReLU into ring slot r % 3
  // (zeros outside the image)
  auto conv1_fin = [&](int r, const f32x4(&acc)[2]) {
    char* slot = smem + kT1 + ((r + 3) % 3) * kSlot;
    const bool ok = r >= 0 && r < H;
    f32x4 t0 = acc[0], t1 = acc[1];
    if constexpr (!DOWN) {
      const f32x4 pa = *reinterpret_cast<const f32x4*>(xp_part);
      const f32x4 pb = *reinterpret_cast<const f32x4*>(xp_part + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // half 0 + half 1 (f32 addition commutes exactly)
        t0[e] += pa[e];
        t1[e] += pb[e];
      }
    }
    const int c0 = 16 * (2 * h + (q & 1)) + 8 * (q >> 1);
    float v[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(t0[e]), __float_as_uint(t1[e]), false, false);
      v[e] = __uint_as_float(sw[0]);
      v[4 + e] = __uint_as_float(sw[1]);
    }
    ld8(bn + c0, sc);
    ld8(bn + 64 + c0, sh);
    affine8<!DOWN>(v, sc, sh);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = ok ? fmaxf(v[e], 0.f) : 0.f;
    *reinterpret_cast<uint4*>(slot + swz(px + 1, c0 >> 3)) = O::store_vals(v);
  };
  // conv2 of output row y, n-tiles 2h, 2h+1, over ring rows y-1..y+1; BN2 + ReLU, rounded:
  // conv3's B fragment of k-step h (channels 32 h + 4 q .. +3 and 32 h + 16 + 4 q .. +3)
  auto conv2_row = [&](int y, auto&& mid) -> uint4 {
    f32x4 acc2[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t == 5) mid();
      const int dy = t / 3, dx = t % 3;
      const char* slot = smem + kT1 + ((y - 1 + dy + 3) % 3) * kSlot;
      const char* Wt = smem + kW2 + t * 8192;
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        uint4 wf[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) wf[j] = *reinterpret_cast<const uint4*>(Wt + swz(16 * (2 * h + j) + r16, 4 * cb + q));
        // ring column px + dx = input pixel px + dx - 1 (columns 0 and 65 are the zero padding)
        const uint4 tf = *reinterpret_cast<const uint4*>(slot + swz(px + dx, 4 * cb + q));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if (kAbl & 1) acc2[j][0] += __uint_as_float(wf[j].x ^ tf.y);
          else O::mma(acc2[j], wf[j], tf);
        }
      }
    }
    const int ca = 32 * h + 4 * q, cb2 = ca + 16;
    const float4 sa = *reinterpret_cast<const float4*>(bn + 128 + ca);
    const float4 sb = *reinterpret_cast<const float4*>(bn + 128 + cb2);
    const float4 ha = *reinterpret_cast<const float4*>(bn + 192 + ca);
    const float4 hb = *reinterpret_cast<const float4*>(bn + 192 + cb2);
    const float s8[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
    const float h8[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    float v[8] = {acc2[0][0], acc2[0][1], acc2[0][2], acc2[0][3], acc2[1][0], acc2[1][1], acc2[1][2], acc2[1][3]};
    affine8<!DOWN>(v, s8, h8);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    return O::store_vals(v);
  };
  // conv3 of output row y, channels 128 h .. 128 h + 127, + BN3 + residual (this wave's half
  // of x row y) + ReLU, 16-B NHWC stores
  // The output row is stored during the NEXT row's step (flush(k), spread over its phases):
  // the stores of all 8 waves at the end of conv3 form a 32 KB burst per CU that stalls the
  // waves behind the CU's store queue.
  uint4 pend[4];
  int pend_off = 0;  // byte offset of the pending output row (wave-uniform)
  auto flush = [&](int k) {
    const uint4 u = pend[k];
    if (kAbl & 4) {
      asm volatile("" ::"v"(u.x), "v"(u.y), "v"(u.z), "v"(u.w));
      return;
    }
    // the row offset goes into the VGPR offset, soffset stays the constant 0: hipcc inserts the
    // wait states of the store-data hazard (a VALU write of the data VGPRs right after a > 64-bit
    // store) only for buffer stores WITHOUT an SGPR soffset, and on gfx950 a store with one
    // stored corrupted values (tools/isa_hazards.py)
    __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned){u.x, u.y, u.z, u.w}, yrs,
                                           lane_off + 64 * k + pend_off, 0, (kAbl & 64) ? 2 : 0);
  };
  auto conv3_row = [&](int y, const uint4(&tb)[2], const uint4(&res)[4]) {
    pend_off = __builtin_amdgcn_readfirstlane((n * H + y) * kRowBytes);
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int qd = 2 * h + qh;
      f32x4 acc3[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc3[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4 wf = *reinterpret_cast<const uint4*>(smem + kW3 + swz(64 * qd + 16 * j + r16, 4 * kb + q));
          if (kAbl & 2) acc3[j][0] += __uint_as_float(wf.x ^ tb[kb].y);
          else O::mma(acc3[j], wf, tb[kb]);
        }
      }
      if constexpr (DOWN) {  // + the downsample of x row y (res = its fragments)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 4; ++j) O::mma(acc3[j], wdf[qh][s][j], res[s]);
      }
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const int s = 2 * qd + jp, c0 = 32 * s + cq;
        float v[8], r[8], sc[8], sh[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc3[2 * jp][e]),
                                                           __float_as_uint(acc3[2 * jp + 1][e]), false, false);
          v[e] = __uint_as_float(sw[0]);
          v[4 + e] = __uint_as_float(sw[1]);
        }
        ld8(bn + 512 + c0, sh);
        if constexpr (DOWN) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] + sh[e], 0.f);
        } else {
          ld8(bn + 256 + c0, sc);
          O::load_vals(res[2 * qh + jp], r);
          affine8<!DOWN>(v, sc, sh);
          add8<!DOWN>(v, r);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        // channels c0 .. c0 + 7 = 128 h + 32 (2 qh + jp) + cq, packed HERE (the empty asm
        // keeps the compiler from sinking the packing, and 8 live f32 per value, into the
        // next row's step where the value is stored: 98 spilled VGPRs without it)
        uint4& pk = pend[2 * qh + jp];
        pk = O::store_vals(v);
        asm("" : "+v"(pk.x), "+v"(pk.y), "+v"(pk.z), "+v"(pk.w));
      }
    }
  };

  // x rows in flight: A = row y (residual of the current output row), B = row y+1 (its
  // conv1 now), C = row y+2, D = row y+3 (prefetched two rows ahead); the roles rotate
  // A<-B<-C<-D each row
  uint4 xa[4], xb[4], xc[4], xd[4];
  f32x4 c1[2];
  load_row(ya - 1, xd);   // the conv1 row above the strip (recomputed; zeros at the top)
  load_row(ya, xa);
  vm_wait<0>();           // w2 / w3 DMAs, w1, BN staging loads, rows ya-1 and ya
  raw_barrier();          // BN params in LDS visible (the DMA'd weights too)
  load_row(ya + 1, xb);
  load_row(ya + 2, xc);
  conv1_part(ya - 1, xd, c1);
  if (!DOWN) raw_barrier();
  conv1_fin(ya - 1, c1);
  if (!DOWN) raw_barrier();  // partial slots free again
  conv1_part(ya, xa, c1);
  if (!DOWN) raw_barrier();
  conv1_fin(ya, c1);

  // one output row, three barriers: (a) conv1 partials of row y+1 exchanged, (b) ring rows
  // y-1..y+1 complete, (c) conv2 halves exchanged.  The ring slot written after (a) held row
  // y-2, whose last reader (conv2 of row y-1) every wave finished before (a); the exchange
  // slots are rewritten only after the next barrier that follows their reads
  auto step = [&](int y, const uint4(&ra)[4], const uint4(&rb)[4], uint4(&rd)[4], bool fl) {
    conv1_part(y + 1, rb, c1);
    load_row(y + 3, rd);
    if (fl) flush(0);
    if (!DOWN) raw_barrier();  // (DOWN: no partials; barrier (c) of the last step freed the slot)
    conv1_fin(y + 1, c1);
    if (fl) flush(1);
    raw_barrier();
    const uint4 mine = conv2_row(y, [&] { if (fl) flush(2); });
    if (fl) flush(3);
    *xt_mine = mine;
    raw_barrier();
    const uint4 part = *xt_part;
    const uint4 tb[2] = {h ? part : mine, h ? mine : part};
    conv3_row(y, tb, ra);
  };
  // first row (nothing pending), then a branch-free body over whole groups of 4 rows (the
  // same vmcnt reason as load_row), then the tail, then the last row's stores
  step(ya, xa, xb, xd, false);
  int y = ya + 1;
  for (; y + 4 <= yb; y += 4) {
    step(y, xb, xc, xa, true);
    step(y + 1, xc, xd, xb, true);
    step(y + 2, xd, xa, xc, true);
    step(y + 3, xa, xb, xd, true);
  }
  if (y < yb) {
    step(y, xb, xc, xa, true);
    if (y + 1 < yb) step(y + 1, xc, xd, xb, true);
    if (y + 2 < yb) step(y + 2, xd, xa, xc, true);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) flush(k);
}

}  // namespace
}  // namespace posu

using namespace posu;

namespace {
int bottleneck_launch(bool down, int dtype, const void* x, int N, int H, int W, int C, int P, const void* w1,
                      const float* s1, const float* b1, const void* w2, const float* s2, const float* b2,
                      const void* w3, const float* s3, const float* b3, void* y, void* stream, const char* what) {
  const std::string wh(what);
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, wh + ": dtype must be BF16 or F16");
  POSU_REQUIRE(x && w1 && s1 && b1 && w2 && s2 && b2 && w3 && (s3 || down) && b3 && y, wh + ": null pointer");
  POSU_REQUIRE(x != y, wh + ": the output must not alias the input");
  POSU_REQUIRE(W == kW && C == (down ? 64 : kC) && P == kP,
               wh + (down ? ": built for W = 64, C = 64, planes = 64 (layer1 block 0 of PoseResNet at 256x256)"
                          : ": built for W = 64, C = 256, planes = 64 (layer1 of PoseResNet at 256x256)"));
  POSU_REQUIRE(N > 0 && H > 0, wh + ": empty input");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * kC * 2 < (1LL << 31) - 256,
               wh + ": activation exceeds the 2 GiB addressing range");
  for (const void* p : {x, static_cast<const void*>(y), w1, w2, w3})
    POSU_REQUIRE((reinterpret_cast<size_t>(p) & 15) == 0, wh + ": pointers must be 16-byte aligned");
  BottleGeom g{};
  g.x = x;
  g.y = y;
  g.w1 = w1;
  g.s1 = s1;
  g.b1 = b1;
  g.w2 = w2;
  g.s2 = s2;
  g.b2 = b2;
  g.w3 = w3;
  g.s3 = s3;
  g.b3 = b3;
  g.N = N;
  g.H = H;
  // strips per image: about one workgroup per CU, whole rows per strip
  int strips = 1;
  while (N * strips * 2 <= 256 && H % (strips * 2) == 0 && H / (strips * 2) >= 2) strips *= 2;
  g.strips = strips;
  g.rows = H / strips;
  hipStream_t s = as_stream(stream);
  const dim3 grid(N * strips), block(512);
  if (dtype == POSU_BF16) {
    if (down) hipLaunchKernelGGL((bottleneck64_kernel<uint16_t, true>), grid, block, 0, s, g);
    else hipLaunchKernelGGL((bottleneck64_kernel<uint16_t, false>), grid, block, 0, s, g);
  } else {
    if (down) hipLaunchKernelGGL((bottleneck64_kernel<f16_t, true>), grid, block, 0, s, g);
    else hipLaunchKernelGGL((bottleneck64_kernel<f16_t, false>), grid, block, 0, s, g);
  }
  return check_launch(what);
}
}  // namespace

extern "C" int posu_bottleneck_fwd(int dtype, const void* x, int N, int H, int W, int C, int P, const void* w1,
                                   const float* s1, const float* b1, const void* w2, const float* s2, const float* b2,
                                   const void* w3, const float* s3, const float* b3, void* y, void* stream) {
  return bottleneck_launch(false, dtype, x, N, H, W, C, P, w1, s1, b1, w2, s2, b2, w3, s3, b3, y, stream,
                           "posu_bottleneck_fwd");
}

extern "C" int posu_bottleneck_down_fwd(int dtype, const void* x, int N, int H, int W, int C, int P,
                                        const void* w1, const float* s1, const float* b1, const void* w2,
                                        const float* s2, const float* b2, const void* w3d, const float* shift3,
                                        void* y, void* stream) {
  return bottleneck_launch(true, dtype, x, N, H, W, C, P, w1, s1, b1, w2, s2, b2, w3d, nullptr, shift3, y, stream,
                           "posu_bottleneck_down_fwd");
}
