// Tail of the identity Bottleneck of layer3 (lib/models/pose_resnet.py:61-99, eval mode, BN
// folded) for PoseResNet at 256x256: t1 [N, H, 16, 256] (conv1's output, BN1 + ReLU applied,
// from the conv kernel), x [N, H, 16, 1024] the block input,
//
//     y = relu( bn3(conv3( relu(bn2(conv2_3x3(t1))) )) + x )
//
// in ONE launch: the 3x3's output tile never leaves the CU (the two separate convolutions
// wrote t2 to HBM and read it back, and each paid its own launch ramp and tail).
//
// One workgroup (8 waves, one per CU) owns 8 image rows x 16 px = 128 output pixels (two per
// image at H = 16: 256 workgroups at batch 128).  LDS:
//   * the t1 window of its rows -- rows y0-1 .. y0+8, columns -1 .. 16 (the 3x3's zero
//     padding, out-of-image rows / columns load as zeros) x 256 channels, staged ONCE (90 KB);
//   * a two-slot 32 KB ring through which ONE stream of stages flows:
//       stages 0-35   conv2, K-tile kt = tap * 4 + c: w2 [256 co][64 ci]   (tap-major K,
//                     exactly conv_igemm's K order: bit-identical accumulators)
//       stages 36-51  conv3, output chunk n (256 co), K-tile c: w3 [256 co][64 ci]
//   * t2 [128 px][256 ch] written over the window once conv2 is done.
// One barrier per stage (its DMA has landed, the other slot is free), the next stage's DMA
// issued right after it.  Waves: pm = w & 1 the pixel half (output rows 4 pm .. 4 pm + 3 =
// m-tiles i), cn = w >> 1 the 64-channel quarter of the 256 outputs (n-tiles j).  MFMA
// operands swapped (A = weights, B = pixels): lane (r16, q) accumulates channels 4q .. 4q+3 of
// pixel r16; v_permlane16_swap pairs n-tiles into 8 consecutive channels for 16-B stores.
// 512-B pixel rows (window, t2): 16-B chunk index XOR (pixel & 15); 128-B weight rows: swz().
#include "gemm_common.h"

// timing ablations (tools/tail3_ablations.sh; never set in the product build):
//   1: no MFMAs   2: no weight DMAs (stale slots)   3: no window DMA   4: no fragment LDS reads
//   5: no MFMAs and no weight DMAs   6: no epilogues (no t2 / y writes)
#ifndef POSU_TAIL3_ABLATE
#define POSU_TAIL3_ABLATE 0
#endif
// store-ordering experiments (tools/store_order.sh; never set in the product build):
//   RAWSTORE 1: y through a raw buffer store with the row offset in soffset
//   EARLYDMA 1: the next chunk's first weight DMA issued BEFORE the chunk's y stores, and
//               waited for with vmcnt(8) (the 8 stores younger than it left in flight)
#ifndef POSU_TAIL3_RAWSTORE
#define POSU_TAIL3_RAWSTORE 0
#endif
#ifndef POSU_TAIL3_EARLYDMA
#define POSU_TAIL3_EARLYDMA 0
#endif

namespace posu {
namespace {

struct Tail3Geom {
  const void* t1;
  const void* x;
  void* y;
  const void* w2;  // [256][2304]  k = (kh * 3 + kw) * 256 + ci
  const float* s2;
  const float* b2;
  const void* w3;  // [1024][256]
  const float* s3;
  const float* b3;
  int N, H;
};

constexpr int kW = 16, kP = 256, kC = 1024, kRows = 8, kPx = kRows * kW;
constexpr int kWinRows = kRows + 2, kWinCols = kW + 2, kWinPix = kWinRows * kWinCols;  // 180
constexpr int kSlotB = 32768;
constexpr int kWin = 0;                              // window: 180 px x 512 B = 92160 B
constexpr int kRing = kWinPix * 512;                 // two 32 KB slots
constexpr int kBN = kRing + 2 * kSlotB;              // s2 b2 (256 each) f32
constexpr int kLds = kBN + 2 * kP * 4;
constexpr int kS3 = kWin + kPx * 512;             // s3 b3 (1024 each) f32, over the window after conv2
static_assert(kS3 + 2 * kC * 4 <= kRing, "t2 and BN3 fit over the window");
static_assert(kLds <= 160 * 1024, "LDS");
constexpr int kConv2Stages = 36;

__device__ __forceinline__ void ld8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// 512-B row (256 bf16 channels) of pixel `pix`, 16-B chunk `chunk` (0..31)
__device__ __forceinline__ int swz32(int pix, int chunk) { return pix * 512 + ((chunk ^ (pix & 15)) << 4); }

template <typename T>
__global__ __launch_bounds__(512, 1) void bottleneck3_tail_kernel(Tail3Geom g) {
  using O = Op<T>;
  constexpr int ES = 2;
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int pm = wid & 1, cn = wid >> 1;
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));
  const int H = g.H;
  const int tiles_per_img = H / kRows;
  const int n = blockIdx.x / tiles_per_img;
  const int y0 = (blockIdx.x - n * tiles_per_img) * kRows;
  float* bn = reinterpret_cast<float*>(smem + kBN);
  if (tid < kP) {
    bn[tid] = g.s2[tid];
    bn[kP + tid] = g.b2[tid];
  }

  const u32x4 t1s = make_srd(g.t1, g.N * H * kW * kP * ES);
  const u32x4 w2s = make_srd(g.w2, kP * 9 * kP * ES);
  const u32x4 w3s = make_srd(g.w3, kC * kP * ES);

  // ---- the t1 window: 90 wave-instructions of 1 KB (2 pixels each), instruction m by wave m & 7
  {
    const int half = lane >> 5, pc = lane & 31;
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int m = wid + 8 * k;
      if (m < kWinPix / 2 && POSU_TAIL3_ABLATE != 3) {  // wave-uniform
        const int pix = 2 * m + half;
        const int wr = pix / kWinCols, wc = pix - wr * kWinCols;
        const int yy = y0 + wr - 1, xx = wc - 1;
        const int lc = pc ^ (pix & 15);
        const bool ok = static_cast<unsigned>(yy) < static_cast<unsigned>(H) && static_cast<unsigned>(xx) < kW;
        dma16(t1s, ok ? (((n * H + yy) * kW + xx) * kP + 8 * lc) * ES : kOOB,
              lds0 + kWin + static_cast<unsigned>(m) * 1024u);
      }
    }
  }
  // ---- weight stages: [256 rows][128 B], 4 DMAs per thread (rows tid >> 3 + 64 i)
  const int cL = (tid & 7) ^ ((tid >> 4) & 7);
  const int drow = tid >> 3;
  auto dma_stage = [&](int u, unsigned slot) {
    if (POSU_TAIL3_ABLATE == 2 || POSU_TAIL3_ABLATE == 5) return;
    const unsigned dst = lds0 + kRing + slot + wid_u * 1024;
    if (u < kConv2Stages) {  // w2 K-tile u: columns 64 u .. 64 u + 63 of [256][2304]
#pragma unroll
      for (int i = 0; i < 4; ++i) dma16(w2s, ((drow + 64 * i) * (9 * kP) + 64 * u + 8 * cL) * ES, dst + i * 8192);
    } else {  // w3 chunk nc = (u - 36) / 4, K-tile c = (u - 36) % 4
      const int v = u - kConv2Stages, nc = v >> 2, c = v & 3;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        dma16(w3s, ((256 * nc + drow + 64 * i) * kP + 64 * c + 8 * cL) * ES, dst + i * 8192);
    }
  };
  auto slot_of = [](int s) { return static_cast<unsigned>((s & 1) * kSlotB); };
  dma_stage(0, slot_of(0));

  f32x4 acc[4][4];  // [m-tile i: output row 4 pm + i][n-tile j: channels 64 cn + 16 j + 4 q ..]
  auto zero = [&] {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto pair = [&](int i, int jp, float* v) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][e]),
                                                       __float_as_uint(acc[i][2 * jp + 1][e]), false, false);
      v[e] = __uint_as_float(sw[0]);
      v[4 + e] = __uint_as_float(sw[1]);
    }
  };
  const int cpair = 16 * (q & 1) + 8 * (q >> 1);  // + 32 jp: a pair's channel offset

  // one 64-channel K-tile: A = weight rows 64 cn + 16 j + r16 of the slot, B = pixel rows
  // `bpix(i)` of the 512-B-row image at `img`, channel chunks 8 kc + 4 cb + q
  auto mma_ktile = [&](unsigned slot, const char* img, int kc, auto bpix) {
    const char* S = smem + kRing + slot;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      uint4 a[4], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a[j] = POSU_TAIL3_ABLATE == 4 ? make_uint4(lane, j, cb, kc)
                                      : *reinterpret_cast<const uint4*>(S + swz(64 * cn + 16 * j + r16, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 4; ++i)
        b[i] = POSU_TAIL3_ABLATE == 4 ? make_uint4(i, lane, kc, cb)
                                      : *reinterpret_cast<const uint4*>(img + swz32(bpix(i), 8 * kc + 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (POSU_TAIL3_ABLATE == 1 || POSU_TAIL3_ABLATE == 5) acc[i][j][0] += __uint_as_float(a[j].x ^ b[i].y);
          else O::mma(acc[i][j], a[j], b[i]);
        }
    }
  };

  // x through a buffer descriptor: a wave-uniform row offset + one lane offset (no 64-bit
  // addresses live across the loop)
  const __amdgpu_buffer_rsrc_t xrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(g.x), 0, g.N * H * kW * kC * ES, 0x00020000);
  // y: plain global stores at a 32-bit offset from this workgroup's first output row (a raw
  // buffer store with the row in soffset corrupted a few elements per launch; not understood)
  char* const ywg = static_cast<char*>(g.y) + static_cast<size_t>(n * H + y0) * kW * kC * ES;
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(g.y, 0, g.N * H * kW * kC * ES, 0x00020000);
  const int lane_off = (r16 * kC + cpair) * ES;
  // byte offset of (output row 4 pm + i, column 0, channel 256 nc + 64 cn + 32 jp), wave-uniform
  auto row_off = [&](int i, int nc, int jp) {
    return __builtin_amdgcn_readfirstlane(((n * H + y0 + 4 * pm + i) * kW * kC + 256 * nc + 64 * cn + 32 * jp) * ES);
  };
  uint4 rv[4][2];
  auto res_load = [&](int nc) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(xrs, lane_off, row_off(i, nc, jp), 0);
        rv[i][jp] = make_uint4(v[0], v[1], v[2], v[3]);
      }
  };

  vm_wait<0>();  // window + stage 0
  // ---- conv2: stages 0 .. 35 (tap-major K-tiles over the window)
#pragma unroll 1
  for (int u = 0; u < kConv2Stages; ++u) {
    vm_wait<0>();
    lds_barrier();
    dma_stage(u + 1, slot_of(u + 1));
    if (u == 0) zero();
    const int tap = u >> 2, kc = u & 3, dy = tap / 3, dx = tap - 3 * (tap / 3);
    mma_ktile(slot_of(u), smem + kWin, kc, [&](int i) { return (4 * pm + i + dy) * kWinCols + r16 + dx; });
  }
  // BN2 + ReLU -> t2 over the window (every wave is done reading it first), BN3 parameters
  // beside it
  lds_barrier();
  if (POSU_TAIL3_ABLATE != 6) {
    float* b3l = reinterpret_cast<float*>(smem + kS3);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      b3l[2 * tid + e] = g.s3[2 * tid + e];
      b3l[kC + 2 * tid + e] = g.b3[2 * tid + e];
    }
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int c0 = 64 * cn + 32 * jp + cpair;
      float sc[8], sh[8];
      ld8(bn + c0, sc);
      ld8(bn + kP + c0, sh);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v[8];
        pair(i, jp, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e], 0.f);
        *reinterpret_cast<uint4*>(smem + kWin + swz32(16 * (4 * pm + i) + r16, c0 >> 3)) = O::store_vals(v);
      }
    }
  }
  // ---- conv3: output chunk nc (256 channels), K-tiles kc = 0 .. 3 of t2; stage u = 36 + 4 nc + kc
#pragma unroll 1
  for (int nc = 0; nc < 4; ++nc) {
#pragma unroll 1
    for (int kc = 0; kc < 4; ++kc) {
      const int u = kConv2Stages + 4 * nc + kc;
      // the chunk's residual loads (issued at kc == 1, after that stage's DMA) are the 8
      // youngest vector-memory ops at kc == 2: its DMA is waited for without them
      if (kc == 2 || (POSU_TAIL3_EARLYDMA && kc == 0 && nc > 0)) vm_wait<8>();
      else vm_wait<0>();
      lds_barrier();
      if (kc == 0) zero();
      // the last stage of a chunk issues the next stage's DMA after its y stores: the next
      // stage's wait then covers both together instead of stalling a later stage behind them
      if (kc != 3 || (POSU_TAIL3_EARLYDMA && nc < 3)) dma_stage(u + 1, slot_of(u + 1));
      if (kc == 1) res_load(nc);  // two stages ahead of the epilogue
      mma_ktile(slot_of(u), smem + kWin, kc, [&](int i) { return 16 * (4 * pm + i) + r16; });
    }
    if (POSU_TAIL3_ABLATE != 6) {  // BN3 + residual + ReLU -> y
      // pixel-major: the two 16-B stores of a pixel's two pairs (one 128-B line of y with the
      // other q-lanes) are issued back to back, so L2 sees whole lines
      float sc[2][8], sh[2][8];
      const float* b3l = reinterpret_cast<const float*>(smem + kS3);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        ld8(b3l + 256 * nc + 64 * cn + 32 * jp + cpair, sc[jp]);
        ld8(b3l + kC + 256 * nc + 64 * cn + 32 * jp + cpair, sh[jp]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int c0 = 256 * nc + 64 * cn + 32 * jp + cpair;
          float vv[8], r[8];
          pair(i, jp, vv);
          O::load_vals(rv[i][jp], r);
#pragma unroll
          for (int e = 0; e < 8; ++e) vv[e] = fmaxf(vv[e] * sc[jp][e] + sh[jp][e] + r[e], 0.f);
          if (POSU_TAIL3_RAWSTORE) {
            const uint4 o = O::store_vals(vv);
            __builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned){o.x, o.y, o.z, o.w},
                                                   yrs, lane_off, row_off(i, nc, jp), 0);
          } else {
            *reinterpret_cast<uint4*>(ywg + ((16 * (4 * pm + i) + r16) * kC + c0) * ES) = O::store_vals(vv);
          }
        }
    }
    if (!POSU_TAIL3_EARLYDMA && nc < 3) dma_stage(kConv2Stages + 4 * nc + 4, slot_of(kConv2Stages + 4 * nc + 4));
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_bottleneck3_tail_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C, int P,
                                         const void* w2, const float* s2, const float* b2, const void* w3,
                                         const float* s3, const float* b3, void* y, void* stream) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, "posu_bottleneck3_tail_fwd: dtype must be BF16 or F16");
  POSU_REQUIRE(t1 && x && w2 && s2 && b2 && w3 && s3 && b3 && y, "posu_bottleneck3_tail_fwd: null pointer");
  POSU_REQUIRE(x != y && t1 != y, "posu_bottleneck3_tail_fwd: the output must not alias an input");
  POSU_REQUIRE(W == kW && C == kC && P == kP,
               "posu_bottleneck3_tail_fwd: built for W = 16, C = 1024, planes = 256 (layer3 of PoseResNet at 256x256)");
  POSU_REQUIRE(N > 0 && H > 0 && H % kRows == 0, "posu_bottleneck3_tail_fwd: H must be a positive multiple of 8");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * 2 < (1LL << 31) - 256,
               "posu_bottleneck3_tail_fwd: activation exceeds the 2 GiB addressing range");
  for (const void* p : {t1, x, static_cast<const void*>(y), w2, w3, static_cast<const void*>(s3),
                        static_cast<const void*>(b3)})
    POSU_REQUIRE((reinterpret_cast<size_t>(p) & 15) == 0, "posu_bottleneck3_tail_fwd: pointers must be 16-byte aligned");
  Tail3Geom g{};
  g.t1 = t1;
  g.x = x;
  g.y = y;
  g.w2 = w2;
  g.s2 = s2;
  g.b2 = b2;
  g.w3 = w3;
  g.s3 = s3;
  g.b3 = b3;
  g.N = N;
  g.H = H;
  const dim3 grid(static_cast<unsigned>(N * (H / kRows)));
  hipStream_t s = as_stream(stream);
  if (dtype == POSU_BF16)
    hipLaunchKernelGGL(bottleneck3_tail_kernel<uint16_t>, grid, dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL(bottleneck3_tail_kernel<f16_t>, grid, dim3(512), 0, s, g);
  return check_launch("posu_bottleneck3_tail_fwd");
}
