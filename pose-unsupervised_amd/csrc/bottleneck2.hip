// Fused identity Bottleneck of layer2 (lib/models/pose_resnet.py:61-99, eval mode, BN
// folded) for PoseResNet at 256x256: x [N, H, 32, 512], planes 128,
//
//     y = relu( bn3(conv3( relu(bn2(conv2_3x3( relu(bn1(conv1(x))) ))) )) + x )
//
// in ONE launch that reads x from HBM once (conv1 input; the residual re-read hits L2 /
// the Infinity Cache) and writes y once: 2 x 134 MB per block at batch 128 against 538 MB
// for the three separate convolutions.
//
// Unlike layer1's kernel (csrc/bottleneck.hip) the weights (w1 128 KB, w2 288 KB, w3 128 KB)
// do not fit in LDS, so they are STREAMED: a workgroup (8 waves, one per CU) walks down a
// strip of one image four rows (128 pixels) per step, and every step runs one continuous
// LDS-DMA stage stream through a two-slot 32 KB ring:
//   stages 0-7    conv1, K-chunk c: [x 128 px x 64 ch | w1 128 x 64]  -> t1 rows 4k+1..4k+4
//   stages 8-16   conv2, tap t:     [w2 tap 128 x 128]                -> t2 rows 4k..4k+3
//   stages 17-20  conv3, chunk c:   [w3 rows 128c.. 128 x 128]        -> y rows 4k..4k+3
// One barrier per stage (the stage's DMA has landed, the other slot is free), the next
// stage's DMA issued right after it.  t1 lives in a 6-row LDS ring [34 px][128 ch] whose
// edge columns are the 3x3's zero padding (every t1 row is computed once: the ring keeps
// rows 4k-1, 4k from the previous step); t2 in a [128 px][128 ch] LDS tile.  Waves: pg =
// w & 3 is the image row of the step, h = w >> 2 the 64-channel half of conv1/conv2's
// outputs (and of each conv3 chunk's 128).  MFMA operands swapped (A = weights, B = pixels):
// lane (r16, q) accumulates channels 4q..4q+3 of pixel r16; v_permlane16_swap pairs n-tiles
// into 8 consecutive channels for 16-B LDS / HBM stores.
//
// Per step: 8 + 9 + 4 stages = 672 KB of L2 -> LDS traffic for 71 MFLOP; the same K order
// per accumulator as the unfused convolutions (conv1: 64-channel chunks, conv2: tap-major,
// conv3: 128 channels) -- bit-identical t1 / t2 / y up to the BN of conv3 and residual,
// which are applied in the same f32 arithmetic.
#include "gemm_common.h"

namespace posu {
namespace {

struct Bottle2Geom {
  const void* x;
  void* y;
  const void* w1;  // [128][512]   (posu_conv2d_fwd packing, k = ci)
  const float* s1;
  const float* b1;
  const void* w2;  // [128][1152]  k = (kh * 3 + kw) * 128 + ci
  const float* s2;
  const float* b2;
  const void* w3;  // [512][128]
  const float* s3;
  const float* b3;
  int N, H;
  int strips, rows;  // strips per image, rows per strip (a multiple of 4)
};

constexpr int kW = 32, kC = 512, kP = 128, kR = 4;
constexpr int kSlotB = 32768;
constexpr int kT1 = 2 * kSlotB;              // t1 ring: 6 rows x [34 px][256 B]     52224 B
constexpr int kT1Row = 34 * 256;
constexpr int kT2 = kT1 + 6 * kT1Row;        // t2: [128 px][256 B]                   32768 B
constexpr int kBN = kT2 + 128 * 256;         // s1 b1 s2 b2 (128 each) s3 b3 (512 each) f32
constexpr int kLds = kBN + (4 * kP + 2 * kC) * 4;
static_assert(kLds <= 160 * 1024, "LDS");

// 256-B LDS rows (128 bf16 channels): 16-B chunk XOR-swizzled by the row's low 4 bits
__device__ __forceinline__ int swz16(int row, int chunk) { return row * 256 + ((chunk ^ (row & 15)) << 4); }

__device__ __forceinline__ void ld8(const float* p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__global__ __launch_bounds__(512, 1) void bottleneck2_kernel(Bottle2Geom g) {
  using O = Op<T>;
  constexpr int ES = 2;
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const int pg = wid & 3, h = wid >> 2;
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));
  const int n = blockIdx.x / g.strips;
  const int ya = (blockIdx.x - n * g.strips) * g.rows;
  const int H = g.H;
  const int nsteps = g.rows / kR;
  float* bn = reinterpret_cast<float*>(smem + kBN);

  // ---- prologue: BN parameters, the ring's zero columns
  if (tid < kP) {
    bn[tid] = g.s1[tid];
    bn[kP + tid] = g.b1[tid];
    bn[2 * kP + tid] = g.s2[tid];
    bn[3 * kP + tid] = g.b2[tid];
  }
  bn[4 * kP + tid] = g.s3[tid];
  bn[4 * kP + kC + tid] = g.b3[tid];
  if (tid < 6 * 2 * 16) {  // 6 rows x 2 edge columns x 16 chunks
    const int r = tid >> 5, side = (tid >> 4) & 1, ch = tid & 15;
    *reinterpret_cast<uint4*>(smem + kT1 + r * kT1Row + side * 33 * 256 + ch * 16) = make_uint4(0, 0, 0, 0);
  }

  // ---- DMA sources
  const u32x4 xs = make_srd(g.x, g.N * H * kW * kC * ES);
  const u32x4 w1s = make_srd(g.w1, kP * kC * ES);
  const u32x4 w2s = make_srd(g.w2, kP * 9 * kP * ES);
  const u32x4 w3s = make_srd(g.w3, kC * kP * ES);
  // 128-B-row images (conv1 stages): thread -> row (tid >> 3) + 64 i, logical chunk cl1
  const int cl1 = (tid & 7) ^ ((tid >> 4) & 7);
  const int row1 = tid >> 3;
  // 256-B-row images (conv2 / conv3 stages): wave instruction i writes rows 4 (w + 8 i) ..,
  // lane -> row 4 (w + 8 i) + (lane >> 4), logical chunk cl2 (row & 15 is the same for all i)
  const int row2 = 4 * wid + (lane >> 4);
  const int cl2 = (lane & 15) ^ (row2 & 15);

  // conv1 stage c of the rows ybase .. ybase + 3: x chunk (OOB rows -> zeros) + w1 chunk
  auto dma_conv1 = [&](int ybase, int c, unsigned slot) {
    const unsigned dst = lds0 + slot + wid_u * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = row1 + 64 * i, yy = ybase + (r >> 5);
      const bool ok = static_cast<unsigned>(yy) < static_cast<unsigned>(H);
      dma16(xs, ok ? (((n * H + yy) * kW + (r & 31)) * kC + 64 * c + 8 * cl1) * ES : kOOB, dst + i * 8192);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(w1s, ((row1 + 64 * i) * kC + 64 * c + 8 * cl1) * ES, dst + 16384 + i * 8192);
  };
  auto dma_w2 = [&](int t, unsigned slot) {
    const unsigned dst = lds0 + slot + wid_u * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      dma16(w2s, ((row2 + 32 * i) * (9 * kP) + t * kP + 8 * cl2) * ES, dst + i * 8192);
  };
  auto dma_w3 = [&](int c, unsigned slot) {
    const unsigned dst = lds0 + slot + wid_u * 1024;
#pragma unroll
    for (int i = 0; i < 4; ++i) dma16(w3s, ((128 * c + row2 + 32 * i) * kP + 8 * cl2) * ES, dst + i * 8192);
  };

  f32x4 acc[2][4];  // [m-tile i: pixels 16 i + r16 of row pg][n-tile j: channels 64 h + 16 j + 4 q ..]
  auto zero = [&] {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // pair (j = 2 jp, 2 jp + 1) -> this lane's 8 consecutive channels 16 (2 jp + (q & 1)) + 8 (q >> 1)
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

  auto conv1_mma = [&](unsigned slot) {
    const char* S = smem + slot;
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      uint4 a[4], b[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const uint4*>(S + 16384 + swz(64 * h + 16 * j + r16, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const uint4*>(S + swz(32 * pg + 16 * i + r16, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) O::mma(acc[i][j], a[j], b[i]);
    }
  };
  auto t1_slot = [&](int yy) { return ((yy % 6) + 6) % 6; };
  // t1 row y1 (BN1 + ReLU; zeros outside the image) into the ring
  auto conv1_out = [&](int y1) {
    const bool ok = static_cast<unsigned>(y1) < static_cast<unsigned>(H);
    char* R = smem + kT1 + t1_slot(y1) * kT1Row;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int c0 = 64 * h + 32 * jp + cpair;
      float sc[8], sh[8];
      ld8(bn + c0, sc);
      ld8(bn + kP + c0, sh);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[8];
        pair(i, jp, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = ok ? fmaxf(v[e] * sc[e] + sh[e], 0.f) : 0.f;
        *reinterpret_cast<uint4*>(R + swz16(16 * i + r16 + 1, c0 >> 3)) = O::store_vals(v);
      }
    }
  };
  // conv2 tap t of output row y2 = ybase + pg: ring rows y2 - 1 + t / 3, columns px + t % 3
  auto conv2_mma = [&](unsigned slot, int t, int y2) {
    const char* S = smem + slot;
    const int dy = t / 3, dx = t % 3;
    const char* R = smem + kT1 + t1_slot(y2 - 1 + dy) * kT1Row;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      uint4 a[4], b[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const uint4*>(S + swz16(64 * h + 16 * j + r16, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const uint4*>(R + swz16(16 * i + r16 + dx, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) O::mma(acc[i][j], a[j], b[i]);
    }
  };
  auto conv2_out = [&] {  // BN2 + ReLU -> t2 tile rows 32 pg + px
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int c0 = 64 * h + 32 * jp + cpair;
      float sc[8], sh[8];
      ld8(bn + 2 * kP + c0, sc);
      ld8(bn + 3 * kP + c0, sh);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[8];
        pair(i, jp, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e], 0.f);
        *reinterpret_cast<uint4*>(smem + kT2 + swz16(32 * pg + 16 * i + r16, c0 >> 3)) = O::store_vals(v);
      }
    }
  };
  auto conv3_mma = [&](unsigned slot) {
    const char* S = smem + slot;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      uint4 a[4], b[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = *reinterpret_cast<const uint4*>(S + swz16(64 * h + 16 * j + r16, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 2; ++i) b[i] = *reinterpret_cast<const uint4*>(smem + kT2 + swz16(32 * pg + 16 * i + r16, 4 * cb + q));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) O::mma(acc[i][j], a[j], b[i]);
    }
  };
  const T* __restrict__ xg = reinterpret_cast<const T*>(g.x);
  T* __restrict__ yg = reinterpret_cast<T*>(g.y);
  // residual chunks of output row y2, chunk c (loaded before the chunk's MMAs)
  auto res_load = [&](int y2, int c, uint4 (&rv)[2][2]) {
    const T* xr = xg + (static_cast<size_t>(n * H + y2) * kW) * kC + 128 * c + 64 * h + cpair;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) rv[i][jp] = *reinterpret_cast<const uint4*>(xr + (16 * i + r16) * kC + 32 * jp);
  };
  auto conv3_out = [&](int y2, int c, const uint4 (&rv)[2][2]) {
    T* yr = yg + (static_cast<size_t>(n * H + y2) * kW) * kC;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int c0 = 128 * c + 64 * h + 32 * jp + cpair;
      float sc[8], sh[8];
      ld8(bn + 4 * kP + c0, sc);
      ld8(bn + 4 * kP + kC + c0, sh);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[8], r[8];
        pair(i, jp, v);
        O::load_vals(rv[i][jp], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e] + r[e], 0.f);
        *reinterpret_cast<uint4*>(yr + (16 * i + r16) * kC + c0) = O::store_vals(v);
      }
    }
  };

  // ---- the stage stream.  gs counts stages from the start (slot = gs & 1); a stage waits
  // for its own DMA (the youngest vector-memory ops after it are the previous conv3
  // chunk's 4 stores, if any), passes the barrier, issues the next stage's DMA, computes.
  unsigned gs = 0;
  auto slot_of = [](unsigned s) { return (s & 1u) * static_cast<unsigned>(kSlotB); };
  // issue the DMA of stage u (0..20) of the step whose t1 rows start at y1base (conv1) and
  // whose output rows start at y1base - 1
  auto dma_stage = [&](int u, int y1base, unsigned slot) {
    if (u < 8) dma_conv1(y1base, u, slot);
    else if (u < 17) dma_w2(u - 8, slot);
    else dma_w3(u - 17, slot);
  };
  // prologue: conv1 of rows ya-3 .. ya (only ya-1, ya are used; rows < 0 are zeros)
  dma_conv1(ya - 3, 0, slot_of(0));
#pragma unroll 1
  for (int c = 0; c < 8; ++c) {
    vm_wait<0>();
    lds_barrier();
    const unsigned cur = slot_of(gs), nxt = slot_of(gs + 1);
    if (c < 7) dma_conv1(ya - 3, c + 1, nxt);
    else dma_conv1(ya + 1, 0, nxt);  // step 0's first stage
    if (c == 0) zero();
    conv1_mma(cur);
    if (c == 7) conv1_out(ya - 3 + pg);
    ++gs;
  }
  uint4 rv[2][2];
#pragma unroll 1
  for (int k = 0; k < nsteps; ++k) {
    const int yo = ya + kR * k;           // output rows yo .. yo+3
    const int y1 = yo + 1;                // t1 rows computed: yo+1 .. yo+4
    const bool last = k + 1 == nsteps;
#pragma unroll 1
    for (int u = 0; u < 21; ++u) {
      // younger than this stage's DMA: the 4 stores of the previous conv3 chunk
      if (u >= 18 || (u == 0 && k > 0)) vm_wait<4>();
      else vm_wait<0>();
      lds_barrier();
      const unsigned cur = slot_of(gs), nxt = slot_of(gs + 1);
      if (u >= 17) res_load(yo + pg, u - 17, rv);
      if (u < 20) dma_stage(u + 1, y1, nxt);
      else if (!last) dma_stage(0, y1 + kR, nxt);
      if (u == 0 || u == 8 || u >= 17) zero();
      if (u < 8) {
        conv1_mma(cur);
        if (u == 7) conv1_out(y1 + pg);
      } else if (u < 17) {
        conv2_mma(cur, u - 8, yo + pg);
        if (u == 16) conv2_out();
      } else {
        conv3_mma(cur);
        conv3_out(yo + pg, u - 17, rv);
      }
      ++gs;
    }
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_bottleneck2_fwd(int dtype, const void* x, int N, int H, int W, int C, int P, const void* w1,
                                    const float* s1, const float* b1, const void* w2, const float* s2,
                                    const float* b2, const void* w3, const float* s3, const float* b3, void* y,
                                    void* stream) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, "posu_bottleneck2_fwd: dtype must be BF16 or F16");
  POSU_REQUIRE(x && w1 && s1 && b1 && w2 && s2 && b2 && w3 && s3 && b3 && y, "posu_bottleneck2_fwd: null pointer");
  POSU_REQUIRE(x != y, "posu_bottleneck2_fwd: the output must not alias the input");
  POSU_REQUIRE(W == kW && C == kC && P == kP,
               "posu_bottleneck2_fwd: built for W = 32, C = 512, planes = 128 (layer2 of PoseResNet at 256x256)");
  POSU_REQUIRE(N > 0 && H > 0 && H % kR == 0, "posu_bottleneck2_fwd: H must be a positive multiple of 4");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * 2 < (1LL << 31) - 256,
               "posu_bottleneck2_fwd: activation exceeds the 2 GiB addressing range");
  for (const void* p : {x, static_cast<const void*>(y), w1, w2, w3})
    POSU_REQUIRE((reinterpret_cast<size_t>(p) & 15) == 0, "posu_bottleneck2_fwd: pointers must be 16-byte aligned");
  Bottle2Geom g{};
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
  int strips = 1;  // about one workgroup per CU, strips of whole 4-row steps
  while (N * strips * 2 <= 256 && H % (strips * 2 * kR) == 0) strips *= 2;
  g.strips = strips;
  g.rows = H / strips;
  hipStream_t s = as_stream(stream);
  if (dtype == POSU_BF16)
    hipLaunchKernelGGL(bottleneck2_kernel<uint16_t>, dim3(N * strips), dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL(bottleneck2_kernel<f16_t>, dim3(N * strips), dim3(512), 0, s, g);
  return check_launch("posu_bottleneck2_fwd");
}
