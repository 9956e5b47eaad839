// Fused Bottleneck block (lib/models/pose_resnet.py:61-99, eval mode, BN folded):
//
//     y = relu( bn3(conv3( relu(bn2(conv2_3x3( relu(bn1(conv1(x))) ))) )) + x )
//
// for the identity-residual blocks of layer1 (x [N, H, 64, 256], planes 64) in ONE
// launch that reads x from HBM exactly once and writes y once: per block 2 x 268 MB at
// batch 128, against 1.07 GB for three separate convolutions (whose two 64-channel
// intermediates and the residual re-read make up the rest).
//
// Streaming structure.  One workgroup (4 waves, 1 per CU: 131 KiB of LDS) walks down a
// strip of output rows of one image, one row (64 pixels) per step; wave w owns pixels
// 16w .. 16w+15 of every row in every phase:
//   conv1    t1 row y+1 = relu(bn1(x row y+1 . w1)): x fragments straight from HBM into
//            VGPRs (prefetched two rows ahead), w1 held in VGPRs for the whole strip.
//            The row goes into a 3-row LDS ring [row][64 px][64 ch] (rows outside the
//            image are zeros = conv2's padding), so every conv1 row is computed once.
//   conv2    3x3 over ring rows y-1, y, y+1 (x-padding = zeroed fragments), w2 [9][64][64]
//            resident in LDS; BN2 + ReLU stay in registers, rounded, and ARE conv3's B
//            fragments: lane (p, q) holds channels 4q..4q+3 of two n-tiles = one MFMA k-step
//            in a permuted channel order, in which conv3's weights are packed.
//   conv3    w3 [256][64] resident in LDS; BN3 + residual + ReLU; 16-B NHWC stores.  The
//            residual is x row y -- the registers conv1 consumed one step earlier: conv1's K
//            order is permuted so that its k-step s of lane q holds exactly the 8 channels
//            the conv3 epilogue of lane q adds for output pair s.
// Per row and wave: 32 + 72 + 32 MFMAs against 64 KB of HBM traffic per CU, so the loop runs
// at HBM speed with the MFMA / LDS work hidden under it.  An image is split into S strips
// (S * N ~ the CU count); a strip recomputes the one conv1 row above it.
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
  const void* w3;  // [256][64], K permuted (bottleneck_conv3_order)
  const float* s3;
  const float* b3;
  int N, H;
  int strips;      // strips per image
  int rows;        // rows per strip (H / strips)
};

constexpr int kP = 64, kW = 64, kC = 256;
constexpr int kW2 = 0;                  // w2: 9 taps x [64 co][128 B]       73728 B
constexpr int kW3 = 73728;              // w3: [256 co][128 B]                32768 B
constexpr int kT1 = 106496;             // t1 ring: 3 x [64 px][128 B]        24576 B
constexpr int kBN = 131072;             // s1 b1 s2 b2 (64 each), s3 b3 (256 each) f32  3072 B
constexpr int kLds = 134144;

// workgroup barrier that also publishes this wave's LDS writes (lgkmcnt(0) first); LDS-DMA
// and global loads stay in flight across it
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void ld8(const float* p, float* v) {  // 8 f32 from LDS
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <typename T>
__global__ __launch_bounds__(256, 1) void bottleneck64_kernel(BottleGeom g) {
  using O = Op<T>;
  constexpr int ES = static_cast<int>(sizeof(T));
  static_assert(ES == 2, "bf16 / f16 activations");
  __shared__ __attribute__((aligned(16))) char smem[kLds];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int r16 = lane & 15, q = lane >> 4;
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const unsigned wid_u = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(wid));

  const int n = blockIdx.x / g.strips;
  const int ya = (blockIdx.x - n * g.strips) * g.rows, yb = ya + g.rows;
  const int H = g.H;
  const T* __restrict__ xg = reinterpret_cast<const T*>(g.x);
  T* __restrict__ yg = reinterpret_cast<T*>(g.y);
  const int px = 16 * wid + r16;                   // this lane's pixel column
  // channel offset of lane q in a 32-channel k-step of conv1 (and of the conv3 epilogue)
  const int cq = 16 * (q & 1) + 8 * (q >> 1);
  const float* bn = reinterpret_cast<const float*>(smem + kBN);

  // ---- prologue: w2 / w3 -> LDS (LDS-DMA, swizzled rows), BN params -> LDS, w1 -> VGPRs
  {
    const u32x4 w2s = make_srd(g.w2, kP * 9 * kP * ES);
    const u32x4 w3s = make_srd(g.w3, kC * kP * ES);
    const int cL = (tid & 7) ^ ((tid >> 4) & 7), drow = tid >> 3;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        dma16(w2s, ((drow + 32 * i) * (9 * kP) + t * kP + cL * 8) * ES,
              lds0 + kW2 + t * 8192 + i * 4096 + wid_u * 1024);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      dma16(w3s, ((drow + 32 * i) * kP + cL * 8) * ES, lds0 + kW3 + i * 4096 + wid_u * 1024);
    float* bw = reinterpret_cast<float*>(smem + kBN);
    if (tid < 64) {
      bw[tid] = g.s1[tid];
      bw[64 + tid] = g.b1[tid];
      bw[128 + tid] = g.s2[tid];
      bw[192 + tid] = g.b2[tid];
    }
    bw[256 + tid] = g.s3[tid];
    bw[512 + tid] = g.b3[tid];
  }
  uint4 w1f[8][4];  // [k-step][n-tile]: rows 16 j + r16, permuted K columns 32 s + 8 q .. + 7
  {
    const T* w1 = reinterpret_cast<const T*>(g.w1);
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        w1f[s][j] = *reinterpret_cast<const uint4*>(w1 + (16 * j + r16) * kC + 32 * s + 8 * q);
  }

  // x row r -> this lane's 8 conv1 fragments (left untouched outside the image)
  auto load_row = [&](int r, uint4(&f)[8]) {
    if (r >= 0 && r < H) {
      const T* xr = xg + (static_cast<size_t>(n * H + r) * kW + px) * kC + cq;
#pragma unroll
      for (int s = 0; s < 8; ++s) f[s] = *reinterpret_cast<const uint4*>(xr + 32 * s);
    }
  };
  // conv1 + BN1 + ReLU of x row r into ring slot r % 3 (zeros outside the image)
  auto conv1_row = [&](int r, const uint4(&f)[8]) {
    char* slot = smem + kT1 + ((r + 3) % 3) * 8192;
    const bool ok = r >= 0 && r < H;
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (ok) {
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) O::mma(acc[j], w1f[s][j], f[s]);
    }
#pragma unroll
    for (int jp = 0; jp < 2; ++jp) {
      const int c0 = 16 * (2 * jp + (q & 1)) + 8 * (q >> 1);
      float v[8], sc[8], sh[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[2 * jp][e]),
                                                         __float_as_uint(acc[2 * jp + 1][e]), false, false);
        v[e] = __uint_as_float(sw[0]);
        v[4 + e] = __uint_as_float(sw[1]);
      }
      ld8(bn + c0, sc);
      ld8(bn + 64 + c0, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = ok ? fmaxf(v[e] * sc[e] + sh[e], 0.f) : 0.f;
      *reinterpret_cast<uint4*>(slot + swz(px, c0 >> 3)) = O::store_vals(v);
    }
  };
  // output row y: conv2 over ring rows y-1..y+1, conv3 + BN3 + residual (x row y) + ReLU
  auto out_row = [&](int y, const uint4(&res)[8]) {
    f32x4 acc2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int dy = t / 3, dx = t % 3;
      const char* slot = smem + kT1 + ((y - 1 + dy + 3) % 3) * 8192;
      const char* Wt = smem + kW2 + t * 8192;
      const int xs = px + dx - 1;
      const bool ok = static_cast<unsigned>(xs) < static_cast<unsigned>(kW);
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        uint4 wf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) wf[j] = *reinterpret_cast<const uint4*>(Wt + swz(16 * j + r16, 4 * cb + q));
        const uint4 tv = *reinterpret_cast<const uint4*>(slot + swz(ok ? xs : 0, 4 * cb + q));
        const uint4 tf = ok ? tv : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 4; ++j) O::mma(acc2[j], wf[j], tf);
      }
    }
    uint4 tb[2];  // conv3's B fragments, k-step kb = n-tiles 2 kb, 2 kb + 1
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const int ca = 32 * kb + 4 * q, cb2 = ca + 16;
      const float4 sa = *reinterpret_cast<const float4*>(bn + 128 + ca);
      const float4 sb = *reinterpret_cast<const float4*>(bn + 128 + cb2);
      const float4 ha = *reinterpret_cast<const float4*>(bn + 192 + ca);
      const float4 hb = *reinterpret_cast<const float4*>(bn + 192 + cb2);
      const float s8[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
      const float h8[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = fmaxf(acc2[2 * kb][e] * s8[e] + h8[e], 0.f);
        v[4 + e] = fmaxf(acc2[2 * kb + 1][e] * s8[4 + e] + h8[4 + e], 0.f);
      }
      tb[kb] = O::store_vals(v);
    }
    T* yr = yg + (static_cast<size_t>(n * H + y) * kW + px) * kC;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      f32x4 acc3[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc3[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint4 wf = *reinterpret_cast<const uint4*>(smem + kW3 + swz(64 * qd + 16 * j + r16, 4 * kb + q));
          O::mma(acc3[j], wf, tb[kb]);
        }
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
        ld8(bn + 256 + c0, sc);
        ld8(bn + 512 + c0, sh);
        O::load_vals(res[s], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e] * sc[e] + sh[e] + r[e], 0.f);
        *reinterpret_cast<uint4*>(yr + c0) = O::store_vals(v);
      }
    }
  };

  // x rows in flight: A = row y (residual of the current output row), B = row y+1 (its
  // conv1 now), C = row y+2, D = row y+3 (prefetched); roles rotate A<-B<-C<-D each row
  uint4 xa[8], xb[8], xc[8], xd[8];
  load_row(ya - 1, xd);   // the conv1 row above the strip (recomputed; zeros at the top)
  load_row(ya, xa);
  vm_wait<0>();           // w2 / w3 DMAs, w1, BN staging loads, rows ya-1 and ya
  raw_barrier();          // BN params in LDS visible (the DMA'd weights too)
  load_row(ya + 1, xb);
  load_row(ya + 2, xc);
  conv1_row(ya - 1, xd);
  conv1_row(ya, xa);

  // one output row: conv1 of row y+1 into the ring slot of row y-2 (free: every wave
  // passed the barrier after its last read), prefetch row y+3, barrier (ring rows
  // y-1..y+1 complete), conv2 + conv3 of row y, barrier (slot of row y-1 may be reused)
  auto step = [&](int y, const uint4(&ra)[8], const uint4(&rb)[8], uint4(&rd)[8]) {
    conv1_row(y + 1, rb);
    if (y + 3 <= yb) load_row(y + 3, rd);
    raw_barrier();
    out_row(y, ra);
    raw_barrier();
  };
  for (int y = ya; y < yb; y += 4) {
    step(y, xa, xb, xd);
    if (y + 1 < yb) step(y + 1, xb, xc, xa);
    if (y + 2 < yb) step(y + 2, xc, xd, xb);
    if (y + 3 < yb) step(y + 3, xd, xa, xc);
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_bottleneck_fwd(int dtype, const void* x, int N, int H, int W, int C, int P, const void* w1,
                                   const float* s1, const float* b1, const void* w2, const float* s2, const float* b2,
                                   const void* w3, const float* s3, const float* b3, void* y, void* stream) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, "posu_bottleneck_fwd: dtype must be BF16 or F16");
  POSU_REQUIRE(x && w1 && s1 && b1 && w2 && s2 && b2 && w3 && s3 && b3 && y, "posu_bottleneck_fwd: null pointer");
  POSU_REQUIRE(x != y, "posu_bottleneck_fwd: the output must not alias the input");
  POSU_REQUIRE(W == kW && C == kC && P == kP,
               "posu_bottleneck_fwd: built for W = 64, C = 256, planes = 64 (layer1 of PoseResNet at 256x256)");
  POSU_REQUIRE(N > 0 && H > 0, "posu_bottleneck_fwd: empty input");
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * 2 < (1LL << 31) - 256,
               "posu_bottleneck_fwd: activation exceeds the 2 GiB addressing range");
  for (const void* p : {x, static_cast<const void*>(y), w1, w2, w3})
    POSU_REQUIRE((reinterpret_cast<size_t>(p) & 15) == 0, "posu_bottleneck_fwd: pointers must be 16-byte aligned");
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
  if (dtype == POSU_BF16)
    hipLaunchKernelGGL(bottleneck64_kernel<uint16_t>, dim3(N * strips), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(bottleneck64_kernel<f16_t>, dim3(N * strips), dim3(256), 0, s, g);
  return check_launch("posu_bottleneck_fwd");
}
