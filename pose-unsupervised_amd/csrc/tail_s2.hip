// Tail of the FIRST Bottleneck of layer2 (lib/models/pose_resnet.py:61-99 with the downsample
// branch, pose_resnet.py:136-141; eval mode, BN folded) of PoseResNet at 256x256:
//
//     y = relu( [w3*s3 | wd*sd] . [ relu(bn2(conv2_3x3_s2(t1))) ; x(2 oy, 2 ox) ] + (b3 + bd) )
//
// t1 [N, H, 64, 128] (conv1's output), x [N, H, 64, 256] (the block input), y [N, H/2, 32, 512].
// The plan ran this as two launches: the 3x3 / stride-2 conv2 (reading t1 with a 1.74x over-fetch
// of its overlapping windows, writing t2) and the two-source 1x1 "dual" GEMM (t2 plus the stride-2
// pixels of x); here t2 never leaves the CU and t1 is read once per tile window.
//
// One workgroup (4 waves, two workgroups per CU) owns 4 output rows x 16 output columns = 64 px:
//   LDS   the t1 window (rows 2 R0 - 1 .. 2 R0 + 7, columns 2 C0 - 1 .. 2 C0 + 31, zeros outside
//         the image = conv2's padding; 9 x 33 px x 256 B, LDS-DMA), BN2; after conv2, over the
//         window: t2 [64 px][128 ch], the tile's stride-2 x pixels [64 px][256 ch] (LDS-DMA) and
//         the shift b3 + bd.
//   wave  cq owns conv2 output channels 32 cq .. + 31 (2 n-tiles) and, in dual chunk nc, output
//         channels 128 nc + 32 cq .. + 31; its 4 m-tiles are the tile's 4 output rows (16 px each).
//   weights  streamed from L2 straight into VGPRs kD k-steps ahead (one contiguous 2 KB per
//         k-step and wave, packing.pack_s2_tail_stream): conv2 tap t, channel step d (k-step
//         4 t + d: conv_igemm's tap-major K order), then per dual chunk its 12 k-steps (t2's 4,
//         then x's 8: the dual GEMM's K order) -- the same MFMA sequence per accumulator as the
//         two launches, so t2 and y are bit-identical to them.
// LDS images are [pixel][channels] rows with the 16-B chunk index XOR (LDS column & 15): the
// stride-2 window reads of a 16-lane group (columns 2 r + dx) and the stride-1 t2 / x reads then
// hit 16 distinct chunk slots.
// MFMA operands swapped (A = weights, B = pixels): lane (r16, q) accumulates channels 4q .. 4q+3
// of pixel r16; v_permlane16_swap pairs the 2 n-tiles into 8 consecutive channels.
#include <type_traits>

#include "gemm_common.h"

namespace posu {
namespace {

struct TailS2Geom {
  const void* t1;
  const void* x;
  void* y;
  const uint4* wst;   // [4 channel groups][kSteps][2 n-tiles][64 lanes] x 16 B
  const float* s2;
  const float* b2;
  const float* shift;  // b3 + bd [512]
  int N, Hin;
  // NEXT (chained): the next identity block's conv1 + BN1 + ReLU over y while it is produced
  // (t1n = relu(y conv1n * s1n + b1n), [N][Hin/2][32][128])
  const float* s1n;
  const float* b1n;
  void* t1n;
  long long wseg;  // the weight stream's 64-B segments (warm-up, gemm_common.h)
  int warm;        // warm-up workgroups (0: none)
};

#ifndef POSU_S2_KD
#define POSU_S2_KD 4
#endif

template <bool NEXT>
struct S2Cfg {
  static constexpr int kWin = 64, kC = 256, kP = 128, kCout = 512, kWout = 32;
  static constexpr int kRows = 4, kTW = 16, kNW = 4, kPx = kRows * kTW;   // 64 output px
  static constexpr int kWR = 2 * kRows + 1, kWC = 2 * kTW + 1;            // 9 x 33 window
  static constexpr int kRowB = kP * 2;                                    // 256 B per t1 / t2 pixel
  static constexpr int kXRowB = kC * 2;                                   // 512 B per x pixel
  static constexpr int kWinInst = (kWR * kWC * kRowB + 1023) / 1024;      // 1 KB DMA instructions
  static constexpr int kBN2 = kWinInst * 1024;                            // s2 b2 behind the window
  static constexpr int kLds = kBN2 + 2 * kP * 4;
  static constexpr int kT2 = 0;                                           // after conv2, over the window
  static constexpr int kX = kT2 + kPx * kRowB;
  static constexpr int kShift = kX + kPx * kXRowB;
  static constexpr int kKT = kP / 32;                                     // k-steps per tap / over t2
  static constexpr int kKX = kC / 32;                                     // k-steps over x
  static constexpr int kNC = kCout / (32 * kNW);                          // dual chunks of 128 channels
  // NEXT: after each dual chunk, the next conv1's kKT k-steps over that chunk's 128 y channels
  static constexpr int kSteps2 = 9 * kKT, kStepsC = kKT + kKX + (NEXT ? kKT : 0);
  static constexpr int kSteps = kSteps2 + kNC * kStepsC;                  // 36 + 4 x 12 = 84 (NEXT: 100)
  static constexpr int kYC = kShift + kCout * 4;                          // NEXT: the y chunk [64 px][128 ch]
  static constexpr int kD = POSU_S2_KD;
  static_assert(kYC + (NEXT ? kPx * kRowB : 0) <= kBN2, "t2, the x pixels, the shift (and the y chunk) fit over the window");
  static_assert(2 * kLds <= 160 * 1024, "two workgroups per CU");
  static_assert(kKT % kD == 0 && kKX % kD == 0 && kSteps2 % kD == 0 && kStepsC % kD == 0,
                "every block starts on ring slot 0");
};

template <typename T, bool NEXT>
__global__ __launch_bounds__(S2Cfg<NEXT>::kNW * 64, 2) void tail_s2_kernel(TailS2Geom g) {
  using O = Op<T>;
  using K = S2Cfg<NEXT>;
  constexpr int ES = 2, kD = K::kD, MT = K::kRows;
  __shared__ __attribute__((aligned(16))) char smem[K::kLds];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int r16 = lane & 15, q = lane >> 4;
  const int cq = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds0 = static_cast<unsigned>(reinterpret_cast<size_t>((__attribute__((address_space(3))) char*)smem));
  const int Hin = g.Hin, Hout = Hin / 2;
  const int tiles_x = K::kWout / K::kTW, tiles_y = Hout / K::kRows;
  const int n = blockIdx.x / (tiles_x * tiles_y);
  const int rem = blockIdx.x - n * tiles_x * tiles_y;
  const int R0 = (rem / tiles_x) * K::kRows, C0 = (rem % tiles_x) * K::kTW;
  float* bn2 = reinterpret_cast<float*>(smem + K::kBN2);
  for (int c = tid; c < K::kP; c += K::kNW * 64) {
    bn2[c] = g.s2[c];
    bn2[K::kP + c] = g.b2[c];
  }

  // ---- the t1 window: 4 px per 1 KB wave-instruction, instruction m by wave m & 3
  {
    const u32x4 t1s = make_srd(g.t1, g.N * Hin * K::kWin * K::kP * ES);
    const int sub = lane >> 4, pc = lane & 15;
#pragma unroll
    for (int k = 0; k < (K::kWinInst + K::kNW - 1) / K::kNW; ++k) {
      const int m = cq + K::kNW * k;
      if (m < K::kWinInst) {  // wave-uniform
        const int pix = 4 * m + sub;
        const int wr = pix / K::kWC, wc = pix - wr * K::kWC;
        const int yy = 2 * R0 - 1 + wr, xx = 2 * C0 - 1 + wc;
        const int lc = pc ^ (wc & 15);
        const bool ok = wr < K::kWR && static_cast<unsigned>(yy) < static_cast<unsigned>(Hin) &&
                        static_cast<unsigned>(xx) < static_cast<unsigned>(K::kWin);
        dma16(t1s, ok ? (((n * Hin + yy) * K::kWin + xx) * K::kP + 8 * lc) * ES : kOOB,
              lds0 + static_cast<unsigned>(m) * 1024u);
      }
    }
  }

  // ---- the weight stream of channel group cq (prefetches past the end reload the last k-step)
  const char* wst = reinterpret_cast<const char*>(g.wst) + cq * (K::kSteps * 2 * 1024);
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
  unsigned wv[kWarmLoads];   // the stream's warm-up (gemm_common.h)
  warm_issue(wv, g.wst, g.wseg, g.warm, K::kNW * 64);
  vm_wait<0>();  // the window (LDS-DMA) and the first fragments
  warm_use(wv);
  lds_barrier();

  f32x4 acc[MT][2];
  f32x4 acc1[MT][2];  // NEXT: the next conv1's accumulators over the whole chunk loop
  auto zero = [&](f32x4 (&a)[MT][2]) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) a[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
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
  // NS k-steps (stream k-steps p0 .., p0 a multiple of kD: the ring slot of k-step d is the
  // compile-time d % kD) over an LDS image of RB-byte pixel rows: k-step d reads, for
  // m-tile i, the pixel lpix + coff(i) at 16-B chunk 4 d + q, XOR the lane's key (its LDS
  // column & 15).  The pixel fragments of k-step d + 1 are read while k-step d's MFMAs run.
  auto block = [&](f32x4 (&acc)[MT][2], auto nsteps, auto rowb, int p0, int base, int lpix, int key, auto coff) {
    constexpr int NS = decltype(nsteps)::value, RB = decltype(rowb)::value;
    uint4 b[2][MT];
    const char* lb = smem + base + lpix * RB + ((q ^ (key & 3)) << 4);
    const char* kb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) kb[k] = lb + ((k ^ (key >> 2)) << 6);
    auto rd = [&](int i, int d) -> uint4 {
      return *reinterpret_cast<const uint4*>(kb[d & 3] + coff(i) * RB + (d & 4) * 64);
    };
#pragma unroll
    for (int i = 0; i < MT; ++i) b[0][i] = rd(i, 0);
#pragma unroll
    for (int d = 0; d < NS; ++d) {
      if (d + 1 < NS) {
#pragma unroll
        for (int i = 0; i < MT; ++i) b[(d + 1) & 1][i] = rd(i, d + 1);
      }
      const int s = d % kD;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) O::mma(acc[i][j], wa[s][j], b[d & 1][i]);
      const int p = p0 + d + kD;
      wa[s][0] = *frag(p, 0);
      wa[s][1] = *frag(p, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using NKT = std::integral_constant<int, K::kKT>;
  using NKX = std::integral_constant<int, K::kKX>;
  using RBT = std::integral_constant<int, K::kRowB>;
  using RBX = std::integral_constant<int, K::kXRowB>;

  // ---- conv2: 9 taps x 4 channel steps; m-tile i = output row i: window row 2 i + dy, column
  // 2 r16 + dx
  zero(acc);
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    const int dy = t / 3, dx = t - 3 * (t / 3);
    block(acc, NKT{}, RBT{}, K::kKT * t, 0, dy * K::kWC + 2 * r16 + dx, (2 * r16 + dx) & 15,
          [&](int i) { return 2 * i * K::kWC; });
  }
  // every wave is done reading the window: the tile's stride-2 x pixels are DMA'd over it while
  // BN2 + ReLU write t2 beside them
  lds_barrier();
  {
    const u32x4 xs = make_srd(g.x, g.N * Hin * K::kWin * K::kC * ES);
    const int sub = lane >> 5, pc = lane & 31;
#pragma unroll
    for (int k = 0; k < K::kPx / 2 / K::kNW; ++k) {
      const int m = cq + K::kNW * k;
      const int px = 2 * m + sub, i = px >> 4, r = px & 15;
      const int lc = (pc & 16) | ((pc ^ r) & 15);
      dma16(xs, (((n * Hin + 2 * (R0 + i)) * K::kWin + 2 * (C0 + r)) * K::kC + 8 * lc) * ES,
            lds0 + static_cast<unsigned>(K::kX + m * 1024));
    }
  }
  {
    float* shl = reinterpret_cast<float*>(smem + K::kShift);
    for (int c = tid; c < K::kCout; c += K::kNW * 64) shl[c] = g.shift[c];
    const int c0 = 32 * cq + cpair;
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = bn2[c0 + e];
      sh[e] = bn2[K::kP + c0 + e];
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8];
      pair(acc, i, v);
      affine8<false>(v, sc, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      *reinterpret_cast<uint4*>(smem + K::kT2 + (16 * i + r16) * K::kRowB + (((c0 >> 3) ^ r16) << 4)) =
          O::store_vals(v);
    }
  }
  vm_wait<0>();  // the x DMA (and the weight prefetches)
  lds_barrier();

  // ---- the dual GEMM, chunk nc: output channels 128 nc + 32 cq ..; K = t2's 128 channels, then
  // the 256 channels of x (2 oy, 2 ox)
  const float* shl = reinterpret_cast<const float*>(smem + K::kShift);
  T* yg = reinterpret_cast<T*>(g.y);
  if constexpr (NEXT) zero(acc1);
#pragma unroll
  for (int nc = 0; nc < K::kNC; ++nc) {
    const int p0 = K::kSteps2 + K::kStepsC * nc;
    zero(acc);
    block(acc, NKT{}, RBT{}, p0, K::kT2, r16, r16, [&](int i) { return 16 * i; });
    block(acc, NKX{}, RBX{}, p0 + K::kKT, K::kX, r16, r16, [&](int i) { return 16 * i; });
    const int c0 = 128 * nc + 32 * cq + cpair;
    float sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) sh[e] = shl[c0 + e];
    if constexpr (NEXT) {
      if (nc > 0) lds_barrier();  // every wave is done reading the previous y chunk
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8];
      pair(acc, i, v);
      add8<false>(v, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      const size_t pix = (static_cast<size_t>(n) * Hout + R0 + i) * K::kWout + C0 + r16;
      const uint4 o = O::store_vals(v);
      *reinterpret_cast<uint4*>(yg + pix * K::kCout + c0) = o;
      // NEXT: the chunk's y (the rounded values just stored), laid out like t2
      if constexpr (NEXT)
        *reinterpret_cast<uint4*>(smem + K::kYC + (16 * i + r16) * K::kRowB + ((((c0 & 127) >> 3) ^ r16) << 4)) = o;
    }
    if constexpr (NEXT) {
      // the next block's conv1 over this K slice (y channels 128 nc ..): the k order of a conv
      // launch over y, so t1n is bit-identical to it
      lds_barrier();
      block(acc1, NKT{}, RBT{}, p0 + K::kKT + K::kKX, K::kYC, r16, r16, [&](int i) { return 16 * i; });
    }
  }
  if constexpr (NEXT) {
    // t1n = relu(conv1n * s1n + b1n): this lane's 8 channels of each m-tile's pixel
    T* tg = reinterpret_cast<T*>(g.t1n);
    const int c0 = 32 * cq + cpair;
    float sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = g.s1n[c0 + e];
      sh[e] = g.b1n[c0 + e];
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v[8];
      pair(acc1, i, v);
      affine8<false>(v, sc, sh);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
      const size_t pix = (static_cast<size_t>(n) * Hout + R0 + i) * K::kWout + C0 + r16;
      *reinterpret_cast<uint4*>(tg + pix * K::kP + c0) = O::store_vals(v);
    }
  }
}

}  // namespace
}  // namespace posu

using namespace posu;

namespace {
int s2_tail_impl(const char* name, int dtype, const void* t1, const void* x, int N, int H, int W, int C, int P,
                 const void* wstream, long long wstream_bytes, const float* s2, const float* b2, const float* shift,
                 int Cout, void* y, const float* s1n, const float* b1n, void* t1n, void* stream) {
  const std::string what = name;
  const bool next = t1n != nullptr;
  using K = S2Cfg<false>;
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F16, what + ": dtype must be BF16 or F16");
  POSU_REQUIRE(t1 && x && wstream && s2 && b2 && shift && y, what + ": null pointer");
  POSU_REQUIRE(y != x && y != t1, what + ": the output must not alias an input");
  POSU_REQUIRE(!next || (s1n && b1n && t1n != y && t1n != x && t1n != t1),
               what + ": the next conv1 needs its BN and an output that aliases no other operand");
  POSU_REQUIRE(W == K::kWin && C == K::kC && P == K::kP && Cout == K::kCout,
               what + ": built for the first Bottleneck of layer2 of PoseResNet at 256x256 (input W = 64, C = 256, "
                      "planes = 128, output channels 512)");
  POSU_REQUIRE(N > 0 && H > 0 && H % (2 * K::kRows) == 0,
               what + ": H must be a positive multiple of " + std::to_string(2 * K::kRows));
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * 2 < (1LL << 31) - 256,
               what + ": activation exceeds the 2 GiB addressing range");
  const long long need = static_cast<long long>(K::kNW) * (next ? S2Cfg<true>::kSteps : K::kSteps) * 2 * 1024;
  POSU_REQUIRE(wstream_bytes == need, what + ": wstream holds " + std::to_string(wstream_bytes) + " bytes, the " +
                                          (next ? "chained" : "plain") + " kernel reads " + std::to_string(need));
  for (const void* p : {t1, x, static_cast<const void*>(y), wstream, static_cast<const void*>(shift),
                        next ? t1n : t1, static_cast<const void*>(next ? s1n : shift),
                        static_cast<const void*>(next ? b1n : shift)})
    POSU_REQUIRE((reinterpret_cast<size_t>(p) & 15) == 0, what + ": pointers must be 16-byte aligned");
  TailS2Geom g{};
  g.t1 = t1;
  g.x = x;
  g.y = y;
  g.wst = static_cast<const uint4*>(wstream);
  g.s2 = s2;
  g.b2 = b2;
  g.shift = shift;
  g.N = N;
  g.Hin = H;
  g.s1n = s1n;
  g.b1n = b1n;
  g.t1n = t1n;
  g.wseg = wstream_bytes / 64;
  g.warm = warm_wgs(wstream_bytes);
  const dim3 grid(static_cast<unsigned>(N * (H / 2 / K::kRows) * (K::kWout / K::kTW)));
  hipStream_t s = as_stream(stream);
  if (dtype == POSU_BF16) {
    if (next) hipLaunchKernelGGL((tail_s2_kernel<uint16_t, true>), grid, dim3(K::kNW * 64), 0, s, g);
    else hipLaunchKernelGGL((tail_s2_kernel<uint16_t, false>), grid, dim3(K::kNW * 64), 0, s, g);
  } else {
    if (next) hipLaunchKernelGGL((tail_s2_kernel<f16_t, true>), grid, dim3(K::kNW * 64), 0, s, g);
    else hipLaunchKernelGGL((tail_s2_kernel<f16_t, false>), grid, dim3(K::kNW * 64), 0, s, g);
  }
  return check_launch(name);
}
}  // namespace

// The tail of the first Bottleneck of layer2 (see the top of this file).  wstream =
// packing.pack_s2_tail_stream(conv2 pack [128][1152], dual pack [512][384]); wstream_bytes its size.
extern "C" int posu_bottleneck_s2_tail_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                           int P, const void* wstream, long long wstream_bytes, const float* s2,
                                           const float* b2, const float* shift, int Cout, void* y, void* stream) {
  return s2_tail_impl("posu_bottleneck_s2_tail_fwd", dtype, t1, x, N, H, W, C, P, wstream, wstream_bytes, s2, b2,
                      shift, Cout, y, nullptr, nullptr, nullptr, stream);
}

// The same, chained with the next (identity) block's conv1 + BN1 + ReLU over y, like
// posu_bottleneck_tail_stream_next_fwd: t1n [N][H/2][32][128] is bit-identical to a conv launch
// over y, and that block skips its conv1 launch.  wstream = packing.pack_s2_tail_stream(conv2
// pack, dual pack, next conv1 pack [128][512]).
extern "C" int posu_bottleneck_s2_tail_next_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                                int P, const void* wstream, long long wstream_bytes, const float* s2,
                                                const float* b2, const float* shift, int Cout, void* y,
                                                const float* s1n, const float* b1n, void* t1n, void* stream) {
  if (!t1n) {
    set_error("posu_bottleneck_s2_tail_next_fwd: null pointer (t1n)");
    return POSU_ERR_ARG;
  }
  return s2_tail_impl("posu_bottleneck_s2_tail_next_fwd", dtype, t1, x, N, H, W, C, P, wstream, wstream_bytes, s2,
                      b2, shift, Cout, y, s1n, b1n, t1n, stream);
}
