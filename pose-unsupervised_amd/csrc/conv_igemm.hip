// Implicit-GEMM convolution on CDNA4 MFMA, NHWC activations.
//
// GEMM view of one launch:  rows m = output pixels (n, oy, ox) of the launch grid,
//                           cols   = output channels,
//                           k      = (kh, kw, ci) taps of the input window.
// A[m][k] is gathered on the fly from the NHWC input (16-byte channel chunks),
// B[k][co] is the packed weight [CoutPad][Kpad] (K contiguous, zero padded).
//
// Block tile BM x BN, K-tile of 128 bytes per row (64 bf16 / 32 f32), 256 threads
// = 4 waves in a 2x2 grid, each wave owning a (BM/2) x (BN/2) accumulator tile made
// of 16x16 MFMA tiles:
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
// Epilogue: accumulators (+BN scale/shift) are staged through LDS as an f32 tile,
// then written as 16-byte NHWC chunks with optional residual add + ReLU (Bottleneck
// tail, lib/models/pose_resnet.py:90-99), or as NCHW f32 heatmaps (+bias) for the
// final 1x1 layer (pose_resnet.py:126-132).
//
// ConvTranspose2d(4, s2, p1) runs as 4 sub-pixel 2x2 stride-1 convolutions, one per
// output parity class (py, px) = blockIdx.z: output (2*qy+py, 2*qx+px) reads inputs
// qy + py - 1 + ty, qx + px - 1 + tx with the deconv tap (3-py-2ty, 3-px-2tx);
// the Python layer packs those taps per class.
#include "posu_common.h"

namespace posu {
namespace {

struct ConvGeom {
  const void* x;
  const void* w;
  const float* scale;
  const float* shift;
  const void* res;
  void* y;
  int N, H, W, C, logC;
  int Ho, Wo, M;  // launch grid: rows = N*Ho*Wo
  int Cout, CoutPad, K, Kpad;
  int KH, KW, stride, pad_h, pad_w;
  int relu;
  int deconv;        // blockIdx.z = parity class
  int out_H, out_W;  // output tensor spatial dims
  int mode;          // 0: NHWC out (dtype), 1: NCHW f32 out
  int mtiles, ntiles;
};

template <typename T>
struct Op;

template <>
struct Op<uint16_t> {  // bf16
  static constexpr int E = 8;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                  __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void load_vals(const uint4& u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ uint4 store_vals(const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = static_cast<uint32_t>(f2bf(v[2 * i])) | (static_cast<uint32_t>(f2bf(v[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
};

template <>
struct Op<float> {
  static constexpr int E = 4;
  static __device__ __forceinline__ void mma(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
  static __device__ __forceinline__ void load_vals(const uint4& u, float* v) {
    v[0] = __uint_as_float(u.x);
    v[1] = __uint_as_float(u.y);
    v[2] = __uint_as_float(u.z);
    v[3] = __uint_as_float(u.w);
  }
  static __device__ __forceinline__ uint4 store_vals(const float* v) {
    return make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]),
                      __float_as_uint(v[3]));
  }
};

__device__ __forceinline__ int swz(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <int BM, int BN>
constexpr int smem_bytes() {
  return (2 * (BM + BN) * 128) > (BM * (BN + 4) * 4) ? (2 * (BM + BN) * 128) : (BM * (BN + 4) * 4);
}

template <typename T, int BM, int BN>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvGeom g) {
  using O = Op<T>;
  constexpr int E = O::E;
  constexpr int BK = 8 * E;  // 128-byte LDS rows
  constexpr int WTM = BM / 2, WTN = BN / 2;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int RA = BM / 32, RB = BN / 32;  // 16-B chunks per thread per K-tile
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  __shared__ __attribute__((aligned(16))) char smem[smem_bytes<BM, BN>()];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int r16 = lane & 15, q = lane >> 4;

  // XCD-aware tile order: blocks b and b+8 share an XCD; give each XCD a
  // contiguous run of tiles so neighbouring tiles (same A rows) share its L2.
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int wg = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int nt = wg % g.ntiles, mt = wg / g.ntiles;
  const int m0 = mt * BM, n0 = nt * BN;

  int pad_h = g.pad_h, pad_w = g.pad_w, oy_off = 0, ox_off = 0, osc = 1;
  const T* __restrict__ wp = reinterpret_cast<const T*>(g.w);
  if (g.deconv) {
    const int cls = blockIdx.z, py = cls >> 1, px = cls & 1;
    pad_h = 1 - py;
    pad_w = 1 - px;
    oy_off = py;
    ox_off = px;
    osc = 2;
    wp += static_cast<size_t>(cls) * g.CoutPad * g.Kpad;
  }
  const T* __restrict__ xp = reinterpret_cast<const T*>(g.x);

  // ---- per-thread A rows (pixel decode once)
  const int cA = tid & 7;
  int hb[RA], wb[RA], nb[RA];
  const int HoWo = g.Ho * g.Wo;
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    if (m < g.M) {
      const int n = m / HoWo, rem = m - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      hb[i] = oy * g.stride - pad_h;
      wb[i] = ox * g.stride - pad_w;
      nb[i] = n * g.H * g.W * g.C;
    } else {
      hb[i] = -(1 << 28);
      wb[i] = 0;
      nb[i] = 0;
    }
  }
  const bool tap_uniform = (g.C % BK) == 0;
  const int nk = g.Kpad / BK;

  // Out-of-window taps read through a buffer descriptor at an offset past
  // num_records: the hardware returns zeros, so the gather needs no branches.
  const __amdgpu_buffer_rsrc_t xrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<T*>(xp), static_cast<short>(0), g.N * g.H * g.W * g.C * static_cast<int>(sizeof(T)),
      0x00020000);
  constexpr int OOB = 0x7ffffff0;

  uint4 ra[RA], rb[RB];
  // global -> registers for K-tile KT (macro, so the staging arrays stay in VGPRs)
#define POSU_LOAD_TILE(KT)                                                                          \
  {                                                                                                 \
    const int kbase = (KT) * BK;                                                                    \
    int kh, kw, ci;                                                                                 \
    bool kvalid;                                                                                    \
    if (tap_uniform) {                                                                              \
      const int tap = kbase >> g.logC;                                                              \
      kh = tap / g.KW;                                                                              \
      kw = tap - kh * g.KW;                                                                         \
      ci = (kbase & (g.C - 1)) + cA * E;                                                            \
      kvalid = true;                                                                                \
    } else {                                                                                        \
      const int k = kbase + cA * E;                                                                 \
      const int tap = k >> g.logC;                                                                  \
      kh = tap / g.KW;                                                                              \
      kw = tap - kh * g.KW;                                                                         \
      ci = k & (g.C - 1);                                                                           \
      kvalid = k < g.K;                                                                             \
    }                                                                                               \
    _Pragma("unroll") for (int i = 0; i < RA; ++i) {                                                \
      const int hi = hb[i] + kh, wi = wb[i] + kw;                                                   \
      const bool ok = kvalid && static_cast<unsigned>(hi) < static_cast<unsigned>(g.H) &&           \
                      static_cast<unsigned>(wi) < static_cast<unsigned>(g.W);                       \
      const int off = ok ? (nb[i] + (hi * g.W + wi) * g.C + ci) * static_cast<int>(sizeof(T)) : OOB; \
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);                         \
      ra[i] = make_uint4(t[0], t[1], t[2], t[3]);                                                   \
    }                                                                                               \
    _Pragma("unroll") for (int i = 0; i < RB; ++i) {                                                \
      const int nrow = n0 + (tid >> 3) + 32 * i;                                                    \
      rb[i] = *reinterpret_cast<const uint4*>(wp + static_cast<size_t>(nrow) * g.Kpad + kbase + cA * E); \
    }                                                                                               \
  }
#define POSU_STORE_TILE(BUF)                                                                        \
  {                                                                                                 \
    char* As_ = smem + (BUF) * STAGE;                                                               \
    char* Bs_ = As_ + A_BYTES;                                                                      \
    _Pragma("unroll") for (int i = 0; i < RA; ++i)                                                  \
      *reinterpret_cast<uint4*>(As_ + swz((tid >> 3) + 32 * i, cA)) = ra[i];                        \
    _Pragma("unroll") for (int i = 0; i < RB; ++i)                                                  \
      *reinterpret_cast<uint4*>(Bs_ + swz((tid >> 3) + 32 * i, cA)) = rb[i];                        \
  }
  // MFMAs over one LDS K-tile
#define POSU_COMPUTE(BUF)                                                                           \
  {                                                                                                 \
    const char* As_ = smem + (BUF) * STAGE;                                                         \
    const char* Bs_ = As_ + A_BYTES;                                                                \
    _Pragma("unroll") for (int cb = 0; cb < 2; ++cb) {                                              \
      const int c = 4 * cb + q;                                                                     \
      uint4 af[TM], bfr[TN];                                                                        \
      _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                \
        af[i] = *reinterpret_cast<const uint4*>(As_ + swz(wm * WTM + i * 16 + r16, c));             \
      _Pragma("unroll") for (int j = 0; j < TN; ++j)                                                \
        bfr[j] = *reinterpret_cast<const uint4*>(Bs_ + swz(wn * WTN + j * 16 + r16, c));            \
      _Pragma("unroll") for (int i = 0; i < TM; ++i)                                                \
        _Pragma("unroll") for (int j = 0; j < TN; ++j) O::mma(acc[i][j], af[i], bfr[j]);            \
    }                                                                                               \
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  POSU_LOAD_TILE(0);
  POSU_STORE_TILE(0);
  __syncthreads();
  for (int kt = 0; kt + 1 < nk; ++kt) {
    const int cur = kt & 1;
    POSU_LOAD_TILE(kt + 1);
    POSU_COMPUTE(cur);
    POSU_STORE_TILE(cur ^ 1);
    __syncthreads();
  }
  POSU_COMPUTE((nk - 1) & 1);
  __syncthreads();

  // ---- epilogue: stage the f32 tile in LDS (after the barrier above)
  constexpr int LD = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = wn * WTN + j * 16 + r16;
    const int co = n0 + col;
    float sc = 1.f, sh = 0.f;
    if (co < g.Cout) {
      if (g.scale) sc = g.scale[co];
      if (g.shift) sh = g.shift[co];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * WTM + i * 16 + q * 4 + e;
        Cs[row * LD + col] = acc[i][j][e] * sc + sh;
      }
  }
  __syncthreads();

  if (g.mode == 0) {
    constexpr int CPR = BN / E;  // output chunks per row
    T* __restrict__ yp = reinterpret_cast<T*>(g.y);
    const T* __restrict__ rp = reinterpret_cast<const T*>(g.res);
    for (int idx = tid; idx < BM * CPR; idx += 256) {
      const int row = idx / CPR, cc = idx - row * CPR;
      const int m = m0 + row, co = n0 + cc * E;
      if (m >= g.M || co >= g.Cout) continue;
      const int n = m / HoWo, rem = m - n * HoWo;
      const int oy = rem / g.Wo, ox = rem - oy * g.Wo;
      const size_t off =
          (static_cast<size_t>(n * g.out_H + oy * osc + oy_off) * g.out_W + (ox * osc + ox_off)) * g.Cout + co;
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
        O::load_vals(*reinterpret_cast<const uint4*>(rp + off), r);
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] += r[e];
      }
      if (g.relu) {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      *reinterpret_cast<uint4*>(yp + off) = O::store_vals(v);
    }
  } else {
    // NCHW f32 (heatmap head): consecutive threads walk pixels of one channel
    float* __restrict__ yp = reinterpret_cast<float*>(g.y);
    const int ncol = min(BN, g.Cout - n0);
    for (int idx = tid; idx < BM * ncol; idx += 256) {
      const int col = idx / BM, row = idx - col * BM;
      const int m = m0 + row;
      if (m >= g.M) continue;
      const int n = m / HoWo, pix = m - n * HoWo;
      float v = Cs[row * LD + col];
      if (g.relu) v = fmaxf(v, 0.f);
      yp[(static_cast<size_t>(n) * g.Cout + n0 + col) * HoWo + pix] = v;
    }
  }
#undef POSU_LOAD_TILE
#undef POSU_STORE_TILE
#undef POSU_COMPUTE
}

int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return ((1 << l) == v) ? l : -1;
}

template <typename T>
int launch(ConvGeom g, int nclass, hipStream_t s, const char* what) {
  const bool wide = g.CoutPad % 128 == 0;
  constexpr int BM = 128;
  const int BN = wide ? 128 : 64;
  g.mtiles = (g.M + BM - 1) / BM;
  g.ntiles = g.CoutPad / BN;
  dim3 grid(g.mtiles * g.ntiles, 1, nclass);
  if (wide)
    hipLaunchKernelGGL((conv_igemm_kernel<T, BM, 128>), grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((conv_igemm_kernel<T, BM, 64>), grid, dim3(256), 0, s, g);
  return check_launch(what);
}

int dispatch(int dtype, ConvGeom& g, int nclass, void* stream, const char* what) {
  hipStream_t s = as_stream(stream);
  if (dtype == POSU_BF16) return launch<uint16_t>(g, nclass, s, what);
  if (dtype == POSU_F32) return launch<float>(g, nclass, s, what);
  set_error(std::string(what) + ": unsupported dtype");
  return POSU_ERR_ARG;
}

int bk_of(int dtype) { return dtype == POSU_F32 ? 32 : 64; }

int common_checks(int dtype, const void* x, const void* w, const void* y, int N, int H, int W, int C,
                  int Cout, const char* what) {
  POSU_REQUIRE(dtype == POSU_BF16 || dtype == POSU_F32, std::string(what) + ": dtype must be F32 or BF16");
  POSU_REQUIRE(x && w && y, std::string(what) + ": null pointer");
  POSU_REQUIRE(N > 0 && H > 0 && W > 0 && Cout > 0, std::string(what) + ": empty shape");
  POSU_REQUIRE(C >= 8 && ilog2(C) >= 0, std::string(what) + ": C must be a power of two >= 8");
  const long long esz = dtype == POSU_F32 ? 4 : 2;
  POSU_REQUIRE(static_cast<long long>(N) * H * W * C * esz < (1LL << 31) - 256,
               std::string(what) + ": input exceeds the 2 GiB buffer-descriptor range");
  return POSU_OK;
}

}  // namespace
}  // namespace posu

using namespace posu;

extern "C" int posu_conv_bk(int dtype) { return bk_of(dtype); }

extern "C" int posu_conv2d_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w, int Cout,
                               int KH, int KW, int stride, int pad, const float* scale, const float* shift,
                               const void* residual, int relu, void* y, int Ho, int Wo, void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_conv2d_fwd")) return st;
  const int E = dtype == POSU_F32 ? 4 : 8;
  POSU_REQUIRE(Cout % E == 0, "posu_conv2d_fwd: Cout must be a multiple of 16 bytes");
  POSU_REQUIRE(KH > 0 && KW > 0 && stride > 0 && pad >= 0, "posu_conv2d_fwd: bad window");
  POSU_REQUIRE(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1,
               "posu_conv2d_fwd: Ho/Wo inconsistent with the window");
  POSU_REQUIRE(static_cast<long long>(N) * Ho * Wo * Cout < (1LL << 31), "posu_conv2d_fwd: output too large");
  ConvGeom g{};
  g.x = x;
  g.w = w;
  g.scale = scale;
  g.shift = shift;
  g.res = residual;
  g.y = y;
  g.N = N;
  g.H = H;
  g.W = W;
  g.C = C;
  g.logC = ilog2(C);
  g.Ho = Ho;
  g.Wo = Wo;
  g.M = N * Ho * Wo;
  g.Cout = Cout;
  g.CoutPad = round_up(Cout, 64);
  g.K = KH * KW * C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = KH;
  g.KW = KW;
  g.stride = stride;
  g.pad_h = pad;
  g.pad_w = pad;
  g.relu = relu;
  g.deconv = 0;
  g.out_H = Ho;
  g.out_W = Wo;
  g.mode = 0;
  return dispatch(dtype, g, 1, stream, "posu_conv2d_fwd");
}

extern "C" int posu_deconv4x4s2_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w,
                                    int Cout, const float* scale, const float* shift, int relu, void* y,
                                    void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_deconv4x4s2_fwd")) return st;
  const int E = dtype == POSU_F32 ? 4 : 8;
  POSU_REQUIRE(Cout % E == 0, "posu_deconv4x4s2_fwd: Cout must be a multiple of 16 bytes");
  POSU_REQUIRE(static_cast<long long>(N) * 4 * H * W * Cout < (1LL << 31),
               "posu_deconv4x4s2_fwd: output too large");
  ConvGeom g{};
  g.x = x;
  g.w = w;
  g.scale = scale;
  g.shift = shift;
  g.res = nullptr;
  g.y = y;
  g.N = N;
  g.H = H;
  g.W = W;
  g.C = C;
  g.logC = ilog2(C);
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.Cout = Cout;
  g.CoutPad = round_up(Cout, 64);
  g.K = 4 * C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = 2;
  g.KW = 2;
  g.stride = 1;
  g.relu = relu;
  g.deconv = 1;
  g.out_H = 2 * H;
  g.out_W = 2 * W;
  g.mode = 0;
  return dispatch(dtype, g, 4, stream, "posu_deconv4x4s2_fwd");
}

extern "C" int posu_head1x1_nchw_fwd(int dtype, const void* x, int N, int H, int W, int C, const void* w,
                                     int Cout, const float* bias, float* y, void* stream) {
  if (int st = common_checks(dtype, x, w, y, N, H, W, C, Cout, "posu_head1x1_nchw_fwd")) return st;
  ConvGeom g{};
  g.x = x;
  g.w = w;
  g.scale = nullptr;
  g.shift = bias;
  g.res = nullptr;
  g.y = y;
  g.N = N;
  g.H = H;
  g.W = W;
  g.C = C;
  g.logC = ilog2(C);
  g.Ho = H;
  g.Wo = W;
  g.M = N * H * W;
  g.Cout = Cout;
  g.CoutPad = round_up(Cout, 64);
  g.K = C;
  g.Kpad = round_up(g.K, bk_of(dtype));
  g.KH = 1;
  g.KW = 1;
  g.stride = 1;
  g.relu = 0;
  g.deconv = 0;
  g.out_H = H;
  g.out_W = W;
  g.mode = 1;
  return dispatch(dtype, g, 1, stream, "posu_head1x1_nchw_fwd");
}
