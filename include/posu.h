/*
 * posu.h — C ABI of libposeu.so, the MI355X (gfx950) kernels behind the
 * pose-unsupervised hot path:
 *
 *   PoseResNet forward (ResNet-18..152 backbone + 3x ConvTranspose head)
 *     -> heatmap soft-argmax / argmax decoding (+ crop affine back to image px)
 *     -> epipolar (fundamental-matrix) consistency loss
 *     -> multi-view DLT triangulation.
 *
 * The reference (LouisNUST/pose-unsupervised) is pure Python/PyTorch; these
 * entry points replace the framework ops its Python functions call.  Each
 * declaration cites the reference interface it replaces (file:line relative to
 * the reference repo root).
 *
 * Conventions (all entry points):
 *   - Every tensor argument is a caller-owned DEVICE pointer (e.g. from
 *     torch.Tensor.data_ptr()).  Shapes are explicit ints; layouts are stated.
 *   - `stream` is a hipStream_t passed as void* (PyTorch's current stream).
 *     Calls only enqueue work; none synchronises, allocates or frees, so every
 *     call is hipGraph-capturable.
 *   - Return value: 0 (POSU_OK) or a POSU_ERR_* code; posu_last_error() then
 *     returns a thread-local message.
 *   - dtype codes: POSU_F32 (fp32 operands, exact-f32 MFMA, the parity mode)
 *                  POSU_BF16 (bf16 operands, f32 accumulate, the fast mode),
 *                  POSU_F16  (IEEE fp16 operands, f32 accumulate: BASELINE configs[4]'s
 *                             fp16 backbone; same kernels and speed as bf16),
 *                  POSU_F16X3 (ABI 13, split fp16: the parity-bearing fast mode).  Every value
 *                             is stored as a pair hi = fp16(v), lo = fp16(v - hi) -- v to ~22
 *                             mantissa bits -- and every product is summed as hi.hi + lo.hi +
 *                             hi.lo (three fp16 MFMAs, f32 accumulate; the lo.lo term dropped).
 *                             Split layout of a tensor of C logical channels (C % 32 == 0): 2C
 *                             fp16 per pixel, logical channel c's hi at (c / 32) * 64 + c % 32
 *                             and its lo 32 elements later ([hi 32 | lo 32] per 32-channel
 *                             block).  Entry points that accept it take LOGICAL channel counts;
 *                             packed weights use the same interleave along K (k = tap * C + ci
 *                             logical, then split per 32-block), so posu_conv_bk = 64 halves =
 *                             32 logical k per K-tile.
 */
#ifndef POSU_H_
#define POSU_H_

#ifdef __cplusplus
extern "C" {
#endif

#define POSU_OK 0
#define POSU_ERR_ARG 1          /* invalid shape / pointer / unsupported config */
#define POSU_ERR_HIP 2          /* a HIP launch failed */

#define POSU_F32 0
#define POSU_BF16 1
#define POSU_F64 2
#define POSU_F16 3
#define POSU_F16X3 4

/* ---------------------------------------------------------------- runtime */
const char* posu_last_error(void);
/* ABI revision: 4 stateless conv knobs; 5 the fused layer1 Bottleneck kernels and batched
 * weight packing; 6 the LDS-tiled packing; 7 the layer3 Bottleneck tail; 8 the crop warp
 * (posu_crop_warp); 9 the chained streamed tail (posu_bottleneck_tail_stream_next_fwd); 10 the
 * BatchNorm statistics in the conv epilogue (measured slower, removed in 11); 11 the streamed
 * tails take their weight stream's byte size, the round-2 LDS-ring layer2 block / layer3 tail
 * kernels removed, the strided tail of layer2's first block (posu_bottleneck_s2_tail_fwd) the
 * one-launch multi-view stem (posu_stem_pool_views_fwd) added, the fused deconv+head takes an
 * optional split-precision head (hw_lo); 12 the chained strided tail
 * (posu_bottleneck_s2_tail_next_fwd); 13 the split-fp16 dtype POSU_F16X3 (conv / dual / deconv /
 * deconv+head / head / pack / s2d pack / max-pool / unpack entry points); 14 (training) the ReLU
 * bit mask (posu_bn_apply_mask / posu_bn_train_bwd_mask) and the fused stem BN + ReLU + max-pool
 * with stored argmax taps (posu_bn_relu_maxpool3x3s2_fwd / posu_maxpool3x3s2_bwd_idx), the training
 * stem's convolution and weight gradient from the NCHW f32 views (posu_stem_conv_views_fwd /
 * posu_stem_wgrad_views); 15 (training) the data gradient on a chosen tile
 * (posu_conv2d_dgrad_tile: the training step autotunes it like the forward convolutions), 3x3
 * sources of the batched deconv packing (the strided 3x3 convs' sub-pixel data gradient), the
 * Adam step (posu_adam_step); 16 (round 6) the split-fp16 dtype in the streamed Bottleneck tails
 * (posu_bottleneck_tail_stream_fwd / _next_fwd, layer1 / layer2 / layer3 at 256x256) and the
 * downsampling first-block tail (posu_bottleneck_down_tail_stream_fwd).  The
 * ctypes binding refuses a library of another revision. */
int posu_abi_version(void);

/* ------------------------------------------------------------ input prep */
/* NCHW fp32 image batch -> NHWC activations with Cpad (>= C) channels,
 * zero-filled above C.  Replaces the implicit layout of the first
 * nn.Conv2d call in PoseResNet.forward (lib/models/pose_resnet.py:192).
 * x: [N, C, H, W] f32.  y: [N, H, W, Cpad] of `dtype`.  hflip != 0 reads the
 * image mirrored along W (the flip test's torch.flip(view, dims=[3]),
 * lib/core/function.py:569). */
int posu_pack_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W,
                           void* y, int Cpad, int hflip, void* stream);

/* NCHW fp32 -> space-to-depth NHWC for the stem: y[n][i][j][(dy*2+dx)*C + c] =
 * x[n][c][2i+dy][2j+dx], zero above 4C.  The 7x7/s2/p3 stem conv then runs as a
 * 4x4/s1 conv with top/left padding 2 over this grid (K = 16 * Cpad instead of
 * 49 * Cpad taps of a Cin-padded 7x7 window).  H, W even; y: [N, H/2, W/2, Cpad];
 * hflip as above. */
int posu_pack_s2d_nchw(int dtype, const float* x, int N, int C, int H, int W,
                       void* y, int Cpad, int hflip, void* stream);

/* Batched weight packing (training: the parameters change every optimizer step).  One
 * launch packs every job of a device-resident table: fp32 PyTorch weights -> the layouts the
 * conv kernels read, in `dtype` (replaces per-layer torch packing; the modes restate
 * lib/posu/packing.py):
 *   POSU_PACK_CONV:   Conv2d [cout][cin][kh][kw] -> [rows][kpad], k = tap * pitch + ci
 *                     (posu_conv2d_fwd's w; pitch = the channel stride of the packed K);
 *   POSU_PACK_DGRAD:  the same weight flipped and transposed -> [rows >= cin][kpad],
 *                     k = tap * pitch + co, value w[co][ci][kh-1-th][kw-1-tw] (co < cout only;
 *                     posu_conv2d_dgrad's weight);
 *   POSU_PACK_DECONV: ConvTranspose2d [cin][cout][4][4] -> [4 classes][rows][kpad],
 *                     k = (ty*2 + tx) * cin + ci (posu_deconv4x4s2_fwd's w).  ABI 15: also a
 *                     [cin][cout][3][3] source (kh = kw = 3), read as its 4x4 zero-padding (tap
 *                     index 3 = 0) -- a Conv2d(3, s2, p1) weight [co][ci][3][3] packed this way
 *                     makes posu_deconv4x4s2_fwd the conv's data gradient (even H, W).
 * Zero outside the source.  block_start: the job's first block; blocks per job =
 * posu_pack_job_blocks(the job's mode .. kpad fields) (-1: kpad not a multiple of 8, a
 * deconv other than 4x4 / 3x3, or a non-positive size); total_blocks = their sum. */
#define POSU_PACK_CONV 0
#define POSU_PACK_DGRAD 1
#define POSU_PACK_DECONV 2
typedef struct posu_pack_job {
  const float* src;
  void* dst;
  long long block_start;
  int mode, cout, cin, kh, kw, pitch, rows, kpad;
} posu_pack_job;
long long posu_pack_job_blocks(int mode, int cout, int cin, int kh, int kw, int pitch, int rows, int kpad);
int posu_pack_weights(int dtype, const posu_pack_job* jobs, int njobs, long long total_blocks, void* stream);

/* NHWC activations -> NCHW fp32 (for returning x1 / f in the reference
 * layout: lib/models/pose_resnet.py:205). */
int posu_nhwc_to_nchw_f32(int dtype, const void* x, int N, int H, int W, int C,
                          float* y, void* stream);

/* ---------------------------------------------------------- convolutions */
/* Implicit-GEMM convolution on MFMA (NHWC), fused eval-mode BatchNorm
 * (per-channel scale/shift), optional residual add and ReLU:
 *     y = act( conv(x, w) * scale[co] + shift[co] + residual )
 * Replaces nn.Conv2d + nn.BatchNorm2d (+ `out += residual`) + nn.ReLU in
 * Bottleneck.forward / BasicBlock.forward (lib/models/pose_resnet.py:42-58,
 * 79-99), the stem (pose_resnet.py:192-194) and the downsample branch
 * (pose_resnet.py:136-141).
 *   x: [N, H, W, C] dtype, C % 8 == 0.
 *   w: packed [CoutPad][Kpad] dtype, k = (kh*KW + kw)*C + ci, zero padded;
 *      CoutPad = round_up(Cout, 64), Kpad = round_up(KH*KW*C, posu_conv_bk(dtype)).
 *   scale/shift: [Cout] f32 (may be NULL: scale 1, shift 0), 16-byte aligned (here and
 *   in posu_conv1x1_dual_fwd / posu_deconv4x4s2_fwd / posu_deconv4x4s2_head_fwd).
 *   residual: NULL or [N, Ho, Wo, Cout] dtype.
 *   y: [N, Ho, Wo, Cout] dtype.  `pad` is the top/left padding; Ho/Wo may be
 *   smaller than (H + 2 pad - KH) / stride + 1 (bottom/right padding implied).
 *   tile (here and in posu_conv1x1_dual_fwd / posu_deconv4x4s2_fwd): -1 = the
 *   built-in heuristic, else a fixed tile configuration cfg + 8 * variant:
 *     cfg 0: 256x64, 1: 128x64, 2: 64x64, 3: 128x128, 4: 64x128 (four waves),
 *         5: 256x256, 6: 256x128 (eight waves);
 *     variant 1: single-slot LDS ring (cfg 0-4), 2: three-slot ring (cfg != 5);
 *     + 32 (bf16 / f16): the persistent K-tile stream;
 *     23 / 31 (bf16 / f16): 256x256 / 256x128 with waves 4-7 staggered by half a K-tile;
 *     7 / 15 (bf16 / f16, ABI 11): 128x128 with eight staggered waves (2x4 / 4x2 wave grids);
 *     39 (bf16 / f16, ABI 13, NHWC outputs): 128x128 with two K groups of four waves (each group
 *        sums every other K-tile over the whole tile, the halves added in LDS at the end: a
 *        different K order, so not bit-identical to the other tiles);
 *     split fp16 (POSU_F16X3): 7 / 15 unstaggered; 31 (ABI 16) staggered, the lagging waves holding a
 *        K-tile's third product hi(w).lo(x) across the barrier; 47 / 55 (ABI 16) the staggered
 *        128x128 eight-wave tiles (2x4 / 4x2 wave grids).
 *   The tile only changes speed (every configuration but 39 computes the same sums in the same
 *   K order); the Python plan picks it per layer by timing every admissible
 *   configuration once (PoseResNetPlan.autotune).  The library keeps no mutable state:
 *   every knob is an argument. */
int posu_conv_bk(int dtype);
/* Fused stem (replaces lib/models/pose_resnet.py:192-195, conv1 -> bn1 -> relu ->
 * maxpool, and the input pack): x NCHW f32 [N, 3, H, W] (the reference's input tensor,
 * mirrored along W when hflip), w packed [64][224] dtype (k = kh*32 + kw*4 + c, zero for
 * kw = 7 / c = 3; posu/packing.py:pack_stem_fused_weight), BN scale/shift [64] f32,
 * y NHWC [N, H/4, W/4, 64] dtype.  BF16 / F16, H % 8 == 0, W in {256, 384}; F16X3 (ABI 13, W = 256):
 * w = the hi plane [64][224] followed by the lo plane [64][224] of the weights (scaled by the
 * caller's power of two, undone in `scale`), the input split into (hi, lo) fp16 as it is staged,
 * three MFMAs per kernel row, y split [N, H/4, W/4, 128]. */
int posu_stem_pool_fwd(int dtype, const float* x, int N, int H, int W, int hflip, const void* w,
                       const float* scale, const float* shift, void* y, void* stream);
/* posu_stem_pool_fwd over the views of one forward in ONE launch (lib/models/multiview_pose_resnet.py
 * runs the backbone per view; the stem needs no per-view statistics in eval mode): views = host
 * array of nviews (1..8) device pointers to [Nv, 3, H, W] f32, y = [nviews * Nv, H/4, W/4, 64]
 * view-major.  Same values as nviews posu_stem_pool_fwd launches. */
int posu_stem_pool_views_fwd(int dtype, const float* const* views, int nviews, int Nv, int H, int W, int hflip,
                             const void* w, const float* scale, const float* shift, void* y, void* stream);
int posu_conv2d_fwd(int dtype, const void* x, int N, int H, int W, int C,
                    const void* w, int Cout, int KH, int KW, int stride, int pad,
                    const float* scale, const float* shift, const void* residual,
                    int relu, void* y, int Ho, int Wo, int tile, void* stream);

/* Two 1x1 convolutions summed into one output (Bottleneck conv3/bn3 + the
 * downsample conv/bn residual branch, lib/models/pose_resnet.py:90-99, 136-141):
 *   y[n,i,j,:] = act( W[:, :C] x[n,i,j,:] + W[:, C:] x2[n, i*stride2, j*stride2, :]
 *                     * scale + shift )
 * with the two BN scales pre-multiplied into W by the caller.
 *   x: [N, H, W, C]; x2: [N, H2, W2, C2]; C, C2 multiples of posu_conv_bk(dtype);
 *   w: [CoutPad][C + C2]; y: [N, H, W, Cout]. */
int posu_conv1x1_dual_fwd(int dtype, const void* x, int N, int H, int W, int C,
                          const void* x2, int H2, int W2, int C2, int stride2,
                          const void* w, int Cout, const float* scale, const float* shift,
                          int relu, void* y, int tile, void* stream);

/* ConvTranspose2d(kernel 4, stride 2, padding 1, output_padding 0) as four
 * stride-1 2x2 sub-pixel convolutions (one per output parity class) in one
 * launch, + fused BN + ReLU.  Replaces _make_deconv_layer's
 * ConvTranspose2d/BatchNorm2d/ReLU triples (lib/models/pose_resnet.py:164-189).
 *   x: [N, H, W, C] dtype.
 *   w: packed [4 classes][CoutPad][Kpad] dtype (see posu_pack_deconv4x4 in
 *      the Python layer), class = py*2 + px, k = (ty*2 + tx)*C + ci.
 *   y: [N, 2H, 2W, Cout] dtype. */
int posu_deconv4x4s2_fwd(int dtype, const void* x, int N, int H, int W, int C,
                         const void* w, int Cout, const float* scale,
                         const float* shift, int relu, void* y, int tile, void* stream);

/* Fused Bottleneck block, eval mode (lib/models/pose_resnet.py:61-99 with the BNs folded):
 *   y = relu( conv3(relu(conv2_3x3(relu(conv1(x) * s1 + b1)) * s2 + b2)) * s3 + b3 + x )
 * in one launch that streams each image's rows once: the two planes-wide intermediates stay
 * in LDS / registers, x is read from HBM once (conv1 input and residual) and y written
 * once.  Identity residual (no downsample), stride 1.  Built for layer1 of PoseResNet at
 * 256x256: W = 64, C = 256, P = 64; dtype BF16 / F16.
 *   x, y: [N, H, W, C] (y must not alias x);
 *   w1: [P][C] with the input channels permuted: column 32 s + 8 q + e holds channel
 *       32 s + 16 (q & 1) + 8 (q >> 1) + e, s1/b1 [P] f32;
 *   w2: [P][9 * P] (posu_conv2d_fwd packing of conv2, k = (kh * 3 + kw) * P + ci), s2/b2 [P];
 *   w3: [C][P] with the input channels of every 32-block permuted: column 32 b + 8 q + e
 *       holds input channel 32 b + 16 (e >> 2) + 4 q + (e & 3) (the order in which conv2's
 *       accumulators become conv3's MFMA operand), s3/b3 [C]. */
int posu_bottleneck_fwd(int dtype, const void* x, int N, int H, int W, int C, int P, const void* w1,
                        const float* s1, const float* b1, const void* w2, const float* s2,
                        const float* b2, const void* w3, const float* s3, const float* b3, void* y,
                        void* stream);

/* The tail of an identity Bottleneck of layer2 (W = 32, C = 512, P = 128) or layer3 (W = 16,
 * C = 1024, P = 256) (lib/models/pose_resnet.py:79-99) with the weights streamed from L2
 * straight into registers (each wave loads its own 2 n-tiles' MFMA fragments a few k-steps
 * ahead; no LDS weight ring): conv2 3x3 + BN2 + ReLU -> conv3 1x1 + BN3 + residual + ReLU.
 * t1 [N, H, W, P] (conv1 output), x [N, H, W, C], y [N, H, W, C], H a multiple of 8.
 * wstream: packing.pack_tail_stream of the conv2 [P][9P] and conv3 [C][P] posu_conv2d_fwd packs,
 * [P/32][9 P/32 + C/32][2][64][8] elements of dtype; wstream_bytes = its size in bytes (checked
 * against what the kernel reads: a pack for another layer or the chained variant's pack is
 * refused, never read past).  Bit-identical to posu_conv2d_fwd(conv2) followed by
 * posu_conv2d_fwd(conv3, residual). */
int posu_bottleneck_tail_stream_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                    int P, const void* wstream, long long wstream_bytes, const float* s2,
                                    const float* b2, const float* s3, const float* b3, void* y, void* stream);

/* posu_bottleneck_tail_stream_fwd chained with the NEXT identity Bottleneck's conv1 (1x1, C -> P)
 * + BN1 + ReLU over this block's output y (lib/models/pose_resnet.py:79-84 of block i+1; the
 * reference runs it as a separate conv over y): each y chunk of P channels is staged in LDS as
 * it is produced and multiplied into the next conv1's accumulators, so y is not re-read and the
 * next block's conv1 launch disappears.  wstream: packing.pack_tail_stream(conv2, conv3, next
 * conv1 [P][C] pack) -- [P/32][9 P/32 + 2 C/32][2][64][8]; s1n/b1n [P] the next conv1's folded
 * BN; t1n [N, H, W, P] out (aliasing no other operand).  y and t1n are bit-identical to this
 * tail followed by posu_conv2d_fwd(next conv1, ReLU) over y. */
int posu_bottleneck_tail_stream_next_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                         int P, const void* wstream, long long wstream_bytes, const float* s2,
                                         const float* b2, const float* s3, const float* b3, void* y,
                                         const float* s1n, const float* b1n, void* t1n, void* stream);

/* (ABI 16) Both tails above also take POSU_F16X3 (split fp16 pairs, [N, H, W, 2 C] storage, C and P
 * logical), at layer1 (W = 64, C = 256, P = 64; 2-row tiles), layer2 (W = 32; 2-row tiles) and
 * layer3 (W = 16; 4-row tiles) of PoseResNet at 256x256: every k-step pair multiplied as hi.hi +
 * lo(w).hi(x) + hi(w).lo(x), bit-identical to the split posu_conv2d_fwd launches they replace;
 * wstream = packing.pack_tail_stream of the split packs (K' = 2 K).
 *
 * The FIRST Bottleneck of layer1 (lib/models/pose_resnet.py:61-99 with its stride-1 downsample,
 * pose_resnet.py:136-141; eval BN folded), split fp16 only: conv2 + the [conv3 | downsample] dual
 * GEMM + ReLU in one launch,
 *   y = relu( [w3*s3 | wd*sd] . [ relu(bn2(conv2_3x3(t1))) ; x ] * s3 + b3 ),
 * = posu_conv2d_fwd(conv2) then posu_conv1x1_dual_fwd(t2, x, stride 1), bit for bit.  t1 [N, H, 64, P]
 * (conv1's output), x [N, H, 64, P] (the block input), y [N, H, 64, C] with C = 256, P = 64
 * (logical channels), H even.  s3 / b3: the dual GEMM's scale (the split weight exponent's 2^-e) and
 * shift (b3 + bd).  s1n / b1n / t1n: optional (all null, or all given) -- the next identity block's
 * conv1 + BN1 + ReLU over y, as posu_bottleneck_tail_stream_next_fwd.  wstream =
 * packing.pack_down_tail_stream(conv2 pack, dual pack[, next conv1 pack]). */
/* (ABI 16) The LAST identity block of a layer chained with the NEXT layer's first conv1 + BN1 + ReLU
 * (1x1 / stride 1 over y, C -> Pn = 2 P at this map size: layer2 / 3 / 4 block 0's conv1,
 * lib/models/pose_resnet.py:79-81) at 256x256: the split fp16 tails of layers 1-3 and the bf16 / fp16 tails of
 * layers 2-3 (their 4-m-tile variants: layer2 2-row, layer3 4-row tiles); Pn = P is
 * posu_bottleneck_tail_stream_next_fwd.  Each y chunk's next-conv1 k-steps run twice, once per half
 * of the Pn outputs (two accumulator sets); t1n [N, H, W, Pn] (logical), s1n / b1n [Pn] f32, wstream =
 * packing.pack_tail_stream(conv2, conv3, next conv1 [Pn][C']).  Bit-identical to the tail followed by
 * posu_conv2d_fwd(next conv1) over y. */
int posu_bottleneck_tail_stream_chain_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                          int P, int Pn, const void* wstream, long long wstream_bytes,
                                          const float* s2, const float* b2, const float* s3, const float* b3,
                                          void* y, const float* s1n, const float* b1n, void* t1n, void* stream);
int posu_bottleneck_down_tail_stream_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C,
                                         int P, const void* wstream, long long wstream_bytes, const float* s2,
                                         const float* b2, const float* s3, const float* b3, void* y,
                                         const float* s1n, const float* b1n, void* t1n, void* stream);

/* The tail of the FIRST Bottleneck of layer2 (lib/models/pose_resnet.py:61-99 with the downsample
 * branch, pose_resnet.py:136-141; eval BN folded) of PoseResNet at 256x256, in one launch:
 *   y = relu( [w3*s3 | wd*sd] . [ relu(bn2(conv2_3x3_stride2(t1))) ; x(2 oy, 2 ox) ] + shift ),
 * i.e. posu_conv2d_fwd(conv2, stride 2) followed by posu_conv1x1_dual_fwd(t2, x, stride 2) with t2
 * kept on chip.  t1 [N, H, 64, 128] (conv1's output), x [N, H, 64, 256] (the block input),
 * y [N, H/2, 32, 512]; H a multiple of 8; BF16 / F16.  s2 / b2: conv2's folded BN [128] f32;
 * shift = b3 + bd [512] f32 (16-B aligned).  wstream: packing.pack_s2_tail_stream of the conv2
 * [128][1152] and dual [512][384] posu_conv2d_fwd / posu_conv1x1_dual_fwd packs,
 * [4][84][2][64][8] elements of dtype; wstream_bytes its size (checked).  Bit-identical to the two
 * launches (same MFMA sequence per accumulator). */
int posu_bottleneck_s2_tail_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C, int P,
                                const void* wstream, long long wstream_bytes, const float* s2, const float* b2,
                                const float* shift, int Cout, void* y, void* stream);

/* The same, chained with the next (identity) Bottleneck's conv1 + BN1 + ReLU (ABI 12), as
 * posu_bottleneck_tail_stream_next_fwd chains the identity tails: while each 128-channel chunk of
 * y is produced, the tail also runs the next block's conv1 over it, and writes
 * t1n = relu(conv1n(y) * s1n + b1n) [N, H/2, 32, 128] -- bit-identical to posu_conv2d_fwd over y
 * (lib/models/pose_resnet.py:79-81 of layer2's block 1), which then has no conv1 launch and y is
 * not re-read for it.  wstream: packing.pack_s2_tail_stream(conv2 pack, dual pack, next conv1
 * pack [128][512]), [4][100][2][64][8]; s1n / b1n the next conv1's folded BN [128] f32 (16-B
 * aligned); t1n must alias no other operand. */
int posu_bottleneck_s2_tail_next_fwd(int dtype, const void* t1, const void* x, int N, int H, int W, int C, int P,
                                     const void* wstream, long long wstream_bytes, const float* s2, const float* b2,
                                     const float* shift, int Cout, void* y, const float* s1n, const float* b1n,
                                     void* t1n, void* stream);

/* The same fused block for the first Bottleneck of layer1 (lib/models/pose_resnet.py:61-99
 * with the downsample branch, pose_resnet.py:136-141): conv3/bn3 and the 1x1 downsample/bn
 * share one accumulator (as in posu_conv1x1_dual_fwd),
 *   y = relu( [w3*s3 | wd*sd] . [t2 ; x] + shift3 ),  t2 = conv2 output as above,
 * x read once (conv1 input and downsample input), y written once.  W = 64, C = P = 64,
 * 4P = 256 output channels; dtype BF16 / F16.
 *   x: [N, H, W, C]; y: [N, H, W, 4P] (must not alias x);
 *   w1: [P][C] (natural channel order), s1/b1 [P]; w2, s2, b2 as posu_bottleneck_fwd;
 *   w3d: [4P][2P]: columns 0..P-1 = conv3 weight * s3 with the posu_bottleneck_fwd column
 *        permutation of w3, columns P..2P-1 = downsample weight * sd (natural order);
 *   shift3: [4P] f32 = b3 + bd. */
int posu_bottleneck_down_fwd(int dtype, const void* x, int N, int H, int W, int C, int P,
                             const void* w1, const float* s1, const float* b1, const void* w2,
                             const float* s2, const float* b2, const void* w3d, const float* shift3,
                             void* y, void* stream);

/* Cross-view Aggregation (multiview_pose_resnet.py:16-58, ChannelWiseFC / Aggregation,
 * NETWORK.AGGRE): the V(V-1) per-pair [HW x HW] matrices form one block matrix with
 * zero diagonal blocks (scaled by 1/(V-1)), so all V aggregated views are ONE GEMM:
 *   posu_pack_view_rows: x[m][o*HW + q] = src[o][m][q]   (src f32 [V][M][HW], M = N*J)
 *   posu_gemm_rows_f32:  out[blk][m][j] = sum_k x[m][k] * wt[blk*vblk + j][k]  (f32,
 *                        view-major output, vblk = HW; wt packed [round_up(Ncol,64)][K])
 * K must be a power of two and a multiple of the K-tile. */
int posu_pack_view_rows(int dtype, const float* src, int V, int M, int HW, void* dst, void* stream);
int posu_gemm_rows_f32(int dtype, const void* x, int M, int K, const void* wt, int Ncol, int vblk,
                       float* out, void* stream);

/* The last deconv stage fused with the final 1x1 head: deconv + BN + ReLU as
 * posu_deconv4x4s2_fwd, then per output pixel hm[n][j][pix] = bias[j] +
 * sum_c hw[j][c] f[c] (lib/models/pose_resnet.py:202-203) from the tile still in LDS,
 * so the 256-channel deconv output need not round-trip through HBM.
 *   y: NULL (do not store f) or [N, 2H, 2W, Cout] dtype; Cout == 256;
 *   hw: packed head weight [>= 16][round_up(Cout, posu_conv_bk)] dtype (rows >= J zero);
 *   hw_lo (ABI 11): NULL, or (BF16 / F16) the head weight's rounding residual w - hw rounded to
 *   the dtype, same layout: the split-precision head -- the deconv output f enters as
 *   round(f) + round(f - round(f)) and the head sums hi.hi + lo.hi + hi.lo products (three MFMAs
 *   per fragment), so the heatmaps carry about twice the dtype's mantissa instead of f's
 *   rounding to the dtype (the largest single source of the 2-byte chains' joint error,
 *   DESIGN.md section 5); f itself is still stored rounded;
 *   hbias: [J] f32; hm: [N, J, 2H, 2W] f32; J <= 16. */
int posu_deconv4x4s2_head_fwd(int dtype, const void* x, int N, int H, int W, int C,
                              const void* w, int Cout, const float* scale, const float* shift,
                              void* y, const void* hw, const void* hw_lo, int J, const float* hbias,
                              float* hm, void* stream);

/* 1x1 convolution (+bias) writing NCHW fp32 heatmaps: PoseResNet.final_layer
 * (lib/models/pose_resnet.py:126-132, 203).
 *   x: [N, H, W, C] dtype; w: packed [CoutPad][Kpad]; bias: [Cout] f32;
 *   y: [N, Cout, H, W] f32. */
int posu_head1x1_nchw_fwd(int dtype, const void* x, int N, int H, int W, int C,
                          const void* w, int Cout, const float* bias, float* y,
                          void* stream);

/* MaxPool2d(3, stride 2, padding 1) on NHWC (lib/models/pose_resnet.py:113,195).
 * y: [N, Ho, Wo, C], Ho = (H - 1) / 2 + 1. */
int posu_maxpool3x3s2_fwd(int dtype, const void* x, int N, int H, int W, int C,
                          void* y, void* stream);

/* ---------------------------------------------------- heatmap -> coords */
/* Soft-argmax (generate_integral_preds_2d_th, lib/utils/transforms.py:149-171):
 *   p = softmax(beta * h) over H*W (beta = 100 in the reference),
 *   x = sum p * col, y = sum p * row,
 * optionally followed by the per-sample crop affine of transform_back_th
 * (lib/utils/transforms.py:174-198): [x, y, 1] @ T^T.
 *   hm: [N, J, H, W] f32 contiguous; affine: NULL or [N, 2, 3] f32;
 *   out: [N, J, 2] f32.  stats: NULL or [N, J, 4] f32 = (max of beta*h,
 *   sum of exp, x, y in heatmap px) kept for the backward pass. */
int posu_softargmax2d_fwd(const float* hm, int N, int J, int H, int W, float beta,
                          const float* affine, float* out, float* stats, void* stream);

/* Gradient of posu_softargmax2d_fwd w.r.t. hm, given gout [N, J, 2]:
 *   dh = beta * p * ((col - x) * gx' + (row - y) * gy'), g' = T_lin^T g.
 * ghm: [N, J, H, W] f32 (overwritten). */
int posu_softargmax2d_bwd(const float* hm, const float* stats, int N, int J, int H, int W,
                          float beta, const float* affine, const float* gout, float* ghm,
                          void* stream);

/* Argmax decoding + quarter-pixel post-process + crop affine back
 * (get_max_preds / get_final_preds, lib/core/inference.py:19-75).
 *   First maximum wins (np.argmax); coords zeroed when maxval <= 0;
 *   post_process != 0 applies the +-0.25 px shift (inference.py:57-66);
 *   affine: NULL or [N, 2, 3] f64 (transform_preds, transforms.py:67-73, which
 *   applies the cv2 float64 matrix in float64 before storing float32).
 *   preds: [N, J, 2] f32; maxvals: [N, J] f32. */
int posu_argmax2d_fwd(const float* hm, int N, int J, int H, int W, int post_process,
                      const double* affine, float* preds, float* maxvals, void* stream);

/* Per-sample 2-D affine of joint coordinates (transform_back_th's
 * `[x, y, 1] @ T^T`, lib/utils/transforms.py:190-195):
 *   transpose == 0: out = [x, y, 1] @ T^T            (forward)
 *   transpose == 1: out = g @ T[:, :, 0:2]            (its gradient w.r.t. pts)
 *   pts: [N, J, 2] f32; T: [N, 2, 3] f32; out: [N, J, 2] f32. */
int posu_affine2d_apply(const float* pts, const float* T, int N, int J, int transpose,
                        float* out, void* stream);

/* Weighted heatmap MSE (JointsMSELoss.forward, lib/core/loss.py:70-86):
 *   loss = sum_j mean_{n,p} (pred*w_nj - gt*w_nj)^2 = sum_{n,j,p} (w (pred-gt))^2 / (N*HW)
 *   pred, gt: [N, J, HW] f32; w: NULL (use_target_weight False) or [N, J] f32;
 *   ws: workspace [N*J] f32 (per-map partial sums, fixed-order final sum);
 *   loss: [1] f32. */
int posu_joints_mse_fwd(const float* pred, const float* gt, const float* w, int N, int J, int HW,
                        float* ws, float* loss, void* stream);

/* Gradient of posu_joints_mse_fwd w.r.t. pred given gloss [1] (device):
 *   gpred = gloss * 2 w^2 (pred - gt) / (N*HW).  gpred: [N, J, HW] f32. */
int posu_joints_mse_bwd(const float* pred, const float* gt, const float* w, int N, int J, int HW,
                        const float* gloss, float* gpred, void* stream);

/* Flip test (lib/core/function.py:566-583): heatmaps of the mirrored input brought
 * back -- W mirrored, joint channels permuted by the dataset's flip pairs
 * (flip_back_th, lib/utils/transforms.py:33-47), optionally shifted right by one
 * column (SHIFT_HEATMAP, function.py:579-582) -- and, when hm is non-NULL, averaged
 * with the plain heatmaps: out = 0.5 * (hm + flip_back(hm_flipped)).
 *   hm_flipped, hm, out: [N, J, H, W] f32 (out may alias hm); perm: NULL or [J] int32
 *   device array, perm[j] = the joint whose flipped map becomes joint j. */
int posu_flip_back(const float* hm_flipped, const int* perm, const float* hm, int N, int J,
                   int H, int W, int shift, float* out, void* stream);

/* ------------------------------------------------------------ data path */
/* The crop of JointsDatasetCompatible.__getitem__ (lib/dataset/joints_dataset_compatible.py
 * :161-172): per sample, cv2.warpAffine(img, trans, (dw, dh), flags=INTER_LINEAR) with the
 * default constant-0 border, computed as OpenCV 3.4 does (the matrix inverted in double,
 * coordinates in 1/1024-px fixed point rounded half to even, 1/32-px bilinear weights, 15-bit
 * fixed-point sum); mode 1 fuses torchvision ToTensor + Normalize (the network input).
 *   src: uint8 HWC images, sample n at byte offset src_off[n] with height / width
 *        src_hw[2n], src_hw[2n + 1], C channels (all device arrays);
 *   M:   [N][2][3] f64 src -> dst matrices (get_affine_transform, not inverted);
 *   mode 0: out uint8 [N, dh, dw, C] (cv2.warpAffine's result);
 *   mode 1: out f32 [N, C, dh, dw] = (v / 255 - mean[c]) / std[c] (mean, std: [C] f32). */
int posu_crop_warp(const unsigned char* src, const long long* src_off, const int* src_hw, int C,
                   const double* M, int N, int dh, int dw, int mode, const float* mean, const float* std,
                   void* out, void* stream);

/* Gaussian target heatmaps of a batch (JointsDatasetCompatible.generate_heatmap,
 * lib/dataset/joints_dataset_compatible.py:215-253): joints [N, J, 2] f32 in crop px,
 * vis [N, J] f32 (joints_vis[:, 0]); target [N, J, hm_h, hm_w] f32, weight [N, J] f32;
 * zero_weight: NULL or [N] uint8 (1 = weights zeroed: H36M samples without pseudo labels). */
int posu_gaussian_targets(const float* joints, const float* vis, int N, int J, int image_w,
                          int image_h, int hm_w, int hm_h, double sigma,
                          const unsigned char* zero_weight, float* target, float* weight,
                          void* stream);
/* Sum-normalised integral coordinates (run/test/test_integral.py:63-70):
 * out[n][j] = (sum x h, sum y h) / sum h  over hm [N, J, H, W] f32 -> [N, J, 2] f32. */
int posu_integral2d_fwd(const float* hm, int N, int J, int H, int W, float* out, void* stream);

/* ------------------------------------------------------------- geometry */
/* Epipolar consistency loss (FundamentalLoss.__call__, lib/core/loss.py:101-133):
 *   loss = sum_{b, (i,j) in permutations(V,2), k} |x~_j^T F_{s(b),i,j} x~_i| * w_i w_j
 *          / (N * V*(V-1) * J)
 *   x: [V, N, J, 2] f32 (image px); w: NULL or [V, N, J] f32 (target weights,
 *   used when non-NULL, i.e. USE_TARGET_WEIGHT_FUND);
 *   F: [S, V*(V-1), 3, 3] f32, pair index p enumerates itertools.permutations
 *   order; subj: [N] int32 in [0, S).
 *   loss: [1] f32 (written, not accumulated); resid: NULL or [N, P, J] f32. */
int posu_epipolar_loss_fwd(const float* x, const float* w, const float* F,
                           const int* subj, int V, int N, int J, int S,
                           float* loss, float* resid, void* stream);

/* d loss / d x given the scalar upstream gradient gloss [1] (device).
 * gx: [V, N, J, 2] f32 (overwritten). */
int posu_epipolar_loss_bwd(const float* x, const float* w, const float* F,
                           const int* subj, int V, int N, int J, int S,
                           const float* gloss, float* gx, void* stream);

/* Multi-view linear triangulation (triangulate_poses / pymvg
 * MultiCameraSystem.find3d, lib/multiviews/triangulate.py:43-99): per
 * (group, joint), undistort each visible view's point with the OpenCV
 * fixed-point model (5 iterations), build 2 DLT rows per view
 * (x*M[2]-M[0], y*M[2]-M[1]) and take the right singular vector of the
 * smallest singular value (one-sided Jacobi SVD, fp64).  Joints seen in < 2
 * views give (0,0,0) (triangulate.py:95-96).
 *   M:    [G, V, 3, 4] f64 projection matrices K[R | -R C];
 *   intr: [G, V, 9] f64 = fx, fy, cx, cy, k1, k2, p1, p2, k3;
 *   xy:   pixel coords in xy_dtype (POSU_F32 or POSU_F64); joint k of view v of
 *         group g at xy[g*xy_stride_g + v*xy_stride_v + 2k] (elements):
 *         [G, V, J, 2] -> (V*J*2, J*2); view-major [V, G, J, 2] -> (J*2, G*J*2);
 *   vis:  NULL (all visible) or [G, V, J] uint8;
 *   undistort: 0 = no_distortion cameras (distortion ignored);
 *   X:    [G, J, 3] f64. */
int posu_triangulate_dlt(const double* M, const double* intr, const void* xy, int xy_dtype,
                         int xy_stride_g, int xy_stride_v, const unsigned char* vis, int G,
                         int V, int J, int undistort, double* X, void* stream);

/* Pseudo-label RANSAC (multiviews/triangulate.py:102-165, ransac): per (group, joint),
 * every pair of visible views (itertools.combinations order) is triangulated (DLT on
 * undistorted points), re-projected into all V views (pymvg find2d: [R|t] = K^-1 M,
 * OpenCV plumb-bob distortion of intr), and views with error < reproj_thre are that
 * pair's inliers; pairs with fewer than min_inliers (>= 1) are skipped; the best pair has
 * the most inliers, ties broken by the smaller mean error.  res_vis[g][v][k] = 1 for the
 * best pair's inliers, else 0.  xy: [G, V, J, 2] f64 (all views, visible or not);
 * vis: NULL or [G, V, J] uint8; 2 <= V <= 4. */
int posu_ransac_inliers(const double* M, const double* intr, const double* xy,
                        const unsigned char* vis, int G, int V, int J, int undistort,
                        double reproj_thre, int min_inliers, unsigned char* res_vis, void* stream);
/* reproject_poses (triangulate.py:168-213): triangulate each joint from its visible
 * views and project into every view: proj [G, V, J, 2] f64 and res_vis = 1 where the
 * joint has >= 2 visible views (zeros otherwise). */
int posu_reproject(const double* M, const double* intr, const double* xy, const unsigned char* vis,
                   int G, int V, int J, int undistort, double* proj, unsigned char* res_vis,
                   void* stream);


/* ----------------------------------------------------------- training path */
/* BASELINE configs[3]: the data-parallel training step (run/pose2d/train.py +
 * core/function.py:91-366: per-view backbone forward in train mode, JointsMSELoss,
 * FundamentalLoss, loss.backward(), optimizer step).  Replaces the autograd of
 * torch.nn.Conv2d / ConvTranspose2d / BatchNorm2d / ReLU / MaxPool2d for the
 * PoseResNet modules (lib/models/pose_resnet.py:21-205). */

/* Data gradient of conv2d x[N,H,W,Cin] -> y[N,Ho,Wo,Cout] (KHxKW, stride 1|2, pad):
 *   dy: [N,Ho,Wo,Cout] dtype; wt: weights flipped + transposed, packed
 *   [round_up(Cin,64)][round_up(KH*KW*Cout, BK)] (K order (kh, kw, co)), i.e. the
 *   forward packing of W[:, :, ::-1, ::-1].transpose(0, 1);
 *   residual: NULL or [N,H,W,Cin] added to dx; dx: [N,H,W,Cin] dtype.
 *   Cout must be a power of two >= 8 (it is the GEMM's reduction channel count).
 *   1x1 / stride 2 / pad 0 with residual == dx: accumulated in place, dx[2i][2j] += dy[i][j] W^T,
 *   a GEMM over dy's pixels (the other pixels keep dx) instead of over the zero-upsampled grid. */
int posu_conv2d_dgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, const void* wt,
                      int Cin, int KH, int KW, int stride, int pad, const void* residual,
                      void* dx, int H, int W, void* stream);
/* ABI 15: the same on tile configuration `tile` (posu_conv2d_fwd's table; -1 = the built-in
 * heuristic, which posu_conv2d_dgrad runs).  Every tile except 39 accumulates in the same K order,
 * so the choice changes speed, not results.  Refused: an unknown tile. */
int posu_conv2d_dgrad_tile(int dtype, const void* dy, int N, int Ho, int Wo, int Cout, const void* wt,
                           int Cin, int KH, int KW, int stride, int pad, const void* residual,
                           void* dx, int H, int W, int tile, void* stream);

/* ABI 15: the Adam step (torch.optim.Adam, utils/utils.py:79-83; core/function.py:366) over a
 * table of f32 parameter tensors: per element g' = g (+ weight_decay p), m = b1 m + (1-b1) g',
 * v = b2 v + (1-b2) g'^2, p -= lr / (1 - b1^step) * m / (sqrt(v) / sqrt(1 - b2^step) + eps),
 * in f32 (within rounding of torch's kernels).  p, m, v updated in place; `step` = the step being
 * taken (>= 1).  The table is host memory, read during the call (the launches carry it). */
typedef struct posu_adam_tensor {
  float* p;
  const float* g;
  float* m;
  float* v;
  long long n;
} posu_adam_tensor;
int posu_adam_step(const posu_adam_tensor* tensors, int ntensors, double lr, double beta1, double beta2,
                   double eps, double weight_decay, long long step, void* stream);

/* Weight gradient dW[Cout][Creal][KH][KW] (f32, the nn.Conv2d weight layout) of a
 * conv over x[N,H,W,C] (C >= Creal, padded channels ignored) with output gradient
 * dy[N,Ho,Wo,Cout].  Also ConvTranspose2d(4, s2, p1): pass x = the transposed
 * conv's output gradient (as a [N,2H,2W,Cout_t] input), dy = its input
 * [N,H,W,Cin_t], KH=KW=4, stride 2, pad 1 -> dW[Cin_t][Cout_t][4][4].
 * workspace >= posu_conv2d_wgrad_workspace(...) bytes (split-K partials). */
long long posu_conv2d_wgrad_workspace(int dtype, int N, int H, int W, int C, int Cout, int KH,
                                      int KW, int stride, int pad);
int posu_conv2d_wgrad(int dtype, const void* dy, const void* x, int N, int H, int W, int C,
                      int Creal, int Cout, int KH, int KW, int stride, int pad, float* dw,
                      void* workspace, long long workspace_bytes, void* stream);

/* Training-mode BatchNorm2d over z[nseg*Pseg, C] (NHWC, nseg batch segments = camera
 * views with separate statistics, torch.nn.functional.batch_norm(training=True)
 * per segment): mean/rstd/scale/shift [nseg, C] f32 out; running_mean/var
 * (optional) updated once per segment in order, unbiased variance. */
long long posu_bn_workspace(int nseg, int C);
int posu_bn_train_fwd(int dtype, const void* z, int nseg, int Pseg, int C, const float* gamma,
                      const float* beta, float eps, float momentum, float* running_mean,
                      float* running_var, float* mean, float* rstd, float* scale, float* shift,
                      void* workspace, long long workspace_bytes, void* stream);
/* y = act(z * scale[seg] + shift[seg] (+ residual)) */
int posu_bn_apply(int dtype, const void* z, int nseg, int Pseg, int C, const float* scale,
                  const float* shift, const void* residual, int relu, void* y, void* stream);
/* Backward of y = relu?(bn(z) (+ r)):  g' = gy * [y > 0]; without a residual the mask
 * can instead be recomputed from z with the forward's per-segment relu_scale/relu_shift
 * ([nseg, C], posu_bn_train_fwd's scale/shift: y > 0 <=> z*scale + shift > 0), which
 * saves reading y; y = relu_scale = NULL: no ReLU.
 * dz = gamma*rstd*(g' - mean(g') - xhat*mean(g'*xhat)) per segment; dgamma/dbeta
 * [C] f32 written (summed over segments); gres (optional) = g'. */
int posu_bn_train_bwd(int dtype, const void* gy, const void* y, const float* relu_scale,
                      const float* relu_shift, const void* z, int nseg, int Pseg,
                      int C, const float* mean, const float* rstd, const float* gamma,
                      float* dgamma, float* dbeta, void* dz, void* gres, void* workspace,
                      long long workspace_bytes, void* stream);
/* ABI 14: the residual Bottleneck output's ReLU mask as bits.  posu_bn_apply_mask = posu_bn_apply
 * with relu = 1 that also writes mask [nseg*Pseg*C/E] bytes (E = 8 for BF16 / F16, 4 for F32:
 * one byte per 16-B chunk, bit e = [y_e > 0] of the stored y); posu_bn_train_bwd_mask =
 * posu_bn_train_bwd reading that mask instead of y (16x fewer bytes than y, read twice per
 * backward).  Replaces the reference's autograd ReLU / BatchNorm2d backward
 * (lib/models/pose_resnet.py:92-97), results identical to the y-masked path. */
int posu_bn_apply_mask(int dtype, const void* z, int nseg, int Pseg, int C, const float* scale,
                       const float* shift, const void* residual, void* y, void* mask, void* stream);
int posu_bn_train_bwd_mask(int dtype, const void* gy, const void* mask, const void* z, int nseg,
                           int Pseg, int C, const float* mean, const float* rstd,
                           const float* gamma, float* dgamma, float* dbeta, void* dz, void* gres,
                           void* workspace, long long workspace_bytes, void* stream);
/* out[c] = sum_p x[p][c] (f32), e.g. the final layer's bias gradient;
 * workspace >= posu_bn_workspace(1, C). */
int posu_channel_sum(int dtype, const void* x, int P, int C, float* out, void* workspace,
                     long long workspace_bytes, void* stream);
/* MaxPool2d(3, 2, 1) backward (PyTorch's first-maximum tie rule), x the forward
 * input [N,H,W,C], gy [N,Ho,Wo,C] -> gx [N,H,W,C]; workspace: argmax taps. */
long long posu_maxpool3x3s2_bwd_workspace(int N, int H, int W, int C);
int posu_maxpool3x3s2_bwd(int dtype, const void* x, int N, int H, int W, int C, const void* gy,
                          void* gx, void* workspace, long long workspace_bytes, void* stream);
/* ABI 14, the training stem (lib/models/pose_resnet.py:192-195: bn1, relu, maxpool): from the
 * raw conv output z [N,H,W,C] (N = nseg equal segments) and posu_bn_train_fwd's scale/shift,
 * y [N,Ho,Wo,C] = maxpool3x3s2(relu(z*scale[seg] + shift[seg]) rounded to dtype) and idx
 * [N,Ho,Wo,C] bytes = the argmax tap 0..8 (first maximum in window order) -- the activation
 * itself is never written.  posu_maxpool3x3s2_bwd_idx: gx [N,H,W,C] from those taps and gy
 * [N,Ho,Wo,C]; identical to posu_maxpool3x3s2_bwd over the activation. */
int posu_bn_relu_maxpool3x3s2_fwd(int dtype, const void* z, int nseg, int N, int H, int W, int C,
                                  const float* scale, const float* shift, void* y, void* idx,
                                  void* stream);
int posu_maxpool3x3s2_bwd_idx(int dtype, const void* idx, const void* gy, int N, int H, int W,
                              int C, void* gx, void* stream);
/* ABI 14, the training stem's convolution (lib/models/pose_resnet.py:192, nn.Conv2d(3, 64, 7, 2, 3,
 * bias=False)) straight from the caller's NCHW f32 views (views[v] = [Nv, 3, H, W], a host array of
 * device pointers, stacked view-major like posu_stem_pool_views_fwd): z [nviews*Nv, H/2, W/2, 64]
 * of dtype (BF16 / F16) from the parameter's own f32 weight w [64][3][7][7]; and its weight
 * gradient dw [64][3][7][7] f32 from dz [nviews*Nv, H/2, W/2, 64] (workspace:
 * posu_stem_wgrad_workspace bytes of per-block partials, summed in a fixed order).  W = 256,
 * H % 8 == 0. */
int posu_stem_conv_views_fwd(int dtype, const float* const* views, int nviews, int Nv, int H, int W,
                             const float* w, void* z, void* stream);
long long posu_stem_wgrad_workspace(int N, int H, int W);
int posu_stem_wgrad_views(int dtype, const float* const* views, int nviews, int Nv, int H, int W,
                          const void* dz, float* dw, void* workspace, long long workspace_bytes,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* POSU_H_ */
