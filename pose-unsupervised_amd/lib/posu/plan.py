"""Inference plan for PoseResNet on the HIP kernels.

A plan is the packed, device-resident form of a PoseResNet (NHWC weights, folded BN)
plus the ordered list of kernel launches of one forward pass
(lib/models/pose_resnet.py:191-205 of the reference):

    pack(NCHW f32 -> NHWC, C 3 -> 8)
    stem conv 7x7/s2 + BN + ReLU          -> maxpool 3x3/s2
    layer1..4: per block conv/BN/ReLU chain, residual (+ downsample conv/BN) fused
               into the last conv's epilogue
    3 x (deconv 4x4/s2 + BN + ReLU)       (sub-pixel, one launch each)
    final 1x1 conv + bias                 -> NCHW f32 heatmaps

All launches go to PyTorch's current stream, so a forward can be captured in a
torch.cuda.CUDAGraph (hipGraph) by the caller.
"""
import torch

from . import ops
from .packing import (fold_bn, pack_bottleneck_conv1_weight, pack_bottleneck_conv3_weight, pack_bottleneck_down_weight,
                      pack_conv_weight, pack_deconv4x4_weight, pack_down_tail_stream,
                      pack_dual_1x1_weight, pack_s2_tail_stream, pack_stem_fused_weight, pack_stem_s2d_weight,
                      pack_tail_stream, split_exponent, to_split)

STEM_CIN_PAD = 8      # direct 7x7 stem (odd input sizes)
STEM_S2D_PAD = 16     # space-to-depth stem: 4 sub-pixels x 3 channels, padded
SPLIT_PAD = 32        # the split dtype's channel granule (the stem pads to it)


def _stem_pads(code):
    """(direct-stem Cin pad, space-to-depth pad) in logical channels (distinct: run_stem tells the
    two packed inputs apart by their channel count; the split dtype's direct stem, for odd input
    sizes only, pads to 2 granules)."""
    return (2 * SPLIT_PAD, SPLIT_PAD) if code == ops.F16X3 else (STEM_CIN_PAD, STEM_S2D_PAD)


def _pack(pk32, code):
    """An f32 / f64 pack in the logical K order -> (pack in the compute dtype, power-of-two weight
    exponent e the epilogue scale must undo: 2^-e; 0 except for the split dtype)."""
    if code == ops.F16X3:
        e = split_exponent(pk32)
        return to_split(pk32, e), e
    return pk32.to(ops.torch_dtype(code)).contiguous(), 0


def _unscale(scale, e):
    return scale if e == 0 else (scale.double() * 2.0 ** -e).float().contiguous()

# fused pack + stem + max-pool kernel (posu_stem_pool_fwd) for bf16 / fp16 plans
FUSED_STEM = True
# bf16 / fp16 plans: the fused deconv+head sums the head in split precision (the deconv output and
# the head weights as hi + lo pairs of the dtype): the rounding of the deconv output to the dtype
# was the largest single term of the 2-byte chains' joint error (tools/precision_attribution.py)
PRECISE_HEAD = True
# the fused stem over all views of a forward in one launch (posu_stem_pool_views_fwd); False: one
# launch per view
STEM_VIEWS = True


class RawViews:
    """pack_input's result when the fused stem applies: the caller's NCHW f32 views
    (stacked on N in order), consumed directly by posu_stem_pool_fwd.  .packed() gives the
    space-to-depth pack of the two-launch path (chunked runs, tools)."""

    def __init__(self, plan, views, hflip):
        self.plan, self.views, self.hflip = plan, views, hflip
        _, _, self.h, self.w = views[0].shape
        self.shape = (sum(v.shape[0] for v in views), self.h, self.w, 3)
        self.device = views[0].device

    def packed(self):
        return self.plan.pack_input(self.views, hflip=self.hflip, fused=False)

    def __getitem__(self, sl):
        """Batch slice (chunked runs): the views' rows [start, stop) of the stacked batch."""
        if not isinstance(sl, slice) or sl.step not in (None, 1):
            raise TypeError('RawViews supports contiguous batch slices only')
        start, stop, _ = sl.indices(self.shape[0])
        out, base = [], 0
        for v in self.views:
            a, b = max(start - base, 0), min(stop - base, v.shape[0])
            if a < b:
                out.append(v[a:b])
            base += v.shape[0]
        return RawViews(self.plan, out, self.hflip)

# the 128x128 eight-wave staggered conv tiles (7 / 15, round 4) among the autotuner's candidates
TILES_128X8 = True
# the 128x128 tile with two K groups of four waves (39, round 5; inference plans only: its K order
# differs from the other tiles', and the training plan relies on every candidate summing alike).
# bf16 / fp16 plans: on again at the end of round 6 -- with this round's plan the headline and configs[1]
# measured 1 % faster with it (2.237 / 2.250 vs 2.267 / 2.270 ms; 1.331 / 1.327 vs 1.345 / 1.342 ms,
# profiles/r06/ksplit_bf16_ab_r6ah.txt; round 5's plan showed no gain), and the line's `control` leg times
# the plan without it.  Where the tuner picks it, the 2-byte plans' last bits depend on the tuned table
# (reproducible under a fixed --tune-file); the parity mode keeps it out (TILES_KSPLIT_F16X3): every
# candidate tile of the split dtype sums alike, so its results do not depend on the tuning
TILES_KSPLIT = True
TILES_KSPLIT_F16X3 = False
# the split dtype's staggered eight-wave tiles (31, 47 / 55; round 6) among its autotuner candidates
TILES_SPLIT_SG = True

# ---- per-layer tile autotuning: geometry key -> conv tile configuration (process-wide,
# shared by every plan, so a re-packed plan does not re-tune)
_TUNE_CACHE = {}
_TUNE_TIMES = {}   # geometry key -> {tile: best ms of the reps}, the last tuning's measurements
_REFINE_TIMES = {}  # geometry key -> {tile: ms per whole forward}, the in-context stage's measurements
# the in-context second tuning stage (PoseResNetPlan._refine_in_context)
REFINE_IN_CONTEXT = True
# its candidates: the per-launch times within REFINE_WITHIN of a geometry's best, at most REFINE_TOP of them
REFINE_WITHIN = 0.25
REFINE_TOP = 3


class _Tuner:
    active = False
    reps = 3
    seen = []   # geometry keys met by the current tuning run, in launch order
    probe = None      # in-context stage: the geometry whose launches are bracketed by HIP events
    probe_events = []


def _tile_candidates(cout, code=None, ksplit=False):
    """Tile ids (include/posu.h): cfg 0..6, cfg + 8 = single-slot ring (four-wave tiles;
    short-K layers: more blocks per CU), cfg + 16 = three-slot ring (two K-tiles in flight),
    cfg + 32 = persistent K-tile stream (epilogue stores overlap the next tile's fetch),
    23 / 31 = 256x256 / 256x128 with waves 4-7 staggered by half a K-tile, 7 / 15 = 128x128 with
    eight staggered waves."""
    cpad = (cout + 63) // 64 * 64
    c = [0, 1, 2]
    if cpad % 128 == 0:
        c += [3, 4, 6]
    if cpad % 256 == 0:
        c.append(5)
    # + 32: the persistent K-tile stream (2-byte dtypes; others ignore the bit);
    # 23 / 31: the eight-wave tiles with waves 4-7 staggered by half a K-tile; 7 / 15: 128x128 with
    # eight staggered waves (2x4 / 4x2 wave grids)
    sg = [23 + 8 * (t == 6) for t in c if t in (5, 6)] + ([7, 15] if cpad % 128 == 0 and TILES_128X8 else [])
    # (tile 32, the persistent 256x64 four-wave instance, is left out: it spills 928 B per lane to
    # scratch and took ~1.2 ms per launch in the tuning trials, 10x the other tiles)
    if code == ops.F16X3:   # the split dtype: plain rings (no persistent stream), the unstaggered (7 / 15)
        # and (round 6) staggered (47 / 55) eight-wave 128x128 tiles, the staggered 256x128 tile (31) and the
        # two-K-group tile (39)
        return c + [t + 8 for t in c if t <= 4] + [t + 16 for t in c if t != 5] + (
            [7, 15] + ([47, 55, 31] if TILES_SPLIT_SG else []) + ([39] if ksplit and TILES_KSPLIT_F16X3 else [])
            if cpad % 128 == 0 else [])
    if ksplit and code in (ops.BF16, ops.F16) and cpad % 128 == 0:
        sg = sg + [39]
    return c + [t + 8 for t in c if t <= 4] + [t + 16 for t in c if t != 5] + [t + 32 for t in c if t != 0] + sg


def _tuned(key, cout, launch):
    """launch(tile) -> output.  While tuning, time every admissible tile once on the real
    operands (HIP events) and keep the fastest for this geometry."""
    cands = _tile_candidates(cout, key[1], ksplit=TILES_KSPLIT and key[0] in ('conv', 'dual', 'deconv'))
    if _Tuner.active and key not in _Tuner.seen:
        _Tuner.seen.append(key)
    # (re)tune a geometry not in the table, or whose tuned tile is no longer a candidate (a plan
    # switch such as TILES_128X8 turned off for a control run)
    if _Tuner.active and (key not in _TUNE_CACHE or _TUNE_CACHE[key] not in cands):
        # two passes over the candidates, the second in reverse order, each tile's best of the two:
        # one pass let the clock ramp and the neighbours' cache state pick tiles that run 20-25 %
        # slower in the graph (layer4 3x3: 75 vs 60 us, profiles/r04/replay_breakdown_r4l.txt)
        times = {}
        for order in (cands, cands[::-1]):
            for t in order:
                launch(t)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(_Tuner.reps):
                    launch(t)
                b.record()
                b.synchronize()
                ms = a.elapsed_time(b)
                times[t] = min(ms, times.get(t, ms))
        _TUNE_CACHE[key] = min(cands, key=lambda t: (times[t], cands.index(t)))
        _TUNE_TIMES[key] = times
    t = _TUNE_CACHE.get(key, -1)
    if _Tuner.probe is not None and key == _Tuner.probe:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = launch(t if t in cands else -1)
        b.record()
        _Tuner.probe_events.append((a, b))
        return out
    return launch(t if t in cands else -1)


def tuned_tiles():
    """The autotuned table (geometry key -> tile), e.g. for logging."""
    return dict(_TUNE_CACHE)


def tuning_times():
    """The last tuning's per-tile times (geometry key -> {tile: ms for the reps}), for diagnostics."""
    return {k: dict(v) for k, v in _TUNE_TIMES.items()}


def refine_times():
    """The in-context stage's times (geometry key -> {tile: median ms of its launches inside a forward})."""
    return {k: dict(v) for k, v in _REFINE_TIMES.items()}


class _Conv:
    __slots__ = ('w', 'scale', 'shift', 'cout', 'k', 'stride', 'pad', 'relu')

    def __init__(self, conv, bn, relu, code, bk, cin_pad=None):
        cin = conv.weight.shape[1]
        # (the split dtype packs 32 logical k per K-tile)
        self.w, e = _pack(pack_conv_weight(conv.weight, cin_pad or cin, 32 if code == ops.F16X3 else bk,
                                           torch.float32), code)
        self.scale, self.shift = fold_bn(bn, conv.bias)
        self.scale = _unscale(self.scale, e)
        self.cout = conv.weight.shape[0]
        self.k = conv.kernel_size[0]
        if conv.kernel_size[0] != conv.kernel_size[1]:
            raise NotImplementedError('square kernels only')
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.relu = relu

    def __call__(self, x, code, residual=None, out=None):
        if out is None:
            ho = (x.shape[1] + 2 * self.pad - self.k) // self.stride + 1
            wo = (x.shape[2] + 2 * self.pad - self.k) // self.stride + 1
            out = torch.empty((x.shape[0], ho, wo, self.cout * ops.cmul(code)), dtype=x.dtype, device=x.device)
        key = ('conv', code, tuple(x.shape), self.cout, self.k, self.stride, self.pad, residual is not None)
        return _tuned(key, self.cout, lambda t: ops.conv2d_nhwc(
            x, self.w, self.cout, self.k, self.k, self.stride, self.pad, self.scale, self.shift, residual, self.relu,
            code, out=out, tile=t))


class _DualTail:
    """Bottleneck conv3/bn3 + downsample conv/bn as one two-source 1x1 GEMM."""
    __slots__ = ('w', 'scale', 'shift', 'cout', 'stride2')

    def __init__(self, conv3, bn3, dconv, dbn, code):
        s3, b3 = fold_bn(bn3, conv3.bias)
        sd, bd = fold_bn(dbn, dconv.bias)
        self.w, e = _pack(pack_dual_1x1_weight(conv3.weight, s3, dconv.weight, sd, torch.float64), code)
        self.shift = (b3.double() + bd.double()).float().contiguous()
        self.cout = conv3.weight.shape[0]
        self.scale = None if e == 0 else torch.full((self.cout,), 2.0 ** -e, device=self.shift.device)
        self.stride2 = dconv.stride[0]

    def __call__(self, mid, x, code, out=None):
        if out is None:
            out = torch.empty(tuple(mid.shape[:3]) + (self.cout * ops.cmul(code),), dtype=mid.dtype, device=mid.device)
        key = ('dual', code, tuple(mid.shape), tuple(x.shape), self.cout)
        return _tuned(key, self.cout, lambda t: ops.conv1x1_dual_nhwc(
            mid, x, self.stride2, self.w, self.cout, self.shift, True, code, out=out, tile=t, scale=self.scale))


# Bottlenecks of layer1 (planes 64, 64x64 maps) as ONE fused launch each in bf16 / fp16 plans
# (posu_bottleneck_fwd; the first block, with its downsample, posu_bottleneck_down_fwd), and the
# identity Bottlenecks of layer2 / layer3 as conv1 (a conv launch) + the register-streamed
# conv2 + conv3 + residual tail (posu_bottleneck_tail_stream_fwd); False runs the convolutions.
# (The round-2 LDS-ring layer2 block / layer3 tail kernels, slower than the streamed tail, were
# removed from the library in round 4.)
FUSED_BOTTLENECK = True
# layer2's first Bottleneck: conv2 (3x3 / stride 2) and the conv3 | downsample dual GEMM as ONE
# launch (posu_bottleneck_s2_tail_fwd) after the conv1 launch; False: two launches
S2_TAIL = True
# consecutive streamed identity tails chained: block i's tail also computes block i+1's conv1
# over its output (posu_bottleneck_tail_stream_next_fwd), so block i+1 has no conv1 launch and y
# is not re-read for it (tools/chain_micro.py: layer2 105.0 vs 130.0 us, layer3 76.3 vs 85.0 us
# for a tail + the next conv1 launch; bit-identical)
CHAINED_TAILS = True
# layer2's strided tail chained with block 1's conv1 (posu_bottleneck_s2_tail_next_fwd, round 4;
# under CHAINED_TAILS too)
S2_CHAIN = True
# the identity Bottlenecks at 384x384 (R152, BASELINE configs[4]) as conv1 + the streamed tail
# (round 5): layer3 at W = 24 (not chained), layer2 at W = 48 (chained)
TAIL_W24 = True
# layer3 at W = 24: the identity tails chained like the 256x256 ones (2-row tiles, three m-tiles per wave,
# round 6).  Off: measured even with each conv1 a launch of its own after the plain 6-row tail (configs[4]
# 9.82 / 10.01 vs 9.97 / 9.97 k frames/s, profiles/r06/w24_chain_ab_r6l.txt) -- the 2-row tiles' weight
# stream (a third of the MFMAs per fragment) costs what the conv1 launches cost
TAIL_W24_CHAIN = False
# the split dtype's identity Bottlenecks of layer1 / layer2 / layer3 as conv1 + the streamed tail
# (chained), layer1's first block as conv1 + the down tail (chained), round 6; False: the conv launches
SPLIT_TAILS = True
# layer1 at 384x384 (96-wide maps, R152 configs[4]) in bf16 / fp16 plans on the streamed tails (round 6):
# the first block as conv1 + the down tail, the identity blocks as the (chained) tail; False: three
# conv launches per block (the fused layer1 kernel is built for 64-wide maps)
TAIL_W96 = True
# split fp16: the last identity block of layers 1-3 chains the NEXT layer's first conv1 too (C -> 2 P,
# posu_bottleneck_tail_stream_chain_fwd, round 6), so that block's conv1 is no launch of its own
CHAIN_LAYERS = True
# the same layer chain in bf16 / fp16 plans (layers 2-3, NX = 2 tails): bit-identical, but measured
# 0.6 % slower on the headline (call r6m: 2.279 vs 2.264 ms; the 2-row NX = 2 tiles halve the layer's
# last tail's rows per workgroup, which costs what the saved conv1 launch gains), so off
CHAIN_LAYERS_2B = False
# round 6: the split dtype's forward runs stem..layer2 and deconv2..head depth-first over two halves
# of the batch by default (run(chunks=None)): its activations are twice the 2-byte ones, so a half
# batch's layer1 / layer2 tensors stay in the 256 MiB Infinity Cache between launches; the layers stay
# chained (layer1 -> layer2 inside a half, layer2 -> layer3 through a whole-batch buffer) -- 5.47-5.64
# vs 5.60-5.75 ms per forward at 32 x 4 (profiles/r06/chunks_ab_r6vwx.txt; 4 chunks slower: the halved
# grids cost more).  The bf16 headline measured slower chunked (2.376 / 2.378 vs 2.325 / 2.346 ms) and
# keeps 1.
CHUNKS_F16X3 = 2
# which ends of the network a chunked run slices (A/B switches; both by default)
CHUNK_EARLY = True   # stem..layer2 (EARLY_LAYERS = 1: stem..layer1)
EARLY_LAYERS = 2     # layers in the chunked early stage (1 .. 3)
CHUNK_LATE = True    # deconv2..head
LATE_CHUNKS = 0      # > 0: the late stage's own slice count (0: the run's chunks)
_FUSED_MAX_BYTES = (1 << 31) - 256   # the fused kernels address x / y with 32-bit byte offsets


def _fused_fits(x, cout):
    """Input and output of a fused Bottleneck kernel inside its 32-bit addressing range (larger
    batches run the convolutions, which use 64-bit addressing)."""
    px = x.shape[0] * x.shape[1] * x.shape[2]
    es = x.element_size()
    return px * max(x.shape[3], cout) * es < _FUSED_MAX_BYTES


class _Block:
    __slots__ = ('convs', 'down', 'dual', 'w1f', 'w3f', 'w3d', 'l1', 'l2', 'l3', 'wst', 'chain', 'wsn', 'ws2', 'ws2n',
                 'wsd', 'wsdn', 'dscale', 'code', 'xchain', 'wsx')

    def __init__(self, blk, code, bk):
        names = ['conv1', 'conv2', 'conv3'] if hasattr(blk, 'conv3') else ['conv1', 'conv2']
        self.convs = []
        self.down = None
        self.dual = None
        self.w1f = self.w3f = None   # conv1 / conv3 packed for the fused kernel (permuted K)
        self.w3d = None              # the fused first block's [w3*s3 | wd*sd] (permuted conv3 K)
        self.l1 = False              # a layer1 identity block on the streamed tail (the split dtype, round 6)
        self.l2 = False              # a layer2 identity block (fused kernel, the convs' own packs)
        self.l3 = False              # a layer3 identity block (conv1, then the fused conv2 + conv3 tail)
        self.wst = None              # layer2 / layer3: the tail's per-wave weight streams (pack_tail_stream)
        self.chain = None            # the next identity block's conv1 (_Conv) when the tails chain
        self.wsn = None              # the streams with that conv1 appended (pack_tail_stream(.., w1n))
        self.ws2 = None              # layer2 block 0: the strided tail's weight streams (pack_s2_tail_stream)
        self.ws2n = None             # ... with the next block's conv1 appended (the chained strided tail)
        self.wsd = None              # split layer1 block 0: the down tail's streams (pack_down_tail_stream)
        self.wsdn = None             # ... with the next block's conv1 appended
        self.dscale = None           # ... the dual GEMM's epilogue scale (2^-e)
        self.code = code
        self.xchain = None           # split: the next layer's first conv1 (_Conv), chained by this last tail
        self.wsx = None              # ... its tail stream (pack_tail_stream(.., that conv1): NX = 2)
        ds = blk.downsample
        if ds is not None and len(names) == 3 and ds[0].kernel_size == (1, 1) and \
                blk.conv3.weight.shape[1] % bk == 0 and ds[0].weight.shape[1] % bk == 0:
            for nm in names[:2]:
                self.convs.append(_Conv(getattr(blk, nm), getattr(blk, 'bn' + nm[-1]), True, code, bk))
            self.dual = _DualTail(blk.conv3, blk.bn3, ds[0], ds[1], code)
            c1, c2 = self.convs
            if code in (ops.BF16, ops.F16) and self.dual.stride2 == 1 and self.dual.cout == 256 and \
                    c1.k == 1 and c1.stride == 1 and c1.w.shape == (64, 64) and \
                    c2.k == 3 and c2.stride == 1 and c2.pad == 1 and c2.w.shape == (64, 576) and \
                    self.dual.w.shape[1] >= 128:
                self.w3d = pack_bottleneck_down_weight(self.dual.w, 64)
            if code == ops.F16X3 and SPLIT_TAILS and self.dual.stride2 == 1 and self.dual.cout == 256 and \
                    c1.k == 1 and c1.stride == 1 and tuple(c1.w.shape) == (64, 128) and \
                    c2.k == 3 and c2.stride == 1 and c2.pad == 1 and tuple(c2.w.shape) == (64, 1152) and \
                    tuple(self.dual.w.shape) == (256, 256):
                self.wsd = pack_down_tail_stream(c2.w, self.dual.w)
                self.dscale = (self.dual.scale if self.dual.scale is not None else
                               torch.ones(256, device=self.dual.shift.device))
            if code in (ops.BF16, ops.F16) and TAIL_W96 and self.dual.stride2 == 1 and self.dual.cout == 256 and \
                    c1.k == 1 and c1.stride == 1 and tuple(c1.w.shape) == (64, 64) and \
                    c2.k == 3 and c2.stride == 1 and c2.pad == 1 and tuple(c2.w.shape) == (64, 576) and \
                    tuple(self.dual.w.shape) == (256, 128):
                self.wsd = pack_down_tail_stream(c2.w, self.dual.w)
                self.dscale = torch.ones(256, device=self.dual.shift.device)
            if code in (ops.BF16, ops.F16) and self.dual.stride2 == 2 and self.dual.cout == 512 and \
                    c1.k == 1 and c1.stride == 1 and c1.w.shape == (128, 256) and \
                    c2.k == 3 and c2.stride == 2 and c2.pad == 1 and c2.w.shape == (128, 1152) and \
                    tuple(self.dual.w.shape) == (512, 384):
                self.ws2 = pack_s2_tail_stream(c2.w, self.dual.w)
            return
        for nm in names:
            self.convs.append(_Conv(getattr(blk, nm), getattr(blk, 'bn' + nm[-1]), True, code, bk))
        if ds is not None:
            self.down = _Conv(ds[0], ds[1], False, code, bk)
        elif code in (ops.BF16, ops.F16) and len(names) == 3 and self._fusable_shape():
            self.w1f = pack_bottleneck_conv1_weight(blk.conv1.weight, ops.torch_dtype(code))
            self.w3f = pack_bottleneck_conv3_weight(blk.conv3.weight, ops.torch_dtype(code))
            # (the same blocks at 96-wide maps run conv1 + the streamed tail: 'l1' at W = 96)
            self.l1 = TAIL_W96 and self._layer1_shape()
            if self.l1:
                self.wst = pack_tail_stream(self.convs[1].w, self.convs[2].w)
        elif code in (ops.BF16, ops.F16, ops.F16X3) and len(names) == 3:
            # (the split dtype: its packs hold 2 K halves per row; layer1 too -- the fused layer1 kernel
            # does not hold pairs -- on the streamed tail, round 6)
            cm = ops.cmul(code)
            self.l1 = code == ops.F16X3 and SPLIT_TAILS and self._layer1_shape(cm)
            self.l2 = (code != ops.F16X3 or SPLIT_TAILS) and self._layer2_shape(cm)
            self.l3 = (code != ops.F16X3 or SPLIT_TAILS) and self._layer3_shape(cm)
            if self.l1 or self.l2 or self.l3:
                self.wst = pack_tail_stream(self.convs[1].w, self.convs[2].w)

    def link_next(self, nxt):
        """Chain this identity block's streamed tail with the next block's conv1 (same layer, same
        kind of tail)."""
        if (self.l1 and nxt.l1) or (self.l2 and nxt.l2) or (self.l3 and nxt.l3):
            self.chain = nxt.convs[0]
            self.wsn = pack_tail_stream(self.convs[1].w, self.convs[2].w, self.chain.w)
        elif self.wsd is not None and nxt.l1:   # split layer1: the down tail and block 1's conv1
            self.chain = nxt.convs[0]
            self.wsdn = pack_down_tail_stream(self.convs[1].w, self.dual.w, self.chain.w)
        elif self.ws2 is not None and nxt.l2:   # layer2's strided tail and block 1's conv1
            self.chain = nxt.convs[0]
            self.ws2n = pack_s2_tail_stream(self.convs[1].w, self.dual.w, self.chain.w)

    def _tail_kind(self, x):
        """'l2' / 'l3' when this block runs as conv1 + the register-streamed tail, else None."""
        if not FUSED_BOTTLENECK or not _fused_fits(x, self.cout):
            return None
        if self.l1 and x.shape[2] == (64 if self.code == ops.F16X3 else 96) and x.shape[1] % 2 == 0:   # 2-row tiles
            return 'l1'
        if self.l2 and x.shape[2] == 32 and x.shape[1] % 4 == 0:
            return 'l2'
        if self.l3 and x.shape[2] == 16 and x.shape[1] % 8 == 0:
            return 'l3'
        split = self.code == ops.F16X3   # (the split tails: 256x256 maps only)
        if self.l3 and x.shape[2] == 24 and x.shape[1] % 6 == 0 and TAIL_W24 and not split:   # R152@384 (configs[4])
            return 'l3w'
        if self.l2 and x.shape[2] == 48 and x.shape[1] % 2 == 0 and TAIL_W24 and not split:   # layer2 at 384x384
            return 'l2w'
        return None

    def link_layer(self, first):
        """Chain this last identity block's tail with the next layer's first block's conv1 (1x1 / stride 1,
        C -> 2 P: posu_bottleneck_tail_stream_chain_fwd): split fp16 layers 1-3, bf16 / fp16 layers 2-3
        (CHAIN_LAYERS_2B)."""
        tails = (self.l1 or self.l2 or self.l3) if self.code == ops.F16X3 else (
            CHAIN_LAYERS_2B and self.code in (ops.BF16, ops.F16) and (self.l2 or self.l3))
        if not (tails and first.dual is not None):
            return
        c1n = first.convs[0]
        planes = self.convs[1].cout
        if c1n.k == 1 and c1n.stride == 1 and c1n.cout == 2 * planes and tuple(c1n.w.shape)[1] == self.convs[0].w.shape[1]:
            self.xchain = c1n
            self.wsx = pack_tail_stream(self.convs[1].w, self.convs[2].w, c1n.w)

    def run(self, x, code, out=None, t1=None, chain_out=False, t1n_out=None):
        """-> (y, t1n): t1n = the next block's conv1 output when this block's tail is chained
        (CHAINED_TAILS; chain_out: the last block of a layer chaining the next layer's first conv1,
        CHAIN_LAYERS), else None; t1 = this block's conv1 output from the previous block's
        chained tail (None: computed here)."""
        kind = self._tail_kind(x)
        if kind is None:
            if t1 is not None:
                if self.dual is None:
                    raise RuntimeError('a chained conv1 output handed to a block without a streamed tail')
                # the first block of a layer whose conv1 the previous layer's last tail computed
                return self.dual(self.convs[1](t1, code), x, code, out=out), None
            if self.wsdn is not None and CHAINED_TAILS and self._down_tail_ok(x):
                c1, c2 = self.convs
                n1 = self.chain
                return ops.bottleneck_down_tail_stream_nhwc(c1(x, code), x, self.wsdn, c2.scale, c2.shift, self.dscale,
                                                            self.dual.shift, code, s1n=n1.scale, b1n=n1.shift, out=out)
            if self.ws2n is not None and CHAINED_TAILS and S2_CHAIN and self._s2_tail_ok(x):
                c1, c2 = self.convs
                n1 = self.chain
                return ops.bottleneck_s2_tail_next_nhwc(c1(x, code), x, self.ws2n, c2.scale, c2.shift, self.dual.shift,
                                                        n1.scale, n1.shift, code, out=out)
            return self(x, code, out=out), None
        c1, c2, c3 = self.convs
        if t1 is None:
            t1 = c1(x, code)
        if chain_out and self.xchain is not None and CHAINED_TAILS and CHAIN_LAYERS and \
                kind in (('l1', 'l2', 'l3') if self.code == ops.F16X3 else ('l2', 'l3')):
            n1 = self.xchain
            return ops.bottleneck_tail_stream_chain_nhwc(t1, x, self.wsx, c2.scale, c2.shift, c3.scale, c3.shift,
                                                         n1.scale, n1.shift, code, out=out, t1n=t1n_out)
        if self.chain is not None and CHAINED_TAILS and (kind != 'l3w' or TAIL_W24_CHAIN):
            n1 = self.chain
            return ops.bottleneck_tail_stream_next_nhwc(t1, x, self.wsn, c2.scale, c2.shift, c3.scale, c3.shift,
                                                        n1.scale, n1.shift, code, out=out)
        return ops.bottleneck_tail_stream_nhwc(t1, x, self.wst, c2.scale, c2.shift, c3.scale, c3.shift, code,
                                               out=out), None

    def _down_tail_ok(self, x):
        """Split layer1's first block runs conv1 + the down tail (SPLIT_TAILS)."""
        return (self.wsd is not None and FUSED_BOTTLENECK and _fused_fits(x, self.cout) and x.shape[1] % 2 == 0 and
                (x.shape[2] == 64 and self.code == ops.F16X3 and SPLIT_TAILS or
                 x.shape[2] == 96 and self.code != ops.F16X3 and TAIL_W96))

    def _s2_tail_ok(self, x):
        """layer2's first block runs conv1 + the strided tail (S2_TAIL)."""
        return (self.ws2 is not None and S2_TAIL and FUSED_BOTTLENECK and _fused_fits(x, self.cout) and
                x.shape[2] == 64 and x.shape[1] % 8 == 0)

    def _tail_shape(self, c, p, cm):
        """An identity Bottleneck C -> P -> P -> C (1x1, 3x3 / 1 / pad 1, 1x1) whose packs hold cm
        stored halves per logical k."""
        c1, c2, c3 = self.convs
        return (c1.k == 1 and c1.stride == 1 and tuple(c1.w.shape) == (p, c * cm) and
                c2.k == 3 and c2.stride == 1 and c2.pad == 1 and tuple(c2.w.shape) == (p, 9 * p * cm) and
                c3.k == 1 and c3.stride == 1 and tuple(c3.w.shape) == (c, p * cm))

    def _layer1_shape(self, cm=1):
        return self._tail_shape(256, 64, cm)

    def _layer2_shape(self, cm=1):
        return self._tail_shape(512, 128, cm)

    def _layer3_shape(self, cm=1):
        return self._tail_shape(1024, 256, cm)

    def _fusable_shape(self):
        c1, c2, c3 = self.convs
        return (c1.k == 1 and c1.stride == 1 and c1.cout == 64 and c1.w.shape == (64, 256) and
                c2.k == 3 and c2.stride == 1 and c2.pad == 1 and c2.cout == 64 and c2.w.shape == (64, 576) and
                c3.k == 1 and c3.stride == 1 and c3.cout == 256)

    @property
    def cout(self):
        return self.dual.cout if self.dual is not None else self.convs[-1].cout

    def __call__(self, x, code, out=None):
        y = x
        fits = _fused_fits(x, self.cout)
        if self.w3d is not None and FUSED_BOTTLENECK and fits and x.shape[2] == 64 and x.shape[3] == 64:
            c1, c2 = self.convs
            return ops.bottleneck_down_nhwc(x, c1.w, c1.scale, c1.shift, c2.w, c2.scale, c2.shift, self.w3d,
                                            self.dual.shift, code, out=out)
        if self._down_tail_ok(x):
            c1, c2 = self.convs
            return ops.bottleneck_down_tail_stream_nhwc(c1(x, code), x, self.wsd, c2.scale, c2.shift, self.dscale,
                                                        self.dual.shift, code, out=out)[0]
        if self._s2_tail_ok(x):
            c1, c2 = self.convs
            return ops.bottleneck_s2_tail_nhwc(c1(x, code), x, self.ws2, c2.scale, c2.shift, self.dual.shift, code,
                                               out=out)
        if self.dual is not None:
            for c in self.convs:
                y = c(y, code)
            return self.dual(y, x, code, out=out)
        if self.w3f is not None and FUSED_BOTTLENECK and fits and x.shape[2] == 64:
            c1, c2, c3 = self.convs
            return ops.bottleneck_nhwc(x, self.w1f, c1.scale, c1.shift, c2.w, c2.scale, c2.shift, self.w3f, c3.scale,
                                       c3.shift, code, out=out)
        if self._tail_kind(x) is not None:
            c1, c2, c3 = self.convs
            return ops.bottleneck_tail_stream_nhwc(c1(x, code), x, self.wst, c2.scale, c2.shift, c3.scale, c3.shift,
                                                   code, out=out)
        res = self.down(x, code) if self.down is not None else x
        for c in self.convs[:-1]:
            y = c(y, code)
        return self.convs[-1](y, code, residual=res, out=out)


class _Deconv:
    __slots__ = ('w', 'scale', 'shift', 'cout')

    def __init__(self, dc, bn, code, bk):
        if dc.stride != (2, 2) or dc.padding != (1, 1) or dc.output_padding != (0, 0):
            raise NotImplementedError('deconv supported for kernel 4, stride 2, padding 1')
        self.w, e = _pack(pack_deconv4x4_weight(dc.weight, 32 if code == ops.F16X3 else bk, torch.float32), code)
        self.scale, self.shift = fold_bn(bn, dc.bias)
        self.scale = _unscale(self.scale, e)
        self.cout = dc.weight.shape[1]

    def __call__(self, x, code, out=None):
        if out is None:
            out = torch.empty((x.shape[0], 2 * x.shape[1], 2 * x.shape[2], self.cout * ops.cmul(code)), dtype=x.dtype,
                              device=x.device)
        key = ('deconv', code, tuple(x.shape), self.cout)
        return _tuned(key, self.cout, lambda t: ops.deconv4x4s2_nhwc(
            x, self.w, self.cout, self.scale, self.shift, True, code, out=out, tile=t))


class PoseResNetPlan:
    """Packed weights + forward launch sequence of one PoseResNet in one compute dtype."""

    def __init__(self, net, code):
        self.code = code
        bk = ops.conv_bk(code)
        self.cin_pad, self.s2d_pad = _stem_pads(code)
        self.stem = _Conv(net.conv1, net.bn1, True, code, bk, cin_pad=self.cin_pad)
        # the same stem as a 4x4/s1 conv over the 2x2 space-to-depth input (even sizes); the same
        # weights, so the same split exponent (the stem's scale is shared)
        if code == ops.F16X3:
            self.stem_s2d_w = to_split(pack_stem_s2d_weight(net.conv1.weight, self.s2d_pad, 32, torch.float32),
                                       split_exponent(net.conv1.weight.float()))
        else:
            self.stem_s2d_w = pack_stem_s2d_weight(net.conv1.weight, self.s2d_pad, bk, ops.torch_dtype(code))
        self.layers = [[_Block(b, code, bk) for b in layer] for layer in
                       (net.layer1, net.layer2, net.layer3, net.layer4)]
        for layer in self.layers:
            for b0, b1 in zip(layer, layer[1:]):
                b0.link_next(b1)
        for la, lb in zip(self.layers, self.layers[1:]):
            la[-1].link_layer(lb[0])
        mods = list(net.deconv_layers)
        self.deconvs = []
        for i in range(0, len(mods), 3):
            self.deconvs.append(_Deconv(mods[i], mods[i + 1], code, bk))
        fl = net.final_layer
        if fl.kernel_size != (1, 1):
            raise NotImplementedError('final layer supported for FINAL_CONV_KERNEL = 1')
        # the fused head reads hi / lo weight halves in the logical channel order (the split dtype
        # too); a separate head launch of the split dtype reads a split pack (head_w_split)
        self.head_w = pack_conv_weight(fl.weight, fl.weight.shape[1], bk, ops.torch_dtype(code))
        self.head_w_lo = None   # the split-precision head's residual weights (2-byte dtypes)
        self.head_w_split = None
        if code in (ops.BF16, ops.F16, ops.F16X3):
            w32 = pack_conv_weight(fl.weight, fl.weight.shape[1], bk, torch.float32)
            self.head_w_lo = (w32 - self.head_w.float()).to(ops.torch_dtype(code)).contiguous()
        if code == ops.F16X3:
            self.head_w_split = to_split(pack_conv_weight(fl.weight, fl.weight.shape[1], 32, torch.float32))
        self.head_b = (fl.bias.detach().float().contiguous() if fl.bias is not None
                       else torch.zeros(fl.weight.shape[0], device=fl.weight.device))
        self.njoints = fl.weight.shape[0]
        last = self.deconvs[-1] if self.deconvs else None
        self.fuse_head = last is not None and last.cout == 256 and self.njoints <= 16
        self.stem_fused_w = None
        if (FUSED_STEM and code in (ops.BF16, ops.F16, ops.F16X3) and tuple(net.conv1.weight.shape) == (64, 3, 7, 7)
                and net.conv1.stride == (2, 2) and net.conv1.padding == (3, 3)):
            if code == ops.F16X3:   # hi plane, then lo plane (posu_stem_pool_fwd); the stem conv's exponent
                v = pack_stem_fused_weight(net.conv1.weight, torch.float64) * 2.0 ** split_exponent(net.conv1.weight)
                hi = v.to(torch.float16)
                self.stem_fused_w = torch.cat([hi, (v - hi.double()).to(torch.float16)], dim=0).contiguous()
            else:
                self.stem_fused_w = pack_stem_fused_weight(net.conv1.weight, ops.torch_dtype(code))

    def pack_input(self, views, hflip=False, fused=True):
        """List of NCHW f32 tensors (same shape) -> one NHWC batch (views stacked on N):
        space-to-depth [N, H/2, W/2, 16] for even H, W, else [N, H, W, 8]; hflip mirrors
        every image along W (flip test).  Where the fused stem applies (bf16 / fp16,
        H % 8 == 0, W in {256, 384}) the views are handed over as they are (RawViews)."""
        n, _, h, w = views[0].shape
        if fused and self.stem_fused_w is not None and h % 8 == 0 and w in ((256,) if self.code == ops.F16X3 else
                                                                             (256, 384)) and views[0].shape[1] == 3:
            return RawViews(self, list(views), hflip)
        s2d = h % 2 == 0 and w % 2 == 0
        cm = ops.cmul(self.code)
        shape = ((n * len(views), h // 2, w // 2, self.s2d_pad * cm) if s2d else
                 (n * len(views), h, w, self.cin_pad * cm))
        x = torch.empty(shape, dtype=ops.torch_dtype(self.code), device=views[0].device)
        for i, v in enumerate(views):
            if s2d:
                ops.pack_s2d_nchw(v, self.code, self.s2d_pad, out=x[i * n:(i + 1) * n], hflip=hflip)
            else:
                ops.pack_nchw_to_nhwc(v, self.code, self.cin_pad, out=x[i * n:(i + 1) * n], hflip=hflip)
        return x

    def stem_pool(self, x):
        """stem + max-pool: one fused launch over the views for RawViews, else two launches."""
        code = self.code
        if isinstance(x, RawViews):
            if STEM_VIEWS and len({tuple(v.shape) for v in x.views}) == 1 and len(x.views) <= 8:
                return ops.stem_pool_views(x.views, self.stem_fused_w, self.stem.scale, self.stem.shift, code,
                                           hflip=x.hflip)
            out = torch.empty((x.shape[0], x.h // 4, x.w // 4, self.stem.cout * ops.cmul(code)),
                              dtype=ops.torch_dtype(code), device=x.device)
            base = 0
            for v in x.views:
                ops.stem_pool(v, self.stem_fused_w, self.stem.scale, self.stem.shift, code,
                              out=out[base:base + v.shape[0]], hflip=x.hflip)
                base += v.shape[0]
            return out
        return ops.maxpool3x3s2_nhwc(self.run_stem(x), code)

    def run_stem(self, x):
        code = self.code
        if isinstance(x, RawViews):
            x = x.packed()
        if x.shape[3] == self.s2d_pad * ops.cmul(code):
            st = self.stem
            out = torch.empty(tuple(x.shape[:3]) + (st.cout * ops.cmul(code),), dtype=x.dtype, device=x.device)
            key = ('stem_s2d', code, tuple(x.shape), st.cout)
            return _tuned(key, st.cout, lambda t: ops.conv2d_nhwc(
                x, self.stem_s2d_w, st.cout, 4, 4, 1, 2, st.scale, st.shift, None, True, code,
                out=out, out_hw=(x.shape[1], x.shape[2]), tile=t))
        return self.stem(x, code)

    def _stage_early(self, x, out=None, keep=None, t1_out=None, nl=2):
        """stem -> maxpool -> layer1 [-> layer2] (nl layers; out: the last one's output slice, keep: layer1
        output slice to fill when nl = 2); each layer's last tail hands the next layer's first block its
        conv1 output as in the whole-batch run (CHAIN_LAYERS): inside the slice, and the last early
        layer's into t1_out (the slice of a whole-batch buffer the next layer takes).  Returns (last early
        layer's out, layer1 out, t1_out if the last tail filled it)."""
        code = self.code
        x = self.stem_pool(x)
        t1 = None
        x1 = None
        for li in range(nl):
            layer = self.layers[li]
            for bi, blk in enumerate(layer):
                last = bi == len(layer) - 1
                dst = out if li == nl - 1 else (keep if li == 0 else None)
                x, t1 = blk.run(x, code, out=dst if last else None, t1=t1,
                                chain_out=last and (li < nl - 1 or t1_out is not None),
                                t1n_out=t1_out if li == nl - 1 and last else None)
            if li == 0:
                x1 = x
        return x, x1, t1

    @staticmethod
    def _run_layer(layer, x, code, out=None):
        """The blocks of one layer in order (out: the last block's output buffer); chained
        streamed tails hand the next block its conv1 output."""
        t1 = None
        for bi, blk in enumerate(layer):
            x, t1 = blk.run(x, code, out=out if bi == len(layer) - 1 else None, t1=t1)
        if t1 is not None:
            raise RuntimeError('the last block of a layer produced a chained conv1 output')
        return x

    def _last_deconv_head(self, x, keep_f, hm_out=None, f_out=None):
        """Last deconv (+BN+ReLU) and the 1x1 head, fused into one launch when possible."""
        code = self.code
        dc = self.deconvs[-1]
        if self.fuse_head:
            return ops.deconv4x4s2_head(x, dc.w, dc.cout, dc.scale, dc.shift, self.head_w, self.njoints, self.head_b,
                                        code, keep_f=keep_f, hm_out=hm_out, f_out=f_out,
                                        head_w_lo=self.head_w_lo if PRECISE_HEAD else None)
        f = dc(x, code, out=f_out)
        hw = self.head_w_split if code == ops.F16X3 else self.head_w
        return ops.head1x1_nchw(f, hw, self.njoints, self.head_b, code, out=hm_out), f

    def _stage_late(self, x, hm_out=None, f_out=None, keep_f=True):
        """deconv2 .. last deconv -> head."""
        code = self.code
        for dc in self.deconvs[1:-1]:
            x = dc(x, code)
        return self._last_deconv_head(x, keep_f, hm_out=hm_out, f_out=f_out)

    @staticmethod
    def _block_cout(blk):
        return blk.cout

    def default_chunks(self):
        """The depth-first slices run(chunks=None) takes: CHUNKS_F16X3 for the split dtype, else 1."""
        return CHUNKS_F16X3 if self.code == ops.F16X3 else 1

    def autotune(self, x, chunks=None, keep_features=True, reps=3):
        """Time every admissible tile configuration of every conv launch of this forward
        (on the packed input x) and keep the fastest per layer geometry; later runs (and
        hipGraph captures) use the tuned tiles."""
        _Tuner.active, _Tuner.reps, _Tuner.seen = True, reps, []
        try:
            with torch.no_grad():
                out = self.run(x, chunks=chunks, keep_features=keep_features)
        finally:
            _Tuner.active = False
        if REFINE_IN_CONTEXT:
            with torch.no_grad():
                self._refine_in_context(x, chunks, keep_features)
        return out

    def _refine_in_context(self, x, chunks, keep_features, within=None, top=None, forwards=6):
        """Second tuning stage: for every geometry of this forward whose best per-launch
        candidates lie within 25 % of each other, run the whole forward with each of its top
        three and keep the one whose launches of that geometry took least INSIDE the forward
        (HIP events around exactly those launches, median over two rounds of `forwards`
        forwards).  The per-launch trials run one launch back to back; inside the network a
        launch follows other kernels at sustained clocks, and the ranking can differ: layer4's
        3x3 took 53 us on two tiles in isolation and 62 vs 75 us on them in the graph
        (profiles/r04/replay_breakdown*.txt).  (Round 4 compared whole-forward times, whose
        run-to-run spread -- ~0.5 % of 2.5 ms -- is as large as the differences it had to
        resolve: deconv1 went to a tile 15 us slower in one tuning, profiles/r05.)"""
        def forward_ms(key):
            self.run(x, chunks=chunks, keep_features=keep_features)
            torch.cuda.synchronize()
            _Tuner.probe, _Tuner.probe_events = key, []
            try:
                for _ in range(forwards):
                    self.run(x, chunks=chunks, keep_features=keep_features)
                torch.cuda.synchronize()
                ms = sorted(a.elapsed_time(b) for a, b in _Tuner.probe_events)
            finally:
                _Tuner.probe, _Tuner.probe_events = None, []
            return ms[len(ms) // 2] if ms else float('inf')
        within = REFINE_WITHIN if within is None else within
        top = REFINE_TOP if top is None else top
        for key in list(_Tuner.seen):
            times = _TUNE_TIMES.get(key)
            if not times or key not in _TUNE_CACHE:
                continue
            best = min(times.values())
            cands = sorted((t for t in times if times[t] <= best * (1 + within)), key=lambda t: times[t])[:top]
            if len(cands) < 2:
                continue
            res = {}
            for order in (cands, cands[::-1]):
                for t in order:
                    _TUNE_CACHE[key] = t
                    ms = forward_ms(key)
                    res[t] = min(ms, res.get(t, ms))
            _TUNE_CACHE[key] = min(cands, key=lambda t: (res[t], cands.index(t)))
            _REFINE_TIMES[key] = res

    def run(self, x, chunks=None, keep_features=True):
        """Packed input -> (heatmaps NCHW f32, layer1 out NHWC, deconv out NHWC).

        chunks > 1 runs the HBM-bound ends of the network (stem..layer2 and
        deconv2..head) depth-first over `chunks` slices of the batch, so their
        activations stay resident in the 256 MiB Infinity Cache between producer and
        consumer; layer3..deconv1 run on the whole batch (None: default_chunks()).
        keep_features=False skips materialising the full layer1 / deconv outputs
        (returned as None)."""
        code = self.code
        if chunks is None:
            chunks = self.default_chunks()
        n = x.shape[0]
        if chunks <= 1 or n % chunks or len(self.deconvs) < 2:
            x = self.stem_pool(x)
            x1 = None
            t1 = None   # a conv1 output handed across a layer boundary (CHAIN_LAYERS)
            for li, layer in enumerate(self.layers):
                for bi, blk in enumerate(layer):
                    x, t1 = blk.run(x, code, t1=t1, chain_out=bi == len(layer) - 1 and li + 1 < len(self.layers))
                if li == 0:
                    x1 = x
            if t1 is not None:
                raise RuntimeError('the last layer produced a chained conv1 output')
            for dc in self.deconvs[:-1]:
                x = dc(x, code)
            hm, f = self._last_deconv_head(x, keep_features)
            return hm, (x1 if keep_features else None), f
        c = n // chunks
        dt = ops.torch_dtype(code)
        dev = x.device
        if x.shape[3] == self.s2d_pad * ops.cmul(code):
            hs, ws = x.shape[1], x.shape[2]
        else:
            hs, ws = (x.shape[1] - 1) // 2 + 1, (x.shape[2] - 1) // 2 + 1
        hp, wp = (hs - 1) // 2 + 1, (ws - 1) // 2 + 1          # after maxpool = layer1 grid
        cm = ops.cmul(code)
        el = max(1, min(EARLY_LAYERS, len(self.layers) - 1))   # layers in the chunked early stage
        he, we = hp, wp
        for _ in range(el - 1):                                  # layers 2.. halve the grid
            he, we = (he - 1) // 2 + 1, (we - 1) // 2 + 1
        x2 = torch.empty((n, he, we, self._block_cout(self.layers[el - 1][-1]) * cm), dtype=dt, device=dev)
        x1 = x2 if el == 1 else (torch.empty((n, hp, wp, self._block_cout(self.layers[0][-1]) * cm), dtype=dt,
                                             device=dev) if keep_features else None)
        # the next layer's first conv1, computed by the last early layer's tail chunk by chunk
        # (CHAIN_LAYERS), else None
        nc1 = self.layers[el][0].convs[0] if len(self.layers) > el and self.layers[el][0].convs else None
        t1 = (torch.empty((n, he, we, nc1.cout * cm), dtype=dt, device=dev)
              if nc1 is not None and self.layers[el - 1][-1].xchain is not None else None)
        chained = []
        ce = chunks if CHUNK_EARLY else 1
        c = n // ce
        for k in range(ce):
            sl = slice(k * c, (k + 1) * c)
            _, _, t1k = self._stage_early(x[sl], out=x2[sl], keep=None if (x1 is None or el == 1) else x1[sl],
                                          t1_out=None if t1 is None else t1[sl], nl=el)
            chained.append(t1k is not None)
        if any(chained) != all(chained):
            raise RuntimeError('the chunks of one batch took different tails')
        t1 = t1 if all(chained) else None
        y = x2
        for li in range(el, len(self.layers)):
            layer = self.layers[li]
            for bi, blk in enumerate(layer):
                last = bi == len(layer) - 1
                y, t1 = blk.run(y, code, t1=t1, chain_out=last and li + 1 < len(self.layers))
        if t1 is not None:
            raise RuntimeError('the last layer produced a chained conv1 output')
        y = self.deconvs[0](y, code)
        hf, wf = y.shape[1] * 2 ** (len(self.deconvs) - 1), y.shape[2] * 2 ** (len(self.deconvs) - 1)
        hm = torch.empty((n, self.njoints, hf, wf), dtype=torch.float32, device=dev)
        f = (torch.empty((n, hf, wf, self.deconvs[-1].cout * cm), dtype=dt, device=dev) if keep_features else None)
        cl = (LATE_CHUNKS if LATE_CHUNKS > 0 and n % LATE_CHUNKS == 0 else chunks) if CHUNK_LATE else 1
        c = n // cl
        for k in range(cl):
            sl = slice(k * c, (k + 1) * c)
            self._stage_late(y[sl], hm_out=hm[sl], f_out=None if f is None else f[sl], keep_f=f is not None)
        return hm, (x1 if keep_features else None), f
