"""Training step of PoseResNet on the HIP kernels (BASELINE configs[3]).

The reference trains with torch autograd over nn.Conv2d / BatchNorm2d / ReLU /
MaxPool2d / ConvTranspose2d (lib/models/pose_resnet.py:21-205, train mode, called once
per camera view by multiview_pose_resnet.py:74-78) and Adam
(core/function.py:364-366, utils/utils.py:79-83).  Here five autograd Functions (stem +
layer1 | layer2 | layer3 | layer4 | deconvs + head, _StageFn) run the network forward and
backward as explicit kernel launches on NHWC activations, so DDP's gradient all-reduce
starts while the earlier stages are still in backward:

  forward   conv (raw, MFMA implicit GEMM) -> per-view batch statistics -> normalise
            (+ residual) + ReLU, for every conv / deconv; max-pool; 1x1 head
  backward  BN/ReLU backward (residual-branch gradient split off), conv weight
            gradient (split-K MFMA, transposed LDS reads), conv data gradient (the
            forward kernel on flipped weights, zero-upsampled input for stride 2, the
            identity-branch gradient added in its epilogue), max-pool backward.

Views are stacked on the batch axis as `nseg` segments: one launch per layer serves
all views while every view keeps its own BatchNorm statistics and its own running-stat
update (in view order), as in the reference's four backbone calls.

Parameters stay NCHW f32 in the nn.Modules (so optimizers, DDP and checkpoints are
unchanged); they are packed into the kernels' layouts in the compute dtype once per
step -- every weight of the network in ONE posu_pack_weights launch into buffers allocated
once (packing.BatchedPacker) -- and their gradients come back f32 in the modules' layouts.
"""
import torch

from . import ops, train_ops as T
from .packing import BatchedPacker

STEM_CIN_PAD = 8
# weight gradients on a side stream, overlapping the data-gradient chain (_Grads)
SIDE_STREAM_WGRAD = True
HEAD_CPAD = 64   # heatmap-gradient channels padded to one 64-channel tile
# round 5: the residual units' ReLU mask kept as bits (bn_apply_mask: the backward reads 1/16 of
# y's bytes, twice) and the stem's BN + ReLU + max-pool in one pass that stores the argmax taps
# (the activation before the pool is never written, the backward needs no argmax pass)
RELU_BITMASK = True
FUSED_STEM_POOL = True
# round 5: the stem's convolution and weight gradient as their own kernels, straight from the NCHW
# f32 views (no NHWC pack; the generic 8-channel-padded conv / weight gradient took 260 / 477 us)
STEM_KERNELS = True
# round 5: with the stem's own kernels (which read the f32 parameter) the step's weight packing
# runs on the side stream beside the stem's forward; layer1 waits for it
PACK_BESIDE_STEM = True
# round 5: a first block's downsample unit (conv + BN statistics + apply) runs on the side stream
# beside its conv1 / conv2 units in the forward (the side stream is idle until the backward)
DOWN_BESIDE = True
# round 6: in the backward, a first block's downsample unit takes the block output's gradient and the
# residual unit's ReLU mask itself (no g' = gy * mask tensor written for it) and runs its BatchNorm
# backward + weight gradient on a third stream beside the main branch's units; only its data gradient
# (accumulated into the main branch's) joins the main stream
DOWN_BWD_BESIDE = True
# round 5: the data-gradient convolutions on autotuned tiles (posu_conv2d_dgrad_tile, ABI 15), like the
# forward ones (_conv_tuned); the in-place 1x1 / stride-2 ones keep the heuristic (a tuning trial
# would accumulate into its output more than once)
TUNE_DGRAD = True
# round 5: a 3x3 / s2 / p1 conv's data gradient (each layer's first block, conv2) as the sub-pixel
# transposed conv -- its 3x3 kernel zero-padded to 4x4 on the deconv layers' kernel: 16 taps per 2x2
# output quad instead of 36 over the zero-upsampled gradient (even input sizes, no residual)
S2_DGRAD_SUBPIXEL = True


def _conv_tuned(x, w, cout, k, stride, pad, code):
    """A raw training convolution (no BN in the epilogue) on the tile the per-layer autotuner
    picked for its geometry (posu.plan's table; every tile accumulates in the same K order, so
    the choice changes speed, not results): tuned while `plan._Tuner.active` (bench.py tunes
    during its first warm-up step), else the stored choice or the built-in heuristic.  The
    stem (C = 8 direct gather) keeps the heuristic."""
    from .plan import _tuned
    n, h, wd, c = x.shape
    ho, wo = (h + 2 * pad - k) // stride + 1, (wd + 2 * pad - k) // stride + 1
    z = torch.empty((n, ho, wo, cout), dtype=x.dtype, device=x.device)
    if c % 64:
        return ops.conv2d_nhwc(x, w, cout, k, k, stride, pad, None, None, None, False, code, out=z)
    key = ('train_conv', code, tuple(x.shape), cout, k, stride, pad)
    return _tuned(key, cout, lambda t: ops.conv2d_nhwc(x, w, cout, k, k, stride, pad, None, None, None, False, code,
                                                      out=z, tile=t))


def _dgrad_tuned(dy, wt, cin, k, stride, pad, hw, code, residual=None, inplace=False):
    """T.conv2d_dgrad on the tile the autotuner picked for its geometry (TUNE_DGRAD; every
    admissible tile gives the same result)."""
    from .plan import _tuned
    will_inplace = (inplace and T.INPLACE_S2_DGRAD and residual is not None and k == 1 and stride == 2
                    and pad == 0)
    if not TUNE_DGRAD or will_inplace or dy.shape[3] % 64 or cin % 64:
        return T.conv2d_dgrad(dy, wt, cin, k, k, stride, pad, hw, code, residual=residual, inplace=inplace)
    out = torch.empty((dy.shape[0], hw[0], hw[1], cin), dtype=dy.dtype, device=dy.device)
    key = ('train_dgrad', code, tuple(dy.shape), cin, k, stride, pad, tuple(hw), residual is not None)
    return _tuned(key, cin, lambda t: T.conv2d_dgrad(dy, wt, cin, k, k, stride, pad, hw, code, residual=residual,
                                                     out=out, tile=t))


class _Grads(dict):
    """parameter -> gradient; weight gradients run on a side stream (`side`), off the
    backward's critical path: the data-gradient chain (BN backward -> dgrad -> next layer)
    stays on the current stream while the compute-bound weight-gradient GEMMs fill the CUs
    the HBM-bound BatchNorm passes leave idle.  join() makes the current stream wait for them."""

    def __init__(self, side):
        super().__init__()
        self.side = side
        self.event = None

    def wgrad(self, param, fn, *inputs):
        if self.side is None:
            self[param] = fn()
            return
        main = torch.cuda.current_stream(inputs[0].device)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            g = fn()
        for t in inputs:        # read on the side stream: not reused by main-stream allocations early
            t.record_stream(self.side)
        g.record_stream(main)   # consumed on the main stream after join()
        self[param] = g

    def join(self, device):
        if self.side is not None:
            torch.cuda.current_stream(device).wait_stream(self.side)

    def close(self):
        """Record the event after this set's last side-stream launch; returns self."""
        self.event = None
        if self.side is not None:
            self.event = torch.cuda.Event()
            self.event.record(self.side)
        return self

    def wait(self):
        """Make the current stream wait for this set's side-stream launches (not for any
        launched after it)."""
        if self.event is not None:
            torch.cuda.current_stream(self.side.device).wait_event(self.event)


class _ConvBN:
    """conv (no bias) -> BatchNorm2d (train) -> [+ residual] -> [ReLU]."""

    def __init__(self, conv, bn, relu, cin_pad=None):
        self.conv, self.bn, self.relu = conv, bn, relu
        self.k = conv.kernel_size[0]
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.cout, self.cin = conv.weight.shape[:2]
        self.cin_pad = cin_pad or self.cin
        if conv.bias is not None:
            raise NotImplementedError('conv + BN with a conv bias')

    def params(self):
        return [self.conv.weight, self.bn.weight, self.bn.bias]

    def pack(self, packer, bk, need_dgrad=True):
        self.w = packer.conv(self.conv.weight, self.cin_pad, bk)
        self.wt = packer.dgrad(self.conv.weight, bk) if need_dgrad else None
        # a 3x3 / s2 / p1 conv's data gradient as the sub-pixel transposed conv (S2_DGRAD_SUBPIXEL)
        self.wdc = (packer.deconv(self.conv.weight, bk)
                    if need_dgrad and S2_DGRAD_SUBPIXEL and self._subpixel_dgrad() else None)

    def _subpixel_dgrad(self):
        c = self.conv
        return (c.kernel_size == (3, 3) and c.stride == (2, 2) and c.padding == (1, 1) and c.dilation == (1, 1)
                and c.groups == 1 and self.cout % 8 == 0 and (self.cout & (self.cout - 1)) == 0 and self.cin % 8 == 0)

    def forward(self, x, nseg, code, residual=None):
        z = _conv_tuned(x, self.w, self.cout, self.k, self.stride, self.pad, code)
        bn = self.bn
        mean, rstd, sc, sh = T.bn_train_fwd(z, nseg, bn.weight, bn.bias, bn.eps, bn.momentum, bn.running_mean,
                                            bn.running_var)
        if RELU_BITMASK and self.relu and residual is not None:
            y, mask = T.bn_apply_mask(z, nseg, sc, sh, residual)
            return y, (x, z, None, mean, rstd, sc, sh, True, mask)
        y = T.bn_apply(z, nseg, sc, sh, residual, self.relu)
        return y, (x, z, y, mean, rstd, sc, sh, residual is not None, None)

    def forward_pooled(self, x, nseg, code):
        """The stem: conv -> BN (train) -> ReLU -> max-pool 3x3 / s2 in one pass after the
        statistics (T.bn_relu_maxpool); returns (pooled, saved, argmax taps).  x: the packed NHWC
        input, or the list of NCHW f32 views (the stem's own convolution kernel, T.stem_conv)."""
        if isinstance(x, (list, tuple)):
            z = T.stem_conv(x, self.conv.weight.detach(), code)
        else:
            z = _conv_tuned(x, self.w, self.cout, self.k, self.stride, self.pad, code)
        bn = self.bn
        mean, rstd, sc, sh = T.bn_train_fwd(z, nseg, bn.weight, bn.bias, bn.eps, bn.momentum, bn.running_mean,
                                            bn.running_var)
        y, idx = T.bn_relu_maxpool(z, nseg, sc, sh)
        return y, (x, z, None, mean, rstd, sc, sh, False, None), idx

    def relu_gate(self, saved):
        """The ReLU mask of this (residual, ReLU) unit's output as bn_train_bwd takes it: (y, bits)."""
        x, z, y, mean, rstd, sc, sh, has_res, mask = saved
        if not (self.relu and has_res):
            raise RuntimeError('relu_gate: a residual unit with ReLU only')
        return (y if mask is None else None), mask

    def backward_bn(self, gy, saved, nseg, code, grads, want_gres=False, gate=None):
        """BatchNorm backward and the weight gradient: -> (dz, gres).  gate = another unit's
        relu_gate(): gy is gated by that unit's ReLU mask first (the downsample unit of a first block,
        whose gradient is the block output's gated by the residual unit's ReLU)."""
        x, z, y, mean, rstd, sc, sh, has_res, mask = saved
        # ReLU mask: the forward's bits, or y after a residual add, else recomputed from z (one
        # tensor read less)
        mask_y = y if (self.relu and has_res and mask is None) else None
        relu_from = (sc, sh) if (self.relu and not has_res) else None
        if gate is not None:
            if self.relu:
                raise RuntimeError('a gated unit has no ReLU of its own')
            mask_y, mask = gate
        dz, gres, dgam, dbet = T.bn_train_bwd(gy, mask_y, z, nseg, mean, rstd, self.bn.weight, want_gres=want_gres,
                                              relu_from=relu_from, mask=mask)
        if isinstance(x, (list, tuple)):   # the stem from the NCHW views (stem_conv): its own kernel
            grads.wgrad(self.conv.weight, lambda: T.stem_wgrad(x, dz, code), dz, *x)
        else:
            grads.wgrad(self.conv.weight, lambda: T.conv2d_wgrad(dz, x, self.cin, self.k, self.k, self.stride,
                                                                 self.pad, code), dz, x)
        grads[self.bn.weight] = dgam
        grads[self.bn.bias] = dbet
        return dz, gres

    def backward(self, gy, saved, nseg, code, grads, want_gres=False, need_dx=True, dx_residual=None,
                 inplace=False, gate=None, dz=None):
        """-> (dx, gres); dz: the BatchNorm backward already run (backward_bn), only the data gradient."""
        gres = None
        if dz is None:
            dz, gres = self.backward_bn(gy, saved, nseg, code, grads, want_gres=want_gres, gate=gate)
        x = saved[0]
        dx = None
        if need_dx and getattr(self, 'wdc', None) is not None and dx_residual is None and x.shape[1] % 2 == 0 \
                and x.shape[2] % 2 == 0:
            # dx of a 3x3 / s2 / p1 conv = ConvTranspose2d(4, s2, p1) of dz with the 3x3 kernel
            # zero-padded to 4x4: four 2x2 sub-pixel classes (16 taps per output quad) instead of the
            # 3x3 conv over the zero-upsampled dz (36), same kernel as the deconv layers
            from .plan import _tuned
            key = ('train_dgrad_s2', code, tuple(dz.shape), self.cin)
            dx = _tuned(key, self.cin, lambda t: ops.deconv4x4s2_nhwc(dz, self.wdc, self.cin, None, None, False, code,
                                                                      tile=t))
        elif need_dx:
            dx = _dgrad_tuned(dz, self.wt, self.cin, self.k, self.stride, self.pad, tuple(x.shape[1:3]), code,
                              residual=dx_residual, inplace=inplace)
        return dx, gres


class _Block:
    def __init__(self, blk):
        self.bottleneck = hasattr(blk, 'conv3')
        names = ['1', '2', '3'] if self.bottleneck else ['1', '2']
        self.units = [_ConvBN(getattr(blk, 'conv' + s), getattr(blk, 'bn' + s), s != names[-1]) for s in names]
        self.units[-1].relu = True   # relu(bn(conv) + residual)
        self.down = None
        if blk.downsample is not None:
            self.down = _ConvBN(blk.downsample[0], blk.downsample[1], False)

    def all_units(self):
        return self.units + ([self.down] if self.down is not None else [])

    def forward(self, x, nseg, code, side=None):
        saved = []
        res, sd = x, None
        joined = None
        if self.down is not None:
            if side is not None:
                # the downsample unit beside conv1 / conv2: the side stream starts after x exists; its
                # tensors are used on the main stream (conv3's residual add, the backward), so the
                # allocator is told (record_stream), and x is read on the side stream
                main = torch.cuda.current_stream(x.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    res, sd = self.down.forward(x, nseg, code)
                joined = torch.cuda.Event()
                joined.record(side)
                x.record_stream(side)
                for t in sd[1:]:
                    if torch.is_tensor(t):
                        t.record_stream(main)
                res.record_stream(main)
            else:
                res, sd = self.down.forward(x, nseg, code)
        y = x
        for u in self.units[:-1]:
            y, s = u.forward(y, nseg, code)
            saved.append(s)
        if joined is not None:
            torch.cuda.current_stream(x.device).wait_event(joined)
        y, s = self.units[-1].forward(y, nseg, code, residual=res)
        saved.append(s)
        return y, (saved, sd)

    def backward(self, gy, saved, nseg, code, grads, beside=None):
        """beside: a stream for the downsample unit's BatchNorm backward + weight gradient
        (DOWN_BWD_BESIDE), or None."""
        su, sd = saved
        u3 = self.units[-1]
        gated = self.down is not None and DOWN_BWD_BESIDE and u3.relu and su[-1][7]
        dz_d = joined = None
        if gated and beside is not None:
            # the downsample's BatchNorm backward from gy and the residual unit's ReLU mask, beside the
            # main branch; gy, the mask and the saved tensors are read there (record_stream), its
            # outputs are used on the main stream after `joined`
            main = torch.cuda.current_stream(gy.device)
            beside.wait_stream(main)
            gate = u3.relu_gate(su[-1])
            with torch.cuda.stream(beside):
                dz_d, _ = self.down.backward_bn(gy, sd, nseg, code, grads, gate=gate)
            joined = torch.cuda.Event()
            joined.record(beside)
            for t in (gy,) + tuple(t for t in gate if t is not None) + tuple(t for t in sd if torch.is_tensor(t)):
                t.record_stream(beside)
            for t in (dz_d, grads[self.down.bn.weight], grads[self.down.bn.bias], grads.get(self.down.conv.weight)):
                if t is not None:
                    t.record_stream(main)
        g, gres = u3.backward(gy, su[-1], nseg, code, grads, want_gres=not gated)
        for u, s in zip(reversed(self.units[:-1]), reversed(su[:-1])):
            if u is self.units[0]:
                break
            g, _ = u.backward(g, s, nseg, code, grads)
        if self.down is None:
            # identity residual: its gradient joins the first conv's data gradient
            dx, _ = self.units[0].backward(g, su[0], nseg, code, grads, dx_residual=gres)
            return dx
        dx_main, _ = self.units[0].backward(g, su[0], nseg, code, grads)
        # dx_main is this block's own temporary: the downsample's 1x1 / stride-2 data gradient
        # accumulates into it in place
        if joined is not None:
            torch.cuda.current_stream(gy.device).wait_event(joined)
            dx, _ = self.down.backward(None, sd, nseg, code, grads, dx_residual=dx_main, inplace=True, dz=dz_d)
        elif gated:
            dx, _ = self.down.backward(gy, sd, nseg, code, grads, dx_residual=dx_main, inplace=True,
                                       gate=u3.relu_gate(su[-1]))
        else:
            dx, _ = self.down.backward(gres, sd, nseg, code, grads, dx_residual=dx_main, inplace=True)
        return dx


class _DeconvBN:
    def __init__(self, dc, bn):
        if dc.stride != (2, 2) or dc.padding != (1, 1) or dc.output_padding != (0, 0) or dc.kernel_size != (4, 4):
            raise NotImplementedError('deconv supported for kernel 4, stride 2, padding 1')
        if dc.bias is not None:
            raise NotImplementedError('deconv with bias')
        self.dc, self.bn = dc, bn
        self.cin, self.cout = dc.weight.shape[:2]

    def params(self):
        return [self.dc.weight, self.bn.weight, self.bn.bias]

    def pack(self, packer, bk):
        self.w = packer.deconv(self.dc.weight, bk)
        # data gradient = conv 4x4 / s2 / p1 with the [Cin][Cout] weight read as conv weights
        self.wd = packer.conv(self.dc.weight, self.cout, bk)

    def forward(self, x, nseg, code):
        z = ops.deconv4x4s2_nhwc(x, self.w, self.cout, None, None, False, code)
        bn = self.bn
        mean, rstd, sc, sh = T.bn_train_fwd(z, nseg, bn.weight, bn.bias, bn.eps, bn.momentum, bn.running_mean,
                                            bn.running_var)
        y = T.bn_apply(z, nseg, sc, sh, None, True)
        return y, (x, z, mean, rstd, sc, sh)

    def backward(self, gy, saved, nseg, code, grads):
        x, z, mean, rstd, sc, sh = saved
        dz, _, dgam, dbet = T.bn_train_bwd(gy, None, z, nseg, mean, rstd, self.bn.weight, relu_from=(sc, sh))
        grads.wgrad(self.dc.weight, lambda: T.deconv4x4s2_wgrad(x, dz, code), x, dz)
        grads[self.bn.weight] = dgam
        grads[self.bn.bias] = dbet
        return _conv_tuned(dz, self.wd, self.cin, 4, 2, 1, code)


class TrainPlan:
    """Forward/backward launch sequence of one PoseResNet in training mode."""

    def __init__(self, net, code):
        self.net = net
        self.code = code
        self.stem = _ConvBN(net.conv1, net.bn1, True, cin_pad=STEM_CIN_PAD)
        self.layers = [[_Block(b) for b in layer] for layer in (net.layer1, net.layer2, net.layer3, net.layer4)]
        mods = list(net.deconv_layers)
        self.deconvs = [_DeconvBN(mods[i], mods[i + 1]) for i in range(0, len(mods), 3)]
        fl = net.final_layer
        if fl.kernel_size != (1, 1):
            raise NotImplementedError('final layer supported for FINAL_CONV_KERNEL = 1')
        self.head = fl
        self.packer = None
        self.side = None
        self.njoints = fl.weight.shape[0]
        if self.njoints > HEAD_CPAD:
            raise NotImplementedError('more than %d joints' % HEAD_CPAD)

    def units(self):
        out = [self.stem]
        for layer in self.layers:
            for b in layer:
                out += b.all_units()
        return out

    def pack(self):
        """Re-pack every weight from the parameters' current values (one launch); the job
        table and the packed buffers are built on the first call."""
        if self.packer is None or self.packer.device != self.head.weight.device:
            code = self.code
            bk = ops.conv_bk(code)
            pk = BatchedPacker(code, self.head.weight.device)
            self.stem.pack(pk, bk, need_dgrad=False)
            for layer in self.layers:
                for b in layer:
                    for u in b.all_units():
                        u.pack(pk, bk)
            for d in self.deconvs:
                d.pack(pk, bk)
            fl = self.head
            self.head_w = pk.conv(fl.weight, fl.weight.shape[1], bk)
            # dgrad of the head over HEAD_CPAD gradient channels (zero above njoints)
            self.head_wt = pk.dgrad(fl.weight, bk, cout_pitch=HEAD_CPAD)
            self.packer = pk
        fl = self.head
        self.head_b = (fl.bias.detach().float().contiguous() if fl.bias is not None else
                       torch.zeros(self.njoints, device=fl.weight.device))
        self.packer.run()

    # ------------------------------------------------------------------ stages
    # The network runs as NSTAGES autograd Functions (stem + layer1 | layer2 | layer3 | layer4 |
    # deconvs + head) so that parameter gradients reach autograd -- and DistributedDataParallel's
    # bucketed all-reduce -- stage by stage during backward instead of all at once at its end
    # (the reference's DDP overlaps its all-reduce with loss.backward(), run/pose2d/train.py:223,
    # lib/core/function.py:366).
    NSTAGES = 5

    def stage_params(self, i):
        """The parameters stage i computes gradients for (every parameter in exactly one stage,
        in the modules' registration order)."""
        if getattr(self, '_stage_params', None) is None:
            net = self.net
            mods = [[net.conv1, net.bn1, net.layer1], [net.layer2], [net.layer3], [net.layer4],
                    [net.deconv_layers, net.final_layer]]
            self._stage_params = [[p for m in ms for p in m.parameters()] for ms in mods]
        return self._stage_params[i]

    def forward_stage(self, i, x, nseg):
        """Stage i's forward: stage 0 takes the list of V NCHW f32 views (stacked on N as nseg
        BatchNorm segments, packed straight into one NHWC batch: no torch.cat), stages 1-3 the
        previous stage's NHWC activation; returns (outputs, saved) -- stage 4's outputs are
        (heatmaps NCHW f32, deconv output NHWC)."""
        code = self.code
        if i == 0:
            n, _, h, w = x[0].shape
            stem_own = FUSED_STEM_POOL and self._stem_kernels(x)
            packed = None
            # (the first pack, which allocates the packer's persistent buffers and job table, runs on
            # the main stream: allocated on the side stream they would return to its pool when the
            # packer is rebuilt, while main-stream kernels may still read them)
            built = self.packer is not None and self.packer.device == self.head.weight.device
            if stem_own and PACK_BESIDE_STEM and SIDE_STREAM_WGRAD and built:
                # the side stream takes the pack after everything before it on this stream (Adam);
                # the stem needs no packed weight, layer1 waits for the pack below
                dev = x[0].device
                if self.side is None:
                    self.side = torch.cuda.Stream(dev)
                main = torch.cuda.current_stream(dev)
                self.side.wait_stream(main)
                with torch.cuda.stream(self.side):
                    self.pack()
                packed = torch.cuda.Event()
                packed.record(self.side)
            else:
                self.pack()
            if stem_own:
                xin = [v.contiguous().float() for v in x]
            else:
                xin = torch.empty((n * len(x), h, w, STEM_CIN_PAD), dtype=ops.torch_dtype(code), device=x[0].device)
                for k, v in enumerate(x):
                    ops.pack_nchw_to_nhwc(v, code, STEM_CIN_PAD, out=xin[k * n:(k + 1) * n])
            if FUSED_STEM_POOL:
                y, s0, idx = self.stem.forward_pooled(xin, nseg, code)
                saved = {'stem': s0, 'pool_idx': idx, 'blocks': []}
            else:
                a0, s0 = self.stem.forward(xin, nseg, code)
                y = ops.maxpool3x3s2_nhwc(a0, code)
                saved = {'stem': s0, 'pool_in': a0, 'blocks': []}
            if packed is not None:
                torch.cuda.current_stream(x[0].device).wait_event(packed)
            for b in self.layers[0]:
                y, sb = b.forward(y, nseg, code, self._down_side(y))
                saved['blocks'].append(sb)
            # num_batches_tracked += nseg for every BatchNorm (the reference's V backbone calls
            # each add 1): one multi-tensor launch instead of one tiny kernel per layer
            nbt = [bn.num_batches_tracked for bn in self._bns() if bn.num_batches_tracked is not None]
            if nbt:
                torch._foreach_add_(nbt, nseg)
            return y, saved
        if i < 4:
            saved = []
            y = x
            for b in self.layers[i]:
                y, sb = b.forward(y, nseg, code, self._down_side(y))
                saved.append(sb)
            return y, saved
        saved = []
        y = x
        for d in self.deconvs:
            y, sd = d.forward(y, nseg, code)
            saved.append(sd)
        hm = ops.head1x1_nchw(y, self.head_w, self.njoints, self.head_b, code)
        return (hm, y), (saved, y)

    def backward_stage(self, i, saved, gouts, nseg):
        """Stage i's backward: gradient of its input activation (None for stage 0) and a _Grads
        of its parameters, whose side-stream launches end with a recorded event."""
        code = self.code
        if SIDE_STREAM_WGRAD and self.side is None:
            dev = self.head.weight.device
            self.side = torch.cuda.Stream(dev)
        grads = _Grads(self.side if SIDE_STREAM_WGRAD else None)
        if i == 4:
            dhm, df = gouts
            dsaved, f = saved
            g = None
            if dhm is not None:
                gh = ops.pack_nchw_to_nhwc(dhm.contiguous().float(), code, HEAD_CPAD)
                fl = self.head
                grads.wgrad(fl.weight, lambda: T.conv2d_wgrad(gh, f, f.shape[3], 1, 1, 1, 0, code)[:self.njoints]
                            .contiguous(), gh, f)
                if fl.bias is not None:
                    grads[fl.bias] = T.channel_sum(gh)[:self.njoints].contiguous()
                g = T.conv2d_dgrad(gh, self.head_wt, f.shape[3], 1, 1, 1, 0, f.shape[1:3], code)
            if df is not None:   # the deconv features used by the caller's loss as well
                df = df.contiguous()
                g = df if g is None else g.add_(df)
            if g is None:
                return None, grads.close()
            for d, sd in zip(reversed(self.deconvs), reversed(dsaved)):
                g = d.backward(g, sd, nseg, code, grads)
            return g, grads.close()
        (g,) = gouts
        if g is None:
            return None, grads.close()
        g = g.contiguous()
        blocks = self.layers[i]
        sblocks = saved['blocks'] if i == 0 else saved
        for b, sb in zip(reversed(blocks), reversed(sblocks)):
            g = b.backward(g, sb, nseg, code, grads, self._down_bwd_stream(g))
        if i == 0:
            if 'pool_idx' in saved:
                g = T.maxpool3x3s2_bwd_idx(saved['pool_idx'], g, saved['stem'][1].shape[1:3])
            else:
                g = T.maxpool3x3s2_bwd(saved['pool_in'], g)
            self.stem.backward(g, saved['stem'], nseg, code, grads, need_dx=False)
            g = None
        return g, grads.close()

    def _down_bwd_stream(self, g):
        """The third stream for DOWN_BWD_BESIDE (created on first use), or None."""
        from .plan import _Tuner
        if not (DOWN_BWD_BESIDE and SIDE_STREAM_WGRAD) or _Tuner.active:
            return None
        if getattr(self, 'beside', None) is None:
            self.beside = torch.cuda.Stream(g.device)
        return self.beside

    def _down_side(self, x):
        """The side stream for DOWN_BESIDE (created on first use), or None."""
        from .plan import _Tuner
        if not (DOWN_BESIDE and SIDE_STREAM_WGRAD) or _Tuner.active:   # (tile trials time alone)
            return None
        if self.side is None:
            self.side = torch.cuda.Stream(x.device)
        return self.side

    def _stem_kernels(self, views):
        """The stem's own conv / weight-gradient kernels apply: 2-byte compute dtype, 3-channel 7x7 /
        s2 / p3 conv1 without bias, 1..8 views of [N, 3, H, 256] with H % 8 == 0."""
        from ._native import BF16, F16
        c = self.stem.conv
        n, ch, h, w = views[0].shape
        return (STEM_KERNELS and self.code in (BF16, F16) and 1 <= len(views) <= 8 and ch == 3 and w == 256
                and h % 8 == 0 and tuple(c.weight.shape) == (64, 3, 7, 7) and c.stride == (2, 2)
                and c.padding == (3, 3) and c.bias is None)

    def _bns(self):
        out = [u.bn for u in self.units()] + [d.bn for d in self.deconvs]
        return out


# Hand-off of a stage's parameter gradients to autograd: 'delayed' returns them from the NEXT
# stage's backward (the earlier layers'), so the current stream waits for a stage's side-stream
# weight gradients one stage later, when they have long finished; 'joined' returns them from
# the stage itself (the current stream waits for the stage's last weight gradient right away)
GRAD_HANDOFF = 'delayed'


class _Stage:
    """One stage of one training forward: the plan, the stage index, the BN segment count and
    the stages' shared hand-off table {stage: (_Grads, its side-stream event)}."""

    def __init__(self, plan, i, nseg, pending):
        self.plan, self.i, self.nseg, self.pending = plan, i, nseg, pending

    def take(self, j):
        grads = self.pending.pop(j, None)
        if grads is None:
            return {}
        grads.wait()
        return grads


def _handoff_stages(i, nstages):
    """Stages whose gradients stage i's backward returns (GRAD_HANDOFF)."""
    if GRAD_HANDOFF == 'joined':
        return [i]
    return ([i] if i == 0 else []) + ([i + 1] if i + 1 < nstages else [])


class _StageFn(torch.autograd.Function):
    """forward(x, stage, *params) -> the stage's outputs; backward returns the input activation's
    gradient and the gradients of `params` (the parameters of the stages _handoff_stages names;
    every other stage's parameters among them get None)."""

    @staticmethod
    def forward(ctx, x, stage, *params):
        ctx.set_materialize_grads(False)
        outs, saved = stage.plan.forward_stage(stage.i, x, stage.nseg)
        ctx.stage, ctx.saved, ctx.params = stage, saved, params
        return outs

    @staticmethod
    def backward(ctx, *gouts):
        st = ctx.stage
        gx, grads = st.plan.backward_stage(st.i, ctx.saved, gouts, st.nseg)
        ctx.saved = None
        st.pending[st.i] = grads
        out = {}
        for j in _handoff_stages(st.i, st.plan.NSTAGES):
            out.update(st.take(j))
        return (gx, None) + tuple(out.get(p) for p in ctx.params)


def _stage_inputs(plan, i):
    js = set(_handoff_stages(i, plan.NSTAGES)) | {i}
    return tuple(p for j in sorted(js) for p in plan.stage_params(j))


def train_forward(net, plan, views, nseg):
    """Differentiable training-mode forward over a list of V views ([B, 3, H, W] each, V = nseg
    BatchNorm segments): (heatmaps NCHW f32, layer1 out, deconv out) -- the features as
    NCHW-shaped channels-last views, differentiable like the reference's (a loss on them adds
    its gradient to the network's backward)."""
    if torch.is_tensor(views):
        views = [views]
    pending = {}
    y = views
    for i in range(plan.NSTAGES - 1):
        y = _StageFn.apply(y, _Stage(plan, i, nseg, pending), *_stage_inputs(plan, i))
        if i == 0:
            x1 = y
    i = plan.NSTAGES - 1
    hm, f = _StageFn.apply(y, _Stage(plan, i, nseg, pending), *_stage_inputs(plan, i))
    return hm, x1.permute(0, 3, 1, 2), f.permute(0, 3, 1, 2)
