"""Algorithmic HBM bytes of one PoseResNet-50 forward at 256x256 in the benched launch order
(measurement bookkeeping for bench.py and tools/pmc_traffic.py; no GPU work).

Per launch: the bytes a kernel must move at least -- every input activation it needs read once
(for a stride-2 1x1 source only its stride-2 pixels), its weights read once, its outputs written
once.  The launch list is the default plan's (plan.py: fused stem over all views, fused layer1
blocks, layer2 conv1 + the strided tail chained with block 1's conv1, chained streamed tails, conv
launches for layer3 block 0 and layer4, deconv1, deconv2, deconv3 with the fused head writing f32
heatmaps only): 30 launches.  Comparing it with the PMC traffic of the same launches
(FETCH_SIZE x 2 + WRITE_SIZE, tools/pmc_traffic.py) gives each kernel's over-fetch.
"""

# R50 PoseResNet stages: (blocks, planes, in channels, out channels, input spatial at 256x256)
_R50 = ((3, 64, 64, 256, 64), (4, 128, 256, 512, 64), (6, 256, 512, 1024, 32), (3, 512, 1024, 2048, 16))


def r50_256_launches(n=128, es=2, joints=17):
    """[(name, read_bytes, write_bytes)] for one forward of n frames (es: activation bytes)."""
    out = []
    act = lambda hw, c: n * hw * hw * c * es  # noqa: E731
    wb = lambda *dims: es * _prod(dims)  # noqa: E731
    # stem: f32 NCHW input, 7x7x3x64 weight, pooled 64x64x64 output
    out.append(('stem_pool (4 views)', n * 3 * 256 * 256 * 4 + wb(64, 147), act(64, 64)))
    # layer1: fused blocks (block 0 with the downsample)
    out.append(('layer1.0 bottleneck64 (down)', act(64, 64) + wb(64, 64) + wb(64, 576) + wb(256, 64) + wb(256, 64),
                act(64, 256)))
    for b in (1, 2):
        out.append(('layer1.%d bottleneck64' % b, act(64, 256) + wb(64, 256) + wb(64, 576) + wb(256, 64),
                    act(64, 256)))
    # layer2: conv1 at 64x64, the strided tail (chained), chained tails, the last tail
    out.append(('layer2.0 conv1', act(64, 256) + wb(128, 256), act(64, 128)))
    # the strided tail chained with block 1's conv1 (S2_CHAIN): y and block 1's t1 written
    out.append(('layer2.0 strided tail + layer2.1 conv1',
                act(64, 128) + act(32, 256) + wb(128, 1152) + wb(512, 384) + wb(128, 512),
                act(32, 512) + act(32, 128)))
    for b in (1, 2):
        out.append(('layer2.%d chained tail' % b, act(32, 128) + act(32, 512) + wb(128, 1152) + wb(512, 128) +
                    wb(128, 512), act(32, 512) + act(32, 128)))
    out.append(('layer2.3 tail', act(32, 128) + act(32, 512) + wb(128, 1152) + wb(512, 128), act(32, 512)))
    # layer3 block 0 as three convs, block 1 conv1, chained tails, the last tail
    out.append(('layer3.0 conv1', act(32, 512) + wb(256, 512), act(32, 256)))
    out.append(('layer3.0 conv2 s2', act(32, 256) + wb(256, 2304), act(16, 256)))
    out.append(('layer3.0 conv3|down', act(16, 256) + act(16, 512) + wb(1024, 768), act(16, 1024)))
    out.append(('layer3.1 conv1', act(16, 1024) + wb(256, 1024), act(16, 256)))
    for b in (1, 2, 3, 4):
        out.append(('layer3.%d chained tail' % b, act(16, 256) + act(16, 1024) + wb(256, 2304) + wb(1024, 256) +
                    wb(256, 1024), act(16, 1024) + act(16, 256)))
    out.append(('layer3.5 tail', act(16, 256) + act(16, 1024) + wb(256, 2304) + wb(1024, 256), act(16, 1024)))
    # layer4: every conv a launch
    out.append(('layer4.0 conv1', act(16, 1024) + wb(512, 1024), act(16, 512)))
    out.append(('layer4.0 conv2 s2', act(16, 512) + wb(512, 4608), act(8, 512)))
    out.append(('layer4.0 conv3|down', act(8, 512) + act(8, 1024) + wb(2048, 1536), act(8, 2048)))
    for b in (1, 2):
        out.append(('layer4.%d conv1' % b, act(8, 2048) + wb(512, 2048), act(8, 512)))
        out.append(('layer4.%d conv2' % b, act(8, 512) + wb(512, 4608), act(8, 512)))
        out.append(('layer4.%d conv3 + residual' % b, act(8, 512) + act(8, 2048) + wb(2048, 512), act(8, 2048)))
    # deconvs (4 parity classes x 4 taps per class of the 4x4 kernel), the fused head
    out.append(('deconv1', act(8, 2048) + wb(256, 2048, 16), act(16, 256)))
    out.append(('deconv2', act(16, 256) + wb(256, 256, 16), act(32, 256)))
    out.append(('deconv3 + head', act(32, 256) + wb(256, 256, 16) + wb(joints, 256), n * joints * 64 * 64 * 4))
    return out


def _prod(dims):
    p = 1
    for d in dims:
        p *= d
    return p


def r50_256_algorithmic_bytes(n=128, es=2):
    return sum(r + w for _, r, w in r50_256_launches(n, es))


# ---- the training step (bench.py --mode train / the train_mode leg): algorithmic bytes by class
def r50_256_train_classes(n=128, es=2, joints=16, fused_bn=False):
    """{class: (read_bytes, write_bytes)} of one training step of n frames (posu.train_plan's launch
    classes): per conv + BatchNorm unit -- conv: x (a stride-2 1x1 only its stride-2 pixels) and the
    packed weight read, z written; BN statistics: z read; BN apply: z (+ the residual) read, y
    written; backward: BN partial sums and BN apply each read gy and z (+ the ReLU bit mask, 1/16 of
    y, where the ReLU follows a residual add: written by that unit's forward apply), the apply writing
    dz (+ the residual branch's gradient); weight gradient: dz and x
    read, the f32 weight gradient written; data gradient: dz and the packed weight read, dx written
    (+ read where it accumulates into the identity branch's gradient).  Max-pool, the 1x1 head,
    packing (f32 parameters read, forward + data-gradient packs written) and Adam (parameters,
    gradients and both moments read, parameters and moments written) complete it.  The stem (round
    5): its conv and weight gradient read the f32 NCHW views; BN + ReLU + max-pool is one pass (z
    read, the pooled activation and its argmax taps written) and the max-pool backward reads the taps.
    Every tensor once per launch: the floor the kernels' PMC traffic is compared with.

    fused_bn (round 6): the IDEAL step with BatchNorm fused into its neighbours instead of passes of its
    own -- the statistics in the producing conv's epilogue, BN + ReLU applied on the consumer's operand
    load (the block outputs after a residual add still materialised: one pass, z + residual read, y
    written), the backward sums in the epilogue of the kernel that writes gy (z read there), dz = f(gy, z)
    formed on the data- and weight-gradient operand loads (z read by each; written only where the
    residual branch needs it).  Its total against the launch-structure floor is what the separate BN
    passes cost."""
    cls = {k: [0, 0] for k in ('conv fwd / dgrad', 'conv wgrad', 'batchnorm', 'maxpool', 'weight packing',
                                 'adam', 'heads / losses')}

    def add(c, r, w):
        cls[c][0] += r
        cls[c][1] += w

    act = lambda hw, c: n * hw * hw * c * es  # noqa: E731
    nparam = [0]

    def unit(hw_in, cin, hw_out, cout, k, stride, residual=False, want_gres=False, dx=True, dx_acc=False,
             relu_after_res=False, stem=False):
        wts = cout * cin * k * k
        nparam[0] += wts + 2 * cout
        xin = act(hw_out, cin) if (k == 1 and stride == 2) else act(hw_in, cin)
        if stem:
            xin = n * cin * hw_in * hw_in * 4                             # the f32 NCHW views
        z = act(hw_out, cout)
        mask = z // 16 if relu_after_res else 0                           # ReLU bits of y
        add('conv fwd / dgrad', xin + wts * (4 if stem else es), z)       # conv
        if fused_bn:
            if residual:                                                  # y materialised after the add
                add('batchnorm', 2 * z, z + mask)
            add('batchnorm', z + 2 * z, z if want_gres else 0)            # sums' z; dgrad / wgrad read z
        else:
            add('batchnorm', z, 0)                                        # statistics
            if not stem:                                                  # (the stem: fused with the pool)
                add('batchnorm', z + (z if residual else 0), z + mask)    # apply (+ residual, + mask)
            extra = mask                                                  # the mask bits
            add('batchnorm', 2 * z + extra, 0)                            # backward partial sums
            add('batchnorm', 2 * z + extra, z + (z if want_gres else 0))  # backward apply
        add('conv wgrad', z + xin, wts * 4)
        if dx:
            add('conv fwd / dgrad', z + wts * es + (act(hw_in, cin) if dx_acc else 0), act(hw_in, cin))
        if not stem:
            add('weight packing', wts * 4, wts * es * (2 if dx else 1))

    # stem (7x7 from the f32 views) + BN / ReLU / max-pool in one pass (taps: 1 byte per output)
    unit(256, 3, 128, 64, 7, 2, dx=False, stem=True)
    add('maxpool', act(128, 64), act(64, 64) + act(64, 64) // 2)         # forward: z -> pooled + taps
    add('maxpool', act(64, 64) // 2 + act(64, 64), act(128, 64))         # backward (taps, gy -> gx)
    hw = 64
    for blocks, planes, cin, cout, hw_in in _R50:
        for b in range(blocks):
            s = 2 if (hw_in != 64 or cin != 64) and b == 0 and planes != 64 else 1
            ci = cin if b == 0 else cout
            h_in = hw_in if b == 0 else hw
            h_out = h_in // s
            unit(h_in, ci, h_in, planes, 1, 1)                                   # conv1
            unit(h_in, planes, h_out, planes, 3, s)                              # conv2
            unit(h_out, planes, h_out, cout, 1, 1, residual=True, want_gres=True, relu_after_res=True)
            if b == 0:
                unit(h_in, ci, h_out, cout, 1, s, dx_acc=True)                   # downsample
            hw = h_out
    # deconvs (4 classes x 4 taps of the 4x4 kernel), BN + ReLU
    for cin, h in ((2048, 8), (256, 16), (256, 32)):
        unit(h, cin, 2 * h, 256, 4, 1)
    # the 1x1 head: forward writes f32 heatmaps; backward its data / weight gradients
    hm = n * joints * 64 * 64 * 4
    add('heads / losses', act(64, 256) + 256 * joints * es, hm)
    add('heads / losses', 3 * hm, hm)                                    # losses + their gradient
    add('conv fwd / dgrad', hm + 256 * 64 * es, act(64, 256))
    add('conv wgrad', hm + act(64, 256), 256 * joints * 4)
    nparam[0] += 256 * joints + joints
    add('adam', 4 * nparam[0] * 4, 3 * nparam[0] * 4)
    return {k: tuple(v) for k, v in cls.items()}


def r50_256_train_algorithmic_bytes(n=128, es=2, fused_bn=False):
    return sum(r + w for r, w in r50_256_train_classes(n, es, fused_bn=fused_bn).values())
