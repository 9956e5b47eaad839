"""Micro-benchmark of the fused layer1 Bottleneck (posu_bottleneck_fwd) at the bench shape
(128 frames x 64 x 64 x 256, bf16) against the same block as three conv launches.  HIP events,
min over rounds; algorithmic HBM bytes = x read once + y written once.

    python tools/bottleneck_micro.py [--n 128] [--reps 20] [--rounds 3] [--lib PATH]

--lib loads another build of libposeu.so, e.g. one of the timing ablations of
csrc/bottleneck.hip (POSU_BNECK_ABLATE, built by tools/bottleneck_ablations.sh).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import _native, ops, packing  # noqa: E402

BF16 = 1


def timeit(fn, reps, rounds):
    best = 1e9
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', type=int, default=128)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--lib', default=None)
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(0)
    dt = torch.bfloat16
    x = torch.randn(a.n, 64, 64, 256, generator=g).to(dev, dt)
    w1 = torch.randn(64, 256, 1, 1, generator=g) * 0.06
    w2 = torch.randn(64, 64, 3, 3, generator=g) * 0.04
    w3 = torch.randn(256, 64, 1, 1, generator=g) * 0.12
    bn = [(torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1) for c in (64, 64, 256)]
    s = [t.to(dev) for p in bn for t in p]
    bk = ops.conv_bk(BF16)
    p1 = packing.pack_conv_weight(w1.to(dev), 256, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(dev), 64, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(dev), 64, bk, dt)
    p1f = packing.pack_bottleneck_conv1_weight(w1.to(dev), dt)
    p3f = packing.pack_bottleneck_conv3_weight(w3.to(dev), dt)
    y = torch.empty_like(x)
    t1 = torch.empty(a.n, 64, 64, 64, device=dev, dtype=dt)
    t2 = torch.empty_like(t1)
    y3 = torch.empty_like(x)

    def fused():
        ops.bottleneck_nhwc(x, p1f, s[0], s[1], p2, s[2], s[3], p3f, s[4], s[5], BF16, out=y)

    def three():
        ops.conv2d_nhwc(x, p1, 64, 1, 1, 1, 0, s[0], s[1], None, True, BF16, out=t1)
        ops.conv2d_nhwc(t1, p2, 64, 3, 3, 1, 1, s[2], s[3], None, True, BF16, out=t2)
        ops.conv2d_nhwc(t2, p3, 256, 1, 1, 1, 0, s[4], s[5], x, True, BF16, out=y3)

    # the first block (64 input channels, downsample as the residual branch)
    x0 = torch.randn(a.n, 64, 64, 64, generator=g).abs().to(dev, dt)
    w10 = torch.randn(64, 64, 1, 1, generator=g) * 0.1
    wd = torch.randn(256, 64, 1, 1, generator=g) * 0.1
    p10 = packing.pack_conv_weight(w10.to(dev), 64, bk, dt)
    pdual = packing.pack_dual_1x1_weight(w3.to(dev), s[4], wd.to(dev), s[4], dt)
    p3d = packing.pack_bottleneck_down_weight(pdual, 64)
    y0 = torch.empty(a.n, 64, 64, 256, device=dev, dtype=dt)
    y03 = torch.empty_like(y0)

    def fused_down():
        ops.bottleneck_down_nhwc(x0, p10, s[0], s[1], p2, s[2], s[3], p3d, s[5], BF16, out=y0)

    def three_down():
        ops.conv2d_nhwc(x0, p10, 64, 1, 1, 1, 0, s[0], s[1], None, True, BF16, out=t1)
        ops.conv2d_nhwc(t1, p2, 64, 3, 3, 1, 1, s[2], s[3], None, True, BF16, out=t2)
        ops.conv1x1_dual_nhwc(t2, x0, 1, pdual, 256, s[5], True, BF16, out=y03)

    # layer2's identity block (32-wide maps, 512 channels, planes 128)
    xl2 = torch.randn(a.n, 32, 32, 512, generator=g).to(dev, dt)
    q1 = packing.pack_conv_weight((torch.randn(128, 512, 1, 1, generator=g) * 0.06).to(dev), 512, bk, dt)
    q2 = packing.pack_conv_weight((torch.randn(128, 128, 3, 3, generator=g) * 0.03).to(dev), 128, bk, dt)
    q3 = packing.pack_conv_weight((torch.randn(512, 128, 1, 1, generator=g) * 0.1).to(dev), 128, bk, dt)
    sl = [torch.rand(c, device=dev) + 0.5 for c in (128, 128, 512)]
    bl = [torch.randn(c, device=dev) * 0.1 for c in (128, 128, 512)]
    yl2 = torch.empty_like(xl2)
    u1 = torch.empty(a.n, 32, 32, 128, device=dev, dtype=dt)
    u2 = torch.empty_like(u1)
    yl23 = torch.empty_like(xl2)

    wst2 = packing.pack_tail_stream(q2, q3)

    def fused_l2():   # conv1 launch + the register-streamed tail (the plan's layer2 identity block)
        ops.conv2d_nhwc(xl2, q1, 128, 1, 1, 1, 0, sl[0], bl[0], None, True, BF16, out=u1)
        ops.bottleneck_tail_stream_nhwc(u1, xl2, wst2, sl[1], bl[1], sl[2], bl[2], BF16, out=yl2)

    def three_l2():
        ops.conv2d_nhwc(xl2, q1, 128, 1, 1, 1, 0, sl[0], bl[0], None, True, BF16, out=u1)
        ops.conv2d_nhwc(u1, q2, 128, 3, 3, 1, 1, sl[1], bl[1], None, True, BF16, out=u2)
        ops.conv2d_nhwc(u2, q3, 512, 1, 1, 1, 0, sl[2], bl[2], xl2, True, BF16, out=yl23)

    nbytes = 2 * x.numel() * 2
    nb0 = (x0.numel() + y0.numel()) * 2
    nb2 = 2 * xl2.numel() * 2
    cases = [('fused', fused, nbytes), ('fused first', fused_down, nb0), ('fused layer2', fused_l2, nb2)]
    if not a.lib:
        cases += [('three launches', three, nbytes), ('first, unfused', three_down, nb0),
                  ('layer2, unfused', three_l2, nb2)]
    for name, fn, nb in cases:
        us = timeit(fn, a.reps, a.rounds)
        print('%-16s %8.1f us  %5.2f TB/s (algorithmic x + y)' % (name, us, nb / us / 1e6))
    if a.lib:
        return
    torch.cuda.synchronize()
    d = (y.float() - y3.float()).abs()
    print('fused vs three: max %.4g mean %.4g' % (float(d.max()), float(d.mean())))
    d = (y0.float() - y03.float()).abs()
    print('fused first vs unfused: max %.4g mean %.4g' % (float(d.max()), float(d.mean())))
    d = (yl2.float() - yl23.float()).abs()
    print('fused layer2 vs unfused: max %.4g mean %.4g' % (float(d.max()), float(d.mean())))


if __name__ == '__main__':
    main()
