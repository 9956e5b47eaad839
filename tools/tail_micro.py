"""Micro-benchmark of the identity-Bottleneck kernels at the bench shape (128 frames, bf16):
layer3 -- the LDS-ring tail (posu_bottleneck3_tail_fwd) vs the register-streamed tail
(posu_bottleneck_tail_stream_fwd); layer2 -- the fused LDS-ring block (posu_bottleneck2_fwd, all
three convs) vs conv1 as a conv launch + the register-streamed tail.  HIP events, min over
rounds; the streamed outputs are checked bit for bit against the other path.

    python tools/tail_micro.py [--n 128] [--reps 20] [--rounds 3]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import ops, packing  # noqa: E402

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
    ap.add_argument('--only', default='layer3,layer2')
    a = ap.parse_args()
    if a.lib:
        from posu import _native
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device('cuda', 0)
    dt = torch.bfloat16
    bk = ops.conv_bk(BF16)
    for layer, (h, w, c, p) in (('layer3', (16, 16, 1024, 256)), ('layer2', (32, 32, 512, 128))):
        if layer not in a.only:
            continue
        g = torch.Generator().manual_seed(0)
        x = torch.randn(a.n, h, w, c, generator=g).to(dev, dt)
        w1 = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
        w2 = torch.randn(p, p, 3, 3, generator=g) * (2.0 / (9 * p)) ** 0.5
        w3 = torch.randn(c, p, 1, 1, generator=g) * (2.0 / p) ** 0.5 * 0.3
        s = [t.to(dev) for ch in (p, p, c) for t in (torch.rand(ch, generator=g) + 0.5, torch.randn(ch, generator=g) * 0.1)]
        p1 = packing.pack_conv_weight(w1.to(dev), c, bk, dt)
        p2 = packing.pack_conv_weight(w2.to(dev), p, bk, dt)
        p3 = packing.pack_conv_weight(w3.to(dev), p, bk, dt)
        wst = packing.pack_tail_stream(p2, p3)
        t1 = ops.conv2d_nhwc(x, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, BF16)
        y_ring, y_str = torch.empty_like(x), torch.empty_like(x)

        def streamed():
            ops.bottleneck_tail_stream_nhwc(t1, x, wst, s[2], s[3], s[4], s[5], BF16, out=y_str)

        def conv1():
            ops.conv2d_nhwc(x, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, BF16, out=t1)

        if layer == 'layer3':
            def ring():
                ops.bottleneck3_tail_nhwc(t1, x, p2, s[2], s[3], p3, s[4], s[5], BF16, out=y_ring)
        else:
            def ring():
                ops.bottleneck2_nhwc(x, p1, s[0], s[1], p2, s[2], s[3], p3, s[4], s[5], BF16, out=y_ring)
        us_r, us_s, us_1 = timeit(ring, a.reps, a.rounds), timeit(streamed, a.reps, a.rounds), \
            timeit(conv1, a.reps, a.rounds)
        torch.cuda.synchronize()
        gf_tail = 2.0 * a.n * h * w * (9 * p * p + p * c) / 1e9
        print('%s batch %d: LDS-ring %s %.1f us | register-streamed tail %.1f us (%.0f TFLOP/s) + conv1 launch %.1f us '
              '= %.1f us | bit-identical %s' % (layer, a.n, 'tail' if layer == 'layer3' else 'block', us_r, us_s,
                                                gf_tail / us_s * 1e3, us_1, us_s + us_1, bool(torch.equal(y_ring, y_str))),
              flush=True)


if __name__ == '__main__':
    main()
