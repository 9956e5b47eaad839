"""Micro-benchmark of the fused layer3 Bottleneck tail (posu_bottleneck3_tail_fwd) at the bench
shape (128 frames x 16 x 16, t1 256 / x 1024 channels, bf16) against conv2 + conv3 as two conv
launches (heuristic tiles and the tiles the bench autotunes).  HIP events, min over rounds.

    python tools/tail3_micro.py [--n 128] [--reps 20] [--rounds 3] [--lib PATH]
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
    t1 = torch.randn(a.n, 16, 16, 256, generator=g).abs().to(dev, dt)
    x = torch.randn(a.n, 16, 16, 1024, generator=g).to(dev, dt)
    w2 = torch.randn(256, 256, 3, 3, generator=g) * 0.03
    w3 = torch.randn(1024, 256, 1, 1, generator=g) * 0.05
    bn = [(torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1) for c in (256, 1024)]
    s = [t.to(dev) for p in bn for t in p]
    bk = ops.conv_bk(BF16)
    p2 = packing.pack_conv_weight(w2.to(dev), 256, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(dev), 256, bk, dt)
    y = torch.empty_like(x)
    t2 = torch.empty_like(t1)
    y2 = torch.empty_like(x)

    def fused():
        ops.bottleneck3_tail_nhwc(t1, x, p2, s[0], s[1], p3, s[2], s[3], BF16, out=y)

    wst = packing.pack_tail_stream(p2, p3)
    y3 = torch.empty_like(x)

    def streamed():
        ops.bottleneck_tail_stream_nhwc(t1, x, wst, s[0], s[1], s[2], s[3], BF16, out=y3)

    def two(t_2=-1, t_3=-1):
        ops.conv2d_nhwc(t1, p2, 256, 3, 3, 1, 1, s[0], s[1], None, True, BF16, out=t2, tile=t_2)
        ops.conv2d_nhwc(t2, p3, 1024, 1, 1, 1, 0, s[2], s[3], x, True, BF16, out=y2, tile=t_3)

    us_f = timeit(fused, a.reps, a.rounds)
    us_s = timeit(streamed, a.reps, a.rounds)
    us_2 = timeit(two, a.reps, a.rounds)
    us_2t = timeit(lambda: two(31, 23), a.reps, a.rounds)
    us_c2 = timeit(lambda: ops.conv2d_nhwc(t1, p2, 256, 3, 3, 1, 1, s[0], s[1], None, True, BF16, out=t2, tile=31),
                   a.reps, a.rounds)
    gf = 2.0 * a.n * 256 * (2304 * 256 + 256 * 1024) / 1e9
    print('layer3 tail, batch %d: register-streamed %.1f us (%.0f TFLOP/s), equal %s | LDS-ring fused %.1f us '
          '(%.0f TFLOP/s) | two launches %.1f us (heuristic tiles), %.1f us (tiles 31 + 23; conv2 alone %.1f us)'
          % (a.n, us_s, gf / us_s * 1e3, bool(torch.equal(y3, y)), us_f, gf / us_f * 1e3, us_2, us_2t, us_c2))


if __name__ == '__main__':
    main()
