"""Micro-benchmark of layer2's first Bottleneck tail at the bench shape (128 frames, bf16):
conv2 (3x3 / stride 2) + the conv3 | downsample dual GEMM as two launches (the plan's autotuned
tiles are not used: heuristic tiles) vs posu_bottleneck_s2_tail_fwd; HIP events, min over rounds,
outputs checked bit for bit.

    python tools/s2tail_micro.py [--n 128] [--reps 20] [--rounds 3]
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
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(0)
    bk = ops.conv_bk(BF16)
    x = torch.randn(a.n, 64, 64, 256, generator=g).abs().to(dev, dt)
    t1 = torch.randn(a.n, 64, 64, 128, generator=g).abs().to(dev, dt)
    p2 = packing.pack_conv_weight((torch.randn(128, 128, 3, 3, generator=g) * 0.04).to(dev), 128, bk, dt)
    pd = packing.pack_dual_1x1_weight((torch.randn(512, 128, 1, 1, generator=g) * 0.1).to(dev),
                                      (torch.rand(512, generator=g) + 0.5).to(dev),
                                      (torch.randn(512, 256, 1, 1, generator=g) * 0.05).to(dev),
                                      (torch.rand(512, generator=g) + 0.5).to(dev), dt)
    s2, b2 = (torch.rand(128, generator=g) + 0.5).to(dev), (torch.randn(128, generator=g) * 0.1).to(dev)
    shift = (torch.randn(512, generator=g) * 0.1).to(dev)
    ws = packing.pack_s2_tail_stream(p2, pd)
    t2 = torch.empty(a.n, 32, 32, 128, device=dev, dtype=dt)
    y2 = torch.empty(a.n, 32, 32, 512, device=dev, dtype=dt)
    y1 = torch.empty_like(y2)

    def two():
        ops.conv2d_nhwc(t1, p2, 128, 3, 3, 2, 1, s2, b2, None, True, BF16, out=t2)
        ops.conv1x1_dual_nhwc(t2, x, 2, pd, 512, shift, True, BF16, out=y2)

    def fused():
        ops.bottleneck_s2_tail_nhwc(t1, x, ws, s2, b2, shift, BF16, out=y1)

    # the chained variant (+ layer2 block 1's conv1 over y) against the tail + a conv1 launch
    p1n = packing.pack_conv_weight((torch.randn(128, 512, 1, 1, generator=g) * 0.06).to(dev), 512, bk, dt)
    s1n, b1n = (torch.rand(128, generator=g) + 0.5).to(dev), (torch.randn(128, generator=g) * 0.1).to(dev)
    wsn = packing.pack_s2_tail_stream(p2, pd, p1n)
    y3 = torch.empty_like(y2)
    t1n = torch.empty(a.n, 32, 32, 128, device=dev, dtype=dt)
    t1r = torch.empty_like(t1n)

    def tail_conv1():
        ops.bottleneck_s2_tail_nhwc(t1, x, ws, s2, b2, shift, BF16, out=y1)
        ops.conv2d_nhwc(y1, p1n, 128, 1, 1, 1, 0, s1n, b1n, None, True, BF16, out=t1r)

    def chained():
        ops.bottleneck_s2_tail_next_nhwc(t1, x, wsn, s2, b2, shift, s1n, b1n, BF16, out=y3, t1n=t1n)

    flop = 2.0 * a.n * 1024 * (1152 * 128 + 384 * 512)
    flop_c = flop + 2.0 * a.n * 1024 * 512 * 128
    nbytes = (t1.numel() + x.numel() // 4 + y1.numel()) * 2
    for name, fn, fl in (('two launches', two, flop), ('strided tail', fused, flop),
                         ('tail + conv1', tail_conv1, flop_c), ('chained tail', chained, flop_c)):
        us = timeit(fn, a.reps, a.rounds)
        print('%-14s %8.1f us  %6.1f TFLOP/s  %5.2f TB/s (algorithmic t1 + x/4 + y)'
              % (name, us, fl / us / 1e6, nbytes / us / 1e6))
    torch.cuda.synchronize()
    print('bit-identical:', bool(torch.equal(y1, y2)), 'chained:', bool(torch.equal(y3, y1)),
          bool(torch.equal(t1n, t1r)))


if __name__ == '__main__':
    main()
