"""Micro-benchmark of the chained streamed tail (posu_bottleneck_tail_stream_next_fwd) at the
bench shape (128 frames, bf16): identity block i's tail + block i+1's conv1 as a separate conv
launch over y, vs the chained tail that produces y and the next conv1 output t1n in one launch.
HIP events, min over rounds; y and t1n checked bit for bit against the two-launch path, with the
chained outputs pre-filled with a NaN sentinel.

    python tools/chain_micro.py [--n 128] [--reps 20] [--rounds 3] [--lib PATH]
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
        w1n = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
        s = [t.to(dev) for ch in (p, p, c, p) for t in (torch.rand(ch, generator=g) + 0.5,
                                                         torch.randn(ch, generator=g) * 0.1)]
        p1 = packing.pack_conv_weight(w1.to(dev), c, bk, dt)
        p2 = packing.pack_conv_weight(w2.to(dev), p, bk, dt)
        p3 = packing.pack_conv_weight(w3.to(dev), p, bk, dt)
        p1n = packing.pack_conv_weight(w1n.to(dev), c, bk, dt)
        wst = packing.pack_tail_stream(p2, p3)
        wsn = packing.pack_tail_stream(p2, p3, p1n)
        t1 = ops.conv2d_nhwc(x, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, BF16)
        y_ref, t1n_ref = torch.empty_like(x), torch.empty_like(t1)
        y_ch = torch.full_like(x, float('nan'))
        t1n_ch = torch.full_like(t1, float('nan'))

        def two():
            ops.bottleneck_tail_stream_nhwc(t1, x, wst, s[2], s[3], s[4], s[5], BF16, out=y_ref)
            ops.conv2d_nhwc(y_ref, p1n, p, 1, 1, 1, 0, s[6], s[7], None, True, BF16, out=t1n_ref)

        def chained():
            ops.bottleneck_tail_stream_next_nhwc(t1, x, wsn, s[2], s[3], s[4], s[5], s[6], s[7], BF16, out=y_ch,
                                                 t1n=t1n_ch)

        two()
        chained()
        torch.cuda.synchronize()
        eq_y, eq_t = bool(torch.equal(y_ref, y_ch)), bool(torch.equal(t1n_ref, t1n_ch))
        ndiff = int((t1n_ref != t1n_ch).sum())
        def plain():
            ops.bottleneck_tail_stream_nhwc(t1, x, wst, s[2], s[3], s[4], s[5], BF16, out=y_ref)

        us_2, us_c = timeit(two, a.reps, a.rounds), timeit(chained, a.reps, a.rounds)
        us_p = timeit(plain, a.reps, a.rounds)
        print('%s batch %d: tail %.1f us | tail + next conv1 launch %.1f us | chained tail %.1f us | y bit-identical '
              '%s, t1n bit-identical %s (%d differ)' % (layer, a.n, us_p, us_2, us_c, eq_y, eq_t, ndiff), flush=True)


if __name__ == '__main__':
    main()
