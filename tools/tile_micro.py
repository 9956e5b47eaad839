"""Times conv tile configurations on the compute-heavy R50@256 batch-128 layer shapes (bf16,
HIP events, min over rounds) and checks that loops with the same K order agree bit for bit.

    python tools/tile_micro.py [--tiles 5,23,37] [--reps 10] [--rounds 3] [--lib PATH] [--flush]

--flush: every launch timed alone (its own HIP events) after a 512 MB write that evicts the L2s
and the Infinity Cache, median over reps x rounds -- the cold-cache figure beside the warm one.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import _native, ops  # noqa: E402

BF16 = 1
# name, kind, (n, h, w, cin), cout, k
SHAPES = [
    ('deconv3 32->64', 'deconv', (128, 32, 32, 256), 256, 4),
    ('deconv2 16->32', 'deconv', (128, 16, 16, 256), 256, 4),
    ('deconv1 8->16', 'deconv', (128, 8, 8, 2048), 256, 4),
    ('l3 c2 3x3 16x16x256', 'conv', (128, 16, 16, 256), 256, 3),
    ('l4 c2 3x3 8x8x512', 'conv', (128, 8, 8, 512), 512, 3),
    ('l2 c2 3x3 32x32x128', 'conv', (128, 32, 32, 128), 128, 3),
    ('l3 c1 1x1 16x16x1024', 'conv', (128, 16, 16, 1024), 256, 1),
    ('l4 c3 1x1 8x8x512', 'conv', (128, 8, 8, 512), 2048, 1),
    ('l4 c1 1x1 8x8x2048', 'conv', (128, 8, 8, 2048), 512, 1),
    ('l3 c3 1x1 16x16x256', 'conv', (128, 16, 16, 256), 1024, 1),
]


def timeit_cold(fn, reps, rounds, junk, touch=()):
    ts = []
    for _ in range(reps * rounds):
        junk.fill_(1.0)
        for t in touch:   # re-read after the eviction (torch reductions): which operand's fetch costs
            t.sum(dtype=torch.float32)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


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
    ap.add_argument('--tiles', default='5,23,37')
    ap.add_argument('--lib', default=None, help='another build of libposeu.so (experiments)')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--only', default='', help='comma-separated substrings of the shape names to run')
    ap.add_argument('--flush', action='store_true', help='cold caches: evict before every timed launch')
    ap.add_argument('--touch', default='', choices=('', 'w', 'x', 'wx'),
                    help='with --flush: re-read the weights (w), the input (x) or both after the eviction')
    a = ap.parse_args()
    tiles = [int(t) for t in a.tiles.split(',')]
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    dt = torch.bfloat16
    bk = ops.conv_bk(BF16)
    junk = torch.empty(128 << 20, device=dev, dtype=torch.float32) if a.flush else None
    for name, kind, (n, h, w, cin), cout, k in SHAPES:
        if a.only and not any(o in name for o in a.only.split(',')):
            continue
        x = torch.randn(n, h, w, cin, device=dev, generator=g).to(dt)
        sc = torch.rand(cout, device=dev, generator=g) + 0.5
        sh = torch.randn(cout, device=dev, generator=g) * 0.1
        if kind == 'deconv':
            wk = (torch.randn(4, cout, 4 * cin, device=dev, generator=g) * 0.03).to(dt)
            flop = 2.0 * n * (2 * h) * (2 * w) * cout * 4 * cin
            fn = lambda t, x=x, wk=wk, cout=cout, sc=sc, sh=sh: ops.deconv4x4s2_nhwc(x, wk, cout, sc, sh, True, BF16, tile=t)
        else:
            kk = k * k * cin
            kp = (kk + bk - 1) // bk * bk
            wk = torch.zeros(cout, kp, device=dev, dtype=dt)
            wk[:, :kk] = (torch.randn(cout, kk, device=dev, generator=g) * 0.03).to(dt)
            flop = 2.0 * n * h * w * cout * kk
            fn = lambda t, x=x, wk=wk, cout=cout, k=k, sc=sc, sh=sh: ops.conv2d_nhwc(
                x, wk, cout, k, k, 1, k // 2, sc, sh, None, True, BF16, tile=t)
        outs, line = {}, []
        for t in tiles:
            try:
                outs[t] = fn(t)
            except RuntimeError as e:
                line.append('%d: n/a' % t)
                continue
            touch = [v for k, v in (('w', wk), ('x', x)) if k in a.touch]
            us = timeit_cold(lambda: fn(t), a.reps, a.rounds, junk, touch) if a.flush else timeit(lambda: fn(t), a.reps, a.rounds)
            line.append('%d: %7.1f us %6.0f TF' % (t, us, flop / us / 1e6))
        torch.cuda.synchronize()
        ref = outs.get(tiles[0])
        same = ' '.join('%d=%s' % (t, 'eq' if torch.equal(ref, o) else 'DIFF %.3g' % float((ref.float() - o.float()).abs().max()))
                        for t, o in outs.items() if t != tiles[0]) if ref is not None else ''
        print('%-24s %s | %s' % (name, ' | '.join(line), same))


if __name__ == '__main__':
    main()
