"""Micro-benchmark of the training BatchNorm passes (posu_bn_train_fwd / posu_bn_apply /
posu_bn_train_bwd) at the R50@256 training-step shapes (128 frames = 4 view segments),
HIP events, one process, min over rounds.  Reports algorithmic HBM bytes / time.

    python tools/bn_micro.py [--reps 20] [--rounds 3]

Run under `rocprofv3 --kernel-trace --stats` for the per-kernel split.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import train_ops as T  # noqa: E402

SHAPES = [(128, 64, 64, 256), (128, 64, 64, 64), (128, 32, 32, 512), (128, 16, 16, 1024), (128, 8, 8, 2048)]
NSEG = 4


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
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--lib', default=None, help='another build of libposeu.so (experiments)')
    ap.add_argument('--frames', type=int, default=128, help='batch of the shapes (32: one view of the 4)')
    ap.add_argument('--nseg', type=int, default=NSEG)
    args = ap.parse_args()
    if args.lib:
        from posu import _native
        _native._LIB_PATH = os.path.abspath(args.lib)
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    total = 0.0
    for shp in SHAPES:
        shp = (args.frames,) + tuple(shp[1:])
        c = shp[-1]
        z = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        r = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        gy = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        gamma = torch.rand(c, device=dev) + 0.5
        beta = torch.randn(c, device=dev)
        nb = z.numel() * 2
        mean, rstd, sc, sh = T.bn_train_fwd(z, args.nseg, gamma, beta, 1e-5, 0.1)
        y = T.bn_apply(z, args.nseg, sc, sh, r, True)
        _, mask = T.bn_apply_mask(z, args.nseg, sc, sh, r)
        out = torch.empty_like(z)
        cases = [
            ('stats', lambda: T.bn_train_fwd(z, args.nseg, gamma, beta, 1e-5, 0.1), 1),
            ('apply', lambda: T.bn_apply(z, args.nseg, sc, sh, None, True, out=out), 2),
            ('apply+res', lambda: T.bn_apply(z, args.nseg, sc, sh, r, True, out=out), 3),
            ('bwd(y,gres)', lambda: T.bn_train_bwd(gy, y, z, args.nseg, mean, rstd, gamma, want_gres=True), 8),
            ('bwd(mask,gres)', lambda: T.bn_train_bwd(gy, None, z, args.nseg, mean, rstd, gamma, want_gres=True,
                                                      mask=mask), 6),
            ('bwd(relu_from)', lambda: T.bn_train_bwd(gy, None, z, args.nseg, mean, rstd, gamma, relu_from=(sc, sh)), 5),
        ]
        for name, fn, passes in cases:
            us = timeit(fn, args.reps, args.rounds)
            total += us
            print('%-22s %-14s %8.1f us  %5.2f TB/s' % (str(shp), name, us, passes * nb / us / 1e6))
    print('TOTAL %.1f us' % total)


if __name__ == '__main__':
    main()
