"""Does a BatchNorm pass pair (statistics then apply; backward sums then apply) run faster one view
segment at a time, so that the second pass re-reads a segment the first left in the Infinity Cache
(256 MB) instead of HBM?  Times, at the training step's large shapes, the pair over all 4 segments
in one call against 4 calls of one segment each (same kernels, nseg = 1 slices), HIP events.

    python tools/bn_seg_micro.py [--reps 20]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import train_ops as T  # noqa: E402

SHAPES = [(128, 64, 64, 256), (128, 64, 64, 64), (128, 32, 32, 512), (128, 32, 32, 128)]
NSEG = 4


def timeit(fn, reps):
    best = 1e9
    for _ in range(3):
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
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for shp in SHAPES:
        n, c = shp[0], shp[-1]
        b = n // NSEG
        z = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        r = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        gy = torch.randn(shp, device=dev, generator=g).to(torch.bfloat16)
        gamma = torch.rand(c, device=dev) + 0.5
        beta = torch.randn(c, device=dev)
        mean, rstd, sc, sh = T.bn_train_fwd(z, NSEG, gamma, beta, 1e-5, 0.1)
        y, mask = T.bn_apply_mask(z, NSEG, sc, sh, r)
        mrows = mask.view(n, -1)
        zs = [z[k * b:(k + 1) * b] for k in range(NSEG)]
        rs = [r[k * b:(k + 1) * b] for k in range(NSEG)]
        gs = [gy[k * b:(k + 1) * b] for k in range(NSEG)]
        ms = [mrows[k * b:(k + 1) * b].reshape(-1) for k in range(NSEG)]

        def fwd_all():
            st = T.bn_train_fwd(z, NSEG, gamma, beta, 1e-5, 0.1)
            T.bn_apply_mask(z, NSEG, st[2], st[3], r)

        def fwd_seg():
            for k in range(NSEG):
                st = T.bn_train_fwd(zs[k], 1, gamma, beta, 1e-5, 0.1)
                T.bn_apply_mask(zs[k], 1, st[2], st[3], rs[k])

        def bwd_all():
            T.bn_train_bwd(gy, None, z, NSEG, mean, rstd, gamma, want_gres=True, mask=mask)

        def bwd_seg():
            for k in range(NSEG):
                T.bn_train_bwd(gs[k], None, zs[k], 1, mean[k], rstd[k], gamma, want_gres=True, mask=ms[k])

        res = [timeit(f, args.reps) for f in (fwd_all, fwd_seg, bwd_all, bwd_seg)]
        print('%-20s fwd (stats+apply) all %7.1f  per-segment %7.1f us | bwd (sums+apply) all %7.1f  per-segment '
              '%7.1f us' % (str(shp), *res))


if __name__ == '__main__':
    main()
