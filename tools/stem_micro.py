"""Micro-benchmark of the fused multi-view stem (posu_stem_pool_views_fwd) at the bench shapes:
4 views x 32 frames at 256x256 (configs[2]) and 4 views x 16 frames at 384x384 (configs[4]).
HIP events, min over rounds; prints a checksum of the output so variant builds
(tools/variant_build.sh, run through tools/with_lib.py) can be compared bit for bit.

    python tools/stem_micro.py [--reps 20] [--rounds 3]
"""
import argparse
import hashlib
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
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--only', type=int, choices=(256, 384), help='one input size (PMC calibration runs)')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    g = torch.Generator().manual_seed(0)
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    wpk = packing.pack_stem_fused_weight(w.to(dev), torch.bfloat16)
    scale = (torch.rand(64, generator=g) + 0.5).to(dev)
    shift = (torch.randn(64, generator=g) * 0.1).to(dev)
    for nv, hw in ((32, 256), (16, 384)):
        if a.only and hw != a.only:
            continue
        views = [torch.randn(nv, 3, hw, hw, generator=g).to(dev) for _ in range(4)]
        out = ops.stem_pool_views(views, wpk, scale, shift, BF16)
        us = timeit(lambda: ops.stem_pool_views(views, wpk, scale, shift, BF16, out=out), a.reps, a.rounds)
        torch.cuda.synchronize()
        digest = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12]
        frames = 4 * nv
        gb = frames * 3 * hw * hw * 4 / 1e9 + out.numel() * 2 / 1e9
        print('stem %d views x %d @%d  %8.1f us  %6.2f TB/s (f32 input + output)  sha1 %s'
              % (4, nv, hw, us, gb / us * 1e6 / 1e3, digest))


if __name__ == '__main__':
    main()
