"""Times the fused last deconv + 1x1 head (posu_deconv4x4s2_head_fwd) on the R50@256 batch-128
shape (bf16, HIP events, min over rounds) for one build of the library, and prints a checksum
of the heatmaps so that builds can be compared bit for bit.

    python tools/head_micro.py [--lib PATH] [--reps 10] [--rounds 3]
"""
import argparse
import hashlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import _native, ops  # noqa: E402

BF16 = 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=None)
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    n, h, w, cin, cout, j = 128, 32, 32, 256, 256, 16
    x = torch.randn(n, h, w, cin, device=dev, generator=g).to(torch.bfloat16)
    wk = (torch.randn(4, cout, 4 * cin, device=dev, generator=g) * 0.03).to(torch.bfloat16)
    sc = torch.rand(cout, device=dev, generator=g) + 0.5
    sh = torch.randn(cout, device=dev, generator=g) * 0.1
    hw = torch.zeros(16, cout, device=dev, dtype=torch.bfloat16)
    hw[:j] = (torch.randn(j, cout, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    hb = torch.randn(j, device=dev, generator=g) * 0.1
    fn = lambda: ops.deconv4x4s2_head(x, wk, cout, sc, sh, hw, j, hb, BF16, keep_f=False)[0]  # noqa: E731
    hm = fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(a.rounds):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / a.reps)
    flop = 2.0 * n * (2 * h) * (2 * w) * cout * (4 * cin + j)
    digest = hashlib.sha1(hm.cpu().numpy().tobytes()).hexdigest()[:16]
    print('deconv3+head %s: %7.1f us %6.0f TF | hm sha1 %s finite %s' % (
        os.path.basename(a.lib or 'libposeu.so'), best, flop / best / 1e6, digest, bool(torch.isfinite(hm).all())))


if __name__ == '__main__':
    main()
