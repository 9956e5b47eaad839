"""Split-K micro-benchmark: for the under-filled conv GEMMs of R50@256 at batch 128 (layer4,
layer3's strided conv2), every plain tile candidate against the split-K candidates
(plan._split_candidates), HIP-event time per launch, best of two passes.
    python tools/splitk_micro.py [--reps 20] [--lib PATH]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

GEOMS = [  # name, input NHWC, cout, k, stride, residual
    ('layer3.0 conv2 s2', (128, 32, 32, 256), 256, 3, 2, False),
    ('layer3.1 conv1', (128, 16, 16, 1024), 256, 1, 1, False),
    ('layer4.0 conv1', (128, 16, 16, 1024), 512, 1, 1, False),
    ('layer4.0 conv2 s2', (128, 16, 16, 512), 512, 3, 2, False),
    ('layer4.x conv1', (128, 8, 8, 2048), 512, 1, 1, False),
    ('layer4.x conv2', (128, 8, 8, 512), 512, 3, 1, False),
    ('layer4.x conv3+res', (128, 8, 8, 512), 2048, 1, 1, True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--lib', default=None)
    a = ap.parse_args()
    if a.lib:
        from posu import _native
        _native._LIB_PATH = os.path.abspath(a.lib)
    from posu import ops, packing, plan as P
    from posu._native import BF16
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    code, dt = BF16, torch.bfloat16
    for name, shp, cout, k, stride, residual in GEOMS:
        n, h, w, c = shp
        pad = k // 2
        ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
        x = torch.randn(shp, device=dev, generator=g).to(dt)
        wt = torch.randn(cout, c, k, k, device=dev, generator=g) * (2.0 / (c * k * k)) ** 0.5
        wp = packing.pack_conv_weight(wt, c, 64, dt)
        sc = torch.rand(cout, device=dev, generator=g) + 0.5
        sh = torch.randn(cout, device=dev, generator=g) * 0.1
        res = torch.randn(n, ho, wo, cout, device=dev, generator=g).to(dt) if residual else None
        out = torch.empty(n, ho, wo, cout, device=dev, dtype=dt)

        def launch(t):
            if t >= 100:
                return ops.conv2d_nhwc_splitk(x, wp, cout, k, k, stride, pad, sc, sh, res, True, code, t % 100,
                                              t // 100, out=out)
            return ops.conv2d_nhwc(x, wp, cout, k, k, stride, pad, sc, sh, res, True, code, out=out, tile=t)
        plain = P._tile_candidates(cout)
        split = P._split_candidates(n * ho * wo, cout, wp.shape[1], code)
        times = {}
        for order in (plain + split, (plain + split)[::-1]):
            for t in order:
                launch(t)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record()
                for _ in range(a.reps):
                    launch(t)
                ev[1].record()
                ev[1].synchronize()
                us = ev[0].elapsed_time(ev[1]) * 1e3 / a.reps
                times[t] = min(us, times.get(t, us))
        flops = 2.0 * n * ho * wo * cout * k * k * c
        bp = min(plain, key=lambda t: times[t])
        line = '%-20s plain best tile %3d %7.1f us (%5.0f TF/s)' % (name, bp, times[bp], flops / times[bp] / 1e6)
        if split:
            bs = min(split, key=lambda t: times[t])
            line += ' | split best %4d %7.1f us (%5.0f TF/s)' % (bs, times[bs], flops / times[bs] / 1e6)
            line += ' | ' + ' '.join('%d:%.1f' % (t, times[t]) for t in split)
        print(line, flush=True)


if __name__ == '__main__':
    main()
