"""Times the weight-gradient launches (posu_conv2d_wgrad: split-K MFMA kernel + fixed-order
reduce) on the R50@256 batch-128 training shapes (bf16, HIP events, min over rounds) and prints
a checksum of every dW, so builds with the same split grouping can be compared bit for bit.

    python tools/wgrad_micro.py [--reps 10] [--rounds 3] [--lib PATH]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import _native, train_ops as T  # noqa: E402

BF16 = 1
# name, x [N, H, W, C], cout, k, stride, pad  (conv: dy [N, Ho, Wo, cout]); deconv: x plays dy
SHAPES = [
    ('l1 c1 1x1 256->64', (128, 64, 64, 256), 64, 1, 1, 0),
    ('l1 c2 3x3 64', (128, 64, 64, 64), 64, 3, 1, 1),
    ('l1 c3 1x1 64->256', (128, 64, 64, 64), 256, 1, 1, 0),
    ('l2 c2 3x3 128', (128, 32, 32, 128), 128, 3, 1, 1),
    ('l2 c1 1x1 512->128', (128, 32, 32, 512), 128, 1, 1, 0),
    ('l3 c2 3x3 256', (128, 16, 16, 256), 256, 3, 1, 1),
    ('l3 c3 1x1 256->1024', (128, 16, 16, 256), 1024, 1, 1, 0),
    ('l4 c2 3x3 512', (128, 8, 8, 512), 512, 3, 1, 1),
    ('l4 c3 1x1 512->2048', (128, 8, 8, 512), 2048, 1, 1, 0),
    ('deconv1 2048->256', 'd', (128, 8, 8, 2048), 256),
    ('deconv3 256->256', 'd', (128, 32, 32, 256), 256),
]


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
    ap.add_argument('--lib', default=None, help='another build of libposeu.so (experiments)')
    ap.add_argument('--reps', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    dt = torch.bfloat16
    total = 0.0
    for sh in SHAPES:
        name = sh[0]
        if sh[1] == 'd':
            n, h, w, cin = sh[2]
            cout = sh[3]
            x = torch.randn(n, h, w, cin, device=dev, generator=g).to(dt)
            dy = torch.randn(n, 2 * h, 2 * w, cout, device=dev, generator=g).to(dt)
            fn = lambda x=x, dy=dy: T.deconv4x4s2_wgrad(x, dy, BF16)  # noqa: E731
            flop = 2.0 * n * h * w * cin * cout * 16
        else:
            (n, h, w, cin), cout, k, stride, pad = sh[1:]
            ho, wo = (h + 2 * pad - k) // stride + 1, (w + 2 * pad - k) // stride + 1
            x = torch.randn(n, h, w, cin, device=dev, generator=g).to(dt)
            dy = torch.randn(n, ho, wo, cout, device=dev, generator=g).to(dt)
            fn = lambda x=x, dy=dy, cin=cin, k=k, stride=stride, pad=pad: T.conv2d_wgrad(  # noqa: E731
                dy, x, cin, k, k, stride, pad, BF16)
            flop = 2.0 * n * ho * wo * cout * k * k * cin
        us = timeit(fn, a.reps, a.rounds)
        total += us
        dw = fn()
        torch.cuda.synchronize()
        print('%-22s %8.1f us %6.0f TF  checksum %.9e' % (name, us, flop / us / 1e6, float(dw.double().sum())),
              flush=True)
    print('sum %.1f us' % total)


if __name__ == '__main__':
    main()
