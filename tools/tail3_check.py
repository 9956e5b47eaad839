"""Bit-exactness check of posu_bottleneck3_tail_fwd against conv2 + conv3 as two launches for a
given build of libposeu.so (diagnostics of kernel variants):  python tools/tail3_check.py [--lib PATH]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import _native, ops, packing  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=None)
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    dev = torch.device('cuda', 0)
    for code, dt in ((1, torch.bfloat16), (3, torch.float16)):
        for n, h in ((2, 16), (128, 16), (3, 24)):
            g = torch.Generator().manual_seed(5 + n)
            t1 = torch.randn(n, h, 16, 256, generator=g).abs().to(dev, dt)
            x = torch.randn(n, h, 16, 1024, generator=g).to(dev, dt)
            w2 = torch.randn(256, 256, 3, 3, generator=g) * 0.03
            w3 = torch.randn(1024, 256, 1, 1, generator=g) * 0.05
            s = [t.to(dev) for t in (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1,
                                     torch.rand(1024, generator=g) + 0.5, torch.randn(1024, generator=g) * 0.1)]
            bk = ops.conv_bk(code)
            p2 = packing.pack_conv_weight(w2.to(dev), 256, bk, dt)
            p3 = packing.pack_conv_weight(w3.to(dev), 256, bk, dt)
            fused = ops.bottleneck3_tail_nhwc(t1, x, p2, s[0], s[1], p3, s[2], s[3], code)
            t2 = ops.conv2d_nhwc(t1, p2, 256, 3, 3, 1, 1, s[0], s[1], None, True, code)
            two = ops.conv2d_nhwc(t2, p3, 1024, 1, 1, 1, 0, s[2], s[3], x, True, code)
            torch.cuda.synchronize()
            d = (fused.float() - two.float()).abs()
            print('code %d n %d h %d: equal %s, differing %d, nan %d' % (
                code, n, h, bool(torch.equal(fused, two)), int((d > 0).sum()), int(torch.isnan(fused).sum())))


if __name__ == '__main__':
    main()
