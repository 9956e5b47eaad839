"""Lost-store / race diagnosis of the fused Bottleneck kernels for one build of libposeu.so:
the output is pre-filled with a NaN sentinel, the fused launch is compared bit for bit with the
unfused launches, and the differing elements are classified (still the sentinel = a store that
never landed; another value = a wrong result) and located (channel chunk, 16-B group, tile row,
column, workgroup).   python tools/store_check.py [--lib PATH] [--reps R]"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import _native, ops, packing  # noqa: E402

SENTINEL = {torch.bfloat16: 0x7fc1, torch.float16: 0x7e01}   # quiet NaNs no kernel produces


def sentinel_like(x):
    out = torch.empty_like(x)
    out.view(torch.int16).fill_(SENTINEL[x.dtype])
    return out


def report(name, fused, ref, row_tile=8):
    lost = fused.view(torch.int16) == SENTINEL[fused.dtype]
    diff = (fused.view(torch.int16) != ref.view(torch.int16))
    nd, nl = int(diff.sum()), int(lost.sum())
    line = '%s: equal %s, differing %d, sentinel left %d' % (name, nd == 0, nd, nl)
    if nd:
        idx = diff.nonzero()
        n, h, w, c = idx.unbind(1)
        def hist(v, m):
            b = torch.bincount(v, minlength=m)
            return ' '.join('%d' % int(x) for x in b[:m])
        line += ('\n   by c//256: %s\n   by (c%%256)//8: %s\n   by h%%%d: %s\n   by w: %s\n   images %s'
                 % (hist(c // 256, (int(c.max()) // 256) + 1), hist((c % 256) // 8, 32), row_tile,
                    hist(h % row_tile, row_tile), hist(w, int(w.max()) + 1),
                    torch.unique(n)[:16].tolist()))
    print(line, flush=True)
    return nd


def tail3(code, dt, n, h, dev, seed):
    g = torch.Generator().manual_seed(seed)
    t1 = torch.randn(n, h, 16, 256, generator=g).abs().to(dev, dt)
    x = torch.randn(n, h, 16, 1024, generator=g).to(dev, dt)
    w2 = torch.randn(256, 256, 3, 3, generator=g) * 0.03
    w3 = torch.randn(1024, 256, 1, 1, generator=g) * 0.05
    s = [t.to(dev) for t in (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1,
                             torch.rand(1024, generator=g) + 0.5, torch.randn(1024, generator=g) * 0.1)]
    bk = ops.conv_bk(code)
    p2 = packing.pack_conv_weight(w2.to(dev), 256, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(dev), 256, bk, dt)
    t2 = ops.conv2d_nhwc(t1, p2, 256, 3, 3, 1, 1, s[0], s[1], None, True, code)
    two = ops.conv2d_nhwc(t2, p3, 1024, 1, 1, 1, 0, s[2], s[3], x, True, code)
    return lambda: ops.bottleneck3_tail_nhwc(t1, x, p2, s[0], s[1], p3, s[2], s[3], code, out=sentinel_like(x)), two


def block(code, dt, n, h, w, c, p, dev, seed, kind):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, h, w, c, generator=g).to(dev, dt)
    w1 = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    w2 = torch.randn(p, p, 3, 3, generator=g) * (2.0 / (9 * p)) ** 0.5
    w3 = torch.randn(c, p, 1, 1, generator=g) * (2.0 / p) ** 0.5 * 0.3
    s = [t.to(dev) for t in (torch.rand(p, generator=g) + 0.5, torch.randn(p, generator=g) * 0.1,
                             torch.rand(p, generator=g) + 0.5, torch.randn(p, generator=g) * 0.1,
                             torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1)]
    bk = ops.conv_bk(code)
    p1 = packing.pack_conv_weight(w1.to(dev), c, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(dev), p, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(dev), p, bk, dt)
    t1 = ops.conv2d_nhwc(x, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, code)
    t2 = ops.conv2d_nhwc(t1, p2, p, 3, 3, 1, 1, s[2], s[3], None, True, code)
    three = ops.conv2d_nhwc(t2, p3, c, 1, 1, 1, 0, s[4], s[5], x, True, code)
    if kind == 'l2':
        return lambda: ops.bottleneck2_nhwc(x, p1, s[0], s[1], p2, s[2], s[3], p3, s[4], s[5], code,
                                            out=sentinel_like(x)), three
    p1f = packing.pack_bottleneck_conv1_weight(w1.to(dev), dt)
    p3f = packing.pack_bottleneck_conv3_weight(w3.to(dev), dt)
    return lambda: ops.bottleneck_nhwc(x, p1f, s[0], s[1], p2, s[2], s[3], p3f, s[4], s[5], code,
                                       out=sentinel_like(x)), three


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', default=None)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--only', default='tail3,l2,l1')
    a = ap.parse_args()
    if a.lib:
        _native._LIB_PATH = os.path.abspath(a.lib)
    print('lib', _native.library_path(), flush=True)
    dev = torch.device('cuda', 0)
    bad = 0
    for code, dt in ((1, torch.bfloat16), (3, torch.float16)):
        cases = []
        if 'tail3' in a.only:
            cases += [('tail3 n%d h%d' % (n, h), 8, tail3(code, dt, n, h, dev, 5 + n)) for n, h in ((2, 16), (128, 16))]
        if 'l2' in a.only:
            cases += [('layer2 n%d' % n, 4, block(code, dt, n, 32, 32, 512, 128, dev, 9 + n, 'l2')) for n in (2, 128)]
        if 'l1' in a.only:
            cases += [('layer1 n%d' % n, 8, block(code, dt, n, 64, 64, 256, 64, dev, 13 + n, 'l1')) for n in (2, 128)]
        for name, rt, (run, ref) in cases:
            for r in range(a.reps):
                fused = run()
                torch.cuda.synchronize()
                bad += report('code %d %s rep %d' % (code, name, r), fused, ref, rt) > 0
    print('cases with differences:', bad, flush=True)


if __name__ == '__main__':
    main()
