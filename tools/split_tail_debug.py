"""Where the split streamed tail and the split conv launches differ (debug aid): per layer, the
differing elements by pixel column / channel / hi-lo half, and each path's distance to fp64."""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pose-unsupervised_amd', 'lib'))
sys.path.insert(0, os.path.join(REPO, 'tests'))
from posu import ops, packing  # noqa: E402
from test_gpu_bottleneck import _block_params, _split_pack  # noqa: E402

S = ops.F16X3
dev = torch.device('cuda', 0)
for layer, (c, p, w, n, h) in {'layer1': (256, 64, 64, 2, 64), 'layer2': (512, 128, 32, 2, 32),
                               'layer3': (1024, 256, 16, 2, 16)}.items():
    g = torch.Generator().manual_seed(131 + h + n + p)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=c, p=p)
    x = torch.randn(n, h, w, c, generator=g, dtype=torch.float64)
    xd = packing.to_split(x).to(dev)
    (p1, e1), (p2, e2), (p3, e3) = (_split_pack(t.to(dev), t.shape[1]) for t in (w1, w2, w3))
    sc = lambda bn, e: ((bn[0].double() * 2.0 ** -e).float().to(dev), bn[1].to(dev))  # noqa: E731
    s1, b1 = sc(bn1, e1)
    s2, b2 = sc(bn2, e2)
    s3, b3 = sc(bn3, e3)
    t1 = ops.conv2d_nhwc(xd, p1, p, 1, 1, 1, 0, s1, b1, None, True, S)
    y = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s2, b2, s3, b3, S)
    t2 = ops.conv2d_nhwc(t1, p2, p, 3, 3, 1, 1, s2, b2, None, True, S)
    two = ops.conv2d_nhwc(t2, p3, c, 1, 1, 1, 0, s3, b3, xd, True, S)
    torch.cuda.synchronize()
    d = (y.view(torch.int16) != two.view(torch.int16))
    idx = d.nonzero()
    print(layer, 'differing', int(d.sum()), 'of', d.numel())
    if len(idx):
        cols = torch.bincount(idx[:, 2], minlength=w)
        rows = torch.bincount(idx[:, 1], minlength=h)
        ch = idx[:, 3]
        half = (ch % 64) >= 32
        print('  by column', cols.tolist())
        print('  by row', rows.tolist()[:16])
        print('  hi %d lo %d; channel blocks' % (int((~half).sum()), int(half.sum())),
              torch.bincount(ch // 64, minlength=2 * c // 64).tolist()[:32])
        yv, tv = ops.widen(y, S), ops.widen(two, S)
        dd = (yv - tv).abs()
        print('  value diff max %.3g mean(over differing) %.3g; |y| max %.3g' % (
            float(dd.max()), float(dd[dd > 0].mean()), float(tv.abs().max())))
    # fp64 reference
    xq = ops.widen(xd, S).double().cpu().permute(0, 3, 1, 2)
    a = [t.double() for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    r1 = ops.widen(t1, S).double().cpu().permute(0, 3, 1, 2)
    r2 = F.relu(F.conv2d(r1, w2.float().double(), padding=1) * a[2].view(1, -1, 1, 1) + a[3].view(1, -1, 1, 1))
    ref = F.relu(F.conv2d(r2, w3.float().double()) * a[4].view(1, -1, 1, 1) + a[5].view(1, -1, 1, 1) + xq)
    for nm, t in (('tail', y), ('launches', two)):
        e = (ops.widen(t, S).double().cpu().permute(0, 3, 1, 2) - ref).abs()
        print('  %s vs fp64 (from the same t1): max %.3g mean %.3g' % (nm, float(e.max()), float(e.mean())))
    t2d = (ops.widen(t2, S).double().cpu().permute(0, 3, 1, 2) - r2).abs()
    print('  t2 launch vs fp64: max %.3g' % float(t2d.max()))
