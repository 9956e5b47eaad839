"""The fused Bottleneck launches (posu_bottleneck_fwd / posu_bottleneck_down_fwd,
csrc/bottleneck.hip) against the unfused launches on the same device and against torch fp32
on CPU (eval-mode Bottleneck, reference lib/models/pose_resnet.py:61-99, downsample
pose_resnet.py:136-141), plus the whole R50 plan with the fused layer1 blocks against the
unfused plan."""
import pytest
import torch
import torch.nn.functional as F

from posu import ops, packing, synthetic as syn
from posu._native import BF16, F16

pytestmark = pytest.mark.gpu


def _block_params(g, c=256, p=64):
    def bn(ch):
        return (torch.rand(ch, generator=g) + 0.5, torch.randn(ch, generator=g) * 0.1)
    w1 = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    w2 = torch.randn(p, p, 3, 3, generator=g) * (2.0 / (9 * p)) ** 0.5
    w3 = torch.randn(c, p, 1, 1, generator=g) * (2.0 / p) ** 0.5 * 0.3
    return w1, bn(p), w2, bn(p), w3, bn(c)


def _sentinel(like, shape=None):
    """Output buffer pre-filled with a quiet-NaN pattern no kernel produces: a store that never
    lands (or lands elsewhere) leaves it behind and fails the comparisons below."""
    out = torch.empty(like.shape if shape is None else shape, dtype=like.dtype, device=like.device)
    out.view(torch.int16).fill_(0x7fc1 if like.dtype == torch.bfloat16 else 0x7e01)
    return out


def _torch_block(x, w1, bn1, w2, bn2, w3, bn3):
    t = F.relu(F.conv2d(x, w1) * bn1[0].view(1, -1, 1, 1) + bn1[1].view(1, -1, 1, 1))
    t = F.relu(F.conv2d(t, w2, padding=1) * bn2[0].view(1, -1, 1, 1) + bn2[1].view(1, -1, 1, 1))
    t = F.conv2d(t, w3) * bn3[0].view(1, -1, 1, 1) + bn3[1].view(1, -1, 1, 1)
    return F.relu(t + x)


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h', [(3, 10), (1, 2), (2, 64), (1, 7), (5, 64), (128, 64)])
def test_fused_bottleneck_matches_three_launches_and_torch(cuda, code, n, h):
    """(128, 64) is the production grid (256 workgroups): against the unfused launches only."""
    g = torch.Generator().manual_seed(17 + h)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g)
    x = torch.randn(n, 256, h, 64, generator=g)
    dt = ops.torch_dtype(code)
    xq = x.to(dt).float()   # the input as the device sees it
    ref = _torch_block(xq, w1, bn1, w2, bn2, w3, bn3) if n < 128 else None
    bk = ops.conv_bk(code)
    xd = xq.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    p1 = packing.pack_conv_weight(w1.to(cuda), 256, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(cuda), 64, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(cuda), 64, bk, dt)
    p3f = packing.pack_bottleneck_conv3_weight(w3.to(cuda), dt)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    p1f = packing.pack_bottleneck_conv1_weight(w1.to(cuda), dt)
    fused = ops.bottleneck_nhwc(xd, p1f, s[0], s[1], p2, s[2], s[3], p3f, s[4], s[5], code, out=_sentinel(xd))
    t1 = ops.conv2d_nhwc(xd, p1, 64, 1, 1, 1, 0, s[0], s[1], None, True, code)
    t2 = ops.conv2d_nhwc(t1, p2, 64, 3, 3, 1, 1, s[2], s[3], None, True, code)
    three = ops.conv2d_nhwc(t2, p3, 256, 1, 1, 1, 0, s[4], s[5], xd, True, code)
    torch.cuda.synchronize()
    # conv1 / conv3 sum their channels in other orders: t1 may differ in its last bit, which
    # conv2 / conv3 carry along (a flipped t1 bit enters 576 products of conv2, a flipped t2
    # bit 64 of conv3): on average a small fraction of an ulp, ~10 ulps at the worst element
    # of the 5 x 64 x 64 x 256 case
    d = (fused.float() - three.float()).abs()
    ulp = (2.0 ** -7 if code == BF16 else 2.0 ** -10) * three.float().abs().clamp_min(2.0 ** -4)
    assert float(d.mean()) < 0.05 * float(ulp.mean()), float(d.mean())
    # the worst of 134 M elements at N = 128 (fp16) sits at ~18 ulp
    assert bool((d <= (16 if n < 128 else 32) * ulp).all()), float((d / ulp).max())
    if ref is None:
        return
    got = fused.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs()
    tol = 0.05 if code == BF16 else 0.01
    assert float(err.max()) <= tol * float(ref.abs().max()) + tol, float(err.max())


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h', [(3, 10), (1, 2), (2, 64), (1, 7), (5, 64), (128, 64)])
def test_fused_first_bottleneck_matches_unfused_launches_and_torch(cuda, code, n, h):
    """Layer1 block 0: 64 input channels, downsample 1x1 + BN as the residual branch."""
    g = torch.Generator().manual_seed(29 + h)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=64)
    w3 = torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5 * 0.3
    bn3 = (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1)
    wd = torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5 * 0.3
    bnd = (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1)
    x = torch.randn(n, 64, h, 64, generator=g).abs()   # a maxpool output of ReLUs
    dt = ops.torch_dtype(code)
    xq = x.to(dt).float()
    t = F.relu(F.conv2d(xq, w1) * bn1[0].view(1, -1, 1, 1) + bn1[1].view(1, -1, 1, 1))
    t = F.relu(F.conv2d(t, w2, padding=1) * bn2[0].view(1, -1, 1, 1) + bn2[1].view(1, -1, 1, 1))
    ref = F.relu(F.conv2d(t, w3) * bn3[0].view(1, -1, 1, 1) + bn3[1].view(1, -1, 1, 1) +
                 F.conv2d(xq, wd) * bnd[0].view(1, -1, 1, 1) + bnd[1].view(1, -1, 1, 1)) if n < 128 else None
    bk = ops.conv_bk(code)
    xd = xq.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    p1 = packing.pack_conv_weight(w1.to(cuda), 64, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(cuda), 64, bk, dt)
    s = [v.to(cuda) for v in (bn1[0], bn1[1], bn2[0], bn2[1])]
    pdual = packing.pack_dual_1x1_weight(w3.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), dt)
    shift = (bn3[1].double() + bnd[1].double()).float().to(cuda)
    fused = ops.bottleneck_down_nhwc(xd, p1, s[0], s[1], p2, s[2], s[3],
                                     packing.pack_bottleneck_down_weight(pdual, 64), shift, code,
                                     out=_sentinel(xd, (n, h, 64, 256)))
    t1 = ops.conv2d_nhwc(xd, p1, 64, 1, 1, 1, 0, s[0], s[1], None, True, code)
    t2 = ops.conv2d_nhwc(t1, p2, 64, 3, 3, 1, 1, s[2], s[3], None, True, code)
    unfused = ops.conv1x1_dual_nhwc(t2, xd, 1, pdual, 256, shift, True, code)
    torch.cuda.synchronize()
    # conv1 sums in the unfused order; conv3 in a permuted one (last-bit differences of t2
    # products only)
    d = (fused.float() - unfused.float()).abs()
    ulp = (2.0 ** -7 if code == BF16 else 2.0 ** -10) * unfused.float().abs().clamp_min(2.0 ** -4)
    assert float(d.mean()) < 0.05 * float(ulp.mean()), float(d.mean())
    assert bool((d <= (16 if n < 128 else 32) * ulp).all()), float((d / ulp).max())
    if ref is None:
        return
    got = fused.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs()
    tol = 0.05 if code == BF16 else 0.01
    assert float(err.max()) <= tol * float(ref.abs().max()) + tol, float(err.max())


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h,w', [(2, 32, 32), (1, 4, 32), (3, 8, 32), (1, 12, 32), (128, 32, 32), (1, 16, 32),
                                   (2, 48, 48), (1, 2, 48), (3, 10, 48), (64, 48, 48)])
def test_fused_layer2_bottleneck_matches_three_launches_and_torch(cuda, code, n, h, w):
    """Layer2's identity block (32-wide maps at 256x256, 48-wide at 384x384; 512 channels, planes
    128) as conv1 + the register-streamed tail (4-row / 2-row tiles): bit-identical to the three unfused launches (same K
    order per accumulator, same epilogue arithmetic) and within the dtype's tolerance of torch
    fp32."""
    g = torch.Generator().manual_seed(41 + h + w)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=512, p=128)
    x = torch.randn(n, 512, h, w, generator=g)
    dt = ops.torch_dtype(code)
    xq = x.to(dt).float()
    ref = _torch_block(xq, w1, bn1, w2, bn2, w3, bn3) if n < 64 else None
    bk = ops.conv_bk(code)
    xd = xq.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    p1 = packing.pack_conv_weight(w1.to(cuda), 512, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(cuda), 128, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(cuda), 128, bk, dt)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 128, 1, 1, 1, 0, s[0], s[1], None, True, code)
    fused = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5],
                                            code, out=_sentinel(xd))
    t2 = ops.conv2d_nhwc(t1, p2, 128, 3, 3, 1, 1, s[2], s[3], None, True, code)
    three = ops.conv2d_nhwc(t2, p3, 512, 1, 1, 1, 0, s[4], s[5], xd, True, code)
    torch.cuda.synchronize()
    d = (fused.float() - three.float()).abs()
    print('layer2 streamed tail vs three launches: max %.3g, differing elements %d'
          % (float(d.max()), int((d > 0).sum())))
    assert torch.equal(fused, three)
    if ref is None:
        return
    got = fused.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs()
    tol = 0.05 if code == BF16 else 0.01
    assert float(err.max()) <= tol * float(ref.abs().max()) + tol, float(err.max())


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h,w', [(2, 16, 16), (1, 8, 16), (3, 24, 16), (128, 16, 16),
                                   (2, 24, 24), (1, 6, 24), (3, 18, 24), (64, 24, 24)])
def test_fused_layer3_tail_matches_two_launches_and_torch(cuda, code, n, h, w):
    """Layer3's identity block tail (16-wide maps at 256x256, 24-wide at 384x384 -- R152's 36
    blocks, m-tiles straddling image rows --, 1024 channels, planes 256): conv2 + conv3 (+
    residual) in one launch, bit-identical to the two unfused launches (conv_igemm's K order per
    accumulator, same epilogue arithmetic) and within the dtype's tolerance of torch fp32.
    (128, 16, 16) / (64, 24, 24): the production grids, against the launches only."""
    g = torch.Generator().manual_seed(71 + h + w)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=1024, p=256)
    x = torch.randn(n, 1024, h, w, generator=g)
    dt = ops.torch_dtype(code)
    xq = x.to(dt).float()
    ref = _torch_block(xq, w1, bn1, w2, bn2, w3, bn3) if n < 64 else None
    bk = ops.conv_bk(code)
    xd = xq.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    p1 = packing.pack_conv_weight(w1.to(cuda), 1024, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(cuda), 256, bk, dt)
    p3 = packing.pack_conv_weight(w3.to(cuda), 256, bk, dt)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 256, 1, 1, 1, 0, s[0], s[1], None, True, code)
    fused = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5],
                                            code, out=_sentinel(xd))
    t2 = ops.conv2d_nhwc(t1, p2, 256, 3, 3, 1, 1, s[2], s[3], None, True, code)
    two = ops.conv2d_nhwc(t2, p3, 1024, 1, 1, 1, 0, s[4], s[5], xd, True, code)
    torch.cuda.synchronize()
    d = (fused.float() - two.float()).abs()
    print('layer3 tail register-streamed vs two launches: max %.3g, differing elements %d'
          % (float(d.max()), int((d > 0).sum())))
    assert torch.equal(fused, two)
    if ref is None:
        return
    got = fused.float().cpu().permute(0, 3, 1, 2)
    err = (got - ref).abs()
    tol = 0.05 if code == BF16 else 0.01
    assert float(err.max()) <= tol * float(ref.abs().max()) + tol, float(err.max())


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h', [(1, 8), (2, 16), (3, 24), (1, 64), (128, 64)])
def test_layer2_first_block_strided_tail_matches_two_launches_and_torch(cuda, code, n, h):
    """Layer2's first block after its conv1 launch: conv2 (3x3 / stride 2) + the conv3 | downsample
    dual GEMM in one launch (posu_bottleneck_s2_tail_fwd), bit-identical to the two launches it
    replaces (same MFMA sequence per accumulator) with every output written (NaN sentinel), and
    within the dtype's tolerance of torch fp32.  (128, 64) is the production grid (2048
    workgroups)."""
    g = torch.Generator().manual_seed(91 + h)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=512, p=128)
    w1 = w1[:, :256].contiguous() * 2 ** 0.5          # conv1 256 -> 128
    wd = torch.randn(512, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5 * 0.3
    bnd = (torch.rand(512, generator=g) + 0.5, torch.randn(512, generator=g) * 0.1)
    x = torch.randn(n, 256, h, 64, generator=g).abs()
    dt = ops.torch_dtype(code)
    xq = x.to(dt).float()
    bk = ops.conv_bk(code)
    xd = xq.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    p1 = packing.pack_conv_weight(w1.to(cuda), 256, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(cuda), 128, bk, dt)
    pdual = packing.pack_dual_1x1_weight(w3.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), dt)
    shift = (bn3[1].double() + bnd[1].double()).float().to(cuda)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 128, 1, 1, 1, 0, s[0], s[1], None, True, code)
    fused = ops.bottleneck_s2_tail_nhwc(t1, xd, packing.pack_s2_tail_stream(p2, pdual), s[2], s[3], shift, code,
                                        out=_sentinel(xd, (n, h // 2, 32, 512)))
    t2 = ops.conv2d_nhwc(t1, p2, 128, 3, 3, 2, 1, s[2], s[3], None, True, code)
    two = ops.conv1x1_dual_nhwc(t2, xd, 2, pdual, 512, shift, True, code)
    torch.cuda.synchronize()
    d = (fused.float() - two.float()).abs()
    print('layer2 strided tail vs two launches: max %.3g, differing elements %d' % (float(d.max()), int((d > 0).sum())))
    assert torch.equal(fused, two)
    if n >= 128:
        return
    t1r = F.relu(F.conv2d(xq, w1) * bn1[0].view(1, -1, 1, 1) + bn1[1].view(1, -1, 1, 1))
    t2r = F.relu(F.conv2d(t1r, w2, stride=2, padding=1) * bn2[0].view(1, -1, 1, 1) + bn2[1].view(1, -1, 1, 1))
    ref = F.relu(F.conv2d(t2r, w3) * bn3[0].view(1, -1, 1, 1) + bn3[1].view(1, -1, 1, 1) +
                 F.conv2d(xq, wd, stride=2) * bnd[0].view(1, -1, 1, 1) + bnd[1].view(1, -1, 1, 1))
    err = (fused.float().cpu().permute(0, 3, 1, 2) - ref).abs()
    tol = 0.05 if code == BF16 else 0.01
    assert float(err.max()) <= tol * float(ref.abs().max()) + tol, float(err.max())


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h', [(1, 8), (2, 16), (3, 24), (128, 64)])
def test_chained_strided_tail_matches_tail_and_next_conv1(cuda, code, n, h):
    """posu_bottleneck_s2_tail_next_fwd: the strided tail computing layer2 block 1's conv1 + BN1 +
    ReLU over its output while it is produced.  y and t1n are bit-identical to the plain strided
    tail followed by a conv launch of that conv1 over y; both outputs start as NaN sentinels."""
    g = torch.Generator().manual_seed(191 + h + n)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=512, p=128)
    w1 = w1[:, :256].contiguous() * 2 ** 0.5
    wd = torch.randn(512, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5 * 0.3
    bnd = (torch.rand(512, generator=g) + 0.5, torch.randn(512, generator=g) * 0.1)
    w1n = torch.randn(128, 512, 1, 1, generator=g) * (2.0 / 512) ** 0.5
    bn1n = (torch.rand(128, generator=g) + 0.5, torch.randn(128, generator=g) * 0.1)
    dt = ops.torch_dtype(code)
    bk = ops.conv_bk(code)
    xd = torch.randn(n, h, 64, 256, generator=g).abs().to(cuda, dt)
    p1 = packing.pack_conv_weight(w1.to(cuda), 256, bk, dt)
    p2 = packing.pack_conv_weight(w2.to(cuda), 128, bk, dt)
    p1n = packing.pack_conv_weight(w1n.to(cuda), 512, bk, dt)
    pdual = packing.pack_dual_1x1_weight(w3.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), dt)
    shift = (bn3[1].double() + bnd[1].double()).float().to(cuda)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn1n[0], bn1n[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 128, 1, 1, 1, 0, s[0], s[1], None, True, code)
    y_ref = ops.bottleneck_s2_tail_nhwc(t1, xd, packing.pack_s2_tail_stream(p2, pdual), s[2], s[3], shift, code)
    t1n_ref = ops.conv2d_nhwc(y_ref, p1n, 128, 1, 1, 1, 0, s[4], s[5], None, True, code)
    y, t1n = ops.bottleneck_s2_tail_next_nhwc(t1, xd, packing.pack_s2_tail_stream(p2, pdual, p1n), s[2], s[3], shift,
                                              s[4], s[5], code, out=_sentinel(xd, (n, h // 2, 32, 512)),
                                              t1n=_sentinel(xd, (n, h // 2, 32, 128)))
    torch.cuda.synchronize()
    dy = int((y.view(torch.int16) != y_ref.view(torch.int16)).sum())
    dt1 = int((t1n.view(torch.int16) != t1n_ref.view(torch.int16)).sum())
    print('chained strided tail n=%d h=%d: y differing %d, t1n differing %d' % (n, h, dy, dt1))
    assert dy == 0 and dt1 == 0


def test_strided_tail_refuses_unsupported_shapes(cuda):
    x = torch.zeros(1, 8, 64, 256, device=cuda, dtype=torch.bfloat16)
    t1 = torch.zeros(1, 8, 64, 128, device=cuda, dtype=torch.bfloat16)
    w2 = torch.zeros(128, 1152, device=cuda, dtype=torch.bfloat16)
    wdual = torch.zeros(512, 384, device=cuda, dtype=torch.bfloat16)
    ws = packing.pack_s2_tail_stream(w2, wdual)
    s = torch.ones(512, device=cuda)
    with pytest.raises(RuntimeError, match='multiple of 8'):
        ops.bottleneck_s2_tail_nhwc(t1[:, :4], x[:, :4], ws, s, s, s, BF16)
    with pytest.raises(RuntimeError, match='first Bottleneck of layer2'):
        ops.bottleneck_s2_tail_nhwc(t1[:, :, :32], x[:, :, :32], ws, s, s, s, BF16)
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_s2_tail_nhwc(t1, x, ws[:3], s, s, s, BF16)
    with pytest.raises(ValueError, match='pack_s2_tail_stream'):
        packing.pack_s2_tail_stream(w2[:64], wdual)
    # the chained variant: its longer stream, an aliasing t1n, a wrong next conv1 pack
    w1n = torch.zeros(128, 512, device=cuda, dtype=torch.bfloat16)
    wsn = packing.pack_s2_tail_stream(w2, wdual, w1n)
    t1n = torch.zeros(1, 4, 32, 128, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_s2_tail_next_nhwc(t1, x, ws, s, s, s, s, s, BF16, t1n=t1n)
    with pytest.raises(RuntimeError, match='alias'):
        ops.bottleneck_s2_tail_next_nhwc(t1, x, wsn, s, s, s, s, s, BF16, t1n=t1)
    with pytest.raises(ValueError, match='next conv1 pack'):
        packing.pack_s2_tail_stream(w2, wdual, w1n[:, :256])


def test_fused_bottleneck_refuses_unsupported_shapes(cuda):
    x = torch.zeros(1, 8, 32, 256, device=cuda, dtype=torch.bfloat16)
    w = torch.zeros(64, 256, device=cuda, dtype=torch.bfloat16)
    s = torch.ones(256, device=cuda)
    with pytest.raises(RuntimeError, match='W = 64'):
        ops.bottleneck_nhwc(x, w, s, s, w, s, s, w, s, s, BF16)
    x = torch.zeros(1, 8, 64, 256, device=cuda, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match='alias'):
        ops.bottleneck_nhwc(x, w, s, s, w, s, s, w, s, s, BF16, out=x)
    with pytest.raises(RuntimeError, match='C = 64'):   # the first-block kernel takes 64 channels
        ops.bottleneck_down_nhwc(x, w, s, s, w, s, s, w, s, BF16)
    # the streamed tails: tile rows, layer shapes, and the weight stream's size (a plain pack handed
    # to the chained entry point, or a layer2 pack to a layer3 launch, is refused, never read past)
    x2 = torch.zeros(1, 6, 32, 512, device=cuda, dtype=torch.bfloat16)
    t2 = torch.zeros(1, 6, 32, 128, device=cuda, dtype=torch.bfloat16)
    p2 = packing.pack_tail_stream(torch.zeros(128, 1152, device=cuda, dtype=torch.bfloat16),
                                  torch.zeros(512, 128, device=cuda, dtype=torch.bfloat16))
    s2 = torch.ones(512, device=cuda)
    with pytest.raises(RuntimeError, match='multiple of 4'):
        ops.bottleneck_tail_stream_nhwc(t2, x2, p2, s2, s2, s2, s2, BF16)
    with pytest.raises(RuntimeError, match='layer2'):
        ops.bottleneck_tail_stream_nhwc(t2[:, :4, :16], x2[:, :4, :16], p2, s2, s2, s2, s2, BF16)
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_tail_stream_next_nhwc(t2[:, :4], x2[:, :4], p2, s2, s2, s2, s2, s2, s2, BF16)
    x3 = torch.zeros(1, 8, 16, 1024, device=cuda, dtype=torch.bfloat16)
    t3 = torch.zeros(1, 8, 16, 256, device=cuda, dtype=torch.bfloat16)
    s3 = torch.ones(1024, device=cuda)
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_tail_stream_nhwc(t3, x3, p2, s3, s3, s3, s3, BF16)
    p3 = packing.pack_tail_stream(torch.zeros(256, 2304, device=cuda, dtype=torch.bfloat16),
                                  torch.zeros(1024, 256, device=cuda, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match='multiple of 8'):   # (H % 4 == 0 small grids run 4-row tiles)
        ops.bottleneck_tail_stream_nhwc(t3[:, :6], x3[:, :6], p3, s3, s3, s3, s3, BF16)
    # a stream that is too LONG is refused too (the kernel would read it with the wrong per-group
    # stride): the chained pack handed to the plain entry point, a layer3 pack to a layer2 launch
    p2n = packing.pack_tail_stream(torch.zeros(128, 1152, device=cuda, dtype=torch.bfloat16),
                                   torch.zeros(512, 128, device=cuda, dtype=torch.bfloat16),
                                   torch.zeros(128, 512, device=cuda, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_tail_stream_nhwc(t2[:, :4], x2[:, :4], p2n, s2, s2, s2, s2, BF16)
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_tail_stream_nhwc(t2[:, :4], x2[:, :4], p3, s2, s2, s2, s2, BF16)
    xs = torch.zeros(1, 8, 64, 256, device=cuda, dtype=torch.bfloat16)
    ts = torch.zeros(1, 8, 64, 128, device=cuda, dtype=torch.bfloat16)
    sh = torch.ones(512, device=cuda)
    ps2n = packing.pack_s2_tail_stream(torch.zeros(128, 1152, device=cuda, dtype=torch.bfloat16),
                                       torch.zeros(512, 384, device=cuda, dtype=torch.bfloat16),
                                       torch.zeros(128, 512, device=cuda, dtype=torch.bfloat16))
    with pytest.raises(RuntimeError, match='wstream holds'):
        ops.bottleneck_s2_tail_nhwc(ts, xs, ps2n, sh, sh, sh, BF16)


@pytest.mark.parametrize('precision', ['bf16', 'fp16'])
def test_plan_with_fused_bottlenecks_matches_unfused_plan(cuda, precision):
    import posu.plan as P
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=50, image_size=256), is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(50, 256)))
    net = net.to(cuda).eval()
    plan = net.plan(cuda)
    assert sum(b.w3f is not None for b in plan.layers[0]) == 2   # layer1 blocks 1 and 2
    assert plan.layers[0][0].w3d is not None                     # layer1 block 0
    assert [b.l2 for b in plan.layers[1]] == [False, True, True, True]   # layer2's identity blocks
    assert [b.l3 for b in plan.layers[2]] == [False] + [True] * 5        # layer3's identity blocks
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 256, seed=12)]
    saved = P.FUSED_BOTTLENECK
    try:
        with torch.no_grad():
            P.FUSED_BOTTLENECK = True
            hm1, x11, _ = plan.run(plan.pack_input(views))
            P.FUSED_BOTTLENECK = False
            hm0, x10, _ = plan.run(plan.pack_input(views))
    finally:
        P.FUSED_BOTTLENECK = saved
    torch.cuda.synchronize()
    dx = (x11.float() - x10.float()).abs().max().item()
    dh = (hm1 - hm0).abs()
    print('%s fused vs unfused plan: layer1 out max %.3g, heatmaps max %.3g mean %.3g'
          % (precision, dx, dh.max(), dh.mean()))
    assert dx < (0.1 if precision == 'bf16' else 0.02)
    assert dh.mean() < (0.01 if precision == 'bf16' else 0.002)


@pytest.mark.parametrize('precision', ['bf16', 'fp16'])
def test_plan_strided_tail_is_bit_identical_to_two_launches(cuda, precision):
    """The R50@256 plan with layer2's first block on the strided tail (S2_TAIL) gives the same heatmaps
    and layer1 features, bit for bit, as with conv2 + the dual GEMM as two launches."""
    import posu.plan as P
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=50, image_size=256), is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(50, 256)))
    net = net.to(cuda).eval()
    plan = net.plan(cuda)
    assert plan.layers[1][0].ws2 is not None and all(b.ws2 is None for b in plan.layers[2] + plan.layers[3])
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 256, seed=13)]
    saved = P.S2_TAIL
    try:
        with torch.no_grad():
            P.S2_TAIL = True
            hm1, _, f1 = plan.run(plan.pack_input(views))
            P.S2_TAIL = False
            hm0, _, f0 = plan.run(plan.pack_input(views))
    finally:
        P.S2_TAIL = saved
    torch.cuda.synchronize()
    assert torch.equal(hm1, hm0) and torch.equal(f1, f0)


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('layer,n,h', [('layer3', 2, 16), ('layer3', 1, 8), ('layer3', 3, 24), ('layer3', 128, 16),
                                       ('layer2', 2, 32), ('layer2', 1, 4), ('layer2', 3, 12), ('layer2', 128, 32),
                                       ('layer2w', 2, 48), ('layer2w', 1, 2), ('layer2w', 3, 10), ('layer2w', 64, 48),
                                       ('layer3w', 2, 24), ('layer3w', 1, 6), ('layer3w', 3, 18), ('layer3w', 64, 24)])
def test_chained_tail_matches_tail_and_next_conv1(cuda, code, layer, n, h):
    """Chained streamed tail (posu_bottleneck_tail_stream_next_fwd): block i's tail computing block
    i+1's conv1 + BN1 + ReLU over its output y.  y and t1n are bit-identical to the plain tail
    followed by a conv launch of the next conv1 over y (the same K order per accumulator); both
    outputs start as NaN sentinels, so a store that never lands fails."""
    c, p, w = {'layer3': (1024, 256, 16), 'layer2': (512, 128, 32), 'layer2w': (512, 128, 48),
               'layer3w': (1024, 256, 24)}[layer]
    g = torch.Generator().manual_seed(97 + h + n)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=c, p=p)
    w1n = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    bn1n = (torch.rand(p, generator=g) + 0.5, torch.randn(p, generator=g) * 0.1)
    dt = ops.torch_dtype(code)
    bk = ops.conv_bk(code)
    xd = torch.randn(n, h, w, c, generator=g).to(cuda, dt)
    p1, p2, p3, p1n = (packing.pack_conv_weight(t.to(cuda), t.shape[1], bk, dt) for t in (w1, w2, w3, w1n))
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1], bn1n[0], bn1n[1])]
    t1 = ops.conv2d_nhwc(xd, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, code)
    y_ref = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5], code)
    t1n_ref = ops.conv2d_nhwc(y_ref, p1n, p, 1, 1, 1, 0, s[6], s[7], None, True, code)
    y, t1n = ops.bottleneck_tail_stream_next_nhwc(t1, xd, packing.pack_tail_stream(p2, p3, p1n), s[2], s[3], s[4],
                                                  s[5], s[6], s[7], code, out=_sentinel(xd),
                                                  t1n=_sentinel(t1))
    torch.cuda.synchronize()
    dy = int((y.view(torch.int16) != y_ref.view(torch.int16)).sum())
    dt1 = int((t1n.view(torch.int16) != t1n_ref.view(torch.int16)).sum())
    print('%s chained tail n=%d h=%d: y differing %d, t1n differing %d' % (layer, n, h, dy, dt1))
    assert dy == 0 and dt1 == 0


def test_chained_tail_refuses_bad_operands(cuda):
    x = torch.zeros(1, 4, 32, 512, device=cuda, dtype=torch.bfloat16)
    t1 = torch.zeros(1, 4, 32, 128, device=cuda, dtype=torch.bfloat16)
    ws = torch.zeros(4, 9 * 4 + 2 * 16, 2, 64, 8, device=cuda, dtype=torch.bfloat16)
    s = torch.ones(512, device=cuda)
    with pytest.raises(RuntimeError, match='alias'):
        ops.bottleneck_tail_stream_next_nhwc(t1, x, ws, s, s, s, s, s, s, BF16, t1n=t1)
    with pytest.raises(RuntimeError, match='multiple of 4'):
        ops.bottleneck_tail_stream_next_nhwc(t1[:, :3], x[:, :3], ws, s, s, s, s, s, s, BF16)
    with pytest.raises(ValueError, match='next conv1 pack'):
        packing.pack_tail_stream(torch.zeros(128, 1152, device=cuda, dtype=torch.bfloat16),
                                 torch.zeros(512, 128, device=cuda, dtype=torch.bfloat16),
                                 torch.zeros(128, 256, device=cuda, dtype=torch.bfloat16))


@pytest.mark.parametrize('precision', ['bf16', 'fp16'])
def test_plan_with_chained_tails_matches_unchained_plan(cuda, precision):
    """The R50 plan with the chained layer2 / layer3 tails (plan.CHAINED_TAILS) gives exactly the
    heatmaps of the plan that runs every conv1 as its own launch."""
    import posu.plan as P
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=50, image_size=256), is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(50, 256)))
    net = net.to(cuda).eval()
    saved2b = P.CHAIN_LAYERS_2B
    P.CHAIN_LAYERS_2B = True   # (off in the benched plans: measured neutral-to-slower, plan.py)
    try:
        plan = net.plan(cuda)
    finally:
        P.CHAIN_LAYERS_2B = saved2b
    # layer2: the strided tail chains block 1's conv1 too (round 4); the last tails of layers 2-3 chain
    # the next layer's first conv1 (CHAIN_LAYERS + CHAIN_LAYERS_2B, round 6)
    assert [b.chain is not None for b in plan.layers[1]] == [True, True, True, False]
    assert [b.chain is not None for b in plan.layers[2]] == [False, True, True, True, True, False]
    assert [layer[-1].xchain is not None for layer in plan.layers] == [False, True, True, False]
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 256, seed=13)]
    saved = P.CHAINED_TAILS
    try:
        with torch.no_grad():
            P.CHAINED_TAILS = True
            hm1, _, f1 = plan.run(plan.pack_input(views))
            P.CHAINED_TAILS = False
            hm0, _, f0 = plan.run(plan.pack_input(views))
    finally:
        P.CHAINED_TAILS = saved
    torch.cuda.synchronize()
    assert torch.equal(hm1, hm0) and torch.equal(f1, f0)


def _split_pack(w, cin):
    """A conv weight -> (split fp16 pack [Cout][2 K], its power-of-two exponent e) as the fp16x3 plan
    packs it (the epilogue scale carries 2^-e)."""
    pk = packing.pack_conv_weight(w, cin, 32, torch.float32)
    e = packing.split_exponent(pk)
    return packing.to_split(pk, e), e


@pytest.mark.parametrize('layer,n,h', [('layer1', 2, 64), ('layer1', 1, 2), ('layer1', 3, 10), ('layer1', 128, 64),
                                       ('layer2', 2, 32), ('layer2', 1, 2), ('layer2', 3, 12), ('layer2', 128, 32),
                                       ('layer3', 2, 16), ('layer3', 1, 4), ('layer3', 3, 12), ('layer3', 128, 16)])
def test_split_tails_match_conv_launches(cuda, layer, n, h):
    """Split fp16 (POSU_F16X3) streamed tails, round 6: the plain tail against the conv2 + conv3
    (+ residual) launches, the chained tail against the plain tail + a conv launch of the next conv1 --
    bit-identical (per accumulator the conv kernel's K order and its hi.hi, lo.hi, hi.lo sequence; the
    same epilogue arithmetic and (hi, lo) split), every output starting as a NaN sentinel; and the
    tail within the split dtype's f32-level error of an fp64 torch block.  (128, ..): the
    production grids."""
    c, p, w = {'layer1': (256, 64, 64), 'layer2': (512, 128, 32), 'layer3': (1024, 256, 16)}[layer]
    S = ops.F16X3
    g = torch.Generator().manual_seed(131 + h + n + p)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=c, p=p)
    w1n = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    bn1n = (torch.rand(p, generator=g) + 0.5, torch.randn(p, generator=g) * 0.1)
    x = torch.randn(n, h, w, c, generator=g, dtype=torch.float64)
    xd = packing.to_split(x).to(cuda)
    (p1, e1), (p2, e2), (p3, e3), (p1n, e1n) = (_split_pack(t.to(cuda), t.shape[1]) for t in (w1, w2, w3, w1n))
    def sc(bn, e):
        return (bn[0].double() * 2.0 ** -e).float().to(cuda), bn[1].to(cuda)
    s1, b1 = sc(bn1, e1)
    s2, b2 = sc(bn2, e2)
    s3, b3 = sc(bn3, e3)
    s1n, b1n = sc(bn1n, e1n)
    t1 = ops.conv2d_nhwc(xd, p1, p, 1, 1, 1, 0, s1, b1, None, True, S)
    y = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s2, b2, s3, b3, S,
                                        out=_sentinel(xd))
    t2 = ops.conv2d_nhwc(t1, p2, p, 3, 3, 1, 1, s2, b2, None, True, S)
    two = ops.conv2d_nhwc(t2, p3, c, 1, 1, 1, 0, s3, b3, xd, True, S)
    yc, t1n = ops.bottleneck_tail_stream_next_nhwc(t1, xd, packing.pack_tail_stream(p2, p3, p1n), s2, b2, s3, b3, s1n,
                                                   b1n, S, out=_sentinel(xd), t1n=_sentinel(t1))
    t1n_ref = ops.conv2d_nhwc(two, p1n, p, 1, 1, 1, 0, s1n, b1n, None, True, S)
    # the layer's last tail chaining the NEXT layer's first conv1 (C -> 2 P, posu_bottleneck_tail_stream_chain_fwd)
    w1x = torch.randn(2 * p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    bn1x = (torch.rand(2 * p, generator=g) + 0.5, torch.randn(2 * p, generator=g) * 0.1)
    p1x, e1x = _split_pack(w1x.to(cuda), c)
    s1x, b1x = sc(bn1x, e1x)
    yx, t1x = ops.bottleneck_tail_stream_chain_nhwc(t1, xd, packing.pack_tail_stream(p2, p3, p1x), s2, b2, s3, b3, s1x,
                                                    b1x, S, out=_sentinel(xd),
                                                    t1n=_sentinel(t1, (n, h, w, 4 * p)))
    t1x_ref = ops.conv2d_nhwc(two, p1x, 2 * p, 1, 1, 1, 0, s1x, b1x, None, True, S)
    torch.cuda.synchronize()
    dy = int((y.view(torch.int16) != two.view(torch.int16)).sum())
    dyc = int((yc.view(torch.int16) != two.view(torch.int16)).sum())
    dt1 = int((t1n.view(torch.int16) != t1n_ref.view(torch.int16)).sum())
    dyx = int((yx.view(torch.int16) != two.view(torch.int16)).sum())
    dt1x = int((t1x.view(torch.int16) != t1x_ref.view(torch.int16)).sum())
    print('split %s tail n=%d h=%d: y differing %d, chained y %d, t1n %d; layer-chained y %d, t1n (2 P) %d'
          % (layer, n, h, dy, dyc, dt1, dyx, dt1x))
    assert dy == 0 and dyc == 0 and dt1 == 0 and dyx == 0 and dt1x == 0
    if n >= 128:
        return
    # fp64 torch on the values the device holds: within the f32 level of sum |w x|
    xq = ops.widen(xd, S).double().cpu().permute(0, 3, 1, 2)
    wq = [t.float().double() for t in (w1, w2, w3)]
    a = [t.double() for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    r1 = F.relu(F.conv2d(xq, wq[0]) * a[0].view(1, -1, 1, 1) + a[1].view(1, -1, 1, 1))
    r2 = F.relu(F.conv2d(r1, wq[1], padding=1) * a[2].view(1, -1, 1, 1) + a[3].view(1, -1, 1, 1))
    ref = F.relu(F.conv2d(r2, wq[2]) * a[4].view(1, -1, 1, 1) + a[5].view(1, -1, 1, 1) + xq)
    got = ops.widen(y, S).double().cpu().permute(0, 3, 1, 2)
    err = float((got - ref).abs().max())
    assert err <= 1e-5 * (1.0 + float(ref.abs().max())), err


def test_split_plan_tails_are_bit_identical_to_conv_launches(cuda):
    """The R50@256 fp16x3 plan with its identity Bottlenecks of layer1-3 on the split streamed tails
    (chained; plan.SPLIT_TAILS) gives the heatmaps and features of the plan that runs every
    convolution as its own launch, bit for bit."""
    import posu.plan as P
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=50, image_size=256), is_train=False, precision='fp16x3')
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(50, 256)))
    net = net.to(cuda).eval()
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 256, seed=14)]
    saved = P.SPLIT_TAILS
    try:
        with torch.no_grad():
            P.SPLIT_TAILS = True
            plan = P.PoseResNetPlan(net, ops.F16X3)
            assert [b.l1 for b in plan.layers[0]] == [False, True, True]
            assert [b.l2 for b in plan.layers[1]] == [False, True, True, True]
            assert [b.l3 for b in plan.layers[2]] == [False] + [True] * 5
            assert plan.layers[0][0].wsdn is not None      # layer1 block 0 on the down tail, chained
            # the last tail of layers 1-3 chains the next layer's first conv1 (CHAIN_LAYERS)
            assert [layer[-1].xchain is not None for layer in plan.layers] == [True, True, True, False]
            assert [b.chain is not None for b in plan.layers[0]] == [True, True, False]
            hm1, x11, f1 = plan.run(plan.pack_input(views))
            P.SPLIT_TAILS = False
            plan0 = P.PoseResNetPlan(net, ops.F16X3)
            assert not any(b.l1 or b.l2 or b.l3 for layer in plan0.layers for b in layer)
            hm0, x10, f0 = plan0.run(plan0.pack_input(views))
    finally:
        P.SPLIT_TAILS = saved
    torch.cuda.synchronize()
    assert torch.equal(x11, x10) and torch.equal(hm1, hm0) and torch.equal(f1, f0)


@pytest.mark.parametrize('n,h', [(2, 64), (1, 2), (3, 10), (128, 64)])
def test_split_down_tail_matches_conv_launches(cuda, n, h):
    """Layer1's first Bottleneck in split fp16 (posu_bottleneck_down_tail_stream_fwd, round 6): conv2 +
    the [conv3 | downsample] dual GEMM in one launch, against the conv2 launch + posu_conv1x1_dual_fwd
    (stride 1) -- bit-identical -- and, chained, its t1n against a conv launch of the next conv1 over
    y; NaN-sentinel outputs."""
    S = ops.F16X3
    c, p, w = 256, 64, 64
    g = torch.Generator().manual_seed(151 + h + n)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=64, p=p)
    w3 = torch.randn(c, p, 1, 1, generator=g) * (2.0 / p) ** 0.5 * 0.3
    bn3 = (torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1)
    wd = torch.randn(c, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5 * 0.3
    bnd = (torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1)
    w1n = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    bn1n = (torch.rand(p, generator=g) + 0.5, torch.randn(p, generator=g) * 0.1)
    x = torch.randn(n, h, w, 64, generator=g, dtype=torch.float64).abs()   # a max-pool output of ReLUs
    xd = packing.to_split(x).to(cuda)
    (p1, e1), (p2, e2), (p1n, e1n) = (_split_pack(t.to(cuda), t.shape[1]) for t in (w1, w2, w1n))
    dual = packing.pack_dual_1x1_weight(w3.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), torch.float64)
    ed = packing.split_exponent(dual)
    pdual = packing.to_split(dual, ed)
    dsc = torch.full((c,), 2.0 ** -ed, device=cuda)
    shift = (bn3[1].double() + bnd[1].double()).float().to(cuda)
    def sc(bn, e):
        return (bn[0].double() * 2.0 ** -e).float().to(cuda), bn[1].to(cuda)
    s1, b1 = sc(bn1, e1)
    s2, b2 = sc(bn2, e2)
    s1n, b1n = sc(bn1n, e1n)
    t1 = ops.conv2d_nhwc(xd, p1, p, 1, 1, 1, 0, s1, b1, None, True, S)
    ysent = _sentinel(xd, (n, h, w, 2 * c))
    y, none = ops.bottleneck_down_tail_stream_nhwc(t1, xd, packing.pack_down_tail_stream(p2, pdual), s2, b2, dsc, shift,
                                                   S, out=ysent)
    t2 = ops.conv2d_nhwc(t1, p2, p, 3, 3, 1, 1, s2, b2, None, True, S)
    ref = ops.conv1x1_dual_nhwc(t2, xd, 1, pdual, c, shift, True, S, scale=dsc)
    yc, t1n = ops.bottleneck_down_tail_stream_nhwc(t1, xd, packing.pack_down_tail_stream(p2, pdual, p1n), s2, b2, dsc,
                                                   shift, S, s1n=s1n, b1n=b1n, out=_sentinel(ysent),
                                                   t1n=_sentinel(t1))
    t1n_ref = ops.conv2d_nhwc(ref, p1n, p, 1, 1, 1, 0, s1n, b1n, None, True, S)
    torch.cuda.synchronize()
    assert none is None
    dy = int((y.view(torch.int16) != ref.view(torch.int16)).sum())
    dyc = int((yc.view(torch.int16) != ref.view(torch.int16)).sum())
    dt1 = int((t1n.view(torch.int16) != t1n_ref.view(torch.int16)).sum())
    print('split down tail n=%d h=%d: y differing %d, chained y %d, t1n %d' % (n, h, dy, dyc, dt1))
    assert dy == 0 and dyc == 0 and dt1 == 0


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('n,h', [(2, 96), (1, 2), (3, 10), (64, 96)])
def test_w96_layer1_tails_match_conv_launches(cuda, code, n, h):
    """Layer1 at 384x384 (96-wide maps, R152 configs[4]; round 6): the identity blocks' streamed tail
    (plain and chained) and the first block's down tail (conv2 + [conv3 | downsample], plain and
    chained) against the conv launches they replace -- bit-identical (64-channel 2-byte LDS rows: 8
    chunks, swizzle keys column & 7); NaN-sentinel outputs.  (64, 96): the production grid."""
    c, p, w = 256, 64, 96
    dt = ops.torch_dtype(code)
    bk = ops.conv_bk(code)
    g = torch.Generator().manual_seed(171 + h + n)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=c, p=p)
    w1n = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    bn1n = (torch.rand(p, generator=g) + 0.5, torch.randn(p, generator=g) * 0.1)
    xd = torch.randn(n, h, w, c, generator=g).to(cuda, dt)
    p1, p2, p3, p1n = (packing.pack_conv_weight(t.to(cuda), t.shape[1], bk, dt) for t in (w1, w2, w3, w1n))
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1], bn1n[0], bn1n[1])]
    t1 = ops.conv2d_nhwc(xd, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, code)
    y = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5], code,
                                        out=_sentinel(xd))
    t2 = ops.conv2d_nhwc(t1, p2, p, 3, 3, 1, 1, s[2], s[3], None, True, code)
    two = ops.conv2d_nhwc(t2, p3, c, 1, 1, 1, 0, s[4], s[5], xd, True, code)
    yc, t1n = ops.bottleneck_tail_stream_next_nhwc(t1, xd, packing.pack_tail_stream(p2, p3, p1n), s[2], s[3], s[4],
                                                   s[5], s[6], s[7], code, out=_sentinel(xd), t1n=_sentinel(t1))
    t1n_ref = ops.conv2d_nhwc(two, p1n, p, 1, 1, 1, 0, s[6], s[7], None, True, code)
    # the first block: 64 input channels, downsample 1x1 + BN beside conv3
    x0 = torch.randn(n, h, w, 64, generator=g).abs().to(cuda, dt)
    w3d = torch.randn(c, p, 1, 1, generator=g) * (2.0 / p) ** 0.5 * 0.3
    wd = torch.randn(c, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5 * 0.3
    bnd = (torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1)
    pdual = packing.pack_dual_1x1_weight(w3d.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), dt)
    shift = (bn3[1].double() + bnd[1].double()).float().to(cuda)
    ones = torch.ones(c, device=cuda)
    p1d = packing.pack_conv_weight(w1[:, :64].contiguous().to(cuda), 64, bk, dt)
    t1d = ops.conv2d_nhwc(x0, p1d, p, 1, 1, 1, 0, s[0], s[1], None, True, code)
    yd, _ = ops.bottleneck_down_tail_stream_nhwc(t1d, x0, packing.pack_down_tail_stream(p2, pdual), s[2], s[3], ones,
                                                 shift, code, out=_sentinel(xd))
    t2d = ops.conv2d_nhwc(t1d, p2, p, 3, 3, 1, 1, s[2], s[3], None, True, code)
    dref = ops.conv1x1_dual_nhwc(t2d, x0, 1, pdual, c, shift, True, code)
    ydc, t1nd = ops.bottleneck_down_tail_stream_nhwc(t1d, x0, packing.pack_down_tail_stream(p2, pdual, p1n), s[2], s[3],
                                                     ones, shift, code, s1n=s[6], b1n=s[7], out=_sentinel(xd),
                                                     t1n=_sentinel(t1))
    t1nd_ref = ops.conv2d_nhwc(dref, p1n, p, 1, 1, 1, 0, s[6], s[7], None, True, code)
    torch.cuda.synchronize()
    diff = lambda a, b: int((a.view(torch.int16) != b.view(torch.int16)).sum())  # noqa: E731
    res = [diff(y, two), diff(yc, two), diff(t1n, t1n_ref), diff(yd, dref), diff(ydc, dref), diff(t1nd, t1nd_ref)]
    print('W = 96 tails n=%d h=%d: y / chained y / t1n / down y / chained down y / its t1n differing %s' % (n, h, res))
    assert res == [0] * 6


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('layer,n,h', [('layer2', 2, 32), ('layer2', 3, 12), ('layer2', 128, 32),
                                       ('layer3', 2, 16), ('layer3', 1, 8), ('layer3', 128, 16)])
def test_layer_chained_tail_matches_tail_and_next_layer_conv1(cuda, code, layer, n, h):
    """A layer's last identity tail chaining the NEXT layer's first conv1 (C -> 2 P,
    posu_bottleneck_tail_stream_chain_fwd, round 6) in bf16 / fp16: y and the 2 P-channel t1n
    bit-identical to the plain tail + a conv launch of that conv1 over y; NaN-sentinel outputs."""
    c, p, w = {'layer3': (1024, 256, 16), 'layer2': (512, 128, 32)}[layer]
    g = torch.Generator().manual_seed(211 + h + n)
    w1, bn1, w2, bn2, w3, bn3 = _block_params(g, c=c, p=p)
    w1x = torch.randn(2 * p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    bn1x = (torch.rand(2 * p, generator=g) + 0.5, torch.randn(2 * p, generator=g) * 0.1)
    dt = ops.torch_dtype(code)
    bk = ops.conv_bk(code)
    xd = torch.randn(n, h, w, c, generator=g).to(cuda, dt)
    p1, p2, p3, p1x = (packing.pack_conv_weight(t.to(cuda), t.shape[1], bk, dt) for t in (w1, w2, w3, w1x))
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1], bn1x[0], bn1x[1])]
    t1 = ops.conv2d_nhwc(xd, p1, p, 1, 1, 1, 0, s[0], s[1], None, True, code)
    y_ref = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5], code)
    t1x_ref = ops.conv2d_nhwc(y_ref, p1x, 2 * p, 1, 1, 1, 0, s[6], s[7], None, True, code)
    y, t1x = ops.bottleneck_tail_stream_chain_nhwc(t1, xd, packing.pack_tail_stream(p2, p3, p1x), s[2], s[3], s[4],
                                                   s[5], s[6], s[7], code, out=_sentinel(xd),
                                                   t1n=_sentinel(t1, (n, h, w, 2 * p)))
    torch.cuda.synchronize()
    dy = int((y.view(torch.int16) != y_ref.view(torch.int16)).sum())
    dt1 = int((t1x.view(torch.int16) != t1x_ref.view(torch.int16)).sum())
    print('%s layer-chained tail n=%d h=%d: y differing %d, t1n (2 P) %d' % (layer, n, h, dy, dt1))
    assert dy == 0 and dt1 == 0
