"""The benchmarked fused bf16 kernels against an exact restatement of their arithmetic
(the 1e-3 gate covers the fp32 plan, which runs the unfused convolutions;
this pins the fused launches the bench times).

Each fused kernel claims: products of bf16 operands summed in f32, the BN affine in f32, and
rounding to bf16 only where the block stores a tensor (t1 and t2 inside the block, y at the
end) -- the reference's eval-mode Bottleneck (lib/models/pose_resnet.py:61-99, downsample
pose_resnet.py:136-141) and stem (pose_resnet.py:192-195) with exactly those roundings.  The
emulation computes that in fp64 on the CPU (weights / inputs rounded as the packing rounds
them, intermediates rounded RNE where the kernel stores them).

What remains is the kernel's f32 arithmetic, and the gate on it is DERIVED, per output element,
not fitted.  Through every stage the emulation carries a bound d on
|kernel value - emulated value| of each stored element:
  * a conv reading inputs off by at most d_in: the pre-rounding value is off by at most
    |s| (sum |w| d_in + gamma_K sum |w a|) + 2u (|v| + D) -- the propagated input error, the
    f32 accumulation of K products (gamma_K = K u / (1 - K u), u = 2^-24, any summation order),
    and the f32 BN affine / residual add roundings;
  * the stored value is the bf16 rounding (after ReLU) of something in [v - D, v + D], so it is
    off by at most max |relu(q(v +- D)) - q(relu(v))| -- zero where that interval holds no
    rounding boundary, i.e. such an element must come out EXACT.
Every kernel output must lie within its bound, and (the regression gate) at most 0.5 % of the
outputs may sit more than half an ulp from the emulation."""
import pytest
import torch
import torch.nn.functional as F

from posu import ops, packing
from posu._native import BF16

pytestmark = pytest.mark.gpu
DT = torch.bfloat16
U32 = 2.0 ** -24


def _q(t):
    """Round an fp64 tensor to bf16 (RNE) and back, as a kernel store does."""
    return t.float().to(DT).double()


def _params(g, c, p):
    def bn(ch):
        return (torch.rand(ch, generator=g) + 0.5, torch.randn(ch, generator=g) * 0.1)
    w1 = torch.randn(p, c, 1, 1, generator=g) * (2.0 / c) ** 0.5
    w2 = torch.randn(p, p, 3, 3, generator=g) * (2.0 / (9 * p)) ** 0.5
    w3 = torch.randn(c, p, 1, 1, generator=g) * (2.0 / p) ** 0.5 * 0.3
    return w1, bn(p), w2, bn(p), w3, bn(c)


def _col(v):
    return v.double().view(1, -1, 1, 1)


def _gamma(k):
    return k * U32 / (1 - k * U32)


class _E:
    """An emulated stored tensor (fp64 values, exactly bf16-representable) and its per-element
    bound d on the kernel's deviation from it."""

    def __init__(self, v, d=None):
        self.v, self.d = v, torch.zeros_like(v) if d is None else d


def _store(v, dv, relu=True):
    """Round (after ReLU) a pre-rounding value v known to within dv: -> _E."""
    act = F.relu if relu else (lambda t: t)
    r = _q(act(v))
    d = torch.maximum((_q(act(v + dv)) - r).abs(), (_q(act(v - dv)) - r).abs())
    return _E(r, d)


def _conv(srcs, scale, shift, residual=None, relu=True):
    """sum over (E input, fp64 weight already rounded as packed, stride, padding) of the convs,
    * scale + shift (+ residual): the emulated stored output and its bound."""
    v = S = P = 0
    k = 0
    for a, w, stride, pad in srcs:
        v = v + F.conv2d(a.v, w, stride=stride, padding=pad)
        S = S + F.conv2d(a.v.abs(), w.abs(), stride=stride, padding=pad)
        P = P + F.conv2d(a.d, w.abs(), stride=stride, padding=pad)
        k += w.shape[1] * w.shape[2] * w.shape[3]
    sc = _col(scale) if scale is not None else 1.0
    v = v * sc + _col(shift)
    dv = abs(sc) * (P + _gamma(k) * S)
    if residual is not None:
        v = v + residual.v
        dv = dv + residual.d
    dv = dv + 2 * U32 * (v.abs() + dv)
    return _store(v, dv, relu)


def _emulate_block(xq, w1, bn1, w2, bn2, w3, bn3):
    """xq: NCHW fp64 holding bf16 values.  conv weights rounded to bf16 as packed."""
    x = _E(xq)
    t1 = _conv([(x, _q(w1.double()), 1, 0)], bn1[0], bn1[1])
    t2 = _conv([(t1, _q(w2.double()), 1, 1)], bn2[0], bn2[1])
    return _conv([(t2, _q(w3.double()), 1, 0)], bn3[0], bn3[1], residual=x)


def _check(name, got_nhwc, emul):
    got = got_nhwc.float().cpu().permute(0, 3, 1, 2).double()
    dev = (got - emul.v).abs()
    ulp = 2.0 ** -7 * emul.v.abs().clamp_min(2.0 ** -4)
    r = dev / ulp
    off = float((r > 0.5).double().mean())
    exact_req = emul.d == 0
    print('%s vs bf16-rounding emulation: exact %.4f, >1/2 ulp %.5f, max %.3g ulp; derived bound: %.3f of the '
          'outputs must be exact, bound max %.3g ulp, largest deviation / bound %.3g'
          % (name, float((r == 0).double().mean()), off, float(r.max()), float(exact_req.double().mean()),
             float((emul.d / ulp).max()), float((dev / emul.d.clamp_min(1e-30)).max())))
    assert torch.isfinite(got).all()
    assert bool((dev <= emul.d).all()), 'deviation beyond the derived bound at %d elements' % int((dev > emul.d).sum())
    assert off < 5e-3, off


def _dev(xq, cuda):
    return xq.float().permute(0, 2, 3, 1).contiguous().to(cuda, DT)


@pytest.mark.parametrize('n,h', [(2, 16), (1, 64)])
def test_layer1_identity_block(cuda, n, h):
    g = torch.Generator().manual_seed(501 + h)
    w1, bn1, w2, bn2, w3, bn3 = _params(g, 256, 64)
    xq = _q(torch.randn(n, 256, h, 64, generator=g).double())
    xd = _dev(xq, cuda)
    bk = ops.conv_bk(BF16)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    got = ops.bottleneck_nhwc(xd, packing.pack_bottleneck_conv1_weight(w1.to(cuda), DT), s[0], s[1],
                              packing.pack_conv_weight(w2.to(cuda), 64, bk, DT), s[2], s[3],
                              packing.pack_bottleneck_conv3_weight(w3.to(cuda), DT), s[4], s[5], BF16)
    torch.cuda.synchronize()
    _check('layer1 block', got, _emulate_block(xq, w1, bn1, w2, bn2, w3, bn3))


@pytest.mark.parametrize('n,h', [(2, 16), (1, 64)])
def test_layer1_first_block_with_downsample(cuda, n, h):
    g = torch.Generator().manual_seed(601 + h)
    w1, bn1, w2, bn2, _, _ = _params(g, 64, 64)
    w3 = torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5 * 0.3
    bn3 = (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1)
    wd = torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5 * 0.3
    bnd = (torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1)
    xq = _q(torch.randn(n, 64, h, 64, generator=g).double().abs())
    xd = _dev(xq, cuda)
    bk = ops.conv_bk(BF16)
    s = [v.to(cuda) for v in (bn1[0], bn1[1], bn2[0], bn2[1])]
    pdual = packing.pack_dual_1x1_weight(w3.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), DT)
    shift = (bn3[1].double() + bnd[1].double()).float()
    got = ops.bottleneck_down_nhwc(xd, packing.pack_conv_weight(w1.to(cuda), 64, bk, DT), s[0], s[1],
                                   packing.pack_conv_weight(w2.to(cuda), 64, bk, DT), s[2], s[3],
                                   packing.pack_bottleneck_down_weight(pdual, 64), shift.to(cuda), BF16)
    torch.cuda.synchronize()
    # the downsample's and conv3's BN scales are folded into the packed weights (one rounding
    # of the fp64 product, pack_dual_1x1_weight); one shift for both branches
    x = _E(xq)
    t1 = _conv([(x, _q(w1.double()), 1, 0)], bn1[0], bn1[1])
    t2 = _conv([(t1, _q(w2.double()), 1, 1)], bn2[0], bn2[1])
    w3s = _q(w3.double() * bn3[0].double().view(-1, 1, 1, 1))
    wds = _q(wd.double() * bnd[0].double().view(-1, 1, 1, 1))
    _check('layer1 block 0', got, _conv([(t2, w3s, 1, 0), (x, wds, 1, 0)], None, shift))


@pytest.mark.parametrize('n,h', [(2, 8), (1, 32)])
def test_layer2_identity_block_streamed_tail(cuda, n, h):
    g = torch.Generator().manual_seed(701 + h)
    w1, bn1, w2, bn2, w3, bn3 = _params(g, 512, 128)
    xq = _q(torch.randn(n, 512, h, 32, generator=g).double())
    xd = _dev(xq, cuda)
    bk = ops.conv_bk(BF16)
    p1 = packing.pack_conv_weight(w1.to(cuda), 512, bk, DT)
    p2 = packing.pack_conv_weight(w2.to(cuda), 128, bk, DT)
    p3 = packing.pack_conv_weight(w3.to(cuda), 128, bk, DT)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 128, 1, 1, 1, 0, s[0], s[1], None, True, BF16)
    streamed = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5], BF16)
    torch.cuda.synchronize()
    _check('layer2 block (conv1 + streamed tail)', streamed, _emulate_block(xq, w1, bn1, w2, bn2, w3, bn3))


@pytest.mark.parametrize('n,h', [(2, 8), (1, 64)])
def test_layer2_first_block_strided_tail(cuda, n, h):
    """conv1 launch + posu_bottleneck_s2_tail_fwd (conv2 3x3 / stride 2, then the conv3 | downsample
    dual GEMM with the BN scales folded into the packed weights)."""
    g = torch.Generator().manual_seed(751 + h)
    _, bn1, w2, bn2, w3, bn3 = _params(g, 512, 128)
    w1 = torch.randn(128, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5
    wd = torch.randn(512, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5 * 0.3
    bnd = (torch.rand(512, generator=g) + 0.5, torch.randn(512, generator=g) * 0.1)
    xq = _q(torch.randn(n, 256, h, 64, generator=g).double().abs())
    xd = _dev(xq, cuda)
    bk = ops.conv_bk(BF16)
    p1 = packing.pack_conv_weight(w1.to(cuda), 256, bk, DT)
    p2 = packing.pack_conv_weight(w2.to(cuda), 128, bk, DT)
    pdual = packing.pack_dual_1x1_weight(w3.to(cuda), bn3[0].to(cuda), wd.to(cuda), bnd[0].to(cuda), DT)
    shift = (bn3[1].double() + bnd[1].double()).float()
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 128, 1, 1, 1, 0, s[0], s[1], None, True, BF16)
    got = ops.bottleneck_s2_tail_nhwc(t1, xd, packing.pack_s2_tail_stream(p2, pdual), s[2], s[3], shift.to(cuda),
                                      BF16)
    torch.cuda.synchronize()
    x = _E(xq)
    t1e = _conv([(x, _q(w1.double()), 1, 0)], bn1[0], bn1[1])
    t2e = _conv([(t1e, _q(w2.double()), 2, 1)], bn2[0], bn2[1])
    w3s = _q(w3.double() * bn3[0].double().view(-1, 1, 1, 1))
    wds = _q(wd.double() * bnd[0].double().view(-1, 1, 1, 1))
    _check('layer2 block 0 (conv1 + strided tail)', got, _conv([(t2e, w3s, 1, 0), (x, wds, 2, 0)], None, shift))


@pytest.mark.parametrize('n,h', [(2, 8), (1, 16)])
def test_layer3_identity_block_streamed_tail(cuda, n, h):
    g = torch.Generator().manual_seed(801 + h)
    w1, bn1, w2, bn2, w3, bn3 = _params(g, 1024, 256)
    xq = _q(torch.randn(n, 1024, h, 16, generator=g).double())
    xd = _dev(xq, cuda)
    bk = ops.conv_bk(BF16)
    p1 = packing.pack_conv_weight(w1.to(cuda), 1024, bk, DT)
    p2 = packing.pack_conv_weight(w2.to(cuda), 256, bk, DT)
    p3 = packing.pack_conv_weight(w3.to(cuda), 256, bk, DT)
    s = [t.to(cuda) for t in (bn1[0], bn1[1], bn2[0], bn2[1], bn3[0], bn3[1])]
    t1 = ops.conv2d_nhwc(xd, p1, 256, 1, 1, 1, 0, s[0], s[1], None, True, BF16)
    got = ops.bottleneck_tail_stream_nhwc(t1, xd, packing.pack_tail_stream(p2, p3), s[2], s[3], s[4], s[5], BF16)
    torch.cuda.synchronize()
    _check('layer3 block (conv1 + streamed tail)', got, _emulate_block(xq, w1, bn1, w2, bn2, w3, bn3))


@pytest.mark.parametrize('size', [256, 384])
def test_fused_stem_pool(cuda, size):
    """posu_stem_pool_fwd: f32 views rounded to bf16 on load, 7x7/s2 conv, BN, ReLU, rounded
    store, 3x3/s2 max-pool (a max of rounded values is exact; a max moves by at most the largest
    bound of its window)."""
    g = torch.Generator().manual_seed(901)
    x = torch.randn(2, 3, size, size, generator=g)
    wt = torch.randn(64, 3, 7, 7, generator=g) * (2.0 / 147) ** 0.5
    sc, sh = torch.rand(64, generator=g) + 0.5, torch.randn(64, generator=g) * 0.1
    got = ops.stem_pool(x.to(cuda), packing.pack_stem_fused_weight(wt.to(cuda), DT), sc.to(cuda), sh.to(cuda), BF16)
    torch.cuda.synchronize()
    stem = _conv([(_E(_q(x.double())), _q(wt.double()), 2, 3)], sc, sh)
    _check('stem + max-pool', got, _E(F.max_pool2d(stem.v, 3, 2, 1), F.max_pool2d(stem.d, 3, 2, 1)))
