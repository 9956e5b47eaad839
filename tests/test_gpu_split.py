"""The split-fp16 dtype (POSU_F16X3, precision='fp16x3'): every value a (hi, lo) pair of fp16 in
[hi 32 | lo 32] blocks, every product hi.hi + lo.hi + hi.lo on the fp16 MFMAs.  Kernel-level parity
against fp64 torch references of the same ops: the split kernels must be as close to the exact
result as an f32 computation is (about 2^-22 relative per value, f32 accumulation), i.e. orders
of magnitude inside the fp16 kernels' error."""
import pytest
import torch
import torch.nn.functional as F

from posu import ops
from posu.packing import pack_conv_weight, pack_deconv4x4_weight, split_exponent, to_split

pytestmark = pytest.mark.gpu

S = ops.F16X3


def to_split_act(x):
    """NCHW f32/f64 -> the split NHWC tensor [N, H, W, 2C] (fp16)."""
    return to_split(x.permute(0, 2, 3, 1).contiguous())


def from_split(y):
    return ops.widen(y, S).permute(0, 3, 1, 2).double()


def rel_err(got, ref, absref):
    """max |got - ref| relative to the magnitude sum that bounds f32 rounding (sum |w x|)."""
    return float(((got - ref).abs() / (absref + 1e-30)).max())


@pytest.mark.parametrize('cin,cout,k,stride,n,hw', [(64, 128, 3, 1, 2, 16), (256, 64, 1, 1, 3, 8),
                                                    (128, 256, 3, 2, 2, 16), (32, 64, 1, 1, 1, 5)])
@pytest.mark.parametrize('tile', [-1, 0, 3, 5, 9, 18, 7, 15, 39, 31, 47, 55])
def test_split_conv_matches_fp64(cuda, cin, cout, k, stride, n, hw, tile):
    torch.manual_seed(cin + cout + k + tile)
    pad = k // 2
    x = torch.randn(n, cin, hw, hw, dtype=torch.float64, device=cuda)
    w = torch.randn(cout, cin, k, k, dtype=torch.float64, device=cuda) * 0.05
    scale = torch.rand(cout, device=cuda) + 0.5
    shift = torch.randn(cout, device=cuda) * 0.1
    res = torch.randn(n, cout, (hw + 2 * pad - k) // stride + 1, (hw + 2 * pad - k) // stride + 1,
                      dtype=torch.float64, device=cuda)
    xs = to_split_act(x)
    xq = from_split(xs)                              # the values the kernel sees (22-bit)
    pk = pack_conv_weight(w.float(), cin, 32, torch.float32)
    e = split_exponent(pk)
    ws = to_split(pk, e)
    rs = to_split_act(res)
    y = ops.conv2d_nhwc(xs, ws, cout, k, k, stride, pad, (scale.double() * 2.0 ** -e).float(), shift, rs, True, S,
                        tile=tile)
    assert y.shape == (n, res.shape[2], res.shape[3], 2 * cout)
    wq = w.float().double()
    ref = F.relu(F.conv2d(xq, wq, stride=stride, padding=pad) * scale.double()[None, :, None, None] +
                 shift.double()[None, :, None, None] + from_split(rs))
    mag = F.conv2d(xq.abs(), wq.abs(), stride=stride, padding=pad) * scale.double()[None, :, None, None] + 1.0
    got = from_split(y)
    # f32 accumulation over K products + the operands' 2^-22 split error: well under 1e-5 of sum |w x|
    assert rel_err(got, ref, mag) < 2e-6
    if tile in (31, 47, 55):   # the staggered split tiles: bit-identical to their unstaggered twins
        twin = {31: 6, 47: 7, 55: 15}[tile]
        y2 = ops.conv2d_nhwc(xs, ws, cout, k, k, stride, pad, (scale.double() * 2.0 ** -e).float(), shift, rs, True, S,
                             tile=twin)
        assert torch.equal(y, y2)


def test_split_dual_and_deconv_head_match_fp64(cuda):
    torch.manual_seed(5)
    n, c, c2, cout, hw = 2, 64, 128, 256, 8
    t = torch.randn(n, c, hw, hw, dtype=torch.float64, device=cuda)
    x = torch.randn(n, c2, 2 * hw, 2 * hw, dtype=torch.float64, device=cuda)
    wa = torch.randn(cout, c, dtype=torch.float64, device=cuda) * 0.05
    wb = torch.randn(cout, c2, dtype=torch.float64, device=cuda) * 0.05
    shift = torch.randn(cout, device=cuda) * 0.1
    pk = torch.cat([wa, wb], dim=1)
    e = split_exponent(pk)
    y = ops.conv1x1_dual_nhwc(to_split_act(t), to_split_act(x), 2, to_split(pk, e), cout, shift, True, S,
                              scale=torch.full((cout,), 2.0 ** -e, device=cuda))
    tq, xq = from_split(to_split_act(t)), from_split(to_split_act(x))[:, :, ::2, ::2]
    ref = F.relu(torch.einsum('oc,nchw->nohw', wa, tq) + torch.einsum('oc,nchw->nohw', wb, xq) +
                 shift.double()[None, :, None, None])
    mag = torch.einsum('oc,nchw->nohw', wa.abs(), tq.abs()) + torch.einsum('oc,nchw->nohw', wb.abs(), xq.abs()) + 1
    assert rel_err(from_split(y), ref, mag) < 2e-6

    # deconv 4x4/s2 + BN + ReLU fused with the 1x1 head (split head weights in the logical order)
    cin, J = 128, 16
    xd = torch.randn(n, cin, hw, hw, dtype=torch.float64, device=cuda)
    wd = torch.randn(cin, cout, 4, 4, dtype=torch.float64, device=cuda) * 0.03
    sc = torch.rand(cout, device=cuda) + 0.5
    sh = torch.randn(cout, device=cuda) * 0.1
    hw_ = torch.randn(J, cout, 1, 1, dtype=torch.float64, device=cuda) * 0.05
    hb = torch.randn(J, device=cuda)
    pd = pack_deconv4x4_weight(wd.float(), 32, torch.float32)
    ed = split_exponent(pd)
    hpk = pack_conv_weight(hw_.float(), cout, 64, torch.float32)
    h_hi = hpk.to(torch.float16)
    h_lo = (hpk - h_hi.float()).to(torch.float16)
    hm, f = ops.deconv4x4s2_head(to_split_act(xd), to_split(pd, ed), cout, (sc.double() * 2.0 ** -ed).float(), sh,
                                 h_hi, J, hb, S, keep_f=True, head_w_lo=h_lo)
    xq = from_split(to_split_act(xd))
    fr = F.relu(F.conv_transpose2d(xq, wd.float().double(), stride=2, padding=1) * sc.double()[None, :, None, None] +
                sh.double()[None, :, None, None])
    fmag = F.conv_transpose2d(xq.abs(), wd.float().double().abs(), stride=2, padding=1) * \
        sc.double()[None, :, None, None] + 1
    assert rel_err(from_split(f), fr, fmag) < 2e-6
    hr = F.conv2d(fr, hw_.float().double()) + hb.double()[None, :, None, None]
    hmag = F.conv2d(fmag, hw_.float().double().abs()) + 1
    assert rel_err(hm.double(), hr, hmag) < 4e-6


def test_split_layout_ops(cuda):
    torch.manual_seed(2)
    x = torch.randn(3, 3, 10, 12, device=cuda)
    # pack (direct and space-to-depth) and unpack round trips: values to the pair's 22 bits
    xs = ops.pack_nchw_to_nhwc(x, S, 32)
    assert xs.shape == (3, 10, 12, 64) and xs.dtype == torch.float16
    back = ops.nhwc_to_nchw_f32(xs, S)
    assert back.shape == (3, 32, 10, 12)
    assert float((back[:, :3] - x).abs().max()) <= float(x.abs().max()) * 2.0 ** -21
    assert float(back[:, 3:].abs().max()) == 0.0
    s2d = ops.pack_s2d_nchw(x, S, 32)
    assert s2d.shape == (3, 5, 6, 64)
    v = ops.widen(s2d, S)
    ref = F.pixel_unshuffle(x, 2).view(3, 3, 4, 5, 6).permute(0, 3, 4, 2, 1).reshape(3, 5, 6, 12)
    assert float((v[..., :12] - ref).abs().max()) <= float(x.abs().max()) * 2.0 ** -21
    # max-pool of pairs = the pair of the max of hi + lo
    a = torch.randn(2, 64, 9, 7, device=cuda)
    a_s = to_split_act(a.double())
    mp = ops.maxpool3x3s2_nhwc(a_s, S)
    ref = F.max_pool2d(from_split(a_s), 3, 2, 1)
    assert torch.equal(from_split(mp), ref)
    assert torch.equal(mp, to_split_act(ref))


@pytest.mark.parametrize('hflip', [False, True])
def test_split_fused_stem_matches_fp64(cuda, hflip):
    """posu_stem_pool_views_fwd in split fp16 (input split while staged, hi / lo weight planes,
    three MFMAs per kernel row, pool first / BN after) against the f64 stem + BN + ReLU + max-pool."""
    from posu.packing import pack_stem_fused_weight
    torch.manual_seed(11)
    views = [torch.randn(3, 3, 256, 256, device=cuda) for _ in range(2)]
    w = torch.randn(64, 3, 7, 7, dtype=torch.float64, device=cuda) * 0.05
    scale = (torch.rand(64, device=cuda) + 0.5) * torch.where(torch.rand(64, device=cuda) < 0.2, -1.0, 1.0)
    shift = torch.randn(64, device=cuda) * 0.1
    e = split_exponent(w)
    v = pack_stem_fused_weight(w.float(), torch.float64) * 2.0 ** e
    hi = v.to(torch.float16)
    wpk = torch.cat([hi, (v - hi.double()).to(torch.float16)], dim=0).contiguous()
    y = ops.stem_pool_views(views, wpk, (scale.double() * 2.0 ** -e).float(), shift, S, hflip=hflip)
    assert y.shape == (6, 64, 64, 128)
    x = torch.cat(views).double()
    if hflip:
        x = x.flip(3)
    xf = x.float()
    xh = xf.half().float()
    xq = (xh.double() + (xf - xh).half().double())     # the input as its (hi, lo) pair
    wq = w.float().double()
    ref = F.max_pool2d(F.relu(F.conv2d(xq, wq, stride=2, padding=3) * scale.double()[None, :, None, None] +
                              shift.double()[None, :, None, None]), 3, 2, 1)
    mag = F.max_pool2d(F.conv2d(xq.abs(), wq.abs(), stride=2, padding=3) * scale.double().abs()[None, :, None, None],
                       3, 2, 1) + 1
    assert rel_err(from_split(y), ref, mag) < 2e-6
