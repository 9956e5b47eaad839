"""Training-path kernels on the MI355X against torch autograd (CPU, fp32) of the same
ops: conv data / weight gradients (incl. strided, padded-channel stem and the
ConvTranspose2d weight gradient), training-mode BatchNorm with per-view segments and
running statistics, its backward through ReLU / residual, channel sums and the max-pool
backward with ties."""
import pytest
import torch
import torch.nn.functional as F

from posu import ops, packing, train_ops as T
from posu._native import BF16, F16, F32

pytestmark = pytest.mark.gpu

FP32_TOL = dict(atol=2e-4, rtol=2e-4)


def _nhwc(t, cuda, dt, cpad=None):
    t = t.permute(0, 2, 3, 1)
    if cpad is not None and cpad > t.shape[-1]:
        t = F.pad(t, (0, cpad - t.shape[-1]))
    return t.contiguous().to(cuda, dt)


def _nchw(t):
    return t.float().cpu().permute(0, 3, 1, 2)


def _close_lowp(got, ref, frac=0.02):
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= frac * scale + 1e-3, (err, scale)


DGRAD_CASES = [
    # n, cin, h, w, cout, k, stride, pad
    (2, 64, 16, 16, 64, 3, 1, 1),
    (2, 64, 17, 15, 128, 3, 2, 1),    # strided 3x3, odd input
    (2, 128, 16, 16, 256, 1, 2, 0),   # downsample 1x1 / s2 (with residual: in place over dy's pixels)
    (2, 64, 15, 17, 128, 1, 2, 0),    # the same, odd input
    (3, 256, 8, 8, 64, 1, 1, 0),
    (2, 128, 8, 8, 64, 4, 2, 1),      # the deconv's data gradient is this forward conv's shape
]


@pytest.mark.parametrize('case', DGRAD_CASES)
@pytest.mark.parametrize('code', [F32, BF16])
def test_conv_dgrad_matches_autograd(cuda, case, code):
    n, cin, h, w, cout, k, s, p = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn(n, cin, h, w, generator=g, requires_grad=True)
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    y = F.conv2d(x, wt, stride=s, padding=p)
    dy = torch.randn_like(y)
    (dx_ref,) = torch.autograd.grad(y, x, dy)
    res = torch.randn_like(dx_ref)
    dt = ops.torch_dtype(code)
    wpk = packing.pack_conv_dgrad_weight(wt.to(cuda), ops.conv_bk(code), dt)
    dx = T.conv2d_dgrad(_nhwc(dy, cuda, dt), wpk, cin, k, k, s, p, (h, w), code)
    dx_r = T.conv2d_dgrad(_nhwc(dy, cuda, dt), wpk, cin, k, k, s, p, (h, w), code, residual=_nhwc(res, cuda, dt))
    torch.cuda.synchronize()
    if code == F32:
        torch.testing.assert_close(_nchw(dx), dx_ref, **FP32_TOL)
        torch.testing.assert_close(_nchw(dx_r), dx_ref + res, **FP32_TOL)
    else:
        _close_lowp(_nchw(dx), dx_ref)
        _close_lowp(_nchw(dx_r), dx_ref + res.to(dt).float())


@pytest.mark.parametrize('case', [DGRAD_CASES[0], DGRAD_CASES[1], DGRAD_CASES[4], (2, 64, 16, 16, 256, 1, 1, 0)])
@pytest.mark.parametrize('code', [BF16, F32])
def test_conv_dgrad_every_tile_equals_the_heuristic(cuda, case, code):
    """ABI 15 (posu_conv2d_dgrad_tile): every tile the training step's autotuner may pick for a data
    gradient (posu.plan._tile_candidates of its output channels) gives the heuristic's dx bit for
    bit, with and without the residual; an unknown tile is refused."""
    from posu import plan as pl
    n, cin, h, w, cout, k, s, p = case
    g = torch.Generator().manual_seed(12)
    dt = ops.torch_dtype(code)
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    dy = torch.randn(n, ho, wo, cout, generator=g).to(cuda, dt)
    res = torch.randn(n, h, w, cin, generator=g).to(cuda, dt)
    wpk = packing.pack_conv_dgrad_weight(wt.to(cuda), ops.conv_bk(code), dt)
    for r in (None, res):
        ref = T.conv2d_dgrad(dy, wpk, cin, k, k, s, p, (h, w), code, residual=r)
        for t in pl._tile_candidates(cin, code):
            got = T.conv2d_dgrad(dy, wpk, cin, k, k, s, p, (h, w), code, residual=r, tile=t)
            assert torch.equal(got, ref), (t, r is None)
    with pytest.raises(RuntimeError, match='unknown tile'):
        T.conv2d_dgrad(dy, wpk, cin, k, k, s, p, (h, w), code, tile=13)


@pytest.mark.parametrize('code', [F32, BF16])
@pytest.mark.parametrize('n,cin,h,w,cout', [(2, 64, 16, 16, 128), (2, 128, 8, 12, 256), (1, 40, 6, 10, 64)])
def test_s2_conv_data_gradient_as_subpixel_deconv(cuda, code, n, cin, h, w, cout):
    """ABI 15 (the training step's first-block conv2 backward): the data gradient of a 3x3 / s2 / p1
    conv as posu_deconv4x4s2_fwd over dz with the conv weight packed as a 3x3 deconv source (its
    4x4 zero-padding) -- four 2x2 sub-pixel classes instead of the 3x3 conv over the zero-upsampled
    gradient -- against autograd, and against posu_conv2d_dgrad (the upsampled form)."""
    g = torch.Generator().manual_seed(17)
    x = torch.randn(n, cin, h, w, generator=g, requires_grad=True)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (2.0 / (cin * 9)) ** 0.5
    y = F.conv2d(x, wt, stride=2, padding=1)
    dy = torch.randn_like(y)
    (dx_ref,) = torch.autograd.grad(y, x, dy)
    dt = ops.torch_dtype(code)
    wdc = packing.pack_deconv4x4_weight(wt.to(cuda), ops.conv_bk(code), dt)
    dx = ops.deconv4x4s2_nhwc(_nhwc(dy, cuda, dt), wdc, cin, None, None, False, code)
    wpk = packing.pack_conv_dgrad_weight(wt.to(cuda), ops.conv_bk(code), dt)
    dx_up = T.conv2d_dgrad(_nhwc(dy, cuda, dt), wpk, cin, 3, 3, 2, 1, (h, w), code)
    torch.cuda.synchronize()
    assert dx.shape == dx_up.shape == (n, h, w, cin)
    if code == F32:
        torch.testing.assert_close(_nchw(dx), dx_ref, **FP32_TOL)
        torch.testing.assert_close(dx, dx_up, atol=1e-5, rtol=1e-5)
    else:
        _close_lowp(_nchw(dx), dx_ref)
        _close_lowp(_nchw(dx), _nchw(dx_up), 0.01)


WGRAD_CASES = [
    # n, cin, cin_pad, h, w, cout, k, stride, pad
    (2, 3, 8, 32, 30, 64, 7, 2, 3),      # direct stem (channels padded to 8)
    (2, 64, 64, 16, 16, 64, 3, 1, 1),    # 64-row tiles, K = 576 (ragged n-tile)
    (2, 64, 64, 17, 15, 128, 3, 2, 1),   # strided, odd
    (3, 256, 256, 8, 8, 512, 1, 1, 0),
    (2, 128, 128, 16, 16, 256, 1, 2, 0),
    (1, 16, 16, 40, 40, 64, 3, 1, 1),    # P = 1600: several splits
]


@pytest.mark.parametrize('case', WGRAD_CASES)
@pytest.mark.parametrize('code', [F32, BF16, F16])
def test_conv_wgrad_matches_autograd(cuda, case, code):
    n, cin, cpad, h, w, cout, k, s, p = case
    g = torch.Generator().manual_seed(12)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = (torch.randn(cout, cin, k, k, generator=g) * 0.1).requires_grad_(True)
    y = F.conv2d(x, wt, stride=s, padding=p)
    dy = torch.randn_like(y)
    (dw_ref,) = torch.autograd.grad(y, wt, dy)
    dt = ops.torch_dtype(code)
    dw = T.conv2d_wgrad(_nhwc(dy, cuda, dt), _nhwc(x, cuda, dt, cpad), cin, k, k, s, p, code)
    torch.cuda.synchronize()
    assert dw.shape == dw_ref.shape
    if code == F32:
        torch.testing.assert_close(dw.cpu(), dw_ref, atol=1e-3, rtol=1e-4)
    else:
        _close_lowp(dw.cpu(), dw_ref)


@pytest.mark.parametrize('code', [F32, BF16])
def test_deconv_weight_and_data_gradients(cuda, code):
    g = torch.Generator().manual_seed(13)
    n, cin, h, w, cout = 2, 128, 6, 5, 64
    x = torch.randn(n, cin, h, w, generator=g, requires_grad=True)
    wt = (torch.randn(cin, cout, 4, 4, generator=g) * 0.05).requires_grad_(True)
    y = F.conv_transpose2d(x, wt, stride=2, padding=1)
    dy = torch.randn_like(y)
    dx_ref, dw_ref = torch.autograd.grad(y, (x, wt), dy)
    dt = ops.torch_dtype(code)
    dyd = _nhwc(dy, cuda, dt)
    dw = T.deconv4x4s2_wgrad(_nhwc(x.detach(), cuda, dt), dyd, code)
    # data gradient = forward conv 4x4 / s2 / p1 of dy with W read as [Cin][Cout] conv weights
    wpk = packing.pack_conv_weight(wt.detach().to(cuda), cout, ops.conv_bk(code), dt)
    dx = ops.conv2d_nhwc(dyd, wpk, cin, 4, 4, 2, 1, None, None, None, False, code)
    torch.cuda.synchronize()
    if code == F32:
        torch.testing.assert_close(dw.cpu(), dw_ref, atol=1e-3, rtol=1e-4)
        torch.testing.assert_close(_nchw(dx), dx_ref, **FP32_TOL)
    else:
        _close_lowp(dw.cpu(), dw_ref)
        _close_lowp(_nchw(dx), dx_ref)


def _bn_ref(z, nseg, gamma, beta, rm, rv, res, relu):
    outs = []
    for zs, rs in zip(z.chunk(nseg), (res.chunk(nseg) if res is not None else [None] * nseg)):
        o = F.batch_norm(zs, rm, rv, gamma, beta, training=True, momentum=0.1, eps=1e-5)
        if rs is not None:
            o = o + rs
        outs.append(F.relu(o) if relu else o)
    return torch.cat(outs)


@pytest.mark.parametrize('c,nseg,residual,relu', [(64, 4, False, True), (256, 2, True, True),
                                                  (2048, 1, False, False), (128, 4, True, True),
                                                  (64, 6, True, True)])  # 6 segments: two finalize passes
@pytest.mark.parametrize('code', [F32, BF16])
@pytest.mark.parametrize('size', [(2, 9, 7), (3, 24, 20)])  # the larger one runs the unrolled loops
def test_bn_train_forward_and_backward_match_autograd(cuda, c, nseg, residual, relu, code, size):
    g = torch.Generator().manual_seed(14)
    b, h, w = size
    dt = ops.torch_dtype(code)
    # activations representable in the compute dtype, so the reference sees the same
    # inputs (and the same ReLU mask) as the kernels
    z = (torch.randn(nseg * b, c, h, w, generator=g) * 2 + 0.5).to(dt).float().requires_grad_(True)
    gamma = (torch.rand(c, generator=g) + 0.5).requires_grad_(True)
    beta = (torch.randn(c, generator=g) * 0.1).requires_grad_(True)
    res = torch.randn(nseg * b, c, h, w, generator=g).to(dt).float().requires_grad_(True) if residual else None
    rm0, rv0 = torch.randn(c, generator=g) * 0.1, torch.rand(c, generator=g) + 0.5
    rm, rv = rm0.clone(), rv0.clone()
    y = _bn_ref(z, nseg, gamma, beta, rm, rv, res, relu)
    gy = torch.randn(y.shape, generator=g).to(dt).float()
    grads = torch.autograd.grad(y, [z, gamma, beta] + ([res] if residual else []), gy)
    zd = _nhwc(z.detach(), cuda, dt)
    rmd, rvd = rm0.clone().to(cuda), rv0.clone().to(cuda)
    mean, rstd, sc, sh = T.bn_train_fwd(zd, nseg, gamma.detach().to(cuda), beta.detach().to(cuda), 1e-5, 0.1,
                                        rmd, rvd)
    rd = _nhwc(res.detach(), cuda, dt) if residual else None
    yd = T.bn_apply(zd, nseg, sc, sh, rd, relu)
    dz, gres, dgam, dbet = T.bn_train_bwd(_nhwc(gy, cuda, dt), yd if relu else None, zd, nseg, mean, rstd,
                                          gamma.detach().to(cuda), want_gres=residual)
    if relu and not residual:  # mask recomputed from z instead of read from y: same result
        dz2, _, dg2, db2 = T.bn_train_bwd(_nhwc(gy, cuda, dt), None, zd, nseg, mean, rstd, gamma.detach().to(cuda),
                                          relu_from=(sc, sh))
        torch.testing.assert_close(dz2, dz, atol=0, rtol=0)
        torch.testing.assert_close(dg2, dgam, atol=0, rtol=0)
        torch.testing.assert_close(db2, dbet, atol=0, rtol=0)
    torch.cuda.synchronize()
    if code == F32:
        tol = dict(atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(rmd.cpu(), rm, **tol)
        torch.testing.assert_close(rvd.cpu(), rv, **tol)
        torch.testing.assert_close(_nchw(yd), y.detach(), **tol)
        torch.testing.assert_close(_nchw(dz), grads[0], atol=1e-4, rtol=1e-3)
        torch.testing.assert_close(dgam.cpu(), grads[1], atol=1e-3, rtol=1e-4)
        torch.testing.assert_close(dbet.cpu(), grads[2], atol=1e-3, rtol=1e-4)
        if residual:
            torch.testing.assert_close(_nchw(gres), grads[3], **tol)
    else:
        torch.testing.assert_close(rmd.cpu(), rm, atol=1e-2, rtol=1e-2)
        _close_lowp(_nchw(yd), y.detach())
        _close_lowp(_nchw(dz), grads[0], 0.03)
        _close_lowp(dgam.cpu(), grads[1], 0.03)
        _close_lowp(dbet.cpu(), grads[2], 0.03)


@pytest.mark.parametrize('code', [F32, BF16, F16])
@pytest.mark.parametrize('c,nseg,size', [(256, 2, (2, 9, 7)), (64, 4, (3, 24, 20)), (2048, 1, (2, 5, 3))])
def test_bn_relu_bitmask_equals_the_y_masked_backward(cuda, code, c, nseg, size):
    """ABI 14: bn_apply_mask writes the same y as bn_apply plus bit e = [y_e > 0] per 16-B chunk,
    and the backward reading those bits equals the one reading y, bit for bit."""
    g = torch.Generator().manual_seed(41)
    b, h, w = size
    dt = ops.torch_dtype(code)
    z = _nhwc(torch.randn(nseg * b, c, h, w, generator=g) * 2 + 0.3, cuda, dt)
    r = _nhwc(torch.randn(nseg * b, c, h, w, generator=g), cuda, dt)
    gy = _nhwc(torch.randn(nseg * b, c, h, w, generator=g), cuda, dt)
    gamma = (torch.rand(c, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(c, generator=g) * 0.1).to(cuda)
    mean, rstd, sc, sh = T.bn_train_fwd(z, nseg, gamma, beta, 1e-5, 0.1)
    y = T.bn_apply(z, nseg, sc, sh, r, True)
    y2, mask = T.bn_apply_mask(z, nseg, sc, sh, r)
    ref = T.bn_train_bwd(gy, y, z, nseg, mean, rstd, gamma, want_gres=True)
    got = T.bn_train_bwd(gy, None, z, nseg, mean, rstd, gamma, want_gres=True, mask=mask)
    torch.cuda.synchronize()
    assert torch.equal(y2, y)
    e = 16 // y.element_size()
    pos = (y.float() > 0).reshape(-1, e).to(torch.int32)
    bits = (pos << torch.arange(e, device=cuda, dtype=torch.int32)).sum(dim=1)
    assert torch.equal(mask.to(torch.int32), bits)
    for a, b_ in zip(got, ref):
        assert torch.equal(a, b_)


@pytest.mark.parametrize('code', [F32, BF16])
@pytest.mark.parametrize('shape', [(4, 17, 16, 64), (2, 32, 30, 64), (2, 9, 9, 128)])
def test_fused_stem_bn_relu_maxpool_equals_the_two_pass_path(cuda, code, shape):
    """ABI 14, the training stem: bn_relu_maxpool = max-pool of bn_apply(relu) bit for bit, and the
    backward from its stored taps = maxpool3x3s2_bwd over the activation (ReLU zeros: many ties)."""
    g = torch.Generator().manual_seed(42)
    n, h, w, c = shape
    nseg = 2
    dt = ops.torch_dtype(code)
    z = (torch.randint(-3, 4, shape, generator=g).float() * 0.5).to(cuda, dt)   # ties in every window
    gamma = (torch.rand(c, generator=g) + 0.5).to(cuda)
    beta = (torch.randn(c, generator=g) * 0.1).to(cuda)
    _, _, sc, sh = T.bn_train_fwd(z, nseg, gamma, beta, 1e-5, 0.1)
    a = T.bn_apply(z, nseg, sc, sh, None, True)
    ref = ops.maxpool3x3s2_nhwc(a, code)
    y, idx = T.bn_relu_maxpool(z, nseg, sc, sh)
    gy = torch.randint(-4, 5, ref.shape, generator=g).float().to(cuda, dt)
    gx_ref = T.maxpool3x3s2_bwd(a, gy)
    gx = T.maxpool3x3s2_bwd_idx(idx, gy, (h, w))
    torch.cuda.synchronize()
    assert torch.equal(y, ref)
    assert torch.equal(gx, gx_ref)


@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('nv,n,h', [(1, 2, 16), (4, 2, 24), (3, 1, 8), (2, 3, 64)])
def test_training_stem_conv_and_weight_gradient(cuda, code, nv, n, h):
    """ABI 14: the training stem's own kernels straight from NCHW f32 views -- the raw 7x7 / s2 / p3
    convolution and its weight gradient -- against torch autograd on the dtype-rounded operands."""
    g = torch.Generator().manual_seed(43)
    views = [torch.randn(n, 3, h, 256, generator=g) for _ in range(nv)]
    wt = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    dt = ops.torch_dtype(code)
    x = torch.cat([v.to(dt).float() for v in views])   # the kernels round the input to the dtype
    wr = wt.to(dt).float().requires_grad_(True)
    y = F.conv2d(x, wr, stride=2, padding=3)
    dy = torch.randn(y.shape, generator=g).to(dt).float()
    (dw_ref,) = torch.autograd.grad(y, wr, dy)
    vd = [v.to(cuda) for v in views]
    z = T.stem_conv(vd, wt.to(cuda), code)
    dw = T.stem_wgrad(vd, _nhwc(dy, cuda, dt), code)
    torch.cuda.synchronize()
    assert z.shape == (nv * n, h // 2, 128, 64) and dw.shape == (64, 3, 7, 7)
    _close_lowp(_nchw(z), y.detach(), 0.01)
    torch.testing.assert_close(dw.cpu(), dw_ref, atol=2e-3 * dw_ref.abs().max().item(), rtol=1e-3)


def test_channel_sum(cuda):
    g = torch.Generator().manual_seed(15)
    x = torch.randn(3, 17, 11, 64, generator=g)
    out = T.channel_sum(x.to(cuda))
    torch.testing.assert_close(out.cpu(), x.double().sum(dim=(0, 1, 2)).float(), atol=1e-4, rtol=1e-5)


@pytest.mark.parametrize('code', [F32, BF16])
def test_maxpool_backward_with_ties_matches_autograd(cuda, code):
    g = torch.Generator().manual_seed(16)
    x = torch.randint(-2, 3, (2, 64, 17, 16), generator=g).float().requires_grad_(True)  # many ties
    y = F.max_pool2d(x, 3, stride=2, padding=1)
    gy = torch.randint(-4, 5, y.shape, generator=g).float()  # exact in bf16
    (gx_ref,) = torch.autograd.grad(y, x, gy)
    dt = ops.torch_dtype(code)
    gx = T.maxpool3x3s2_bwd(_nhwc(x.detach(), cuda, dt), _nhwc(gy, cuda, dt))
    torch.testing.assert_close(_nchw(gx), gx_ref, atol=0, rtol=0)


@pytest.mark.parametrize('code', [F32])
def test_bn_train_statistics_with_a_large_mean_offset(cuda, code):
    """Channels whose mean is large against their spread (|mean| / std ~ 1e4): the partial
    sums are taken about the segment's first pixel, so the variance survives f32 partials
    (a plain E[z^2] - mean^2 loses it entirely at this ratio)."""
    g = torch.Generator().manual_seed(31)
    nseg, b, c, h, w = 2, 4, 64, 24, 20
    dt = ops.torch_dtype(code)
    offset = torch.linspace(-300, 300, c).view(1, c, 1, 1)
    z = (offset + 0.03 * torch.randn(nseg * b, c, h, w, generator=g)).to(dt).float()
    gamma, beta = torch.ones(c), torch.zeros(c)
    rm, rv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    mean, rstd, sc, sh = T.bn_train_fwd(_nhwc(z, cuda, dt), nseg, gamma.to(cuda), beta.to(cuda), 1e-5, 0.1, rm, rv)
    torch.cuda.synchronize()
    zs = z.double().view(nseg, b, c, h, w)
    mu = zs.mean(dim=(1, 3, 4))
    var = zs.var(dim=(1, 3, 4), unbiased=False)
    torch.testing.assert_close(mean.cpu().double().view(nseg, c), mu, atol=1e-4, rtol=1e-6)
    torch.testing.assert_close(rstd.cpu().double().view(nseg, c), 1 / torch.sqrt(var + 1e-5), atol=0, rtol=2e-3)


@pytest.mark.parametrize('code', [F32, BF16, F16])
def test_batched_weight_packing_equals_the_torch_packs(cuda, code):
    """posu_pack_weights (one launch for the whole training step) against packing.py's torch
    restatements, bit for bit: conv (padded stem channels, 3x3, 1x1), conv data-gradient
    (flipped + transposed, and the head's padded gradient channels), deconv parity classes and
    the deconv's data-gradient conv view."""
    g = torch.Generator(device=cuda).manual_seed(3)
    dt, bk = ops.torch_dtype(code), ops.conv_bk(code)
    w_stem = torch.randn(64, 3, 7, 7, device=cuda, generator=g)
    w3 = torch.randn(96, 40, 3, 3, device=cuda, generator=g)
    w1 = torch.randn(130, 64, 1, 1, device=cuda, generator=g)
    wdc = torch.randn(72, 48, 4, 4, device=cuda, generator=g)     # ConvTranspose2d [Cin][Cout][4][4]
    wh = torch.randn(17, 256, 1, 1, device=cuda, generator=g)
    pk = packing.BatchedPacker(code, cuda)
    outs = [
        (pk.conv(w_stem, 8, bk), packing.pack_conv_weight(w_stem, 8, bk, dt)),
        (pk.conv(w3, 40, bk), packing.pack_conv_weight(w3, 40, bk, dt)),
        (pk.dgrad(w3, bk), packing.pack_conv_dgrad_weight(w3, bk, dt)),
        (pk.conv(w1, 64, bk), packing.pack_conv_weight(w1, 64, bk, dt)),
        (pk.dgrad(w1, bk), packing.pack_conv_dgrad_weight(w1, bk, dt)),
        (pk.deconv(wdc, bk), packing.pack_deconv4x4_weight(wdc, bk, dt)),
        (pk.conv(wdc, 48, bk), packing.pack_conv_weight(wdc, 48, bk, dt)),
        # ABI 15: a 3x3 conv weight as a deconv source (zero-padded to 4x4), LDS-tiled and element-wise
        (pk.deconv(w3, bk), packing.pack_deconv4x4_weight(w3, bk, dt)),
        (pk.deconv(w3[:44, :24].contiguous(), bk), packing.pack_deconv4x4_weight(w3[:44, :24], bk, dt)),
    ]
    wpad = torch.zeros(64, 256, 1, 1, device=cuda)
    wpad[:17] = wh
    outs.append((pk.dgrad(wh, bk, cout_pitch=64), packing.pack_conv_dgrad_weight(wpad, bk, dt)))
    pk.run()
    torch.cuda.synchronize()
    for i, (got, ref) in enumerate(outs):
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        assert torch.equal(got, ref), (i, float((got.float() - ref.float()).abs().max()))
    # the parameters change in place (an optimizer step): run() re-packs the new values
    with torch.no_grad():
        w3.mul_(-0.5)
    pk.run()
    assert torch.equal(outs[1][0], packing.pack_conv_weight(w3, 40, bk, dt))


@pytest.mark.parametrize('code', [F32, BF16])
def test_batched_weight_packing_network_sizes(cuda, code):
    """The LDS-tiled packing paths at PoseResNet-50 sizes (several rows / tiles per block,
    multi-tile deconv classes) against the torch restatements, bit for bit."""
    g = torch.Generator(device=cuda).manual_seed(5)
    dt, bk = ops.torch_dtype(code), ops.conv_bk(code)
    w3 = torch.randn(512, 512, 3, 3, device=cuda, generator=g)
    w1 = torch.randn(256, 1024, 1, 1, device=cuda, generator=g)
    wdc = torch.randn(2048, 256, 4, 4, device=cuda, generator=g)
    pk = packing.BatchedPacker(code, cuda)
    outs = [
        (pk.conv(w3, 512, bk), packing.pack_conv_weight(w3, 512, bk, dt)),
        (pk.dgrad(w3, bk), packing.pack_conv_dgrad_weight(w3, bk, dt)),
        (pk.conv(w1, 1024, bk), packing.pack_conv_weight(w1, 1024, bk, dt)),
        (pk.dgrad(w1, bk), packing.pack_conv_dgrad_weight(w1, bk, dt)),
        (pk.deconv(wdc, bk), packing.pack_deconv4x4_weight(wdc, bk, dt)),
        (pk.conv(wdc, 256, bk), packing.pack_conv_weight(wdc, 256, bk, dt)),
        (pk.deconv(w3, bk), packing.pack_deconv4x4_weight(w3, bk, dt)),
    ]
    pk.run()
    torch.cuda.synchronize()
    for i, (got, ref) in enumerate(outs):
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        assert torch.equal(got, ref), (i, float((got.float() - ref.float()).abs().max()))
