"""Kernel-level parity on the MI355X: every libposeu.so entry point against the CPU
oracle / a torch fp32 reference of the same op, on seeded inputs."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import geometry_ref as G
from posu import ops, packing, synthetic as syn
from posu._native import BF16, F16, F32

pytestmark = pytest.mark.gpu


def _conv_case(cuda, code, n, cin, h, w, cout, k, stride, pad, residual, relu, seed=0, tile=-1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    ref = F.conv2d(x, wt, stride=stride, padding=pad) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    res = None
    if residual:
        res = torch.randn_like(ref)
        ref = ref + res
    if relu:
        ref = F.relu(ref)
    dt = ops.torch_dtype(code)
    cin_pad = max(8, cin)
    xd = torch.zeros(n, h, w, cin_pad)
    xd[..., :cin] = x.permute(0, 2, 3, 1)
    xd = xd.to(cuda, dt)
    wp = packing.pack_conv_weight(wt.to(cuda), cin_pad, ops.conv_bk(code), dt)
    rd = res.permute(0, 2, 3, 1).contiguous().to(cuda, dt) if residual else None
    out = ops.conv2d_nhwc(xd, wp, cout, k, k, stride, pad, sc.to(cuda), sh.to(cuda), rd, relu, code, tile=tile)
    torch.cuda.synchronize()
    return out.float().cpu().permute(0, 3, 1, 2), ref


CONV_CASES = [
    # n, cin, h, w, cout, k, stride, pad, residual, relu
    (2, 3, 40, 36, 64, 7, 2, 3, False, True),      # stem (Cin padded to 8)
    (2, 64, 16, 16, 64, 1, 1, 0, False, True),
    (2, 64, 17, 15, 64, 3, 1, 1, False, True),     # ragged spatial
    (2, 128, 16, 16, 128, 3, 2, 1, False, True),   # strided 3x3
    (3, 64, 16, 16, 256, 1, 1, 0, True, True),     # bottleneck tail with residual
    (2, 256, 8, 8, 512, 1, 2, 0, False, False),    # downsample
    (1, 512, 4, 4, 512, 3, 1, 1, False, True),     # small M (< one tile)
]


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv2d_fp32_matches_torch(cuda, case):
    got, ref = _conv_case(cuda, F32, *case)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv2d_bf16_close_to_torch(cuda, case):
    got, ref = _conv_case(cuda, BF16, *case)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 0.03 * scale + 0.02, (err, scale)


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv2d_fp16_close_to_torch(cuda, case):
    got, ref = _conv_case(cuda, F16, *case)
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 0.004 * scale + 0.004, (err, scale)


@pytest.mark.parametrize('code,tol', [(F32, 1e-4), (BF16, 0.05), (F16, 0.01)])
def test_deconv4x4s2_matches_conv_transpose(cuda, code, tol):
    g = torch.Generator().manual_seed(3)
    n, cin, h, w, cout = 2, 64, 6, 5, 64
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cin, cout, 4, 4, generator=g) * (2.0 / (cin * 4)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    ref = F.relu(F.conv_transpose2d(x, wt, stride=2, padding=1) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    dt = ops.torch_dtype(code)
    wp = packing.pack_deconv4x4_weight(wt.to(cuda), ops.conv_bk(code), dt)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    out = ops.deconv4x4s2_nhwc(xd, wp, cout, sc.to(cuda), sh.to(cuda), True, code)
    got = out.float().cpu().permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('code,tol', [(F32, 1e-4), (BF16, 0.05), (F16, 0.01)])
def test_head1x1_writes_nchw_heatmaps(cuda, code, tol):
    g = torch.Generator().manual_seed(4)
    x = torch.randn(3, 256, 16, 16, generator=g)
    wt = torch.randn(16, 256, 1, 1, generator=g) * 0.06
    b = torch.randn(16, generator=g)
    ref = F.conv2d(x, wt, b)
    dt = ops.torch_dtype(code)
    wp = packing.pack_conv_weight(wt.to(cuda), 256, ops.conv_bk(code), dt)
    out = ops.head1x1_nchw(x.permute(0, 2, 3, 1).contiguous().to(cuda, dt), wp, 16, b.to(cuda), code)
    torch.testing.assert_close(out.cpu(), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('code', [F32, BF16, F16])
def test_maxpool_pack_unpack(cuda, code):
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, 3, 33, 30, generator=g)
    dt = ops.torch_dtype(code)
    xp = ops.pack_nchw_to_nhwc(x.to(cuda), code, 8)
    assert xp.shape == (2, 33, 30, 8)
    back = xp.float().cpu().permute(0, 3, 1, 2)
    torch.testing.assert_close(back[:, :3], x.to(dt).float())
    assert torch.all(back[:, 3:] == 0)
    y = torch.randn(2, 64, 17, 16, generator=g).to(dt)
    yn = y.permute(0, 2, 3, 1).contiguous().to(cuda)
    mp = ops.maxpool3x3s2_nhwc(yn, code)
    ref = F.max_pool2d(y.float(), 3, stride=2, padding=1)
    torch.testing.assert_close(mp.float().cpu().permute(0, 3, 1, 2), ref)
    un = ops.nhwc_to_nchw_f32(yn, code)
    torch.testing.assert_close(un.cpu(), y.float())


def test_softargmax_matches_reference_golden(cuda, golden):
    g = golden('decode.npz')
    hm = torch.from_numpy(g['heatmaps']).to(cuda)
    sa = ops.softargmax2d(hm)
    np.testing.assert_allclose(sa.cpu().numpy(), g['softargmax'], atol=2e-4, rtol=0)
    T = torch.from_numpy(g['inv_affines']).float()
    fused = ops.softargmax2d(hm, affine=T.to(cuda))
    np.testing.assert_allclose(fused.cpu().numpy(), g['transform_back'], atol=5e-3, rtol=0)
    tb = ops.affine2d(sa, T.to(cuda))
    np.testing.assert_allclose(tb.cpu().numpy(), g['transform_back'], atol=5e-3, rtol=0)


def test_softargmax_backward_matches_autograd(cuda):
    r = np.random.default_rng(0)
    hm = torch.from_numpy((0.03 * r.standard_normal((3, 5, 16, 12))).astype(np.float32))
    T = torch.from_numpy(r.uniform(-2, 2, size=(3, 2, 3)).astype(np.float32))
    gout = torch.from_numpy(r.standard_normal((3, 5, 2)).astype(np.float32))
    a = hm.clone().requires_grad_(True)
    ref = G.softargmax2d(a)
    ref = torch.einsum('njc,nkc->njk', torch.cat([ref, torch.ones(3, 5, 1)], 2), T)
    (ref * gout).sum().backward()
    b = hm.to(cuda).requires_grad_(True)
    out = ops.softargmax2d(b, affine=T.to(cuda))
    (out * gout.to(cuda)).sum().backward()
    torch.testing.assert_close(out.detach().cpu(), ref.detach(), atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(b.grad.cpu(), a.grad, atol=1e-4, rtol=1e-3)


def test_argmax_decoding_matches_reference_golden(cuda, golden):
    g = golden('decode.npz')
    hm = torch.from_numpy(g['heatmaps']).to(cuda)
    p, v = ops.argmax2d(hm, post_process=False)
    np.testing.assert_array_equal(p.cpu().numpy(), g['max_preds'])
    np.testing.assert_array_equal(v.cpu().numpy(), g['max_vals'])
    T = torch.from_numpy(g['inv_affines'])
    fp, fv = ops.argmax2d(hm, post_process=True, affine64=T.to(cuda))
    np.testing.assert_allclose(fp.cpu().numpy(), g['final_preds'], atol=1e-4, rtol=0)
    np.testing.assert_array_equal(fv.cpu().numpy(), g['final_vals'])
    fp0, _ = ops.argmax2d(hm, post_process=False, affine64=T.to(cuda))
    np.testing.assert_allclose(fp0.cpu().numpy(), g['final_preds_nopost'], atol=1e-4, rtol=0)


@pytest.mark.parametrize('tag,utw', [('w', True), ('nw', False)])
def test_epipolar_loss_and_grad_match_reference_golden(cuda, golden, tag, utw):
    from core.loss import FundamentalLoss
    g = golden('losses.npz')
    F_dict = {tuple(int(v) for v in k): f for k, f in zip(g['F_keys'], g['F_vals'])}
    cfg = syn.make_cfg(use_target_weight_fund=utw)
    crit = FundamentalLoss(cfg, fundamental_matrix_dict=F_dict, device=cuda)
    joints = [torch.tensor(j, device=cuda, requires_grad=True) for j in g['joints']]
    weights = [torch.from_numpy(w).to(cuda) for w in g['weights']]
    meta = [{'subject': torch.from_numpy(g['subjects'])} for _ in range(4)]
    loss = crit(joints, weights, meta)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g['fund_loss_' + tag], rtol=1e-5)
    grad = np.stack([j.grad.cpu().numpy() for j in joints])
    np.testing.assert_allclose(grad, g['fund_grad_' + tag], rtol=1e-5, atol=1e-9)


@pytest.mark.parametrize('tag,utw', [('w', True), ('nw', False)])
def test_joints_mse_matches_reference_golden(cuda, golden, tag, utw):
    from core.loss import JointsMSELoss
    g = golden('losses.npz')
    pred = torch.tensor(g['mse_pred'], device=cuda, requires_grad=True)
    loss = JointsMSELoss(utw)(pred, torch.from_numpy(g['mse_gt']).to(cuda), torch.from_numpy(g['mse_w']).to(cuda))
    loss.backward()
    np.testing.assert_allclose(loss.item(), g['mse_loss_' + tag], rtol=1e-5)
    np.testing.assert_allclose(pred.grad.cpu().numpy(), g['mse_grad_' + tag], rtol=1e-5, atol=1e-9)


def test_triangulation_known_answer_exact(cuda, golden):
    """Noise-free pinhole projections from the reference camera code -> exact 3-D joints."""
    from multiviews.triangulate import triangulate_poses
    g = golden('cameras.npz')
    n = g['poses3d'].shape[0]
    cams = syn.group_cameras(n, distortion=False)
    X = triangulate_poses(cams, g['proj_nodist'], no_distortion=True)
    assert X.shape == (n, 16, 3) and X.dtype == np.float64
    np.testing.assert_allclose(X, g['poses3d'], atol=1e-6, rtol=0)  # well inside the 1e-2 mm gate


def test_triangulation_matches_oracle_on_noisy_distorted_views(cuda, golden):
    from multiviews.triangulate import triangulate_poses
    g = golden('cameras.npz')
    n = g['poses3d'].shape[0]
    cams = syn.group_cameras(n, distortion=True)
    r = np.random.default_rng(1)
    p2d = g['proj'] + r.normal(0, 3.0, size=g['proj'].shape)
    vis = (r.uniform(size=p2d.shape[:2]) > 0.15).astype(np.float64)
    vis[0:4, 2] = 0          # joint unseen everywhere
    vis[4:7, 7] = 0          # seen by one view only
    ref = G.triangulate_poses(cams, p2d, joints_vis=vis, no_distortion=False)
    got = triangulate_poses(cams, p2d, joints_vis=vis, no_distortion=False)
    np.testing.assert_allclose(got, ref, atol=1e-2, rtol=0)   # 1e-2 mm gate (BASELINE.json)
    assert np.abs(got - ref).max() < 1e-5
    assert np.all(got[0, 2] == 0) and np.all(got[1, 7] == 0)
    # float32 inputs (as the h5 'locations' are) promote exactly
    got32 = triangulate_poses(cams, p2d.astype(np.float32), joints_vis=vis)
    ref32 = G.triangulate_poses(cams, p2d.astype(np.float32).astype(np.float64), joints_vis=vis)
    np.testing.assert_allclose(got32, ref32, atol=1e-2, rtol=0)


def test_triangulate_one_point_api(cuda, golden):
    from multiviews.triangulate import build_multi_camera_system, triangulate_one_point
    g = golden('cameras.npz')
    cams = syn.group_cameras(1, distortion=False)
    system = build_multi_camera_system([('camera_%d' % v, cams[v]) for v in range(4)], no_distortion=True)
    pts = [('camera_%d' % v, g['proj_nodist'][v, 4]) for v in (0, 2, 3)]
    X = triangulate_one_point(system, pts)
    np.testing.assert_allclose(X, g['poses3d'][0, 4], atol=1e-6)


@pytest.mark.parametrize('nviews', [5, 8, 12])
def test_triangulation_more_than_four_views(cuda, golden, nviews):
    """More than 4 views (posu_triangulate_dlt's 16-view kernel, rows folded into a 4 x 4 R factor by
    Givens rotations, round 6): exact on noise-free pinhole projections, and the oracle's numpy-SVD
    restatement of pymvg find3d on noisy distorted ones."""
    from multiviews.triangulate import build_multi_camera_system
    g = golden('cameras.npz')
    cams = syn.group_cameras(3, distortion=True)[:nviews]   # two subject rigs: up to 12 distinct cameras
    r = np.random.default_rng(nviews)
    for nodist in (True, False):
        system = build_multi_camera_system([('c%d' % i, c) for i, c in enumerate(cams)], no_distortion=nodist)
        oc = [G._camera(c, nodist) for c in cams]
        for X in g['poses3d'][0, :6]:
            pts = [system.find2d('c%d' % i, X, distorted=not nodist) for i in range(nviews)]
            if not nodist:
                pts = [p + r.normal(0, 2.0, size=2) for p in pts]
            got = system.find3d([('c%d' % i, p) for i, p in enumerate(pts)])
            ref = G.find3d([c[0] for c in oc], [c[1] for c in oc], [c[2] for c in oc], pts)
            if nodist:
                np.testing.assert_allclose(got, X, atol=1e-6, rtol=0)
            np.testing.assert_allclose(got, ref, atol=1e-6, rtol=0)


@pytest.mark.parametrize('code,tol', [(F32, 1e-4), (BF16, 0.05), (F16, 0.01)])
def test_s2d_stem_matches_torch(cuda, code, tol):
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 3, 36, 40, generator=g)
    w = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    sc = torch.rand(64, generator=g) + 0.5
    sh = torch.randn(64, generator=g) * 0.1
    ref = F.relu(F.conv2d(x, w, stride=2, padding=3) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    dt = ops.torch_dtype(code)
    xs = ops.pack_s2d_nchw(x.to(cuda), code, 16)
    assert xs.shape == (2, 18, 20, 16)
    wp = packing.pack_stem_s2d_weight(w.to(cuda), 16, ops.conv_bk(code), dt)
    out = ops.conv2d_nhwc(xs, wp, 64, 4, 4, 1, 2, sc.to(cuda), sh.to(cuda), None, True, code, out_hw=(18, 20))
    torch.testing.assert_close(out.float().cpu().permute(0, 3, 1, 2), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('code,tol', [(F32, 1e-4), (BF16, 0.05), (F16, 0.01)])
@pytest.mark.parametrize('stride', [1, 2])
def test_dual_1x1_tail_matches_torch(cuda, code, tol, stride):
    g = torch.Generator().manual_seed(7)
    mid, cin, cout, h = 64, 128, 256, 9
    a = torch.relu(torch.randn(3, mid, h, h, generator=g))
    x = torch.randn(3, cin, h * stride, h * stride, generator=g)
    w3 = torch.randn(cout, mid, 1, 1, generator=g) * 0.1
    wd = torch.randn(cout, cin, 1, 1, generator=g) * 0.1
    s3, sd = torch.rand(cout, generator=g) + 0.5, torch.rand(cout, generator=g) + 0.5
    b = torch.randn(cout, generator=g) * 0.1
    ref = F.relu(F.conv2d(a, w3) * s3.view(1, -1, 1, 1) + F.conv2d(x, wd, stride=stride) * sd.view(1, -1, 1, 1)
                 + b.view(1, -1, 1, 1))
    dt = ops.torch_dtype(code)
    wp = packing.pack_dual_1x1_weight(w3.to(cuda), s3.to(cuda), wd.to(cuda), sd.to(cuda), dt)
    out = ops.conv1x1_dual_nhwc(a.permute(0, 2, 3, 1).contiguous().to(cuda, dt),
                                x.permute(0, 2, 3, 1).contiguous().to(cuda, dt), stride, wp, cout, b.to(cuda), True,
                                code)
    torch.testing.assert_close(out.float().cpu().permute(0, 3, 1, 2), ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('code,tol', [(F32, 1e-4), (BF16, 0.05), (F16, 0.01)])
@pytest.mark.parametrize('keep_f', [True, False])
@pytest.mark.parametrize('shape', [(3, 5, 6, 16), (2, 24, 20, 13)])
def test_fused_deconv_head_matches_unfused(cuda, code, tol, keep_f, shape):
    """Last deconv + BN + ReLU + 1x1 head in one launch: bf16 / f16 on the 256x256
    register-epilogue tile (partial heatmaps of the four column waves summed in LDS), f32
    on the 64x256 LDS tile; ragged M, several tiles, J < 16."""
    _fused_deconv_head_case(cuda, code, tol, keep_f, shape)


def _fused_deconv_head_case(cuda, code, tol, keep_f, shape):
    g = torch.Generator().manual_seed(8)
    n, h, w, J = shape
    cin, cout = 64, 256
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cin, cout, 4, 4, generator=g) * (2.0 / (cin * 4)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    hw = torch.randn(J, cout, 1, 1, generator=g) * 0.06
    hb = torch.randn(J, generator=g)
    f_ref = F.relu(F.conv_transpose2d(x, wt, stride=2, padding=1) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    hm_ref = F.conv2d(f_ref, hw, hb)
    dt = ops.torch_dtype(code)
    wp = packing.pack_deconv4x4_weight(wt.to(cuda), ops.conv_bk(code), dt)
    hwp = packing.pack_conv_weight(hw.to(cuda), cout, ops.conv_bk(code), dt)
    xd = x.permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    hm, f = ops.deconv4x4s2_head(xd, wp, cout, sc.to(cuda), sh.to(cuda), hwp, J, hb.to(cuda), code, keep_f=keep_f)
    torch.testing.assert_close(hm.cpu(), hm_ref, atol=tol, rtol=tol)
    if keep_f:
        torch.testing.assert_close(f.float().cpu().permute(0, 3, 1, 2), f_ref, atol=tol, rtol=tol)
    else:
        assert f is None
    # identical to the two-launch path on the same device (same rounding of f)
    f2 = ops.deconv4x4s2_nhwc(xd, wp, cout, sc.to(cuda), sh.to(cuda), True, code)
    hm2 = ops.head1x1_nchw(f2, hwp, J, hb.to(cuda), code)
    torch.testing.assert_close(hm, hm2, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize('code', [BF16, F16])
def test_split_precision_head(cuda, code):
    """The fused deconv + head with the split-precision head (hw_lo, ABI 11): against the head
    computed in fp64 from the deconv output of the SAME rounded operands (so only the head's own
    arithmetic differs), at least 20x closer than the plain head, whose input is the deconv output
    rounded to the dtype; f (stored) is unchanged by the split."""
    g = torch.Generator().manual_seed(18)
    n, h, w, J = 2, 24, 20, 16
    cin, cout = 64, 256
    dt = ops.torch_dtype(code)
    x = torch.randn(n, cin, h, w, generator=g).to(dt).double()
    wt = (torch.randn(cin, cout, 4, 4, generator=g) * (2.0 / (cin * 4)) ** 0.5).to(dt).double()
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    hw = torch.randn(J, cout, 1, 1, generator=g) * 0.06
    hb = torch.randn(J, generator=g)
    f64 = F.relu(F.conv_transpose2d(x, wt, stride=2, padding=1) * sc.double().view(1, -1, 1, 1) +
                 sh.double().view(1, -1, 1, 1))
    hm64 = F.conv2d(f64, hw.double(), hb.double())
    bk = ops.conv_bk(code)
    wp = packing.pack_deconv4x4_weight(wt.float().to(cuda), bk, dt)
    hw32 = packing.pack_conv_weight(hw.to(cuda), cout, bk, torch.float32)
    hwp = hw32.to(dt)
    hwl = (hw32 - hwp.float()).to(dt)
    xd = x.float().permute(0, 2, 3, 1).contiguous().to(cuda, dt)
    args = (xd, wp, cout, sc.to(cuda), sh.to(cuda), hwp, J, hb.to(cuda), code)
    hm1, f1 = ops.deconv4x4s2_head(*args)
    hm2, f2 = ops.deconv4x4s2_head(*args, head_w_lo=hwl)
    torch.cuda.synchronize()
    e1 = float((hm1.double().cpu() - hm64).abs().max())
    e2 = float((hm2.double().cpu() - hm64).abs().max())
    print('head vs fp64: plain %.3g, split %.3g (%.0fx)' % (e1, e2, e1 / max(e2, 1e-30)))
    assert torch.equal(f1, f2)
    assert e2 * 20 < e1
    assert e2 < (3e-4 if code == BF16 else 1e-4)


@pytest.mark.parametrize('case', CONV_CASES[1:5])
def test_conv2d_three_stage_ring_matches_torch(cuda, case):
    got, ref = _conv_case(cuda, F32, *case, tile=16 + (1 if case[4] < 128 else 3))
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize('cfg', [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 15, 16, 17, 18, 19, 20, 22, 23, 31, 33, 37,
                                 39])
@pytest.mark.parametrize('code', [F32, BF16, F16])
def test_every_tile_configuration_matches_torch(cuda, cfg, code):
    """Each tile shape (incl. LDS rings above 64 KiB, eight-wave blocks, the single- /
    three-slot variants, the staggered and persistent loops) on ragged shapes: 3x3 with
    residual, 1x1 strided."""
    cout = 256 if (cfg & 7) in (3, 4, 5, 6, 7) else 64
    for case in [(2, 64, 17, 15, cout, 3, 1, 1, True, True), (3, 128, 12, 12, cout, 1, 2, 0, False, False)]:
        got, ref = _conv_case(cuda, code, *case, tile=cfg)
        if code == F32:
            torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)
        else:
            assert (got - ref).abs().max().item() <= 0.03 * ref.abs().max().item() + 0.02


def test_invalid_tile_is_refused(cuda):
    x = torch.zeros(1, 8, 8, 64, device=cuda, dtype=torch.bfloat16)
    w = torch.zeros(64, 64, device=cuda, dtype=torch.bfloat16)
    # (7 / 15: the 128x128 eight-wave tiles since round 4; 39 round 5; 47 / 55 split fp16, round 6)
    for bad in (63, 29, 64, 70, 40 + 5):
        with pytest.raises(RuntimeError, match='tile must be'):
            ops.conv2d_nhwc(x, w, 64, 1, 1, 1, 0, None, None, None, False, BF16, tile=bad)


@pytest.mark.parametrize('cfg', [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize('code', [BF16, F16])
def test_persistent_stream_bit_exact_vs_one_block_per_tile(cuda, cfg, code):
    """The persistent K-tile stream (tile + 32) walks each tile's K in the same order as the
    one-block-per-tile kernel: outputs equal bit for bit for 3x3 + residual (ragged M,
    K-tiles >> ring), 1x1 + residual with one K-tile per tile (several epilogues inside the
    ring window), strided 1x1, ConvTranspose(4, s2) and the two-source Bottleneck tail."""
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=cuda).manual_seed(7)
    cout = 256
    sc = torch.rand(cout, device=cuda, generator=g) + 0.5
    sh = torch.randn(cout, device=cuda, generator=g) * 0.1

    def rnd(*shape, scale=1.0):
        return (torch.randn(*shape, device=cuda, generator=g) * scale).to(dt)

    x = rnd(7, 21, 19, 128)
    x64 = rnd(7, 21, 19, 64)
    res = rnd(7, 21, 19, cout)
    x2 = rnd(7, 42, 38, 64)
    w3 = rnd(cout, 9 * 128, scale=0.03)
    w1 = rnd(cout, 64, scale=0.1)
    wd = rnd(cout, 128 + 64, scale=0.05)
    wdc = rnd(4, cout, 4 * 128, scale=0.03)
    outs = {}
    for t in (cfg, cfg + 32):
        outs[t] = [
            ops.conv2d_nhwc(x, w3, cout, 3, 3, 1, 1, sc, sh, res, True, code, tile=t),
            ops.conv2d_nhwc(x64, w1, cout, 1, 1, 1, 0, sc, sh, res, True, code, tile=t),
            ops.conv2d_nhwc(x, w3[:, :128].contiguous(), cout, 1, 1, 2, 0, sc, sh, None, False, code, tile=t),
            ops.deconv4x4s2_nhwc(x, wdc, cout, sc, sh, True, code, tile=t),
            ops.conv1x1_dual_nhwc(x, x2, 2, wd, cout, sh, True, code, tile=t),
        ]
    torch.cuda.synchronize()
    for a, b in zip(outs[cfg], outs[cfg + 32]):
        assert torch.equal(a, b)


@pytest.mark.parametrize('code', [F32, BF16, F16])
def test_staggered_tiles_bit_exact_vs_two_slot(cuda, code):
    """The staggered loops (tiles 23 / 31: waves 4-7 half a K-tile behind) keep each
    accumulator's K order, so their outputs equal the two-slot loops (tiles 5 / 6) bit for
    bit: 3x3 + residual (ragged M), strided 1x1, ConvTranspose(4, s2) and the two-source
    Bottleneck tail.  (f32 has no staggered loop: its 23 / 31 run as 5 / 6.)"""
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=cuda).manual_seed(5)
    sc = torch.rand(256, device=cuda, generator=g) + 0.5
    sh = torch.randn(256, device=cuda, generator=g) * 0.1
    bk = ops.conv_bk(code)

    def rnd(*shape):
        return torch.randn(*shape, device=cuda, generator=g).to(dt)

    x = rnd(9, 33, 31, 128)
    res = rnd(9, 33, 31, 256)
    w3 = (rnd(256, 9 * 128).float() * 0.03).to(dt)
    x2 = rnd(9, 66, 62, 64)
    wd = (rnd(256, 128 + 64).float() * 0.05).to(dt)
    wdc = (rnd(4, 256, 4 * 128).float() * 0.03).to(dt)
    assert (9 * 128) % bk == 0
    outs = {}
    for t in (5, 23, 6, 31, 3, 7, 15):
        outs[t] = [
            ops.conv2d_nhwc(x, w3, 256, 3, 3, 1, 1, sc, sh, res, True, code, tile=t),
            ops.conv2d_nhwc(x, w3[:, :128].contiguous(), 256, 1, 1, 2, 0, sc, sh, None, False, code, tile=t),
            ops.deconv4x4s2_nhwc(x, wdc, 256, sc, sh, True, code, tile=t),
            ops.conv1x1_dual_nhwc(x, x2, 2, wd, 256, sh, True, code, tile=t),
        ]
    torch.cuda.synchronize()
    for t, base in ((23, 5), (31, 6), (7, 3), (15, 3)):   # 7 / 15: 128x128 eight-wave staggered (round 4)
        for a, b in zip(outs[base], outs[t]):
            assert torch.equal(a, b), (t, float((a.float() - b.float()).abs().max()))


@pytest.mark.parametrize('code', [F32, BF16])
def test_training_conv_tiles_bit_identical(cuda, code):
    """The training convolutions (raw, no BN epilogue: train_plan._conv_tuned) run on whichever
    tile the autotuner timed fastest; the claim that the choice changes speed, not results,
    holds only if every candidate of plan._tile_candidates accumulates in the same K order.
    One raw conv per geometry class (3x3 / 1x1, stride 1 / 2, ragged M) on every candidate
    tile, outputs equal bit for bit."""
    from posu.plan import _tile_candidates
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=cuda).manual_seed(11)
    for cin, h, w, cout, k, stride, pad in [(64, 17, 15, 256, 3, 1, 1), (256, 13, 11, 64, 1, 1, 0),
                                             (128, 18, 14, 128, 3, 2, 1), (256, 18, 14, 512, 1, 2, 0)]:
        x = torch.randn(3, h, w, cin, device=cuda, generator=g).to(dt)
        wt = (torch.randn(cout, k * k * cin, device=cuda, generator=g) * (k * k * cin) ** -0.5).to(dt)
        outs = {t: ops.conv2d_nhwc(x, wt, cout, k, k, stride, pad, None, None, None, False, code, tile=t)
                for t in _tile_candidates(cout)}
        torch.cuda.synchronize()
        t0 = _tile_candidates(cout)[0]
        for t, o in outs.items():
            assert torch.equal(o, outs[t0]), (cin, k, stride, cout, t)


@pytest.mark.parametrize('code,tol', [(F32, 1e-4), (BF16, None)])
@pytest.mark.parametrize('cout', [256, 384])
def test_conv2d_big_tiles_match_torch(cuda, code, tol, cout):
    """Large grids take the eight-wave 256 x 256 tiles (residual epilogue in passes) when
    Cout % 256 == 0; 384 channels take the automatic fallback (128 x 128)."""
    case = (64, 64, 32, 32, cout, 3, 1, 1, True, True)  # M = 65536: >= 256 big tiles
    got, ref = _conv_case(cuda, code, *case)
    if tol is None:
        assert (got - ref).abs().max().item() <= 0.03 * ref.abs().max().item() + 0.02
    else:
        torch.testing.assert_close(got, ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('distortion', [False, True])
def test_ransac_and_reprojection_match_oracle(cuda, distortion):
    """Pseudo-label geometry (triangulate.py:102-213): inlier masks bit-exact and
    re-projections to 1e-4 px against the numpy restatement, on noisy views with gross
    outliers and partial visibility."""
    from multiviews.triangulate import camera_tables
    ng = 8
    cams = syn.group_cameras(ng, distortion=distortion)
    poses = syn.synthetic_poses3d(ng)
    r = np.random.default_rng(17)
    p2d = np.zeros((ng * 4, 16, 2))
    for gi in range(ng):
        for v in range(4):
            M, K, D = G._camera(cams[gi * 4 + v], no_distortion=not distortion)
            p2d[gi * 4 + v] = [G.find2d(M, K, D, X) for X in poses[gi]]
    p2d += r.normal(0, 1.5, size=p2d.shape)
    bad = r.uniform(size=p2d.shape[:2]) < 0.15
    p2d[bad] += r.choice([-1, 1], size=(bad.sum(), 2)) * r.uniform(60, 120, size=(bad.sum(), 2))
    vis = (r.uniform(size=p2d.shape[:2]) > 0.1).astype(np.int64)
    ref_vis = G.ransac(p2d, cams, vis, reproj_thre=10, num_inliers=2, no_distortion=not distortion)
    ref_proj, ref_rv = G.reproject_poses(p2d, cams, vis, no_distortion=not distortion)
    M, intr = camera_tables(cams, 4, no_distortion=not distortion)
    Md, Id = torch.from_numpy(M).to(cuda), torch.from_numpy(intr).to(cuda)
    xy = torch.from_numpy(p2d.reshape(ng, 4, 16, 2)).to(cuda)
    vd = torch.from_numpy(vis.reshape(ng, 4, 16)).to(cuda)
    got = ops.ransac_inliers(Md, Id, xy, vd, 10.0, 2).cpu().numpy().reshape(ng * 4, 16)
    np.testing.assert_array_equal(got, ref_vis)
    proj, rv = ops.reproject(Md, Id, xy, vd)
    np.testing.assert_array_equal(rv.cpu().numpy().reshape(ng * 4, 16), ref_rv)
    np.testing.assert_allclose(proj.cpu().numpy().reshape(ng * 4, 16, 2), ref_proj, atol=1e-4, rtol=0)
    # the drop-in functions (reference signatures) give the same answers
    from multiviews.triangulate import ransac, reproject_poses
    cfg = syn.make_cfg()
    cfg.DATASET.NO_DISTORTION = not distortion
    cfg.PSEUDO_LABEL.NUM_INLIERS, cfg.PSEUDO_LABEL.REPROJ_THRE = 2, 10
    np.testing.assert_array_equal(ransac(p2d, cams, vis, cfg), ref_vis)
    pr, rvis = reproject_poses(p2d, cams, vis, no_distortion=not distortion)
    np.testing.assert_allclose(pr, ref_proj, atol=1e-4, rtol=0)


@pytest.mark.parametrize('size', [256, 384])
@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('hflip', [False, True])
def test_fused_stem_pool_matches_two_launch_path(cuda, size, code, hflip):
    """posu_stem_pool_fwd (input pack + 7x7/s2 stem + BN + ReLU + 3x3/s2 max-pool in one
    launch) against the pack -> space-to-depth stem -> max-pool launches on the same
    inputs: equal up to the f32 summation order of the stem (one rounding step at most),
    including the padded top row / left column, odd batch and the flip test's mirror."""
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=cuda).manual_seed(21)
    n = 3
    x = torch.randn(n, 3, size, size, device=cuda, generator=g)
    wt = torch.randn(64, 3, 7, 7, device=cuda, generator=g) * (2.0 / 147) ** 0.5
    sc = torch.rand(64, device=cuda, generator=g) + 0.5
    sh = torch.randn(64, device=cuda, generator=g) * 0.1
    got = ops.stem_pool(x, packing.pack_stem_fused_weight(wt, dt), sc, sh, code, hflip=hflip)
    xp = ops.pack_s2d_nchw(x, code, 16, hflip=hflip)
    ws = packing.pack_stem_s2d_weight(wt, 16, ops.conv_bk(code), dt)
    stem = ops.conv2d_nhwc(xp, ws, 64, 4, 4, 1, 2, sc, sh, None, True, code, out_hw=(size // 2, size // 2))
    ref = ops.maxpool3x3s2_nhwc(stem, code)
    torch.cuda.synchronize()
    assert got.shape == ref.shape == (n, size // 4, size // 4, 64)
    d = (got.float() - ref.float()).abs()
    ulp = (2.0 ** -7 if code == BF16 else 2.0 ** -10) * ref.float().abs()
    assert bool((d <= 2 * ulp + 1e-3).all()), float(d.max())
    assert float((d > 0).float().mean()) < 0.05


@pytest.mark.parametrize('size,nv', [(256, 32), (384, 16)])
@pytest.mark.parametrize('code', [BF16, F16])
@pytest.mark.parametrize('hflip', [False, True])
def test_stem_pool_views_one_launch(cuda, size, nv, code, hflip):
    """posu_stem_pool_views_fwd at the bench shapes (4 views x 32 frames at 256, x 16 at 384: strips
    of 16 / 24 consecutive pool-row pairs per block, the rolling input ring and the carried stem
    row): against the two-launch path per view (one rounding step at most), and bit-identical to
    one posu_stem_pool_fwd launch per view (every stem value is the same MFMA sequence)."""
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=cuda).manual_seed(23)
    views = [torch.randn(nv, 3, size, size, device=cuda, generator=g) for _ in range(4)]
    wt = torch.randn(64, 3, 7, 7, device=cuda, generator=g) * (2.0 / 147) ** 0.5
    sc = torch.rand(64, device=cuda, generator=g) + 0.5
    sh = torch.randn(64, device=cuda, generator=g) * 0.1
    wpk = packing.pack_stem_fused_weight(wt, dt)
    out = torch.empty(4 * nv, size // 4, size // 4, 64, device=cuda, dtype=dt)
    out.view(torch.int16).fill_(0x7fc1 if code == BF16 else 0x7e01)   # NaN sentinel: every pixel written
    got = ops.stem_pool_views(views, wpk, sc, sh, code, out=out, hflip=hflip)
    per_view = torch.cat([ops.stem_pool(v, wpk, sc, sh, code, hflip=hflip) for v in views])
    ws = packing.pack_stem_s2d_weight(wt, 16, ops.conv_bk(code), dt)
    refs = []
    for v in views:
        stem = ops.conv2d_nhwc(ops.pack_s2d_nchw(v, code, 16, hflip=hflip), ws, 64, 4, 4, 1, 2, sc, sh, None, True,
                               code, out_hw=(size // 2, size // 2))
        refs.append(ops.maxpool3x3s2_nhwc(stem, code))
    ref = torch.cat(refs)
    torch.cuda.synchronize()
    assert torch.equal(got, per_view)
    d = (got.float() - ref.float()).abs()
    ulp = (2.0 ** -7 if code == BF16 else 2.0 ** -10) * ref.float().abs()
    assert bool((d <= 2 * ulp + 1e-3).all()), float(d.max())
    assert float((d > 0).float().mean()) < 0.05


@pytest.mark.parametrize('code', [BF16, F16])
def test_ksplit_tile_close_to_the_plain_tile(cuda, code):
    """Tile 39 (two K groups of four waves, partial sums added in LDS): the same products as the
    plain 128 x 128 tile, summed in another order -- outputs within a rounding step of it, every
    epilogue path (residual, stride 2, deconv parity classes, the dual GEMM, ragged M, an odd
    K-tile count)."""
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=cuda).manual_seed(9)
    sc = torch.rand(256, device=cuda, generator=g) + 0.5
    sh = torch.randn(256, device=cuda, generator=g) * 0.1

    def rnd(*shape, s=1.0):
        return (torch.randn(*shape, device=cuda, generator=g) * s).to(dt)

    x = rnd(5, 23, 19, 128)
    res = rnd(5, 23, 19, 256)
    w3 = rnd(256, 9 * 128, s=0.03)
    x2 = rnd(5, 46, 38, 64)
    wd = rnd(256, 128 + 64, s=0.05)   # K = 192: three K-tiles (the last pair half empty)
    wdc = rnd(4, 256, 4 * 128, s=0.03)
    outs = {}
    for t in (3, 39):
        outs[t] = [
            ops.conv2d_nhwc(x, w3, 256, 3, 3, 1, 1, sc, sh, res, True, code, tile=t),
            ops.conv2d_nhwc(x, w3[:, :128].contiguous(), 256, 1, 1, 2, 0, sc, sh, None, False, code, tile=t),
            ops.deconv4x4s2_nhwc(x, wdc, 256, sc, sh, True, code, tile=t),
            ops.conv1x1_dual_nhwc(x, x2, 2, wd, 256, sh, True, code, tile=t),
        ]
    torch.cuda.synchronize()
    ulp = 2.0 ** (-7 if code == BF16 else -10)
    for a, b in zip(outs[3], outs[39]):
        a, b = a.float(), b.float()
        d = (a - b).abs()
        assert float(d.max()) <= 2 * ulp * float(a.abs().max()) + 1e-6
        assert float((d > 0).float().mean()) < 0.1   # most outputs round identically
