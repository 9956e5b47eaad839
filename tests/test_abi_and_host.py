"""CPU-side checks: the C-ABI library loads and exports every declared symbol, and the
host logic (weight packing / sub-pixel deconv decomposition, crop affines, camera
tables, synthetic data determinism) is right.  No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from posu import _native, packing, synthetic as syn

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    src = open(os.path.join(REPO, 'include', 'posu.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(posu_\w+)\s*\(', src)))


def test_library_exports_every_declared_symbol():
    lib = _native.load()
    declared = _declared_symbols()
    assert len(declared) >= 18
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(declared) == _native.exported_symbols()
    assert lib.posu_abi_version() == _native.ABI_VERSION == 16
    assert lib.posu_conv_bk(_native.BF16) == 64 and lib.posu_conv_bk(_native.F32) == 32
    assert lib.posu_conv_bk(_native.F16X3) == 64   # halves: 32 logical k per K-tile


def test_argument_errors_are_reported_without_a_gpu():
    # shape validation happens on the host before any launch
    lib = _native.load()
    st = lib.posu_conv2d_fwd(_native.BF16, None, 1, 8, 8, 8, None, 64, 3, 3, 1, 1, None, None, None, 1, None, 8, 8,
                             -1, None)
    assert st == 1 and 'null pointer' in _native.last_error()
    st = lib.posu_triangulate_dlt(None, None, None, _native.F32, 128, 32, None, 1, 4, 16, 1, None, None)
    assert st == 1
    # the split dtype needs logical channel counts in 32-channel granules, and is inference-only
    p = ctypes.c_void_p(16)
    st = lib.posu_conv2d_fwd(_native.F16X3, p, 1, 8, 8, 16, p, 64, 3, 3, 1, 1, None, None, None, 1, p, 8, 8, -1, None)
    assert st == 1 and 'multiples of 32' in _native.last_error()
    st = lib.posu_conv2d_dgrad(_native.F16X3, p, 1, 8, 8, 64, p, 64, 3, 3, 1, 1, None, p, 8, 8, None)
    assert st == 1 and 'inference-only' in _native.last_error()


def test_split_pack_layout():
    """packing.to_split: per 32-k block [hi 32 | lo 32], hi = fp16(v 2^e), lo = fp16(v 2^e - hi)."""
    torch.manual_seed(3)
    w = torch.randn(64, 96, dtype=torch.float32) * 0.03
    e = packing.split_exponent(w)
    assert 2.0 ** (packing.SPLIT_WEIGHT_EXP - 1) < float(w.abs().max()) * 2.0 ** e <= 2.0 ** packing.SPLIT_WEIGHT_EXP
    s = packing.to_split(w, e)
    assert s.shape == (64, 192) and s.dtype == torch.float16
    blk = s.view(64, 3, 2, 32).double()
    v = (blk[:, :, 0] + blk[:, :, 1]).reshape(64, 96) * 2.0 ** -e
    assert float((v - w.double()).abs().max()) <= float(w.abs().max()) * 2.0 ** -21
    assert torch.equal(blk[:, :, 0].reshape(64, 96).half(), (w.double() * 2.0 ** e).half())


def _im2col_nhwc(x, kh, kw, stride, pad):
    """[N, H, W, C] -> [N*Ho*Wo, kh*kw*C] with k = (kh, kw, c) (the kernel's A operand)."""
    n, h, w, c = x.shape
    xp = F.pad(x.permute(0, 3, 1, 2), (pad, pad, pad, pad)).permute(0, 2, 3, 1)
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (w + 2 * pad - kw) // stride + 1
    cols = []
    for i in range(kh):
        for j in range(kw):
            cols.append(xp[:, i:i + stride * ho:stride, j:j + stride * wo:stride, :])
    return torch.cat(cols, dim=3).reshape(n * ho * wo, kh * kw * c), ho, wo


@pytest.mark.parametrize('cin,cout,k,stride,pad,cin_pad', [(3, 64, 7, 2, 3, 8), (64, 64, 3, 1, 1, 64),
                                                           (128, 256, 1, 2, 0, 128), (256, 16, 1, 1, 0, 256)])
def test_conv_weight_packing_is_the_implicit_gemm_B_operand(cin, cout, k, stride, pad, cin_pad):
    torch.manual_seed(0)
    w = torch.randn(cout, cin, k, k)
    x = torch.randn(2, cin, 13, 11)
    ref = F.conv2d(x, w, stride=stride, padding=pad)
    bk = 64
    wp = packing.pack_conv_weight(w, cin_pad, bk, torch.float32)
    assert wp.shape[0] % 64 == 0 and wp.shape[1] % bk == 0
    xn = torch.zeros(2, 13, 11, cin_pad)
    xn[..., :cin] = x.permute(0, 2, 3, 1)
    A, ho, wo = _im2col_nhwc(xn, k, k, stride, pad)
    Kd = A.shape[1]
    out = A @ wp[:cout, :Kd].t()
    got = out.reshape(2, ho, wo, cout).permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_deconv_subpixel_decomposition_matches_conv_transpose():
    torch.manual_seed(1)
    cin, cout, h, w = 16, 24, 5, 7
    wt = torch.randn(cin, cout, 4, 4)
    x = torch.randn(2, cin, h, w)
    ref = F.conv_transpose2d(x, wt, stride=2, padding=1)
    wp = packing.pack_deconv4x4_weight(wt, 32, torch.float32)  # [4, CoutPad, Kpad]
    xn = x.permute(0, 2, 3, 1)
    out = torch.zeros(2, 2 * h, 2 * w, cout)
    for py in range(2):
        for px in range(2):
            # class (py, px): inputs qy + py - 1 + ty -> pad (1-py) before, py after
            xp = F.pad(xn.permute(0, 3, 1, 2), (1 - px, px, 1 - py, py)).permute(0, 2, 3, 1)
            A, ho, wo = _im2col_nhwc(xp, 2, 2, 1, 0)
            assert (ho, wo) == (h, w)
            o = A @ wp[py * 2 + px, :cout, :4 * cin].t()
            out[:, py::2, px::2, :] = o.reshape(2, h, w, cout)
    torch.testing.assert_close(out.permute(0, 3, 1, 2), ref, atol=1e-4, rtol=1e-4)


def test_bn_folding_matches_eval_batchnorm():
    bn = torch.nn.BatchNorm2d(8)
    bn.eval()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_()
        bn.running_mean.normal_()
        bn.running_var.uniform_(0.5, 2)
    bias = torch.randn(8)
    x = torch.randn(3, 8, 4, 4)
    sc, sh = packing.fold_bn(bn, bias)
    torch.testing.assert_close(x * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1),
                               bn(x + bias.view(1, -1, 1, 1)), atol=1e-5, rtol=1e-5)


def test_crop_affine_matches_reference(golden):
    from utils.transforms import get_affine_transform, transform_preds
    g = golden('decode.npz')
    for c, s, ref in zip(g['centers'], g['scales'], g['inv_affines']):
        np.testing.assert_allclose(get_affine_transform(c, s, 0, [64, 64], inv=1), ref, rtol=1e-12, atol=1e-9)
    pts = g['max_preds'][1]
    out = transform_preds(pts, g['centers'][1], g['scales'][1], [64, 64])
    np.testing.assert_allclose(out[:, :2], pts @ g['inv_affines'][1][:, :2].T + g['inv_affines'][1][:, 2],
                               rtol=1e-9)


def test_camera_tables_project_like_the_reference(golden):
    from multiviews.triangulate import camera_tables
    from multiviews.cameras import project_pose, camera_to_world_frame, world_to_camera_frame
    g = golden('cameras.npz')
    G_ = g['poses3d'].shape[0]
    cams = syn.group_cameras(G_, distortion=False)
    M, intr = camera_tables(cams, 4, no_distortion=True)
    assert M.shape == (G_, 4, 3, 4) and intr.shape == (G_, 4, 9)
    Xh = np.concatenate([g['poses3d'], np.ones((G_, 16, 1))], axis=2)
    for gi in range(G_):
        for v in range(4):
            uvw = Xh[gi] @ M[gi, v].T
            np.testing.assert_allclose(uvw[:, :2] / uvw[:, 2:], g['proj_nodist'][gi * 4 + v], rtol=1e-10)
            np.testing.assert_allclose(project_pose(g['poses3d'][gi], cams[gi * 4 + v]),
                                       g['proj_nodist'][gi * 4 + v], rtol=1e-12, atol=1e-9)
    cams_d = syn.group_cameras(G_, distortion=True)
    for gi in range(G_):
        np.testing.assert_allclose(project_pose(g['poses3d'][gi], cams_d[gi * 4]), g['proj'][gi * 4], rtol=1e-12,
                                   atol=1e-9)
    c0 = cams_d[0]
    np.testing.assert_allclose(world_to_camera_frame(g['poses3d'][0], c0['R'], c0['T']), g['cam_frame'][0],
                               rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(camera_to_world_frame(g['cam_frame'][0], c0['R'], c0['T']), g['world_back'][0],
                               rtol=1e-12, atol=1e-9)


def test_synthetic_state_dict_is_deterministic_and_keyed_like_the_reference():
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=50), is_train=False)
    sd1 = syn.synthetic_state_dict(net.state_dict(), seed=0)
    sd2 = syn.synthetic_state_dict(net.state_dict(), seed=0)
    assert list(sd1) == list(net.state_dict())
    assert len(sd1) == 338  # reference R50 PoseResNet state entries
    for k in sd1:
        assert torch.equal(sd1[k], sd2[k])
    net.load_state_dict(sd1)
    assert 'deconv_layers.6.weight' in sd1 and 'final_layer.bias' in sd1
    assert sum(p.numel() for p in net.parameters()) == 33_999_376 or \
        abs(sum(p.numel() for p in net.parameters()) - 34.0e6) < 0.1e6


def test_seeded_init_weights_draw_the_reference_tensors(golden):
    """get_pose_net(is_train=True) after torch.manual_seed(s) draws bit-identical tensors
    to the reference's (pose_resnet.py:234-247, module construction order included) on the
    host the golden was made on (torch's CPU RNG kernels may draw differently on another
    CPU, so the GPU trajectory test starts from the numpy-drawn init below)."""
    from models.pose_resnet import get_pose_net
    g = golden('adam_r18_128.npz')
    torch.manual_seed(int(g['init_seed']))
    net = get_pose_net(syn.make_cfg(num_layers=int(g['num_layers']), image_size=int(g['image_size'])), is_train=True)
    assert [n for n, _ in net.named_parameters()] == list(g['param_names'])
    sums = np.array([float(p.detach().double().sum()) for p in net.parameters()])
    if not np.array_equal(sums, g['torch_init_sums']):
        t = torch.empty(1000)
        torch.manual_seed(0)
        t.normal_()
        pytest.skip('torch CPU RNG draws differ on this host (first normal %.9g)' % float(t[0]))
    # the numpy-drawn init of the Adam trajectory golden
    net.load_state_dict(syn.reference_init_state_dict(net.state_dict(), seed=int(g['init_seed'])))
    sums = np.array([float(p.detach().double().sum()) for p in net.parameters()])
    np.testing.assert_allclose(sums, g['init_sums'], rtol=1e-10, atol=1e-12)


def test_fundamental_loss_missing_pair_raises_like_the_reference():
    """The reference looks F up per (subject, i, j) (loss.py:127): a missing key is a
    KeyError, not a zero matrix."""
    from core.loss import FundamentalLoss
    F = syn.fundamental_dict()
    fl = FundamentalLoss(syn.make_cfg(), fundamental_matrix_dict=F, device=torch.device('cpu'))
    assert fl.subject_indices([9, 11]).tolist() == [fl.subjects.index(9), fl.subjects.index(11)]
    broken = dict(F)
    del broken[(11, 2, 1)]
    fl = FundamentalLoss(syn.make_cfg(), fundamental_matrix_dict=broken, device=torch.device('cpu'))
    fl.subject_indices([9, 9])  # subject 9 is complete
    with pytest.raises(KeyError):
        fl.subject_indices([9, 11])
    with pytest.raises(KeyError):
        fl.subject_indices([5])


def test_forward_refuses_cpu_tensors():
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=18, image_size=64), is_train=False).eval()
    with pytest.raises(RuntimeError, match='cuda'):
        net(torch.zeros(1, 3, 64, 64))
    net.train()  # the training path refuses CPU tensors the same way
    with pytest.raises(RuntimeError, match='cuda'):
        net(torch.zeros(1, 3, 64, 64))
    net.precision = 'fp16'  # fp16 training would need loss scaling: refused
    with pytest.raises(NotImplementedError):
        net.train_plan()


def _s2d(x, cpad):
    n, c, h, w = x.shape
    out = torch.zeros(n, h // 2, w // 2, cpad)
    for dy in range(2):
        for dx in range(2):
            sub = dy * 2 + dx
            out[..., sub * c:(sub + 1) * c] = x[:, :, dy::2, dx::2].permute(0, 2, 3, 1)
    return out


def test_space_to_depth_stem_equals_7x7_stride2_conv():
    torch.manual_seed(2)
    x = torch.randn(2, 3, 20, 18)
    w = torch.randn(64, 3, 7, 7)
    ref = F.conv2d(x, w, stride=2, padding=3)
    wp = packing.pack_stem_s2d_weight(w, 16, 64, torch.float32)
    xs = _s2d(x, 16)
    # 4x4 / stride 1 / top-left pad 2 (bottom/right pad 1) over the s2d grid
    xp = F.pad(xs.permute(0, 3, 1, 2), (2, 1, 2, 1)).permute(0, 2, 3, 1)
    A, ho, wo = _im2col_nhwc(xp, 4, 4, 1, 0)
    assert (ho, wo) == (10, 9)
    got = (A @ wp[:64, :256].t()).reshape(2, ho, wo, 64).permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_dual_tail_weight_folds_both_bn_branches():
    torch.manual_seed(3)
    mid, cin, cout = 16, 24, 32
    w3, wd = torch.randn(cout, mid, 1, 1), torch.randn(cout, cin, 1, 1)
    s3, sd = torch.rand(cout) + 0.5, torch.rand(cout) + 0.5
    a, x = torch.randn(2, mid, 5, 5), torch.randn(2, cin, 10, 10)
    ref = F.conv2d(a, w3) * s3.view(1, -1, 1, 1) + F.conv2d(x, wd, stride=2) * sd.view(1, -1, 1, 1)
    wp = packing.pack_dual_1x1_weight(w3, s3, wd, sd, torch.float32)
    assert wp.shape == (64, mid + cin)
    feat = torch.cat([a.permute(0, 2, 3, 1), x[:, :, ::2, ::2].permute(0, 2, 3, 1)], dim=3)
    got = (feat @ wp[:cout].t()).permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=1e-4, rtol=1e-4)


def test_bottleneck_conv3_order_is_the_accumulator_fragment_order():
    """conv2's 16x16x32 accumulators (lane (p, q): channels 4q..4q+3 of n-tiles 2b and 2b+1)
    read as conv3's B fragment (lane (p, q): k = 8q + e) map k-step b's k = 8q + e to channel
    32b + 16(e >> 2) + 4q + (e & 3); the packed conv3 weight reads the same channel there, so
    the product sums every channel exactly once."""
    order = packing.bottleneck_conv3_order(64)
    assert sorted(order) == list(range(64))
    for b in range(2):
        for q in range(4):
            acc_channels = [32 * b + 4 * q + e for e in range(4)] + [32 * b + 16 + 4 * q + e for e in range(4)]
            assert order[32 * b + 8 * q:32 * b + 8 * q + 8] == acc_channels
    w = torch.randn(256, 64, 1, 1)
    wp = packing.pack_bottleneck_conv3_weight(w, torch.float32)
    t = torch.randn(64)
    torch.testing.assert_close(wp @ t[order], w.view(256, 64) @ t)
    # conv1: lane q of k-step s reads the residual chunk of output pair s (epilogue lane q:
    # channels 32 s + 16 (q & 1) + 8 (q >> 1) .. + 7)
    o1 = packing.bottleneck_conv1_order(256)
    assert sorted(o1) == list(range(256))
    for s in range(8):
        for q in range(4):
            assert o1[32 * s + 8 * q:32 * s + 8 * q + 8] == [32 * s + 16 * (q & 1) + 8 * (q >> 1) + e for e in range(8)]
    w1 = torch.randn(64, 256, 1, 1)
    x = torch.randn(256)
    torch.testing.assert_close(packing.pack_bottleneck_conv1_weight(w1, torch.float32) @ x[o1], w1.view(64, 256) @ x)


@pytest.mark.parametrize('planes,c', [(128, 512), (256, 1024)])
def test_chained_tail_stream_interleaves_the_next_conv1(planes, c):
    """pack_tail_stream(w2, w3, w1n): the plain tail's stream with, after conv3 chunk nc, the next
    conv1's KT k-steps over that chunk's channels (wave cq: n-tiles 2 cq, 2 cq + 1), so the kernel
    walks one linear stream of equal KT-step blocks (csrc/tail_stream.hip, NEXT)."""
    w2, w3, w1n = torch.randn(planes, 9 * planes), torch.randn(c, planes), torch.randn(planes, c)
    plain, chained = packing.pack_tail_stream(w2, w3), packing.pack_tail_stream(w2, w3, w1n)
    ncq = kt = planes // 32
    nc = c // planes
    assert chained.shape == (ncq, 9 * kt + 2 * nc * kt, 2, 64, 8)
    assert torch.equal(plain[:, :9 * kt], chained[:, :9 * kt])
    f1 = packing.mfma_fragments(w1n)
    for n in range(nc):
        base = 9 * kt + 2 * n * kt
        assert torch.equal(plain[:, 9 * kt + n * kt:9 * kt + (n + 1) * kt], chained[:, base:base + kt])
        for q in range(ncq):
            for j in range(2):
                assert torch.equal(chained[q, base + kt:base + 2 * kt, j], f1[2 * q + j, n * kt:(n + 1) * kt])
    with pytest.raises(ValueError):
        packing.pack_tail_stream(w2, w3, torch.randn(planes, c // 2))


def test_fused_bottleneck_byte_guard():
    """Batches whose activations pass the fused kernels' 32-bit byte offsets take the
    convolution path (plan._fused_fits) instead of a RuntimeError from the kernel's check."""
    from posu import plan as P
    ok = torch.empty((128, 64, 64, 64), dtype=torch.bfloat16, device='meta')
    assert P._fused_fits(ok, 256)                        # layer1 block 0 at batch 128
    big = torch.empty((1024, 64, 64, 256), dtype=torch.bfloat16, device='meta')
    assert not P._fused_fits(big, 256)                   # 2 GiB of layer1 output
    assert not P._fused_fits(torch.empty((1024, 64, 64, 64), dtype=torch.bfloat16, device='meta'), 256)
    assert P._fused_fits(torch.empty((1023, 64, 64, 256), dtype=torch.bfloat16, device='meta'), 256)


def test_u2a_indices_and_mpjpe_follow_test_triangulate():
    """posu.metrics against run/test/test_triangulate.py:84-102 written out: the u2a mapping
    (union index -> dataset index, '*' dropped, sorted by union index), pred3d[:, u] only for GT
    2-D inputs, gt3d[:, a], per-joint Euclidean error mean / std / max."""
    import numpy as np
    from posu.metrics import mpjpe_stats, u2a_indices
    u2a = {5: 2, 0: 0, 3: '*', 1: 4, 7: 1, 2: '*', 6: 3, 4: 5}
    u, a = u2a_indices(u2a)
    np.testing.assert_array_equal(u, [0, 1, 4, 5, 6, 7])
    np.testing.assert_array_equal(a, [0, 4, 5, 2, 3, 1])
    rng = np.random.default_rng(3)
    pred_union = rng.normal(0, 500, (7, 8, 3))        # triangulated from GT 2-D: union order
    gt = rng.normal(0, 500, (7, 6, 3))                # dataset order
    st = mpjpe_stats(pred_union, gt, u, a, pred_in_union_order=False)
    norm = np.linalg.norm(pred_union[:, u, :] - gt[:, a, :], axis=2)
    assert st['mean'] == np.mean(norm) and st['std'] == np.std(norm) and st['max'] == np.amax(norm)
    pred_sel = pred_union[:, u, :]                     # read from the validate() h5 (already u-selected)
    st2 = mpjpe_stats(pred_sel, gt, u, a, pred_in_union_order=True)
    assert st2['mean'] == st['mean'] and np.array_equal(st2['per_joint'], norm)


def test_bench_plan_flags_boolean_and_integer(monkeypatch):
    """bench.py --plan-flag: booleans take 0 / 1, integer switches an integer; anything else exits."""
    import bench
    from posu import plan as P
    monkeypatch.setattr(P, 'S2_CHAIN', True)
    monkeypatch.setattr(P, 'STEM_CIN_PAD', 8)
    bench.apply_plan_flags(['S2_CHAIN=0', 'STEM_CIN_PAD=16'])
    assert P.S2_CHAIN is False and P.STEM_CIN_PAD == 16
    for bad in ('S2_CHAIN=2', 'STEM_CIN_PAD=x', 'NO_SUCH_SWITCH=1'):
        with pytest.raises(SystemExit):
            bench.apply_plan_flags([bad])
