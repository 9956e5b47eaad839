"""Model-level parity on the MI355X: the HIP PoseResNet against heatmaps the reference
produced (fp32 mode, 1e-3 gate from BASELINE.json), the bf16 / fp16 deviation, the multi-view
wrapper, and the full 4-view pipeline against the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import geometry_ref as G
from oracle import pose_resnet_ref as PR
from posu import synthetic as syn

pytestmark = pytest.mark.gpu

HEATMAP_TOL = 1e-3  # BASELINE.json: heatmaps within 1e-3 of the reference CPU path


def _model(num_layers, size, seed, precision, device):
    from models.pose_resnet import get_pose_net
    net = get_pose_net(syn.make_cfg(num_layers=num_layers, image_size=size), is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=seed,
                                                 bn_stats=syn.load_bn_stats(num_layers, size)))
    return net.to(device).eval()


@pytest.mark.parametrize('precision', ['fp32', 'fp16x3'])
@pytest.mark.parametrize('num_layers,size', [(18, 128), (50, 256), (152, 384)])
def test_pose_resnet_fp32_matches_reference_heatmaps(cuda, golden, num_layers, size, precision):
    """fp32 and the split-fp16 mode (fp16x3) both at the 1e-3 parity gate."""
    g = golden('pose_resnet_r%d_%d.npz' % (num_layers, size))
    net = _model(num_layers, size, int(g['seed']), precision, cuda)
    x = torch.cat(syn.synthetic_views(1, int(g['batch']), size, seed=int(g['input_seed'])), 0)
    with torch.no_grad():
        hm, x1, f = net(x.to(cuda))
    assert hm.shape == g['heatmaps'].shape and hm.dtype == torch.float32
    np.testing.assert_allclose(hm.cpu().numpy(), g['heatmaps'], atol=HEATMAP_TOL, rtol=0)
    # intermediate features: same 1e-3 gate as the heatmaps
    np.testing.assert_allclose(x1.float().mean(dim=(0, 2, 3)).cpu().numpy(), g['x1_mean'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(x1[:, :8, :8, :8].float().cpu().numpy(), g['x1_slice'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(f.float().mean(dim=(0, 2, 3)).cpu().numpy(), g['f_mean'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(f[:, :8, :8, :8].float().cpu().numpy(), g['f_slice'], atol=1e-3, rtol=0)


@pytest.mark.parametrize('precision,num_layers,size,max_mean,max_abs', [
    # measured (round 2): bf16 R50 mean 0.0226 max 0.145; fp16 R50 0.0029 / 0.021; fp16 R152@384 0.0122 / 0.088
    ('bf16', 50, 256, 0.03, 0.2),
    ('fp16', 50, 256, 0.004, 0.03),
    ('fp16', 152, 384, 0.016, 0.12),  # BASELINE configs[4]: R152@384 fp16 backbone
])
def test_pose_resnet_low_precision_deviation_is_bounded(cuda, golden, precision, num_layers, size, max_mean,
                                                        max_abs):
    """bf16 / fp16 operands with f32 accumulation against the reference's fp32 heatmaps:
    report-only accuracy gates (not the 1e-3 parity gate, which is the fp32 mode's)."""
    g = golden('pose_resnet_r%d_%d.npz' % (num_layers, size))
    net = _model(num_layers, size, int(g['seed']), precision, cuda)
    x = torch.cat(syn.synthetic_views(1, int(g['batch']), size, seed=int(g['input_seed'])), 0)
    with torch.no_grad():
        hm, x1, f = net(x.to(cuda))
    # the reference's f32 features whatever the plan's operand type (pose_resnet.py:197-205)
    assert x1.dtype == torch.float32 and f.dtype == torch.float32 and torch.isfinite(x1).all()
    hm = hm.cpu().numpy()
    assert np.isfinite(hm).all()
    err = np.abs(hm - g['heatmaps'])
    print('%s R%d@%d heatmap deviation vs reference: max %.4f mean %.5f' % (precision, num_layers, size,
                                                                          err.max(), err.mean()))
    assert err.mean() < max_mean and err.max() < max_abs


def test_multiview_forward_equals_per_view_forward(cuda):
    from models.multiview_pose_resnet import get_multiview_pose_net
    net = _model(18, 128, 1, 'fp32', cuda)
    mv = get_multiview_pose_net(net, syn.make_cfg(num_layers=18, image_size=128))
    views = [v.to(cuda) for v in syn.synthetic_views(4, 3, 128, seed=9)]
    with torch.no_grad():
        single, multi, low, high = mv(views)
        assert len(single) == 4 and multi == [] and len(low) == 4 and len(high) == 4
        for v, hm in zip(views, single):
            ref, _, _ = net(v)
            torch.testing.assert_close(hm, ref, atol=1e-5, rtol=1e-5)
        assert single[0].shape == (3, 16, 32, 32)
        assert low[0].shape == (3, 64, 32, 32) and high[0].shape == (3, 256, 32, 32)  # BasicBlock: 64-ch layer1


def test_pipeline_matches_cpu_oracle(cuda):
    """forward -> soft-argmax + affine -> epipolar loss -> triangulation vs the oracle chain."""
    from posu.pipeline import MultiViewPipeline, synthetic_meta
    ng, size = 4, 128
    net = _model(18, size, 1, 'fp32', cuda)
    meta, host = synthetic_meta(ng, cuda, image_size=size)
    views = [v.to(cuda) for v in syn.synthetic_views(4, ng, size, seed=21)]
    with torch.no_grad():
        hm, coords, loss, X = MultiViewPipeline(net).step(views, meta)
    torch.cuda.synchronize()
    # oracle chain on CPU
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    x_all = torch.cat([v.cpu() for v in views], 0)
    hm_ref, _, _ = PR.pose_resnet_forward(x_all, sd, 18)
    np.testing.assert_allclose(hm.cpu().numpy(), hm_ref.numpy(), atol=HEATMAP_TOL, rtol=0)
    sa = G.softargmax2d(hm.cpu())  # decode the device heatmaps: isolates the decode/geometry stages
    img = G.transform_back(sa, host['centers'].reshape(-1, 2), host['scales'].reshape(-1, 2), [32, 32])
    np.testing.assert_allclose(coords.reshape(-1, 16, 2).cpu().numpy(), img.numpy(), atol=5e-3, rtol=0)
    joints = [torch.from_numpy(coords[v].cpu().numpy()) for v in range(4)]
    ones = [torch.ones(ng, 16, 1) for _ in range(4)]
    lref = G.fundamental_loss(joints, ones, host['subjects'], host['F_dict'])
    np.testing.assert_allclose(loss.item(), lref.item(), rtol=1e-4)
    p2d = coords.permute(1, 0, 2, 3).reshape(ng * 4, 16, 2).double().cpu().numpy()
    Xref = G.triangulate_poses(host['cams'], p2d.astype(np.float32).astype(np.float64))
    np.testing.assert_allclose(X.cpu().numpy(), Xref, atol=1e-2, rtol=1e-9)


@pytest.mark.parametrize('chunks,early', [(2, 2), (4, 2), (2, 1), (2, 3)])
def test_chunked_depth_first_run_equals_whole_batch(cuda, chunks, early):
    from posu import plan as P
    net = _model(50, 128, 0, 'fp32', cuda)
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 128, seed=4)]
    plan = net.plan(cuda)
    x = plan.pack_input(views)
    saved = P.EARLY_LAYERS
    try:
        P.EARLY_LAYERS = early   # the chunked early stage: stem..layer2 (2) or stem..layer1 (1)
        with torch.no_grad():
            hm0, x10, f0 = plan.run(x)
            hm1, x11, f1 = plan.run(x, chunks=chunks)
            hm2, x12, f2 = plan.run(x, chunks=chunks, keep_features=False)
    finally:
        P.EARLY_LAYERS = saved
    assert x12 is None and f2 is None
    torch.testing.assert_close(hm1, hm0, atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(hm2, hm0, atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(x11, x10, atol=1e-6, rtol=1e-6)
    torch.testing.assert_close(f1, f0, atol=1e-6, rtol=1e-6)


@pytest.mark.parametrize('early', [2, 1, 3])
def test_split_plan_runs_chunked_by_default_and_equals_whole_batch(cuda, early):
    """fp16x3 (round 6): run() takes plan.CHUNKS_F16X3 = 2 depth-first halves by default, the layers'
    last tails chaining the next layers' first conv1 inside each half and across into the whole-batch
    part -- heatmaps, layer1 output and deconv features bit-identical to the whole-batch run (every
    kernel's per-pixel sums are the same)."""
    from posu import plan as P
    net = _model(50, 256, 0, 'fp16x3', cuda)
    views = [v.to(cuda) for v in syn.synthetic_views(4, 2, 256, seed=6)]
    plan = net.plan(cuda)
    assert plan.default_chunks() == P.CHUNKS_F16X3 == 2
    x = plan.pack_input(views)
    saved = P.EARLY_LAYERS
    try:
        P.EARLY_LAYERS = early
        with torch.no_grad():
            hm0, x10, f0 = plan.run(x, chunks=1)
            hm1, x11, f1 = plan.run(x)
            hm2, _, _ = plan.run(x, keep_features=False)
    finally:
        P.EARLY_LAYERS = saved
    torch.cuda.synchronize()
    assert torch.equal(hm1, hm0) and torch.equal(hm2, hm0)
    assert torch.equal(x11, x10) and torch.equal(f1, f0)


def test_chunked_run_with_fused_stem_equals_whole_batch(cuda):
    """bf16 at 256x256 hands the views to the fused stem (RawViews); chunked runs slice
    them per chunk (a chunk may cover part of a view) and give the whole-batch result."""
    from posu.plan import RawViews
    net = _model(50, 256, 0, 'bf16', cuda)
    views = [v.to(cuda) for v in syn.synthetic_views(4, 3, 256, seed=5)]
    plan = net.plan(cuda)
    x = plan.pack_input(views)
    assert isinstance(x, RawViews) and x.shape[0] == 12
    assert [v.shape[0] for v in x[2:7].views] == [1, 3, 1]
    with torch.no_grad():
        hm0, _, _ = plan.run(x, keep_features=False)
        hm1, _, _ = plan.run(x, chunks=4, keep_features=False)
    torch.testing.assert_close(hm1, hm0, atol=1e-3, rtol=0)
