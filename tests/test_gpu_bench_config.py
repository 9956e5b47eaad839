"""Parity at the benchmarked configuration (BASELINE configs[2]): exactly the plan
bench.py times -- R50@256, 32 groups x 4 views, per-layer autotuned tiles (bf16), the fused
stem / deconv+head launches, the two hipGraphs -- against the CPU oracle chain (fp32
reference network -> soft-argmax -> crop affine -> FundamentalLoss -> fp64 triangulation)
on bench's first input batch, compared by bench.compare_with_reference (the numbers the
bench line reports as mpjpe_vs_ref_mm):

  heatmap error; joint error in image px; epipolar-loss relative error;
  triangulation_same_2d_mm -- the device triangulation vs the oracle's on the same 2-D
      joints (BASELINE.json: 1e-2 mm);
  mean / max (mm) -- the pipeline's 2-D deviation from the reference chain laid on the
      synthetic poses' projections and triangulated (run/test/test_triangulate.py:98-102).

The raw end-to-end X of a random-weight network is not gated: its views' soft-argmax
joints do not correspond, so the DLT solution is ill-conditioned (see compare_with_reference).

Gates: fp32 and fp16x3 (the parity modes; fp16x3 is the bench line's parity_mode leg, autotuned
like the headline, its split tiles chosen in-run, round 6) -- heatmaps 1e-3 (BASELINE.json),
triangulation 1e-2 mm on the same 2-D joints, loss 1e-5 relative, joints and pipeline mm within
measured bands, and within 4x the reference fp32 path's own deviation from fp64.  bf16
(benchmarked mode) -- bands from the measured deviation: soft-argmax at
beta = 100 on the peakless heatmaps of a random-weight network turns bf16's ~0.02 heatmap
deviation into joint moves of tens of pixels."""
import numpy as np
import pytest
import torch

import bench
from posu import synthetic as syn
from posu.pipeline import synthetic_meta

pytestmark = pytest.mark.gpu

GROUPS, LAYERS, SIZE = 32, 50, 256
# measured on MI355X (round 2: fp32 hm 2.3e-5 / px 0.005 / mm 0.029; bf16 hm 0.19-0.21 / px 38-39).
# bf16 has no mm gate here: with random weights the heatmaps are flat noise and soft-argmax at
# beta = 100 turns a 0.02 heatmap difference into a jump between noise maxima (tens of px),
# which the DLT over four mutually inconsistent views turns into metres (472-3269 mm mean
# between runs of the same code).  The mm gates of BASELINE.json (1e-2 mm, fp32) and of the
# benched bf16 mode are in tests/test_gpu_peaked.py, on a fitted network's peaked heatmaps.
# fp32 mm band: 0.05 (measured 0.029) -- on peakless maps the reference's OWN fp32 path sits
# as far from its fp64 run (the 4x checks below), so 1e-2 mm is not reachable by any fp32 chain.
BANDS = {
    'fp32': {'hm_max': 1e-3, 'tri_max': 1e-2, 'loss_rel': 1e-5, 'px_mean': 0.02, 'mm_mean': 0.05},
    'fp16x3': {'hm_max': 1e-3, 'tri_max': 1e-2, 'loss_rel': 1e-5, 'px_mean': 0.02, 'mm_mean': 0.05},
    'bf16': {'hm_max': 0.5, 'hm_mean': 0.05, 'tri_max': 1e-2, 'loss_rel': 1e-2, 'px_mean': 100.0, 'mm_mean': None},
}


@pytest.fixture(scope='module')
def oracle_run():
    from models.pose_resnet import get_pose_net
    torch.set_num_threads(16)
    net = get_pose_net(syn.make_cfg(num_layers=LAYERS, image_size=SIZE), is_train=False)
    sd = syn.synthetic_state_dict(net.state_dict(), seed=0, bn_stats=syn.load_bn_stats(LAYERS, SIZE))
    _, host = synthetic_meta(GROUPS, 'cpu', image_size=SIZE)
    views = syn.group_views(4, range(GROUPS), SIZE, seed=100)   # = bench.input_views(all groups, batch 0)
    ref = bench.oracle_chain(sd, LAYERS, SIZE, views, host, full=True)
    ref['host'] = host
    # the reference path's own fp32 error: the same forward in fp64 (the oracle is
    # dtype-generic), heatmaps and soft-argmax coordinates
    from oracle import geometry_ref as G
    from oracle import pose_resnet_ref as PR
    hm64, _, _ = PR.pose_resnet_forward(torch.cat(views, 0).double(), {k: v.double() if v.is_floating_point() else v
                                                                      for k, v in sd.items()}, LAYERS)
    ref['hm64'] = hm64
    ref['sa64'] = G.softargmax2d(hm64)
    return ref


def _bench_plan_outputs(cuda, precision, autotune, layers=LAYERS, size=SIZE, groups=GROUPS):
    from posu import plan as P
    net = bench.build_model(layers, size, precision, cuda)
    meta, _ = synthetic_meta(groups, cuda, image_size=size)
    plan = net.plan(cuda)
    rep = bench.Replayer(plan, bench.input_views(list(range(groups)), size, 0, cuda), meta, groups, 1, True, cuda)
    with torch.no_grad():
        rep.stage_geo(rep.stage_net())
        if autotune:
            plan.autotune(plan.pack_input(rep.views), keep_features=False, reps=2)
            # every unfused conv geometry of the plan: layer2 block 0's conv1 (64x64 input), layer3
            # block 0's three convs + block 1's conv1, layer4's six distinct geometries, deconv1,
            # deconv2; layer2 block 0's conv2 and dual GEMM run in the strided tail (else +2), which
            # also computes block 1's conv1 when chained (else +1: a 32x32 conv1 launch)
            s2 = P.S2_TAIL and P.FUSED_BOTTLENECK
            expect = 12 + (0 if s2 else 2) + (0 if s2 and P.S2_CHAIN and P.CHAINED_TAILS else 1)
            assert len(P.tuned_tiles()) >= expect
        rep.capture()
        rep.run_geo(rep.run_net())
        coords, loss, X = rep.run_geo(rep.run_net())
        torch.cuda.synchronize()
    return {'hm0': rep.hm.cpu(), 'coords0': coords.cpu().numpy(), 'loss0': float(loss), 'X0': X.cpu().numpy(),
            'meta': meta}


@pytest.mark.parametrize('precision', ['fp32', 'fp16x3', 'bf16'])
def test_bench_configuration_matches_the_oracle_chain(cuda, oracle_run, precision):
    out = _bench_plan_outputs(cuda, precision, autotune=precision != 'fp32')
    c = bench.compare_with_reference(out, oracle_run, out['meta'], cuda)
    print('%s bench config vs oracle: %s' % (precision, c))
    b = BANDS[precision]
    assert np.isfinite(out['X0']).all()
    assert c['heatmap_abs_err']['max'] < b['hm_max']
    if 'hm_mean' in b:
        assert c['heatmap_abs_err']['mean'] < b['hm_mean']
    assert c['triangulation_same_2d_mm']['max'] < b['tri_max']
    assert c['epipolar_loss_rel_err'] < b['loss_rel']
    assert c['joints_px_err']['mean'] < b['px_mean']
    if b['mm_mean'] is not None:
        assert c['mean'] < b['mm_mean']
    # against fp64: the HIP path's error next to the reference fp32 path's own error
    from oracle import geometry_ref as G
    ours_hm = (out['hm0'].double() - oracle_run['hm64']).abs().max().item()
    ref_hm = (oracle_run['heatmaps'].double() - oracle_run['hm64']).abs().max().item()
    ours_sa = (G.softargmax2d(out['hm0']).double() - oracle_run['sa64']).norm(dim=-1)
    ref_sa = (G.softargmax2d(oracle_run['heatmaps']).double() - oracle_run['sa64']).norm(dim=-1)
    print('vs fp64: heatmap max |err| ours %.3g, reference fp32 path %.3g; soft-argmax heatmap-px err mean/max '
          'ours %.3g / %.3g, reference fp32 path %.3g / %.3g'
          % (ours_hm, ref_hm, ours_sa.mean(), ours_sa.max(), ref_sa.mean(), ref_sa.max()))
    if precision in ('fp32', 'fp16x3'):  # within a small factor of the reference's own fp32 precision
        assert ours_hm < 4 * ref_hm + 1e-6
        assert ours_sa.mean() < 4 * ref_sa.mean() + 1e-5


def test_r152_384_fp16_pipeline_matches_the_oracle_chain(cuda, monkeypatch):
    """configs[4]'s per-GPU pipeline at its per-GPU shape: R152 backbone at 384x384, fp16 compute,
    fp64 triangulation, 16 groups x 4 views, per-layer AUTOTUNED tiles, bench's replay path
    (hipGraph, fused stem; layer1 at 96x96 maps as conv1 + the chained down tail, the chained tail and
    the plain tail (round 6); layer3's 35 identity blocks as conv1 + the W = 24 streamed tail -- both
    asserted taken).
      * oracle subset (CPU-feasible): groups 0-1 against the fp32 CPU oracle chain;
      * full size, property checks: every output finite; the device triangulation of all 16
        groups against the oracle's DLT on the same device joints (BASELINE's 1e-2 mm); the
        device epipolar loss against the oracle FundamentalLoss of the device joints; batch
        invariance -- groups 0-1 of the 16-group autotuned run equal, bit for bit, a 2-group run
        with the heuristic tiles (every tile sums K in the same order)."""
    layers, size, groups, sub = 152, 384, 16, 2
    from models.pose_resnet import get_pose_net
    from oracle import geometry_ref as G
    torch.set_num_threads(16)
    net = get_pose_net(syn.make_cfg(num_layers=layers, image_size=size), is_train=False)
    sd = syn.synthetic_state_dict(net.state_dict(), seed=syn.calibrated_seed(layers, size),
                                  bn_stats=syn.load_bn_stats(layers, size))
    from posu import ops, plan as P
    calls = []

    def counting(fn, tag):
        def counted(t1, x, *a, **k):
            calls.append((tag,) + tuple(x.shape))
            return fn(t1, x, *a, **k)
        return counted
    for name in ('bottleneck_tail_stream_nhwc', 'bottleneck_tail_stream_next_nhwc', 'bottleneck_down_tail_stream_nhwc'):
        monkeypatch.setattr(ops, name, counting(getattr(ops, name), name))
    # (the two-K-group tile 39 sums K in another order: kept out of this bit-for-bit batch
    # invariance check)
    monkeypatch.setattr(P, 'TILES_KSPLIT', False)
    full = _bench_plan_outputs(cuda, 'fp16', True, layers=layers, size=size, groups=groups)
    # layer3's 35 identity blocks (W = 24): 34 chained tails + the plain last one per forward (round 6)
    n_full = sum(1 for c in calls if c[1:] == (64, 24, 24, 1024) and c[0] in ('bottleneck_tail_stream_nhwc',
                                                                             'bottleneck_tail_stream_next_nhwc'))
    # layer1 (96x96): per eager forward one down tail, one chained tail, one plain tail
    l1 = [sum(1 for c in calls if c == (nm, 64, 96, 96, ch)) for nm, ch in
          (('bottleneck_down_tail_stream_nhwc', 64), ('bottleneck_tail_stream_next_nhwc', 256),
           ('bottleneck_tail_stream_nhwc', 256))]
    small = _bench_plan_outputs(cuda, 'fp16', False, layers=layers, size=size, groups=sub)
    # every eager forward of the plan runs layer3's 35 identity blocks on the W = 24 tails
    assert n_full > 0 and n_full % 35 == 0, n_full
    assert l1[0] > 0 and l1[0] == l1[1] == l1[2] == n_full // 35, (l1, n_full)
    _, host = synthetic_meta(groups, 'cpu', image_size=size)
    # full size: triangulation and loss consistency of every group
    V, J = 4, full['coords0'].shape[2]
    assert np.isfinite(full['X0']).all() and np.isfinite(full['coords0']).all() and torch.isfinite(full['hm0']).all()
    p2d = full['coords0'].transpose(1, 0, 2, 3).reshape(groups * V, J, 2).astype(np.float64)
    tri = np.linalg.norm(full['X0'] - G.triangulate_poses(host['cams'], p2d), axis=-1)
    lref = G.fundamental_loss([torch.from_numpy(full['coords0'][v]) for v in range(V)], [torch.ones(groups, J, 1)] * V,
                              host['subjects'], host['F_dict'])
    print('R152@384 fp16, 16 groups: triangulation vs oracle DLT on the device joints max %.3g mm; epipolar loss '
          'rel %.3g' % (tri.max(), abs(full['loss0'] / float(lref) - 1)))
    assert tri.max() < 1e-2
    assert abs(full['loss0'] / float(lref) - 1) < 1e-4
    # batch invariance (autotuned 16-group plan vs heuristic-tile 2-group plan)
    rows = [v * groups + g for v in range(V) for g in range(sub)]
    assert torch.equal(full['hm0'][rows], small['hm0'])
    # the oracle subset: groups 0-1 against the fp32 CPU oracle chain
    _, hsub = synthetic_meta(sub, 'cpu', image_size=size)
    ref = bench.oracle_chain(sd, layers, size, syn.group_views(4, range(sub), size, seed=100), hsub, full=True)
    ref['host'] = hsub
    c = bench.compare_with_reference(small, ref, small['meta'], cuda)
    print('R152@384 fp16 pipeline (groups 0-1) vs oracle: %s' % c)
    assert c['heatmap_abs_err']['mean'] < 0.05 and c['heatmap_abs_err']['max'] < 0.5
    assert c['triangulation_same_2d_mm']['max'] < 1e-2      # the DLT itself: BASELINE's 1e-2 mm
    assert c['epipolar_loss_rel_err'] < 0.1


def test_configs1_batch64_plan_end_to_end(cuda, monkeypatch):
    """BASELINE configs[1]'s plan exactly as bench.time_configs1 runs it -- R50@256 bf16, ONE batch of 64
    frames, autotuned tiles (layer3's 4-row streamed tails at this grid), captured in a hipGraph --
    end to end: every heatmap finite, and rows 0-1 bit-identical to a 2-frame plan on the heuristic
    tiles (tile 39, which sums K in another order, kept out of the tuning here), whose heatmaps are
    checked against the fp32 CPU oracle at the bf16 band."""
    from oracle import pose_resnet_ref as PR
    from posu import plan as P
    monkeypatch.setattr(P, 'TILES_KSPLIT', False)
    net = bench.build_model(50, 256, 'bf16', cuda)
    plan = net.plan(cuda)
    views = [v.to(cuda) for v in syn.synthetic_views(1, 64, 256, seed=300)]
    with torch.no_grad():
        plan.autotune(plan.pack_input(views), keep_features=False, reps=2)
        s = torch.cuda.Stream(cuda)
        s.wait_stream(torch.cuda.current_stream(cuda))
        with torch.cuda.stream(s):
            plan.run(plan.pack_input(views), keep_features=False)
        torch.cuda.current_stream(cuda).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            hm = plan.run(plan.pack_input(views), keep_features=False)[0]
        g.replay()
        torch.cuda.synchronize()
        hm64 = hm.clone()
        from posu import plan as P
        saved = dict(P._TUNE_CACHE)
        P._TUNE_CACHE.clear()
        try:
            hm2 = plan.run(plan.pack_input([v[:2] for v in views]), keep_features=False)[0]
        finally:
            P._TUNE_CACHE.update(saved)
        torch.cuda.synchronize()
    assert torch.isfinite(hm64).all()
    assert torch.equal(hm64[:2], hm2)
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    ref, _, _ = PR.pose_resnet_forward(views[0][:2].cpu(), sd, 50)
    err = (hm2.cpu() - ref).abs()
    print('configs1 batch-64 plan: rows 0-1 vs the oracle, heatmaps max %.3g mean %.3g' % (err.max(), err.mean()))
    assert float(err.max()) < BANDS['bf16']['hm_max'] and float(err.mean()) < BANDS['bf16']['hm_mean']
