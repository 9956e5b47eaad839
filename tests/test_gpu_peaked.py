"""Parity of the BENCHED chains on peaked, trained-like heatmaps (the verdict's round-2 gap:
random-weight heatmaps are flat, so their soft-argmax joints measure nothing).

R50@256 is fitted on the GPU through the product training path (tools/peaked.py: bf16, per-view
BatchNorm, Adam lr 1e-3, 1200 steps, ~15 s) to Gaussian targets at the projections of synthetic
3-D poses, on crops that show a coloured blob per joint; its heatmaps then peak (~0.9) where the
poses project and the oracle chain triangulates them to ~10 mm of the synthetic ground truth.
Then bench's chain (eval plan -> soft-argmax + crop affine -> fp64 DLT) in bf16 and in fp32 is
compared with the CPU oracle chain (fp32 reference forward -> soft-argmax -> transform_back ->
triangulate_poses, run/test/test_triangulate.py:98-101 arithmetic) on the same weights.

Gates: fp32 and fp16x3 (the split-fp16 mode, round 5) -- BASELINE.json's bars: heatmaps 1e-3,
triangulated joints 1e-2 mm (mean AND max).  bf16 and fp16 (the plan's default split-precision head, plan.PRECISE_HEAD) -- 2 x the
deviation measured at round 4 (profiles/r04/precision_attribution_r4e.json, deterministic: the
same fitted net and the same chains give the same figures run to run):
    bf16  heatmaps 0.0163 max / 3.2e-4 mean, joints 0.131 px mean, 0.656 mm mean / 3.03 mm max
    fp16  heatmaps 0.00205 max / 3.9e-5 mean, joints 0.0147 px mean, 0.068 mm mean / 0.209 mm max"""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))


@pytest.fixture(scope='module')
def fitted(cuda):
    import peaked
    torch.set_num_threads(16)
    net, task = peaked.fit_peaked(cuda, steps=1200)
    res32, ref = peaked.parity(net, task, cuda, 'fp32')
    res16, _ = peaked.parity(net, task, cuda, 'bf16', ref)
    resh, _ = peaked.parity(net, task, cuda, 'fp16', ref)
    ress, _ = peaked.parity(net, task, cuda, 'fp16x3', ref)
    print('fp32:', res32)
    print('bf16:', res16)
    print('fp16:', resh)
    print('fp16x3:', ress)
    return res32, res16, resh, ress


def test_fitted_network_is_trained_like(fitted):
    res32 = fitted[0]
    assert res32['heatmap_peak_mean'] > 0.8 and res32['heatmap_peak_min'] > 0.4
    assert res32['oracle_mpjpe_vs_gt_mm'] < 25.0


@pytest.mark.parametrize('which', [0, 3], ids=['fp32', 'fp16x3'])
def test_chain_meets_the_baseline_bars_on_peaked_heatmaps(fitted, which):
    r = fitted[which]
    assert r['heatmap_abs_err']['max'] < 1e-3
    assert r['mpjpe_vs_ref_mm']['mean'] < 1e-2 and r['mpjpe_vs_ref_mm']['max'] < 1e-2


def test_bf16_chain_on_peaked_heatmaps(fitted):
    from posu import plan
    assert plan.PRECISE_HEAD, 'the bands below are the split-precision head\'s'
    r = fitted[1]
    assert r['heatmap_abs_err']['max'] < 0.033 and r['heatmap_abs_err']['mean'] < 6.4e-4
    assert r['joints_px_err']['mean'] < 0.27
    assert r['mpjpe_vs_ref_mm']['mean'] < 1.32 and r['mpjpe_vs_ref_mm']['max'] < 6.1


def test_fp16_chain_on_peaked_heatmaps(fitted):
    r = fitted[2]
    assert r['heatmap_abs_err']['max'] < 4.2e-3 and r['heatmap_abs_err']['mean'] < 7.8e-5
    assert r['joints_px_err']['mean'] < 0.03
    assert r['mpjpe_vs_ref_mm']['mean'] < 0.14 and r['mpjpe_vs_ref_mm']['max'] < 0.42
