"""Parity of the BENCHED chains on peaked, trained-like heatmaps (the verdict's round-2 gap:
random-weight heatmaps are flat, so their soft-argmax joints measure nothing).

R50@256 is fitted on the GPU through the product training path (tools/peaked.py: bf16, per-view
BatchNorm, Adam lr 1e-3, 1200 steps, ~15 s) to Gaussian targets at the projections of synthetic
3-D poses, on crops that show a coloured blob per joint; its heatmaps then peak (~0.9) where the
poses project and the oracle chain triangulates them to ~10 mm of the synthetic ground truth.
Then bench's chain (eval plan -> soft-argmax + crop affine -> fp64 DLT) in bf16 and in fp32 is
compared with the CPU oracle chain (fp32 reference forward -> soft-argmax -> transform_back ->
triangulate_poses, run/test/test_triangulate.py:98-101 arithmetic) on the same weights.

Gates: fp32 -- BASELINE.json's bars: heatmaps 1e-3, triangulated joints 1e-2 mm (mean AND
max).  bf16 -- bands from the measured deviation (round 3: heatmaps 0.038 max / 7.6e-4 mean,
joints 0.26 px mean, 1.34 mm mean / 6.5 mm max MPJPE against the fp32 reference chain)."""
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
    print('fp32:', res32)
    print('bf16:', res16)
    return res32, res16


def test_fitted_network_is_trained_like(fitted):
    res32, _ = fitted
    assert res32['heatmap_peak_mean'] > 0.8 and res32['heatmap_peak_min'] > 0.4
    assert res32['oracle_mpjpe_vs_gt_mm'] < 25.0


def test_fp32_chain_meets_the_baseline_bars_on_peaked_heatmaps(fitted):
    r, _ = fitted
    assert r['heatmap_abs_err']['max'] < 1e-3
    assert r['mpjpe_vs_ref_mm']['mean'] < 1e-2 and r['mpjpe_vs_ref_mm']['max'] < 1e-2


def test_bf16_chain_on_peaked_heatmaps(fitted):
    _, r = fitted
    assert r['heatmap_abs_err']['max'] < 0.1 and r['heatmap_abs_err']['mean'] < 5e-3
    assert r['joints_px_err']['mean'] < 1.0
    assert r['mpjpe_vs_ref_mm']['mean'] < 5.0 and r['mpjpe_vs_ref_mm']['max'] < 25.0
