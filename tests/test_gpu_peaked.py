"""Parity of the BENCHED chains on peaked, trained-like heatmaps (the verdict's round-2 gap:
random-weight heatmaps are flat, so their soft-argmax joints measure nothing).

R50@256 is fitted on the GPU through the product training path (tools/peaked.py: fp32 since round 6,
per-view BatchNorm, Adam lr 1e-3, 1200 steps, ~30 s) to Gaussian targets at the projections of
synthetic 3-D poses, on crops that show a coloured blob per joint; its heatmaps then peak (~0.9) where
the poses project and the oracle chain triangulates them to ~9 mm of the synthetic ground truth.
Then bench's chains (eval plan -> soft-argmax + crop affine -> fp64 DLT) are compared with the CPU
oracle chain (fp32 reference forward -> soft-argmax -> transform_back -> triangulate_poses,
run/test/test_triangulate.py:98-101 arithmetic) on the same weights.

Gates: fp32 and fp16x3 (the split-fp16 parity mode; also with its tiles autotuned on the task, as
the bench's parity_mode leg tunes them) -- BASELINE.json's bars: heatmaps 1e-3, triangulated joints
1e-2 mm (mean AND max).  bf16 and fp16 (the plan's default split-precision head, plan.PRECISE_HEAD) --
absolute bands at 2 x the deviation measured on this fitted net (round 6, call r6e):
    bf16  heatmaps 0.0185 max / 3.2e-4 mean, joints 0.147 px mean, 0.701 mm mean / 3.76 mm max
    fp16  heatmaps 0.00191 max / 4.0e-5 mean, joints 0.0193 px mean, 0.095 mm mean / 0.393 mm max
and fp16 at <= 1/4 of the same net's bf16 (3 more mantissa bits).  Round 5 fitted through the bf16
training path, and the fitted net -- with the heavy-tailed max-over-joints of the 2-byte chains -- moved
whenever the bf16 training kernels' summation order changed (fp16 max 0.209 -> 0.481 mm); the fp32
fit does not depend on the bf16 kernels, so the bands are absolute again."""
import os
import sys

import numpy as np
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
    rest, _ = peaked.parity(net, task, cuda, 'fp16x3', ref, autotune=True)   # the tuner's split tiles
    print('fp32:', res32)
    print('bf16:', res16)
    print('fp16:', resh)
    print('fp16x3:', ress)
    print('fp16x3 autotuned:', rest)
    return res32, res16, resh, ress, net, task, rest


def _res(fitted, which):
    return fitted[6] if which == 6 else fitted[which]


def test_fitted_network_is_trained_like(fitted):
    res32 = fitted[0]
    assert res32['heatmap_peak_mean'] > 0.8 and res32['heatmap_peak_min'] > 0.4
    assert res32['oracle_mpjpe_vs_gt_mm'] < 25.0


@pytest.mark.parametrize('which', [0, 3, 6], ids=['fp32', 'fp16x3', 'fp16x3-autotuned'])
def test_chain_meets_the_baseline_bars_on_peaked_heatmaps(fitted, which):
    r = _res(fitted, which)
    assert r['heatmap_abs_err']['max'] < 1e-3
    assert r['mpjpe_vs_ref_mm']['mean'] < 1e-2 and r['mpjpe_vs_ref_mm']['max'] < 1e-2


def test_bf16_chain_on_peaked_heatmaps(fitted):
    from posu import plan
    assert plan.PRECISE_HEAD, 'the bands below are the split-precision head\'s'
    r = fitted[1]
    assert r['heatmap_abs_err']['max'] < 0.037 and r['heatmap_abs_err']['mean'] < 6.4e-4
    assert r['joints_px_err']['mean'] < 0.29
    assert r['mpjpe_vs_ref_mm']['mean'] < 1.4 and r['mpjpe_vs_ref_mm']['max'] < 7.5


def test_fp16_chain_on_peaked_heatmaps(fitted):
    r, rb = fitted[2], fitted[1]
    assert r['heatmap_abs_err']['max'] < 3.8e-3 and r['heatmap_abs_err']['mean'] < 8e-5
    assert r['joints_px_err']['mean'] < 0.039
    assert r['mpjpe_vs_ref_mm']['mean'] < 0.19 and r['mpjpe_vs_ref_mm']['max'] < 0.79
    # the same fitted net's bf16 chain: fp16's 3 extra mantissa bits, at least 4x closer (module doc)
    assert r['mpjpe_vs_ref_mm']['mean'] <= rb['mpjpe_vs_ref_mm']['mean'] / 4
    assert r['mpjpe_vs_ref_mm']['max'] <= rb['mpjpe_vs_ref_mm']['max'] / 4


@pytest.mark.parametrize('fund_weight', [5.0, 0.0], ids=['mse+fund5', 'mse-only'])
def test_bf16_train_step_on_peaked_network(fitted, cuda, fund_weight):
    """The bf16 training step (JointsMSE + fund_weight x FundamentalLoss, per-view batch BN) on the
    FITTED network, whose heatmaps peak, against the oracle's autograd of the same step: with
    peaked heatmaps the soft-argmax joints no longer follow the heatmaps' rounding noise, so this
    separates the bf16 backward's own deviation from the FundamentalLoss's amplification of flat
    heatmaps (test_gpu_train.py's random-init network)."""
    from models.pose_resnet import get_pose_net
    from posu import synthetic as syn
    from test_gpu_train import _step
    from test_oracle_golden import train_step_oracle
    net0, task = fitted[4], fitted[5]
    net = get_pose_net(syn.make_cfg(num_layers=50, image_size=256), is_train=False, precision='bf16')
    net.load_state_dict(net0.state_dict())
    net = net.to(cuda)
    groups = task['groups']
    host = task['host']
    # targets 2 heatmap px right of the fitted ones: the net (fitted in fp32 to the unshifted targets) sits
    # at the fp32 optimum of those, where the MSE gradient is rounding noise; against shifted targets
    # the MSE gradient is a real signal for the bf16 backward to reproduce
    targets = torch.roll(task['target'], shifts=2, dims=-1).cpu().numpy()
    g = {'num_layers': 50, 'image_size': 256, 'nviews': 4, 'batch': groups, 'seed': 0, 'fund_weight': fund_weight,
         'targets': targets, 'target_weight': np.ones((4, groups, 16, 1), np.float32),
         'centers': host['centers'], 'scales': host['scales'], 'subjects': np.asarray(host['subjects'])}
    sd = {k: v.detach().cpu().clone() for k, v in net.state_dict().items()}
    net, hm, joints, mse, fund = _step(cuda, g, 'bf16', net=net, views=task['views'])
    params, _, hm_r, _, mse_r, fund_r = train_step_oracle(g, sd=sd, views=[v.cpu() for v in task['views']])
    named = dict(net.named_parameters())
    names = list(named)
    rel = np.abs(np.array([named[n].grad.norm().item() / params[n].grad.norm().item() - 1 for n in names]))
    ga = torch.cat([named[n].grad.detach().double().cpu().ravel() for n in names])
    gr = torch.cat([params[n].grad.detach().double().ravel() for n in names])
    cos = float(ga @ gr / (ga.norm() * gr.norm()))
    hm_err = float((torch.stack(hm).detach().cpu() - hm_r.detach()).abs().max())
    # attribution: the FundamentalLoss gradient w.r.t. the heatmaps, by the oracle's own autograd
    # (soft-argmax -> transform_back -> FundamentalLoss, all fp32 CPU), taken once at the bf16
    # forward's heatmaps and once at the oracle's -- how much of the parameter-gradient deviation the
    # forward's heatmap rounding alone accounts for, whatever the backward's precision
    from oracle import geometry_ref as G
    hcos = float('nan')
    if fund_weight > 0:
        def fund_hm_grad(maps):
            hs = [m.detach().float().cpu().clone().requires_grad_(True) for m in maps]
            joints = [G.transform_back(G.softargmax2d(h), host['centers'][v],
                                       host['scales'][v], [64, 64]) for v, h in enumerate(hs)]
            G.fundamental_loss(joints, [torch.ones(groups, 16, 1)] * 4, host['subjects'],
                               syn.fundamental_dict()).backward()
            return torch.cat([h.grad.double().ravel() for h in hs])
        ha, hr = fund_hm_grad(hm), fund_hm_grad(list(hm_r))
        hcos = float(ha @ hr / (ha.norm() * hr.norm()))
    print('peaked bf16 train step (fund_weight %g) vs oracle: heatmaps max %.3g, mse %.6g vs %.6g, fund %.6g vs %.6g, '
          'grad-norm rel median %.3g max %.3g (%s), cosine %.6f; FundamentalLoss d/d(heatmaps) at the bf16 vs the '
          'oracle forward\'s heatmaps (oracle autograd): cosine %.6f'
          % (fund_weight, hm_err, mse.item(), mse_r.item(), float(fund.detach()), float(fund_r.detach()), np.median(rel), rel.max(),
             names[int(rel.argmax())], cos, hcos))
    b = PEAKED_TRAIN_BF16[fund_weight > 0]
    assert hm_err < b['hm']
    assert abs(mse.item() / mse_r.item() - 1) < b['loss']
    assert np.median(rel) < b['norm_median'] and cos > b['cos']


# about 2 x the round-6 measurement (call r6g; the fp32-fitted net, targets shifted 2 px): heatmaps
# 0.0351 max, MSE 1.8e-3 relative; gradients with the FundamentalLoss x 5 (the reference's fund5 config)
# median 0.034 / cosine 0.751, JointsMSE only 0.0089 / 0.917 (the worst tensor: final_layer.bias, whose
# gradient -- the heatmaps' summed residual -- nearly cancels).  Why the FundamentalLoss step stays near
# 0.75: the oracle's own autograd of the FundamentalLoss w.r.t. the heatmaps, taken at the bf16
# forward's heatmaps against the oracle's, agrees only to cosine 0.715 -- the soft-argmax at beta = 100
# turns the bf16 forward's heatmap rounding (0.035 max) into a different gradient before any backward
# kernel runs, so no backward precision can lift it (the faithful training step is the fp32 mode,
# test_gpu_train.py)
PEAKED_TRAIN_BF16 = {True: {'hm': 0.07, 'loss': 0.03, 'norm_median': 0.07, 'cos': 0.5},
                     False: {'hm': 0.07, 'loss': 0.03, 'norm_median': 0.02, 'cos': 0.83}}
