"""A trained-like PoseResNet for parity measurements on peaked heatmaps (test / bench harness,
not product code).

With random synthetic weights the heatmaps are flat noise, and the reference's soft-argmax
(softmax of 100 x heatmap, lib/utils/transforms.py:149-171) turns a 0.02 heatmap difference
into a jump between noise maxima -- a joint deviation that measures nothing about the kernels.
Here the network is first fitted, on the GPU through the product training path (fp32 since round 6 --
the fitted net then does not move when the bf16 training kernels' summation order changes, which
moved the 2-byte chains' heavy-tailed max-over-joints in round 5; per-view BatchNorm, Adam lr 1e-3 as
in the reference), to Gaussian targets (sigma 2, NETWORK.SIGMA of
the reference config) at the projections of synthetic 3-D poses into the four cameras of each
group; its heatmaps then peak where the poses project, like a trained network's, and the
benched bf16 / fp32 chains can be compared with the CPU oracle chain on them (heatmaps, image-px
joints, triangulated joints in mm).

    fit_peaked(dev, groups=8, steps=300, precision='fp32') -> (net [eval mode], task dict)
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

SCALE = 2.0           # 400-px crops (H36M-like person boxes), 6.25 image px per heatmap px
POSE_SIGMA = 120.0    # mm: every joint inside the crop
SIGMA = 2.0           # target Gaussian (heatmap px)
BLOB = 6.0            # rendered joint blob (crop px)


def make_task(groups, dev, seed=0, size=256, njoints=16):
    """Views, metadata and Gaussian targets of `groups` synthetic 4-view groups."""
    from multiviews.cameras import project_pose
    from posu import synthetic as syn
    from posu.pipeline import synthetic_meta
    meta, host = synthetic_meta(groups, dev, image_size=size, scale=SCALE, pose_sigma=POSE_SIGMA)
    noise = syn.group_views(4, range(groups), size, seed=500 + seed)
    hs = size // 4
    aff = host['affines'].reshape(4, groups, 2, 3)                    # heatmap px -> image px
    joints_hm = np.zeros((4, groups, njoints, 2))
    for v in range(4):
        for g in range(groups):
            img = project_pose(host['poses3d'][g], host['cams'][g * 4 + v])
            A = aff[v, g]
            joints_hm[v, g] = np.linalg.solve(A[:, :2], (img - A[:, 2]).T).T
    ys, xs = np.meshgrid(np.arange(hs), np.arange(hs), indexing='ij')
    t = np.exp(-((xs - joints_hm[..., 0, None, None]) ** 2 + (ys - joints_hm[..., 1, None, None]) ** 2)
               / (2 * SIGMA ** 2)).astype(np.float32)
    # the crops: 0.3 x N(0, 1) noise + one coloured Gaussian blob per joint at its projection
    # (crop px = 4 x heatmap px), a joint-specific colour from a fixed spread of directions
    rc = np.random.default_rng(12345)
    col = rc.standard_normal((njoints, 3))
    col = 2.5 * col / np.linalg.norm(col, axis=1, keepdims=True)
    yi, xi = np.meshgrid(np.arange(size), np.arange(size), indexing='ij')
    views = []
    for v in range(4):
        img = 0.3 * noise[v].numpy()
        for g in range(groups):
            for j in range(njoints):
                cx, cy = 4 * joints_hm[v, g, j]
                blob = np.exp(-((xi - cx) ** 2 + (yi - cy) ** 2) / (2 * BLOB ** 2))
                img[g] += col[j][:, None, None] * blob[None]
        views.append(torch.from_numpy(img.astype(np.float32)).to(dev))
    return {'views': views, 'meta': meta, 'host': host, 'target': torch.from_numpy(t).to(dev),
            'joints_hm': joints_hm, 'groups': groups}


def fit_peaked(dev, groups=8, steps=300, seed=0, lr=1e-3, log=None, precision='fp32'):
    """Fit R50@256 (synthetic init, calibrated BN statistics) to the task's targets; returns the
    network in eval mode and the task."""
    from core.loss import JointsMSELoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from models.pose_resnet import get_pose_net
    from posu import synthetic as syn
    torch.manual_seed(seed)
    cfg = syn.make_cfg(num_layers=50, image_size=256)
    net = get_pose_net(cfg, is_train=False, precision=precision)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=syn.calibrated_seed(50, 256),
                                                 bn_stats=syn.load_bn_stats(50, 256)))
    net = net.to(dev).train()
    model = get_multiview_pose_net(net, cfg)
    task = make_task(groups, dev, seed=seed)
    w = torch.ones(groups, 16, 1, device=dev)
    mse = JointsMSELoss(use_target_weight=True)
    opt = torch.optim.Adam(net.parameters(), lr=lr, fused=True)
    for it in range(steps):
        raw, _, _, _ = model(task['views'])
        loss = sum(mse(raw[v], task['target'][v], w) for v in range(4))
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        if log is not None and (it % 50 == 0 or it == steps - 1):
            log('step %d loss %.6f peak %.3f' % (it, float(loss.detach()),
                                                 float(torch.cat(raw).detach().amax(dim=(2, 3)).mean())))
    net.eval()
    return net, task


def parity(net, task, dev, precision, ref=None, autotune=False):
    """The benched chain on the task's views (eval-mode plan in `precision`: forward -> soft-argmax +
    crop affine -> fp64 DLT triangulation) against the CPU oracle chain on the same weights (fp32
    reference forward -> soft-argmax -> transform_back -> triangulate_poses).  autotune: the plan's
    tiles autotuned on these views first (as bench.py does), so the tiles the tuner picks -- the split
    dtype's two-K-group tile among them -- are the ones measured.  Returns (metrics dict, the oracle
    outputs for reuse)."""
    from oracle import geometry_ref as G
    from oracle import pose_resnet_ref as PR
    from posu import ops
    from posu.metrics import mpjpe_stats
    host, meta, groups = task['host'], task['meta'], task['groups']
    if ref is None:
        sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
        hm_ref, _, _ = PR.pose_resnet_forward(torch.cat([v.cpu() for v in task['views']]), sd, 50)
        sa = G.softargmax2d(hm_ref)
        img = G.transform_back(sa, host['centers'].reshape(-1, 2), host['scales'].reshape(-1, 2), [64, 64])
        joints = img.view(4, groups, -1, 2)
        p2d = joints.permute(1, 0, 2, 3).reshape(groups * 4, -1, 2).double().numpy()
        ref = {'hm': hm_ref, 'joints': joints, 'X': G.triangulate_poses(host['cams'], p2d)}
    saved = net.precision
    try:
        net.precision = precision
        with torch.no_grad():
            plan = net.plan(dev)
            if autotune:
                plan.autotune(plan.pack_input(task['views']), keep_features=False, reps=2)
            hm = plan.run(plan.pack_input(task['views']), keep_features=False)[0]
            coords = ops.softargmax2d(hm, beta=100.0, affine=meta.affines).view(4, groups, hm.shape[1], 2)
            X = ops.triangulate_dlt(meta.M, meta.intr, coords, None, undistort=True, view_major=True)
        torch.cuda.synchronize()
    finally:
        net.precision = saved
    hm_err = (hm.cpu() - ref['hm']).abs()
    jerr = (coords.cpu() - ref['joints']).norm(dim=-1)
    st = mpjpe_stats(X.cpu().numpy(), ref['X'])
    gt = mpjpe_stats(ref['X'], host['poses3d'])
    r6 = lambda v: float('%.6g' % float(v))  # noqa: E731
    peak = hm.amax(dim=(2, 3))
    return ({'precision': precision, 'autotuned': bool(autotune), 'heatmap_peak_mean': r6(peak.mean()), 'heatmap_peak_min': r6(peak.min()),
             'heatmap_abs_err': {'max': r6(hm_err.max()), 'mean': r6(hm_err.mean())},
             'joints_px_err': {'mean': r6(jerr.mean()), 'max': r6(jerr.max())},
             'mpjpe_vs_ref_mm': {'mean': r6(st['mean']), 'std': r6(st['std']), 'max': r6(st['max'])},
             'oracle_mpjpe_vs_gt_mm': r6(gt['mean'])}, ref)


if __name__ == '__main__':
    import time
    dev = torch.device('cuda', 0)
    t0 = time.time()
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    lr = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-3
    net, task = fit_peaked(dev, steps=steps, lr=lr, log=print)
    torch.cuda.synchronize()
    print('fitted in %.1f s' % (time.time() - t0))
    with torch.no_grad():
        plan = net.plan(dev)
        hm = plan.run(plan.pack_input(task['views']))[0]
    mx = hm.amax(dim=(2, 3))
    print('eval heatmap peak: mean %.3f min %.3f' % (float(mx.mean()), float(mx.min())))
    t1 = time.time()
    res, ref = parity(net, task, dev, 'fp32')
    print(res)
    for p, tune in (('fp16x3', False), ('fp16x3', True), ('fp16', False), ('bf16', False)):
        print(parity(net, task, dev, p, ref, autotune=tune)[0])
    print('parity in %.1f s' % (time.time() - t1))
