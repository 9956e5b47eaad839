"""Generate the golden fixtures in tests/golden/ by importing the REFERENCE
(/root/reference/lib) in this container.  Run once (not on the GPU box):

    python tests/golden/make_golden.py

What it imports and how (all in-process, nothing is copied into the repo):
  * models.pose_resnet (imports as-is) -- PoseResNet R18/R50/R152 heatmaps; also a
    train-mode calibration pass whose BN running statistics become
    pose-unsupervised_amd/data/synthetic_bn_r*_*.npz (momentum 1.0 = one batch's stats);
  * utils.transforms, core.inference, core.loss -- these import OpenCV, which is not
    installed; a stand-in module provides only cv2.getAffineTransform (the 6x6 linear
    solve OpenCV performs).  generate_integral_preds_2d_th calls Tensor.get_device(),
    which is -1 on CPU tensors: it is patched to return 'cpu' while generating.
    FundamentalLoss.__init__ needs torch.distributed + CUDA: the object is built with
    __new__ and given its fundamental-matrix dict directly;
  * one training step of the reference model (train mode, per-view calls, the reference's
    JointsMSELoss / soft-argmax / transform_back / FundamentalLoss, loss.backward()):
    tests/golden/train_step_r50_128.npz (gradients, losses, BN buffers after the step);
  * multiviews.cameras (imports as-is) -- projection of known 3-D points, used as the
    exact known-answer input of the triangulation tests (pymvg is not importable).
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_LIB = '/root/reference/lib'

def _load_synthetic():
    # loaded by file path: the build's lib/ must not shadow the reference's packages here
    import importlib.util
    path = os.path.join(REPO, 'pose-unsupervised_amd', 'lib', 'posu', 'synthetic.py')
    spec = importlib.util.spec_from_file_location('posu_synthetic', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


syn = _load_synthetic()  # deterministic inputs, no reference code


def _install_cv2_standin():
    m = types.ModuleType('cv2')

    def getAffineTransform(src, dst):
        a = np.zeros((6, 6))
        b = np.zeros(6)
        src = np.asarray(src, np.float64)
        dst = np.asarray(dst, np.float64)
        for i in range(3):
            a[2 * i, :3] = [src[i, 0], src[i, 1], 1]
            a[2 * i + 1, 3:] = [src[i, 0], src[i, 1], 1]
            b[2 * i:2 * i + 2] = dst[i]
        return np.linalg.solve(a, b).reshape(2, 3)

    m.getAffineTransform = getAffineTransform
    m.INTER_LINEAR = 1
    sys.modules['cv2'] = m


def _import_reference():
    _install_cv2_standin()
    for p in (REF_LIB, os.path.join(REF_LIB, 'core')):
        if p not in sys.path:
            sys.path.insert(0, p)
    import models.pose_resnet as ref_pr  # noqa
    import utils.transforms as ref_tf  # noqa
    import core.inference as ref_inf  # noqa
    import core.loss as ref_loss  # noqa
    import multiviews.cameras as ref_cam  # noqa
    return ref_pr, ref_tf, ref_inf, ref_loss, ref_cam


def _patched_get_device():
    orig = torch.Tensor.get_device

    def gd(self):
        return 'cpu' if not self.is_cuda else orig(self)
    return orig, gd


def pose_resnet_golden(ref_pr, num_layers, image_size, batch, seed):
    cfg = syn.make_cfg(num_layers=num_layers, image_size=image_size)
    block, layers = ref_pr.resnet_spec[num_layers]
    net = ref_pr.PoseResNet(block, layers, cfg)
    sd = syn.synthetic_state_dict(net.state_dict(), seed=seed)
    net.load_state_dict(sd)
    # calibration: one train-mode pass with momentum 1 sets running stats = batch stats
    for m in net.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = 1.0
    calib = torch.cat(syn.synthetic_views(1, 4, image_size, seed=777), 0)
    net.train()
    with torch.no_grad():
        net(calib)
    stats = {k: v.detach().numpy().copy() for k, v in net.state_dict().items()
             if k.endswith('running_mean') or k.endswith('running_var')}
    os.makedirs(syn.DATA_DIR, exist_ok=True)
    np.savez_compressed(syn.bn_stats_file(num_layers, image_size), **stats)
    net.eval()
    x = torch.cat(syn.synthetic_views(1, batch, image_size, seed=seed + 1), 0)
    with torch.no_grad():
        hm, x1, f = net(x)
    np.savez_compressed(os.path.join(HERE, 'pose_resnet_r%d_%d.npz' % (num_layers, image_size)),
                        seed=seed, input_seed=seed + 1, batch=batch, heatmaps=hm.numpy(),
                        x1_mean=x1.mean(dim=(0, 2, 3)).numpy(), x1_slice=x1[:, :8, :8, :8].numpy(),
                        f_mean=f.mean(dim=(0, 2, 3)).numpy(), f_slice=f[:, :8, :8, :8].numpy())
    print('pose_resnet r%d@%d: |hm| max %.3f' % (num_layers, image_size, hm.abs().max()))


def peaked_heatmaps(n, j, h, w, seed):
    r = np.random.default_rng(seed)
    hm = 0.02 * r.standard_normal((n, j, h, w)).astype(np.float32)
    ys, xs = np.mgrid[0:h, 0:w]
    for a in range(n):
        for b in range(j):
            cy, cx = r.uniform(2, h - 3), r.uniform(2, w - 3)
            hm[a, b] += np.exp(-((ys - cy) ** 2 + (xs - cx) ** 2) / (2 * 2.0 ** 2)).astype(np.float32)
    return hm


def decode_golden(ref_tf, ref_inf):
    n, j, h, w = 6, 16, 64, 64
    hm = peaked_heatmaps(n, j, h, w, seed=5)
    hm[0, 0] = -1.0 - np.abs(hm[0, 0])          # all-negative map -> coords zeroed
    hm[0, 1] = 0.0
    hm[0, 1, 10, 20] = hm[0, 1, 30, 5] = 2.0    # tie -> first index wins
    hm[0, 2] = 0.0
    hm[0, 2, 0, 63] = 1.0                       # border peak -> no post-process shift
    hm[0, 3] = 0.0
    hm[0, 3, 1, 1] = 1.0                        # px == 1 -> no shift (strict 1 < px)
    centers = np.random.default_rng(6).uniform(300, 700, size=(n, 2))
    scales = np.random.default_rng(7).uniform(3.5, 6.0, size=(n, 2))
    orig, gd = _patched_get_device()
    torch.Tensor.get_device = gd
    try:
        t = torch.from_numpy(hm)
        sa = ref_tf.generate_integral_preds_2d_th(t)
        meta = [{'center': torch.from_numpy(centers), 'scale': torch.from_numpy(scales)}]
        cfg = syn.make_cfg()
        tb = ref_tf.transform_back_th(cfg, [sa], meta)[0]
    finally:
        torch.Tensor.get_device = orig
    maxp, maxv = ref_inf.get_max_preds(hm.copy())
    cfg = syn.make_cfg(post_process=True)
    fp, fv = ref_inf.get_final_preds(cfg, hm.copy(), centers, scales)
    cfg.TEST.POST_PROCESS = False
    fp0, _ = ref_inf.get_final_preds(cfg, hm.copy(), centers, scales)
    affs = np.stack([ref_tf.get_affine_transform(c, s, 0, [w, h], inv=1) for c, s in zip(centers, scales)])
    np.savez_compressed(os.path.join(HERE, 'decode.npz'), heatmaps=hm, centers=centers, scales=scales,
                        softargmax=sa.numpy(), transform_back=tb.numpy(), max_preds=maxp, max_vals=maxv,
                        final_preds=fp, final_vals=fv, final_preds_nopost=fp0, inv_affines=affs)
    print('decode: softargmax range', sa.min().item(), sa.max().item())


def loss_golden(ref_loss):
    V, B, J = 4, 6, 16
    r = np.random.default_rng(11)
    F_dict = syn.fundamental_dict()
    joints = [torch.tensor(r.uniform(100, 900, size=(B, J, 2)).astype(np.float32), requires_grad=True)
              for _ in range(V)]
    weights = [torch.from_numpy((r.uniform(size=(B, J, 1)) > 0.2).astype(np.float32)) for _ in range(V)]
    subjects = np.array([9, 11, 11, 9, 9, 11])
    meta = [{'subject': torch.from_numpy(subjects)} for _ in range(V)]
    out = {}
    for utw in (True, False):
        fl = ref_loss.FundamentalLoss.__new__(ref_loss.FundamentalLoss)
        fl.use_target_weight = utw
        fl.fundamental_matrix_dict = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in F_dict.items()}
        for jt in joints:
            jt.grad = None
        loss = fl(joints, weights, meta)
        loss.backward()
        tag = 'w' if utw else 'nw'
        out['fund_loss_' + tag] = loss.detach().numpy()
        out['fund_grad_' + tag] = np.stack([jt.grad.numpy() for jt in joints])
    pred = torch.tensor(r.standard_normal((B, J, 32, 32)).astype(np.float32), requires_grad=True)
    gt = torch.from_numpy(r.standard_normal((B, J, 32, 32)).astype(np.float32))
    tw = torch.from_numpy(r.uniform(size=(B, J, 1)).astype(np.float32))
    for utw in (True, False):
        pred.grad = None
        crit = ref_loss.JointsMSELoss(use_target_weight=utw)
        loss = crit(pred, gt, tw)
        loss.backward()
        tag = 'w' if utw else 'nw'
        out['mse_loss_' + tag] = loss.detach().numpy()
        out['mse_grad_' + tag] = pred.grad.numpy()
    keys = sorted(F_dict)
    np.savez_compressed(os.path.join(HERE, 'losses.npz'), joints=np.stack([j.detach().numpy() for j in joints]),
                        weights=np.stack([w.numpy() for w in weights]), subjects=subjects,
                        F_keys=np.array(keys), F_vals=np.stack([F_dict[k] for k in keys]),
                        mse_pred=pred.detach().numpy(), mse_gt=gt.numpy(), mse_w=tw.numpy(), **out)
    print('losses:', {k: float(v) for k, v in out.items() if 'loss' in k})


def camera_golden(ref_cam):
    G = 6
    cams = syn.group_cameras(G, distortion=True)
    cams_nd = syn.group_cameras(G, distortion=False)
    poses = syn.synthetic_poses3d(G, seed=3)
    proj = np.zeros((G * 4, 16, 2))
    proj_nd = np.zeros((G * 4, 16, 2))
    for g in range(G):
        for v in range(4):
            proj[g * 4 + v] = ref_cam.project_pose(poses[g], cams[g * 4 + v])
            proj_nd[g * 4 + v] = ref_cam.project_pose(poses[g], cams_nd[g * 4 + v])
    cam0 = cams[0]
    xc = np.stack([ref_cam.world_to_camera_frame(poses[g], cam0['R'], cam0['T']) for g in range(G)])
    back = np.stack([ref_cam.camera_to_world_frame(xc[g], cam0['R'], cam0['T']) for g in range(G)])
    np.savez_compressed(os.path.join(HERE, 'cameras.npz'), poses3d=poses, proj=proj, proj_nodist=proj_nd,
                        cam_frame=xc, world_back=back)
    print('cameras: proj range', proj.min(), proj.max())


MPII_FLIP_PAIRS = [[0, 5], [1, 4], [2, 3], [10, 15], [11, 14], [12, 13]]


def flip_golden(ref_tf):
    """Flip test (function.py:566-583): reference flip_back (numpy form of flip_back_th,
    transforms.py:20-31), SHIFT_HEATMAP's one-column shift and the average."""
    r = np.random.default_rng(21)
    hm = r.standard_normal((3, 16, 12, 10)).astype(np.float32)
    hmf = r.standard_normal((3, 16, 12, 10)).astype(np.float32)
    back = ref_tf.flip_back(hmf.copy(), MPII_FLIP_PAIRS)
    shifted = back.copy()
    shifted[:, :, :, 1:] = shifted.copy()[:, :, :, 0:-1]
    avg = (hm + shifted) * 0.5
    # PCK accuracy of validate() (core/evaluate.py:42-73)
    import core.evaluate as ref_eval
    target = peaked_heatmaps(6, 16, 32, 32, seed=23)
    target[0, 0] = 0.0
    target[0, 0, 1, 20] = 1.0                      # peak on row 1 -> excluded (-1 distance)
    output = target + 0.3 * r.standard_normal(target.shape).astype(np.float32)
    acc, avg_acc, cnt, pred = ref_eval.accuracy(output.copy(), target.copy())
    np.savez_compressed(os.path.join(HERE, 'flip.npz'), hm=hm, hm_flipped=hmf, pairs=np.array(MPII_FLIP_PAIRS),
                        flip_back=back, avg_shift=avg, avg_noshift=(hm + back) * 0.5,
                        acc_output=output, acc_target=target, acc=acc, avg_acc=avg_acc, cnt=cnt, acc_pred=pred)
    print('flip: done; accuracy', avg_acc, cnt)


TRAIN_FUND_WEIGHT = 10.0
TRAIN_PARAMS_FULL = ['conv1.weight', 'bn1.weight', 'bn1.bias', 'layer1.0.conv1.weight', 'layer1.0.bn3.weight',
                     'layer4.2.bn3.bias', 'deconv_layers.4.weight', 'final_layer.weight', 'final_layer.bias']
TRAIN_BUFFERS = ['bn1.running_mean', 'bn1.running_var', 'bn1.num_batches_tracked', 'layer4.2.bn3.running_mean',
                 'layer4.2.bn3.running_var', 'deconv_layers.7.running_mean', 'deconv_layers.7.running_var']


def train_step_golden(ref_pr, ref_tf, ref_loss, num_layers=50, image_size=128, nviews=4, batch=2, seed=3):
    """One reference training step (core/function.py:154-366 without the optimizer):
    per-view train-mode backbone calls, JointsMSELoss(use_target_weight) per view, and
    FundamentalLoss on soft-argmax -> transform_back coordinates; loss.backward()."""
    cfg = syn.make_cfg(num_layers=num_layers, image_size=image_size)
    block, layers = ref_pr.resnet_spec[num_layers]
    net = ref_pr.PoseResNet(block, layers, cfg)
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=seed))
    net.train()
    views = syn.synthetic_views(nviews, batch, image_size, seed=seed + 1)
    hms = image_size // 4
    targets = peaked_heatmaps(nviews * batch, 16, hms, hms, seed=seed + 2).reshape(nviews, batch, 16, hms, hms)
    r = np.random.default_rng(seed + 3)
    tw = (r.uniform(size=(nviews, batch, 16, 1)) > 0.15).astype(np.float32)
    centers = r.uniform(400, 600, size=(nviews, batch, 2))
    scales = np.full((nviews, batch, 2), 5.0)
    subjects = np.array([9, 11][:batch] + [9] * max(0, batch - 2))
    meta = [{'center': torch.from_numpy(centers[v]), 'scale': torch.from_numpy(scales[v]),
             'subject': torch.from_numpy(subjects)} for v in range(nviews)]
    outs = [net(v)[0] for v in views]
    crit = ref_loss.JointsMSELoss(use_target_weight=True)
    mse = 0
    for v in range(nviews):
        mse = mse + crit(outs[v], torch.from_numpy(targets[v]), torch.from_numpy(tw[v]))
    orig, gd = _patched_get_device()
    torch.Tensor.get_device = gd
    try:
        joints = ref_tf.transform_back_th(cfg, [ref_tf.generate_integral_preds_2d_th(o) for o in outs], meta)
    finally:
        torch.Tensor.get_device = orig
    fl = ref_loss.FundamentalLoss.__new__(ref_loss.FundamentalLoss)
    fl.use_target_weight = True
    fl.fundamental_matrix_dict = {k: torch.from_numpy(np.asarray(v, np.float32))
                                  for k, v in syn.fundamental_dict().items()}
    fund = fl(joints, [torch.from_numpy(w) for w in tw], meta) * TRAIN_FUND_WEIGHT
    loss = mse + fund
    loss.backward()
    named = dict(net.named_parameters())
    sd = net.state_dict()
    out = dict(num_layers=num_layers, image_size=image_size, nviews=nviews, batch=batch, seed=seed,
               fund_weight=TRAIN_FUND_WEIGHT, targets=targets, target_weight=tw, centers=centers, scales=scales,
               subjects=subjects, loss_mse=mse.detach().numpy(), loss_fund=fund.detach().numpy(),
               heatmaps=torch.stack([o.detach() for o in outs]).numpy(),
               joints=torch.stack([j.detach() for j in joints]).numpy(),
               grad_names=np.array(list(named)),
               grad_norms=np.array([named[k].grad.norm().item() for k in named]))
    for k in TRAIN_PARAMS_FULL:
        out['grad__' + k] = named[k].grad.numpy()
    for k in TRAIN_BUFFERS:
        out['buf__' + k] = sd[k].numpy()
    np.savez_compressed(os.path.join(HERE, 'train_step_r%d_%d.npz' % (num_layers, image_size)), **out)
    print('train step r%d@%d: mse %.6g fund %.6g' % (num_layers, image_size, mse.item(), fund.item()))


ADAM_STEPS = 6


def adam_golden(ref_pr, ref_loss, num_layers=18, image_size=128, nviews=4, batch=2, init_seed=123):
    """Seeded reference optimisation trajectory: the reference's random init
    (pose_resnet.py:234-247: N(0, 0.001) weights, BN 1 / 0) drawn from numpy
    (posu.synthetic.reference_init_state_dict -- torch's CPU RNG kernels can draw different
    floats on another host CPU, the GPU box's), then ADAM_STEPS steps of
    torch.optim.Adam(lr=1e-3) on the per-view JointsMSELoss(use_target_weight) of fixed
    synthetic targets in the reference's train mode (per-view BN batch statistics,
    core/function.py:154-182, 365-367).  Also recorded: the sums of the tensors the
    reference's own get_pose_net(is_train=True) draws after torch.manual_seed(init_seed)
    here, which the build's get_pose_net must reproduce bit for bit on this host."""
    cfg = syn.make_cfg(num_layers=num_layers, image_size=image_size)
    torch.manual_seed(init_seed)
    seeded = ref_pr.get_pose_net(cfg, is_train=True)
    torch_init_sums = np.array([float(p.detach().double().sum()) for p in seeded.parameters()])
    net = ref_pr.get_pose_net(cfg, is_train=False)
    net.load_state_dict(syn.reference_init_state_dict(net.state_dict(), seed=init_seed))
    init_sums = np.array([float(p.detach().double().sum()) for p in net.parameters()])
    net.train()
    views = syn.synthetic_views(nviews, batch, image_size, seed=init_seed + 1)
    hms = image_size // 4
    targets = peaked_heatmaps(nviews * batch, 16, hms, hms, seed=init_seed + 2).reshape(nviews, batch, 16, hms, hms)
    tw = (np.random.default_rng(init_seed + 3).uniform(size=(nviews, batch, 16, 1)) > 0.15).astype(np.float32)
    def trajectory(model, dtype):
        model = model.to(dtype)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        crit = ref_loss.JointsMSELoss(use_target_weight=True)
        losses, norms = [], []
        for _ in range(ADAM_STEPS):
            outs = [model(v.to(dtype))[0] for v in views]
            loss = sum(crit(outs[v], torch.from_numpy(targets[v]).to(dtype), torch.from_numpy(tw[v]).to(dtype))
                       for v in range(nviews))
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.item())
            norms.append([float(p.detach().norm()) for p in model.parameters()])
        return losses, norms
    import copy
    net64 = copy.deepcopy(net)
    losses, norms = trajectory(net, torch.float32)
    # the same trajectory in fp64: the reference's own fp32 rounding moves an Adam
    # trajectory (sign-like first steps on near-zero gradients), measured against this
    losses64, norms64 = trajectory(net64, torch.float64)
    np.savez_compressed(os.path.join(HERE, 'adam_r%d_%d.npz' % (num_layers, image_size)),
                        num_layers=num_layers, image_size=image_size, nviews=nviews, batch=batch,
                        init_seed=init_seed, lr=1e-3, init_sums=init_sums, torch_init_sums=torch_init_sums,
                        targets=targets, target_weight=tw,
                        losses=np.array(losses), param_norms=np.array(norms),
                        losses_f64=np.array(losses64), param_norms_f64=np.array(norms64),
                        param_names=np.array([n for n, _ in net.named_parameters()]))
    print('adam r%d@%d: losses %s' % (num_layers, image_size, ['%.6f' % v for v in losses]))


def main():
    torch.manual_seed(0)
    torch.set_num_threads(8)
    ref_pr, ref_tf, ref_inf, ref_loss, ref_cam = _import_reference()
    if len(sys.argv) > 1 and sys.argv[1] == 'adam':  # only the Adam trajectory
        adam_golden(ref_pr, ref_loss)
        return
    pose_resnet_golden(ref_pr, 50, 256, batch=2, seed=0)
    pose_resnet_golden(ref_pr, 18, 128, batch=2, seed=1)
    pose_resnet_golden(ref_pr, 152, 384, batch=1, seed=2)
    decode_golden(ref_tf, ref_inf)
    loss_golden(ref_loss)
    camera_golden(ref_cam)
    train_step_golden(ref_pr, ref_tf, ref_loss)
    flip_golden(ref_tf)
    adam_golden(ref_pr, ref_loss)


if __name__ == '__main__':
    main()
