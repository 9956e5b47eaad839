"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import geometry_ref as G
from oracle import pose_resnet_ref as PR
from posu import synthetic as syn


def _model_inputs(golden, num_layers, size):
    g = golden('pose_resnet_r%d_%d.npz' % (num_layers, size))
    template = {k: v for k, v in _reference_shaped_state(num_layers, size).items()}
    sd = syn.synthetic_state_dict(template, seed=int(g['seed']), bn_stats=syn.load_bn_stats(num_layers, size))
    x = torch.cat(syn.synthetic_views(1, int(g['batch']), size, seed=int(g['input_seed'])), 0)
    return g, sd, x


def _reference_shaped_state(num_layers, size):
    # the build's module tree has the reference's state_dict keys and shapes
    from models.pose_resnet import get_pose_net
    return get_pose_net(syn.make_cfg(num_layers=num_layers, image_size=size), is_train=False).state_dict()


@pytest.mark.parametrize('num_layers,size', [(18, 128), (50, 256), (152, 384)])
def test_oracle_pose_resnet_matches_reference(golden, num_layers, size):
    torch.set_num_threads(8)
    g, sd, x = _model_inputs(golden, num_layers, size)
    hm, x1, f = PR.pose_resnet_forward(x, sd, num_layers)
    assert hm.shape == g['heatmaps'].shape
    np.testing.assert_allclose(hm.numpy(), g['heatmaps'], atol=2e-5, rtol=0)
    np.testing.assert_allclose(x1.mean(dim=(0, 2, 3)).numpy(), g['x1_mean'], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(x1[:, :8, :8, :8].numpy(), g['x1_slice'], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(f.mean(dim=(0, 2, 3)).numpy(), g['f_mean'], atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(f[:, :8, :8, :8].numpy(), g['f_slice'], atol=1e-5, rtol=1e-5)


def test_oracle_decode_matches_reference(golden):
    g = golden('decode.npz')
    hm = torch.from_numpy(g['heatmaps'])
    sa = G.softargmax2d(hm)
    np.testing.assert_allclose(sa.numpy(), g['softargmax'], atol=1e-5, rtol=0)
    tb = G.transform_back(sa, g['centers'], g['scales'], [64, 64])
    np.testing.assert_allclose(tb.numpy(), g['transform_back'], atol=1e-3, rtol=0)
    mp, mv = G.get_max_preds(g['heatmaps'].copy())
    np.testing.assert_array_equal(mp, g['max_preds'])
    np.testing.assert_array_equal(mv, g['max_vals'])
    fp, fv = G.get_final_preds(g['heatmaps'].copy(), g['centers'], g['scales'], post_process=True)
    np.testing.assert_allclose(fp, g['final_preds'], atol=1e-4, rtol=0)
    fp0, _ = G.get_final_preds(g['heatmaps'].copy(), g['centers'], g['scales'], post_process=False)
    np.testing.assert_allclose(fp0, g['final_preds_nopost'], atol=1e-4, rtol=0)
    for i in range(len(g['centers'])):
        np.testing.assert_allclose(G.crop_affine(g['centers'][i], g['scales'][i], [64, 64]), g['inv_affines'][i],
                                   rtol=1e-12, atol=1e-9)


def _F_dict(g):
    return {tuple(int(v) for v in k): f for k, f in zip(g['F_keys'], g['F_vals'])}


@pytest.mark.parametrize('tag,utw', [('w', True), ('nw', False)])
def test_oracle_losses_match_reference(golden, tag, utw):
    g = golden('losses.npz')
    joints = [torch.tensor(j, requires_grad=True) for j in g['joints']]
    weights = [torch.from_numpy(w) for w in g['weights']]
    loss = G.fundamental_loss(joints, weights, g['subjects'], _F_dict(g), use_target_weight=utw)
    loss.backward()
    np.testing.assert_allclose(loss.item(), g['fund_loss_' + tag], rtol=1e-5)
    np.testing.assert_allclose(np.stack([j.grad.numpy() for j in joints]), g['fund_grad_' + tag], rtol=1e-5,
                               atol=1e-9)
    pred = torch.tensor(g['mse_pred'], requires_grad=True)
    ml = G.joints_mse(pred, torch.from_numpy(g['mse_gt']), torch.from_numpy(g['mse_w']) if utw else None)
    ml.backward()
    np.testing.assert_allclose(ml.item(), g['mse_loss_' + tag], rtol=1e-5)
    np.testing.assert_allclose(pred.grad.numpy(), g['mse_grad_' + tag], rtol=1e-5, atol=1e-9)


def test_oracle_camera_projection_matches_reference(golden):
    g = golden('cameras.npz')
    G_ = g['poses3d'].shape[0]
    cams = syn.group_cameras(G_, distortion=True)
    cams_nd = syn.group_cameras(G_, distortion=False)
    for gi in range(G_):
        for v in range(4):
            np.testing.assert_allclose(G.project_pose(g['poses3d'][gi], cams[gi * 4 + v]), g['proj'][gi * 4 + v],
                                       rtol=1e-12, atol=1e-9)
            np.testing.assert_allclose(G.project_pose(g['poses3d'][gi], cams_nd[gi * 4 + v]),
                                       g['proj_nodist'][gi * 4 + v], rtol=1e-12, atol=1e-9)


def test_oracle_triangulation_known_answer(golden):
    """Noise-free pinhole projections (made by the reference's cameras.project_pose)
    triangulate back to the known 3-D joints."""
    g = golden('cameras.npz')
    G_ = g['poses3d'].shape[0]
    cams = syn.group_cameras(G_, distortion=False)
    X = G.triangulate_poses(cams, g['proj_nodist'], no_distortion=True)
    np.testing.assert_allclose(X, g['poses3d'], atol=1e-6, rtol=0)
    # joints visible in fewer than two views stay at the origin (triangulate.py:95-96)
    vis = np.ones((G_ * 4, 16))
    vis[0:4, 3] = 0
    vis[1:4, 5] = 0
    X2 = G.triangulate_poses(cams, g['proj_nodist'], joints_vis=vis, no_distortion=True)
    assert np.all(X2[0, 3] == 0) and np.all(X2[0, 5] == 0)
    np.testing.assert_allclose(np.delete(X2[0], [3, 5], axis=0), np.delete(g['poses3d'][0], [3, 5], axis=0),
                               atol=1e-6)


def test_oracle_undistort_inverts_opencv_model():
    """The restated pymvg undistortion inverts the OpenCV distortion model it targets."""
    K = np.array([[1145.0, 0, 512.0], [0, 1145.0, 515.0], [0, 0, 1]])
    D = np.array([-0.207, 0.247, -0.0009, -0.0016, -0.003])
    rng = np.random.default_rng(0)
    for _ in range(20):
        x, y = rng.uniform(-0.2, 0.2, size=2)
        r2 = x * x + y * y
        rad = 1 + D[0] * r2 + D[1] * r2 ** 2 + D[4] * r2 ** 3
        xd = x * rad + 2 * D[2] * x * y + D[3] * (r2 + 2 * x * x)
        yd = y * rad + D[2] * (r2 + 2 * y * y) + 2 * D[3] * x * y
        u = np.array([xd * K[0, 0] + K[0, 2], yd * K[1, 1] + K[1, 2]])
        und = G.undistort_point(u, K, D)
        np.testing.assert_allclose(und, [x * K[0, 0] + K[0, 2], y * K[1, 1] + K[1, 2]], atol=0.05)


def test_find2d_restatement_is_the_pinhole_projection_of_the_reference(golden):
    """No distortion: pymvg find2d (restated) == the reference's cameras.project_pose
    (fx == fy, so its average-focal model coincides) -- the known-answer pin; the
    distorted branch follows pymvg's OpenCV model (parity unpinned)."""
    g = golden('cameras.npz')
    cams = syn.group_cameras(g['poses3d'].shape[0], distortion=False)
    for gi in range(g['poses3d'].shape[0]):
        for v in range(4):
            M, K, D = G._camera(cams[gi * 4 + v], no_distortion=True)
            got = np.stack([G.find2d(M, K, D, X) for X in g['poses3d'][gi]])
            np.testing.assert_allclose(got, g['proj_nodist'][gi * 4 + v], rtol=1e-10, atol=1e-8)


def test_ransac_oracle_known_answers():
    """Noise-free views are all inliers; a view moved by 80 px is rejected; a joint seen
    by one view stays 0 (triangulate.py:134-136)."""
    ng = 3
    cams = syn.group_cameras(ng, distortion=False)
    poses = syn.synthetic_poses3d(ng)
    p2d = np.zeros((ng * 4, 16, 2))
    for gi in range(ng):
        for v in range(4):
            M, K, D = G._camera(cams[gi * 4 + v], no_distortion=True)
            p2d[gi * 4 + v] = [G.find2d(M, K, D, X) for X in poses[gi]]
    vis = np.ones((ng * 4, 16), dtype=np.int64)
    p2d[1 * 4 + 2, 5] += 80.0
    vis[2 * 4 + 1:2 * 4 + 4, 7] = 0
    res = G.ransac(p2d, cams, vis, reproj_thre=10, num_inliers=2, no_distortion=True)
    assert res.sum() == ng * 4 * 16 - 1 - 4
    assert res[1 * 4 + 2, 5] == 0 and res[1 * 4 + 0, 5] == 1
    assert res[2 * 4:2 * 4 + 4, 7].sum() == 0
    proj, rv = G.reproject_poses(p2d, cams, vis, no_distortion=True)
    np.testing.assert_allclose(proj[0], p2d[0], atol=1e-6)
    assert rv[2 * 4:2 * 4 + 4, 7].sum() == 0


def train_step_oracle(g, num_layers=None, size=None, sd=None, views=None):
    """The reference's training step (core/function.py:154-366, train mode, per-view BatchNorm)
    restated on the oracle: -> (params, buffers, heatmaps [V, B, J, h, w], joints [V, B, J, 2],
    mse, fund); the loss is back-propagated into params[k].grad.  sd / views (CPU): another
    network's state and crops than the golden's seeded ones."""
    nl = int(g['num_layers']) if num_layers is None else num_layers
    size = int(g['image_size']) if size is None else size
    nv, b, seed = int(g['nviews']), int(g['batch']), int(g['seed'])
    if sd is None:
        sd = syn.synthetic_state_dict(_reference_shaped_state(nl, size), seed=seed)
    params = {k: v.detach().float().clone().requires_grad_(True) for k, v in sd.items()
              if not ('running_' in k or 'num_batches' in k)}
    bufs = {k: v.clone() for k, v in sd.items() if 'running_' in k}
    if views is None:
        views = syn.synthetic_views(nv, b, size, seed=seed + 1)
    hms, joints, mse = [], [], 0
    for v in range(nv):
        hm, _, _ = PR.pose_resnet_train_forward(views[v], params, bufs, nl)
        hms.append(hm)
        mse = mse + G.joints_mse(hm, torch.from_numpy(g['targets'][v]), torch.from_numpy(g['target_weight'][v]))
        sa = G.softargmax2d(hm)
        joints.append(G.transform_back(sa, g['centers'][v], g['scales'][v], [size // 4] * 2))
    fund = G.fundamental_loss(joints, [torch.from_numpy(w) for w in g['target_weight']], g['subjects'],
                              syn.fundamental_dict()) * float(g['fund_weight'])
    (mse + fund).backward()
    return params, bufs, torch.stack(hms), torch.stack(joints), mse, fund


def test_oracle_train_step_matches_reference(golden):
    """The oracle's train-mode forward (pose_resnet_train_forward) + losses + autograd against the
    reference's own training step (tests/golden/train_step_r50_128.npz): heatmaps, joints, losses,
    every parameter gradient's norm, the full gradients held in the golden, running statistics."""
    torch.set_num_threads(8)
    g = golden('train_step_r50_128.npz')
    params, bufs, hm, joints, mse, fund = train_step_oracle(g)
    np.testing.assert_allclose(hm.detach().numpy(), g['heatmaps'], atol=1e-5, rtol=0)
    np.testing.assert_allclose(joints.detach().numpy(), g['joints'], atol=1e-3, rtol=0)
    np.testing.assert_allclose(mse.item(), g['loss_mse'], rtol=1e-5)
    np.testing.assert_allclose(fund.item(), g['loss_fund'], rtol=1e-5)
    norms = np.array([params[n].grad.norm().item() for n in g['grad_names']])
    np.testing.assert_allclose(norms, g['grad_norms'], rtol=1e-4)
    for k in g:
        if k.startswith('grad__'):
            np.testing.assert_allclose(params[k[6:]].grad.numpy(), g[k], atol=1e-4 * np.abs(g[k]).max(), rtol=1e-3,
                                       err_msg=k)
        if k.startswith('buf__') and 'num_batches' not in k:   # F.batch_norm keeps no counter
            np.testing.assert_allclose(bufs[k[5:]].numpy(), g[k], atol=1e-6, rtol=1e-5, err_msg=k)
