"""The evaluation slice: flip test, PCK accuracy and the
validate() batch body (core/function.py:555-644) on the MI355X, against
reference-generated goldens (tests/golden/flip.npz) and the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import geometry_ref as G
from oracle import pose_resnet_ref as PR
from posu import ops, synthetic as syn
from posu._native import BF16, F32

pytestmark = pytest.mark.gpu


def _perm(pairs, j=16):
    from utils.transforms import flip_pair_order
    return flip_pair_order(j, [list(p) for p in pairs])


def test_flip_back_matches_reference_golden(cuda, golden):
    g = golden('flip.npz')
    hm, hmf = torch.from_numpy(g['hm']).to(cuda), torch.from_numpy(g['hm_flipped']).to(cuda)
    perm = _perm(g['pairs'])
    np.testing.assert_array_equal(ops.flip_back(hmf, perm).cpu().numpy(), g['flip_back'])
    np.testing.assert_array_equal(ops.flip_back(hmf, perm, hm=hm, shift=True).cpu().numpy(), g['avg_shift'])
    np.testing.assert_array_equal(ops.flip_back(hmf, perm, hm=hm, shift=False).cpu().numpy(), g['avg_noshift'])
    # in place over the plain heatmaps (the validate loop's output buffer)
    out = hm.clone()
    ops.flip_back(hmf, perm, hm=out, shift=True, out=out)
    np.testing.assert_array_equal(out.cpu().numpy(), g['avg_shift'])


def test_flip_back_th_drop_in(cuda, golden):
    from utils.transforms import flip_back_th
    g = golden('flip.npz')
    views = [torch.from_numpy(g['hm_flipped']).to(cuda) for _ in range(4)]
    for v in flip_back_th(views, g['pairs'].tolist()):
        np.testing.assert_array_equal(v.cpu().numpy(), g['flip_back'])


def test_accuracy_matches_reference_golden(cuda, golden):
    from core.evaluate import accuracy
    g = golden('flip.npz')
    acc, avg, cnt, pred = accuracy(g['acc_output'].copy(), g['acc_target'].copy())
    np.testing.assert_allclose(acc, g['acc'], rtol=0, atol=1e-12)
    assert cnt == int(g['cnt'])
    np.testing.assert_allclose(avg, g['avg_acc'], rtol=0, atol=1e-12)
    np.testing.assert_array_equal(pred, g['acc_pred'])
    # cuda tensors in: same answer
    acc2, _, _, _ = accuracy(torch.from_numpy(g['acc_output']).to(cuda), torch.from_numpy(g['acc_target']).to(cuda))
    np.testing.assert_allclose(acc2, g['acc'], rtol=0, atol=1e-12)


@pytest.mark.parametrize('code', [F32, BF16])
def test_hflip_input_pack_equals_packing_the_flipped_image(cuda, code):
    x = torch.randn(2, 3, 16, 12, generator=torch.Generator().manual_seed(3)).to(cuda)
    xf = torch.flip(x, dims=[3])
    torch.testing.assert_close(ops.pack_s2d_nchw(x, code, 16, hflip=True), ops.pack_s2d_nchw(xf, code, 16),
                               atol=0, rtol=0)
    torch.testing.assert_close(ops.pack_nchw_to_nhwc(x, code, 8, hflip=True), ops.pack_nchw_to_nhwc(xf, code, 8),
                               atol=0, rtol=0)


def test_validate_batch_with_flip_test_matches_oracle(cuda, golden):
    from core.function import validate_batch
    from core.loss import JointsMSELoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from models.pose_resnet import get_pose_net
    pairs = golden('flip.npz')['pairs'].tolist()
    size, n = 128, 2
    cfg = syn.make_cfg(num_layers=18, image_size=size, flip_test=True, shift_heatmap=True)
    net = get_pose_net(cfg, is_train=False, precision='fp32')
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=1, bn_stats=syn.load_bn_stats(18, 128)))
    net = net.to(cuda).eval()
    model = get_multiview_pose_net(net, cfg)
    views = [v.to(cuda) for v in syn.synthetic_views(4, n, size, seed=33)]
    r = np.random.default_rng(34)
    centers = r.uniform(400, 600, size=(4, n, 2))
    scales = np.full((4, n, 2), 5.0)
    meta = [{'center': torch.from_numpy(centers[v]), 'scale': torch.from_numpy(scales[v])} for v in range(4)]
    target = [torch.rand(n, 16, 32, 32) for _ in range(4)]
    weight = [torch.ones(n, 16, 1) for _ in range(4)]
    res = validate_batch(cfg, model, views, target, weight, meta, flip_pairs=pairs,
                         criterion=JointsMSELoss(use_target_weight=True))
    # oracle: plain + mirrored forward, reference flip-back / shift / average, per view
    sd = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    perm = _perm(pairs)
    for k in range(4):
        x = views[k].cpu()
        hm, _, _ = PR.pose_resnet_forward(x, sd, 18)
        hmf, _, _ = PR.pose_resnet_forward(torch.flip(x, dims=[3]), sd, 18)
        back = torch.flip(hmf, dims=[3])[:, perm]
        back[:, :, :, 1:] = back.clone()[:, :, :, :-1]
        ref = ((hm + back) * 0.5).numpy()
        got = res['heatmaps'][k::4]
        np.testing.assert_allclose(got, ref, atol=1e-3, rtol=0)
        # decode of the device heatmaps vs the oracle decode (isolates the argmax stage)
        p, mv = G.get_final_preds(got, centers[k], scales[k], post_process=True)
        np.testing.assert_allclose(res['preds'][k::4, :, :2], p, atol=1e-4, rtol=0)
        np.testing.assert_allclose(res['preds'][k::4, :, 2:], mv, atol=1e-6, rtol=0)
    assert res['loss'] is not None and np.isfinite(res['loss'])
    assert 0.0 <= res['acc'] <= 1.0


def test_validate_batch_aggre_loss_terms(cuda):
    """AGGRE validation loss (function.py:589-609): JointsMSE on the raw outputs + the
    consistent loss (plain mean MSE between raw and aggregated heatmaps of the H36M samples)
    + the pseudo-label MSE of the fused outputs x MSE_LOSS_WEIGHT, against the same sums
    taken with torch ops on CPU from the model's own raw / aggregated heatmaps."""
    from core.function import fuse_routing, validate_batch
    from core.loss import JointsMSELoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from models.pose_resnet import get_pose_net
    size, n = 64, 3
    cfg = syn.make_cfg(num_layers=18, image_size=size)
    cfg.NETWORK.AGGRE = True
    cfg.TEST.FUSE_OUTPUT = True
    cfg.LOSS.USE_CONSISTENT_LOSS = True
    cfg.LOSS.MSE_LOSS_WEIGHT = 0.7
    cfg.DATASET.PSEUDO_LABEL_PATH = 'pseudo.pkl'
    net = get_pose_net(cfg, is_train=False, precision='fp32')
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=2))
    net = net.to(cuda).eval()
    model = get_multiview_pose_net(net, cfg).to(cuda)
    views = [v.to(cuda) for v in syn.synthetic_views(4, n, size, seed=35)]
    meta = [{'center': torch.full((n, 2), 500.0, dtype=torch.float64), 'scale': torch.full((n, 2), 5.0,
             dtype=torch.float64), 'source': ['h36m', 'mpii', 'h36m']} for _ in range(4)]
    g = torch.Generator().manual_seed(36)
    target = [torch.rand(n, 16, 16, 16, generator=g) for _ in range(4)]
    weight = [(torch.rand(n, 16, 1, generator=g) > 0.2).float() for _ in range(4)]
    crit = {'mse_weights': JointsMSELoss(use_target_weight=True)}
    res = validate_batch(cfg, model, views, target, weight, meta, criterion_dict=crit)
    with torch.no_grad():
        raw, agg, _, _ = model(views)
        out = fuse_routing(raw, agg, True, meta)
    raw = [r.cpu() for r in raw]
    agg = [a.cpu() for a in agg]
    out = [o.cpu() for o in out]
    ref = sum(G.joints_mse(r, t, w) for r, t, w in zip(raw, target, weight))
    sel = torch.tensor([True, False, True])
    ref = ref + torch.nn.functional.mse_loss(torch.cat([r[sel] for r in raw]), torch.cat([a[sel] for a in agg]))
    ref = ref + sum(G.joints_mse(o, t, w) for o, t, w in zip(out, target, weight)) * 0.7
    np.testing.assert_allclose(res['loss'], float(ref), rtol=1e-5)


class _FakeH5:
    """Stands in for h5py (absent from this image): records what validate() writes."""

    def __init__(self):
        self.files = {}

    def File(self, name, mode):   # noqa: N802 -- h5py's name
        rec = self.files.setdefault(name, {'mode': mode})

        class _F(dict):
            def __enter__(self):
                return self

            def __exit__(self, *a):
                rec.update(self)
                return False

            def close(self):
                rec.update(self)
        return _F()


class _FakeDataset:
    subset, dataset_type = 'validation', 'multiview_h36m'
    flip_pairs = [[0, 5], [1, 4], [2, 3], [10, 15], [11, 14], [12, 13]]

    def __init__(self, ngroups):
        self.n = ngroups
        # union-joint index -> dataset joint name ('*' = not annotated): 14 of 16 kept, out of order
        names = ['j%d' % k for k in range(16)]
        names[6] = names[9] = '*'
        self.u2a_mapping = {k: names[k] for k in (3, 0, 1, 2, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 14)}
        self.evaluated = None

    def __len__(self):
        return self.n

    def evaluate(self, preds, output_dir):
        self.evaluated = preds.copy()
        return {'mpjpe': 1.0}, 0.5


@pytest.mark.parametrize('flip', [False, True])
def test_validate_end_to_end_writes_the_reference_arrays(cuda, monkeypatch, tmp_path, flip):
    """validate() over a two-batch loader (core/function.py:155-188, reference function.py:529-690):
    the arrays handed to the h5 writer are the reference's -- heatmaps[:, u], locations[:, u]
    (get_final_preds + maxvals, views interleaved view-minor per batch), joint_names_order = u
    (the sorted annotated union joints) -- and dataset.evaluate gets all_preds[:, u]."""
    import sys
    from core import function as fn
    from core.loss import JointsMSELoss
    from models.multiview_pose_resnet import get_multiview_pose_net
    from models.pose_resnet import get_pose_net
    fake = _FakeH5()
    monkeypatch.setitem(sys.modules, 'h5py', fake)
    cfg = syn.make_cfg(num_layers=18, image_size=64, flip_test=flip, shift_heatmap=flip)
    net = get_pose_net(cfg, is_train=False, precision='fp32')
    net.load_state_dict(syn.synthetic_state_dict(net.state_dict(), seed=4))
    model = get_multiview_pose_net(net.to(cuda), cfg)
    ds = _FakeDataset(ngroups=5)
    rng = np.random.default_rng(0)
    loader = []
    for nb in (3, 2):
        views = [torch.from_numpy(rng.standard_normal((nb, 3, 64, 64)).astype(np.float32)) for _ in range(4)]
        target = [torch.from_numpy(rng.random((nb, 16, 16, 16)).astype(np.float32)) for _ in range(4)]
        weight = [torch.ones(nb, 16, 1) for _ in range(4)]
        meta = [{'center': torch.from_numpy(rng.uniform(100, 900, (nb, 2))),
                 'scale': torch.from_numpy(rng.uniform(1, 3, (nb, 2))), 'source': ['h36m'] * nb} for _ in range(4)]
        loader.append((views, target, weight, meta))
    perf = fn.validate(cfg, loader, ds, {'base_model': model}, {'mse_weights': JointsMSELoss(True)}, str(tmp_path),
                       None, 0)
    assert perf == 0.5
    (name, rec), = fake.files.items()
    assert name.endswith('heatmaps_locations_validation_multiview_h36m.h5') and rec['mode'] == 'w'
    u = np.array([0, 1, 2, 3, 4, 5, 7, 8, 10, 11, 12, 13, 14, 15])
    np.testing.assert_array_equal(rec['joint_names_order'], u)
    # expected: per batch, the views' heatmaps interleaved view-minor, decoded by the oracle
    exp_hm, exp_loc = [], []
    perm = torch.tensor(_perm(ds.flip_pairs), dtype=torch.int32, device=cuda)
    for views, _, _, meta in loader:
        nb = views[0].shape[0]
        with torch.no_grad():
            outs = [net(v.to(cuda))[0] for v in views]
            if flip:
                outf = [net(torch.flip(v, dims=[3]).to(cuda))[0] for v in views]
                outs = [ops.flip_back(f, perm, hm=o, shift=True) for o, f in zip(outs, outf)]
        hm = np.zeros((4 * nb, 16, 16, 16), np.float32)
        loc = np.zeros((4 * nb, 16, 3), np.float32)
        for k, (o, m) in enumerate(zip(outs, meta)):
            o = o.cpu().numpy()
            p, mv = G.get_final_preds(o, m['center'].numpy(), m['scale'].numpy())
            hm[k::4] = o
            loc[k::4, :, :2] = p
            loc[k::4, :, 2:] = mv
        exp_hm.append(hm)
        exp_loc.append(loc)
    exp_hm, exp_loc = np.concatenate(exp_hm), np.concatenate(exp_loc)
    assert rec['heatmaps'].shape == (20, 14, 16, 16) and rec['locations'].shape == (20, 14, 3)
    np.testing.assert_allclose(rec['heatmaps'], exp_hm[:, u], rtol=0, atol=1e-6)
    np.testing.assert_allclose(rec['locations'], exp_loc[:, u], rtol=0, atol=2e-3)
    np.testing.assert_array_equal(ds.evaluated, rec['locations'])
