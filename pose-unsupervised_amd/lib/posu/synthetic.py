"""Deterministic synthetic workloads (no datasets or checkpoints exist offline).

* ``synthetic_state_dict``: He-initialised PoseResNet weights keyed like the reference
  ``state_dict`` (per-tensor seeds from the key name, numpy PCG64: identical on every
  machine), BatchNorm affine terms random around (1, 0); running statistics come
  from a calibration file (one train-mode pass, written by tests/golden/make_golden.py)
  so that activations stay O(1) through 50-150 layers, or default to (0, 1).
* ``h36m_like_cameras`` / ``synthetic_poses3d`` / ``fundamental_table``: 4-camera
  H36M-like rigs (fx = fy = 1145, principal point (512, 515), H36M distortion values,
  cameras 5 m from the subject), 16-joint poses, analytic fundamental matrices.
* ``synthetic_views``: seeded N(0, 1) NCHW crops (the post-normalisation domain).
"""
import itertools
import os
import zlib
from types import SimpleNamespace

import numpy as np
import torch

DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), 'data')


def _ns(**kw):
    return SimpleNamespace(**kw)


def make_cfg(num_layers=50, image_size=256, num_joints=16, deconv_with_bias=False, use_target_weight_fund=True,
             post_process=True, data_root='', flip_test=False, shift_heatmap=False):
    """The config fields the hot path reads (reference lib/core/config.py defaults)."""
    hm = image_size // 4
    return _ns(
        POSE_RESNET=_ns(NUM_LAYERS=num_layers, DECONV_WITH_BIAS=deconv_with_bias, NUM_DECONV_LAYERS=3,
                        NUM_DECONV_FILTERS=[256, 256, 256], NUM_DECONV_KERNELS=[4, 4, 4], FINAL_CONV_KERNEL=1),
        NETWORK=_ns(NUM_JOINTS=num_joints, PRETRAINED='', AGGRE=False, IMAGE_SIZE=np.array([image_size] * 2),
                    HEATMAP_SIZE=np.array([hm, hm])),
        LOSS=_ns(USE_TARGET_WEIGHT=True, USE_TARGET_WEIGHT_FUND=use_target_weight_fund, USE_FUNDAMENTAL_LOSS=True,
                 FUNDAMENTAL_LOSS_WEIGHT=5.0, MSE_LOSS_WEIGHT=1.0),
        TEST=_ns(POST_PROCESS=post_process, FUSE_OUTPUT=False, FLIP_TEST=flip_test, SHIFT_HEATMAP=shift_heatmap),
        DATASET=_ns(ROOT=data_root, NO_DISTORTION=False),
        DEBUG=_ns(SAVE_ALL_PREDS=False),
        PSEUDO_LABEL=_ns(NUM_INLIERS=4, REPROJ_THRE=10, IF_RANSAC=True, USE_REPROJ=False),
        PRINT_FREQ=100,
    )


def _rng(name, seed):
    return np.random.default_rng((zlib.crc32(name.encode()) ^ (seed * 2654435761)) & 0xFFFFFFFF)


def bn_stats_file(num_layers, image_size):
    return os.path.join(DATA_DIR, 'synthetic_bn_r%d_%d.npz' % (num_layers, image_size))


def _is_residual_tail(name, template):
    parts = name.split('.')
    if len(parts) != 4 or not parts[0].startswith('layer') or not parts[2].startswith('bn'):
        return False
    nxt = '%s.%s.bn%d.weight' % (parts[0], parts[1], int(parts[2][2:]) + 1)
    return nxt not in template


def synthetic_state_dict(template, seed=0, bn_stats=None):
    """template: a state_dict (names + shapes) of the reference-shaped model."""
    out = {}
    for name, t in template.items():
        shape = tuple(t.shape)
        r = _rng(name, seed)
        if name.endswith('num_batches_tracked'):
            out[name] = torch.zeros((), dtype=torch.long)
            continue
        if name.endswith('running_mean'):
            v = np.zeros(shape, np.float32)
        elif name.endswith('running_var'):
            v = np.ones(shape, np.float32)
        elif len(shape) == 4:
            if name.startswith('deconv_layers'):
                fan_in = shape[0] * shape[2] * shape[3] / 4.0  # stride-2 deconv: 1/4 of the taps per output
            else:
                fan_in = shape[1] * shape[2] * shape[3]
            gain = 1.0 if name.startswith('final_layer') else 2.0
            v = (r.standard_normal(shape) * np.sqrt(gain / fan_in)).astype(np.float32)
        elif name.endswith('weight'):  # BN gamma
            if _is_residual_tail(name, template):
                # last BN of a residual branch: small gamma keeps every block close to the
                # identity, so the random network is well conditioned (perturbations do
                # not grow exponentially with depth, as they would not in a trained net)
                v = r.uniform(0.1, 0.3, size=shape).astype(np.float32)
            else:
                v = r.uniform(0.5, 1.5, size=shape).astype(np.float32)
        else:  # BN beta / conv bias
            v = (0.1 * r.standard_normal(shape)).astype(np.float32)
        out[name] = torch.from_numpy(v)
    if bn_stats is not None:
        for k, v in bn_stats.items():
            if k in out:
                out[k] = torch.from_numpy(np.asarray(v, dtype=np.float32).reshape(tuple(out[k].shape)))
    return out


def reference_init_state_dict(template, seed=0):
    """The reference's random init (get_pose_net(is_train=True) without a pretrained file,
    pose_resnet.py:234-247) drawn from numpy PCG64 instead of torch's global RNG, so the
    same tensors come out on every machine: conv / deconv weights N(0, 0.001), BN weight 1,
    bias 0, running stats (0, 1); the final conv's bias keeps PyTorch's default Conv2d
    init, U(-1/sqrt(fan_in), 1/sqrt(fan_in)), which that init leaves in place."""
    out = {}
    for name, t in template.items():
        shape = tuple(t.shape)
        r = _rng(name, seed)
        if name.endswith('num_batches_tracked'):
            out[name] = torch.zeros((), dtype=torch.long)
            continue
        if len(shape) == 4:
            v = r.normal(0.0, 0.001, size=shape)
        elif name.endswith('running_var') or (name.endswith('weight') and len(shape) == 1):
            v = np.ones(shape)
        elif name.startswith('final_layer') and name.endswith('bias'):
            fan_in = template[name[:-4] + 'weight'][0].numel()
            v = r.uniform(-1.0, 1.0, size=shape) / np.sqrt(fan_in)
        else:
            v = np.zeros(shape)
        out[name] = torch.from_numpy(v.astype(np.float32))
    return out


# the weight seed each committed BN calibration (data/synthetic_bn_r*_*.npz) was made with
# (tests/golden/make_golden.py: the pose_resnet goldens' seeds); other seeds with these running
# statistics give un-normalised activations
CALIBRATED_SEED = {(18, 128): 1, (50, 256): 0, (152, 384): 2}


def calibrated_seed(num_layers, image_size):
    return CALIBRATED_SEED.get((num_layers, image_size), 0)


def load_bn_stats(num_layers, image_size):
    path = bn_stats_file(num_layers, image_size)
    if not os.path.exists(path):
        return None
    with np.load(path) as z:
        return {k: z[k] for k in z.files}


def synthetic_views(nviews, batch, image_size, seed=0, device='cpu'):
    """V x [batch, 3, S, S] f32 N(0, 1) crops (seed 1000 * seed + view)."""
    views = []
    for v in range(nviews):
        r = np.random.default_rng(1000 * seed + v)
        views.append(torch.from_numpy(r.standard_normal((batch, 3, image_size, image_size)).astype(np.float32))
                     .to(device))
    return views


def group_views(nviews, groups, image_size, seed=0, device='cpu'):
    """V x [len(groups), 3, S, S] f32 N(0, 1) crops of the listed groups of a global batch:
    group g's V crops are drawn from its own generator (seed, g), so a rank that holds a shard
    of the groups (posu.dist.shard_groups) gets exactly those groups' crops of the batch that
    one process would see."""
    out = np.empty((nviews, len(groups), 3, image_size, image_size), dtype=np.float32)
    for k, g in enumerate(groups):
        r = np.random.default_rng([seed, int(g)])
        out[:, k] = r.standard_normal((nviews, 3, image_size, image_size), dtype=np.float32)
    return [torch.from_numpy(out[v]).to(device) for v in range(nviews)]


# ---------------------------------------------------------------- geometry
H36M_K = np.array([-0.207, 0.247, -0.003])
H36M_P = np.array([-0.0009, -0.0016])
YAWS = (0.3, 1.9, 3.5, 5.0)
SUBJECTS = (9, 11)


def _look_at(C, target):
    z = target - C
    z = z / np.linalg.norm(z)
    x = np.cross(z, np.array([0.0, 0.0, 1.0]))
    x = x / np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z], axis=0)


def h36m_like_cameras(subject=9, distortion=True):
    """4 camera dicts in the H36M layout (R 3x3, T 3x1 centre, fx/fy/cx/cy (1,), k (3,1), p (2,1))."""
    cams = []
    rs = np.random.default_rng(subject)
    for yaw in YAWS:
        dist = 5000.0 + rs.uniform(-300, 300)
        height = 1600.0 + rs.uniform(-200, 200)
        C = np.array([dist * np.cos(yaw), dist * np.sin(yaw), height])
        R = _look_at(C, np.array([0.0, 0.0, 900.0]))
        cams.append({
            'R': R, 'T': C.reshape(3, 1),
            'fx': np.array([1145.0]), 'fy': np.array([1145.0]),
            'cx': np.array([512.0]), 'cy': np.array([515.0]),
            'k': (H36M_K if distortion else np.zeros(3)).reshape(3, 1).copy(),
            'p': (H36M_P if distortion else np.zeros(2)).reshape(2, 1).copy(),
            'name': 'cam%d' % len(cams),
        })
    return cams


def synthetic_poses3d(ngroups, njoints=16, seed=0, sigma=400.0):
    r = np.random.default_rng(seed)
    root = np.array([0.0, 0.0, 900.0])
    return root + r.normal(0.0, sigma, size=(ngroups, njoints, 3))


def group_subjects(ngroups):
    return np.array([SUBJECTS[g % len(SUBJECTS)] for g in range(ngroups)], dtype=np.int64)


def group_cameras(ngroups, distortion=True):
    """Group-major list of G*4 camera dicts (subject rig alternates per group)."""
    rigs = {s: h36m_like_cameras(s, distortion) for s in SUBJECTS}
    out = []
    for s in group_subjects(ngroups):
        out.extend(rigs[int(s)])
    return out


def fundamental(cam_i, cam_j):
    """F with x_j^T F x_i = 0 (pinhole), normalised to F[2, 2] = 1."""
    def K(c):
        return np.array([[float(c['fx'][0]), 0, float(c['cx'][0])], [0, float(c['fy'][0]), float(c['cy'][0])],
                         [0, 0, 1.0]])
    Ri, Rj = cam_i['R'], cam_j['R']
    Ci, Cj = cam_i['T'].reshape(3), cam_j['T'].reshape(3)
    R = Rj @ Ri.T
    t = Rj @ (Ci - Cj)
    tx = np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])
    F = np.linalg.inv(K(cam_j)).T @ tx @ R @ np.linalg.inv(K(cam_i))
    return F / F[2, 2]


def fundamental_dict(distortion=True):
    """{(subject, i, j): 3x3} like the reference fundamental_matrix.pkl."""
    out = {}
    for s in SUBJECTS:
        cams = h36m_like_cameras(s, distortion)
        for i, j in itertools.permutations(range(4), 2):
            out[(s, i, j)] = fundamental(cams[i], cams[j]).astype(np.float32)
    return out
