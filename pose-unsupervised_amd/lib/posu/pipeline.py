"""The batched 4-view hot path as one device-resident step.

    views (V x [B, 3, S, S] NCHW f32, B groups of V cameras)
      -> PoseResNet forward over the V*B frames as one batch      (plan.PoseResNetPlan)
      -> soft-argmax + per-frame crop affine -> image px          (posu_softargmax2d_fwd)
      -> epipolar loss over the V(V-1) ordered view pairs         (posu_epipolar_loss_fwd)
      -> fp64 DLT triangulation of every (group, joint)           (posu_triangulate_dlt)

This is the composition of the reference's train step slice (function.py:299-310:
generate_integral_preds_2d_th -> transform_back_th -> FundamentalLoss) and its
evaluation tail (test_triangulate.py -> triangulate_poses), run per batch without any
host round trip.  Per-batch metadata (crop affines, camera tables, subject index,
F table) is uploaded once and stays resident in HBM.
"""
import numpy as np
import torch

from . import ops
from .synthetic import fundamental_dict


class MultiViewBatchMeta:
    """Device-resident per-batch metadata of B groups x V views."""

    def __init__(self, affines, M, intr, F, subj, weights=None, undistort=True):
        self.affines = affines      # [V*B, 2, 3] f32 (view-major frame order)
        self.M = M                  # [B, V, 3, 4] f64
        self.intr = intr            # [B, V, 9] f64
        self.F = F                  # [S, V(V-1), 3, 3] f32
        self.subj = subj            # [B] int32
        self.weights = weights      # [V, B, J] f32 or None
        self.undistort = undistort


class MultiViewPipeline:
    def __init__(self, model, nviews=4, chunks=None):
        self.model = model
        self.nviews = nviews
        self.chunks = chunks

    def step(self, views, meta):
        """One batch: returns (heatmaps [V*B, J, h, w], coords [V, B, J, 2], loss [], X [B, J, 3] f64)."""
        plan = self.model.plan(views[0].device)
        hm, _, _ = plan.run(plan.pack_input(views), chunks=self.chunks, keep_features=False)
        nb = views[0].shape[0]
        j = hm.shape[1]
        coords = ops.softargmax2d(hm, beta=100.0, affine=meta.affines).view(self.nviews, nb, j, 2)
        loss = ops.epipolar_loss(coords, meta.weights, meta.F, meta.subj)
        X = ops.triangulate_dlt(meta.M, meta.intr, coords, None, undistort=meta.undistort, view_major=True)
        return hm, coords, loss, X


def subset_meta(meta, host, groups):
    """The metadata of the listed groups of a batch (a rank's shard, posu.dist.shard_groups):
    device tables indexed on their group axis, host camera / pose lists likewise."""
    nv = meta.M.shape[1]
    nb = meta.M.shape[0]
    gi = torch.as_tensor(list(groups), dtype=torch.long, device=meta.M.device)
    fi = (torch.arange(nv, device=gi.device)[:, None] * nb + gi[None, :]).reshape(-1)   # view-major frames
    sub = MultiViewBatchMeta(
        affines=meta.affines[fi].contiguous(), M=meta.M[gi].contiguous(), intr=meta.intr[gi].contiguous(),
        F=meta.F, subj=meta.subj[gi].contiguous(),
        weights=None if meta.weights is None else meta.weights[:, gi].contiguous(), undistort=meta.undistort)
    g = list(groups)
    hs = dict(host)
    hs['cams'] = [c for k in g for c in host['cams'][k * nv:(k + 1) * nv]]
    hs['poses3d'] = host['poses3d'][g]
    hs['centers'] = host['centers'][:, g]
    hs['scales'] = host['scales'][:, g]
    hs['affines'] = host['affines'].reshape(nv, nb, 2, 3)[:, g].reshape(-1, 2, 3)
    hs['subjects'] = host['subjects'][g]
    return sub, hs


def synthetic_meta(ngroups, device, image_size=256, njoints=16, distortion=True, nviews=4, scale=5.0,
                   pose_sigma=400.0):
    """Crop affines / cameras / F table of a synthetic H36M-like batch (posu.synthetic): crops
    centred on each group's projected root joint, `scale` x 200 px wide."""
    from utils.transforms import batch_inverse_affines
    from multiviews.triangulate import camera_tables
    from . import synthetic as syn
    cams = syn.group_cameras(ngroups, distortion=distortion)
    poses = syn.synthetic_poses3d(ngroups, njoints, sigma=pose_sigma)
    from multiviews.cameras import project_pose
    centers = np.zeros((nviews, ngroups, 2))
    for g in range(ngroups):
        for v in range(nviews):
            centers[v, g] = project_pose(poses[g, :1], cams[g * nviews + v])[0]
    scales = np.full((nviews, ngroups, 2), float(scale))
    hm = image_size // 4
    aff = batch_inverse_affines(centers.reshape(-1, 2), scales.reshape(-1, 2), [hm, hm])
    M, intr = camera_tables(cams, nviews, no_distortion=not distortion)
    fd = fundamental_dict(distortion)
    subjects = sorted({k[0] for k in fd})
    pairs = [(i, j) for i in range(nviews) for j in range(nviews) if i != j]
    F = np.stack([np.stack([fd[(s, i, j)] for (i, j) in pairs]) for s in subjects]).astype(np.float32)
    sidx = np.array([subjects.index(int(s)) for s in syn.group_subjects(ngroups)], dtype=np.int32)
    meta = MultiViewBatchMeta(
        affines=torch.from_numpy(aff).to(device=device, dtype=torch.float32),
        M=torch.from_numpy(M).to(device), intr=torch.from_numpy(intr).to(device),
        F=torch.from_numpy(F).to(device), subj=torch.from_numpy(sidx).to(device),
        weights=torch.ones((nviews, ngroups, njoints), dtype=torch.float32, device=device),
        undistort=True)
    host = dict(cams=cams, poses3d=poses, centers=centers, scales=scales, affines=aff, F_dict=fd,
                subjects=syn.group_subjects(ngroups))
    return meta, host
