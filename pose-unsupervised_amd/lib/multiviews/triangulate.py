"""Multi-view DLT triangulation (reference lib/multiviews/triangulate.py) on the HIP
fp64 triangulation kernel (libposeu.so posu_triangulate_dlt).

The reference builds a pymvg ``MultiCameraSystem`` per 4-view group and calls
``find3d`` per joint from a Python double loop (triangulate.py:57-99).  Here the
camera system is reduced to the two tables the arithmetic needs -- the projection
matrix M = K [R | -R T] (triangulate.py:29-36) and the intrinsics/distortion row
(fx, fy, cx, cy, k1, k2, p1, p2, k3) in pymvg's OpenCV order (triangulate.py:33) --
and every (group, joint) of a batch is solved in one launch.

pymvg is not vendored by the reference and is absent here; the kernel restates
its published algorithm (CameraModel.undistort: OpenCV fixed-point, 5 iterations,
skipped when all coefficients are zero; MultiCameraSystem.find3d: rows
x*M[2]-M[0], y*M[2]-M[1], smallest right singular vector).  See DESIGN.md for how
this is pinned.
"""
import numpy as np
import torch

from posu import ops
from multiviews.cameras import unfold_camera_param

NVIEWS = 4


def _scalar(v):
    return float(np.ravel(np.asarray(v, dtype=np.float64))[0])


def camera_table(camera, no_distortion=False):
    """(M [3, 4], intr [9]) float64 of one H36M camera dict."""
    R, T, f, c, k, p = unfold_camera_param(camera, avg_f=False)
    fx, fy = _scalar(f[0]), _scalar(f[1])
    cx, cy = _scalar(c[0]), _scalar(c[1])
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], dtype=float)
    R = np.asarray(R, dtype=float)
    t = -np.matmul(R, np.asarray(T, dtype=float).reshape(3, 1))
    M = K.dot(np.concatenate((R, t), axis=1))
    kk = np.ravel(np.asarray(k, dtype=float))
    pp = np.ravel(np.asarray(p, dtype=float))
    dist = np.zeros(5) if no_distortion else np.array([kk[0], kk[1], pp[0], pp[1], kk[2]])
    intr = np.array([fx, fy, cx, cy, dist[0], dist[1], dist[2], dist[3], dist[4]])
    return M, intr


class MultiCameraSystem:
    """Camera tables of one group (what build_multi_camera_system returns)."""

    def __init__(self, names, M, intr):
        self.names = list(names)
        self.M = M        # [V, 3, 4]
        self.intr = intr  # [V, 9]
        self._index = {n: i for i, n in enumerate(self.names)}

    def find3d(self, pts):
        """pts: list of (camera_name, xy) -> X [3] float64 (needs >= 2 views)."""
        v = len(self.names)
        xy = np.zeros((1, v, 1, 2))
        vis = np.zeros((1, v, 1), dtype=np.uint8)
        for name, p in pts:
            i = self._index[name]
            xy[0, i, 0] = np.ravel(p)[:2]
            vis[0, i, 0] = 1
        X = _solve(self.M[None], self.intr[None], xy, vis)
        return X[0, 0]

    def find2d(self, camera_name, xyz, distorted=True):
        """pymvg find2d: project a world point into one camera (OpenCV distortion of
        the camera row unless distorted=False) -> [2] float64.  Host arithmetic: a
        single point; the batched path is posu_reproject / posu_ransac_inliers."""
        i = self._index[camera_name]
        M, c = self.M[i], self.intr[i]
        X = np.append(np.ravel(np.asarray(xyz, dtype=np.float64))[:3], 1.0)
        P = M.dot(X)
        fx, fy, cx, cy = c[:4]
        k1, k2, p1, p2, k3 = c[4:] if distorted else (0.0,) * 5
        x = (P[0] - cx * P[2]) / fx / P[2]
        y = (P[1] - cy * P[2]) / fy / P[2]
        r2 = x * x + y * y
        radial = 1.0 + ((k3 * r2 + k2) * r2 + k1) * r2
        xd = x * radial + 2.0 * p1 * x * y + p2 * (r2 + 2.0 * x * x)
        yd = y * radial + p1 * (r2 + 2.0 * y * y) + 2.0 * p2 * x * y
        return np.array([fx * xd + cx, fy * yd + cy])


def build_multi_camera_system(cameras, no_distortion=False):
    """cameras: list of (name, camera dict) -> MultiCameraSystem (triangulate.py:17-40)."""
    tabs = [camera_table(cam, no_distortion) for _, cam in cameras]
    return MultiCameraSystem([n for n, _ in cameras], np.stack([t[0] for t in tabs]),
                             np.stack([t[1] for t in tabs]))


def triangulate_one_point(camera_system, points_2d_set):
    return camera_system.find3d(points_2d_set)


def camera_tables(camera_params, nviews=NVIEWS, no_distortion=False):
    """List of G*V camera dicts (group-major) -> M [G, V, 3, 4], intr [G, V, 9] float64."""
    tabs = [camera_table(c, no_distortion) for c in camera_params]
    g = len(camera_params) // nviews
    M = np.stack([t[0] for t in tabs])[:g * nviews].reshape(g, nviews, 3, 4)
    intr = np.stack([t[1] for t in tabs])[:g * nviews].reshape(g, nviews, 9)
    return M, intr


def _solve(M, intr, xy, vis, device=None):
    if not torch.cuda.is_available():
        raise RuntimeError('pose-unsupervised_amd triangulates on the GPU; no cuda device is visible')
    dev = device or torch.device('cuda', torch.cuda.current_device())
    X = ops.triangulate_dlt(torch.from_numpy(np.ascontiguousarray(M)).to(dev),
                            torch.from_numpy(np.ascontiguousarray(intr)).to(dev),
                            torch.from_numpy(np.ascontiguousarray(xy)).to(dev),
                            None if vis is None else torch.from_numpy(np.ascontiguousarray(vis)).to(dev),
                            undistort=True)
    return X.cpu().numpy()


def triangulate_poses(camera_params, poses2d, joints_vis=None, no_distortion=False):
    """camera_params: G*4 camera dicts; poses2d [G*4, J, 2] (group-major, view-minor);
    joints_vis [G*4, J] -> poses3d [G, J, 3] float64 (joints seen by < 2 views stay 0)."""
    njoints = poses2d.shape[1]
    ninstances = len(camera_params) // NVIEWS
    if joints_vis is not None:
        assert np.all(np.asarray(joints_vis).shape == tuple(poses2d.shape[:2]))
    M, intr = camera_tables(camera_params, NVIEWS, no_distortion)
    if isinstance(poses2d, torch.Tensor):
        dev = poses2d.device
        xy = poses2d[:ninstances * NVIEWS].reshape(ninstances, NVIEWS, njoints, 2)
        vis = None
        if joints_vis is not None:
            vis = torch.as_tensor(joints_vis, device=dev)[:ninstances * NVIEWS].reshape(
                ninstances, NVIEWS, njoints).ne(0).to(torch.uint8)
        return ops.triangulate_dlt(torch.from_numpy(M).to(dev), torch.from_numpy(intr).to(dev), xy, vis)
    poses2d = np.asarray(poses2d)
    xy = poses2d[:ninstances * NVIEWS].reshape(ninstances, NVIEWS, njoints, 2)
    if xy.dtype != np.float32:
        xy = xy.astype(np.float64)
    vis = None
    if joints_vis is not None:
        vis = (np.asarray(joints_vis)[:ninstances * NVIEWS] != 0).astype(np.uint8).reshape(
            ninstances, NVIEWS, njoints)
    return _solve(M, intr, xy, vis)


def _group_arrays(camera_params, poses2d, joints_vis, no_distortion):
    njoints = poses2d.shape[1]
    ninstances = len(camera_params) // NVIEWS
    assert np.all(np.asarray(joints_vis).shape == tuple(poses2d.shape[:2]))
    M, intr = camera_tables(camera_params, NVIEWS, no_distortion)
    if not torch.cuda.is_available():
        raise RuntimeError('pose-unsupervised_amd runs the pseudo-label geometry on the GPU; no cuda device is visible')
    dev = poses2d.device if isinstance(poses2d, torch.Tensor) else torch.device('cuda', torch.cuda.current_device())
    xy = torch.as_tensor(poses2d, dtype=torch.float64, device=dev)[:ninstances * NVIEWS].reshape(
        ninstances, NVIEWS, njoints, 2)
    vis = torch.as_tensor(joints_vis, device=dev)[:ninstances * NVIEWS].reshape(ninstances, NVIEWS, njoints).ne(0)
    return torch.from_numpy(M).to(dev), torch.from_numpy(intr).to(dev), xy, vis.to(torch.uint8), ninstances


def ransac(poses2d, camera_params, joints_vis, config):
    """Reference triangulate.py:102-165: per group and joint, the view pair whose
    triangulation re-projects within PSEUDO_LABEL.REPROJ_THRE in the most views (ties:
    smaller mean error; at least PSEUDO_LABEL.NUM_INLIERS) -> res_vis [N, J] (its inliers).
    One posu_ransac_inliers launch for the whole batch."""
    M, intr, xy, vis, ng = _group_arrays(camera_params, poses2d, joints_vis, config.DATASET.NO_DISTORTION)
    res = ops.ransac_inliers(M, intr, xy, vis, float(config.PSEUDO_LABEL.REPROJ_THRE),
                             int(config.PSEUDO_LABEL.NUM_INLIERS))
    out = np.zeros_like(np.asarray(joints_vis))
    out[:ng * NVIEWS] = res.reshape(ng * NVIEWS, -1).cpu().numpy().astype(out.dtype)
    return out


def reproject_poses(poses2d, camera_params, joints_vis, no_distortion=False):
    """Reference triangulate.py:168-213 -> (proj_2d [N, J, 2], res_vis [N, J])."""
    M, intr, xy, vis, ng = _group_arrays(camera_params, poses2d, joints_vis, no_distortion)
    proj, res = ops.reproject(M, intr, xy, vis)
    proj_2d = np.zeros(np.asarray(poses2d).shape, dtype=np.asarray(poses2d).dtype)
    res_vis = np.zeros_like(np.asarray(joints_vis))
    proj_2d[:ng * NVIEWS] = proj.reshape(ng * NVIEWS, -1, 2).cpu().numpy()
    res_vis[:ng * NVIEWS] = res.reshape(ng * NVIEWS, -1).cpu().numpy().astype(res_vis.dtype)
    return proj_2d, res_vis
