"""H36M camera model helpers (reference lib/multiviews/cameras.py).

Host-side numpy on per-camera metadata (these feed the triangulation kernel's
camera tables and build ground truth; they are not per-pixel work).
Camera dict: R 3x3, T 3x1 (camera centre in world mm), fx, fy, cx, cy, k 3x1, p 2x1.
"""
from __future__ import division

import numpy as np


def unfold_camera_param(camera, avg_f=True):
    R, T = camera['R'], camera['T']
    f = 0.5 * (camera['fx'] + camera['fy']) if avg_f else np.array([camera['fx'], camera['fy']])
    c = np.array([camera['cx'], camera['cy']])
    return R, T, f, c, camera['k'], camera['p']


def project_point_radial(x, R, T, f, c, k, p):
    """World points [N, 3] -> pixels [N, 2] with the H36M radial + tangential model
    (reference cameras.py:25-49): y = xcam[:2] / xcam[2];
    y_d = y * (1 + k1 r^2 + k2 r^4 + k3 r^6 + p0 y1 + p1 y0) + [p1, p0] r^2; px = f y_d + c."""
    xcam = R.dot(x.T - T)
    y = xcam[:2] / xcam[2]
    r2 = np.sum(y ** 2, axis=0)
    kk = np.asarray(k).reshape(-1)
    pp = np.asarray(p).reshape(-1)
    radial = 1 + (kk[0] * r2 + kk[1] * r2 ** 2 + kk[2] * r2 ** 3)
    tan = pp[0] * y[1] + pp[1] * y[0]
    y = y * np.tile(radial + tan, (2, 1)) + np.outer(np.array([pp[1], pp[0]]), r2)
    return ((f * y) + np.asarray(c, dtype=np.float64).reshape(2, 1)).T


def project_pose(x, camera):
    R, T, f, c, k, p = unfold_camera_param(camera)
    return project_point_radial(x, R, T, f, c, k, p)


def world_to_camera_frame(x, R, T):
    return R.dot(x.T - T).T


def camera_to_world_frame(x, R, T):
    return (R.T.dot(x.T) + T).T
