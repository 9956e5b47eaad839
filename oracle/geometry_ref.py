"""CPU ORACLE (test infrastructure only): restatement of the reference's heatmap
decoding, losses, camera model and triangulation.

Sources (paths relative to the reference repo):
  softargmax2d        lib/utils/transforms.py:149-171 (torch-CPU fp32, same op order)
  crop affine         lib/utils/transforms.py:76-135 (+ cv2.getAffineTransform's 6x6 solve)
  transform_back      lib/utils/transforms.py:174-198
  get_max_preds       lib/core/inference.py:19-47
  get_final_preds     lib/core/inference.py:50-75, transforms.py:67-73, 112-120
  fundamental_loss    lib/core/loss.py:101-133
  joints_mse          lib/core/loss.py:70-86
  project_point_radial lib/multiviews/cameras.py:25-49
  warp_affine_linear  lib/dataset/joints_dataset_compatible.py:161-164 cv2.warpAffine(INTER_LINEAR,
                      BORDER_CONSTANT 0) as OpenCV 3.4 (requirements.txt: opencv-python
                      3.4.1.15) computes it: the affine inverted in double, coordinates in
                      1/1024-px fixed point (cvRound), 1/32-px bilinear weight table, 15-bit
                      fixed-point sum -- OpenCV is absent here: PARITY UNPINNED
  to_tensor_normalize torchvision ToTensor + Normalize (run/pose2d/train.py:151-158)
  triangulate_poses   lib/multiviews/triangulate.py:17-99 with pymvg's
                      CameraModel.undistort (OpenCV fixed point, 5 iterations) and
                      MultiCameraSystem.find3d (DLT rows, numpy SVD) restated
                      (pymvg is an unpinned, un-vendored dependency).
"""
import itertools
import math

import numpy as np
import torch


# ---------------------------------------------------------------- crop warp (data path)
def _cv_round(x):
    """cvRound on doubles: round half to even (lrint), as int64."""
    return np.rint(x).astype(np.int64)


def warp_affine_linear(src, M, dsize):
    """cv2.warpAffine(src, M, dsize, flags=INTER_LINEAR) for uint8 [H, W, C] (border 0).
    M: the 2x3 src -> dst matrix (get_affine_transform); dsize: (width, height)."""
    src = np.asarray(src, dtype=np.uint8)
    if src.ndim == 2:
        src = src[:, :, None]
    H, W, C = src.shape
    dw, dh = int(dsize[0]), int(dsize[1])
    m = np.asarray(M, dtype=np.float64).reshape(6).copy()
    D = m[0] * m[4] - m[1] * m[3]                     # cv::warpAffine: invert (no WARP_INVERSE_MAP)
    D = 1.0 / D if D != 0 else 0.0
    a11, a22 = m[4] * D, m[0] * D
    m[0], m[1], m[3], m[4] = a11, m[1] * -D, m[3] * -D, a22
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    AB_BITS, INTER_BITS, TAB = 10, 5, 32
    AB_SCALE = 1 << AB_BITS
    round_delta = AB_SCALE // TAB // 2
    xs = np.arange(dw, dtype=np.float64)
    ys = np.arange(dh, dtype=np.float64)
    adelta = _cv_round(m[0] * xs * AB_SCALE)
    bdelta = _cv_round(m[3] * xs * AB_SCALE)
    X0 = _cv_round((m[1] * ys + m[2]) * AB_SCALE) + round_delta
    Y0 = _cv_round((m[4] * ys + m[5]) * AB_SCALE) + round_delta
    X = (X0[:, None] + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx = np.clip(X >> INTER_BITS, -32768, 32767)
    sy = np.clip(Y >> INTER_BITS, -32768, 32767)
    fx, fy = X & (TAB - 1), Y & (TAB - 1)
    # the bilinear table entries: (1 - fy/32, fy/32) x (1 - fx/32, fx/32) x 32768, exact integers
    w = [(TAB - fy) * (TAB - fx) * 32, (TAB - fy) * fx * 32, fy * (TAB - fx) * 32, fy * fx * 32]
    out = np.zeros((dh, dw, C), dtype=np.uint8)
    outside = (sx >= W) | (sx + 1 < 0) | (sy >= H) | (sy + 1 < 0)   # whole pixel = the border value
    acc = np.zeros((dh, dw, C), dtype=np.int64)
    for k, (ox, oy) in enumerate(((0, 0), (1, 0), (0, 1), (1, 1))):
        tx, ty = sx + ox, sy + oy
        ok = (tx >= 0) & (tx < W) & (ty >= 0) & (ty < H)
        v = src[np.clip(ty, 0, H - 1), np.clip(tx, 0, W - 1)].astype(np.int64)
        acc += np.where(ok[..., None], v, 0) * w[k][..., None]
    val = (acc + (1 << 14)) >> 15
    out[:] = np.clip(val, 0, 255).astype(np.uint8)
    out[outside] = 0
    return out


def to_tensor_normalize(img_u8, mean, std):
    """torchvision ToTensor (HWC uint8 -> CHW float32 / 255) + Normalize ((x - mean) / std), f32."""
    x = np.asarray(img_u8).transpose(2, 0, 1).astype(np.float32) / np.float32(255)
    m = np.asarray(mean, dtype=np.float32)[:, None, None]
    s = np.asarray(std, dtype=np.float32)[:, None, None]
    return ((x - m) / s).astype(np.float32)


# ---------------------------------------------------------------- heatmaps
def softargmax2d(hm):
    """[N, J, h, w] f32 CPU tensor -> [N, J, 2] (x, y)."""
    n, j, h, w = hm.shape
    p = torch.softmax((hm * 100).view(n, j, -1), dim=-1).view(n, j, h, w)
    accu_w = p.sum(dim=2)
    accu_h = p.sum(dim=3)
    xs = torch.sum(accu_w * torch.arange(w, dtype=torch.float32).view(1, 1, -1), dim=2)
    ys = torch.sum(accu_h * torch.arange(h, dtype=torch.float32).view(1, 1, -1), dim=2)
    return torch.stack([xs, ys], dim=2)


def _solve_affine(src, dst):
    a = np.zeros((6, 6))
    b = np.zeros(6)
    src = np.asarray(src, np.float32).astype(np.float64)
    dst = np.asarray(dst, np.float32).astype(np.float64)
    for i in range(3):
        a[2 * i, :3] = [src[i, 0], src[i, 1], 1]
        a[2 * i + 1, 3:] = [src[i, 0], src[i, 1], 1]
        b[2 * i:2 * i + 2] = dst[i]
    return np.linalg.solve(a, b).reshape(2, 3)


def crop_affine(center, scale, output_size, inv=1):
    scale = np.asarray(scale, dtype=np.float64) * 200.0
    half = scale[0] * -0.5
    src = np.zeros((3, 2), np.float32)
    dst = np.zeros((3, 2), np.float32)
    src[0] = center
    src[1] = np.asarray(center) + np.array([0.0, half])  # rot = 0
    dst[0] = [output_size[0] * 0.5, output_size[1] * 0.5]
    dst[1] = np.array([output_size[0] * 0.5, output_size[1] * 0.5]) + np.array([0, output_size[0] * -0.5],
                                                                                 np.float32)
    for m in (src, dst):
        d = m[0] - m[1]
        m[2] = m[1] + np.array([-d[1], d[0]], np.float32)
    return _solve_affine(dst, src) if inv else _solve_affine(src, dst)


def transform_back(coords, centers, scales, hm_size):
    """coords [N, J, 2] f32 tensor (heatmap px) -> image px (fp32 matrices, like the reference)."""
    out = []
    for i in range(coords.shape[0]):
        T = torch.from_numpy(crop_affine(centers[i], scales[i], hm_size)).float()
        p = torch.cat([coords[i], torch.ones(coords.shape[1], 1)], dim=1)
        out.append(p @ T.t())
    return torch.stack(out, 0)


def get_max_preds(hm):
    n, j, h, w = hm.shape
    flat = hm.reshape(n, j, -1)
    idx = np.argmax(flat, 2).reshape(n, j, 1)
    maxvals = np.amax(flat, 2).reshape(n, j, 1)
    preds = np.tile(idx, (1, 1, 2)).astype(np.float32)
    preds[:, :, 0] = preds[:, :, 0] % w
    preds[:, :, 1] = np.floor(preds[:, :, 1] / w)
    preds *= np.tile(np.greater(maxvals, 0.0), (1, 1, 2)).astype(np.float32)
    return preds, maxvals


def get_final_preds(hm, centers, scales, post_process=True):
    coords, maxvals = get_max_preds(hm)
    h, w = hm.shape[2], hm.shape[3]
    if post_process:
        for n in range(coords.shape[0]):
            for p in range(coords.shape[1]):
                m = hm[n][p]
                px = int(math.floor(coords[n][p][0] + 0.5))
                py = int(math.floor(coords[n][p][1] + 0.5))
                if 1 < px < w - 1 and 1 < py < h - 1:
                    diff = np.array([m[py][px + 1] - m[py][px - 1], m[py + 1][px] - m[py - 1][px]])
                    coords[n][p] += np.sign(diff) * .25
    preds = coords.copy()
    for i in range(coords.shape[0]):
        T = crop_affine(centers[i], scales[i], [w, h])
        pt = np.concatenate((coords[i][:, :2], np.ones((coords.shape[1], 1))), axis=-1)
        preds[i][:, :2] = np.dot(pt, T.T)
    return preds, maxvals


# ------------------------------------------------------------------ losses
def fundamental_loss(joints, weights, subjects, F_dict, use_target_weight=True):
    """joints: V x [B, J, 2] f32 tensors; weights: V x [B, J, 1]; subjects [B]."""
    nv = len(joints)
    b, j = joints[0].shape[:2]
    homo = [torch.cat([p, torch.ones(b, j, 1)], dim=2) for p in joints]
    pairs = list(itertools.permutations(range(nv), 2))
    loss = 0
    for idx, s in enumerate(subjects):
        for (pi, pj) in pairs:
            Fm = torch.as_tensor(np.asarray(F_dict[(int(s), pi, pj)]), dtype=torch.float32)
            r = torch.abs(torch.sum(torch.mm(homo[pj][idx], Fm) * homo[pi][idx], dim=1))
            if use_target_weight:
                r = r * torch.squeeze(weights[pj][idx] * weights[pi][idx])
            loss = loss + r.sum()
    return loss / (b * len(pairs) * j)


def joints_mse(pred, gt, w=None):
    n, j = pred.shape[:2]
    hp = pred.reshape(n, j, -1)
    hg = gt.reshape(n, j, -1)
    loss = 0
    for k in range(j):
        a, c = hp[:, k], hg[:, k]
        if w is not None:
            a = a * w[:, k]
            c = c * w[:, k]
        loss = loss + torch.mean((a - c) ** 2)
    return loss


# ------------------------------------------------------------------ camera
def project_point_radial(x, R, T, f, c, k, p):
    xcam = R.dot(x.T - T)
    y = xcam[:2] / xcam[2]
    r2 = np.sum(y ** 2, axis=0)
    k = np.asarray(k).reshape(-1)
    p = np.asarray(p).reshape(-1)
    radial = 1 + (k[0] * r2 + k[1] * r2 ** 2 + k[2] * r2 ** 3)
    tan = p[0] * y[1] + p[1] * y[0]
    y = y * np.tile(radial + tan, (2, 1)) + np.outer(np.array([p[1], p[0]]), r2)
    return (f * y + np.asarray(c, np.float64).reshape(2, 1)).T


def project_pose(x, cam):
    f = 0.5 * (cam['fx'] + cam['fy'])
    return project_point_radial(x, cam['R'], cam['T'], f, np.array([cam['cx'], cam['cy']]), cam['k'], cam['p'])


# ------------------------------------------------------------- triangulate
def _camera(cam, no_distortion):
    f = [float(np.ravel(cam['fx'])[0]), float(np.ravel(cam['fy'])[0])]
    c = [float(np.ravel(cam['cx'])[0]), float(np.ravel(cam['cy'])[0])]
    K = np.array([[f[0], 0, c[0]], [0, f[1], c[1]], [0, 0, 1]], dtype=float)
    R = np.asarray(cam['R'], float)
    t = -np.matmul(R, np.asarray(cam['T'], float).reshape(3, 1))
    M = K.dot(np.concatenate((R, t), axis=1))
    k = np.ravel(cam['k'])
    p = np.ravel(cam['p'])
    D = np.zeros(5) if no_distortion else np.array([k[0], k[1], p[0], p[1], k[2]], float)
    return M, K, D


def undistort_point(xy, K, D):
    """pymvg CameraModel.undistort restated (OpenCV cvUndistortPoints fixed point)."""
    if np.sum(np.abs(D)) == 0.0:
        return np.asarray(xy, dtype=np.float64)
    fx, cx, fy, cy = K[0, 0], K[0, 2], K[1, 1], K[1, 2]
    xd = (xy[0] - cx) / fx
    yd = (xy[1] - cy) / fy
    k1, k2, t1, t2, k3 = D
    x, y = xd, yd
    for _ in range(5):
        r2 = x * x + y * y
        icdist = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
        dx = 2 * t1 * x * y + t2 * (r2 + 2 * x * x)
        dy = t1 * (r2 + 2 * y * y) + 2 * t2 * x * y
        x = (xd - dx) * icdist
        y = (yd - dy) * icdist
    return np.array([x * fx + cx, y * fy + cy])


def find3d(Ms, Ks, Ds, pts):
    A = []
    for M, K, D, xy in zip(Ms, Ks, Ds, pts):
        u, v = undistort_point(np.asarray(xy, dtype=np.float64), K, D)
        A.append(u * M[2] - M[0])
        A.append(v * M[2] - M[1])
    _, _, vt = np.linalg.svd(np.array(A))
    return vt[-1, :3] / vt[-1, 3]


def triangulate_poses(cameras, poses2d, joints_vis=None, no_distortion=False):
    nviews = 4
    nj = poses2d.shape[1]
    g = len(cameras) // nviews
    if joints_vis is None:
        joints_vis = np.ones(poses2d.shape[:2])
    out = np.zeros((g, nj, 3))
    for i in range(g):
        cams = [_camera(cameras[i * nviews + v], no_distortion) for v in range(nviews)]
        for k in range(nj):
            sel = [v for v in range(nviews) if joints_vis[i * nviews + v, k]]
            if len(sel) < 2:
                continue
            out[i, k] = find3d([cams[v][0] for v in sel], [cams[v][1] for v in sel], [cams[v][2] for v in sel],
                               [poses2d[i * nviews + v, k] for v in sel])
    return out


# ---------------------------------------------- pseudo-label RANSAC / reprojection
def find2d(M, K, D, X):
    """pymvg CameraModel.project_3d_to_pixel restated: [R|t] = K^-1 M, OpenCV plumb-bob
    distortion (k1, k2, p1, p2, k3) in normalised coordinates, back through K."""
    P = M.dot(np.append(np.asarray(X, np.float64)[:3], 1.0))
    Rt = np.linalg.solve(K, P)
    x, y = Rt[0] / Rt[2], Rt[1] / Rt[2]
    k1, k2, p1, p2, k3 = D
    r2 = x * x + y * y
    radial = 1 + k1 * r2 + k2 * r2 ** 2 + k3 * r2 ** 3
    xd = x * radial + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * radial + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.array([K[0, 0] * xd + K[0, 2], K[1, 1] * yd + K[1, 2]])


def ransac(poses2d, cameras, joints_vis, reproj_thre, num_inliers, no_distortion=False):
    """multiviews/triangulate.py:102-165 (ransac) with the pymvg calls restated."""
    import itertools
    nviews = 4
    nj = poses2d.shape[1]
    res_vis = np.zeros_like(joints_vis)
    for i in range(len(cameras) // nviews):
        cams = [_camera(cameras[i * nviews + v], no_distortion) for v in range(nviews)]
        for k in range(nj):
            pts = [(v, poses2d[i * nviews + v, k, :]) for v in range(nviews) if joints_vis[i * nviews + v, k]]
            if len(pts) < 2:
                continue
            best_inliers, best_error = [], 10000
            for pair in itertools.combinations(pts, 2):
                X = find3d([cams[v][0] for v, _ in pair], [cams[v][1] for v, _ in pair],
                           [cams[v][2] for v, _ in pair], [p for _, p in pair])
                in_thre, mean_error = [], 0
                for j in range(nviews):
                    err = np.linalg.norm(find2d(*cams[j], X) - poses2d[i * nviews + j, k, :])
                    if err < reproj_thre:
                        in_thre.append(j)
                        mean_error += err
                if len(in_thre) < num_inliers:
                    continue
                mean_error /= len(in_thre)
                if len(in_thre) > len(best_inliers) or (len(in_thre) == len(best_inliers) and mean_error < best_error):
                    best_inliers, best_error = in_thre, mean_error
            for v in best_inliers:
                res_vis[i * nviews + v, k] = 1
    return res_vis


def reproject_poses(poses2d, cameras, joints_vis, no_distortion=False):
    """multiviews/triangulate.py:168-213 with the pymvg calls restated."""
    nviews = 4
    proj = np.zeros_like(poses2d, dtype=np.float64)
    res_vis = np.zeros_like(joints_vis)
    for i in range(len(cameras) // nviews):
        cams = [_camera(cameras[i * nviews + v], no_distortion) for v in range(nviews)]
        for k in range(poses2d.shape[1]):
            sel = [v for v in range(nviews) if joints_vis[i * nviews + v, k]]
            if len(sel) < 2:
                continue
            X = find3d([cams[v][0] for v in sel], [cams[v][1] for v in sel], [cams[v][2] for v in sel],
                       [poses2d[i * nviews + v, k] for v in sel])
            for j in range(nviews):
                proj[i * nviews + j, k] = find2d(*cams[j], X)
                res_vis[i * nviews + j, k] = 1
    return proj, res_vis
