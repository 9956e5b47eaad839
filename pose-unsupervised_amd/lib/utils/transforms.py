"""Crop-affine geometry and heatmap decoding (reference lib/utils/transforms.py).

Host side (numpy, float64 like cv2): get_affine_transform / affine_transform /
transform_preds -- the per-sample crop matrices are tiny metadata.  The affine solve
is a restatement of cv2.getAffineTransform (the 6x6 linear system for the 2x3 matrix
mapping three point pairs), so OpenCV is not needed.

Device side (HIP kernels, libposeu.so): generate_integral_preds_2d_th (soft-argmax),
transform_back_th (per-sample affine), flip_back_th, plus the fused
integral_preds_image_th (soft-argmax + affine in one pass over the heatmaps).
"""
import numpy as np
import torch

from posu import ops


def get_dir(src_point, rot_rad):
    sn, cs = np.sin(rot_rad), np.cos(rot_rad)
    return [src_point[0] * cs - src_point[1] * sn, src_point[0] * sn + src_point[1] * cs]


def get_3rd_point(a, b):
    d = a - b
    return b + np.array([-d[1], d[0]], dtype=np.float32)


def affine_from_3_points(src, dst):
    """2x3 float64 matrix M with M @ [x, y, 1] = dst for the 3 (float32) point pairs
    (the system cv2.getAffineTransform solves)."""
    src = np.asarray(src, dtype=np.float32).astype(np.float64)
    dst = np.asarray(dst, dtype=np.float32).astype(np.float64)
    a = np.zeros((6, 6))
    b = np.zeros(6)
    for i in range(3):
        a[2 * i, 0:3] = (src[i, 0], src[i, 1], 1.0)
        a[2 * i + 1, 3:6] = (src[i, 0], src[i, 1], 1.0)
        b[2 * i], b[2 * i + 1] = dst[i, 0], dst[i, 1]
    return np.linalg.solve(a, b).reshape(2, 3)


def get_affine_transform(center, scale, rot, output_size, shift=np.array([0, 0], dtype=np.float32), inv=0):
    """Crop affine of reference transforms.py:76-109 (float64 2x3)."""
    if not isinstance(scale, np.ndarray) and not isinstance(scale, list):
        scale = np.array([scale, scale])
    scale_px = np.asarray(scale) * 200.0
    src_w = scale_px[0]
    dst_w, dst_h = output_size[0], output_size[1]
    rot_rad = np.pi * rot / 180
    src_dir = get_dir([0, src_w * -0.5], rot_rad)
    dst_dir = np.array([0, dst_w * -0.5], np.float32)
    src = np.zeros((3, 2), dtype=np.float32)
    dst = np.zeros((3, 2), dtype=np.float32)
    src[0, :] = center + scale_px * shift
    src[1, :] = center + src_dir + scale_px * shift
    dst[0, :] = [dst_w * 0.5, dst_h * 0.5]
    dst[1, :] = np.array([dst_w * 0.5, dst_h * 0.5]) + dst_dir
    src[2:, :] = get_3rd_point(src[0, :], src[1, :])
    dst[2:, :] = get_3rd_point(dst[0, :], dst[1, :])
    return affine_from_3_points(dst, src) if inv else affine_from_3_points(src, dst)


def affine_transform(pt, t):
    """pt [N, 2] or [2]; t [2, 3] -> homogeneous transform (float64)."""
    if pt.ndim == 1:
        pt = pt[np.newaxis, ...]
    pt = np.concatenate((pt, np.ones((pt.shape[0], 1))), axis=-1)
    return np.dot(pt, t.T).squeeze()


def transform_preds(coords, center, scale, output_size):
    target = np.zeros(coords.shape)
    trans = get_affine_transform(center, scale, 0, output_size, inv=1)
    target[:, :2] = affine_transform(coords[:, :2], trans)
    return target


def batch_inverse_affines(centers, scales, output_size):
    """[N, 2] centers / scales -> [N, 2, 3] float64 heatmap->image affines."""
    centers = np.asarray(centers)
    scales = np.asarray(scales)
    return np.stack([get_affine_transform(c, s, 0, output_size, inv=1) for c, s in zip(centers, scales)], axis=0)


# ------------------------------------------------------------------ device
def generate_integral_preds_2d_th(heatmaps):
    """Soft-argmax of reference transforms.py:149-171: [N, J, h, w] -> [N, J, 2] (x, y)."""
    return ops.softargmax2d(heatmaps, beta=100.0)


def integral_preds_image_th(heatmaps, affine):
    """Fused soft-argmax + crop affine: [N, J, h, w], [N, 2, 3] -> [N, J, 2] image px."""
    return ops.softargmax2d(heatmaps, beta=100.0, affine=affine)


def _meta_np(v):
    return v.numpy() if isinstance(v, torch.Tensor) else np.asarray(v)


def transform_back_th(cfg, joints_2d_list, meta):
    """Reference transforms.py:174-198: per view, heatmap px -> image px with the
    per-sample inverse crop affine (matrices built on the host, applied on device)."""
    out = []
    size = [cfg.NETWORK.HEATMAP_SIZE[0], cfg.NETWORK.HEATMAP_SIZE[1]]
    for p, m in zip(joints_2d_list, meta):
        trans = batch_inverse_affines(_meta_np(m['center']), _meta_np(m['scale']), size)
        T = torch.from_numpy(trans).to(device=p.device, dtype=torch.float32)
        res = ops.affine2d(p, T)
        assert len(res) == p.shape[0]
        out.append(res)
    return out


def flip_pair_order(num_joints, matched_parts):
    """perm[j] = joint whose flipped heatmap becomes joint j (transforms.py:40-44)."""
    order = list(range(num_joints))
    for a, b in matched_parts:
        order[a] = b
        order[b] = a
    return order


def flip_back_th(output_flipped, matched_parts):
    """Reference transforms.py:33-47 (flip test): mirror columns and swap L/R joints,
    one posu_flip_back launch per view."""
    assert len(output_flipped) == 4
    assert output_flipped[0].dim() == 4
    perm = torch.tensor(flip_pair_order(output_flipped[0].size(1), matched_parts), dtype=torch.int32,
                        device=output_flipped[0].device)
    return [ops.flip_back(v, perm) for v in output_flipped]
