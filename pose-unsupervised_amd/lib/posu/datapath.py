"""Batch data-path kernels: the crop of
JointsDatasetCompatible.__getitem__ (cv2.warpAffine INTER_LINEAR, optionally fused with
ToTensor + Normalize; lib/dataset/joints_dataset_compatible.py:161-172) for a whole batch in one
launch, Gaussian target heatmaps (JointsDatasetCompatible.generate_heatmap,
joints_dataset_compatible.py:215-253) in one launch, and the sum-normalised integral decode of
run/test/test_integral.py:63-70.  cuda tensors only.
"""
import numpy as np
import torch

from ._native import call, ptr, stream_of, require_cuda

# run/pose2d/train.py:322-323 (transforms.Normalize after ToTensor)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def crop_warp(images, trans, image_size, device, out='f32', mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """images: N uint8 [H, W, C] arrays (numpy or cuda tensors, sizes may differ); trans: [N, 2, 3]
    src -> dst affines (utils.transforms.get_affine_transform(center, scale, rot, image_size));
    image_size (w, h).  out='u8': cv2.warpAffine's uint8 [N, h, w, C]; out='f32': the network input
    ToTensor + Normalize would give, f32 [N, C, h, w]."""
    if out not in ('u8', 'f32'):
        raise ValueError("out must be 'u8' or 'f32'")
    n = len(images)
    dw, dh = int(image_size[0]), int(image_size[1])
    shapes = [tuple(im.shape) for im in images]
    if any(len(sh) != 3 for sh in shapes) or len({sh[2] for sh in shapes}) > 1:
        raise ValueError('images must be [H, W, C] with one channel count')
    c = shapes[0][2] if shapes else 3
    offs = np.cumsum([0] + [int(np.prod(sh)) for sh in shapes])
    flat = [im.reshape(-1) if torch.is_tensor(im) else torch.from_numpy(np.ascontiguousarray(im).reshape(-1))
            for im in images]
    if any(f.dtype != torch.uint8 for f in flat):
        raise TypeError('crop_warp expects uint8 images (cv2.imread)')
    src = torch.cat([f.to(device) for f in flat]) if flat else torch.empty(0, dtype=torch.uint8, device=device)
    off = torch.tensor(offs[:-1], dtype=torch.int64, device=device)
    hw = torch.tensor([[sh[0], sh[1]] for sh in shapes], dtype=torch.int32, device=device).reshape(-1)
    M = torch.as_tensor(np.asarray(trans, dtype=np.float64).reshape(n, 6), device=device).contiguous()
    require_cuda(src)
    if out == 'u8':
        res = torch.empty((n, dh, dw, c), dtype=torch.uint8, device=device)
        m = s = None
    else:
        res = torch.empty((n, c, dh, dw), dtype=torch.float32, device=device)
        m = torch.tensor(mean, dtype=torch.float32, device=device)
        s = torch.tensor(std, dtype=torch.float32, device=device)
        if m.numel() != c or s.numel() != c:
            raise ValueError('mean / std need one value per channel')
    call('posu_crop_warp', ptr(src), ptr(off), ptr(hw), c, ptr(M), n, dh, dw, 0 if out == 'u8' else 1, ptr(m), ptr(s),
         ptr(res), stream_of(device))
    return res


def crop_batch(images, centers, scales, rotations, image_size, device, out='f32'):
    """The crops of a batch as __getitem__ makes them: trans = get_affine_transform(center,
    scale, rotation, image_size) per sample (host, float64), then crop_warp."""
    from utils.transforms import get_affine_transform
    trans = np.stack([get_affine_transform(np.asarray(c, dtype=np.float64), np.asarray(s, dtype=np.float64), r,
                                           image_size) for c, s, r in zip(centers, scales, rotations)])
    return crop_warp(images, trans, image_size, device, out=out), trans


def generate_heatmaps(joints, joints_vis, image_size, heatmap_size, sigma=2, zero_weight=None):
    """joints [N, J, 2] (crop px), joints_vis [N, J] or [N, J, k] (column 0 used) ->
    (target [N, J, hm_h, hm_w] f32, target_weight [N, J, 1] f32).  zero_weight: optional
    [N] bool, samples whose weights are zeroed (H36M without pseudo labels)."""
    require_cuda(joints)
    j = joints.float().contiguous()
    v = joints_vis.to(device=j.device, dtype=torch.float32)
    if v.dim() == 3:
        v = v[..., 0]
    v = v.contiguous()
    n, nj, _ = j.shape
    hw, hh = int(heatmap_size[0]), int(heatmap_size[1])
    target = torch.empty((n, nj, hh, hw), dtype=torch.float32, device=j.device)
    weight = torch.empty((n, nj, 1), dtype=torch.float32, device=j.device)
    zw = None
    if zero_weight is not None:
        zw = torch.as_tensor(zero_weight, device=j.device).to(torch.uint8).contiguous()
    call('posu_gaussian_targets', ptr(j), ptr(v), n, nj, int(image_size[0]), int(image_size[1]), hw, hh,
         float(sigma), ptr(zw), ptr(target), ptr(weight), stream_of(j.device))
    return target, weight


def integral_preds(heatmaps):
    """[N, J, H, W] -> [N, J, 2] (x, y) sum-normalised integral coordinates."""
    require_cuda(heatmaps)
    h = heatmaps.float().contiguous()
    n, nj, hh, ww = h.shape
    out = torch.empty((n, nj, 2), dtype=torch.float32, device=h.device)
    call('posu_integral2d_fwd', ptr(h), n, nj, hh, ww, ptr(out), stream_of(h.device))
    return out
