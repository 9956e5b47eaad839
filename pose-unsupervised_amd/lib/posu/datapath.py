"""Batch data-path kernels: Gaussian target heatmaps
(JointsDatasetCompatible.generate_heatmap, lib/dataset/joints_dataset_compatible.py
:215-253) for a whole batch in one launch, and the sum-normalised integral decode of
run/test/test_integral.py:63-70.  cuda tensors only.
"""
import torch

from ._native import call, ptr, stream_of, require_cuda


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
