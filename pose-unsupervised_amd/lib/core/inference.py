"""Argmax heatmap decoding (reference lib/core/inference.py) on the HIP argmax kernel.

``get_max_preds`` / ``get_final_preds`` keep the reference signatures and return
types: numpy in -> numpy out (the batch is staged to the current cuda device, decoded
there, and copied back), cuda tensor in -> cuda tensors out (no host round trip).
Semantics follow inference.py:19-75: first maximum wins, coordinates zeroed where the
maximum is <= 0, optional +-0.25 px shift toward the larger neighbour
(TEST.POST_PROCESS), then the inverse crop affine (float64 matrix, float32 result).
"""
import numpy as np
import torch

from posu import ops
from utils.transforms import batch_inverse_affines


def _to_device(batch_heatmaps):
    if isinstance(batch_heatmaps, torch.Tensor):
        return batch_heatmaps, False
    assert isinstance(batch_heatmaps, np.ndarray), 'batch_heatmaps should be numpy.ndarray'
    if not torch.cuda.is_available():
        raise RuntimeError('pose-unsupervised_amd decodes heatmaps on the GPU; no cuda device is visible')
    return torch.from_numpy(np.ascontiguousarray(batch_heatmaps, dtype=np.float32)).cuda(), True


def get_max_preds(batch_heatmaps):
    """[N, J, h, w] -> (coords [N, J, 2] f32, maxvals [N, J, 1] f32)."""
    hm, was_np = _to_device(batch_heatmaps)
    assert hm.dim() == 4, 'batch_images should be 4-ndim'
    preds, maxvals = ops.argmax2d(hm, post_process=False, affine64=None)
    if was_np:
        return preds.cpu().numpy(), maxvals.cpu().numpy()
    return preds, maxvals


def get_final_preds(config, batch_heatmaps, center, scale):
    """Argmax + post-process + transform back to image px (inference.py:50-75)."""
    hm, was_np = _to_device(batch_heatmaps)
    h, w = hm.shape[2], hm.shape[3]
    trans = batch_inverse_affines(np.asarray(center), np.asarray(scale), [w, h])
    T = torch.from_numpy(trans).to(device=hm.device, dtype=torch.float64)
    preds, maxvals = ops.argmax2d(hm, post_process=bool(config.TEST.POST_PROCESS), affine64=T)
    if was_np:
        return preds.cpu().numpy(), maxvals.cpu().numpy()
    return preds, maxvals
