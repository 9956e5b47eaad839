"""PCK-style heatmap accuracy (reference lib/core/evaluate.py), used by validate().

The argmax of output and target heatmaps runs on the HIP argmax kernel
(core.inference.get_max_preds); the per-joint distance / threshold arithmetic on the
[N, J] coordinates is the reference's, on the host, with the same return values:
(acc [J+1], avg_acc, cnt, pred).
"""
import numpy as np

from core.inference import get_max_preds


def calc_dists(preds, target, normalize):
    """evaluate.py:17-29: [J, N] normalised distances, -1 where the target is not
    inside the map (target x or y <= 1)."""
    preds = preds.astype(np.float32)
    target = target.astype(np.float32)
    valid = (target[:, :, 0] > 1) & (target[:, :, 1] > 1)
    d = np.linalg.norm(preds / normalize[:, None, :] - target / normalize[:, None, :], axis=2)
    return np.where(valid, d, -1.0).T


def dist_acc(dists, thr=0.5):
    """Fraction below `thr` ignoring -1 entries; -1 if there are none (evaluate.py:32-39)."""
    dist_cal = np.not_equal(dists, -1)
    num_dist_cal = dist_cal.sum()
    if num_dist_cal > 0:
        return np.less(dists[dist_cal], thr).sum() * 1.0 / num_dist_cal
    return -1


def _np(x):
    return x.detach().cpu().numpy() if hasattr(x, 'detach') else x


def accuracy(output, target, hm_type='gaussian', thr=0.5):
    """evaluate.py:42-73 (output / target: [N, J, h, w] numpy or cuda tensors)."""
    idx = list(range(output.shape[1]))
    norm = 1.0
    if hm_type == 'gaussian':
        pred, _ = get_max_preds(output)
        target, _ = get_max_preds(target)
        pred, target = _np(pred), _np(target)
        h = output.shape[2]
        w = output.shape[3]
        norm = np.ones((pred.shape[0], 2)) * np.array([h, w]) / 10
    dists = calc_dists(pred, target, norm)
    acc = np.zeros((len(idx) + 1))
    avg_acc = 0
    cnt = 0
    for i in range(len(idx)):
        acc[i + 1] = dist_acc(dists[idx[i]])
        if acc[i + 1] >= 0:
            avg_acc = avg_acc + acc[i + 1]
            cnt += 1
    if cnt != 0:
        avg_acc = avg_acc / cnt
        acc[0] = avg_acc
    return acc, avg_acc, cnt, pred
