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
    """Fraction of the entries != -1 below `thr`; -1 when every entry is -1 (evaluate.py:32-39)."""
    valid = dists != -1
    n = int(np.count_nonzero(valid))
    return np.count_nonzero(dists[valid] < thr) * 1.0 / n if n else -1


def _np(x):
    return x.detach().cpu().numpy() if hasattr(x, 'detach') else x


def accuracy(output, target, hm_type='gaussian', thr=0.5):
    """evaluate.py:42-73 (output / target: [N, J, h, w] numpy or cuda tensors) -> (acc [J+1],
    avg_acc, cnt, pred): both argmaxes from the HIP kernel, then every joint's PCK at once over the
    [J, N] distance table (acc[0] = the mean over the joints that have a valid target)."""
    if hm_type != 'gaussian':
        raise NotImplementedError("accuracy: hm_type 'gaussian' only (the reference defines pred for it alone)")
    pred, tgt = (_np(get_max_preds(t)[0]) for t in (output, target))
    norm = np.tile(np.array([output.shape[2], output.shape[3]], dtype=np.float64) / 10, (pred.shape[0], 1))
    dists = calc_dists(pred, tgt, norm)                      # [J, N], -1: target outside the map
    valid = dists != -1
    nval = valid.sum(axis=1)
    hits = np.logical_and(dists < thr, valid).sum(axis=1)
    per_joint = np.where(nval > 0, hits * 1.0 / np.maximum(nval, 1), -1.0)
    acc = np.concatenate([[0.0], per_joint])
    counted = per_joint[per_joint >= 0]
    cnt = len(counted)
    avg_acc = 0
    for a in counted:   # accumulated joint by joint, as the reference does
        avg_acc = avg_acc + a
    if cnt:
        avg_acc = avg_acc / cnt
        acc[0] = avg_acc
    return acc, avg_acc, cnt, pred
