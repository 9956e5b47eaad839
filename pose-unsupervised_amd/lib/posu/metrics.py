"""MPJPE, as the reference's evaluation harness computes it (run/test/test_triangulate.py:84-102).

The harness maps both joint sets into one order (``u2a_mapping``: union index u ->
dataset index a, entries marked '*' dropped, sorted by u; test_triangulate.py:84-88),
selects ``pred3d[:, u]`` only when the 2-D inputs were the dataset's own (GT) joints
(:90-93, predictions read from the h5 file are already in union order) and
``gt3d[:, a]`` (:96), then reports the per-joint Euclidean error's mean, std, max and the
share of joints beyond mean + std (:98-102).

``mpjpe_stats`` is that arithmetic on host arrays (numpy, fp64); ``mpjpe_sums`` is the
device form used by the multi-rank evaluation: per-rank (error sum, squared-error sum,
count, max) that one small all-reduce combines (posu.dist.sum_over_ranks)."""
import numpy as np
import torch


def u2a_indices(u2a_mapping):
    """(u, a) index arrays of test_triangulate.py:84-88 from a dataset's u2a mapping
    ({union index: dataset index or '*'})."""
    items = sorted(((k, v) for k, v in u2a_mapping.items() if v != '*'), key=lambda kv: kv[0])
    return np.array([k for k, _ in items]), np.array([v for _, v in items])


def mpjpe_stats(pred3d, gt3d, u=None, a=None, pred_in_union_order=True):
    """pred3d [N, J, 3], gt3d [N, Jd, 3] (mm) -> dict(mean, std, max, frac_above_mean_std,
    per_joint [N, J]).  u / a: the u2a index arrays (None: identity, same joint order)."""
    pred3d = np.asarray(pred3d, dtype=np.float64)
    gt3d = np.asarray(gt3d, dtype=np.float64)
    assert len(pred3d) == len(gt3d)
    pred = pred3d if (u is None or pred_in_union_order) else pred3d[:, u, :]
    gt = gt3d if a is None else gt3d[:, a, :]
    norm = np.linalg.norm(pred - gt, axis=2)
    mean, std = float(np.mean(norm)), float(np.std(norm))
    return {'mean': mean, 'std': std, 'max': float(np.amax(norm)),
            'frac_above_mean_std': float(np.sum(norm > mean + std) / norm.size), 'per_joint': norm}


def mpjpe_sums(pred3d, gt3d):
    """Device tensors [N, J, 3] -> [sum |e|, sum |e|^2, count, max |e|] (f64) for a
    multi-rank mean / std / max (combine the sums with a SUM and the max with a MAX)."""
    e = torch.linalg.norm(pred3d.double() - gt3d.double(), dim=2)
    return torch.stack([e.sum(), (e * e).sum(), torch.tensor(float(e.numel()), dtype=torch.float64,
                                                             device=e.device), e.max()])


def stats_from_sums(s, sq, count, mx):
    mean = s / count
    return {'mean': mean, 'std': float(np.sqrt(max(sq / count - mean * mean, 0.0))), 'max': mx}
