"""Hot-path losses (reference lib/core/loss.py) on HIP kernels.

* JointsMSELoss (loss.py:64-86): weighted per-joint heatmap MSE, one fused
  reduction kernel + its backward.
* FundamentalLoss (loss.py:89-133): epipolar residual |x_j^T F_{s,i,j} x_i| over the
  V(V-1) ordered view pairs, one kernel for the whole batch (the reference issues
  B x 12 small matmuls from a Python loop) + its backward.  The fundamental matrices
  are read from ``<DATASET.ROOT>/testdata/fundamental_matrix.pkl`` like the reference
  ({(subject, i, j): 3x3}), or given directly as a dict.

The MI / InfoNCE / JSD discriminator losses of the reference are outside this build.
"""
import itertools
import os
import pickle

import numpy as np
import torch

from posu import ops


class JointsMSELoss(torch.nn.Module):
    def __init__(self, use_target_weight):
        super(JointsMSELoss, self).__init__()
        self.use_target_weight = use_target_weight

    def forward(self, output, target, target_weight):
        w = target_weight if self.use_target_weight else None
        return ops.joints_mse(output, target, w)


class FundamentalLoss:
    def __init__(self, cfg, fundamental_matrix_dict=None, device=None):
        self.use_target_weight = cfg.LOSS.USE_TARGET_WEIGHT_FUND
        if fundamental_matrix_dict is None:
            path = os.path.join(cfg.DATASET.ROOT, 'testdata', 'fundamental_matrix.pkl')
            with open(path, 'rb') as f:  # the user's own data file, as in the reference
                fundamental_matrix_dict = pickle.load(f)
        if device is None:
            if torch.distributed.is_available() and torch.distributed.is_initialized():
                device = torch.device('cuda', torch.distributed.get_rank() % max(torch.cuda.device_count(), 1))
            else:
                device = torch.device('cuda', torch.cuda.current_device())
        self.device = device
        self.fundamental_matrix_dict = fundamental_matrix_dict
        keys = list(fundamental_matrix_dict.keys())
        self.subjects = sorted({k[0] for k in keys})
        self.nviews = 1 + max(max(k[1], k[2]) for k in keys)
        self.pairs = list(itertools.permutations(range(self.nviews), 2))
        table = np.zeros((len(self.subjects), len(self.pairs), 3, 3), dtype=np.float32)
        self._missing = {}  # subject -> first (subject, i, j) key absent from the dict
        for si, s in enumerate(self.subjects):
            for pi, (i, j) in enumerate(self.pairs):
                if (s, i, j) in fundamental_matrix_dict:
                    table[si, pi] = np.asarray(fundamental_matrix_dict[(s, i, j)], dtype=np.float32)
                else:
                    self._missing.setdefault(s, (s, i, j))
        self.F = torch.from_numpy(table).to(device)
        self._subj_index = {s: i for i, s in enumerate(self.subjects)}

    def subject_indices(self, subjects):
        """Rows of the F table; a subject without an entry, or with a (subject, i, j) pair
        missing from the dict, raises KeyError like the reference's dict lookup
        (loss.py:127) -- never a silent zero matrix."""
        subjects = np.asarray(subjects).tolist()
        for s in subjects:
            if s in self._missing:
                raise KeyError(self._missing[s])
        idx = np.array([self._subj_index[s] for s in subjects], dtype=np.int32)
        return torch.from_numpy(idx).to(self.device)

    def __call__(self, joints_2d_list, target_weight, meta):
        """joints_2d_list: V x [K, J, 2] image px (cuda); target_weight: V x [K, J, 1]; meta: V dicts."""
        assert isinstance(joints_2d_list[0], torch.Tensor)
        batch_size = joints_2d_list[0].shape[0]
        subject = meta[0]['subject']
        subject = subject.numpy() if isinstance(subject, torch.Tensor) else np.asarray(subject)
        assert batch_size == len(subject)
        assert len(joints_2d_list) == self.nviews
        x = torch.stack(joints_2d_list, dim=0)
        w = None
        if self.use_target_weight:
            w = torch.stack([t.reshape(batch_size, -1) for t in target_weight], dim=0)
        return ops.epipolar_loss(x, w, self.F, self.subject_indices(subject))
