"""Multi-view wrapper (reference lib/models/multiview_pose_resnet.py).

``MultiViewPose.forward(list of V [N, 3, H, W])`` returns
``(single_views, multi_views, low_features, high_features)`` like the reference
(multiview_pose_resnet.py:69-84).  The V views run as ONE backbone pass over a V*N
batch and the outputs are split back per view: in eval mode BN is a per-channel affine,
so this equals V separate passes; in train mode every view is a separate BatchNorm
segment (own batch statistics, own running-stat update in view order), which equals
the reference's V backbone calls.  A single tensor input behaves like
``PoseResNet.forward``.

``Aggregation`` (AGGRE: true) keeps the reference's parameters -- V(V-1) = 12
``ChannelWiseFC`` [HW, HW] matrices in ``aggre`` (state_dict keys ``aggre.<i>.weight``)
-- and runs all of them as ONE block-matrix MFMA GEMM (posu.aggregate), differentiable.
"""
import torch
import torch.nn as nn

from posu import ops
from posu.aggregate import aggregate, channel_fc


class ChannelWiseFC(nn.Module):
    """multiview_pose_resnet.py:16-29: out[n, c] = in[n, c].flatten() @ weight."""

    def __init__(self, size, precision='fp32'):
        super(ChannelWiseFC, self).__init__()
        self.weight = nn.Parameter(torch.Tensor(size, size))
        self.weight.data.uniform_(0, 0.1)
        self.precision = precision

    def forward(self, input):
        """One MFMA rows GEMM ([N*C, HW] x [HW, HW]); inside Aggregation all twelve run as
        one block-matrix GEMM instead."""
        if not input.is_cuda:
            raise RuntimeError('ChannelWiseFC runs on the MI355X HIP path only: input must be a cuda tensor')
        return channel_fc(input, self.weight, ops.dtype_code(self.precision))


class Aggregation(nn.Module):
    """multiview_pose_resnet.py:32-58: warped_i = sum_{o != i} fc_(i,o)(x_o) / (V - 1)."""

    def __init__(self, cfg, weights=[0.4, 0.2, 0.2, 0.2], precision='fp32'):
        super(Aggregation, self).__init__()
        NUM_NETS = 12
        size = int(cfg.NETWORK.HEATMAP_SIZE[0])
        self.weights = weights
        self.precision = precision
        self.aggre = nn.ModuleList()
        for i in range(NUM_NETS):
            self.aggre.append(ChannelWiseFC(size * size, precision))

    def forward(self, inputs):
        for t in inputs:
            if not t.is_cuda:
                raise RuntimeError('Aggregation runs on the MI355X HIP path only: inputs must be cuda tensors')
        nviews = len(inputs)
        if nviews * (nviews - 1) != len(self.aggre):
            raise ValueError('Aggregation built for %d view pairs, got %d views' % (len(self.aggre), nviews))
        return aggregate(inputs, [fc.weight for fc in self.aggre], ops.dtype_code(self.precision))


class MultiViewPose(nn.Module):

    def __init__(self, PoseResNet, Aggre, CFG):
        super(MultiViewPose, self).__init__()
        self.config = CFG
        self.resnet = PoseResNet
        self.aggre_layer = Aggre

    def forward(self, views):
        if not isinstance(views, list):
            return self.resnet(views)
        nv, n = len(views), views[0].shape[0]
        if any(v.shape != views[0].shape for v in views):
            raise ValueError('all views must share one shape')
        hm, x1, f = self.resnet._run_views(views)
        single_views = list(torch.split(hm, n, dim=0))
        low_features = list(torch.split(x1, n, dim=0))
        high_features = list(torch.split(f, n, dim=0))
        assert len(single_views) == nv
        multi_views = []
        if self.config.NETWORK.AGGRE:
            multi_views = self.aggre_layer(single_views)
        return single_views, multi_views, low_features, high_features


def get_multiview_pose_net(PoseResNet, CFG):
    Aggre = Aggregation(CFG, precision=getattr(PoseResNet, 'precision', 'fp32')) if CFG.NETWORK.AGGRE else None
    return MultiViewPose(PoseResNet, Aggre, CFG)
