"""Multi-view wrapper (reference lib/models/multiview_pose_resnet.py).

``MultiViewPose.forward(list of V [N, 3, H, W])`` returns
``(single_views, multi_views, low_features, high_features)`` like the reference
(multiview_pose_resnet.py:69-84).  The V views run as ONE backbone pass over a V*N
batch and the outputs are split back per view: in eval mode BN is a per-channel affine,
so this equals V separate passes; in train mode every view is a separate BatchNorm
segment (own batch statistics, own running-stat update in view order), which equals
the reference's V backbone calls.  A single tensor input behaves like
``PoseResNet.forward``.

The cross-view ``Aggregation`` fusion (AGGRE: true, 12 dense HW x HW maps) is not on
this round's path: constructing it raises, rather than running a non-HIP fallback.
"""
import torch
import torch.nn as nn


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
    if CFG.NETWORK.AGGRE:
        raise NotImplementedError(
            'pose-unsupervised_amd: NETWORK.AGGRE (ChannelWiseFC aggregation) is not on this build\'s HIP path yet')
    return MultiViewPose(PoseResNet, None, CFG)
