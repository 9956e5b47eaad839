"""PoseResNet ("SimpleBaselines") on MI355X HIP kernels.

Drop-in for the reference ``models.pose_resnet`` (lib/models/pose_resnet.py):
same class names, constructor signatures, sub-module names (so ``state_dict`` keys
such as ``conv1.weight``, ``layer1.0.bn2.running_var``, ``deconv_layers.3.weight``,
``final_layer.bias`` load unchanged), ``init_weights`` semantics and forward return
tuple ``(heatmaps, layer1_out, deconv_out)`` (pose_resnet.py:191-205).

The modules hold the parameters in the reference's NCHW fp32 layout; forward runs a
:class:`posu.plan.PoseResNetPlan` (NHWC, MFMA implicit-GEMM kernels, BN folded into
the conv epilogues) that is re-packed whenever a parameter or buffer changes.

Compute dtype: ``precision='fp32'`` (the default: exact-f32 MFMA, the reference's fp32
numerics -- heatmaps within 1e-3 of the reference, so an unchanged reference script gets
reference results), ``'bf16'`` (opt-in fast mode: bf16 operands / f32 accumulate,
~16x the fp32 MFMA rate; heatmaps deviate ~0.02 mean / 0.15 max from the fp32 path on
R50@256) or ``'fp16'`` (IEEE fp16 operands / f32 accumulate, the fp16
setting of BASELINE configs[4]).  Heatmaps are always returned as NCHW float32;
``layer1_out`` / ``deconv_out`` are returned as NCHW-shaped channels-last views of the
NHWC activations in the compute dtype (zero-copy; fp32 in the default mode, like the
reference's).

Training mode (``model.train()``) runs posu.train_plan: batch-statistics BN per view,
differentiable through five stage Functions whose backward is the HIP kernel chain;
parameter gradients land in ``.grad`` as usual, stage by stage (optimizers / DDP unchanged;
DDP's bucketed all-reduce overlaps the rest of the backward).  ``layer1_out`` and
``deconv_out`` are differentiable in training mode, as in the reference.
"""
import logging
import os

import torch
import torch.nn as nn

from posu import ops
from posu.plan import PoseResNetPlan
from posu.train_plan import TrainPlan, train_forward

BN_MOMENTUM = 0.1
logger = logging.getLogger(__name__)


def _bn(c):
    return nn.BatchNorm2d(c, momentum=BN_MOMENTUM)


class BasicBlock(nn.Module):
    """3x3 -> 3x3 residual block (reference pose_resnet.py:29-58)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super(BasicBlock, self).__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = _bn(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = _bn(planes)
        self.downsample = downsample
        self.stride = stride


class Bottleneck(nn.Module):
    """1x1 -> 3x3(stride) -> 1x1 residual block (reference pose_resnet.py:61-99)."""
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super(Bottleneck, self).__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = _bn(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = _bn(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = _bn(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


_DECONV_CFG = {4: (1, 0), 3: (1, 1), 2: (0, 0)}  # kernel -> (padding, output_padding)


class PoseResNet(nn.Module):

    def __init__(self, block, layers, cfg, precision='fp32', **kwargs):
        super(PoseResNet, self).__init__()
        extra = cfg.POSE_RESNET
        self.inplanes = 64
        self.deconv_with_bias = extra.DECONV_WITH_BIAS
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.deconv_layers = self._make_deconv_layer(
            extra.NUM_DECONV_LAYERS, extra.NUM_DECONV_FILTERS, extra.NUM_DECONV_KERNELS)
        k = extra.FINAL_CONV_KERNEL
        self.final_layer = nn.Conv2d(extra.NUM_DECONV_FILTERS[-1], cfg.NETWORK.NUM_JOINTS,
                                     kernel_size=k, stride=1, padding=1 if k == 3 else 0)
        self.precision = precision
        self._plan = None
        self._plan_key = None
        self._train_plan = None

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                _bn(planes * block.expansion))
        mods = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        mods += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def _make_deconv_layer(self, num_layers, num_filters, num_kernels):
        assert num_layers == len(num_filters), \
            'ERROR: num_deconv_layers is different len(num_deconv_filters)'
        assert num_layers == len(num_kernels), \
            'ERROR: num_deconv_layers is different len(num_deconv_filters)'
        mods = []
        for planes, kernel in zip(num_filters, num_kernels):
            padding, output_padding = _DECONV_CFG[kernel]
            mods += [nn.ConvTranspose2d(self.inplanes, planes, kernel_size=kernel, stride=2, padding=padding,
                                        output_padding=output_padding, bias=self.deconv_with_bias),
                     _bn(planes), nn.ReLU(inplace=True)]
            self.inplanes = planes
        return nn.Sequential(*mods)

    # ------------------------------------------------------------------ plan
    def _state_key(self, device):
        versions = tuple(t._version for t in self.parameters()) + tuple(t._version for t in self.buffers())
        return (str(device), ops.dtype_code(self.precision), versions,
                tuple(t.data_ptr() for t in self.parameters()))

    def plan(self, device=None):
        """The packed HIP plan for the current parameters (rebuilt when they change)."""
        device = device or self.conv1.weight.device
        key = self._state_key(device)
        if self._plan is None or self._plan_key != key:
            with torch.no_grad():
                self._plan = PoseResNetPlan(self, ops.dtype_code(self.precision))
            self._plan_key = key
        return self._plan

    def train_plan(self):
        """The training-mode launch sequence (posu.train_plan.TrainPlan); packs per step."""
        code = ops.dtype_code(self.precision)
        if code in (ops.F16, ops.F16X3):
            raise NotImplementedError('training in fp16 / fp16x3 needs loss scaling; use precision bf16 or fp32')
        if self._train_plan is None or self._train_plan.code != code:
            self._train_plan = TrainPlan(self, code)
        return self._train_plan

    def _run_views(self, views):
        for v in views:
            if not v.is_cuda:
                raise RuntimeError('PoseResNet runs on the MI355X HIP path only: input must be a cuda tensor')
            if v.dim() != 4 or v.shape[1] != 3:
                raise ValueError('expected [N, 3, H, W] input, got %s' % (tuple(v.shape),))
        if self.conv1.weight.device != views[0].device:
            raise RuntimeError('model parameters are on %s but input is on %s'
                               % (self.conv1.weight.device, views[0].device))
        if self.training:
            # batch-statistics BN per view (one segment per view), differentiable; the views
            # are packed straight into one NHWC batch (no torch.cat)
            return train_forward(self, self.train_plan(), list(views), len(views))
        plan = self.plan(views[0].device)
        hm, x1, f = plan.run(plan.pack_input(views))
        # the reference returns f32 features (pose_resnet.py:197-205): a 2-byte plan's layer1 /
        # deconv outputs are widened once here (the heatmaps are f32 already); NHWC ->
        # NCHW-shaped channels-last views
        if x1.dtype != torch.float32:
            x1, f = ops.widen(x1, plan.code), ops.widen(f, plan.code)
        return hm, x1.permute(0, 3, 1, 2), f.permute(0, 3, 1, 2)

    def forward(self, x):
        return self._run_views([x])

    def init_weights(self, pretrained=''):
        """Reference semantics (pose_resnet.py:207-247): load an ImageNet checkpoint
        (non-strict) and re-init the head, or N(0, 0.001) init everything."""
        if os.path.isfile(pretrained):
            state = torch.load(pretrained, map_location='cpu', weights_only=True)
            logger.info('=> loading pretrained model {}'.format(pretrained))
            self.load_state_dict(state, strict=False)
            heads = list(self.deconv_layers.modules()) + list(self.final_layer.modules())
        else:
            logger.info('=> init weights from normal distribution')
            heads = list(self.modules())
        for m in heads:
            if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
                nn.init.normal_(m.weight, std=0.001)
                if m.bias is not None and (isinstance(m, nn.ConvTranspose2d) or os.path.isfile(pretrained)):
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)


resnet_spec = {18: (BasicBlock, [2, 2, 2, 2]),
               34: (BasicBlock, [3, 4, 6, 3]),
               50: (Bottleneck, [3, 4, 6, 3]),
               101: (Bottleneck, [3, 4, 23, 3]),
               152: (Bottleneck, [3, 8, 36, 3])}


def get_pose_net(cfg, is_train, **kwargs):
    """Reference factory (pose_resnet.py:257-267); extra kwarg ``precision`` = 'fp32' (default,
    reference numerics) | 'fp16x3' (split fp16: reference-parity numerics on the fp16 MFMAs) |
    'bf16' | 'fp16' (opt-in fast modes)."""
    block_class, layers = resnet_spec[cfg.POSE_RESNET.NUM_LAYERS]
    model = PoseResNet(block_class, layers, cfg, **kwargs)
    if is_train:
        model.init_weights(cfg.NETWORK.PRETRAINED)
    return model
