"""CPU ORACLE (test infrastructure only): functional restatement of the reference
PoseResNet eval-mode forward in torch-CPU fp32.

Follows /root/reference lib/models/pose_resnet.py:
  stem conv 7x7/s2/p3 -> BN -> ReLU -> maxpool 3/s2/p1       (pose_resnet.py:109-113, 192-195)
  Bottleneck: 1x1 -> BN -> ReLU -> 3x3(stride)/p1 -> BN -> ReLU -> 1x1 -> BN
              (+ downsample 1x1(stride) -> BN) -> add -> ReLU  (pose_resnet.py:61-99, 134-149)
  BasicBlock: 3x3(stride) -> BN -> ReLU -> 3x3 -> BN (+ds) -> add -> ReLU (pose_resnet.py:29-58)
  3 x ConvTranspose2d(4, s2, p1, bias=DECONV_WITH_BIAS) -> BN -> ReLU (pose_resnet.py:164-189)
  final 1x1 conv + bias                                     (pose_resnet.py:126-132)
returning (heatmaps, layer1 output, deconv output)          (pose_resnet.py:191-205).
Parameters are read from a reference-keyed state_dict.
"""
import torch
import torch.nn.functional as F

BN_EPS = 1e-5
LAYERS = {18: ('basic', [2, 2, 2, 2]), 34: ('basic', [3, 4, 6, 3]), 50: ('bottleneck', [3, 4, 6, 3]),
          101: ('bottleneck', [3, 4, 23, 3]), 152: ('bottleneck', [3, 8, 36, 3])}


def _bn(x, sd, p):
    return F.batch_norm(x, sd[p + '.running_mean'], sd[p + '.running_var'], sd[p + '.weight'], sd[p + '.bias'],
                        training=False, eps=BN_EPS)


def _block(x, sd, p, kind, stride):
    if kind == 'bottleneck':
        out = F.relu(_bn(F.conv2d(x, sd[p + '.conv1.weight']), sd, p + '.bn1'))
        out = F.relu(_bn(F.conv2d(out, sd[p + '.conv2.weight'], stride=stride, padding=1), sd, p + '.bn2'))
        out = _bn(F.conv2d(out, sd[p + '.conv3.weight']), sd, p + '.bn3')
    else:
        out = F.relu(_bn(F.conv2d(x, sd[p + '.conv1.weight'], stride=stride, padding=1), sd, p + '.bn1'))
        out = _bn(F.conv2d(out, sd[p + '.conv2.weight'], padding=1), sd, p + '.bn2')
    if p + '.downsample.0.weight' in sd:
        res = _bn(F.conv2d(x, sd[p + '.downsample.0.weight'], stride=stride), sd, p + '.downsample.1')
    else:
        res = x
    return F.relu(out + res)


@torch.no_grad()
def pose_resnet_forward(x, sd, num_layers=50):
    """x: [N, 3, H, W] f32 CPU; sd: reference-keyed state_dict (CPU f32)."""
    kind, blocks = LAYERS[num_layers]
    x = F.relu(_bn(F.conv2d(x, sd['conv1.weight'], stride=2, padding=3), sd, 'bn1'))
    x = F.max_pool2d(x, 3, stride=2, padding=1)
    x1 = None
    for li, nb in enumerate(blocks):
        for b in range(nb):
            stride = 2 if (li > 0 and b == 0) else 1
            x = _block(x, sd, 'layer%d.%d' % (li + 1, b), kind, stride)
        if li == 0:
            x1 = x
    i = 0
    while 'deconv_layers.%d.weight' % i in sd:
        w = sd['deconv_layers.%d.weight' % i]
        x = F.conv_transpose2d(x, w, bias=sd.get('deconv_layers.%d.bias' % i), stride=2, padding=1)
        x = F.relu(_bn(x, sd, 'deconv_layers.%d' % (i + 1)))
        i += 3
    f = x
    hm = F.conv2d(f, sd['final_layer.weight'], sd.get('final_layer.bias'))
    return hm, x1, f


def _bn_train(x, params, buffers, p, momentum):
    """Train-mode BatchNorm2d (batch statistics; running statistics updated in `buffers` as
    nn.BatchNorm2d does, pose_resnet.py:18 BN_MOMENTUM = 0.1)."""
    return F.batch_norm(x, buffers[p + '.running_mean'], buffers[p + '.running_var'], params[p + '.weight'],
                        params[p + '.bias'], training=True, momentum=momentum, eps=BN_EPS)


def pose_resnet_train_forward(x, params, buffers, num_layers=50, momentum=0.1):
    """The reference PoseResNet.forward in train mode (pose_resnet.py:191-205 with every
    BatchNorm2d on batch statistics), differentiable: x [N, 3, H, W] f32 CPU; params: reference-keyed
    leaf tensors (requires_grad as the caller wants); buffers: running statistics, updated in
    place.  One call = one view of MultiViewPose (multiview_pose_resnet.py:26-45 runs the backbone
    per view, so each view has its own batch statistics).  -> (heatmaps, layer1 out, deconv out)."""
    kind, blocks = LAYERS[num_layers]

    def bn(t, p):
        return _bn_train(t, params, buffers, p, momentum)

    x = F.relu(bn(F.conv2d(x, params['conv1.weight'], stride=2, padding=3), 'bn1'))
    x = F.max_pool2d(x, 3, stride=2, padding=1)
    x1 = None
    for li, nb in enumerate(blocks):
        for b in range(nb):
            stride = 2 if (li > 0 and b == 0) else 1
            p = 'layer%d.%d' % (li + 1, b)
            if kind == 'bottleneck':
                out = F.relu(bn(F.conv2d(x, params[p + '.conv1.weight']), p + '.bn1'))
                out = F.relu(bn(F.conv2d(out, params[p + '.conv2.weight'], stride=stride, padding=1), p + '.bn2'))
                out = bn(F.conv2d(out, params[p + '.conv3.weight']), p + '.bn3')
            else:
                out = F.relu(bn(F.conv2d(x, params[p + '.conv1.weight'], stride=stride, padding=1), p + '.bn1'))
                out = bn(F.conv2d(out, params[p + '.conv2.weight'], padding=1), p + '.bn2')
            if p + '.downsample.0.weight' in params:
                res = bn(F.conv2d(x, params[p + '.downsample.0.weight'], stride=stride), p + '.downsample.1')
            else:
                res = x
            x = F.relu(out + res)
        if li == 0:
            x1 = x
    i = 0
    while 'deconv_layers.%d.weight' % i in params:
        x = F.conv_transpose2d(x, params['deconv_layers.%d.weight' % i], bias=params.get('deconv_layers.%d.bias' % i),
                               stride=2, padding=1)
        x = F.relu(bn(x, 'deconv_layers.%d' % (i + 1)))
        i += 3
    f = x
    hm = F.conv2d(f, params['final_layer.weight'], params.get('final_layer.bias'))
    return hm, x1, f
