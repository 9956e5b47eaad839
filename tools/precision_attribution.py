"""Where the bf16 / fp16 chains' joint error comes from (measurement tool, not product code).

On the fitted peaked-heatmap R50@256 of tools/peaked.py, an fp32 functional forward on the GPU
(torch convolutions, not the HIP kernels) emulates the product's rounding points one stage at a
time: in a rounded stage every conv weight is rounded to the compute dtype as the plan packs it
(raw weights, BN applied in f32 by the epilogue; the downsample block's [w3*s3 | wd*sd] with the
scales folded in, as packing.pack_dual_1x1_weight / pack_bottleneck_down_weight do) and every
activation a conv of that stage reads is rounded (the plan stores activations in the dtype).
Each configuration runs the rest of the chain as the CPU oracle does (soft-argmax, crop affine,
fp64 triangulation) and is compared with the oracle chain: per-stage contribution to heatmap
error, image-px joint error and MPJPE (mm).  'all' rounds every stage (= the emulated product
chain); the real HIP chains (peaked.parity) are reported beside it.

    python tools/precision_attribution.py [fit_steps] > out.json
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO, os.path.join(REPO, 'tools')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

STAGES = ('stem', 'layer1', 'layer2', 'layer3', 'layer4', 'deconv1', 'deconv2', 'deconv3', 'head')
BN_EPS = 1e-5
BLOCKS = [3, 4, 6, 3]


def _fold(sd, p):
    s = sd[p + '.weight'].double() / torch.sqrt(sd[p + '.running_var'].double() + BN_EPS)
    b = sd[p + '.bias'].double() - sd[p + '.running_mean'].double() * s
    return s.float(), b.float()


def _q(t, dt, on):
    return t.to(dt).float() if on else t


def forward(x, sd, rounded, dt):
    """fp32 forward of R50 PoseResNet with the stages in `rounded` at dtype dt's rounding points."""
    def conv_bn(x, wkey, bnkey, on, relu=True, stride=1, pad=0, res=None):
        s, b = _fold(sd, bnkey)
        y = F.conv2d(_q(x, dt, on), _q(sd[wkey], dt, on), stride=stride, padding=pad)
        y = y * s[None, :, None, None] + b[None, :, None, None]
        if res is not None:
            y = y + res
        return F.relu(y) if relu else y

    on = 'stem' in rounded
    x = conv_bn(x, 'conv1.weight', 'bn1', on, stride=2, pad=3)
    x = F.max_pool2d(x, 3, stride=2, padding=1)
    for li, nb in enumerate(BLOCKS):
        on = 'layer%d' % (li + 1) in rounded
        for bi in range(nb):
            p = 'layer%d.%d' % (li + 1, bi)
            stride = 2 if (li > 0 and bi == 0) else 1
            t = conv_bn(x, p + '.conv1.weight', p + '.bn1', on)
            t = conv_bn(t, p + '.conv2.weight', p + '.bn2', on, stride=stride, pad=1)
            if bi == 0:
                # conv3 | downsample as one GEMM with both BN scales folded into the weights
                s3, b3 = _fold(sd, p + '.bn3')
                sdn, bd = _fold(sd, p + '.downsample.1')
                w3 = _q((sd[p + '.conv3.weight'].double() * s3.double()[:, None, None, None]).float(), dt, on)
                wd = _q((sd[p + '.downsample.0.weight'].double() * sdn.double()[:, None, None, None]).float(), dt, on)
                y = F.conv2d(_q(t, dt, on), w3) + F.conv2d(_q(x, dt, on), wd, stride=stride)
                x = F.relu(y + (b3.double() + bd.double()).float()[None, :, None, None])
            else:
                x = conv_bn(t, p + '.conv3.weight', p + '.bn3', on, res=_q(x, dt, on))
    for i, st in zip((0, 3, 6), ('deconv1', 'deconv2', 'deconv3')):
        on = st in rounded
        s, b = _fold(sd, 'deconv_layers.%d' % (i + 1))
        y = F.conv_transpose2d(_q(x, dt, on), _q(sd['deconv_layers.%d.weight' % i], dt, on), stride=2, padding=1)
        x = F.relu(y * s[None, :, None, None] + b[None, :, None, None])
    # 'head' rounds both head operands; 'head_act' / 'head_w' only the deconv output / the weights
    on_a = 'head' in rounded or 'head_act' in rounded
    on_w = 'head' in rounded or 'head_w' in rounded
    return F.conv2d(_q(x, dt, on_a), _q(sd['final_layer.weight'], dt, on_w), sd.get('final_layer.bias'))


def _split(t, dt, scale=0):
    """hi + lo pair of t in dtype dt (lo = the rounding residual rounded again), both as f32;
    scale: a power-of-two exponent applied before the split (the weight scaling of the split pack)."""
    t = t * (2.0 ** scale)
    hi = t.to(dt).float()
    lo = (t - hi).to(dt).float()
    return hi, lo


def forward_split(x, sd, dt, wscale=None, two=()):
    """fp32 forward of R50 PoseResNet at the split-precision plan's rounding points: every activation
    stored as a (hi, lo) pair of dt, every weight likewise (wscale: per-tensor power-of-two
    exponent so that max |w| sits at 2^wscale before the split, undone in the f32 epilogue), every
    conv summing hi.hi + lo.hi + hi.lo in f32 (the lo.lo term dropped).  two: the stages (STAGES
    names) run as TWO products, hi(w).hi(x) + hi(w).lo(x) -- the weights a single (scaled) dt value,
    the activations still pairs (round 6: the verdict's per-stage two-MFMA scheme)."""
    cur = {'stage': 'stem'}
    def store(t):
        h, l = _split(t, dt)
        return h + l

    def conv(x, w, stride=1, pad=0, transpose=False):
        e = 0
        if wscale is not None:
            e = wscale - int(torch.ceil(torch.log2(w.abs().max())).item())
        xh, xl = _split(x, dt)
        wh, wl = _split(w, dt, e)
        f = (lambda a, b: F.conv_transpose2d(a, b, stride=stride, padding=pad)) if transpose else \
            (lambda a, b: F.conv2d(a, b, stride=stride, padding=pad))
        if cur['stage'] in two:
            return (f(xh, wh) + f(xl, wh)) * (2.0 ** -e)
        return (f(xh, wh) + f(xl, wh) + f(xh, wl)) * (2.0 ** -e)

    def conv_bn(x, wkey, bnkey, relu=True, stride=1, pad=0, res=None):
        s, b = _fold(sd, bnkey)
        y = conv(x, sd[wkey], stride=stride, pad=pad)
        y = y * s[None, :, None, None] + b[None, :, None, None]
        if res is not None:
            y = y + res
        return store(F.relu(y) if relu else y)

    x = conv_bn(store(x), 'conv1.weight', 'bn1', stride=2, pad=3)
    x = F.max_pool2d(x, 3, stride=2, padding=1)
    for li, nb in enumerate(BLOCKS):
        cur['stage'] = 'layer%d' % (li + 1)
        for bi in range(nb):
            p = 'layer%d.%d' % (li + 1, bi)
            stride = 2 if (li > 0 and bi == 0) else 1
            t = conv_bn(x, p + '.conv1.weight', p + '.bn1')
            t = conv_bn(t, p + '.conv2.weight', p + '.bn2', stride=stride, pad=1)
            if bi == 0:
                s3, b3 = _fold(sd, p + '.bn3')
                sdn, bd = _fold(sd, p + '.downsample.1')
                w3 = (sd[p + '.conv3.weight'].double() * s3.double()[:, None, None, None]).float()
                wd = (sd[p + '.downsample.0.weight'].double() * sdn.double()[:, None, None, None]).float()
                # one GEMM over [t | x(stride)]: one weight exponent for both halves
                if wscale is not None:
                    e = wscale - int(torch.ceil(torch.log2(torch.maximum(w3.abs().max(), wd.abs().max()))).item())
                else:
                    e = 0
                th, tl = _split(t, dt)
                xs = x[:, :, ::stride, ::stride]
                xh, xl = _split(xs, dt)
                w3h, w3l = _split(w3, dt, e)
                wdh, wdl = _split(wd, dt, e)
                y = F.conv2d(th, w3h) + F.conv2d(tl, w3h) + F.conv2d(xh, wdh) + F.conv2d(xl, wdh)
                if cur['stage'] not in two:
                    y = y + F.conv2d(th, w3l) + F.conv2d(xh, wdl)
                y = y * (2.0 ** -e)
                x = store(F.relu(y + (b3.double() + bd.double()).float()[None, :, None, None]))
            else:
                x = conv_bn(t, p + '.conv3.weight', p + '.bn3', res=x)
    for k, i in enumerate((0, 3, 6)):
        cur['stage'] = 'deconv%d' % (k + 1)
        s, b = _fold(sd, 'deconv_layers.%d' % (i + 1))
        y = conv(x, sd['deconv_layers.%d.weight' % i], stride=2, pad=1, transpose=True)
        x = store(F.relu(y * s[None, :, None, None] + b[None, :, None, None]))
    cur['stage'] = 'head'
    return conv(x, sd['final_layer.weight']) + sd['final_layer.bias'][None, :, None, None]


def chain_metrics(hm, ref, task):
    from oracle import geometry_ref as G
    from posu.metrics import mpjpe_stats
    host, groups = task['host'], task['groups']
    hm = hm.float().cpu()
    sa = G.softargmax2d(hm)
    img = G.transform_back(sa, host['centers'].reshape(-1, 2), host['scales'].reshape(-1, 2), [64, 64])
    joints = img.view(4, groups, -1, 2)
    p2d = joints.permute(1, 0, 2, 3).reshape(groups * 4, -1, 2).double().numpy()
    X = G.triangulate_poses(host['cams'], p2d)
    st = mpjpe_stats(X, ref['X'])
    jerr = (joints - ref['joints']).norm(dim=-1)
    r6 = lambda v: float('%.6g' % float(v))  # noqa: E731
    return {'heatmap_abs_err_max': r6((hm - ref['hm']).abs().max()), 'joints_px_mean': r6(jerr.mean()),
            'joints_px_max': r6(jerr.max()), 'mpjpe_mm_mean': r6(st['mean']), 'mpjpe_mm_max': r6(st['max'])}


def main():
    import peaked
    dev = torch.device('cuda', 0)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1200
    only_split = len(sys.argv) > 2 and sys.argv[2] in ('split', 'split2')
    two_mfma = len(sys.argv) > 2 and sys.argv[2] == 'split2'
    torch.set_num_threads(16)
    t0 = time.time()
    net, task = peaked.fit_peaked(dev, steps=steps)
    torch.cuda.synchronize()
    out = {'fit_steps': steps, 'fit_s': round(time.time() - t0, 1), 'hip_chains': {}}
    ref = None
    from posu import plan as pl
    for prec in (('fp32',) if only_split else ('fp32', 'bf16', 'fp16')):
        out['hip_chains'][prec], ref = peaked.parity(net, task, dev, prec, ref)
        if prec != 'fp32':   # the plain head (round 3's chain) beside the split-precision one
            pl.PRECISE_HEAD = False
            out['hip_chains'][prec + '_plain_head'], _ = peaked.parity(net, task, dev, prec, ref)
            pl.PRECISE_HEAD = True
    sd = {k: v.detach().float() for k, v in net.state_dict().items() if v.is_floating_point()}
    x = torch.cat(task['views'])
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    with torch.no_grad():
        out['emulated'] = {'none': chain_metrics(forward(x, sd, (), torch.float32), ref, task)}
        # split-precision schemes (hi + lo operands, three MFMAs per product) for a parity-bearing
        # 2-byte mode: fp16 / bf16 pairs, with and without the weights' power-of-two scaling
        out['emulated']['split'] = {
            'fp16x3': chain_metrics(forward_split(x, sd, torch.float16), ref, task),
            'fp16x3_wscale14': chain_metrics(forward_split(x, sd, torch.float16, wscale=14), ref, task),
            'bf16x3': chain_metrics(forward_split(x, sd, torch.bfloat16), ref, task)}
        if two_mfma:
            # the two-product scheme stage by stage (the other stages fp16x3), and everywhere
            res = {st: chain_metrics(forward_split(x, sd, torch.float16, wscale=14, two=(st,)), ref, task)
                   for st in STAGES}
            res['all'] = chain_metrics(forward_split(x, sd, torch.float16, wscale=14, two=STAGES), ref, task)
            out['emulated']['split2_fp16'] = res
        if only_split:
            print(json.dumps(out, indent=1))
            return
        for dname, dt in (('bf16', torch.bfloat16), ('fp16', torch.float16)):
            res = {'all': chain_metrics(forward(x, sd, STAGES, dt), ref, task),
                   # the plan's split-precision head (PRECISE_HEAD): every stage rounded but the head
                   'all_but_head': chain_metrics(forward(x, sd, STAGES[:-1], dt), ref, task)}
            for s in STAGES + ('head_act', 'head_w'):
                res[s] = chain_metrics(forward(x, sd, (s,), dt), ref, task)
            out['emulated'][dname] = res
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
