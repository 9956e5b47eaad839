"""Tensor-level wrappers over the training-path entry points of libposeu.so
(include/posu.h, "training path"): conv data / weight gradients, training-mode
BatchNorm (per-view statistics), its backward, channel sums and the max-pool
backward.  NHWC activations in the compute dtype, f32 statistics and gradients of
parameters.  cuda tensors only; no fallback.
"""
import torch

from . import _native as nat
from ._native import call, ptr, stream_of, require_cuda

_WS = {}
# 1x1 / stride-2 data gradients accumulated in place over dy's pixels (22.62 vs 23.02 ms per
# training step A/B); False runs them over the zero-upsampled grid
INPLACE_S2_DGRAD = True


def workspace(device, nbytes, slot='default'):
    """Grow-only scratch buffer per (device, slot, current stream), reused by consecutive
    launches on that stream only: a buffer is allocated, used and (when it grows) released on
    one stream, so the caching allocator orders its reuse behind every launch that used it (the
    training step runs weight gradients on a side stream, train_plan._Grads)."""
    key = (str(device), slot, torch.cuda.current_stream(device).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def conv2d_dgrad(dy, wt_packed, cin, kh, kw, stride, pad, hw, code, residual=None, out=None, inplace=False,
                 tile=None):
    """dx [N, H, W, cin] of a conv x -> dy; `hw` = (H, W) of x; optional residual added.
    inplace=True (1x1 / stride-2 convolutions with a residual only) accumulates into `residual`
    itself and returns it -- the caller gives up that tensor; otherwise nothing is mutated.
    tile: a conv tile configuration (posu_conv2d_dgrad_tile, ABI 15), None = the heuristic."""
    require_cuda(dy)
    n, ho, wo, cout = dy.shape
    h, w = hw
    if inplace and INPLACE_S2_DGRAD and out is None and residual is not None and kh == kw == 1 and stride == 2 \
            and pad == 0:
        out = residual  # accumulated in place over dy's pixels (posu_conv2d_dgrad)
    if out is None:
        out = torch.empty((n, h, w, cin), dtype=dy.dtype, device=dy.device)
    if tile is None:
        call('posu_conv2d_dgrad', code, ptr(dy), n, ho, wo, cout, ptr(wt_packed), cin, kh, kw, stride, pad,
             ptr(residual), ptr(out), h, w, stream_of(dy.device))
    else:
        call('posu_conv2d_dgrad_tile', code, ptr(dy), n, ho, wo, cout, ptr(wt_packed), cin, kh, kw, stride, pad,
             ptr(residual), ptr(out), h, w, int(tile), stream_of(dy.device))
    return out


def conv2d_wgrad(dy, x, creal, kh, kw, stride, pad, code, out=None):
    """dW [Cout, creal, kh, kw] f32 of a conv over x [N, H, W, C >= creal] with output grad dy."""
    require_cuda(dy, x)
    n, h, w, c = x.shape
    cout = dy.shape[3]
    need = nat.load().posu_conv2d_wgrad_workspace(code, n, h, w, c, cout, kh, kw, stride, pad)
    if need <= 0:
        raise RuntimeError('posu_conv2d_wgrad: partial buffer too large for this shape')
    ws = workspace(dy.device, need, 'wgrad')
    if out is None:
        out = torch.empty((cout, creal, kh, kw), dtype=torch.float32, device=dy.device)
    call('posu_conv2d_wgrad', code, ptr(dy), ptr(x), n, h, w, c, creal, cout, kh, kw, stride, pad, ptr(out),
         ptr(ws), ws.numel(), stream_of(dy.device))
    return out


def deconv4x4s2_wgrad(x, dy, code, out=None):
    """dW [Cin, Cout, 4, 4] f32 of ConvTranspose2d(4, s2, p1) with input x [N,H,W,Cin], output grad dy."""
    return conv2d_wgrad(x, dy, dy.shape[3], 4, 4, 2, 1, code, out=out)


def _bn_ws(device, nseg, c):
    return workspace(device, nat.load().posu_bn_workspace(nseg, c), 'bn')


def bn_train_fwd(z, nseg, gamma, beta, eps, momentum, running_mean=None, running_var=None):
    """Per-segment batch statistics of z [nseg*B, H, W, C]: (mean, rstd, scale, shift) each [nseg, C] f32."""
    require_cuda(z)
    c = z.shape[-1]
    pix = z.numel() // c
    if pix % nseg:
        raise ValueError('batch does not split into %d equal segments' % nseg)
    st = torch.empty((4, nseg, c), dtype=torch.float32, device=z.device)
    ws = _bn_ws(z.device, nseg, c)
    call('posu_bn_train_fwd', nat.dtype_code_of(z), ptr(z), nseg, pix // nseg, c, ptr(gamma), ptr(beta),
         float(eps), float(momentum), ptr(running_mean), ptr(running_var), ptr(st[0]), ptr(st[1]), ptr(st[2]),
         ptr(st[3]), ptr(ws), ws.numel(), stream_of(z.device))
    return st[0], st[1], st[2], st[3]


def bn_apply(z, nseg, scale, shift, residual=None, relu=True, out=None):
    require_cuda(z)
    c = z.shape[-1]
    pix = z.numel() // c
    if out is None:
        out = torch.empty_like(z)
    call('posu_bn_apply', nat.dtype_code_of(z), ptr(z), nseg, pix // nseg, c, ptr(scale), ptr(shift),
         ptr(residual), int(relu), ptr(out), stream_of(z.device))
    return out


def bn_apply_mask(z, nseg, scale, shift, residual=None):
    """y = relu(bn(z) (+ residual)) and its ReLU bit mask (uint8, one byte per 16-B chunk of y,
    bit e = [y_e > 0]) for bn_train_bwd(mask=...): the backward reads 1/16 of y's bytes."""
    require_cuda(z)
    c = z.shape[-1]
    pix = z.numel() // c
    y = torch.empty_like(z)
    mask = torch.empty(z.numel() * z.element_size() // 16, dtype=torch.uint8, device=z.device)
    call('posu_bn_apply_mask', nat.dtype_code_of(z), ptr(z), nseg, pix // nseg, c, ptr(scale), ptr(shift),
         ptr(residual), ptr(y), ptr(mask), stream_of(z.device))
    return y, mask


def bn_train_bwd(gy, y, z, nseg, mean, rstd, gamma, want_gres=False, dgamma=None, dbeta=None, relu_from=None,
                 mask=None):
    """Backward of y = relu?(bn(z) (+ r)); y=None and relu_from=None means no ReLU;
    relu_from=(scale, shift) recomputes the ReLU mask from z (no residual) instead of reading y;
    mask (bn_apply_mask's bits) replaces y.
    Returns (dz, gres or None, dgamma [C] f32, dbeta [C] f32)."""
    require_cuda(gy, z)
    c = z.shape[-1]
    pix = z.numel() // c
    dz = torch.empty_like(z)
    gres = torch.empty_like(z) if want_gres else None
    if dgamma is None:
        dgamma = torch.empty((c,), dtype=torch.float32, device=z.device)
    if dbeta is None:
        dbeta = torch.empty((c,), dtype=torch.float32, device=z.device)
    ws = _bn_ws(z.device, nseg, c)
    if mask is not None:
        if y is not None or relu_from is not None:
            raise ValueError('bn_train_bwd: give one ReLU mask source (mask, y or relu_from)')
        call('posu_bn_train_bwd_mask', nat.dtype_code_of(z), ptr(gy), ptr(mask), ptr(z), nseg, pix // nseg, c,
             ptr(mean), ptr(rstd), ptr(gamma), ptr(dgamma), ptr(dbeta), ptr(dz), ptr(gres), ptr(ws), ws.numel(),
             stream_of(z.device))
        return dz, gres, dgamma, dbeta
    msc, msh = relu_from if relu_from is not None else (None, None)
    call('posu_bn_train_bwd', nat.dtype_code_of(z), ptr(gy), ptr(y), ptr(msc), ptr(msh), ptr(z), nseg, pix // nseg, c,
         ptr(mean),
         ptr(rstd), ptr(gamma), ptr(dgamma), ptr(dbeta), ptr(dz), ptr(gres), ptr(ws), ws.numel(),
         stream_of(z.device))
    return dz, gres, dgamma, dbeta


def channel_sum(x, out=None):
    """sum over pixels of an NHWC tensor -> [C] f32."""
    require_cuda(x)
    c = x.shape[-1]
    if out is None:
        out = torch.empty((c,), dtype=torch.float32, device=x.device)
    ws = _bn_ws(x.device, 1, c)
    call('posu_channel_sum', nat.dtype_code_of(x), ptr(x), x.numel() // c, c, ptr(out), ptr(ws), ws.numel(),
         stream_of(x.device))
    return out


def maxpool3x3s2_bwd(x, gy):
    require_cuda(x, gy)
    n, h, w, c = x.shape
    ws = workspace(x.device, nat.load().posu_maxpool3x3s2_bwd_workspace(n, h, w, c), 'maxpool')
    gx = torch.empty_like(x)
    call('posu_maxpool3x3s2_bwd', nat.dtype_code_of(x), ptr(x), n, h, w, c, ptr(gy), ptr(gx), ptr(ws), ws.numel(),
         stream_of(x.device))
    return gx


def bn_relu_maxpool(z, nseg, scale, shift):
    """Training stem: (maxpool3x3s2(relu(bn(z))), argmax taps uint8) without writing the
    activation; the backward is maxpool3x3s2_bwd_idx(taps, gy, (H, W))."""
    require_cuda(z)
    n, h, w, c = z.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    y = torch.empty((n, ho, wo, c), dtype=z.dtype, device=z.device)
    idx = torch.empty((n, ho, wo, c), dtype=torch.uint8, device=z.device)
    call('posu_bn_relu_maxpool3x3s2_fwd', nat.dtype_code_of(z), ptr(z), nseg, n, h, w, c, ptr(scale), ptr(shift),
         ptr(y), ptr(idx), stream_of(z.device))
    return y, idx


def maxpool3x3s2_bwd_idx(idx, gy, hw):
    """Max-pool backward from stored argmax taps: gx [N, H, W, C], (H, W) = hw."""
    require_cuda(idx, gy)
    n, _, _, c = gy.shape
    h, w = hw
    gx = torch.empty((n, h, w, c), dtype=gy.dtype, device=gy.device)
    call('posu_maxpool3x3s2_bwd_idx', nat.dtype_code_of(gy), ptr(idx), ptr(gy), n, h, w, c, ptr(gx),
         stream_of(gy.device))
    return gx


def _views_arg(views):
    """A list of NCHW f32 [Nv, 3, H, W] cuda views of one shape -> (ctypes pointer array, Nv, H, W); the
    array object must stay alive until the call returns (the kernel arguments are copied at launch)."""
    import ctypes
    if not views or not all(v.is_cuda and v.dtype == torch.float32 and v.is_contiguous() for v in views):
        raise TypeError('stem views: contiguous f32 cuda tensors expected')
    n, c, h, w = views[0].shape
    if c != 3 or any(tuple(v.shape) != (n, c, h, w) for v in views):
        raise ValueError('stem views: views of one shape [N, 3, H, W] expected')
    arr = (ctypes.c_void_p * len(views))(*[v.data_ptr() for v in views])
    return arr, n, h, w


def stem_conv(views, weight, code):
    """The training stem's raw 7x7 / s2 / p3 convolution of the views (stacked view-major) from the f32
    parameter itself: z [V * Nv, H/2, W/2, 64] in the compute dtype (posu_stem_conv_views_fwd)."""
    import ctypes
    arr, n, h, w = _views_arg(views)
    require_cuda(weight)
    if weight.dtype != torch.float32 or tuple(weight.shape) != (64, 3, 7, 7) or not weight.is_contiguous():
        raise ValueError('stem_conv: a contiguous f32 [64, 3, 7, 7] weight expected')
    z = torch.empty((n * len(views), h // 2, w // 2, 64), dtype=nat_dtype(code), device=views[0].device)
    call('posu_stem_conv_views_fwd', code, ctypes.cast(arr, ctypes.c_void_p), len(views), n, h, w, ptr(weight),
         ptr(z), stream_of(z.device))
    return z


def stem_wgrad(views, dz, code, out=None):
    """dW [64, 3, 7, 7] f32 of the stem convolution from its output gradient dz (posu_stem_wgrad_views)."""
    import ctypes
    arr, n, h, w = _views_arg(views)
    require_cuda(dz)
    need = nat.load().posu_stem_wgrad_workspace(n * len(views), h, w)
    if need <= 0:
        raise ValueError('stem_wgrad: unsupported shape')
    ws = workspace(dz.device, need, 'stem_wgrad')
    if out is None:
        out = torch.empty((64, 3, 7, 7), dtype=torch.float32, device=dz.device)
    call('posu_stem_wgrad_views', code, ctypes.cast(arr, ctypes.c_void_p), len(views), n, h, w, ptr(dz), ptr(out),
         ptr(ws), ws.numel(), stream_of(dz.device))
    return out


def nat_dtype(code):
    from . import ops
    return ops.torch_dtype(code)
