"""Tensor-level wrappers over libposeu.so entry points.

Every function here takes/returns torch tensors on a cuda (HIP) device, launches on
PyTorch's current stream, and raises if given CPU tensors: there is no fallback
path.  Autograd Functions wrap the kernels that the training step differentiates
through (soft-argmax, crop affine, epipolar loss, heatmap MSE).
"""
import torch

from . import _native as nat
from ._native import F32, BF16, F64, F16, F16X3, ptr, call, stream_of, require_cuda

_TORCH_OF = {F32: torch.float32, BF16: torch.bfloat16, F16: torch.float16, F16X3: torch.float16}


def dtype_code(dtype):
    if dtype in ('bf16', torch.bfloat16, BF16):
        return BF16
    if dtype in ('fp32', 'f32', torch.float32, F32):
        return F32
    if dtype in ('fp16', 'f16', torch.float16, F16):
        return F16
    if dtype in ('fp16x3', F16X3):
        return F16X3
    raise ValueError('unsupported compute dtype %r (bf16 | fp16 | fp16x3 | fp32)' % (dtype,))


def torch_dtype(code):
    return _TORCH_OF[code]


def cmul(code):
    """Stored elements per logical channel: 2 for the split dtype (a (hi, lo) fp16 pair,
    [hi 32 | lo 32] per 32-channel block, include/posu.h), else 1."""
    return 2 if code == F16X3 else 1


def channels(x, code):
    """Logical channel count of an NHWC activation tensor."""
    return x.shape[3] // cmul(code)


def widen(x, code):
    """NHWC activations -> f32 values (the split dtype's pairs summed: hi + lo is exact in f32)."""
    if code != F16X3:
        return x.float()
    n, h, w, c2 = x.shape
    t = x.view(n, h, w, c2 // 64, 2, 32).float()
    return (t[..., 0, :] + t[..., 1, :]).reshape(n, h, w, c2 // 2)


def conv_bk(code):
    return nat.load().posu_conv_bk(code)


# ---------------------------------------------------------------- layout ops
def pack_nchw_to_nhwc(x, code, cpad, out=None, hflip=False):
    """[N, C, H, W] f32 -> [N, H, W, cpad] (zero channels above C); hflip mirrors W."""
    require_cuda(x)
    x = x.contiguous().float()
    n, c, h, w = x.shape
    if out is None:
        out = torch.empty((n, h, w, cpad * cmul(code)), dtype=torch_dtype(code), device=x.device)
    call('posu_pack_nchw_to_nhwc', code, ptr(x), n, c, h, w, ptr(out), cpad, int(hflip), stream_of(x.device))
    return out


def pack_s2d_nchw(x, code, cpad, out=None, hflip=False):
    """[N, C, H, W] f32 -> space-to-depth [N, H/2, W/2, cpad] (channel (dy*2+dx)*C + c); hflip mirrors W."""
    require_cuda(x)
    x = x.contiguous().float()
    n, c, h, w = x.shape
    if out is None:
        out = torch.empty((n, h // 2, w // 2, cpad * cmul(code)), dtype=torch_dtype(code), device=x.device)
    call('posu_pack_s2d_nchw', code, ptr(x), n, c, h, w, ptr(out), cpad, int(hflip), stream_of(x.device))
    return out


def nhwc_to_nchw_f32(x, code):
    require_cuda(x)
    n, h, w, c = x.shape
    c //= cmul(code)
    out = torch.empty((n, c, h, w), dtype=torch.float32, device=x.device)
    call('posu_nhwc_to_nchw_f32', code, ptr(x), n, h, w, c, ptr(out), stream_of(x.device))
    return out


# ------------------------------------------------------------------ conv ops
def conv2d_nhwc(x, wpk, cout, kh, kw, stride, pad, scale, shift, residual, relu, code, out=None, out_hw=None,
                tile=-1):
    n, h, w, c = x.shape
    c //= cmul(code)
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (w + 2 * pad - kw) // stride + 1
    if out_hw is not None:
        ho, wo = out_hw
    if out is None:
        out = torch.empty((n, ho, wo, cout * cmul(code)), dtype=x.dtype, device=x.device)
    call('posu_conv2d_fwd', code, ptr(x), n, h, w, c, ptr(wpk), cout, kh, kw, stride, pad,
         ptr(scale), ptr(shift), ptr(residual), int(relu), ptr(out), ho, wo, int(tile), stream_of(x.device))
    return out


def conv1x1_dual_nhwc(x, x2, stride2, wpk, cout, shift, relu, code, out=None, tile=-1, scale=None):  # noqa: D401
    """act((W[:, :C] x + W[:, C:] x2[::stride2, ::stride2]) * scale + shift) (two 1x1 sources, one
    output; scale None = 1)."""
    n, h, w, c = x.shape
    _, h2, w2, c2 = x2.shape
    c //= cmul(code)
    c2 //= cmul(code)
    if out is None:
        out = torch.empty((n, h, w, cout * cmul(code)), dtype=x.dtype, device=x.device)
    call('posu_conv1x1_dual_fwd', code, ptr(x), n, h, w, c, ptr(x2), h2, w2, c2, int(stride2), ptr(wpk), cout,
         ptr(scale), ptr(shift), int(relu), ptr(out), int(tile), stream_of(x.device))
    return out


def bottleneck_nhwc(x, w1, s1, b1, w2, s2, b2, w3, s3, b3, code, out=None):
    """Fused identity-residual Bottleneck (posu_bottleneck_fwd): x [N, H, W, C] -> y."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty_like(x)
    call('posu_bottleneck_fwd', code, ptr(x), n, h, w, c, w1.shape[0], ptr(w1), ptr(s1), ptr(b1), ptr(w2), ptr(s2),
         ptr(b2), ptr(w3), ptr(s3), ptr(b3), ptr(out), stream_of(x.device))
    return out


def bottleneck_tail_stream_nhwc(t1, x, wstream, s2, b2, s3, b3, code, out=None):
    """conv2 + conv3 (+ residual) of a layer2 / layer3 identity Bottleneck with the weights
    streamed into registers (posu_bottleneck_tail_stream_fwd, csrc/tail_stream.hip; the split dtype
    also at layer1's shape); wstream = packing.pack_tail_stream(conv2 pack, conv3 pack)."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty_like(x)
    call('posu_bottleneck_tail_stream_fwd', code, ptr(t1), ptr(x), n, h, w, c // cmul(code), t1.shape[3] // cmul(code),
         ptr(wstream),
         wstream.numel() * wstream.element_size(), ptr(s2), ptr(b2), ptr(s3), ptr(b3), ptr(out), stream_of(x.device))
    return out


def bottleneck_s2_tail_nhwc(t1, x, wstream, s2, b2, shift, code, out=None):
    """conv2 (3x3 / stride 2) + the conv3 | downsample dual GEMM of layer2's first Bottleneck in one
    launch (posu_bottleneck_s2_tail_fwd, csrc/tail_s2.hip): t1 [N, H, 64, 128], x [N, H, 64, 256] ->
    y [N, H/2, 32, 512]; wstream = packing.pack_s2_tail_stream(conv2 pack, dual pack)."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, h // 2, w // 2, shift.numel()), dtype=x.dtype, device=x.device)
    call('posu_bottleneck_s2_tail_fwd', code, ptr(t1), ptr(x), n, h, w, c, t1.shape[3], ptr(wstream),
         wstream.numel() * wstream.element_size(), ptr(s2), ptr(b2), ptr(shift), shift.numel(), ptr(out),
         stream_of(x.device))
    return out


def bottleneck_s2_tail_next_nhwc(t1, x, wstream, s2, b2, shift, s1n, b1n, code, out=None, t1n=None):
    """The strided tail chained with the next identity block's conv1 + BN1 + ReLU over y
    (posu_bottleneck_s2_tail_next_fwd); wstream = packing.pack_s2_tail_stream(conv2 pack, dual pack,
    next conv1 pack).  Returns (y, t1n) with t1n [N, H/2, 32, 128] bit-identical to a conv launch of
    the next conv1 over y."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, h // 2, w // 2, shift.numel()), dtype=x.dtype, device=x.device)
    if t1n is None:
        t1n = torch.empty((n, h // 2, w // 2, s1n.numel()), dtype=x.dtype, device=x.device)
    call('posu_bottleneck_s2_tail_next_fwd', code, ptr(t1), ptr(x), n, h, w, c, t1.shape[3], ptr(wstream),
         wstream.numel() * wstream.element_size(), ptr(s2), ptr(b2), ptr(shift), shift.numel(), ptr(out), ptr(s1n),
         ptr(b1n), ptr(t1n), stream_of(x.device))
    return out, t1n


def bottleneck_tail_stream_next_nhwc(t1, x, wstream, s2, b2, s3, b3, s1n, b1n, code, out=None, t1n=None):
    """The tail above chained with the NEXT identity block's conv1 + BN1 + ReLU over its output
    (posu_bottleneck_tail_stream_next_fwd); wstream = packing.pack_tail_stream(conv2 pack, conv3
    pack, next conv1 pack).  Returns (y, t1n): t1n is what a conv launch of the next conv1 over y
    would produce, bit for bit."""
    n, h, w, c = x.shape
    p = t1.shape[3]
    if out is None:
        out = torch.empty_like(x)
    if t1n is None:
        t1n = torch.empty((n, h, w, p), dtype=x.dtype, device=x.device)
    cm = cmul(code)
    call('posu_bottleneck_tail_stream_next_fwd', code, ptr(t1), ptr(x), n, h, w, c // cm, p // cm, ptr(wstream),
         wstream.numel() * wstream.element_size(), ptr(s2), ptr(b2), ptr(s3), ptr(b3), ptr(out), ptr(s1n), ptr(b1n),
         ptr(t1n), stream_of(x.device))
    return out, t1n


def bottleneck_tail_stream_chain_nhwc(t1, x, wstream, s2, b2, s3, b3, s1n, b1n, code, out=None, t1n=None):
    """The last identity block's tail of a layer chained with the NEXT layer's first conv1 + BN1 + ReLU
    (C -> Pn = s1n.numel() = 2 P; posu_bottleneck_tail_stream_chain_fwd, split fp16): (y, t1n [N, H, W, Pn])."""
    n, h, w, c = x.shape
    cm = cmul(code)
    p, pn = t1.shape[3] // cm, s1n.numel()
    if out is None:
        out = torch.empty_like(x)
    if t1n is None:
        t1n = torch.empty((n, h, w, pn * cm), dtype=x.dtype, device=x.device)
    call('posu_bottleneck_tail_stream_chain_fwd', code, ptr(t1), ptr(x), n, h, w, c // cm, p, pn, ptr(wstream),
         wstream.numel() * wstream.element_size(), ptr(s2), ptr(b2), ptr(s3), ptr(b3), ptr(out), ptr(s1n), ptr(b1n),
         ptr(t1n), stream_of(x.device))
    return out, t1n


def bottleneck_down_tail_stream_nhwc(t1, x, wstream, s2, b2, s3, b3, code, s1n=None, b1n=None, out=None, t1n=None):
    """Layer1's first Bottleneck after its conv1 in split fp16 (posu_bottleneck_down_tail_stream_fwd):
    conv2 + the [conv3 | downsample] dual GEMM (scale s3, shift b3) + ReLU in one launch, t1 / x
    [N, H, 64, 64] -> y [N, H, 64, 256] (logical channels); with s1n / b1n also the next identity block's
    conv1 + BN1 + ReLU over y.  Returns (y, t1n or None)."""
    n, h, w, _ = x.shape
    cm = cmul(code)
    c = s3.numel()
    if out is None:
        out = torch.empty((n, h, w, c * cm), dtype=x.dtype, device=x.device)
    if s1n is not None and t1n is None:
        t1n = torch.empty_like(t1)
    call('posu_bottleneck_down_tail_stream_fwd', code, ptr(t1), ptr(x), n, h, w, c, t1.shape[3] // cm, ptr(wstream),
         wstream.numel() * wstream.element_size(), ptr(s2), ptr(b2), ptr(s3), ptr(b3), ptr(out), ptr(s1n), ptr(b1n),
         ptr(t1n if s1n is not None else None), stream_of(x.device))
    return out, (t1n if s1n is not None else None)


def bottleneck_down_nhwc(x, w1, s1, b1, w2, s2, b2, w3d, shift3, code, out=None):
    """Fused first Bottleneck of layer1 with its downsample (posu_bottleneck_down_fwd):
    x [N, H, W, C] -> y [N, H, W, w3d.shape[0]]."""
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, h, w, w3d.shape[0]), dtype=x.dtype, device=x.device)
    call('posu_bottleneck_down_fwd', code, ptr(x), n, h, w, c, w1.shape[0], ptr(w1), ptr(s1), ptr(b1), ptr(w2),
         ptr(s2), ptr(b2), ptr(w3d), ptr(shift3), ptr(out), stream_of(x.device))
    return out


def deconv4x4s2_nhwc(x, wpk, cout, scale, shift, relu, code, out=None, tile=-1):
    n, h, w, c = x.shape
    c //= cmul(code)
    if out is None:
        out = torch.empty((n, 2 * h, 2 * w, cout * cmul(code)), dtype=x.dtype, device=x.device)
    call('posu_deconv4x4s2_fwd', code, ptr(x), n, h, w, c, ptr(wpk), cout, ptr(scale), ptr(shift),
         int(relu), ptr(out), int(tile), stream_of(x.device))
    return out


def deconv4x4s2_head(x, wpk, cout, scale, shift, head_w, njoints, head_b, code, keep_f=True, hm_out=None,
                     f_out=None, head_w_lo=None):
    """Last deconv + BN + ReLU fused with the 1x1 head: returns (heatmaps NCHW f32, f NHWC or None).
    head_w_lo (2-byte dtypes): the head weight's rounding residual -> the split-precision head."""
    n, h, w, c = x.shape
    c //= cmul(code)
    if hm_out is None:
        hm_out = torch.empty((n, njoints, 2 * h, 2 * w), dtype=torch.float32, device=x.device)
    if keep_f and f_out is None:
        f_out = torch.empty((n, 2 * h, 2 * w, cout * cmul(code)), dtype=x.dtype, device=x.device)
    call('posu_deconv4x4s2_head_fwd', code, ptr(x), n, h, w, c, ptr(wpk), cout, ptr(scale), ptr(shift),
         ptr(f_out if keep_f else None), ptr(head_w), ptr(head_w_lo), njoints, ptr(head_b), ptr(hm_out),
         stream_of(x.device))
    return hm_out, (f_out if keep_f else None)


def head1x1_nchw(x, wpk, cout, bias, code, out=None):
    n, h, w, c = x.shape
    c //= cmul(code)
    if out is None:
        out = torch.empty((n, cout, h, w), dtype=torch.float32, device=x.device)
    call('posu_head1x1_nchw_fwd', code, ptr(x), n, h, w, c, ptr(wpk), cout, ptr(bias), ptr(out),
         stream_of(x.device))
    return out


def stem_pool_views(views, wpk, scale, shift, code, out=None, hflip=False):
    """stem_pool over the views of one forward in ONE launch (posu_stem_pool_views_fwd): a list of
    NCHW f32 [Nv, 3, H, W] tensors (same shape) -> NHWC [V * Nv, H/4, W/4, 64], view-major."""
    import ctypes
    if not views or not all(v.is_cuda for v in views):
        raise RuntimeError('stem_pool_views: HIP op needs GPU tensors')
    n, c, h, w = views[0].shape
    if c != 3 or any(tuple(v.shape) != (n, c, h, w) for v in views):
        raise ValueError('stem_pool_views: views of one shape [N, 3, H, W] expected')
    views = [v.contiguous().float() for v in views]
    if out is None:
        out = torch.empty((n * len(views), h // 4, w // 4, 64 * cmul(code)), dtype=torch_dtype(code),
                          device=views[0].device)
    arr = (ctypes.c_void_p * len(views))(*[v.data_ptr() for v in views])
    call('posu_stem_pool_views_fwd', code, ctypes.cast(arr, ctypes.c_void_p), len(views), n, h, w, int(bool(hflip)),
         ptr(wpk), ptr(scale), ptr(shift), ptr(out), stream_of(views[0].device))
    return out


def stem_pool(x, wpk, scale, shift, code, out=None, hflip=False):
    """Fused input pack + 7x7/s2 stem + BN + ReLU + 3x3/s2 max-pool: NCHW f32 [N, 3, H, W]
    -> NHWC [N, H/4, W/4, 64] (compute dtype)."""
    if not x.is_cuda:
        raise RuntimeError('stem_pool: HIP op needs a GPU tensor')
    n, c, h, w = x.shape
    if c != 3:
        raise ValueError('stem_pool: 3 input channels expected')
    x = x.contiguous().float()
    if out is None:
        out = torch.empty((n, h // 4, w // 4, 64 * cmul(code)), dtype=torch_dtype(code), device=x.device)
    call('posu_stem_pool_fwd', code, ptr(x), n, h, w, int(bool(hflip)), ptr(wpk), ptr(scale), ptr(shift), ptr(out),
         stream_of(x.device))
    return out


def maxpool3x3s2_nhwc(x, code, out=None):
    n, h, w, c = x.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    if out is None:
        out = torch.empty((n, ho, wo, c), dtype=x.dtype, device=x.device)
    call('posu_maxpool3x3s2_fwd', code, ptr(x), n, h, w, c // cmul(code), ptr(out), stream_of(x.device))
    return out


# ------------------------------------------------------------ heatmap decode
class _SoftArgmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hm, beta, affine):
        hm = hm.contiguous()
        n, j, h, w = hm.shape
        out = torch.empty((n, j, 2), dtype=torch.float32, device=hm.device)
        stats = torch.empty((n, j, 4), dtype=torch.float32, device=hm.device)
        call('posu_softargmax2d_fwd', ptr(hm), n, j, h, w, float(beta), ptr(affine), ptr(out), ptr(stats),
             stream_of(hm.device))
        ctx.save_for_backward(hm, stats, affine)
        ctx.beta = beta
        return out

    @staticmethod
    def backward(ctx, gout):
        hm, stats, affine = ctx.saved_tensors
        n, j, h, w = hm.shape
        gout = gout.contiguous().float()
        ghm = torch.empty_like(hm)
        call('posu_softargmax2d_bwd', ptr(hm), ptr(stats), n, j, h, w, float(ctx.beta), ptr(affine), ptr(gout),
             ptr(ghm), stream_of(hm.device))
        return ghm, None, None


def softargmax2d(hm, beta=100.0, affine=None):
    """[N, J, H, W] f32 heatmaps -> [N, J, 2] (x=col, y=row); affine [N, 2, 3] maps to image px."""
    require_cuda(hm, affine)
    if hm.dtype != torch.float32:
        raise TypeError('soft-argmax expects float32 heatmaps (got %s)' % hm.dtype)
    if affine is not None:
        affine = affine.to(device=hm.device, dtype=torch.float32).contiguous()
    return _SoftArgmax.apply(hm, beta, affine)


class _Affine2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pts, T):
        pts = pts.contiguous().float()
        n, j, _ = pts.shape
        out = torch.empty_like(pts)
        call('posu_affine2d_apply', ptr(pts), ptr(T), n, j, 0, ptr(out), stream_of(pts.device))
        ctx.save_for_backward(T)
        return out

    @staticmethod
    def backward(ctx, g):
        (T,) = ctx.saved_tensors
        g = g.contiguous().float()
        n, j, _ = g.shape
        gin = torch.empty_like(g)
        call('posu_affine2d_apply', ptr(g), ptr(T), n, j, 1, ptr(gin), stream_of(g.device))
        return gin, None


def affine2d(pts, T):
    """[N, J, 2] @ per-sample [N, 2, 3] affine (homogeneous)."""
    require_cuda(pts)
    T = T.to(device=pts.device, dtype=torch.float32).contiguous()
    return _Affine2d.apply(pts, T)


def argmax2d(hm, post_process=True, affine64=None):
    """get_final_preds on device: returns (preds [N, J, 2] f32, maxvals [N, J, 1] f32)."""
    require_cuda(hm)
    hm = hm.contiguous().float()
    n, j, h, w = hm.shape
    if affine64 is not None:
        affine64 = affine64.to(device=hm.device, dtype=torch.float64).contiguous()
    preds = torch.empty((n, j, 2), dtype=torch.float32, device=hm.device)
    maxv = torch.empty((n, j, 1), dtype=torch.float32, device=hm.device)
    call('posu_argmax2d_fwd', ptr(hm), n, j, h, w, int(bool(post_process)), ptr(affine64), ptr(preds), ptr(maxv),
         stream_of(hm.device))
    return preds, maxv


def flip_back(hm_flipped, perm=None, hm=None, shift=False, out=None):
    """Flip-test heatmaps back (mirror W, permute joints by `perm`, optional one-column
    shift) and, with `hm`, average: 0.5 * (hm + flip_back(hm_flipped))."""
    require_cuda(hm_flipped)
    hf = hm_flipped.contiguous().float()
    n, j, h, w = hf.shape
    if perm is not None and not isinstance(perm, torch.Tensor):
        perm = torch.tensor(list(perm), dtype=torch.int32)
    if perm is not None:
        perm = perm.to(device=hf.device, dtype=torch.int32).contiguous()
    if hm is not None:
        hm = hm.contiguous().float()
    if out is None:
        out = torch.empty_like(hf)
    call('posu_flip_back', ptr(hf), ptr(perm), ptr(hm), n, j, h, w, int(bool(shift)), ptr(out), stream_of(hf.device))
    return out


# ----------------------------------------------------------------- losses
class _Epipolar(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, F, subj):
        x = x.contiguous().float()
        v, n, j, _ = x.shape
        s = F.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        call('posu_epipolar_loss_fwd', ptr(x), ptr(w), ptr(F), ptr(subj), v, n, j, s, ptr(loss), None,
             stream_of(x.device))
        ctx.save_for_backward(x, w, F, subj)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        x, w, F, subj = ctx.saved_tensors
        v, n, j, _ = x.shape
        gloss = gloss.contiguous().float().reshape(1)
        gx = torch.empty_like(x)
        call('posu_epipolar_loss_bwd', ptr(x), ptr(w), ptr(F), ptr(subj), v, n, j, F.shape[0], ptr(gloss),
             ptr(gx), stream_of(x.device))
        return gx, None, None, None


def epipolar_loss(x, w, F, subj):
    """x [V, N, J, 2] image px; w [V, N, J] or None; F [S, V(V-1), 3, 3]; subj [N] int32."""
    require_cuda(x, w, F, subj)
    if w is not None:
        w = w.contiguous().float()
    return _Epipolar.apply(x, w, F.contiguous().float(), subj.contiguous().int())


def epipolar_residuals(x, w, F, subj):
    """Per (sample, pair, joint) weighted |x_j^T F x_i| [N, P, J] (no autograd)."""
    require_cuda(x, w, F, subj)
    x = x.contiguous().float()
    v, n, j, _ = x.shape
    p = v * (v - 1)
    loss = torch.empty((), dtype=torch.float32, device=x.device)
    resid = torch.empty((n, p, j), dtype=torch.float32, device=x.device)
    call('posu_epipolar_loss_fwd', ptr(x), ptr(None if w is None else w.contiguous().float()),
         ptr(F.contiguous().float()), ptr(subj.contiguous().int()), v, n, j, F.shape[0], ptr(loss), ptr(resid),
         stream_of(x.device))
    return resid, loss


class _JointsMSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, w):
        n, j = pred.shape[:2]
        hw = pred[0, 0].numel()
        pred = pred.contiguous().float()
        gt = gt.contiguous().float()
        ws = torch.empty((n * j,), dtype=torch.float32, device=pred.device)
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        call('posu_joints_mse_fwd', ptr(pred), ptr(gt), ptr(w), n, j, hw, ptr(ws), ptr(loss), stream_of(pred.device))
        ctx.save_for_backward(pred, gt, w)
        return loss

    @staticmethod
    def backward(ctx, gloss):
        pred, gt, w = ctx.saved_tensors
        n, j = pred.shape[:2]
        hw = pred[0, 0].numel()
        gloss = gloss.contiguous().float().reshape(1)
        gpred = torch.empty_like(pred)
        call('posu_joints_mse_bwd', ptr(pred), ptr(gt), ptr(w), n, j, hw, ptr(gloss), ptr(gpred),
             stream_of(pred.device))
        return gpred, None, None


def joints_mse(pred, gt, w=None):
    require_cuda(pred, gt, w)
    if w is not None:
        w = w.reshape(pred.shape[0], pred.shape[1]).contiguous().float()
    return _JointsMSE.apply(pred, gt, w)


# -------------------------------------------------------------- triangulation
def triangulate_dlt(M, intr, xy, vis=None, undistort=True, view_major=False):
    """M [G, V, 3, 4] f64, intr [G, V, 9] f64, xy [G, V, J, 2] (or [V, G, J, 2] with view_major) f32|f64,
    vis [G, V, J] u8 -> X [G, J, 3] f64."""
    require_cuda(M, intr, xy, vis)
    if view_major:
        v, g, j, _ = xy.shape
        sg, sv = j * 2, g * j * 2
    else:
        g, v, j, _ = xy.shape
        sg, sv = v * j * 2, j * 2
    M = M.contiguous().double()
    intr = intr.contiguous().double()
    xy = xy.contiguous()
    if xy.dtype == torch.float64:
        code = F64
    else:
        xy = xy.float()
        code = F32
    if vis is not None:
        vis = vis.contiguous().to(torch.uint8)
    X = torch.empty((g, j, 3), dtype=torch.float64, device=xy.device)
    call('posu_triangulate_dlt', ptr(M), ptr(intr), ptr(xy), code, sg, sv, ptr(vis), g, v, j, int(bool(undistort)),
         ptr(X), stream_of(xy.device))
    return X


def ransac_inliers(M, intr, xy, vis=None, reproj_thre=20.0, min_inliers=2, undistort=True):
    """multiviews.triangulate.ransac on device: M [G, V, 3, 4] f64, intr [G, V, 9] f64,
    xy [G, V, J, 2], vis [G, V, J] -> res_vis [G, V, J] uint8."""
    require_cuda(M, intr, xy)
    g, v, j, _ = xy.shape
    xy = xy.to(torch.float64).contiguous()
    if vis is not None:
        vis = vis.to(device=xy.device, dtype=torch.uint8).contiguous()
    out = torch.empty((g, v, j), dtype=torch.uint8, device=xy.device)
    call('posu_ransac_inliers', ptr(M.contiguous()), ptr(intr.contiguous()), ptr(xy), ptr(vis), g, v, j,
         int(bool(undistort)), float(reproj_thre), int(min_inliers), ptr(out), stream_of(xy.device))
    return out


def reproject(M, intr, xy, vis=None, undistort=True):
    """multiviews.triangulate.reproject_poses on device -> (proj [G, V, J, 2] f64, res_vis [G, V, J] uint8)."""
    require_cuda(M, intr, xy)
    g, v, j, _ = xy.shape
    xy = xy.to(torch.float64).contiguous()
    if vis is not None:
        vis = vis.to(device=xy.device, dtype=torch.uint8).contiguous()
    proj = torch.empty((g, v, j, 2), dtype=torch.float64, device=xy.device)
    res = torch.empty((g, v, j), dtype=torch.uint8, device=xy.device)
    call('posu_reproject', ptr(M.contiguous()), ptr(intr.contiguous()), ptr(xy), ptr(vis), g, v, j,
         int(bool(undistort)), ptr(proj), ptr(res), stream_of(xy.device))
    return proj, res
