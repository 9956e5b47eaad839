"""Cross-view heatmap aggregation (reference lib/models/multiview_pose_resnet.py:16-58,
``ChannelWiseFC`` / ``Aggregation``, NETWORK.AGGRE) as ONE MFMA GEMM per direction.

The reference runs V(V-1) = 12 separate [N*J, HW] x [HW, HW] matmuls and sums them per
target view.  Written as a block matrix over the concatenated source views,

    out[m][i*HW + p] = sum_{o != i} sum_q x_o[m][q] * W_{fc(i,o)}[q][p] / (V-1)
                     = sum_k X[m][k] * B[k][i*HW + p],   X[m][o*HW + q] = x_o[m][q],

every target view comes out of one launch (posu_gemm_rows_f32, view-major f32), with
B's diagonal blocks zero.  Backward: dX = dOut . B^T (the same kernel on B's other
packing) and dB = X^T dOut (the conv weight-gradient kernel with a 1x1 window), from
which each pair's dW is a block of dB.
"""
import torch

from . import ops, train_ops as T
from ._native import call, ptr, stream_of, require_cuda


def fc_index(nviews):
    """(target i, source o) -> index into the reference's aggre ModuleList
    (multiview_pose_resnet.py:46-55: for i, for o != i, fc_idx += 1)."""
    idx, out = 0, {}
    for i in range(nviews):
        for o in range(nviews):
            if o != i:
                out[(i, o)] = idx
                idx += 1
    return out


def pack_block_weight(weights, nviews, hw, transpose_for_forward, dtype):
    """weights: list of V(V-1) [HW, HW] f32.  Forward packing (rows = outputs n = i*HW+p,
    K = o*HW+q): Bt[n][k] = W_fc(i,o)[q][p] / (V-1); backward packing (rows = k): B[k][n]."""
    n = nviews * hw
    dev = weights[0].device
    out = torch.zeros((n, n), dtype=torch.float32, device=dev)
    idx = fc_index(nviews)
    s = 1.0 / (nviews - 1)
    for (i, o), f in idx.items():
        w = weights[f].detach().float() * s           # [q][p]
        if transpose_for_forward:
            out[i * hw:(i + 1) * hw, o * hw:(o + 1) * hw] = w.t()
        else:
            out[o * hw:(o + 1) * hw, i * hw:(i + 1) * hw] = w
    return out.to(dtype).contiguous()


def pack_rows(views_vm, code):
    """[V, M, HW] f32 (view-major) -> X [M, V*HW] in the compute dtype."""
    require_cuda(views_vm)
    v, m, hw = views_vm.shape
    x = torch.empty((m, v * hw), dtype=ops.torch_dtype(code), device=views_vm.device)
    call('posu_pack_view_rows', code, ptr(views_vm.contiguous()), v, m, hw, ptr(x), stream_of(views_vm.device))
    return x


def gemm_rows(x, wt, ncol, vblk, code):
    """out [ncol / vblk, M, vblk] f32 = blocks of x [M, K] . wt^T (wt [ncol, K])."""
    m, k = x.shape
    out = torch.empty((ncol // vblk, m, vblk), dtype=torch.float32, device=x.device)
    call('posu_gemm_rows_f32', code, ptr(x), m, k, ptr(wt), ncol, vblk, ptr(out), stream_of(x.device))
    return out


class _AggregateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hm_vm, code, *weights):
        v, n, j, h, w = hm_vm.shape
        hw = h * w
        x = pack_rows(hm_vm.reshape(v, n * j, hw), code)
        bt = pack_block_weight(weights, v, hw, True, ops.torch_dtype(code))
        out = gemm_rows(x, bt, v * hw, hw, code)
        ctx.save_for_backward(x, *weights)
        ctx.code, ctx.shape = code, (v, n, j, h, w)
        return out.reshape(v, n, j, h, w)

    @staticmethod
    def backward(ctx, gout):
        x, *weights = ctx.saved_tensors
        code = ctx.code
        v, n, j, h, w = ctx.shape
        hw = h * w
        g = pack_rows(gout.float().reshape(v, n * j, hw), code)           # [M, V*HW]
        dhm = None
        if ctx.needs_input_grad[0]:
            b = pack_block_weight(weights, v, hw, False, ops.torch_dtype(code))
            dhm = gemm_rows(g, b, v * hw, hw, code).reshape(v, n, j, h, w)  # per source view o
        grads = [None] * len(weights)
        if any(ctx.needs_input_grad[2:]):
            m = n * j
            # dBt[n][k] = sum_m g[m][n] x[m][k]: the 1x1 weight gradient over M "pixels"
            dbt = T.conv2d_wgrad(g.view(m, 1, 1, v * hw), x.view(m, 1, 1, v * hw), v * hw, 1, 1, 1, 0,
                                 code).view(v * hw, v * hw)
            s = 1.0 / (v - 1)
            for (i, o), f in fc_index(v).items():
                if ctx.needs_input_grad[2 + f]:
                    grads[f] = (dbt[i * hw:(i + 1) * hw, o * hw:(o + 1) * hw].t() * s).contiguous()
        return (dhm, None) + tuple(grads)


def aggregate(views, weights, code):
    """views: list of V [N, J, H, W] f32 cuda heatmaps; weights: the V(V-1) ChannelWiseFC
    matrices -> list of V aggregated heatmaps (Aggregation.forward)."""
    hm_vm = torch.stack([t.float() for t in views], 0)
    out = _AggregateFn.apply(hm_vm, code, *weights)
    return list(out.unbind(0))


class _ChannelFCFn(torch.autograd.Function):
    """ChannelWiseFC.forward (multiview_pose_resnet.py:23-28): out[n, c] = in[n, c].flatten() @ W
    as one rows GEMM (posu_gemm_rows_f32); backward dX = dOut . W^T (same kernel, W as the
    packed operand) and dW = X^T . dOut (the 1x1 weight-gradient kernel over M rows)."""

    @staticmethod
    def forward(ctx, inp, weight, code):
        n, c, h, w = inp.shape
        hw = h * w
        x = pack_rows(inp.float().reshape(1, n * c, hw), code)                      # [M, HW]
        wt = weight.detach().float().t().contiguous().to(ops.torch_dtype(code))    # [p][q]
        out = gemm_rows(x, wt, hw, hw, code)                                         # [1, M, HW]
        ctx.save_for_backward(x, weight)
        ctx.code, ctx.shape = code, (n, c, h, w)
        return out.reshape(n, c, h, w)

    @staticmethod
    def backward(ctx, gout):
        x, weight = ctx.saved_tensors
        code = ctx.code
        n, c, h, w = ctx.shape
        hw, m = h * w, n * c
        g = pack_rows(gout.float().reshape(1, m, hw), code)
        dinp = dw = None
        if ctx.needs_input_grad[0]:
            wq = weight.detach().float().contiguous().to(ops.torch_dtype(code))     # [q][p]
            dinp = gemm_rows(g, wq, hw, hw, code).reshape(n, c, h, w)
        if ctx.needs_input_grad[1]:
            dbt = T.conv2d_wgrad(g.view(m, 1, 1, hw), x.view(m, 1, 1, hw), hw, 1, 1, 1, 0, code).view(hw, hw)
            dw = dbt.t().contiguous()
        return dinp, dw, None


def channel_fc(inp, weight, code):
    """[N, C, H, W] cuda heatmaps x ChannelWiseFC weight [HW, HW] -> [N, C, H, W] f32.
    H*W must be a power of two (the rows GEMM's K; 64x64 / 32x32 heatmaps)."""
    require_cuda(inp, weight)
    hw = inp.shape[2] * inp.shape[3]
    if hw & (hw - 1) or hw < 64:
        raise NotImplementedError('ChannelWiseFC on the HIP path needs H*W a power of two >= 64 (got %d)' % hw)
    return _ChannelFCFn.apply(inp, weight, code)
