"""Weight packing: reference (PyTorch NCHW) parameters -> the layouts the HIP kernels read.

* Conv2d weight [Cout, Cin, KH, KW] -> [CoutPad][Kpad], k = (kh*KW + kw)*CinPad + ci
  (K contiguous per output channel, the B^T operand of the implicit GEMM).
* ConvTranspose2d(4, s2, p1) weight [Cin, Cout, 4, 4] -> [4 classes][CoutPad][Kpad]:
  output parity class (py, px) is a 2x2 stride-1 convolution whose tap (ty, tx) is the
  deconv tap (3 - py - 2ty, 3 - px - 2tx) (see csrc/conv_igemm.hip).
* Eval-mode BatchNorm2d -> per-channel (scale, shift) f32, folded in fp64:
  scale = gamma / sqrt(var + eps), shift = beta - mean * scale (+ conv bias * scale).
"""
import numpy as np
import torch

COUT_ALIGN = 64


def round_up(x, m):
    return (x + m - 1) // m * m


def pack_conv_weight(w, cin_pad, bk, dtype):
    cout, cin, kh, kw = w.shape
    k = kh * kw * cin_pad
    wt = torch.zeros((cout, kh, kw, cin_pad), dtype=torch.float32, device=w.device)
    wt[..., :cin] = w.detach().float().permute(0, 2, 3, 1)
    out = torch.zeros((round_up(cout, COUT_ALIGN), round_up(k, bk)), dtype=torch.float32, device=w.device)
    out[:cout, :k] = wt.reshape(cout, k)
    return out.to(dtype).contiguous()


def mfma_fragments(wpk):
    """[Cout][K] (posu_conv2d_fwd packing) -> [Cout/16][K/32][64 lanes][8]: the MFMA A operand of
    n-tile nt and k-step ks as one contiguous 1 KB block -- lane q * 16 + r holds row 16 nt + r,
    columns 32 ks + 8 q .. + 7 (v_mfma_f32_16x16x32 operand layout)."""
    co, k = wpk.shape
    return wpk.reshape(co // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(co // 16, k // 32, 64, 8)


def pack_s2_tail_stream(w2pk, wdual, w1n=None):
    """The per-wave weight streams of posu_bottleneck_s2_tail_fwd (csrc/tail_s2.hip) from the conv2
    [128][1152] (posu_conv2d_fwd) and dual [512][384] (pack_dual_1x1_weight) packs:
    [4 channel groups][84 k-steps][2 n-tiles][64 lanes][8].  Group cq, k-step p < 36: conv2 n-tile
    2 cq + j, k-step p (tap-major K); p = 36 + 12 nc + c: dual n-tile 8 nc + 2 cq + j, k-step c
    (t2's 4 k-steps, then x's 8).

    w1n (the next identity block's conv1 pack [128][512], posu_bottleneck_s2_tail_next_fwd): after
    dual chunk nc's 12 k-steps come the next conv1's 4 k-steps over that chunk's 128 y channels --
    [4][100][2][64][8], p = 36 + 16 nc + 12 + c: conv1n n-tile 2 cq + j, k-step 4 nc + c."""
    if tuple(w2pk.shape) != (128, 1152) or tuple(wdual.shape) != (512, 384):
        raise ValueError('pack_s2_tail_stream: conv2 pack [128][1152] and dual pack [512][384] expected, got %s / %s'
                         % (tuple(w2pk.shape), tuple(wdual.shape)))
    f2 = mfma_fragments(w2pk)                                     # [8][36][64][8]
    s2 = f2.reshape(4, 2, 36, 64, 8).permute(0, 2, 1, 3, 4)       # [cq][36][j][64][8]
    fd = mfma_fragments(wdual)                                    # [32][12][64][8]
    sd = fd.reshape(4, 4, 2, 12, 64, 8).permute(1, 0, 3, 2, 4, 5)  # [cq][nc][12][j][64][8]
    if w1n is None:
        return torch.cat([s2, sd.reshape(4, 48, 2, 64, 8)], dim=1).contiguous()
    if tuple(w1n.shape) != (128, 512):
        raise ValueError('pack_s2_tail_stream: the next conv1 pack must be [128][512], got %s' % (tuple(w1n.shape),))
    f1 = mfma_fragments(w1n)                                      # [8][16][64][8]
    s1 = f1.reshape(4, 2, 4, 4, 64, 8).permute(0, 2, 3, 1, 4, 5)  # [cq][nc][4][j][64][8]
    sdn = torch.cat([sd, s1], dim=2)                              # [cq][nc][16][j][64][8]
    return torch.cat([s2, sdn.reshape(4, 64, 2, 64, 8)], dim=1).contiguous()


def pack_tail_stream(w2pk, w3pk, w1n=None):
    """The per-wave weight streams of posu_bottleneck_tail_stream_fwd (csrc/tail_stream.hip) from
    the conv2 [P][9P] and conv3 [C][P] posu_conv2d_fwd packs: [NCQ][9 KT + NC KT][2][64][8] with
    NCQ = P / 32 channel groups, KT = P / 32 k-steps per tap, NC = C / P conv3 chunks.  Group cq,
    k-step p < 9 KT: conv2 n-tile 2 cq + j, k-step p; p = 9 KT + KT nc + c: conv3 n-tile
    2 NCQ nc + 2 cq + j, k-step c.

    w1n (the next identity block's conv1 pack [P][C], posu_bottleneck_tail_stream_next_fwd):
    after conv3 chunk nc come the next conv1's KT k-steps over that chunk's channels -- p =
    9 KT + 2 KT nc + c: conv3 as above; p = 9 KT + 2 KT nc + KT + c: conv1n n-tile 2 cq + j,
    k-step KT nc + c.

    Split fp16 packs (to_split: K' = 2 K, [hi 32 | lo 32] per 32 k) give KT = 2 P / 32: every pair of
    k-steps is the hi and the lo half of the same 32 channels, which the split tail multiplies as
    hi.hi + lo(w).hi(x) + hi(w).lo(x)."""
    planes, c = w2pk.shape[0], w3pk.shape[0]
    ncq, kt, nc = planes // 32, w3pk.shape[1] // 32, c // planes
    cm = kt * 32 // planes   # stored halves per logical channel (2: split packs)
    # (w1n may have 2 P rows: the next LAYER's first conv1, chained by a layer's last tail -- its k-steps
    # come per chunk as two halves of P output channels, posu_bottleneck_tail_stream_chain_fwd)
    f2 = mfma_fragments(w2pk)                                    # [2 ncq][9 kt][64][8]
    f3 = mfma_fragments(w3pk)                                    # [2 ncq nc][kt][64][8]
    s2 = f2.reshape(ncq, 2, 9 * kt, 64, 8).permute(0, 2, 1, 3, 4)
    s3 = f3.reshape(nc, ncq, 2, kt, 64, 8).permute(1, 0, 3, 2, 4, 5)              # [ncq][nc][kt][2][64][8]
    if w1n is None:
        return torch.cat([s2, s3.reshape(ncq, nc * kt, 2, 64, 8)], dim=1).contiguous()
    if w1n.shape[0] not in (planes, 2 * planes) or w1n.shape[1] != c * cm:
        raise ValueError('pack_tail_stream: the next conv1 pack must be [%d or %d][%d]' % (planes, 2 * planes, c * cm))
    nx = w1n.shape[0] // planes
    f1 = mfma_fragments(w1n)                                     # [2 ncq nx][nc kt][64][8]
    s1 = f1.reshape(nx, ncq, 2, nc, kt, 64, 8).permute(1, 3, 0, 4, 2, 5, 6)      # [ncq][nc][nx][kt][2][64][8]
    s31 = torch.cat([s3.unsqueeze(2), s1], dim=2).reshape(ncq, nc * (1 + nx) * kt, 2, 64, 8)
    return torch.cat([s2, s31], dim=1).contiguous()


def pack_down_tail_stream(w2pk, wdual, w1n=None):
    """The per-wave weight streams of posu_bottleneck_down_tail_stream_fwd (layer1's first Bottleneck,
    split fp16): conv2 [P][9 P'] as pack_tail_stream, then per output chunk nc (P channels) the dual
    GEMM's KT k-steps over t2 followed by its KT k-steps over the block input (pack_dual_1x1_weight's
    K order [conv3 | downsample], split: [C][2 P' ]), then (w1n) the next conv1's KT k-steps over the
    chunk -- [P/32][9 KT + NC (2 + (w1n given)) KT][2][64][8], KT = P' / 32 (P' the stored halves of P)."""
    planes, c = w2pk.shape[0], wdual.shape[0]
    ncq, kt2, nc = planes // 32, wdual.shape[1] // 32, c // planes
    kt = kt2 // 2
    if w2pk.shape[1] != 9 * kt * 32:
        raise ValueError('pack_down_tail_stream: conv2 pack [%d][%d] and dual pack [%d][%d] disagree on the planes'
                         % (tuple(w2pk.shape) + tuple(wdual.shape)))
    f2 = mfma_fragments(w2pk)
    s2 = f2.reshape(ncq, 2, 9 * kt, 64, 8).permute(0, 2, 1, 3, 4)
    fd = mfma_fragments(wdual)                                                    # [C/16][2 kt][64][8]
    sd = fd.reshape(nc, ncq, 2, kt2, 64, 8).permute(1, 0, 3, 2, 4, 5)            # [ncq][nc][2 kt][2][64][8]
    if w1n is not None:
        if tuple(w1n.shape) != (planes, c * kt * 32 // planes):
            raise ValueError('pack_down_tail_stream: the next conv1 pack must be [%d][%d]'
                             % (planes, c * kt * 32 // planes))
        f1 = mfma_fragments(w1n)
        s1 = f1.reshape(ncq, 2, nc, kt, 64, 8).permute(0, 2, 3, 1, 4, 5)          # [ncq][nc][kt][2][64][8]
        sd = torch.cat([sd, s1], dim=2)
    return torch.cat([s2, sd.reshape(ncq, -1, 2, 64, 8)], dim=1).contiguous()


def bottleneck_conv3_order(planes):
    """Input-channel order of the fused Bottleneck's conv3 K (csrc/bottleneck.hip): column
    32 b + 8 q + e reads channel 32 b + 16 (e >> 2) + 4 q + (e & 3) -- the order in which
    lane (pixel, q) of conv2's 16x16 accumulators (channels 4q..4q+3 of two n-tiles) forms
    an MFMA k-step."""
    idx = []
    for b in range(planes // 32):
        for q in range(4):
            for e in range(8):
                idx.append(32 * b + 16 * (e >> 2) + 4 * q + (e & 3))
    return idx


def bottleneck_conv1_order(cin):
    """Input-channel order of the fused Bottleneck's conv1 K: column 32 s + 8 q + e reads
    channel 32 s + 16 (q & 1) + 8 (q >> 1) + e, so lane q's x fragment of k-step s is the
    8-channel chunk its conv3 epilogue adds as the residual of output pair s."""
    return [32 * s + 16 * (q & 1) + 8 * (q >> 1) + e for s in range(cin // 32) for q in range(4) for e in range(8)]


def pack_bottleneck_conv1_weight(w, dtype):
    """conv1 weight [P, C, 1, 1] -> [P][C] with the K columns in bottleneck_conv1_order."""
    p, cin = w.shape[:2]
    if cin % 32 or w.shape[2:] != (1, 1):
        raise NotImplementedError('fused Bottleneck conv1: 1x1 kernel, input channels a multiple of 32')
    order = torch.tensor(bottleneck_conv1_order(cin), device=w.device)
    return w.detach().float().reshape(p, cin)[:, order].to(dtype).contiguous()


def pack_bottleneck_conv3_weight(w, dtype):
    """conv3 weight [C, P, 1, 1] -> [C][P] with the K columns in bottleneck_conv3_order."""
    cout, p = w.shape[:2]
    if p % 32 or w.shape[2:] != (1, 1):
        raise NotImplementedError('fused Bottleneck conv3: 1x1 kernel, planes a multiple of 32')
    wf = w.detach().float().reshape(cout, p)
    order = torch.tensor(bottleneck_conv3_order(p), device=w.device)
    return wf[:, order].to(dtype).contiguous()


def pack_bottleneck_down_weight(dual_w, planes):
    """Packed two-source tail weight [C][>= 2P] ([w3*s3 | wd*sd], pack_dual_1x1_weight) ->
    [C][2P] for posu_bottleneck_down_fwd: the conv3 columns 0..P-1 in bottleneck_conv3_order,
    the downsample columns P..2P-1 unchanged."""
    order = torch.tensor(bottleneck_conv3_order(planes) + list(range(planes, 2 * planes)), device=dual_w.device)
    return dual_w[:, order].contiguous()


def pack_stem_s2d_weight(w, cpad, bk, dtype):
    """7x7 / stride 2 / pad 3 stem weight [Cout, Cin, 7, 7] -> the equivalent 4x4 / stride 1 /
    top-left pad 2 weight over the 2x2 space-to-depth input (channel (dy*2+dx)*Cin + c):
    tap (ty, tx, dy, dx) is the 7x7 tap (2ty+dy-1, 2tx+dx-1) (zero where that is -1)."""
    cout, cin, kh, kw = w.shape
    if (kh, kw) != (7, 7) or 4 * cin > cpad:
        raise NotImplementedError('space-to-depth stem needs a 7x7 kernel and 4*Cin <= cpad')
    wf = w.detach().float()
    ws = torch.zeros((cout, 4, 4, cpad), dtype=torch.float32, device=w.device)
    for ty in range(4):
        for tx in range(4):
            for dy in range(2):
                for dx in range(2):
                    r, c = 2 * ty + dy - 1, 2 * tx + dx - 1
                    if 0 <= r < 7 and 0 <= c < 7:
                        sub = dy * 2 + dx
                        ws[:, ty, tx, sub * cin:(sub + 1) * cin] = wf[:, :, r, c]
    k = 16 * cpad
    out = torch.zeros((round_up(cout, COUT_ALIGN), round_up(k, bk)), dtype=torch.float32, device=w.device)
    out[:cout, :k] = ws.reshape(cout, k)
    return out.to(dtype).contiguous()


def pack_stem_fused_weight(w, dtype):
    """7x7 stem weight [64, 3, 7, 7] -> [64][224] for posu_stem_pool_fwd:
    k = kh*32 + kw*4 + c (kw < 7, c < 3; the 8th tap and the 4th channel are zeros)."""
    cout, cin, kh, kw = w.shape
    if (cin, kh, kw) != (3, 7, 7):
        raise NotImplementedError('fused stem needs a 3-channel 7x7 kernel')
    out = torch.zeros((cout, 7, 8, 4), dtype=torch.float32, device=w.device)
    out[:, :, :7, :3] = w.detach().float().permute(0, 2, 3, 1)
    return out.reshape(cout, 224).to(dtype).contiguous()


def pack_dual_1x1_weight(w_a, scale_a, w_b, scale_b, dtype):
    """Two 1x1 conv weights with their BN scales folded in, concatenated along K:
    [CoutPad][Ca + Cb] = [W_a * s_a | W_b * s_b] (fp64 product, one rounding)."""
    cout = w_a.shape[0]
    a = w_a.detach().double().reshape(cout, -1) * scale_a.double().view(-1, 1)
    b = w_b.detach().double().reshape(cout, -1) * scale_b.double().view(-1, 1)
    out = torch.zeros((round_up(cout, COUT_ALIGN), a.shape[1] + b.shape[1]), dtype=torch.float64, device=w_a.device)
    out[:cout] = torch.cat([a, b], dim=1)
    return out.to(dtype).contiguous()


def pack_deconv4x4_weight(w, bk, dtype):
    """ConvTranspose2d(4, s2, p1) weight [Cin][Cout][4][4] -> [4 classes][CoutPad][Kpad].  A 3x3
    weight [Cin][Cout][3][3] packs as its 4x4 zero-padding (tap index 3 = 0): a Conv2d(3, s2, p1)
    weight [co][ci][3][3] packed so makes the sub-pixel deconv that conv's data gradient."""
    cin, cout, kh, kw = w.shape
    wf = w.detach().float()
    if (kh, kw) == (3, 3):
        wf = torch.nn.functional.pad(wf, (0, 1, 0, 1))
    elif (kh, kw) != (4, 4):
        raise NotImplementedError('sub-pixel deconv kernel supports kernel 4 / stride 2 / padding 1 only')
    k = 4 * cin
    out = torch.zeros((4, round_up(cout, COUT_ALIGN), round_up(k, bk)), dtype=torch.float32, device=w.device)
    for py in range(2):
        for px in range(2):
            taps = []
            for ty in range(2):
                for tx in range(2):
                    taps.append(wf[:, :, 3 - py - 2 * ty, 3 - px - 2 * tx].t())  # [Cout, Cin]
            out[py * 2 + px, :cout, :k] = torch.cat(taps, dim=1)
    return out.to(dtype).contiguous()


# the split dtype (POSU_F16X3) scales each packed weight by a power of two so that its largest
# entry sits at 2^SPLIT_WEIGHT_EXP before the (hi, lo) split: the lo halves of small weights stay
# out of the fp16 subnormal range (tools/precision_attribution.py 'fp16x3_wscale14'); the kernels'
# f32 epilogue scale takes the inverse power (exact)
SPLIT_WEIGHT_EXP = 14


def split_exponent(w):
    """Power-of-two exponent e with max |w| * 2^e in (2^(SPLIT_WEIGHT_EXP - 1), 2^SPLIT_WEIGHT_EXP]."""
    m = float(w.detach().abs().max())
    if m == 0.0:
        return 0
    return SPLIT_WEIGHT_EXP - int(np.ceil(np.log2(m)))


def to_split(wpk, e=0):
    """An f32 / f64 pack [..., K] (K % 32 == 0, k in the kernel's logical order) -> the split fp16
    pack [..., 2K]: per 32-k block [hi 32 | lo 32] of wpk * 2^e, hi = fp16(v), lo = fp16(v - hi)."""
    v = wpk.double() * (2.0 ** e)
    if v.shape[-1] % 32:
        raise ValueError('split packs need K a multiple of 32 (got %d)' % v.shape[-1])
    hi = v.to(torch.float16)
    lo = (v - hi.double()).to(torch.float16)
    blk = v.shape[:-1] + (v.shape[-1] // 32, 1, 32)
    out = torch.cat([hi.reshape(blk), lo.reshape(blk)], dim=-2)
    return out.reshape(v.shape[:-1] + (2 * v.shape[-1],)).contiguous()


def fold_bn(bn, conv_bias=None):
    """(scale, shift) f32 of an eval-mode BatchNorm2d (optionally after a biased conv)."""
    gamma = bn.weight.detach().double() if bn.weight is not None else torch.ones_like(bn.running_mean.double())
    beta = bn.bias.detach().double() if bn.bias is not None else torch.zeros_like(bn.running_mean.double())
    mean = bn.running_mean.detach().double()
    var = bn.running_var.detach().double()
    scale = gamma / torch.sqrt(var + bn.eps)
    shift = beta - mean * scale
    if conv_bias is not None:
        shift = shift + conv_bias.detach().double() * scale
    return scale.float().contiguous(), shift.float().contiguous()


def pack_conv_dgrad_weight(w, bk, dtype):
    """Data-gradient weight of a Conv2d [Cout, Cin, KH, KW]: the forward packing of
    W[:, :, ::-1, ::-1].transpose(0, 1), i.e. [CinPad][Kpad] with k = (kh*KW + kw)*Cout + co
    (see posu_conv2d_dgrad)."""
    wt = w.detach().float().flip(2, 3).transpose(0, 1)
    return pack_conv_weight(wt, wt.shape[1], bk, dtype)


# ---- batched packing (posu_pack_weights): every weight of a training step in one launch
PACK_CONV, PACK_DGRAD, PACK_DECONV = 0, 1, 2
_JOB = np.dtype([('src', '<u8'), ('dst', '<u8'), ('block_start', '<i8'), ('mode', '<i4'), ('cout', '<i4'),
                 ('cin', '<i4'), ('kh', '<i4'), ('kw', '<i4'), ('pitch', '<i4'), ('rows', '<i4'), ('kpad', '<i4')],
                align=True)
assert _JOB.itemsize == 56   # sizeof(posu_pack_job)


class BatchedPacker:
    """Packs a fixed set of fp32 parameters into preallocated kernel-layout buffers with one
    posu_pack_weights launch (the per-layer torch packs above, restated in HIP).  add() returns
    the destination buffer (stable across steps); run() re-packs from the parameters' current
    values.  The job table is rebuilt if a parameter's storage moved."""

    def __init__(self, code, device):
        self.code, self.device = code, device
        self.jobs, self.srcs, self.dsts = [], [], []
        self.table, self.total, self._ptrs = None, 0, None

    def add(self, mode, w, cout, cin, kh, kw, pitch, rows, kpad):
        from . import ops
        from ._native import load
        if w.dtype != torch.float32 or not w.is_contiguous():
            raise TypeError('batched packing reads contiguous f32 parameters')
        n = rows * kpad * (4 if mode == PACK_DECONV else 1)
        dst = torch.empty(((4, rows, kpad) if mode == PACK_DECONV else (rows, kpad)), dtype=ops.torch_dtype(self.code),
                          device=self.device)
        assert dst.numel() == n
        blocks = int(load().posu_pack_job_blocks(mode, cout, cin, kh, kw, pitch, rows, kpad))
        if blocks <= 0:
            raise ValueError('posu_pack_weights cannot pack this weight (mode %d, %s)' % (mode, tuple(w.shape)))
        self.jobs.append([mode, cout, cin, kh, kw, pitch, rows, kpad, blocks])
        self.srcs.append(w)
        self.dsts.append(dst)
        self.table = None
        return dst

    def conv(self, w, cin_pad, bk):
        cout, cin, kh, kw = w.shape
        return self.add(PACK_CONV, w, cout, cin, kh, kw, cin_pad, round_up(cout, COUT_ALIGN),
                        round_up(kh * kw * cin_pad, bk))

    def dgrad(self, w, bk, cout_pitch=None):
        cout, cin, kh, kw = w.shape
        pitch = cout_pitch or cout
        return self.add(PACK_DGRAD, w, cout, cin, kh, kw, pitch, round_up(cin, COUT_ALIGN), round_up(kh * kw * pitch, bk))

    def deconv(self, w, bk):
        """A ConvTranspose2d(4, s2, p1) weight [cin][cout][4][4], or a 3x3 one read as its 4x4
        zero-padding (a Conv2d(3, s2, p1) weight: its data gradient, train_plan)."""
        cin, cout, kh, kw = w.shape
        return self.add(PACK_DECONV, w, cout, cin, kh, kw, cin, round_up(cout, COUT_ALIGN), round_up(4 * cin, bk))

    def _build(self):
        arr = np.zeros(len(self.jobs), dtype=_JOB)
        start = 0
        for i, (job, w, d) in enumerate(zip(self.jobs, self.srcs, self.dsts)):
            mode, cout, cin, kh, kw, pitch, rows, kpad, blocks = job
            arr[i] = (w.data_ptr(), d.data_ptr(), start, mode, cout, cin, kh, kw, pitch, rows, kpad)
            start += blocks
        self.table = torch.from_numpy(arr.view(np.uint8)).to(self.device)
        self.total = start
        self._ptrs = [w.data_ptr() for w in self.srcs]

    def run(self):
        from ._native import call, ptr, stream_of
        if self.table is None or self._ptrs != [w.data_ptr() for w in self.srcs]:
            self._build()
        call('posu_pack_weights', self.code, ptr(self.table), len(self.jobs), self.total, stream_of(self.device))
