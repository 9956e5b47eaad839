"""Micro-benchmark of single conv launches on random operands (HIP events, one process).

    python tools/conv_micro.py [--cases deconv3,l3c2] [--tiles -1,5,3] [--reps 50] [--rounds 3]

Each case is one PoseResNet-50@256 layer shape at batch 128 (bf16); every (case, tile)
pair is timed in interleaved rounds (methodology: one process, min over rounds).  Used to
A/B conv main-loop variants and as the target of `rocprofv3 --pmc` passes (--only).
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import ops  # noqa: E402

B = 128
# name: (kind, H, W, C, Cout, k, stride, pad)
CASES = {
    'stem': ('conv', 128, 128, 16, 64, 4, 1, 2),
    'l1c1': ('conv', 64, 64, 256, 64, 1, 1, 0),
    'l1c2': ('conv', 64, 64, 64, 64, 3, 1, 1),
    'l1c3': ('conv', 64, 64, 64, 256, 1, 1, 0),
    'l1c3r': ('conv', 64, 64, 64, 256, 1, 1, 0),  # with the residual add (Bottleneck tail)
    'l2c2': ('conv', 32, 32, 128, 128, 3, 1, 1),
    'l2c3': ('conv', 32, 32, 128, 512, 1, 1, 0),
    'l2c3r': ('conv', 32, 32, 128, 512, 1, 1, 0),
    'l2c1': ('conv', 32, 32, 512, 128, 1, 1, 0),
    'l3c1': ('conv', 16, 16, 1024, 256, 1, 1, 0),
    'l3c2': ('conv', 16, 16, 256, 256, 3, 1, 1),
    'l3c3': ('conv', 16, 16, 256, 1024, 1, 1, 0),
    'l3c3r': ('conv', 16, 16, 256, 1024, 1, 1, 0),
    'l4c2': ('conv', 8, 8, 512, 512, 3, 1, 1),
    'deconv1': ('deconv', 8, 8, 2048, 256, 4, 2, 1),
    'deconv2': ('deconv', 16, 16, 256, 256, 4, 2, 1),
    'deconv3': ('deconv', 32, 32, 256, 256, 4, 2, 1),
}


def flops(case):
    kind, h, w, c, co, k, s, p = CASES[case]
    if kind == 'deconv':
        return 2.0 * B * (2 * h) * (2 * w) * co * 4 * c
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    if case == 'stem':
        return 2.0 * B * ho * wo * co * 147
    return 2.0 * B * ho * wo * co * k * k * c


def make(case, dev, code):
    kind, h, w, c, co, k, s, p = CASES[case]
    dt = ops.torch_dtype(code)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, h, w, c, device=dev, generator=g).to(dt)
    bk = ops.conv_bk(code)
    kk = (4 if kind == 'deconv' else k * k) * c
    kp = (kk + bk - 1) // bk * bk
    cp = (co + 63) // 64 * 64
    nw = 4 if kind == 'deconv' else 1
    wt = (torch.randn(nw, cp, kp, device=dev, generator=g) * (1.0 / kk) ** 0.5).to(dt)
    scale = torch.ones(co, device=dev)
    shift = torch.zeros(co, device=dev)
    if kind == 'deconv':
        out = torch.empty(B, 2 * h, 2 * w, co, device=dev, dtype=dt)
        return lambda t: ops.deconv4x4s2_nhwc(x, wt, co, scale, shift, True, code, out=out, tile=t)
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    if case == 'stem':
        ho, wo = 128, 128
    out = torch.empty(B, ho, wo, co, device=dev, dtype=dt)
    res = torch.randn(B, ho, wo, co, device=dev, generator=g).to(dt) if case.endswith('r') else None
    return lambda t: ops.conv2d_nhwc(x, wt[0], co, k, k, s, p, scale, shift, res, True, code, out=out,
                                     out_hw=(ho, wo), tile=t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cases', default=','.join(CASES))
    ap.add_argument('--tiles', default='-1')
    ap.add_argument('--reps', type=int, default=50)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--precision', default='bf16')
    ap.add_argument('--stamps', action='store_true', help='per-block s_memtime breakdown of one launch')
    ap.add_argument('--epilogue', default='1', help='comma list of posu_set_conv_epilogue modes to A/B')
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    code = ops.dtype_code({'bf16': torch.bfloat16, 'fp16': torch.float16, 'fp32': torch.float32}[args.precision])
    cases = args.cases.split(',')
    tiles = [int(t) for t in args.tiles.split(',')]
    epis = [int(e) for e in args.epilogue.split(',')]
    if len(epis) > 1:  # A/B the epilogue: tile ids carry the mode as +100
        tiles = [t + 100 * e for e in epis for t in tiles]
    raw = {c: make(c, dev, code) for c in cases}

    def wrap(f):
        def run(t):
            if t >= 90 or len(epis) > 1:
                ops.set_conv_epilogue((t + 10) // 100)
                t = (t + 10) % 100 - 10
            return f(t)
        return run

    fns = {c: wrap(f) for c, f in raw.items()}
    best = {}
    for _ in range(args.rounds):
        for c in cases:
            for t in tiles:
                fn = fns[c]
                try:
                    fn(t)
                except RuntimeError as e:  # tile not admissible for this shape
                    best[(c, t)] = None
                    print('skip', c, t, e)
                    continue
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.reps):
                    fn(t)
                b.record()
                torch.cuda.synchronize()
                us = a.elapsed_time(b) * 1e3 / args.reps
                prev = best.get((c, t))
                best[(c, t)] = us if prev is None else min(prev, us)
    if args.stamps:
        from posu._native import call
        buf = torch.zeros(4 * 65536, dtype=torch.int64, device=dev)
        for c in cases:
            for t in tiles:
                buf.zero_()
                fns[c](t)
                call('posu_debug_conv_stamps', ctypes.c_void_p(buf.data_ptr()))
                fns[c](t)
                torch.cuda.synchronize()
                call('posu_debug_conv_stamps', None)
                st = buf.view(-1, 4).cpu()
                st = st[st[:, 2] > 0].double()
                t0 = st[:, 0].min()
                main = st[:, 1] - st[:, 0]
                epi = st[:, 2] - st[:, 1]
                span = st[:, 2].max() - t0
                cu = ((st[:, 3].long() >> 8) & 15) + 16 * ((st[:, 3].long() >> 13) & 7)
                print('%-8s tile %3d blocks %d span %.0f clk | per block: main %.0f (min %.0f max %.0f) epi %.0f '
                      '(min %.0f max %.0f) | busy %.3f | blocks/CU-slot %.2f' % (
                          c, t, st.shape[0], span, main.mean(), main.min(), main.max(), epi.mean(), epi.min(),
                          epi.max(), ((st[:, 2] - st[:, 0]).sum() / span / max(1, len(set(cu.tolist())))).item(),
                          st.shape[0] / max(1, len(set(cu.tolist())))), flush=True)
    for c in cases:
        for t in tiles:
            us = best.get((c, t))
            if us is None:
                continue
            print('%-8s tile %3d %9.1f us %8.1f TF' % (c, t, us, flops(c) / us / 1e6), flush=True)


if __name__ == '__main__':
    main()
