"""Per-launch timing of the PoseResNet plan (HIP events, many repetitions per layer).

    python tools/bench_layers.py [--layers 50] [--size 256] [--batch 128] [--precision bf16]

Prints one line per launch: shape, microseconds, TFLOP/s (algorithmic MACs x 2) and the
HBM bytes of its inputs+outputs / time (GB/s), to see which layers are MFMA- or HBM-bound.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

from posu import ops  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--layers', type=int, default=50)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--batch', type=int, default=128)
    ap.add_argument('--precision', default='bf16')
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--autotune', action='store_true', help='per-layer tile autotuning first')
    args = ap.parse_args()
    import bench
    dev = torch.device('cuda', 0)
    net = bench.build_model(args.layers, args.size, args.precision, dev)
    plan = net.plan(dev)
    code = plan.code
    esz = 2 if code == ops.BF16 else 4
    x_in = [torch.randn(args.batch, 3, args.size, args.size, device=dev)]
    rows = []

    def rec(name, fn, flops, nbytes):
        us = timeit(fn, args.reps)
        rows.append((name, us, flops, nbytes))
        print('%-22s %9.1f us %8.1f TF %8.0f GB/s' % (name, us, flops / us / 1e6, nbytes / us / 1e3), flush=True)

    xp = plan.pack_input(x_in, fused=False)
    if args.autotune:
        from posu.plan import tuned_tiles
        plan.autotune(xp, keep_features=False)
        for k, v in tuned_tiles().items():
            print('tile', v, k)
    rec('pack', lambda: plan.pack_input(x_in, fused=False), 0, x_in[0].numel() * 4 + xp.numel() * esz)
    y = plan.run_stem(xp)
    n, ho, wo, co = y.shape
    rec('stem', lambda: plan.run_stem(xp), 2 * n * ho * wo * co * 147, xp.numel() * esz + y.numel() * esz)
    p = ops.maxpool3x3s2_nhwc(y, code)
    rec('maxpool', lambda: ops.maxpool3x3s2_nhwc(y, code), 0, (y.numel() + p.numel()) * esz)
    raw = plan.pack_input(x_in)
    if not isinstance(raw, torch.Tensor):
        rec('pack+stem+pool(fused)', lambda: plan.stem_pool(raw), 2 * n * ho * wo * co * 147,
            x_in[0].numel() * 4 + p.numel() * esz)
    x = p
    for li, layer in enumerate(plan.layers):
        for bi, blk in enumerate(layer):
            res = x
            if blk.down is not None:
                d = blk.down
                res = d(x, code)
                k = x.shape[3]
                rec('l%d.%d.down' % (li + 1, bi), lambda d=d, x=x: d(x, code),
                    2 * res.shape[0] * res.shape[1] * res.shape[2] * res.shape[3] * k, (x.numel() + res.numel()) * esz)
            out = x
            last_i = len(blk.convs) - (0 if blk.dual is not None else 1)
            for ci, c in enumerate(blk.convs):
                last = ci == last_i
                o = c(out, code, residual=res if last else None)
                k = out.shape[3] * c.k * c.k
                nb = (out.numel() + o.numel() + (res.numel() if last else 0)) * esz
                rec('l%d.%d.c%d' % (li + 1, bi, ci + 1),
                    lambda c=c, out=out, r=(res if last else None): c(out, code, residual=r),
                    2 * o.shape[0] * o.shape[1] * o.shape[2] * o.shape[3] * k, nb)
                out = o
            if blk.dual is not None:
                dl = blk.dual
                o = dl(out, x, code)
                k = out.shape[3] + x.shape[3]
                nb = (out.numel() + x.numel() // (dl.stride2 ** 2) + o.numel()) * esz
                rec('l%d.%d.c3+down' % (li + 1, bi), lambda dl=dl, out=out, x=x: dl(out, x, code),
                    2 * o.numel() * k, nb)
                out = o
            x = out
    for i, dc in enumerate(plan.deconvs):
        xs_last = x
        o = dc(x, code)
        rec('deconv%d' % (i + 1), lambda dc=dc, x=x: dc(x, code),
            2 * o.numel() * x.shape[3] * 4, (x.numel() + o.numel()) * esz)
        x = o
    if plan.fuse_head:
        dc = plan.deconvs[-1]
        xin = xs_last
        rec('deconv3+head(fused)', lambda: ops.deconv4x4s2_head(xin, dc.w, dc.cout, dc.scale, dc.shift, plan.head_w,
                                                                  plan.njoints, plan.head_b, code, keep_f=False),
            2 * x.numel() * xin.shape[3] * 4 + 2 * x.shape[0] * x.shape[1] * x.shape[2] * 16 * 256,
            xin.numel() * esz + x.shape[0] * 16 * x.shape[1] * x.shape[2] * 4)
    hm = ops.head1x1_nchw(x, plan.head_w, plan.njoints, plan.head_b, code)
    rec('head', lambda: ops.head1x1_nchw(x, plan.head_w, plan.njoints, plan.head_b, code),
        2 * hm.numel() * x.shape[3], x.numel() * esz + hm.numel() * 4)
    tot = sum(r[1] for r in rows)
    fl = sum(r[2] for r in rows)
    print('TOTAL %.1f us  %.1f TF (conv FLOPs / all launch time)' % (tot, fl / tot / 1e6))


if __name__ == '__main__':
    main()
