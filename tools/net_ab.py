"""A/B whole-network settings in ONE process (methodology: interleaved rounds, one device).

    python tools/net_ab.py --settings "epi=1" "epi=2" "epi=2,nt=16" [--rounds 5 --reps 20]

Each setting is a comma list of knob=value (epi: posu_set_conv_epilogue, nt: streaming-store
threshold in MiB, stages, big, early, cand: autotune candidate set -- "all" (default), "base"
(no persistent +32 tiles), "halo" (all + halo tiles 64..68)).  Every setting is autotuned
under its own knobs and gets its own captured hipGraph of the R50@256 128-frame forward;
replays are timed with HIP events in interleaved rounds, per-setting median / min printed.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from posu import ops, synthetic as syn  # noqa: E402


def apply(setting):
    from posu import plan as P
    kv = dict(x.split('=') for x in setting.split(',') if x)
    cand = kv.get('cand', 'all')
    if not hasattr(P, '_orig_candidates'):
        P._orig_candidates = P._tile_candidates
    base = P._orig_candidates
    if cand == 'base':
        P._tile_candidates = lambda cout: [t for t in base(cout) if t < 32]
    elif cand == 'halo':
        P._tile_candidates = lambda cout: base(cout) + [64, 65, 66, 67, 68]
    else:
        P._tile_candidates = base
    ops.set_conv_epilogue(int(kv.get('epi', 1)))
    ops.set_conv_nt_threshold(int(float(kv.get('nt', 0)) * 2 ** 20))
    ops.set_conv_stages(int(kv.get('stages', 2)))
    ops.set_conv_tiles(int(kv.get('big', 1)))
    ops.set_conv_early_residual(int(kv.get('early', 8)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--settings', nargs='+', required=True)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--layers', type=int, default=50)
    ap.add_argument('--size', type=int, default=256)
    ap.add_argument('--groups', type=int, default=32)
    args = ap.parse_args()
    import bench
    dev = torch.device('cuda', 0)
    net = bench.build_model(args.layers, args.size, 'bf16', dev)
    views = [v.to(dev) for v in syn.synthetic_views(4, args.groups, args.size, seed=100)]
    plan = net.plan(dev)
    graphs = {}
    with torch.no_grad():
        apply('')
        for _ in range(2):
            plan.run(plan.pack_input(views), keep_features=False)
        from posu import plan as P
        for st in args.settings:
            apply(st)
            kv = dict(x.split('=') for x in st.split(',') if x)
            saved = P.CHAIN_BLOCKS
            P.CHAIN_BLOCKS = {'off': False, 'on': True, 'auto': 'auto'}[kv.get('chain', 'auto')]
            plan = P.PoseResNetPlan(net, plan.code)
            P.CHAIN_BLOCKS = saved
            P._TUNE_CACHE.clear()
            plan.autotune(plan.pack_input(views), keep_features=False)
            torch.cuda.synchronize()
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):
                    plan.run(plan.pack_input(views), keep_features=False)
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                plan.run(plan.pack_input(views), keep_features=False)
            torch.cuda.synchronize()
            graphs[st] = (g, plan)
        apply('')
        times = {st: [] for st in args.settings}
        for _ in range(args.rounds):
            for st in args.settings:
                g = graphs[st][0]
                g.replay()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.reps):
                    g.replay()
                b.record()
                torch.cuda.synchronize()
                times[st].append(a.elapsed_time(b) / args.reps)
    for st in args.settings:
        t = np.array(times[st])
        print('%-30s median %.4f ms  min %.4f ms' % (st, np.median(t), t.min()), flush=True)


if __name__ == '__main__':
    main()
