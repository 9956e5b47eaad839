"""Is the configs[3] training step host-bound?  Times, per step after a sync, how long the host
takes to enqueue each phase (loss forward, zero_grad + backward, Adam) and when the GPU finishes,
then a free-running loop of steps (the bench's timing).  Same batch / model / optimizer as
bench.py --mode train.

    python tools/train_host_time.py [--steps 10] [bench.py train options, e.g. --plan-flag X=0]
"""
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pose-unsupervised_amd', 'lib'), REPO]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], '--mode', 'train'] + sys.argv[1:]
    args = bench.parse()
    bench.apply_plan_flags(args.plan_flag)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    tb = bench.train_batch(args, dev)
    if args.adam == 'posu':   # bench.py's default optimizer
        from posu.optim import Adam as PosuAdam
        opt = PosuAdam(tb['net'].parameters(), lr=1e-3)
    else:
        opt = torch.optim.Adam(tb['net'].parameters(), lr=1e-3, fused=args.adam == 'fused')
    from posu import plan as pplan

    def phases():
        t = [time.perf_counter()]
        loss = tb['loss']()
        t.append(time.perf_counter())
        opt.zero_grad(set_to_none=True)
        loss.backward()
        t.append(time.perf_counter())
        opt.step()
        t.append(time.perf_counter())
        return t

    pplan._Tuner.active, pplan._Tuner.reps = True, 3
    try:
        phases()
    finally:
        pplan._Tuner.active = False
    for _ in range(3):
        phases()
    torch.cuda.synchronize()
    rows = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t = phases()
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        rows.append([(b - t[0]) * 1e3 for b in t[1:]])
    med = [statistics.median(r[i] for r in rows) for i in range(4)]
    print('per step after a sync (ms from step start, median of %d): forward+loss enqueued %.2f, backward '
          'enqueued %.2f, Adam enqueued %.2f, GPU done %.2f' % (args.steps, *med))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = []
    for _ in range(args.steps):
        t = phases()
        host.append((t[-1] - t[0]) * 1e3)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print('free-running %d steps: host enqueue %.2f ms per step (median), wall %.2f ms per step, host ahead at '
          'the end by %.2f ms' % (args.steps, statistics.median(host), (t2 - t0) * 1e3 / args.steps,
                                  (t2 - t1) * 1e3))
    if os.environ.get('POSU_HOST_PROFILE'):   # where the host time goes: cProfile over free-running steps
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.steps):
            phases()
        torch.cuda.synchronize()
        pr.disable()
        pstats.Stats(pr).sort_stats('tottime').print_stats(40)
        pstats.Stats(pr).sort_stats('cumulative').print_stats(40)


if __name__ == '__main__':
    main()
