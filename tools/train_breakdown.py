"""Per-step kernel breakdown of the training bench from a rocprofv3 kernel-trace CSV.

    python tools/train_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--steps 2] [--launches]

A step = the dispatches from one forward stem kernel (the first conv of the network) up to
the next one.  Prints, averaged over the last --steps steps: the step span, the summed
kernel time per category (conv fwd/dgrad, wgrad, BN, pool, torch, ...), and with
--launches every launch of the last step in order with its duration."""
import argparse
import collections
import csv
import re


def short(name):
    name = name.replace('(anonymous namespace)::', '').replace('posu::', '')
    name = re.sub(r'\(.*', '', name)
    return name[:90]


def category(n):
    if 'conv_wgrad' in n or 'wgrad_reduce' in n:
        return 'conv wgrad'
    if 'conv_igemm' in n or 'conv_persist' in n:
        return 'conv fwd / dgrad'
    if 'bn_' in n or 'channel_sum' in n:
        return 'batchnorm'
    if 'maxpool' in n:
        return 'maxpool'
    if 'pack' in n or 'weights' in n:
        return 'weight packing'
    if 'softargmax' in n or 'epipolar' in n or 'mse' in n:
        return 'heads / losses'
    if 'adam_kernel' in n:
        return 'adam (posu)'
    if 'multi_tensor_apply' in n:
        return 'adam (torch)'
    if 'nccl' in n.lower() or 'rccl' in n.lower():
        return 'rccl'
    return 'torch / other'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--steps', type=int, default=2)
    ap.add_argument('--first', default='pack_weights', help='substring of the first kernel of a step')
    ap.add_argument('--launches', action='store_true')
    ap.add_argument('--gaps', type=float, default=0.0,
                    help='also list the idle intervals (no kernel on any stream) longer than this many us')
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'],
                         r.get('Stream_Id') or r.get('Queue_Id') or '?'))
    rows.sort()
    streams = {}
    for r in rows:
        streams.setdefault(r[3], 0)
    rows_s = rows
    rows = [r[:3] for r in rows]
    starts = [i for i, r in enumerate(rows) if a.first in r[2]]
    if len(starts) < 2:
        raise SystemExit('fewer than two steps found (first-kernel marker %r)' % a.first)
    steps = [rows[starts[i]:starts[i + 1]] for i in range(len(starts) - 1)][-a.steps:]
    cat = collections.defaultdict(float)
    span = busy = 0.0
    for st in steps:
        span += (st[-1][1] - st[0][0]) / 1e3
        for s, e, n in st:
            cat[category(n)] += (e - s) / 1e3
            busy += (e - s) / 1e3
    k = len(steps)
    union = 0.0  # time with at least one kernel running (streams overlap)
    for st in steps:
        end = None
        for s, e, _ in sorted(st):
            if end is None or s >= end:
                union += (e - s) / 1e3
                end = e
            elif e > end:
                union += (e - end) / 1e3
                end = e
    print('%d steps: span %.1f us per step, kernel busy %.1f us (summed), %.1f us (union over streams), '
          '%d launches per step' % (k, span / k, busy / k, union / k, len(steps[-1])))
    for c, v in sorted(cat.items(), key=lambda x: -x[1]):
        print('  %-18s %9.1f us' % (c, v / k))
    # per stream (rocprofv3's Stream_Id / Queue_Id): kernel time and categories of the last steps
    lo, hi = steps[0][0][0], steps[-1][-1][1]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for s_, e_, n_, sid in rows_s:
        if lo <= s_ <= hi:
            per[sid][category(n_)] += (e_ - s_) / 1e3
    for sid, cats in sorted(per.items(), key=lambda x: -sum(x[1].values())):
        print('  stream %s: %.1f us per step (%s)' % (sid, sum(cats.values()) / k,
              ', '.join('%s %.0f' % (c, v / k) for c, v in sorted(cats.items(), key=lambda x: -x[1]))))
    if a.launches:
        t0 = steps[-1][0][0]
        for s, e, n in steps[-1]:
            print('%9.1f us  %s  @%.1f' % ((e - s) / 1e3, short(n), (s - t0) / 1e3))
    if a.gaps > 0:
        st = sorted(steps[-1])
        end, prev, total = None, None, 0.0
        print('idle intervals > %.1f us in the last step:' % a.gaps)
        for s, e, n in st:
            if end is not None and s > end:
                g = (s - end) / 1e3
                total += g
                if g > a.gaps:
                    print('  %8.1f us idle @%.1f after %s, before %s' % (g, (end - st[0][0]) / 1e3, short(prev),
                                                                      short(n)))
            if end is None or e > end:
                end, prev = e, n
        print('  idle total %.1f us' % total)


if __name__ == '__main__':
    main()
