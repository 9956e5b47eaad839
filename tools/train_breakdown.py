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
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
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
    if a.launches:
        for s, e, n in steps[-1]:
            print('%9.1f us  %s' % ((e - s) / 1e3, short(n)))


if __name__ == '__main__':
    main()
