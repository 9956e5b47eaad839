"""Per-launch timeline of network replays from a rocprofv3 kernel-trace CSV.

    python tools/replay_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--last 5]

A replay = the dispatches from the first of a run of stem_pool_kernel launches (one per view in
the round-3 plan, one for all views since round 4) up to (not including) the next soft-argmax
kernel.  (The round-3 version restarted a replay at EVERY stem launch, so its breakdowns counted
one of the four per-view stem launches of that plan.)  Prints, for the chosen replays, each launch's median duration (us)
its gap to the previous launch's end (negative: overlap), with its kernel name, and the replay's launch-time sum and wall span (first start to last
end: the sum plus the gaps between launches).  The side-stream weight prefetches (prefetch_kernel,
plan.PREFETCH) run beside the network's launches: they are listed apart, not in the sequence."""
import argparse
import csv
import re
import statistics


def short(name):
    name = name.replace('(anonymous namespace)::', '').replace('posu::', '')
    name = re.sub(r'\(.*', '', name)
    return name[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('csv')
    ap.add_argument('--last', type=int, default=5, help='replays (from the end of the trace) to aggregate')
    ap.add_argument('--start', default='stem_pool_kernel',
                    help='kernel-name substring of a replay\'s first launch(es) (pack_split_kernel: the fp16x3 plan)')
    a = ap.parse_args()
    st = a.start
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    pre = [r for r in rows if 'prefetch_kernel' in r[2]]
    rows = [r for r in rows if 'prefetch_kernel' not in r[2]]
    replays, cur = [], None
    for s, e, n in rows:
        if st in n:
            if cur is not None and len(cur) and all(st in c[2] for c in cur) and s - cur[-1][1] <= 20000:
                cur.append((s, e, n))   # the next view's stem launch of the same replay
            else:
                cur = [(s, e, n)]
        elif cur is not None:
            if s - cur[-1][1] > 20000:   # a graph replay runs back to back: a gap ends it (incomplete)
                cur = None
            elif 'softargmax' in n:   # only complete replays (the configs1 leg has no soft-argmax)
                replays.append(cur)
                cur = None
            else:
                cur.append((s, e, n))
    replays = [r for r in replays if len(r) == len(replays[-1])][-a.last:]
    if not replays:
        raise SystemExit('no replay found')
    k = len(replays[0])
    print('%d replays of %d launches' % (len(replays), k))
    tot = 0.0
    for i in range(k):
        d = statistics.median((r[i][1] - r[i][0]) / 1e3 for r in replays)
        g = statistics.median((r[i][0] - r[i - 1][1]) / 1e3 for r in replays) if i else 0.0
        tot += d
        print('%3d %9.1f us  gap %6.1f  %s' % (i, d, g, short(replays[0][i][2])))
    span = statistics.median((r[-1][1] - r[0][0]) / 1e3 for r in replays)
    print('sum of launches %.1f us, replay span %.1f us (gaps %.1f us)' % (tot, span, span - tot))
    if pre:
        a0, a1 = replays[0][0][0], replays[-1][-1][1]
        inside = [r for r in pre if a0 <= r[0] <= a1]
        if inside:
            print('side-stream prefetches: %d launches per replay, %.1f us each on median (overlapped)'
                  % (round(len(inside) / len(replays)), statistics.median((e - s) / 1e3 for s, e, _ in inside)))


if __name__ == '__main__':
    main()
