"""Per-launch timeline of network replays from a rocprofv3 kernel-trace CSV.

    python tools/replay_breakdown.py gpurun_out/prof/run_kernel_trace.csv [--last 5]

A replay = the network kernels from the first of a run of stem_pool_kernel launches (one per view in
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
    ap.add_argument('--per', type=int, default=1,
                    help='start launches per replay: a forward run depth-first over N chunks starts N stem runs '
                         '(plan.CHUNKS_F16X3 = 2); each chunk\'s early segment is merged with what follows it')
    a = ap.parse_args()
    st = a.start
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    pre = [r for r in rows if 'prefetch_kernel' in r[2]]
    rows = [r for r in rows if 'prefetch_kernel' not in r[2]]
    # the network's own kernels only (the decode / loss / triangulation graph runs on another
    # stream and may overlap the next replay); a replay starts at the first of a run of stem launches
    net = ('conv_igemm_kernel', 'conv_persist_kernel', 'bottleneck', 'tail_stream_kernel', 'tail_s2_kernel',
           'maxpool', 'pack_s2d_kernel', 'pack_kernel', 'pack_split_kernel', 'unpack', st)
    rows = [r for r in rows if any(k in r[2] for k in net)]
    replays, cur = [], None
    for s, e, n in rows:
        if st in n and (cur is None or st not in cur[-1][2]):
            if cur is not None:
                replays.append(cur)
            cur = [(s, e, n)]
        elif cur is not None:
            if s - cur[-1][1] > 20000:   # a graph replay runs back to back: a gap ends it (incomplete)
                cur = None
            else:
                cur.append((s, e, n))
    if cur is not None:
        replays.append(cur)
    if a.per > 1:
        # chunked forwards: the early segments of chunks 1 .. N-1 (each shorter than the last chunk's
        # segment, which runs on through the rest of the network) are merged with the segments after them
        merged, i = [], 0
        while i + a.per - 1 < len(replays):
            grp = replays[i:i + a.per]
            lens = [len(g) for g in grp]
            contiguous = all(grp[j + 1][0][0] - grp[j][-1][1] <= 20000 for j in range(a.per - 1))
            if contiguous and all(l == lens[0] for l in lens[:-1]) and lens[-1] > lens[0]:
                merged.append([x for g in grp for x in g])
                i += a.per
            else:
                i += 1
        replays = merged
    if replays:   # complete replays: the most common length
        k = statistics.mode(len(r) for r in replays)
        replays = [r for r in replays if len(r) == k]
    replays = replays[-a.last:]
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
