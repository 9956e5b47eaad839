"""HBM traffic of one network forward from rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D1 -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d D2 -o run --output-format csv -- python3 bench.py ...
(the benched hipGraph replays themselves since round 4; the round-3 reductions came from eager
--no-graph runs whose launch list differed from the graph's)
    python tools/pmc_traffic.py D1/run_counter_collection.csv D2/run_counter_collection.csv [launches_per_forward]

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B stores.  Infinity-Cache hits are counted too.
The JSON line carries the commit the passes ran at (env POSU_COMMIT, set by
tools/profile_round.sh).
Takes the LAST forward's network launches (pack + conv stack + maxpool), found from the
last run of input-pack launches unless a launch count is given.
"""
import csv
import json
import os
import sys

NET_KERNELS = ('conv_igemm_kernel', 'conv_persist_kernel', 'bottleneck', 'tail_stream_kernel', 'tail_s2_kernel',
               'stem_pool_kernel',
               'maxpool_kernel',
               'pack_s2d_kernel', 'pack_kernel')


def load(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        if r.get('Counter_Name') == counter:
            out.append((int(r['Dispatch_Id']), r['Kernel_Name'], float(r['Counter_Value'])))
    out.sort()
    return [x for x in out if any(k in x[1] for k in NET_KERNELS)]


def main():
    fetch = load(sys.argv[1], 'FETCH_SIZE')
    write = load(sys.argv[2], 'WRITE_SIZE')
    if len(sys.argv) > 3:
        per_fwd = int(sys.argv[3])
    else:  # the last forward starts at the first input-pack launch of the final run of packs
        names = [x[1] for x in fetch]
        i = len(names) - 1
        while i >= 0 and not any(k in names[i] for k in ('pack', 'stem_pool')):
            i -= 1
        while i > 0 and any(k in names[i - 1] for k in ('pack', 'stem_pool')):
            i -= 1
        per_fwd = len(names) - i
    f = fetch[-per_fwd:]
    w = write[-per_fwd:]
    fb = sum(x[2] for x in f) * 2 * 1024
    wb = sum(x[2] for x in w) * 1024
    print(json.dumps({'launches': len(f), 'fetch_bytes_corrected': fb, 'write_bytes': wb,
                      'traffic_bytes': fb + wb, 'commit': os.environ.get('POSU_COMMIT')}))
    for a, b in zip(f, w):
        print('%-60s fetch %8.1f MB  write %8.1f MB' % (a[1][:60], a[2] * 2 * 1024 / 1e6, b[2] * 1024 / 1e6))


if __name__ == '__main__':
    main()
