"""HBM traffic of one network forward from rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d D1 -o run --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d D2 -o run --output-format csv -- python3 bench.py ...
(the benched hipGraph replays themselves since round 4; the round-3 reductions came from eager
--no-graph runs whose launch list differed from the graph's)
    python tools/pmc_traffic.py D1/run_counter_collection.csv D2/run_counter_collection.csv [launches_per_forward]

Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of wide (16 B/lane) coalesced streaming reads, so it
is doubled; WRITE_SIZE is exact for 16-B stores.  Infinity-Cache hits are counted too.
The stem's f32 input reads are calibrated on their own (tools/stem_micro.py under a FETCH_SIZE
pass against the known input bytes, profiles/r04/stem_fetch_calibration.txt): --stem-fetch-scale
is the factor that calibration found (default 2, the guide's).
With the default plan's launch count (posu.roofline), each launch is printed beside its algorithmic bytes
(posu.roofline.r50_256_launches: inputs read once, weights once, outputs written once) and the
JSON line carries the total and traffic / algorithmic.
The JSON line carries the commit the passes ran at (env POSU_COMMIT, set by
tools/profile_round.sh).
Takes the LAST forward's network launches (pack + conv stack + maxpool), found from the
last run of input-pack launches unless a launch count is given.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'pose-unsupervised_amd',
                                'lib'))

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
    ap = argparse.ArgumentParser()
    ap.add_argument('fetch_csv')
    ap.add_argument('write_csv')
    ap.add_argument('launches', nargs='?', type=int, help='launches per forward (default: from the last stem)')
    ap.add_argument('--stem-fetch-scale', type=float, default=2.0)
    ap.add_argument('--stems', type=int, default=1,
                    help='runs of stem / input-pack launches per forward (a forward run depth-first over N chunks '
                         'has N: plan.CHUNKS_F16X3 = 2)')
    a = ap.parse_args()
    fetch = load(a.fetch_csv, 'FETCH_SIZE')
    write = load(a.write_csv, 'WRITE_SIZE')
    if a.launches:
        per_fwd = a.launches
    else:  # the last forward starts at the first input-pack launch of the final run of packs
        names = [x[1] for x in fetch]
        i = len(names)
        for _ in range(a.stems):   # back over --stems runs of stem / pack launches
            i -= 1
            while i >= 0 and not any(k in names[i] for k in ('pack', 'stem_pool')):
                i -= 1
            while i > 0 and any(k in names[i - 1] for k in ('pack', 'stem_pool')):
                i -= 1
        per_fwd = len(names) - i
    f = fetch[-per_fwd:]
    w = write[-per_fwd:]
    scale = [a.stem_fetch_scale if 'stem_pool' in x[1] else 2.0 for x in f]
    fb = [x[2] * s * 1024 for x, s in zip(f, scale)]
    wb = [x[2] * 1024 for x in w]
    line = {'launches': len(f), 'fetch_bytes_corrected': sum(fb), 'write_bytes': sum(wb),
            'traffic_bytes': sum(fb) + sum(wb), 'stem_fetch_scale': a.stem_fetch_scale,
            'commit': os.environ.get('POSU_COMMIT')}
    alg = None
    from posu import roofline
    split = any('f16s_t' in x[1] for x in f)   # the fp16x3 plan: its own launch list (no algorithmic table)
    line['plan'] = 'fp16x3' if split else 'default (bf16 / fp16)'
    if not split and len(f) == len(roofline.r50_256_launches()):
        alg = roofline.r50_256_launches()
        line['algorithmic_bytes'] = sum(r + wr for _, r, wr in alg)
        line['traffic_over_algorithmic'] = round(line['traffic_bytes'] / line['algorithmic_bytes'], 4)
    print(json.dumps(line))
    for i, (x, b, c) in enumerate(zip(f, fb, wb)):
        row = '%-40s fetch %8.1f MB  write %8.1f MB' % (x[1].replace('void posu::(anonymous namespace)::', '')[:40],
                                                         b / 1e6, c / 1e6)
        if alg:
            n, r, wr = alg[i]
            row += ' | %-44s alg read %7.1f write %7.1f MB  x%.2f' % (n, r / 1e6, wr / 1e6, (b + c) / (r + wr))
        print(row)


if __name__ == '__main__':
    main()
