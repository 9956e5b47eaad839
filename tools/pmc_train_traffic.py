"""HBM traffic of one training step from rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE
runs of `bench.py --mode train`, no other tracing):

    python tools/pmc_train_traffic.py D1/run_counter_collection.csv D2/run_counter_collection.csv

The step = every dispatch from the last weight-packing launch (the first launch of a training step,
posu_pack_weights) to the end of the run, both streams.  FETCH_SIZE is doubled per the gfx950
correction of MI355X_MICROARCH.md (wide streaming reads report half their bytes); WRITE_SIZE is
taken as is; both are KiB.  The JSON line carries the commit (env POSU_COMMIT).
"""
import collections
import csv
import json
import os
import sys


def load(path, counter):
    rows = {}
    for r in csv.DictReader(open(path)):
        if r.get('Counter_Name') == counter:
            d = int(r['Dispatch_Id'])
            name, v = r['Kernel_Name'], float(r['Counter_Value'])
            prev = rows.get(d)
            rows[d] = (name, v + (prev[1] if prev else 0.0))
    return [(d,) + rows[d] for d in sorted(rows)]


def last_step(rows):
    starts = [i for i, (_, n, _) in enumerate(rows) if 'pack_weights_kernel' in n]
    if not starts:
        raise SystemExit('no pack_weights_kernel launch in the trace')
    return rows[starts[-1]:]


def category(n):
    for key, cat in (('wgrad', 'conv wgrad'), ('conv_igemm', 'conv fwd / dgrad'), ('conv_persist', 'conv fwd / dgrad'),
                     ('bn_', 'batchnorm'), ('channel_sum', 'batchnorm'), ('maxpool', 'maxpool'),
                     ('pack', 'weight packing'), ('multi_tensor_apply', 'adam (torch)')):
        if key in n:
            return cat
    return 'other'


def main():
    f = last_step(load(sys.argv[1], 'FETCH_SIZE'))
    w = last_step(load(sys.argv[2], 'WRITE_SIZE'))
    fb = sum(x[2] for x in f) * 2 * 1024
    wb = sum(x[2] for x in w) * 1024
    print(json.dumps({'launches': len(f), 'fetch_bytes_corrected': fb, 'write_bytes': wb,
                      'traffic_bytes': fb + wb, 'commit': os.environ.get('POSU_COMMIT')}))
    by = collections.defaultdict(lambda: [0.0, 0.0])
    for x in f:
        by[category(x[1])][0] += x[2] * 2 * 1024
    for x in w:
        by[category(x[1])][1] += x[2] * 1024
    for c, (a, b) in sorted(by.items(), key=lambda t: -(t[1][0] + t[1][1])):
        print('%-20s fetch %9.1f MB  write %9.1f MB' % (c, a / 1e6, b / 1e6))


if __name__ == '__main__':
    main()
