"""HBM traffic of one training step from rocprofv3 PMC passes (separate FETCH_SIZE and WRITE_SIZE
runs of `bench.py --mode train`, no other tracing):

    python tools/pmc_train_traffic.py D1/run_counter_collection.csv D2/run_counter_collection.csv

The step = every dispatch from the last weight-packing launch (the first launch of a training step,
posu_pack_weights) to the end of the run, both streams.  FETCH_SIZE is doubled per the gfx950
correction of MI355X_MICROARCH.md (wide streaming reads report half their bytes); WRITE_SIZE is
taken as is; both are KiB.  Each class is set beside posu.roofline.r50_256_train_classes (every
tensor once per launch of the default bf16 batch-32 step).  The JSON line carries the commit (env POSU_COMMIT).
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pose-unsupervised_amd', 'lib'))
from posu import roofline as _rl  # noqa: E402


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
                     ('pack', 'weight packing'), ('adam_kernel', 'adam'), ('multi_tensor_apply', 'adam')):
        if key in n:
            return cat
    return 'heads / losses'


def main():
    f = last_step(load(sys.argv[1], 'FETCH_SIZE'))
    w = last_step(load(sys.argv[2], 'WRITE_SIZE'))
    fb = sum(x[2] for x in f) * 2 * 1024
    wb = sum(x[2] for x in w) * 1024
    alg = _rl.r50_256_train_classes()
    total_alg = sum(r + w for r, w in alg.values())
    print(json.dumps({'launches': len(f), 'fetch_bytes_corrected': fb, 'write_bytes': wb,
                      'traffic_bytes': fb + wb, 'algorithmic_bytes': total_alg,
                      'traffic_over_algorithmic': round((fb + wb) / total_alg, 4),
                      'commit': os.environ.get('POSU_COMMIT')}))
    by = collections.defaultdict(lambda: [0.0, 0.0])
    for x in f:
        by[category(x[1])][0] += x[2] * 2 * 1024
    for x in w:
        by[category(x[1])][1] += x[2] * 1024
    for c, (a, b) in sorted(by.items(), key=lambda t: -(t[1][0] + t[1][1])):
        r, w_ = alg.get(c, (0, 0))
        print('%-20s fetch %9.1f MB  write %9.1f MB  algorithmic read %9.1f MB  write %9.1f MB  traffic/alg %s'
              % (c, a / 1e6, b / 1e6, r / 1e6, w_ / 1e6, '%.3f' % ((a + b) / (r + w_)) if r + w_ else '-'))


if __name__ == '__main__':
    main()
