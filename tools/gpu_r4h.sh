#!/bin/bash
# r4h: stem A-fragment row reuse / prefetch depth; stem FETCH_SIZE calibration against its known input bytes
set -o pipefail
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k stem > $O/stem_tests.log 2>&1 || { tail -20 $O/stem_tests.log; exit 1; }
tail -1 $O/stem_tests.log
echo "lib default (PFD 1, row reuse)"; timeout -k 10 120 python3 tools/stem_micro.py || exit 1
for v in head pfd2 abl1 abl7; do
  echo "lib $v"; timeout -k 10 120 python3 tools/with_lib.py pose-unsupervised_amd/build/r4g/libposeu_$v.so tools/stem_micro.py || exit 1
done
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/cal_$c -o run -- python3 tools/stem_micro.py --only 256 --reps 2 --rounds 1 > $O/cal_$c.log 2>&1 || { tail -5 $O/cal_$c.log; exit 1; }
done
python3 - <<'PY' || exit 1
import csv, glob
for c in ('FETCH_SIZE', 'WRITE_SIZE'):
    f = glob.glob('gpurun_out/r4h/cal_%s/**/run_counter_collection.csv' % c, recursive=True)[0]
    v = [float(r['Counter_Value']) for r in csv.DictReader(open(f)) if r['Counter_Name'] == c and 'stem_pool' in r['Kernel_Name']]
    print(c, 'per stem dispatch (KiB -> MB):', ['%.1f' % (x * 1024 / 1e6) for x in v])
PY
echo done
