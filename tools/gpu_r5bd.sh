#!/bin/bash
# BN finalize, second form (block per 16 channels, lane sums met in LDS) vs the round-2 form:
# tests, per-kernel durations under the tracer (bn_micro), training step A/B
OUT=gpurun_out/r5bd
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_train.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in main fin1; do
  if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/ab13/libposeu_$v.so"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o run -- \
    python3 tools/bn_micro.py --reps 10 --rounds 1 $L > $OUT/micro_$v.txt 2> $OUT/micro_$v.err || exit 1
  python3 - $OUT/prof_$v/run_kernel_stats.csv $v <<'PY' | tee -a $OUT/finalize.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'finalize' in r['Name'] or 'bn_partial' in r['Name']:
        print(sys.argv[2], r['Name'][:60], r['Calls'], r['AverageNs'])
PY
done
for r in 1 2; do
  for v in main fin1; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/ab13/libposeu_$v.so"; fi
    timeout -k 10 300 python -u $L bench.py --mode train --steps 20 --warmup 3 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'])
PY
  done
done
