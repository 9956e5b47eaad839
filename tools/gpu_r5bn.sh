#!/bin/bash
# posu.optim.Adam (posu_adam_step) vs torch's fused Adam in the training step: tests, A/B, kernel stats
OUT=gpurun_out/r5bn
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_optim.py tests/test_abi_and_host.py tests/test_gpu_train.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in posu fused; do
    timeout -k 10 300 python -u bench.py --mode train --steps 20 --warmup 3 --adam $v > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'], 'loss', d['loss'])
PY
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --mode train --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit 1
grep -h "adam" $OUT/prof/run_kernel_stats.csv | cut -c1-160 | tee -a $OUT/ab.txt
rm -f $OUT/prof/run_kernel_trace.csv
