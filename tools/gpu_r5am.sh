#!/bin/bash
# stem weight-gradient reduction in 16 lanes per output: stem tests, training step
OUT=gpurun_out/r5am
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_kernels.py -k "stem" > $OUT/stem_tests.log 2>&1
rc=$?; tail -2 $OUT/stem_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --mode train --steps 20 --warmup 3 > $OUT/on_$r.json 2> $OUT/on_$r.err || exit $?
  python - "$OUT/on_$r.json" "on run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'])
PY
done
