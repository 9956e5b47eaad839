#!/bin/bash
# BackwardAdam (per-stage fused Adam on the side stream inside the backward) vs torch fused Adam
# after the backward: tests, training step A/B
OUT=gpurun_out/r5be
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_train.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in backward fused; do
    timeout -k 10 300 python -u bench.py --mode train --steps 20 --warmup 3 --adam $v > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'], 'loss', d['loss'])
PY
  done
done
