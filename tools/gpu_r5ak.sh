#!/bin/bash
# training stem kernels (conv + weight gradient from the NCHW views): kernel tests, training tests,
# then the step A/B (STEM_KERNELS on / off), alternating
OUT=gpurun_out/r5ak
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_train_kernels.py -k "stem" > $OUT/stem_tests.log 2>&1
rc=$?; tail -3 $OUT/stem_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_train.py tests/test_gpu_train_full.py > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
Q="--mode train --steps 20 --warmup 3"
for r in 1 2; do
  for v in on off; do
    case $v in
      off) F="--plan-flag STEM_KERNELS=0";;
      on) F="";;
    esac
    timeout -k 10 300 python -u bench.py $Q $F > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'])
PY
  done
done
