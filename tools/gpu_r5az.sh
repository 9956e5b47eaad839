#!/bin/bash
# scratch-free BN / stem weight-gradient kernels (value selects instead of address selects): tests + step
OUT=gpurun_out/r5az
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_train.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode train --steps 20 --warmup 3 > $OUT/train.json 2> $OUT/train.err || exit $?
python - "$OUT/train.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('ms_per_step', d['ms_per_step'], 'value', d['value'])
PY
