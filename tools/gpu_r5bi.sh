#!/bin/bash
# 3x3 s2 data gradient as the sub-pixel deconv (S2_DGRAD_SUBPIXEL) vs the zero-upsampled conv: tests, training step A/B
OUT=gpurun_out/r5bi
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_train.py tests/test_abi_and_host.py tests/test_gpu_train_full.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in sub up; do
    if [ $v = sub ]; then F=""; else F="--plan-flag S2_DGRAD_SUBPIXEL=0"; fi
    timeout -k 10 300 python -u bench.py --mode train --steps 20 --warmup 3 $F > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'], 'loss', d['loss'])
PY
  done
done
