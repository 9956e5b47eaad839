#!/bin/bash
# BN passes with the ReLU-mask source / residual presence as template parameters (no dummy loads)
# vs the run-time value-select form: tests, bn_micro, training step A/B
OUT=gpurun_out/r5bm
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_train_kernels.py tests/test_gpu_train.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for v in main prev; do
  if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/ab15/libposeu_$v.so"; fi
  echo "== $v" >> $OUT/micro.txt
  timeout -k 10 200 python -u tools/bn_micro.py $L >> $OUT/micro.txt 2> $OUT/micro_$v.err || exit $?
done
for r in 1 2; do
  for v in main prev; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/ab15/libposeu_$v.so"; fi
    timeout -k 10 300 python -u $L bench.py --mode train --steps 20 --warmup 3 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'], 'loss', d['loss'])
PY
  done
done
grep -E "==|TOTAL" $OUT/micro.txt
