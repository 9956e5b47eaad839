#!/bin/bash
OUT=gpurun_out/r5e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -s tests/test_gpu_train.py \
  tests/test_gpu_train_full.py tests/test_gpu_peaked.py > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|vs oracle|vs the fp32|FAIL|Error" $OUT/tests.log | tail -30
exit $rc
