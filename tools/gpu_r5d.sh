#!/bin/bash
# r5d: the new / changed GPU tests (split dtype, training gates by cause, full-size training step,
# tail stream refusals), then the smoke and the default bench line (with the parity_mode leg).
OUT=gpurun_out/r5d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_split.py \
  tests/test_gpu_train.py tests/test_gpu_train_full.py tests/test_gpu_peaked.py tests/test_gpu_bottleneck.py \
  > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|vs oracle|vs the fp32|FAIL|Error" $OUT/tests.log | tail -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?
tail -c 400 $OUT/bench.json
exit $rc
