#!/bin/bash
# soft-argmax: one map per 64-lane block, 16-B backward: tests + per-kernel durations in
# the training bench
OUT=gpurun_out/r5bl
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_train.py tests/test_gpu_validate.py tests/test_gpu_ddp.py tests/test_gpu_peaked.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --mode train --steps 5 --warmup 1 > $OUT/prof.log 2>&1 || exit 1
grep -h "softargmax\|mse_" $OUT/prof/run_kernel_stats.csv | cut -c1-160 | tee $OUT/stats.txt
grep '^{' $OUT/prof.log | tail -1 | cut -c1-200
rm -f $OUT/prof/run_kernel_trace.csv
