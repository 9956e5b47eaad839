#!/bin/bash
OUT=gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -k "ksplit or every_tile or invalid_tile or persistent or staggered or training_conv" > $OUT/tests.log 2>&1
rc=$?
tail -3 $OUT/tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/tile_micro.py --tiles 4,20,3,7,15,39,5,23 --reps 20 --rounds 3 > $OUT/tile_micro.txt 2>&1
rc=$?
cat $OUT/tile_micro.txt
exit $rc
