#!/bin/bash
# r4t: weight-stream depth 8 -- strided tail (POSU_S2_KD=8; main = 4 with the tap loop unrolled,
# s2head = the committed kernel) and the plain layer3 streamed tail (POSU_TS_KD=8)
set -o pipefail
O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bottleneck.py -k "strided" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in main kd8 s2head; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/r4t/libposeu_$v.so"; fi
    echo "lib $v"; timeout -k 10 120 python3 $L tools/s2tail_micro.py | grep -E "strided tail|chained tail|identical" || exit 1
  done
  for v in main tskd8; do
    if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/r4t/libposeu_$v.so"; fi
    echo "lib $v"; timeout -k 10 120 python3 tools/chain_micro.py $L || exit 1
  done
done
echo done
