#!/bin/bash
# r4y: the stem with two barriers per item (the first one was redundant with the pool's) vs the
# committed stem; stem GPU tests
set -o pipefail
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_rounding_emulation.py -k "stem" > $O/stem_tests.log 2>&1 || { tail -20 $O/stem_tests.log; exit 1; }
tail -1 $O/stem_tests.log
for r in 1 2; do
  echo "lib main"; timeout -k 10 120 python3 tools/stem_micro.py || exit 1
  echo "lib stemhead"; timeout -k 10 120 python3 tools/with_lib.py pose-unsupervised_amd/build/r4y/libposeu_stemhead.so tools/stem_micro.py || exit 1
done
echo done
