#!/bin/bash
# r4g: stem pipeline depth + timing ablations; stem tests at HEAD
set -o pipefail
O=gpurun_out/r4g; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k stem > $O/stem_tests.log 2>&1 || { tail -20 $O/stem_tests.log; exit 1; }
tail -1 $O/stem_tests.log
echo "lib default (PFD 2, pool first)"; timeout -k 10 120 python3 tools/stem_micro.py || exit 1
for v in prev pfd1 abl1 abl2 abl4 abl7; do
  echo "lib $v"; timeout -k 10 120 python3 tools/with_lib.py pose-unsupervised_amd/build/r4g/libposeu_$v.so tools/stem_micro.py || exit 1
done
echo done
