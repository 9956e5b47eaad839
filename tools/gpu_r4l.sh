#!/bin/bash
# r4l: the bench-config test (tile-count fix), then r4k's A/Bs
set -o pipefail
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench_config.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
sed -e 's#gpurun_out/r4j#gpurun_out/r4l#' -e '/pytest tests\/test_gpu_kernels.py/,+1d' tools/gpu_r4j.sh > /tmp/r4l_ab.sh
bash /tmp/r4l_ab.sh
