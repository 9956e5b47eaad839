#!/bin/bash
# r4k: full GPU suite at this tree, then the A/Bs of r4j (packed epilogues, the committed conv
# kernel, the chained strided tail) and a replay breakdown
set -o pipefail
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -40 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
sed -e 's#gpurun_out/r4j#gpurun_out/r4k#' -e '/pytest tests\/test_gpu_kernels.py/,+1d' tools/gpu_r4j.sh > /tmp/r4k_ab.sh
bash /tmp/r4k_ab.sh
