#!/bin/bash
# training step per launch with start offsets and the idle intervals (HEAD, ABI 14)
set -o pipefail
O=gpurun_out/r5aq
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/train" -o run -- \
  python3 bench.py --mode train --steps 4 --warmup 2 > "$O/train_bench.log" 2>&1 || exit 1
python3 tools/train_breakdown.py "$O"/train/run_kernel_trace.csv --steps 2 --launches --gaps 5 > "$O/train_launches.txt"
python3 tools/train_breakdown.py "$O"/train/run_kernel_trace.csv --steps 2 | grep stream; rm -rf $O/train
head -12 $O/train_launches.txt
