#!/bin/bash
# kernel trace + per-launch replay breakdown of one bench configuration:
#   tools/gpu_trace.sh OUT START_KERNEL [bench args...]
set -euo pipefail
OUT=$1; START=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $OUT/tiles.json"
timeout -k 10 300 python3 bench.py $COMMON "$@" > $OUT/tune.json 2> $OUT/tune.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py $COMMON "$@" --steps 10 --warmup 3 > $OUT/trace_bench.json 2> $OUT/trace_bench.err
python3 tools/replay_breakdown.py $OUT/trace/run_kernel_trace.csv --last 5 --start $START > $OUT/replay_breakdown.txt
cat $OUT/replay_breakdown.txt
