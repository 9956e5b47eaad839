#!/bin/bash
# r5c: first timing of the split-fp16 (fp16x3) pipeline: bench line (headline in fp16x3, tuned),
# then a kernel trace of the tuned replays for the per-launch breakdown.
set -euo pipefail
OUT=gpurun_out/${1:-r5c}
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--precision fp16x3 --no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $OUT/tiles.json"
timeout -k 10 300 python3 bench.py $COMMON > $OUT/bench_fp16x3.json 2> $OUT/bench_fp16x3.err
tail -c 1500 $OUT/bench_fp16x3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/infer -o run -- \
  python3 bench.py $COMMON --steps 10 --warmup 3 > $OUT/infer_bench.log 2>&1
python3 tools/replay_breakdown.py $OUT/infer/run_kernel_trace.csv --last 5 --start stem_pool_kernel > $OUT/replay_breakdown.txt
cat $OUT/replay_breakdown.txt
