#!/bin/bash
# r4f: in-graph per-kernel times of the network with and without the strided layer2 tail
# (kernel trace + replay breakdown, tuned tiles loaded from one table).
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $O/tiles.json"
timeout -k 10 300 python3 bench.py $C > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
for f in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s2_$f -o run -- \
    python3 bench.py $C --steps 10 --warmup 3 --plan-flag S2_TAIL=$f > $O/s2_$f.log 2>&1 || { tail -5 $O/s2_$f.log; exit 1; }
  python3 tools/replay_breakdown.py $O/s2_$f/run_kernel_trace.csv --last 5 > $O/replay_s2_$f.txt || exit 1
  echo "S2_TAIL=$f"; head -14 $O/replay_s2_$f.txt; tail -1 $O/replay_s2_$f.txt
done
