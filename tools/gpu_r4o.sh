#!/bin/bash
# r4o: the default bench line at this tree, then the autotuner stability check (tools/gpu_r4n.sh)
set -o pipefail
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
grep "^bench:" $O/bench_default.err | head -5
tail -c 1200 $O/bench_default.json
bash tools/gpu_r4n.sh
