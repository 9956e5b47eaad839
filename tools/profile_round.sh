#!/bin/bash
# Profiles for profiles/<round>/ (run on the GPU box from the repo root):
#   kernel-trace --stats of the inference bench and of the training bench, and the two
#   separate PMC passes (FETCH_SIZE, WRITE_SIZE) of the inference network, reduced by
#   tools/pmc_traffic.py (FETCH doubled per the gfx950 correction).
set -euo pipefail
OUT=${1:-gpurun_out/profile}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/infer" -o run -- \
  python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/infer_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train" -o run -- \
  python3 bench.py --mode train --steps 4 --warmup 1 > "$OUT/train_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT"/pmc_fetch/run_counter_collection.csv "$OUT"/pmc_write/run_counter_collection.csv \
  > "$OUT/pmc_traffic_network.txt"
echo profile done
python3 tools/roofline_check.py "$OUT"/infer/run_kernel_trace.csv "$OUT"/infer_bench.log > "$OUT/roofline_check.txt"
timeout -k 10 400 python3 tools/bench_layers.py --autotune > "$OUT/layers_autotuned.txt" 2>&1
echo profile all done
