#!/bin/bash
# Profiles for profiles/<round>/ (run on the GPU box from the repo root):
#     tools/profile_round.sh OUT_DIR COMMIT
# 1. one bench run that autotunes the conv tiles and saves them (OUT/tiles.json), so the
#    profiled runs below load the table and their traces hold graph replays, not tuning trials;
# 2. kernel-trace --stats of the inference bench (tuned, hipGraph) + the per-launch replay
#    breakdown (tools/replay_breakdown.py) + the trace-vs-HIP-event check;
# 3. two separate PMC passes (FETCH_SIZE, WRITE_SIZE; no other tracing) of the tuned network's
#    hipGraph replays (the launch sequence the bench times), reduced by tools/pmc_traffic.py
#    (FETCH doubled per the gfx950 correction), stamped with COMMIT;
# 4. kernel-trace --stats of the training bench.
set -euo pipefail
OUT=${1:-gpurun_out/profile}
COMMIT=${2:-unknown}
mkdir -p "$OUT"
export TMPDIR=/tmp
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $OUT/tiles.json"
timeout -k 10 300 python3 bench.py $COMMON > "$OUT/tune_bench.log" 2>&1
echo tuned
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/infer" -o run -- \
  python3 bench.py $COMMON --steps 10 --warmup 3 > "$OUT/infer_bench.log" 2>&1
python3 tools/replay_breakdown.py "$OUT"/infer/run_kernel_trace.csv --last 5 > "$OUT/replay_breakdown.txt"
python3 tools/roofline_check.py "$OUT"/infer/run_kernel_trace.csv "$OUT"/infer_bench.log > "$OUT/roofline_check.txt"
echo infer profiled
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- \
  python3 bench.py $COMMON --steps 2 --warmup 1 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- \
  python3 bench.py $COMMON --steps 2 --warmup 1 > "$OUT/pmc_write.log" 2>&1
POSU_COMMIT=$COMMIT python3 tools/pmc_traffic.py "$OUT"/pmc_fetch/run_counter_collection.csv \
  "$OUT"/pmc_write/run_counter_collection.csv > "$OUT/pmc_traffic_network.txt"
echo pmc done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train" -o run -- \
  python3 bench.py --mode train --steps 4 --warmup 1 > "$OUT/train_bench.log" 2>&1
echo profile all done
python3 tools/train_breakdown.py "$OUT"/train/run_kernel_trace.csv --steps 2 > "$OUT/train_breakdown.txt"
