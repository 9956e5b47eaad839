#!/bin/bash
# training step at HEAD: kernel-trace --stats + breakdown (per stream), and its HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes) beside posu.roofline's training classes
OUT=gpurun_out/r5bo
COMMIT=${1:-unknown}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/train" -o run -- \
  python3 bench.py --mode train --steps 4 --warmup 1 > "$OUT/train_bench.log" 2>&1 || exit $?
python3 tools/train_breakdown.py "$OUT"/train/run_kernel_trace.csv --steps 2 > "$OUT/train_breakdown.txt"
cp "$OUT"/train/run_kernel_stats.csv "$OUT/kernel_stats_train_bench.csv"
rm -f "$OUT"/train/*.csv
echo traced
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/tf" -o run -- \
  python3 bench.py --mode train --steps 2 --warmup 1 > "$OUT/tf.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/tw" -o run -- \
  python3 bench.py --mode train --steps 2 --warmup 1 > "$OUT/tw.log" 2>&1 || exit $?
POSU_COMMIT=$COMMIT python3 tools/pmc_train_traffic.py "$OUT"/tf/run_counter_collection.csv \
  "$OUT"/tw/run_counter_collection.csv > "$OUT/pmc_traffic_train.txt"
rm -f "$OUT"/tf/*.csv "$OUT"/tw/*.csv
cat $OUT/train_breakdown.txt $OUT/pmc_traffic_train.txt
