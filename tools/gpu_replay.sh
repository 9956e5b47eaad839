# tuned-table replay breakdown of the inference network at HEAD: gpurun_out/<name>/replay_breakdown.txt
set -o pipefail
OUT=gpurun_out/${1:-replay}
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --tune-file $OUT/tiles.json"
timeout -k 10 300 python3 bench.py $COMMON > "$OUT/tune_bench.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/infer" -o run -- \
  python3 bench.py $COMMON --steps 10 --warmup 3 > "$OUT/infer_bench.log" 2>&1 || exit 1
python3 tools/replay_breakdown.py "$OUT"/infer/run_kernel_trace.csv --last 5 > "$OUT/replay_breakdown.txt"
rm -f "$OUT"/infer/run_kernel_trace.csv
cat "$OUT/replay_breakdown.txt"
