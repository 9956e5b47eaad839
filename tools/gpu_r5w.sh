#!/bin/bash
# weight prefetch (plan.PREFETCH, posu_prefetch): GPU tests, headline A/B alternating, and a
# kernel trace of the prefetching network (per-launch replay breakdown)
OUT=gpurun_out/r5w
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prefetch.py \
  tests/test_gpu_bench_config.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --c1-steps 0 --steps 40"
for r in 1 2; do
  for v in 0 1; do
    timeout -k 10 200 python -u bench.py $Q --plan-flag PREFETCH=$v > $OUT/pf${v}_$r.json 2> $OUT/pf${v}_$r.err || exit $?
    python - "$OUT/pf${v}_$r.json" "PREFETCH=$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])
PY
  done
done
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/infer" -o run -- \
  python3 bench.py $COMMON --steps 10 --warmup 3 > "$OUT/infer_bench.log" 2>&1 || exit $?
python3 tools/replay_breakdown.py "$OUT"/infer/run_kernel_trace.csv --last 5 > "$OUT/replay_breakdown.txt"
rm -f "$OUT"/infer/*.csv
cat $OUT/replay_breakdown.txt
