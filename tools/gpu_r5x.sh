#!/bin/bash
# weight prefetch variants (workgroups per prefetch, first prefetched layer) against none,
# alternating, headline only; then the kernel trace of the default plan
OUT=gpurun_out/r5x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prefetch.py \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --c1-steps 0 --steps 40"
for r in 1 2; do
  for v in off wg32 wg8 wg32l4 wg1024l4; do
    case $v in
      off) F="--plan-flag PREFETCH=0";;
      wg32) F="--plan-flag PREFETCH_WORKGROUPS=32";;
      wg8) F="--plan-flag PREFETCH_WORKGROUPS=8";;
      wg32l4) F="--plan-flag PREFETCH_WORKGROUPS=32 --plan-flag PREFETCH_FROM_LAYER=3";;
      wg1024l4) F="--plan-flag PREFETCH_WORKGROUPS=1024 --plan-flag PREFETCH_FROM_LAYER=3";;
    esac
    timeout -k 10 200 python -u bench.py $Q $F > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])
PY
  done
done
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/infer$v" -o run -- \
    python3 bench.py $COMMON --steps 10 --warmup 3 --plan-flag PREFETCH=$v > "$OUT/infer_bench$v.log" 2>&1 || exit $?
  python3 tools/replay_breakdown.py "$OUT"/infer$v/run_kernel_trace.csv --last 5 > "$OUT/replay_breakdown$v.txt"
done
paste $OUT/replay_breakdown0.txt $OUT/replay_breakdown1.txt | cut -c1-200
