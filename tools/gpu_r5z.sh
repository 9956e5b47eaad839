#!/bin/bash
# weight warm-up in the streamed / strided tails too, and its size threshold: tail GPU tests, then
# headline A/B alternating: no warm-up / >= 1 MiB tensors (default) / >= 64 KiB tensors
OUT=gpurun_out/r5z
mkdir -p $OUT
export TMPDIR=/tmp
AB=pose-unsupervised_amd/build/ab5
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bottleneck.py \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --steps 40"
for r in 1 2 3; do
  for v in nowarm w1m w64k; do
    if [ $v = w1m ]; then L=""; else L="tools/with_lib.py $AB/libposeu_$v.so"; fi
    timeout -k 10 200 python -u $L bench.py $Q > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'], 'configs1', d['configs1']['network_ms'])
PY
  done
done
