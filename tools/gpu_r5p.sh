#!/bin/bash
# A/B of layer3's 4-row tail tiles: headline (batch 128) and configs1 (batch 64), alternating libs
OUT=gpurun_out/r5p
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bottleneck.py -k "layer3_tail or chained_tail" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -le 1 ] || exit $rc
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --steps 40 --c1-steps 40"
for r in 1 2; do
  for v in l3r4 l3r8; do
    timeout -k 10 200 python -u tools/with_lib.py pose-unsupervised_amd/build/ab5/libposeu_$v.so bench.py $Q > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'configs1 ms', d['configs1']['network_ms'], 'frac', d['configs1']['roofline']['frac'])
PY
  done
done
