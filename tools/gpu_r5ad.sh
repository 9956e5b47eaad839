#!/bin/bash
# layer2 streamed-tail phase stagger (POSU_TS_STAGGER variants) vs the product library, alternating
OUT=gpurun_out/r5ad
mkdir -p $OUT
AB=pose-unsupervised_amd/build/ab5
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --c1-steps 0 --steps 40"
for r in 1 2; do
  for v in base s4b8 s4b3 s2b8 s8b8; do
    if [ $v = base ]; then L=""; else L="tools/with_lib.py $AB/libposeu_$v.so"; fi
    timeout -k 10 200 python -u $L bench.py $Q > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])
PY
  done
done
