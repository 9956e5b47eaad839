#!/bin/bash
# weight-gradient blocks per launch (POSU_WG_BLOCKS 128 default vs 96 / 192) at the round-end step
OUT=gpurun_out/r5bp
mkdir -p $OUT
for r in 1 2; do
  for v in main wgb96 wgb192; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/ab16/libposeu_$v.so"; fi
    timeout -k 10 300 python -u $L bench.py --mode train --steps 20 --warmup 3 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'], 'loss', d['loss'])
PY
  done
done
