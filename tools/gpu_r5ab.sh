#!/bin/bash
# the two-K-group tile 39 among the candidates or not, with the weight warm-up in place: headline
# A/B in separate processes, alternating, tile tables dumped
OUT=gpurun_out/r5ab
mkdir -p $OUT
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --steps 40"
for r in 1 2 3; do
  for v in 1 0; do
    POSU_DUMP_TILES=$OUT/tiles_ks${v}_$r.json timeout -k 10 200 python -u bench.py $Q --plan-flag TILES_KSPLIT=$v > $OUT/ks${v}_$r.json 2> $OUT/ks${v}_$r.err || exit $?
    python - "$OUT/ks${v}_$r.json" "KSPLIT=$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'], 'configs1', d['configs1']['network_ms'])
PY
  done
done
python - $OUT <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + '/tiles_*.json')):
    t = json.load(open(f))
    print(f.split('/')[-1], ' '.join(str(r[1]) for r in t))
PY
