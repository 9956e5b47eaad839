#!/bin/bash
# tuner stability with the in-context per-launch refinement: three independent tunings (headline
# only), their tile tables and network times
OUT=gpurun_out/r5k
mkdir -p $OUT
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --steps 40"
for r in 1 2 3; do
  POSU_DUMP_TILES=$OUT/tiles_$r.json timeout -k 10 200 python -u bench.py $Q > $OUT/bench_$r.json 2> $OUT/bench_$r.err || exit $?
  python -c "import json; d=json.loads(open('$OUT/bench_$r.json').read().strip().splitlines()[-1]); print('run $r network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])" | tee -a $OUT/summary.txt
done
python - <<'PY' | tee -a $OUT/summary.txt
import json
ts = [{e[0]: (e[1], e[3]) for e in json.load(open('gpurun_out/r5k/tiles_%d.json' % r))} for r in (1, 2, 3)]
for k in ts[0]:
    ch = [t[k][0] if k in t else None for t in ts]
    print(('SAME ' if len(set(ch)) == 1 else 'DIFF ') + k[:90], ch, ts[0][k][1])
PY
