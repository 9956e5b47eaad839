#!/bin/bash
# r4n: autotuner stability -- three independent tunings (two-pass, per-tile min), their tile
# tables with the measured per-tile times, and each table's in-graph network time
set -o pipefail
O=gpurun_out/r4n; mkdir -p $O
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"
for r in 1 2 3; do
  POSU_DUMP_TILES=$O/dump_$r.json timeout -k 10 300 python3 bench.py $C --tune-file $O/tiles_$r.json --steps 30 > $O/tune_$r.json 2> $O/tune_$r.err || { tail -5 $O/tune_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/tune_$r.json').read().strip().splitlines()[-1]);print('tuning $r', d['value'], d['network_ms'])"
done
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py $C --tune-file $O/tiles_$r.json --steps 30 > $O/run_$r.json 2> $O/run_$r.err || { tail -5 $O/run_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/run_$r.json').read().strip().splitlines()[-1]);print('table $r', d['value'], d['network_ms'])"
done
python3 - <<'PY'
import json
d = [json.load(open('gpurun_out/r4n/dump_%d.json' % r)) for r in (1, 2, 3)]
for rows in zip(*d):
    k = rows[0][0]
    tiles = [r[1] for r in rows]
    print(('SAME ' if len(set(tiles)) == 1 else 'DIFF ') + k[:70], tiles)
PY
echo done
