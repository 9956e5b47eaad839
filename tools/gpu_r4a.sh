#!/bin/bash
# r4a: precision attribution (bf16 / fp16 per stage on peaked heatmaps), the training leg's
# 21.6 vs 23.98 ms question (the default line's legs toggled, tile tables dumped), fp16 line.
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O


timeout -k 10 240 python -u tools/precision_attribution.py 1200 > $O/attribution.json 2> $O/attribution.err || exit 1
echo attribution done
C="--no-cpu-baseline --no-mpjpe"
POSU_DUMP_TILES=$O/tiles_t1.json timeout -k 10 200 python -u bench.py --mode train --steps 10 --warmup 3 > $O/t1.json 2> $O/t1.err || exit 1
POSU_DUMP_TILES=$O/tiles_full.json timeout -k 10 300 python -u bench.py $C > $O/full.json 2> $O/full.err || exit 1
POSU_DUMP_TILES=$O/tiles_nofp32.json timeout -k 10 300 python -u bench.py $C --fp32-steps 0 > $O/nofp32.json 2> $O/nofp32.err || exit 1
POSU_DUMP_TILES=$O/tiles_noc1.json timeout -k 10 300 python -u bench.py $C --c1-steps 0 > $O/noc1.json 2> $O/noc1.err || exit 1
POSU_DUMP_TILES=$O/tiles_t2.json timeout -k 10 200 python -u bench.py --mode train --steps 10 --warmup 3 > $O/t2.json 2> $O/t2.err || exit 1
python - <<'PY'
import json
O = 'gpurun_out/r4a'
for n in ('t1', 'full', 'nofp32', 'noc1', 't2'):
    d = json.loads(open('%s/%s.json' % (O, n)).read().strip().splitlines()[-1])
    tm = d if 'train_mode' not in d else d['train_mode']
    print(n, 'train ms', tm and tm['ms_per_step'], 'infer', d.get('value'), d.get('network_ms'))
PY
timeout -k 10 300 python -u bench.py --precision fp16 --train-steps 0 --no-cpu-baseline > $O/fp16.json 2> $O/fp16.err || exit 1
tail -c 400 $O/fp16.json
