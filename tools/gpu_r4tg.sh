#!/bin/bash
# call r4tg: the training step captured in one hipGraph vs eager steps (bench --mode train);
# the in-context tuning stage (network with / without)
set -o pipefail
O=gpurun_out/r4tg; mkdir -p $O
for m in on off on; do
  timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 --train-graph $m > $O/train_$m.json 2> $O/train_$m.err || { tail -20 $O/train_$m.err; exit 1; }
  echo "$m $(python3 -c "import json; d=json.loads(open('$O/train_$m.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['loss'], d['config']['step_launch'])")" | tee -a $O/ab.txt
  grep -i "refused" $O/train_$m.err || true
done
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --steps 30"
for r in 1 2; do
  POSU_DUMP_TILES=$O/tiles_ctx$r.json timeout -k 10 300 python -u bench.py $COMMON > $O/ctx$r.json 2> $O/ctx$r.err || exit 1
  POSU_DUMP_TILES=$O/tiles_noctx$r.json timeout -k 10 300 python -u bench.py $COMMON --plan-flag REFINE_IN_CONTEXT=0 > $O/noctx$r.json 2> $O/noctx$r.err || exit 1
done
for f in ctx1 noctx1 ctx2 noctx2; do python3 -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('network_ms'), d['roofline']['frac'])"; done | tee $O/ctx_ab.txt
