#!/bin/bash
# A/B of the two-K-group tile in one call (headline only, 40 steps, alternating), then the bf16 profile set
OUT=gpurun_out/r5j
mkdir -p $OUT
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --steps 40"
for r in 1 2; do
  for f in 1 0; do
    timeout -k 10 200 python -u bench.py $Q --plan-flag TILES_KSPLIT=$f > $OUT/ab_ks${f}_$r.json 2> $OUT/ab_ks${f}_$r.err || exit $?
    python -c "import json,sys; d=json.loads(open('$OUT/ab_ks${f}_$r.json').read().strip().splitlines()[-1]); print('KS=$f run $r network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])" | tee -a $OUT/ab.txt
  done
done
tools/profile_round.sh $OUT/prof $(cat COMMIT_STAMP) > $OUT/profile.log 2>&1
rc=$?
tail -2 $OUT/profile.log
exit $rc
