#!/bin/bash
# streamed tails: y stores trickled from LDS during the next conv1 (POSU_TS_TRICKLE)
# tail micro (bit-identity checked) and the headline network, alternating
OUT=gpurun_out/r5bb
mkdir -p $OUT
VS="main trickle"
for v in $VS; do
  if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/ab12/libposeu_$v.so"; fi
  echo "== $v" >> $OUT/micro.txt
  timeout -k 10 120 python -u tools/chain_micro.py $L >> $OUT/micro.txt 2> $OUT/micro_$v.err || exit $?
done
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --c1-steps 0 --steps 40"
for r in 1 2; do
  for v in $VS; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/ab12/libposeu_$v.so"; fi
    timeout -k 10 200 python -u $L bench.py $Q > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])
PY
  done
done
cat $OUT/micro.txt
