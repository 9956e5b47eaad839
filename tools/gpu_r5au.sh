#!/bin/bash
# training step: main stream high priority (--train-stream high) x weight-gradient blocks 128 / 192 / 256
OUT=gpurun_out/r5au
mkdir -p $OUT
for r in 1 2; do
  for v in main_n main_h b192_h b256_h; do
    case $v in
      main_n) L=""; F="";;
      main_h) L=""; F="--train-stream high";;
      b192_h) L="tools/with_lib.py pose-unsupervised_amd/build/ab9/libposeu_b192.so"; F="--train-stream high";;
      b256_h) L="tools/with_lib.py pose-unsupervised_amd/build/ab9/libposeu_b256.so"; F="--train-stream high";;
    esac
    timeout -k 10 300 python -u $L bench.py --mode train --steps 20 --warmup 3 $F > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'ms_per_step', d['ms_per_step'], 'value', d['value'])
PY
  done
done
