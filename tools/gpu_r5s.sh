#!/bin/bash
# spill-free streamed tails (buffer-descriptor x / y / t1n): tests, then A/B against the previous
# build (64-bit addresses, layer3 chained tail spilling 34 VGPRs), headline only, alternating
OUT=gpurun_out/r5s
mkdir -p $OUT
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --c1-steps 0 --steps 40"
for r in 1 2; do
  for v in base kd4 kd4nb2 kd2nb2; do
    timeout -k 10 200 python -u tools/with_lib.py pose-unsupervised_amd/build/ab5/libposeu_$v.so bench.py $Q > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])
PY
  done
done
