#!/bin/bash
# in-kernel weight warm-up (conv_igemm, POSU_IG_WARM): conv GPU tests, cold-cache tile timings
# with / without it, headline A/B alternating (control: the library built with POSU_IG_WARM=0)
OUT=gpurun_out/r5y
mkdir -p $OUT
export TMPDIR=/tmp
NOW=pose-unsupervised_amd/build/ab5/libposeu_nowarm.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_split.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
T="--tiles 20,15,39,23 --only l4,deconv1 --reps 10 --rounds 3 --flush --touch x"
timeout -k 10 200 python -u tools/tile_micro.py $T > $OUT/tiles_warm.txt 2>&1 || exit $?
timeout -k 10 200 python -u tools/with_lib.py $NOW tools/tile_micro.py $T > $OUT/tiles_nowarm.txt 2>&1 || exit $?
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --c1-steps 0 --steps 40"
for r in 1 2 3; do
  for v in nowarm warm; do
    if [ $v = warm ]; then L=""; else L="tools/with_lib.py $NOW"; fi
    timeout -k 10 200 python -u $L bench.py $Q > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || exit $?
    python - "$OUT/${v}_$r.json" "$v run $r" <<'PY' | tee -a $OUT/ab.txt
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], 'network_ms', d['network_ms'], 'ms_per_step', d['ms_per_step'])
PY
  done
done
grep -v amdgpu.ids $OUT/tiles_nowarm.txt; grep -v amdgpu.ids $OUT/tiles_warm.txt
