#!/bin/bash
OUT=gpurun_out/${1:-r5l}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_bottleneck.py \
  -k "layer3_tail or layer2_bottleneck or chained_tail or refuses" tests/test_gpu_bench_config.py::test_r152_384_fp16_pipeline_matches_the_oracle_chain \
  > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|FAIL|Error|R152|layer3 tail" $OUT/tests.log | tail -30
[ $rc -le 1 ] || exit $rc
Q="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --control-steps 0 --steps 5"
for f in 1 0; do
  timeout -k 10 300 python -u bench.py $Q --plan-flag TAIL_W24=$f > $OUT/c4_w24_$f.json 2> $OUT/c4_w24_$f.err || exit $?
  python -c "import json; d=json.loads(open('$OUT/c4_w24_$f.json').read().strip().splitlines()[-1])['configs4']; print('TAIL_W24=$f', d['value'], d['network_ms'], d['roofline']['frac'])" | tee -a $OUT/ab.txt
done
