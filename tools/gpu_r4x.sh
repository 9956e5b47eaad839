#!/bin/bash
# r4x: layer1 Bottleneck with two barriers per row (conv1 of row y+2 beside conv2 of row y) vs the
# committed three-barrier kernel: GPU tests of the fused blocks, micro-benchmark, network A/B
set -o pipefail
O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bottleneck.py tests/test_gpu_rounding_emulation.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  echo "lib main"; timeout -k 10 120 python3 tools/bottleneck_micro.py | head -3 || exit 1
  echo "lib bnhead"; timeout -k 10 120 python3 tools/bottleneck_micro.py --lib pose-unsupervised_amd/build/r4x/libposeu_bnhead.so | head -3 || exit 1
done
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $O/tiles.json"
timeout -k 10 300 python3 bench.py $C > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
for r in 1 2; do
  for v in main bnhead; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/r4x/libposeu_$v.so"; fi
    timeout -k 10 200 python3 $L bench.py $C --steps 30 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['network_ms'])"
  done
done
bash tools/gpu_r4y.sh
echo done
