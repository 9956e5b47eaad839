#!/bin/bash
# r4x: layer1 Bottleneck with two barriers per row (conv1 of row y+2 beside conv2 of row y) vs the
# committed three-barrier kernel: GPU tests of the fused blocks, micro-benchmark, network A/B
set -o pipefail
O=gpurun_out/r4x; mkdir -p $O
for r in 1 2; do
  echo "lib main"; timeout -k 10 120 python3 tools/bottleneck_micro.py > $O/bm_main.txt 2>&1 || exit 1
  grep -E "^fused" $O/bm_main.txt
  echo "lib bnhead"; timeout -k 10 120 python3 tools/bottleneck_micro.py --lib pose-unsupervised_amd/build/r4x/libposeu_bnhead.so > $O/bm_head.txt 2>&1 || exit 1
  grep -E "^fused" $O/bm_head.txt
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
