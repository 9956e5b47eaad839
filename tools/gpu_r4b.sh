#!/bin/bash
# r4b: GPU tests of the fused Bottleneck kernels (ABI 11, the strided layer2 tail), its micro-benchmark
# and the network A/B (S2_TAIL on / off in one call), then r4a's attribution / training-leg / fp16 runs.
set -o pipefail
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bottleneck.py -q -x --timeout 120 --timeout-method thread > $O/bneck_tests.log 2>&1 || { tail -30 $O/bneck_tests.log; exit 1; }
tail -2 $O/bneck_tests.log
timeout -k 10 120 python -u tools/s2tail_micro.py > $O/s2tail_micro.txt 2>&1 || { cat $O/s2tail_micro.txt; exit 1; }
cat $O/s2tail_micro.txt
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0"
for f in 1 0 1 0; do
  timeout -k 10 200 python -u bench.py $C --plan-flag S2_TAIL=$f > $O/ab_s2_$f.json 2> $O/ab_s2_$f.err || exit 1
  python -c "import json;d=json.loads(open('$O/ab_s2_$f.json').read().strip().splitlines()[-1]);print('S2_TAIL=$f',d['value'],d['network_ms'])"
done
bash tools/gpu_r4a.sh
