#!/bin/bash
# r4e: kernel / model GPU tests (split-precision head, 128x128 eight-wave tiles), precision
# attribution with the split head, speed A/Bs in one call (PRECISE_HEAD on/off; bf16 vs fp16),
# then the training side-stream hardware-queue probe (r4d).
set -o pipefail
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
grep "head vs fp64" $O/tests.log
timeout -k 10 300 python -u tools/precision_attribution.py 1200 > $O/attribution.json 2> $O/attribution.err || { tail -5 $O/attribution.err; exit 1; }
echo attribution done
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"
for f in "--precision bf16" "--precision bf16 --plan-flag PRECISE_HEAD=0" "--precision fp16" "--precision bf16" "--precision fp16" "--precision fp16 --plan-flag PRECISE_HEAD=0"; do
  timeout -k 10 200 python -u bench.py $C $f > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['network_ms'])"
done
bash tools/gpu_r4d.sh
