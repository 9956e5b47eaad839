#!/bin/bash
# r4c: GPU tests of the new kernels (multi-view strip stem, strided layer2 tail) and the ABI-11
# Bottleneck tests, micro-benchmark, network A/Bs in one call, then r4a's attribution / training
# leg / fp16 runs.
set -o pipefail
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "stem" > $O/stem_tests.log 2>&1 || { tail -30 $O/stem_tests.log; exit 1; }
tail -2 $O/stem_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_bottleneck.py -q -x --timeout 120 --timeout-method thread > $O/bneck_tests.log 2>&1 || { tail -30 $O/bneck_tests.log; exit 1; }
tail -2 $O/bneck_tests.log
timeout -k 10 120 python -u tools/s2tail_micro.py > $O/s2tail_micro.txt 2>&1 || { cat $O/s2tail_micro.txt; exit 1; }
cat $O/s2tail_micro.txt
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"
for f in "S2_TAIL=1" "S2_TAIL=0 --plan-flag STEM_VIEWS=0 --plan-flag TILES_128X8=0" "S2_TAIL=0" "STEM_VIEWS=0" "TILES_128X8=0" "S2_TAIL=1"; do
  timeout -k 10 200 python -u bench.py $C --plan-flag $f > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['network_ms'])"
done
# layer2 tails with 2-row tiles (4 m-tiles per wave, three workgroups per CU) vs the default
if [ -f pose-unsupervised_amd/build/ab/libposeu_l2mt4.so ]; then
  timeout -k 10 120 python -u tools/chain_micro.py --only layer2 > $O/chain_default.txt 2>&1 || { cat $O/chain_default.txt; exit 1; }
  timeout -k 10 120 python -u tools/chain_micro.py --only layer2 --lib pose-unsupervised_amd/build/ab/libposeu_l2mt4.so > $O/chain_l2mt4.txt 2>&1 || { cat $O/chain_l2mt4.txt; exit 1; }
  cat $O/chain_default.txt $O/chain_l2mt4.txt
  for lib in default l2mt4 default l2mt4; do
    if [ $lib = default ]; then
      timeout -k 10 200 python -u bench.py $C > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
    else
      timeout -k 10 200 python -u tools/with_lib.py pose-unsupervised_amd/build/ab/libposeu_$lib.so bench.py $C > $O/ab.json 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
    fi
    python -c "import json;d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]);print('lib $lib',d['value'],d['network_ms'])"
  done
fi
bash tools/gpu_r4a.sh
