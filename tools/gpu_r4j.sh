#!/bin/bash
# r4j: packed-FMA epilogues (BN / residual as v_pk_fma_f32 / v_pk_add_f32) vs scalar loops:
# layer1 block micro, network A/B (same tile table), GPU kernel tests of the touched kernels;
# the chained strided tail (S2_CHAIN) A/B in the network; cibase = the committed conv kernel (the
# fused head in every 256x256 instance, scalar epilogue) with this tree's other kernels
set -o pipefail
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bottleneck.py tests/test_gpu_rounding_emulation.py -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in main nopk; do
  if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/r4j/libposeu_nopk.so"; fi
  echo "lib $v"; timeout -k 10 200 python3 tools/bottleneck_micro.py $L > $O/bneck_$v.txt 2>&1 || { tail -5 $O/bneck_$v.txt; exit 1; }
  grep -i "fused\|us" $O/bneck_$v.txt | head -6
done
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $O/tiles.json"
timeout -k 10 300 python3 bench.py $C > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
for r in 1 2; do
  for v in main nopk cibase; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/r4j/libposeu_$v.so"; fi
    timeout -k 10 200 python3 $L bench.py $C --steps 30 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['network_ms'])"
  done
  for f in 1 0; do
    timeout -k 10 200 python3 bench.py $C --steps 30 --plan-flag S2_CHAIN=$f > $O/chain_$f.json 2> $O/chain_$f.err || { tail -5 $O/chain_$f.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/chain_$f.json').read().strip().splitlines()[-1]);print('S2_CHAIN=$f', d['value'], d['network_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py $C --steps 10 --warmup 3 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/replay_breakdown.py $O/kt/run_kernel_trace.csv --last 5 > $O/replay.txt || exit 1
cat $O/replay.txt
echo done
