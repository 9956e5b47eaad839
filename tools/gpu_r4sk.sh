#!/bin/bash
# call r4sk: split-K conv -- parity tests, micro-benchmark, tuned network with / without split-K
set -o pipefail
O=gpurun_out/r4sk; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "splitk" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/splitk_micro.py > $O/micro.txt 2>&1 || { cat $O/micro.txt; exit 1; }
cat $O/micro.txt
COMMON="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"
POSU_DUMP_TILES=$O/tiles_split.json timeout -k 10 300 python -u bench.py $COMMON --steps 30 > $O/bench_split.json 2> $O/bench_split.err || exit 1
timeout -k 10 300 python -u bench.py $COMMON --steps 30 --plan-flag SPLIT_K=0 > $O/bench_nosplit.json 2> $O/bench_nosplit.err || exit 1
timeout -k 10 300 python -u bench.py $COMMON --steps 30 > $O/bench_split2.json 2> $O/bench_split2.err || exit 1
for f in split nosplit split2; do python3 -c "import json; d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('network_ms'), d['roofline']['frac'])"; done
