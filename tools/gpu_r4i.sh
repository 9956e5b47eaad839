#!/bin/bash
# r4i: the fused head as its own conv instance (no scratch in the 256x256 tiles): full GPU suite,
# network A/B against the committed conv kernel (same tile table), replay breakdown at HEAD
set -o pipefail
O=gpurun_out/r4i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $O/tiles.json"
timeout -k 10 300 python3 bench.py $C > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
for r in 1 2; do
  for v in main cibase; do
    if [ $v = main ]; then L=""; else L="tools/with_lib.py pose-unsupervised_amd/build/r4j/libposeu_cibase.so"; fi
    timeout -k 10 200 python3 $L bench.py $C --steps 30 > $O/ab_$v.json 2> $O/ab_$v.err || { tail -5 $O/ab_$v.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['network_ms'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- \
  python3 bench.py $C --steps 10 --warmup 3 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 tools/replay_breakdown.py $O/kt/run_kernel_trace.csv --last 5 > $O/replay.txt || exit 1
cat $O/replay.txt
echo done
