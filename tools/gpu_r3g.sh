set -o pipefail
# GPU call: full GPU suite, then the default bench line with and without the layer2 streamed tail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -4 $O/gputests.log; [ $rc -le 1 ] || exit $rc
Q="--no-cpu-baseline --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --no-mpjpe"
timeout -k 10 300 python -u bench.py $Q --tune-file $O/tiles.json > $O/b_on1.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py $Q --tune-file $O/tiles.json --plan-flag STREAMED_LAYER2_TAIL=0 > $O/b_off1.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py $Q --tune-file $O/tiles.json > $O/b_on2.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py $Q --tune-file $O/tiles.json --plan-flag STREAMED_LAYER2_TAIL=0 > $O/b_off2.json 2>/dev/null || exit 1
for f in on1 off1 on2 off2; do python -c "import json,sys;d=json.loads(open('$O/b_$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['network_ms'])"; done
