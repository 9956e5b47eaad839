set -o pipefail
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bottleneck.py tests/test_gpu_bench_config.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 > $O/bench_on.json 2> $O/bench_on.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --plan-flag CHAINED_TAILS=0 > $O/bench_off.json 2> $O/bench_off.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 > $O/bench_on2.json 2> $O/bench_on2.err || exit 1
for f in bench_on bench_off bench_on2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['network_ms'],d['roofline']['frac'])"; done
