set -o pipefail
O=gpurun_out/r3ab
mkdir -p $O
B="bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0"
timeout -k 10 300 python -u $B > $O/b_pipe.json 2> $O/b_pipe.err || exit 1
timeout -k 10 300 python -u $B --serial-geo > $O/b_serial.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $B > $O/b_pipe2.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $B --serial-geo > $O/b_serial2.json 2>/dev/null || exit 1
for f in b_pipe b_serial b_pipe2 b_serial2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['network_ms'],d['decode_geometry_ms'],d['roofline']['frac'])"; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_config.py -q -x --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; exit $rc
