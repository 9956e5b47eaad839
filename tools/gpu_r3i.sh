set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "train or wgrad or adam or ddp" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > $O/train.json 2> $O/train.err || exit 1
python -c "import json;d=json.loads(open('$O/train.json').read().strip().splitlines()[-1]);print('train',d['value'],d['ms_per_step'])"
