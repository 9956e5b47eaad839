set -o pipefail
O=gpurun_out/r3ag
mkdir -p $O
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > $O/t1.json 2>/dev/null || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --c1-steps 0 --peaked-steps 0 > $O/d1.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > $O/t2.json 2>/dev/null || exit 1
python -c "import json;[print(f,json.loads(open('$O/'+f).read().strip().splitlines()[-1])['ms_per_step']) for f in ('t1.json','t2.json')]"
python -c "import json;d=json.loads(open('$O/d1.json').read().strip().splitlines()[-1]);print('default-line train leg',d['train_mode']['ms_per_step'],'infer',d['value'])"
