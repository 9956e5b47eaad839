set -o pipefail
O=gpurun_out/r3ah
mkdir -p $O
timeout -k 10 600 python -u bench.py --layers 152 --size 384 --precision fp16 --groups 16 --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 > $O/r152.json 2> $O/r152.err || { tail -5 $O/r152.err; exit 1; }
python -c "import json;d=json.loads(open('$O/r152.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['network_ms'],d['roofline']['frac'])"
