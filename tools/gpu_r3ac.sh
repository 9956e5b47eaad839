set -o pipefail
O=gpurun_out/r3ac
mkdir -p $O
B="bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0"
timeout -k 10 300 python -u $B --overlap-front > $O/b_ov.json 2> $O/b_ov.err || { tail -5 $O/b_ov.err; exit 1; }
timeout -k 10 300 python -u $B > $O/b_pipe.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $B --overlap-front > $O/b_ov2.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $B > $O/b_pipe2.json 2>/dev/null || exit 1
for f in b_ov b_pipe b_ov2 b_pipe2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['network_ms'],d['decode_geometry_ms'])"; done
