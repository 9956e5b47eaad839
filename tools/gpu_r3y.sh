set -o pipefail
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 100 python tools/head_micro.py > $O/head.txt 2>&1 || exit 1
timeout -k 10 100 python tools/head_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_headold.so >> $O/head.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/head.txt
B="bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0"
timeout -k 10 300 python -u $B > $O/b_new.json 2>/dev/null || exit 1
timeout -k 10 300 python -u tools/with_lib.py pose-unsupervised_amd/build/abl/libposeu_headold.so $B > $O/b_old.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $B > $O/b_new2.json 2>/dev/null || exit 1
timeout -k 10 300 python -u tools/with_lib.py pose-unsupervised_amd/build/abl/libposeu_headold.so $B > $O/b_old2.json 2>/dev/null || exit 1
for f in b_new b_old b_new2 b_old2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['network_ms'])"; done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
tail -3 $O/gputests.log; exit $rc
