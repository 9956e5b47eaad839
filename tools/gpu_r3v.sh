set -o pipefail
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_train_kernels.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
T="bench.py --mode train --steps 10 --warmup 3"
timeout -k 10 300 python -u $T > $O/train_new.json 2>/dev/null || exit 1
timeout -k 10 300 python -u tools/with_lib.py pose-unsupervised_amd/build/abl/libposeu_bnold.so $T > $O/train_old.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $T > $O/train_new2.json 2>/dev/null || exit 1
timeout -k 10 300 python -u tools/with_lib.py pose-unsupervised_amd/build/abl/libposeu_bnold.so $T > $O/train_old2.json 2>/dev/null || exit 1
for f in train_new train_old train_new2 train_old2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'])"; done
