set -o pipefail
O=gpurun_out/r3ae
mkdir -p $O
# the training tests with the fused BN statistics switched on (train_plan.FUSED_BN_STATS)
timeout -k 10 400 python -u -c "
import sys; sys.path[:0] = ['pose-unsupervised_amd/lib', '.']
import posu.train_plan as t; t.FUSED_BN_STATS = True
import pytest; sys.exit(pytest.main(['tests/test_gpu_train_kernels.py', 'tests/test_gpu_train.py', '-q', '-x', '--timeout', '120', '--timeout-method', 'thread']))
" > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
T="bench.py --mode train --steps 10 --warmup 3"
timeout -k 10 300 python -u $T --plan-flag FUSED_BN_STATS=1 > $O/t_on.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $T --plan-flag FUSED_BN_STATS=0 > $O/t_off.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $T --plan-flag FUSED_BN_STATS=1 > $O/t_on2.json 2>/dev/null || exit 1
timeout -k 10 300 python -u $T --plan-flag FUSED_BN_STATS=0 > $O/t_off2.json 2>/dev/null || exit 1
for f in t_on t_off t_on2 t_off2; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['ms_per_step'],d['loss'])"; done
