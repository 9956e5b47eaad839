#!/bin/bash
# call r4z: the BatchNorm finalize fused into the partial pass -- tests, micro A/B, training A/B
set -o pipefail
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for lib in main nofin; do
  L=pose-unsupervised_amd/lib/posu/libposeu.so; [ $lib = nofin ] && L=pose-unsupervised_amd/build/r4z/libposeu_nofin.so
  echo "lib $lib" >> $O/bn_micro.txt
  timeout -k 10 120 python -u tools/bn_micro.py --lib $L >> $O/bn_micro.txt 2>&1 || exit 1
done
cat $O/bn_micro.txt
for lib in main nofin main nofin; do
  L=pose-unsupervised_amd/lib/posu/libposeu.so; [ $lib = nofin ] && L=pose-unsupervised_amd/build/r4z/libposeu_nofin.so
  timeout -k 10 300 python -u tools/run_with_lib.py $L bench.py --mode train --steps 10 --warmup 3 > $O/train_$lib.json 2> $O/train_$lib.err || exit 1
  echo "$lib $(python3 -c "import json,sys; d=json.loads(open('$O/train_$lib.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('loss'))")" | tee -a $O/train_ab.txt
done
