#!/bin/bash
# call r4bn: BatchNorm pass unroll depth (backward partial pixels in flight, apply chunks in flight)
set -o pipefail
O=gpurun_out/r4bn; mkdir -p $O
for v in main u1_8 segu_8 both_8 u1_2; do
  L=pose-unsupervised_amd/lib/posu/libposeu.so; [ $v != main ] && L=pose-unsupervised_amd/build/r4bn/libposeu_$v.so
  echo "lib $v" >> $O/bn_micro.txt
  timeout -k 10 120 python -u tools/bn_micro.py --lib $L 2>&1 | grep -v amdgpu.ids >> $O/bn_micro.txt || exit 1
done
grep -E "lib|TOTAL" $O/bn_micro.txt
