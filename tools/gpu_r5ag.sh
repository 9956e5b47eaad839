#!/bin/bash
# BN backward partial pass: threads per block (POSU_BN_BS1) A/B at the training shapes
OUT=gpurun_out/r5ag
mkdir -p $OUT
for r in 1 2; do
for v in main bs512 bs1024 bs1024u8; do
  if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/ab6/libposeu_$v.so"; fi
  echo "== $v run $r" >> $OUT/bn.txt
  timeout -k 10 120 python -u tools/bn_micro.py $L >> $OUT/bn.txt 2> $OUT/$v.err || exit $?
done
done
cat $OUT/bn.txt
