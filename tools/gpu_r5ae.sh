#!/bin/bash
# streamed-tail timing ablations at HEAD (POSU_TS_ABLATE: 1 no MFMA, 2 no weight loads, 8 no
# residual loads / y stores, 16 no window DMA, 32 no y stores, 64 no residual loads; wrong results)
OUT=gpurun_out/r5ae
mkdir -p $OUT
for v in main a1 a2 a8 a32 a64 a16; do
  if [ $v = main ]; then L=""; else L="--lib pose-unsupervised_amd/build/ab6/libposeu_$v.so"; fi
  echo "== $v" >> $OUT/abl.txt
  timeout -k 10 120 python -u tools/chain_micro.py $L >> $OUT/abl.txt 2> $OUT/$v.err || exit $?
done
cat $OUT/abl.txt
