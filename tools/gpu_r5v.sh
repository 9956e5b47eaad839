#!/bin/bash
# cold-cache tile timings with the weights / the input re-read after the eviction: which fetch
# makes layer4's in-graph launches slower than the warm micro
OUT=gpurun_out/r5v
mkdir -p $OUT
T="--tiles 20,15,39,23 --only l4,deconv1 --reps 10 --rounds 3"
for m in warm cold w x wx; do
  case $m in warm) A="";; cold) A="--flush";; *) A="--flush --touch $m";; esac
  echo "== $m" >> $OUT/tiles.txt
  timeout -k 10 200 python -u tools/tile_micro.py $T $A >> $OUT/tiles.txt 2>&1 || exit $?
done
cat $OUT/tiles.txt
