#!/bin/bash
# r4u: layer2's chained tail with 4 m-tiles per wave and a deeper weight stream (kD 4, two pixel
# fragment sets; at 3 and at 2 workgroups per CU) against the default (8 m-tiles, kD 1, one set)
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
for r in 1 2; do
  echo "lib main"; timeout -k 10 120 python3 tools/chain_micro.py --only layer2 || exit 1
  for v in l2mt4kd2 l2mt4kd4 l2mt4kd4o2; do
    echo "lib $v"; timeout -k 10 120 python3 tools/chain_micro.py --only layer2 --lib pose-unsupervised_amd/build/r4u/libposeu_$v.so || exit 1
  done
done
echo done
