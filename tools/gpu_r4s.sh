#!/bin/bash
# r4s: strided tail weight-stream depth (POSU_S2_KD 1 / 2 / 4 = default), plain and chained
set -o pipefail
O=gpurun_out/r4s; mkdir -p $O
for r in 1 2; do
  echo "lib kd4 (default)"; timeout -k 10 120 python3 tools/s2tail_micro.py || exit 1
  for v in kd1 kd2; do
    echo "lib $v"; timeout -k 10 120 python3 tools/with_lib.py pose-unsupervised_amd/build/r4s/libposeu_$v.so tools/s2tail_micro.py || exit 1
  done
done
echo done
