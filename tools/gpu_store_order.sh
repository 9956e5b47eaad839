#!/bin/bash
# GPU side of tools/store_order.sh: the lost-store / race check of every variant, one process each.
set -o pipefail
out=${1:-gpurun_out/store}
mkdir -p $out
timeout -k 10 150 python -u tools/store_check.py --reps 2 > $out/main.log 2>&1 || exit $?
for v in r0e0 r1e0 r0e1 r1e1 old old_g old_w0; do
  timeout -k 10 90 python -u tools/store_check.py --only tail3 --reps 3 \
    --lib pose-unsupervised_amd/build/var/libposeu_$v.so > $out/$v.log 2>&1 || exit $?
done
