#!/bin/bash
# GPU side of tools/tail_ablations.sh: the micro-benchmark of every built variant, one process each.
out=${1:-gpurun_out/tail_abl}
mkdir -p $out
timeout -k 10 90 python -u tools/tail_micro.py > $out/base.log 2>&1 || exit $?
for f in pose-unsupervised_amd/build/abl/libposeu_ts_*.so; do
  m=$(basename $f .so)
  timeout -k 10 90 python -u tools/tail_micro.py --lib $f > $out/$m.log 2>&1 || exit $?
done
