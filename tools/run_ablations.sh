#!/bin/bash
# GPU side of tools/bottleneck_ablations.sh: times every built variant (one process each).
for f in pose-unsupervised_amd/build/abl/libposeu_*.so; do
  echo "== $(basename $f .so)"
  timeout -k 10 60 python tools/bottleneck_micro.py --lib "$f" 2>&1 | grep -v amdgpu.ids || exit 1
done
