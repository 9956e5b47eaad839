#!/bin/bash
# Builds timing-ablation variants of libposeu.so (csrc/bottleneck3.hip with POSU_TAIL3_ABLATE=m,
# see the kernel) under pose-unsupervised_amd/build/abl/ -- run here, on the CPU; then on the
# GPU box:  python tools/tail3_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_tail3_m.so
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
make -s
mkdir -p build/abl
OTHERS=$(ls build/*.o | grep -v '/bottleneck3.o$')
for m in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPOSU_TAIL3_ABLATE=$m -c csrc/bottleneck3.hip -o build/abl/bottleneck3_$m.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/abl/bottleneck3_$m.o -o build/abl/libposeu_tail3_$m.so
done
