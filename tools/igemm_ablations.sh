#!/bin/bash
# Builds timing-ablation variants of libposeu.so (csrc/conv_igemm.hip's staggered loop with
# POSU_IG_ABLATE=m, see the kernel) under pose-unsupervised_amd/build/abl/libposeu_ig_m.so --
# run here, on the CPU; then on the GPU box:
#   python tools/tile_micro.py --tiles 23 --lib pose-unsupervised_amd/build/abl/libposeu_ig_m.so
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
make -s
mkdir -p build/abl
OTHERS=$(ls build/*.o | grep -v '/conv_igemm.o$')
for m in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPOSU_IG_ABLATE=$m -c csrc/conv_igemm.hip -o build/abl/conv_igemm_$m.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/abl/conv_igemm_$m.o -o build/abl/libposeu_ig_$m.so
done
