#!/bin/bash
# Builds prefetch-depth variants of csrc/tail_stream.hip (POSU_TS_KD=k) as
# pose-unsupervised_amd/build/abl/libposeu_kd_k.so (run here; time on the box with tools/tail_micro.py --lib)
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
make -s
mkdir -p build/abl
OTHERS=$(ls build/*.o | grep -v '/tail_stream.o$')
for k in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPOSU_TS_KD=$k -c csrc/tail_stream.hip -o build/abl/tail_stream_kd$k.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/abl/tail_stream_kd$k.o -o build/abl/libposeu_kd_$k.so
done
