#!/bin/bash
# Builds timing-ablation variants of libposeu.so (csrc/tail_stream.hip with POSU_TS_ABLATE=m, see
# the kernel) under pose-unsupervised_amd/build/abl/libposeu_ts_m.so -- run here, on the CPU; then
# on the GPU box: python tools/tail_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_ts_m.so
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
make -s
mkdir -p build/abl
OTHERS=$(ls build/*.o | grep -v '/tail_stream.o$')
for m in "$@"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPOSU_TS_ABLATE=$m -c csrc/tail_stream.hip -o build/abl/tail_stream_$m.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/abl/tail_stream_$m.o -o build/abl/libposeu_ts_$m.so
done
