#!/bin/bash
# Builds timing-ablation variants of libposeu.so (csrc/bottleneck.hip with POSU_BNECK_ABLATE=m,
# see the kernel) under pose-unsupervised_amd/build/abl/ -- run here, on the CPU; then on the
# GPU box:  for m in ...; do python tools/bottleneck_micro.py --lib .../libposeu_$m.so; done
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
make -s
mkdir -p build/abl
OTHERS=$(ls build/*.o | grep -v '/bottleneck.o$')
# an argument m builds POSU_BNECK_ABLATE=m; "m:e" also sets POSU_BNECK_EXP=e (experiments)
for arg in "$@"; do
  m=${arg%%:*}; e=0; [[ $arg == *:* ]] && e=${arg#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPOSU_BNECK_ABLATE=$m -DPOSU_BNECK_EXP=$e -c csrc/bottleneck.hip -o build/abl/bottleneck_${m}_$e.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/abl/bottleneck_${m}_$e.o -o build/abl/libposeu_${m}_$e.so
done
