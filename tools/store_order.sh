#!/bin/bash
# Builds the store-ordering experiment variants of libposeu.so (csrc/bottleneck3.hip with
# POSU_TAIL3_RAWSTORE r and POSU_TAIL3_EARLYDMA e, see the kernel) under
# pose-unsupervised_amd/build/var/libposeu_r<r>e<e>.so -- run here, on the CPU; then on the GPU
# box:  python tools/store_check.py --lib pose-unsupervised_amd/build/var/libposeu_r1e0.so
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
make -s
mkdir -p build/var
OTHERS=$(ls build/*.o | grep -v '/bottleneck3.o$')
for r in 0 1; do
  for e in 0 1; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DPOSU_TAIL3_RAWSTORE=$r -DPOSU_TAIL3_EARLYDMA=$e \
      -c csrc/bottleneck3.hip -o build/var/bottleneck3_r${r}e${e}.o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/var/bottleneck3_r${r}e${e}.o \
      -o build/var/libposeu_r${r}e${e}.so
  done
done
# the round-2 kernel that failed its bit-exactness test (commit 74f82b6: one stage loop, the next
# chunk's DMA before the y stores and vmcnt(8) at the chunk's first stage, raw-buffer y stores),
# and that kernel with ONE change each: plain global y stores (old_g) / vmcnt(0) there (old_w0)
cd ..
git show 74f82b6:pose-unsupervised_amd/csrc/bottleneck3.hip > pose-unsupervised_amd/build/var/b3_old.hip
python3 - <<'PY'
src = open('pose-unsupervised_amd/build/var/b3_old.hip').read()
raw = ('__builtin_amdgcn_raw_buffer_store_b128((__attribute__((ext_vector_type(4))) unsigned){u.x, u.y, u.z, u.w},\n'
       '                                                   yrs, lane_off, row_off(i, nc, jp), 0);')
assert raw in src
g = src.replace(raw, '*reinterpret_cast<uint4*>(static_cast<char*>(g.y) + static_cast<size_t>(lane_off + row_off(i, nc, jp))) = u;')
w8 = 'if (u > kConv2Stages && ((u - kConv2Stages) & 3) == 0) vm_wait<8>();'
assert w8 in src
w0 = src.replace(w8, 'if (u > kConv2Stages && ((u - kConv2Stages) & 3) == 0) vm_wait<0>();')
open('pose-unsupervised_amd/build/var/b3_old_g.hip', 'w').write(g)
open('pose-unsupervised_amd/build/var/b3_old_w0.hip', 'w').write(w0)
PY
cd pose-unsupervised_amd
for v in old old_g old_w0; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc -c build/var/b3_$v.hip -o build/var/b3_$v.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/var/b3_$v.o -o build/var/libposeu_$v.so
done
