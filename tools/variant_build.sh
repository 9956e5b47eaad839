#!/bin/bash
# Builds a variant of libposeu.so with one source file compiled under extra defines:
#     tools/variant_build.sh NAME SOURCE.hip -DFOO=1 [-DBAR=2 ...]
#     tools/variant_build.sh NAME ALL -DFOO=1      (every source file under the defines)
# -> pose-unsupervised_amd/build/abl/libposeu_NAME.so (run here, on the CPU; the GPU tools take
# it with --lib).  Timing ablations and tile experiments only; never the product library.
set -euo pipefail
cd "$(dirname "$0")/../pose-unsupervised_amd"
name=$1; src=$2; shift 2
make -s
mkdir -p build/${POSU_AB_DIR:-abl}
if [ "$src" = ALL ]; then
  objs=""
  for f in csrc/*.hip; do
    b=$(basename "$f" .hip)
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c "$f" -o build/${POSU_AB_DIR:-abl}/${b}_$name.o
    objs="$objs build/${POSU_AB_DIR:-abl}/${b}_$name.o"
  done
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $objs -o build/${POSU_AB_DIR:-abl}/libposeu_$name.so
  echo built build/${POSU_AB_DIR:-abl}/libposeu_$name.so
  exit 0
fi
base=$(basename "$src" .hip)
OTHERS=$(ls build/*.o | grep -v "/$base.o\$")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c csrc/$base.hip -o build/${POSU_AB_DIR:-abl}/${base}_$name.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -shared $OTHERS build/${POSU_AB_DIR:-abl}/${base}_$name.o -o build/${POSU_AB_DIR:-abl}/libposeu_$name.so
echo built build/${POSU_AB_DIR:-abl}/libposeu_$name.so
