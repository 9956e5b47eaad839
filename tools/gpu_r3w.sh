set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 150 python tools/tile_micro.py --tiles 23,31 > $O/abl.txt 2>&1 || exit 1
echo "== ig_16 (no epilogue)" >> $O/abl.txt
timeout -k 10 150 python tools/tile_micro.py --tiles 23,31 --lib pose-unsupervised_amd/build/abl/libposeu_ig_16.so >> $O/abl.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/abl.txt
