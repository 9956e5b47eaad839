set -o pipefail
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 100 python tools/head_micro.py > $O/head.txt 2>&1 || exit 1
for v in headold ig_16 ig_32; do timeout -k 10 100 python tools/head_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_$v.so >> $O/head.txt 2>&1 || exit 1; done
timeout -k 10 100 python tools/head_micro.py >> $O/head.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/head.txt
