set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 120 python tools/tail_micro.py --only layer2 > $O/tail_var.txt 2>&1 || exit 1
for v in ts8 ts32 ts64; do
  echo "== $v" >> $O/tail_var.txt
  timeout -k 10 120 python tools/tail_micro.py --only layer2 --lib pose-unsupervised_amd/build/abl/libposeu_$v.so >> $O/tail_var.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/tail_var.txt
