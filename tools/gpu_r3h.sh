set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
for v in wgs2 wgs3; do
  echo "== $v" >> $O/wg.txt
  timeout -k 10 120 python tools/wgrad_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_$v.so >> $O/wg.txt 2>&1 || exit 1
done
echo "== wgs4 (product)" >> $O/wg.txt
timeout -k 10 120 python tools/wgrad_micro.py >> $O/wg.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/wg.txt
