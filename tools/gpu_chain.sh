set -o pipefail
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 120 python tools/chain_micro.py > $O/chain.txt 2>&1 || exit 1
for v in k4n1 k2n2 k4n2 k1n1; do
  echo "== $v" >> $O/chain.txt
  timeout -k 10 120 python tools/chain_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_$v.so >> $O/chain.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/chain.txt
