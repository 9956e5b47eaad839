set -o pipefail
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 120 python tools/chain_micro.py --only layer2 > $O/chain.txt 2>&1 || exit 1
for v in w1k4n2 w1k2n2; do
  echo "== $v" >> $O/chain.txt
  timeout -k 10 120 python tools/chain_micro.py --only layer2 --lib pose-unsupervised_amd/build/abl/libposeu_$v.so >> $O/chain.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/chain.txt
