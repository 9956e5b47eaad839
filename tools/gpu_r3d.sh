set -o pipefail
# GPU call: training kernels' tests + un-profiled training step after the BN-finalize revert,
# then the round's profiles at HEAD (tools/profile_round.sh).
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_rounding_emulation.py tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread -k "train or rounding or tiles_bit" > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > $O/train.json 2> $O/train.err || exit 1
tail -c 500 $O/train.json
bash tools/profile_round.sh $O/prof $(cat COMMIT_STAMP 2>/dev/null || echo unknown)
for v in l2r8 ts1 ts2 ts8; do
  echo "== $v" >> $O/tail_var.txt
  timeout -k 10 120 python tools/tail_micro.py --lib pose-unsupervised_amd/build/abl/libposeu_$v.so >> $O/tail_var.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/tail_var.txt
