set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 400 python -u -m pytest tests/test_gpu_train_kernels.py tests/test_gpu_train.py tests/test_gpu_rounding_emulation.py -q -s --timeout 120 --timeout-method thread > gpurun_out/r3b/trk.log 2>&1
rc=$?; tail -30 gpurun_out/r3b/trk.log; [ $rc -le 1 ] || exit $rc
for m in 0 1 2 4 6 8; do
  echo "== ig_$m" >> gpurun_out/r3b/abl.txt
  timeout -k 10 120 python tools/tile_micro.py --tiles 23 --reps 10 --rounds 3 --lib pose-unsupervised_amd/build/abl/libposeu_ig_$m.so >> gpurun_out/r3b/abl.txt 2>&1 || exit 1
done
cat gpurun_out/r3b/abl.txt | grep -v amdgpu.ids
tools/profile_round.sh gpurun_out/prof_r3a daed434
