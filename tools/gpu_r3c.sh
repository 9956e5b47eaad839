set -o pipefail
# GPU call: full GPU suite, staggered-loop timing ablations, default bench line, kernel trace of
# the tuned inference bench.  Stops at the first GPU step that faults, aborts or times out.
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -15 $O/gputests.log; [ $rc -le 1 ] || exit $rc
for m in 0 1 2 4 6 8; do
  echo "== ig_$m" >> $O/abl.txt
  timeout -k 10 120 python tools/tile_micro.py --tiles 23 --reps 10 --rounds 3 --lib pose-unsupervised_amd/build/abl/libposeu_ig_$m.so >> $O/abl.txt 2>&1 || exit 1
done
grep -v amdgpu.ids $O/abl.txt
timeout -k 10 120 python tools/tail_micro.py > $O/tail_micro.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/tail_micro.txt
timeout -k 10 400 python -u bench.py --tune-file $O/tiles.json > $O/bench.json 2> $O/bench.err || exit 1
tail -c 400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/infer -o run -- \
  python3 bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --tune-file $O/tiles.json --steps 10 --warmup 3 > $O/infer_bench.log 2>&1 || exit 1
python3 tools/replay_breakdown.py $O/infer/run_kernel_trace.csv --last 5 > $O/replay_breakdown.txt
echo done
