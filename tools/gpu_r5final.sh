#!/bin/bash
# Round-5 validation in one call: GPU test suite + default bench line (gpu_round.sh), smoke, then
# the HEAD profile set (inference replay + PMC, training trace) -- each step under its own limit,
# nothing more after a failure.
OUT=${1:-gpurun_out/r5final}
COMMIT=${2:-unknown}
mkdir -p $OUT
bash tools/gpu_round.sh $OUT || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
bash tools/profile_round.sh $OUT/prof $COMMIT || exit $?
cp $OUT/prof/infer/run_kernel_stats.csv $OUT/prof/kernel_stats_infer_bench.csv 2>/dev/null
rm -rf $OUT/prof/infer $OUT/prof/pmc_fetch $OUT/prof/pmc_write
cp $OUT/prof/train/run_kernel_stats.csv $OUT/prof/kernel_stats_train_bench.csv 2>/dev/null
rm -rf $OUT/prof/train
cat $OUT/prof/replay_breakdown.txt | tail -3
