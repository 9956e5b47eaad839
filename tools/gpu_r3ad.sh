set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3ad
mkdir -p $O
T="$R/bench.py --mode train --steps 2 --warmup 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f -o run -- python3 $T > $O/f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/w -o run -- python3 $T > $O/w.log 2>&1 || exit 1
POSU_COMMIT=$(cat $R/COMMIT_STAMP) python3 $R/tools/pmc_train_traffic.py $O/f/run_counter_collection.csv $O/w/run_counter_collection.csv > $O/pmc_traffic_train.txt
rm -f $O/f/run_kernel_trace.csv $O/w/run_kernel_trace.csv
cat $O/pmc_traffic_train.txt
