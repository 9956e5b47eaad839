set -o pipefail
O=${1:-gpurun_out/r3q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/train" -o run -- \
  python3 bench.py --mode train --steps 4 --warmup 2 > "$O/train_bench.log" 2>&1 || exit 1
python3 tools/train_breakdown.py "$O"/train/run_kernel_trace.csv --steps 2 --launches > "$O/train_launches.txt"
rm -f $O/train/run_kernel_trace.csv
head -12 $O/train_launches.txt
