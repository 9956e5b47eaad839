set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/train -o run -- \
  python3 bench.py --mode train --steps 4 --warmup 2 > $O/train_bench.log 2>&1 || exit 1
python3 tools/train_breakdown.py $O/train/run_kernel_trace.csv --steps 2 --launches > $O/train_breakdown.txt
head -12 $O/train_breakdown.txt
