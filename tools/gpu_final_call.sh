set -o pipefail
OUT=${1:-gpurun_out/final}
bash tools/gpu_round.sh ${OUT:-gpurun_out/final} || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > ${OUT:-gpurun_out/final}/smoke.log 2>&1
