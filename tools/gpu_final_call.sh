set -o pipefail
bash tools/gpu_round.sh gpurun_out/r4final2 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4final2/smoke.log 2>&1
