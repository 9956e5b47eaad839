set -o pipefail
mkdir -p gpurun_out/pmc1
export TMPDIR=/tmp
timeout -k 10 120 python tools/conv_micro.py --tiles=-1,3,5,6 > gpurun_out/pmc1/micro.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc1/counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc1/a -o run -- python3 tools/conv_micro.py --cases deconv3,l3c2,l1c2 --tiles=-1 --reps 5 --rounds 1 > gpurun_out/pmc1/a.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc1/b -o run -- python3 tools/conv_micro.py --cases deconv3,l3c2,l1c2 --tiles=-1 --reps 5 --rounds 1 > gpurun_out/pmc1/b.log 2>&1 || exit 3
echo done
