set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2/a -o run -- python3 tools/conv_micro.py --cases deconv3,l3c2 --tiles=5,29 --reps 3 --rounds 1 > gpurun_out/pmc2/a.log 2>&1 || exit 2
timeout -s KILL 90 rocprofv3 --pmc TA_BUFFER_READ_LDS_WAVEFRONTS_sum TA_DATA_STALLED_BY_TC_CYCLES_sum SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d gpurun_out/pmc2/b -o run -- python3 tools/conv_micro.py --cases deconv3,l3c2 --tiles=5,29 --reps 3 --rounds 1 > gpurun_out/pmc2/b.log 2>&1 || exit 3
echo done
