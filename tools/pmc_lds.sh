set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcl
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p1 -o run -- python3 $R/tools/conv_micro.py --cases deconv3 --tiles=5 --reps 3 --rounds 1 > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM TA_TA_BUSY TA_BUSY_avr TD_TD_BUSY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p2 -o run -- python3 $R/tools/conv_micro.py --cases deconv3 --tiles=5 --reps 3 --rounds 1 > $O/p2.log 2>&1
