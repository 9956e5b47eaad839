# PMC counters of the staggered 256x256 conv loop (tile 23) on deconv2 (tools/tile_micro.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcc
mkdir -p $O
RUN="python3 $R/tools/tile_micro.py --tiles 23 --only deconv2,l3 --reps 3 --rounds 1"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p1 -o run -- $RUN > $O/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_MFMA TA_TA_BUSY TA_BUSY_avr GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p2 -o run -- $RUN > $O/p2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/p3 -o run -- $RUN > $O/p3.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections, os
O=os.environ['GRAFT_REPO_ROOT']+'/gpurun_out/pmcc'
for p in ('p1','p2','p3'):
    f=glob.glob(O+'/'+p+'/**/*counter_collection.csv', recursive=True)
    if not f: print(p,'no csv'); continue
    agg=collections.defaultdict(lambda: collections.defaultdict(float)); cnt=collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k=r['Kernel_Name'][:60]
        if 'conv_igemm' not in k and 'conv_persist' not in k: continue
        agg[k][r['Counter_Name']]+=float(r['Counter_Value'])
    for k,d in agg.items():
        print(p,k); [print('   %-28s %.4g'%(c,v)) for c,v in sorted(d.items())]
PY
