#!/bin/bash
# r4q: stem instruction mix (SQ counters on tools/stem_micro.py --only 256), and the head's
# rounding split by operand (precision_attribution head_act / head_w)
set -o pipefail
O=gpurun_out/r4q; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 tools/stem_micro.py --only 256 --reps 2 --rounds 1 > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 tools/stem_micro.py --only 256 --reps 2 --rounds 1 > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
python3 - <<'PY' || exit 1
import csv, glob, collections
for d in ('sq1', 'sq2'):
    f = glob.glob('gpurun_out/r4q/%s/**/run_counter_collection.csv' % d, recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'stem_pool' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in sorted(acc.items()):
        print('%-24s %14.0f (last of %d dispatches)' % (k, v[-1], len(v)))
PY
timeout -k 10 400 python3 tools/precision_attribution.py > $O/attribution.json 2> $O/attribution.err || { tail -5 $O/attribution.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/r4q/attribution.json'))
for dt in ('bf16', 'fp16'):
    for s in ('head', 'head_act', 'head_w', 'all', 'all_but_head'):
        v = d['emulated'][dt][s]
        print(dt, s, v['mpjpe_mm_mean'], v['mpjpe_mm_max'], v['heatmap_abs_err_max'])
PY
echo done
