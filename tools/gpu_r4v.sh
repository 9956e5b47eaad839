#!/bin/bash
# r4v: SQ counters of the layer1 identity Bottleneck kernel (tools/bottleneck_micro.py) -- instruction
# mix and wait cycles, to see what bounds its row loop
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/sq1 -o run -- python3 tools/bottleneck_micro.py --reps 2 --rounds 1 > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq2 -o run -- python3 tools/bottleneck_micro.py --reps 2 --rounds 1 > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
python3 - <<'PY' || exit 1
import csv, glob, collections
for d in ('sq1', 'sq2'):
    f = glob.glob('gpurun_out/r4v/%s/**/run_counter_collection.csv' % d, recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        if 'bottleneck64' in r['Kernel_Name']:
            kind = 'down' if 'true' in r['Kernel_Name'] else 'identity'
            acc[kind][r['Counter_Name']].append(float(r['Counter_Value']))
    for kind, cs in acc.items():
        for k, v in sorted(cs.items()):
            print('%-9s %-24s %14.0f (last of %d dispatches)' % (kind, k, v[-1], len(v)))
PY
echo done
