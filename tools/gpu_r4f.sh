#!/bin/bash
# r4f: in-graph per-kernel times of the network with and without the strided layer2 tail
# (kernel trace + replay breakdown, tuned tiles loaded from one table).
set -o pipefail
O=gpurun_out/r4f
mkdir -p $O
export TMPDIR=/tmp
C="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $O/tiles.json"
timeout -k 10 300 python3 bench.py $C > $O/tune.log 2>&1 || { tail -5 $O/tune.log; exit 1; }
for f in 1 0; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s2_$f -o run -- \
    python3 bench.py $C --steps 10 --warmup 3 --plan-flag S2_TAIL=$f > $O/s2_$f.log 2>&1 || { tail -5 $O/s2_$f.log; exit 1; }
  python3 tools/replay_breakdown.py $O/s2_$f/run_kernel_trace.csv --last 5 > $O/replay_s2_$f.txt || exit 1
  echo "S2_TAIL=$f"; head -14 $O/replay_s2_$f.txt; tail -1 $O/replay_s2_$f.txt
done
# L2 hit rate per kernel of one network replay (one PMC pass: TCC_HIT_sum, TCC_MISS_sum)
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/pmc_l2 -o run -- \
  python3 bench.py $C --steps 2 --warmup 1 > $O/pmc_l2.log 2>&1 || { tail -5 $O/pmc_l2.log; exit 1; }
python3 - <<'PY' > $O/l2_hit_rate.txt
import csv, collections
rows = collections.defaultdict(dict)
for r in csv.DictReader(open('gpurun_out/r4f/pmc_l2/run_counter_collection.csv')):
    rows[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
    rows[int(r['Dispatch_Id'])]['name'] = r['Kernel_Name']
ids = sorted(rows)
# the last network replay: from the last stem launch to the next soft-argmax
last = max(i for i in ids if 'stem_pool' in rows[i]['name'])
for i in ids:
    if i < last:
        continue
    n = rows[i]['name']
    if 'softargmax' in n:
        break
    h, m = rows[i].get('TCC_HIT_sum', 0), rows[i].get('TCC_MISS_sum', 0)
    print('%-70s hit %.3f  (%.1f M requests)' % (n.split('(')[0][:70], h / max(h + m, 1), (h + m) / 1e6))
PY
cat $O/l2_hit_rate.txt
# the counter names of this rocprofv3 (for the next PMC passes)
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -c "" $O/counters.txt
# fp16 per-kernel times (the fp16 line ran ~1.6 % slower than bf16 in r4e)
timeout -k 10 300 python3 bench.py $C --precision fp16 --tune-file $O/tiles16.json > $O/tune16.log 2>&1 || { tail -5 $O/tune16.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/f16 -o run -- \
  python3 bench.py --no-cpu-baseline --no-mpjpe --fp32-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0 --tune-file $O/tiles16.json --precision fp16 --steps 10 --warmup 3 > $O/f16.log 2>&1 || { tail -5 $O/f16.log; exit 1; }
python3 tools/replay_breakdown.py $O/f16/run_kernel_trace.csv --last 5 > $O/replay_f16.txt || exit 1
tail -1 $O/replay_f16.txt
# the training leg behind the other legs (the round-3 order), with and without emptying the allocator cache
L="--no-cpu-baseline --no-mpjpe --peaked-steps 0"
for e in "" "--empty-cache-before-train"; do
  timeout -k 10 400 python3 bench.py $L --train-last $e > $O/trainlast.json 2> $O/trainlast.err || { tail -5 $O/trainlast.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/trainlast.json').read().strip().splitlines()[-1]);print('train-last $e', d['train_mode']['ms_per_step'], d['network_ms'])"
done
timeout -k 10 200 python3 bench.py --mode train --steps 10 --warmup 3 > $O/t.json 2> $O/t.err || exit 1
python3 -c "import json;d=json.loads(open('$O/t.json').read().strip().splitlines()[-1]);print('standalone', d['ms_per_step'])"
