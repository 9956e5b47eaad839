#!/bin/bash
# r4p: HBM traffic of one training step at this commit (separate FETCH_SIZE / WRITE_SIZE passes
# of bench.py --mode train, both streams), for the training line's roofline.traffic
set -o pipefail
O=gpurun_out/r4p; mkdir -p $O
export TMPDIR=/tmp
C=${1:-unknown}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/t_$c -o run -- \
    python3 bench.py --mode train --steps 2 --warmup 1 > $O/t_$c.log 2>&1 || { tail -5 $O/t_$c.log; exit 1; }
done
POSU_COMMIT=$C python3 tools/pmc_train_traffic.py $O/t_FETCH_SIZE/run_counter_collection.csv $O/t_WRITE_SIZE/run_counter_collection.csv > $O/pmc_traffic_train.txt || exit 1
head -12 $O/pmc_traffic_train.txt
timeout -k 10 200 python3 bench.py --mode train --steps 10 --warmup 3 > $O/train.json 2> $O/train.err || { tail -5 $O/train.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/train.json').read().strip().splitlines()[-1]);print('train', d['value'], d['ms_per_step'])"
echo done
