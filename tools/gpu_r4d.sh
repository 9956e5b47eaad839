#!/bin/bash
# r4d: the training step vs the number of torch pool streams taken before it (hypothesis: the
# weight-gradient side stream shares a hardware queue with the main stream for some pool
# indices; GPU_MAX_HW_QUEUES = 4 on this pool)
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
for k in 0 1 2 3 4 5; do
  POSU_STREAM_SKIP=$k timeout -k 10 200 python -u bench.py --mode train --steps 10 --warmup 3 > $O/t_$k.json 2> $O/t_$k.err || { tail -5 $O/t_$k.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/t_$k.json').read().strip().splitlines()[-1]);print('skip $k', d['ms_per_step'])"
done
for k in 0 1; do
  GPU_MAX_HW_QUEUES=8 POSU_STREAM_SKIP=$k timeout -k 10 200 python -u bench.py --mode train --steps 10 --warmup 3 > $O/q8_$k.json 2> $O/q8_$k.err || { tail -5 $O/q8_$k.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/q8_$k.json').read().strip().splitlines()[-1]);print('hwq8 skip $k', d['ms_per_step'])"
done
