#!/bin/bash
# round-5 mid-session validation at HEAD: GPU suite + default bench line, then smoke
OUT=gpurun_out/r5av
bash tools/gpu_round.sh $OUT || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -2 $OUT/smoke.log
