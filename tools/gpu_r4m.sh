#!/bin/bash
# r4m: smoke, the profile round (kernel trace + replay breakdown, PMC traffic on graph replays,
# training trace) and the default bench line, at 4e5b0a7
set -o pipefail
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 1100 bash tools/profile_round.sh $O/prof 4e5b0a7 || exit 1
head -1 $O/prof/pmc_traffic_network.txt
tail -1 $O/prof/replay_breakdown.txt
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 1500 $O/bench_default.json
echo done
