#!/bin/bash
# default bench line + the profile set of the HEAD plan (tools/profile_round.sh)
OUT=gpurun_out/r5i
mkdir -p $OUT
timeout -k 10 500 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -c 300 $OUT/bench.json
tools/profile_round.sh $OUT/prof $(cat COMMIT_STAMP 2>/dev/null || echo head) > $OUT/profile.log 2>&1
rc=$?
tail -3 $OUT/profile.log
exit $rc
