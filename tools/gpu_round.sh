#!/bin/bash
# One GPU call: the GPU test suite, then (unless a test run faulted or hung: exit status > 1)
# the default bench line.  Usage: tools/gpu_round.sh OUTDIR [extra bench args]
out=${1:-gpurun_out/round}; shift
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/gputests.log 2>&1
rc=$?
tail -3 $out/gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py "$@" > $out/bench.json 2> $out/bench.err
rc=$?
tail -c 600 $out/bench.json
exit $rc
