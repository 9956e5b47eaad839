#!/bin/bash
# full GPU suite + smoke (round-5 state)
OUT=gpurun_out/${1:-r5n}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $OUT/gputests.log 2>&1
rc=$?
tail -5 $OUT/gputests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
tail -1 $OUT/smoke.log
exit $rc
