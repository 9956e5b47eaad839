set -o pipefail
# Round-3 refresh at HEAD: full GPU suite, smoke, default bench line, round profiles.
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -3 $O/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 --train-stream default > $O/train_default.json 2>/dev/null || exit 1
python -c "import json;[print(f,json.loads(open('$O/'+f).read().strip().splitlines()[-1])['ms_per_step']) for f in ('train_default.json',)]"
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('infer',d['value'],d['network_ms'],d['roofline']['frac'],'train(high prio)',d['train_mode']['ms_per_step'])"
bash tools/profile_round.sh $O/prof $(cat COMMIT_STAMP)
