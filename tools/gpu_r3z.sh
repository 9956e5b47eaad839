set -o pipefail
# Round-3 refresh at HEAD: smoke, default bench line, round profiles.
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('infer',d['value'],d['network_ms'],d['roofline']['frac'],'train',d['train_mode']['ms_per_step'],'c1',d['configs1']['value'])"
bash tools/profile_round.sh $O/prof $(cat COMMIT_STAMP)
