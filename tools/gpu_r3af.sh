set -o pipefail
# end-of-session check at HEAD: full GPU suite, smoke, default bench line
O=gpurun_out/r3af
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1
rc=$?; tail -3 $O/gputests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('infer',d['value'],d['ms_per_step'],d['network_ms'],d['roofline']['frac'],d['roofline']['traffic'],'train',d['train_mode']['ms_per_step'],d['train_mode']['traffic'],'c1',d['configs1']['value'],'mpjpe',d['mpjpe_vs_ref_mm']['mean'])"
