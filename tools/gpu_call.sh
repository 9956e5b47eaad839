#!/bin/bash
# One parametrised GPU call (replaces round 5's one-off gpu_r5*.sh recipes).  Every step runs under
# its own time limit; the call stops at the first step that fails, faults or times out (no retries).
#
#   bash tools/gpu_call.sh OUTDIR STEP [STEP ...]
#
# STEP (arguments inside a step separated by commas; a '+' inside an argument is a space, e.g.
# tests:tests/test_gpu_kernels.py,-k,split+or+triang):
#   tests:ARGS          pytest -m gpu over ARGS (files, -k expressions), e.g. tests:tests/test_gpu_split.py,-k,tail
#   suite               the whole GPU test suite
#   smoke               __graft_entry__.smoke()
#   bench[@NAME]:ARGS   python bench.py ARGS -> OUTDIR/NAME.json (default name bench)
#   replay@NAME:ARGS    tuned bench forward under rocprofv3 --kernel-trace -> OUTDIR/NAME_replay_breakdown.txt
#                       (ARGS: extra bench args, e.g. --precision,fp16x3)
#   pmc@NAME:ARGS       HBM traffic per forward launch (FETCH_SIZE, WRITE_SIZE passes) -> OUTDIR/NAME_pmc_traffic.txt
#   profile:COMMIT      tools/profile_round.sh (the HEAD profile set)
#   ab@NAME:FLAG:ARGS   bench ARGS with --plan-flag FLAG=1 and =0, twice each, alternating -> OUTDIR/NAME_ab.txt
#   run@NAME:ARGS       python3 -u ARGS (a tool script and its arguments) -> OUTDIR/NAME.txt
set -o pipefail
OUT=${1:?usage: gpu_call.sh OUTDIR STEP...}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
LEAN="--no-cpu-baseline --no-mpjpe --fp32-steps 0 --parity-steps 0 --train-steps 0 --c1-steps 0 --peaked-steps 0 --c4-steps 0 --control-steps 0"

fail() { echo "step '$1' failed (exit $2)"; exit "$2"; }

summ() {  # the one-line JSON of a bench run -> a short summary
  python3 - "$1" "$2" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
except Exception as e:
    print(sys.argv[2], 'no JSON line:', e); sys.exit(0)
keys = ('value', 'ms_per_step', 'network_ms')
print(sys.argv[2], {k: d.get(k) for k in keys},
      'parity_mode', {k: (d.get('parity_mode') or {}).get(k) for k in ('value', 'network_ms', 'within_baseline_bars')})
PY
}

for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  name=${kind#*@}
  kind=${kind%%@*}
  [ "$name" = "$kind" ] && name=$kind
  IFS=',' read -ra argv <<< "$rest"
  argv=("${argv[@]//+/ }")
  args=${rest//,/ }
  echo "== $kind ($name) $args"
  case $kind in
    tests)
      log="$OUT/tests_${name}_$(date +%s).log"
      timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 200 --timeout-method thread "${argv[@]}" > "$log" 2>&1
      rc=$?; tail -3 "$log"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
        > "$OUT/gputests.log" 2>&1
      rc=$?; tail -3 "$OUT/gputests.log"; [ $rc -eq 0 ] || fail "$step" $rc ;;
    smoke)
      timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail "$step" $?
      tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python3 -u bench.py $args > "$OUT/$name.json" 2> "$OUT/$name.err" || fail "$step" $?
      summ "$OUT/$name.json" "$name" ;;
    replay|pmc)
      # stem runs per forward: --chunks N, else the plan's default (2 for the split dtype's halves)
      spf=1
      [[ " $args " == *" fp16x3 "* ]] && spf=2
      if [[ " $args " =~ " --chunks "([0-9]+)" " ]]; then spf=${BASH_REMATCH[1]}; [ "$spf" -lt 1 ] && spf=1; fi
      ;;&
    replay)
      timeout -k 10 300 python3 bench.py $LEAN --tune-file "$OUT/${name}_tiles.json" $args \
        > "$OUT/${name}_tune.json" 2> "$OUT/${name}_tune.err" || fail "$step" $?
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${name}_trace" -o run -- \
        python3 bench.py $LEAN --tune-file "$OUT/${name}_tiles.json" --steps 10 --warmup 3 $args \
        > "$OUT/${name}_traced.log" 2>&1 || fail "$step" $?
      python3 tools/replay_breakdown.py "$OUT/${name}_trace/run_kernel_trace.csv" --last 5 --start stem_pool_kernel --per $spf \
        > "$OUT/${name}_replay_breakdown.txt" || fail "$step" $?
      cp "$OUT/${name}_trace/run_kernel_stats.csv" "$OUT/${name}_kernel_stats.csv" 2>/dev/null
      rm -rf "$OUT/${name}_trace"
      tail -2 "$OUT/${name}_replay_breakdown.txt" ;;
    pmc)
      timeout -k 10 300 python3 bench.py $LEAN --tune-file "$OUT/${name}_tiles.json" $args \
        > "$OUT/${name}_tune.json" 2> "$OUT/${name}_tune.err" || fail "$step" $?
      for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$OUT/${name}_pmc_$ctr" -o run -- \
          python3 bench.py $LEAN --tune-file "$OUT/${name}_tiles.json" --steps 2 --warmup 1 $args \
          > "$OUT/${name}_pmc_$ctr.log" 2>&1 || fail "$step" $?
      done
      POSU_COMMIT=${POSU_COMMIT:-unknown} python3 tools/pmc_traffic.py "$OUT/${name}_pmc_FETCH_SIZE/run_counter_collection.csv" \
        "$OUT/${name}_pmc_WRITE_SIZE/run_counter_collection.csv" --stems $spf > "$OUT/${name}_pmc_traffic.txt" || fail "$step" $?
      rm -rf "$OUT/${name}_pmc_FETCH_SIZE" "$OUT/${name}_pmc_WRITE_SIZE"
      head -3 "$OUT/${name}_pmc_traffic.txt" ;;
    profile)
      bash tools/profile_round.sh "$OUT/prof" "${rest:-unknown}" || fail "$step" $? ;;
    ab)
      flag=${rest%%:*}
      bargs=${rest#*:}; [ "$bargs" = "$rest" ] && bargs=""
      bargs=${bargs//,/ }
      for r in 1 2; do
        for v in 1 0; do
          timeout -k 10 400 python3 -u bench.py $LEAN --plan-flag "$flag=$v" $bargs \
            > "$OUT/${name}_${v}_$r.json" 2> "$OUT/${name}_${v}_$r.err" || fail "$step" $?
          summ "$OUT/${name}_${v}_$r.json" "$flag=$v run $r" | tee -a "$OUT/${name}_ab.txt"
        done
      done ;;
    run)
      timeout -k 10 600 python3 -u "${argv[@]}" > "$OUT/$name.txt" 2>&1 || fail "$step" $?
      tail -5 "$OUT/$name.txt" ;;
    *)
      echo "unknown step kind: $kind"; exit 2 ;;
  esac
done
