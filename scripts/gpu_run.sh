#!/bin/bash
# One parameterised GPU lease: run named steps in order, each under its own time limit, stop at the first
# failure (no further GPU step after a failed, faulted or timed-out one).  Output: gpurun_out/TAG/.
#
#   scripts/gpu_run.sh TAG STEP [STEP ...]
#
# Steps (ARGS after ':' are passed through; use ',' for spaces inside one step):
#   tests[:PYTEST_ARGS]        pytest -m gpu over tests/ (or the given files / -k expression)
#   smoke                      __graft_entry__.smoke()
#   bench[:BENCH_ARGS]         one bench.py line -> bench_<n>.json (default: the driver's command)
#   ab:REPS:BENCH_ARGS:V1|V2   interleaved A/B of bench.py variants (scripts/bench_variants.sh); each Vi is an
#                              environment assignment list, e.g. "X=0|GICP_LIB_VARIANT=base"
#   tail[:N,ARGS]              tail-build stage stamps of one registration (scripts/tail_run.py, GICP_TAIL build)
#   timeline[:ARGS]            the waves that end each pass (scripts/last_waves.py, GICP_TIMELINE build)
#   odo[:ARGS]                 the C5 stream bench (bench_odometry.py)
#   c1                         the C1 latency bench (bench_small.py)
#   profile[:PD]               scripts/profile_round.sh (kernel trace, PMC passes, traffic) into PD
#   extras                     scripts/round_extras.sh (C2, 2-D, C5, per-pass instruction counts)
#   cmd:SHELL_COMMAND          anything else (',' -> ' '), under the step time limit
# STEP_TIMEOUT (s, default 600) bounds each step.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
TL=${STEP_TIMEOUT:-600}
n=0
for step in "$@"; do
  n=$((n+1))
  kind=${step%%:*}
  arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  arg=${arg//,/ }
  log=$OUT/s${n}_${kind}.log
  echo "== step $n: $kind $arg"
  case $kind in
    tests)
      timeout -k 10 $TL python3 -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $log 2>&1
      rc=$?; tail -1 $log ;;
    smoke)
      timeout -k 10 $TL python3 -c "import __graft_entry__ as g; g.smoke()" > $log 2>&1; rc=$?; tail -1 $log ;;
    bench)
      timeout -k 10 $TL python3 bench.py ${arg:---gpus 1 --steps 20 --warmup 5} > $OUT/bench_$n.json 2> $log; rc=$?
      [ $rc = 0 ] && python3 -c "import json;d=json.load(open('$OUT/bench_$n.json'));p=d.get('passes',{});print(round(d['value'],1),d['unit'],'frac',round(d['roofline']['frac'],4),'moving',round(p.get('moving_pass_us',0),1),'conv',round(p.get('converged_pass_us',0),1));print(' '.join(f'{x:.0f}' for x in p.get('k_corr_us_per_iteration',[])))" ;;
    ab)
      reps=${arg%%:*}; rest=${arg#*:}; bargs=${rest%%:*}; vars=${rest#*:}
      IFS='|' read -ra V <<< "$vars"
      BENCH_ARGS="$bargs" timeout -k 10 $TL bash scripts/bench_variants.sh $TAG/ab_$n $reps "${V[@]}" > $log 2>&1; rc=$?; cat $log ;;
    tail)
      GICP_LIB_VARIANT=${TAIL_VARIANT:-tail} timeout -k 10 $TL python3 scripts/tail_run.py ${arg:---steps 20 --reps 1} > $OUT/tail_$n.txt 2> $log
      rc=$?; tail -22 $OUT/tail_$n.txt ;;
    timeline)
      GICP_LIB_VARIANT=${TL_VARIANT:-tl} timeout -k 10 $TL python3 scripts/last_waves.py ${arg} > $OUT/last_waves_$n.txt 2> $log
      rc=$?; grep -E "^pass" $OUT/last_waves_$n.txt ;;
    odo)
      timeout -k 10 $TL python3 bench_odometry.py $arg > $OUT/odo_$n.json 2> $log; rc=$?
      [ $rc = 0 ] && python3 -c "import json;d=json.load(open('$OUT/odo_$n.json'));print(round(d['frames_per_s'],1),'frames/s setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3))" ;;
    c1)
      timeout -k 10 $TL python3 bench_small.py > $OUT/c1_$n.json 2> $log; rc=$?
      [ $rc = 0 ] && python3 -c "import json;d=json.load(open('$OUT/c1_$n.json'));print('C1',d['summary'])" ;;
    profile)
      timeout -k 10 $TL bash scripts/profile_round.sh ${TAG}_prof ${arg:-profiles/r06} > $log 2>&1; rc=$?; tail -5 $log ;;
    extras)
      timeout -k 10 $TL bash scripts/round_extras.sh ${TAG}_extras > $log 2>&1; rc=$?; tail -8 $log ;;
    cmd)
      timeout -k 10 $TL bash -c "$arg" > $log 2>&1; rc=$?; tail -20 $log ;;
    *)
      echo "unknown step $kind"; exit 2 ;;
  esac
  if [ $rc != 0 ]; then
    echo "step $n ($kind) failed: rc=$rc"; tail -30 $log; exit 1
  fi
done
