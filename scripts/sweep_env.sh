#!/bin/bash
# Per-iteration k_corr profile of the default bench for several values of one environment knob.
#   bash scripts/sweep_env.sh VAR v1 v2 ...
export TMPDIR=/tmp
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/sweep_$v -o t --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/sweep_$v.json 2>/dev/null || { echo "run $v failed"; exit 1; }
  echo "$VAR=$v it/s $(python3 -c "import json;print(round(json.load(open('gpurun_out/sweep_$v.json'))['value'],1))")"
  python3 scripts/trace_iters.py gpurun_out/sweep_$v 30 | head -1
done
