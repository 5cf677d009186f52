#!/bin/bash
# Time the default library under environment settings, interleaved: bash scripts/variants_env.sh "A=1" "B=2" ...
export TMPDIR=/tmp
for round in $(seq ${ROUNDS:-2}); do
for e in "" "$@"; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/venv.json 2> gpurun_out/venv.err || { echo "env $e failed"; tail -3 gpurun_out/venv.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/venv.json'));print('env','${e:-default}','it/s',round(d['value'],1),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
done
done
