#!/bin/bash
# env-toggle comparison at three workloads: "" vs each VAR=VAL given
export TMPDIR=/tmp
for args in "--steps 30" "--steps 200" "--n 100000 --steps 200"; do
for v in "" $@; do
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline $args > gpurun_out/env.json 2> gpurun_out/env.err || { echo "$v failed"; tail -3 gpurun_out/env.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/env.json'));print('$args','env','${v:-default}','it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
done
done
