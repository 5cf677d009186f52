#!/bin/bash
# variants at three workloads: 1M 30 steps, 1M 200 steps, 100k 200 steps
export TMPDIR=/tmp
for args in "--steps 30" "--steps 200" "--n 100000 --steps 200"; do
for v in "" $@; do
  GICP_LIB_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline $args > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var_$v.json'));print('$args','variant','${v:-main}','it/s',round(d['value'],1),'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'pairs',d['valu']['pairs_per_launch'])"
done
done
