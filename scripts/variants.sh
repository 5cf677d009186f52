#!/bin/bash
# Time k_corr variants (GICP_LIB_VARIANT) on the 1M/1M bench, interleaved, one process each.
export TMPDIR=/tmp
for round in $(seq ${ROUNDS:-2}); do
for v in "" $@; do
  GICP_LIB_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/var_$v.err; exit 1; }
  python -c "import json,sys;d=json.load(open('gpurun_out/var_$v.json'));print('variant','${v:-main}','it/s',round(d['value'],1),'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'pairs',d['valu']['pairs_per_launch'])"
done
done
