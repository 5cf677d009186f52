#!/bin/bash
# round 5: the match gather from one 64-B position+covariance record (main) vs two 32-B gathers (base)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05rec
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05rec/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05rec/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05rec/pytest_gpu.log
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05rec_1m 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
bash scripts/bench_variants.sh r05rec_1m30 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05rec_c2 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh r05rec_sim8 1 "X=0" "GICP_LIB_VARIANT=base" || exit 1
for v in main base; do
  if [ $v = main ]; then unset GICP_LIB_VARIANT; else export GICP_LIB_VARIANT=$v; fi
  timeout -k 10 300 python3 bench_odometry.py > gpurun_out/r05rec/odo_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r05rec/odo_$v.json'));print('C5 $v',round(d['frames_per_s'],1))"
done
