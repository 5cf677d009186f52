#!/bin/bash
# round 5: kernel arguments in host memory (HIP_FORCE_DEV_KERNARG=0) vs the default device kernarg pool
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05w_1m 2 "X=0" "HIP_FORCE_DEV_KERNARG=0" || exit 1
BENCH_ARGS="--n 20000 --shard-sim 2 --steps 100" bash scripts/bench_variants.sh r05w_20k 2 "X=0" "HIP_FORCE_DEV_KERNARG=0" || exit 1
for v in 1 0; do
  HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python3 bench_odometry.py > gpurun_out/r05w_1m/odo_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r05w_1m/odo_$v.json'));print('C5 devkernarg=$v',round(d['frames_per_s'],1))"
done
