#!/bin/bash
# Unit-map schedules on the smaller workloads: C2 (100k/100k), one 8-GPU shard of C3, the C5 stream.
set -o pipefail
OUT=gpurun_out/umaps; mkdir -p $OUT
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh umaps/c2 2 "GICP_MOVING_ITERS=0" "GICP_MOVING_ITERS=5" "GICP_MOVING_ITERS=0 GICP_UNIT_MAP=8" > $OUT/c2.txt 2>&1 || exit 1
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh umaps/sh8 1 "GICP_MOVING_ITERS=0" "GICP_MOVING_ITERS=5" "GICP_MOVING_ITERS=0 GICP_UNIT_MAP=8" > $OUT/sh8.txt 2>&1 || exit 1
for v in "GICP_MOVING_ITERS=0" "GICP_MOVING_ITERS=5" "GICP_MOVING_ITERS=0 GICP_UNIT_MAP=8"; do
  echo "== $v"; env $v timeout -k 10 200 python bench_odometry.py --frames 300 2>&1 | tail -1
done > $OUT/odo.txt || exit 1
