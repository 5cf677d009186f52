#!/bin/bash
# round 5: one-level reduction threshold (kFlatUnits 128, default) vs 512 / 64 on the small and mid grids
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05fl_c2 2 "X=0" "GICP_LIB_VARIANT=flat512" || exit 1
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh r05fl_sim8 1 "X=0" "GICP_LIB_VARIANT=flat512" || exit 1
BENCH_ARGS="--n 20000 --shard-sim 2 --steps 100" bash scripts/bench_variants.sh r05fl_20k 1 "X=0" "GICP_LIB_VARIANT=flat64" || exit 1
