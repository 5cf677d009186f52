#!/bin/bash
# round 5: re-tune the moving passes' unit map (GICP_MOVING_MAP chunk / GICP_MOVING_ITERS) at the current kernel
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05v 2 "X=0" "GICP_MOVING_MAP=4" "GICP_MOVING_MAP=16" "GICP_MOVING_ITERS=3" "GICP_MOVING_ITERS=10" "GICP_MOVING_ITERS=20" || exit 1
