#!/bin/bash
# round 5: tile-count budget (GICP_TILE_BUDGET, both clouds; default 1.35) on the driver command and C2
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05r_1m 2 "X=0" "GICP_TILE_BUDGET=1.15" "GICP_TILE_BUDGET=1.25" "GICP_TILE_BUDGET=1.5" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05r_c2 1 "X=0" "GICP_TILE_BUDGET=1.15" "GICP_TILE_BUDGET=1.5" || exit 1
