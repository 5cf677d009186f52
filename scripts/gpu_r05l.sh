#!/bin/bash
# round 5: source tiles of 32 / 16 points (GICP_SRC_TILE) -- A/B on the small grids and the driver command,
# then the GPU suite with 16-point source tiles
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh r05l_sim8 2 "X=0" "GICP_SRC_TILE=32" "GICP_SRC_TILE=16" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05l_c2 2 "X=0" "GICP_SRC_TILE=32" "GICP_SRC_TILE=16" || exit 1
BENCH_ARGS="--n 20000 --shard-sim 2 --steps 100" bash scripts/bench_variants.sh r05l_20k 1 "X=0" "GICP_SRC_TILE=32" "GICP_SRC_TILE=16" || exit 1
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05l_1m 1 "X=0" "GICP_SRC_TILE=32" || exit 1
mkdir -p gpurun_out/r05l_tests
GICP_SRC_TILE=16 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05l_tests/pytest_gpu.log 2>&1; tail -3 gpurun_out/r05l_tests/pytest_gpu.log
