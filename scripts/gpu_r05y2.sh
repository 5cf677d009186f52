#!/bin/bash
# round 5: calm tiles (cert_pass bit 30: the last pass needed no search) skip the rel32 read -- GPU suite, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05y2
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05y2/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05y2/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05y2/pytest_gpu.log
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05y2_1m 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
bash scripts/bench_variants.sh r05y2_1m30 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05y2_c2 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh r05y2_sim8 1 "X=0" "GICP_LIB_VARIANT=base" || exit 1
