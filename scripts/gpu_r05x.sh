#!/bin/bash
# round 5: the walk's fp32 screen coordinates of the source points from the fp64 points the epilogue reads anyway
# (relx build, GICP_REL_FROM_XYZ) instead of the rel32 array: 16 B per point less to read where the second read
# of the fp64 point hits the cache.  Parity tests with the variant, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05x
GICP_LIB_VARIANT=relx timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -k "not native_library" > gpurun_out/r05x/tests.log 2>&1 || { tail -30 gpurun_out/r05x/tests.log; exit 1; }
tail -1 gpurun_out/r05x/tests.log
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05x_1m 2 "X=0" "GICP_LIB_VARIANT=relx" || exit 1
bash scripts/bench_variants.sh r05x_1m30 1 "X=0" "GICP_LIB_VARIANT=relx" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05x_c2 2 "X=0" "GICP_LIB_VARIANT=relx" || exit 1
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh r05x_sim8 1 "X=0" "GICP_LIB_VARIANT=relx" || exit 1
