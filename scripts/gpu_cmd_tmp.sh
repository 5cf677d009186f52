#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/t8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t8/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/t8/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/t8/pytest_gpu.log
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh ab8s20 3 "GICP_LIB_VARIANT=base" "GICP_LIB_VARIANT=vb" "X=0" || exit 1
bash scripts/bench_variants.sh ab8 2 "GICP_LIB_VARIANT=base" "GICP_LIB_VARIANT=vb" "X=0"
