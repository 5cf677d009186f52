#!/bin/bash
# round 5: parity suite with target lists + kappa_far, then A/B against the revision before them
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05d
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log
[ $rc = 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit 1; }
( cd $OUT && for v in 0 1; do echo "HIP_FORCE_DEV_KERNARG=$v"; HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 ../../scripts/probes/launch_gap || exit 1; done > launch_gap.txt 2>&1 ) || exit 1
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05d/ab 2 "GICP_LIB_VARIANT=base5" "GICP_NO_TLISTS=1 GICP_CERT_KAPPA_FAR=0.002" "GICP_NO_TLISTS=1" "X=0" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05d/ab_c2 1 "GICP_LIB_VARIANT=base5" "X=0" || exit 1
