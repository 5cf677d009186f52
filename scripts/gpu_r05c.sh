#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05c
( cd gpurun_out/r05c && for v in 0 1; do echo "HIP_FORCE_DEV_KERNARG=$v"; HIP_FORCE_DEV_KERNARG=$v timeout -k 10 120 ../../scripts/probes/launch_gap || exit 1; done > launch_gap.txt 2>&1 ) || exit 1
cat gpurun_out/r05c/launch_gap.txt
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05c/ab_kfar 2 "GICP_CERT_KAPPA_FAR=0.002" "GICP_CERT_KAPPA_FAR=0.04" "GICP_CERT_KAPPA_FAR=0.1" || exit 1
SKIP_TAIL=1 bash scripts/gpu_tail.sh r05c
