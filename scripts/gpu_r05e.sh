#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05e
mkdir -p $OUT
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05e/ab 2 "GICP_LIB_VARIANT=base5" "GICP_NO_TLISTS=1" "X=0" || exit 1
GICP_LIB_VARIANT=tail timeout -k 10 200 python3 scripts/tail_run.py --n 1000000 --steps 20 --reps 1 > $OUT/tail_1m.txt 2>&1 || { tail $OUT/tail_1m.txt; exit 1; }
tail -22 $OUT/tail_1m.txt
