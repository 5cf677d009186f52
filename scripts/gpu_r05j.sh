#!/bin/bash
# round 5: descent outcomes per pass (tail build), then the full GPU suite at the current kernel
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p $OUT
GICP_LIB_VARIANT=tail timeout -k 10 300 python3 scripts/tail_run.py --steps 20 --reps 1 > $OUT/tail_1m.txt 2> $OUT/tail.err || { echo tail failed; tail $OUT/tail.err; exit 1; }
tail -22 $OUT/tail_1m.txt
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo suite failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
