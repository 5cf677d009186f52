#!/bin/bash
# round 5: the new multi-rank / full-size tests, then the baseline benches + tail breakdown
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_new.log 2>&1; rc=$?
tail -3 $OUT/pytest_new.log
[ $rc = 0 ] || { grep -E "FAILED|Error" $OUT/pytest_new.log | head; exit 1; }
bash scripts/gpu_tail.sh r05a
