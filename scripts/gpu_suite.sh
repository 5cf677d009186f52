#!/bin/bash
# Full GPU test suite + smoke, then the quick benches + tail breakdown.  Output: gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-suite}
mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log
[ $rc = 0 ] || { grep -E "FAILED|Error" $OUT/pytest_gpu.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
echo smoke ok
bash scripts/gpu_tail.sh ${1:-suite}
