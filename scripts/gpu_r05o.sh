#!/bin/bash
# round 5: spin-wait on the batch end (GICP_SPIN_WAIT=1, default) vs the stream sync; C5 and the driver command;
# odometry + extension tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_odometry.py tests/test_gpu_extensions.py -m gpu > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in 1 0; do
    GICP_SPIN_WAIT=$v timeout -k 10 300 python3 bench_odometry.py > $OUT/odo_${v}_$r.json 2> $OUT/odo_${v}_$r.err || { echo odo $v failed; tail $OUT/odo_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/odo_${v}_$r.json'));print('spin $v rep $r',round(d['frames_per_s'],1),'fps setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3))"
  done
done
bash scripts/bench_variants.sh r05o_1m 2 "X=0" "GICP_SPIN_WAIT=0" || exit 1
