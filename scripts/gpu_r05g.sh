#!/bin/bash
# round 5: the multi-rank tests with the full-slot peer probe; C5 with the adaptive first batch vs batches of 8
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multirank.py > $OUT/multirank.log 2>&1 || { echo multirank failed; tail -30 $OUT/multirank.log; exit 1; }
tail -2 $OUT/multirank.log
for r in 1 2; do
  for v in main b8; do
    if [ $v = main ]; then unset GICP_LIB_VARIANT; else export GICP_LIB_VARIANT=$v; fi
    timeout -k 10 300 python3 bench_odometry.py > $OUT/odo_${v}_$r.json 2> $OUT/odo_${v}_$r.err || { echo odo $v failed; tail $OUT/odo_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/odo_${v}_$r.json'));print('$v $r',round(d['frames_per_s'],1),'fps setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3),'it/frame',round(d['iterations_per_frame'],2))"
  done
done
unset GICP_LIB_VARIANT
