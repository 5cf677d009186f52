#!/bin/bash
# round 5: C5 frame overheads -- reset_tile_state in one launch, exchange timing cleared with the state upload,
# no host sync in commit / target_to_source (main) vs HEAD (base); odometry + multirank tests first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05n
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_odometry.py tests/test_gpu_multirank.py -m gpu > $OUT/tests.log 2>&1 || { echo tests failed; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for v in main base; do
    if [ $v = main ]; then unset GICP_LIB_VARIANT; else export GICP_LIB_VARIANT=$v; fi
    timeout -k 10 300 python3 bench_odometry.py > $OUT/odo_${v}_$r.json 2> $OUT/odo_${v}_$r.err || { echo odo $v failed; tail $OUT/odo_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/odo_${v}_$r.json'));print('$v $r',round(d['frames_per_s'],1),'fps setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3),'it/frame',round(d['iterations_per_frame'],2))"
  done
done
unset GICP_LIB_VARIANT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o t --output-format csv -- python3 bench_odometry.py --frames 300 > $OUT/odo_trace.json 2> $OUT/odo_trace.err || { echo trace failed; exit 1; }
python3 scripts/c5_frame_trace.py $OUT/trace | tee $OUT/c5_frames.txt
