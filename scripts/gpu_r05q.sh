#!/bin/bash
# round 5: the host doorbell for converging registrations (GICP_DOORBELL=1, default) vs batches; full GPU suite first
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo suite failed; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  for v in 1 0; do
    GICP_DOORBELL=$v timeout -k 10 300 python3 bench_odometry.py > $OUT/odo_${v}_$r.json 2> $OUT/odo_${v}_$r.err || { echo odo $v failed; tail $OUT/odo_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/odo_${v}_$r.json'));print('doorbell $v rep $r',round(d['frames_per_s'],1),'fps setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3),'it/frame',round(d['iterations_per_frame'],2))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o t --output-format csv -- python3 bench_odometry.py --frames 300 > $OUT/odo_trace.json 2> $OUT/odo_trace.err || { echo trace failed; exit 1; }
python3 scripts/c5_frame_trace.py $OUT/trace | tee $OUT/c5_frames.txt
