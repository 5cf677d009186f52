#!/bin/bash
# round 5: where a C5 frame's time goes (kernel trace of 300 frames)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05m
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o t --output-format csv -- python3 bench_odometry.py --frames 300 > $OUT/odo.json 2> $OUT/odo.err || { echo trace failed; tail $OUT/odo.err; exit 1; }
python3 scripts/c5_frame_trace.py $OUT/trace | tee $OUT/c5_frames.txt
