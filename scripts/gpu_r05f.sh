#!/bin/bash
# round 5: benches at the current kernel (padded tickets, one-level reduction), C1 with the native CG, C5 with
# borrowed / copied staging, and the tail breakdown
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05f
mkdir -p $OUT
bash scripts/gpu_tail.sh r05f || exit 1
timeout -k 10 600 python3 bench_small.py > $OUT/bench_c1.json 2> $OUT/bench_c1.err || { echo c1 failed; tail $OUT/bench_c1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c1.json'));print('C1',d['summary'])"
timeout -k 10 600 python3 bench_odometry.py > $OUT/bench_odometry_borrow.json 2> $OUT/odo1.err || { echo odo failed; tail $OUT/odo1.err; exit 1; }
timeout -k 10 600 python3 bench_odometry.py --copy > $OUT/bench_odometry_copy.json 2> $OUT/odo2.err || { echo odo2 failed; tail $OUT/odo2.err; exit 1; }
for f in bench_odometry_borrow bench_odometry_copy; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['frames_per_s'],1),'fps',round(d['value'],1),'it/s setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3),'it/frame',round(d['iterations_per_frame'],2))"; done
