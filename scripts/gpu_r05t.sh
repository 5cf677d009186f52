#!/bin/bash
# round 5: C5 without the sampled per-launch HIP events (default now) vs with them (--kernel-times)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05t
mkdir -p $OUT
for r in 1 2; do
  for v in noev ev; do
    F=""; [ $v = ev ] && F="--kernel-times"
    timeout -k 10 300 python3 bench_odometry.py $F > $OUT/odo_${v}_$r.json 2> $OUT/odo_${v}_$r.err || { echo odo failed; tail $OUT/odo_${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/odo_${v}_$r.json'));print('$v rep $r',round(d['frames_per_s'],1),'fps setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3))"
  done
done
