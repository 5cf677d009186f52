#!/bin/bash
# round 5 final: the round-end set at the final code (tests, smoke, driver-command profile and bench line),
# then the C5 lines
set -o pipefail
export TMPDIR=/tmp
SKIP_EXTRAS=1 bash scripts/round_end.sh r05final || exit 1
OUT=gpurun_out/r05final_extras
mkdir -p $OUT
timeout -k 10 400 python3 bench_odometry.py > $OUT/bench_odometry_staged.json 2> $OUT/odo.err || { echo odometry failed; exit 1; }
timeout -k 10 400 python3 bench_odometry.py --copy > $OUT/bench_odometry_staged_copy.json 2> $OUT/odo_copy.err || { echo odometry copy failed; exit 1; }
timeout -k 10 400 python3 bench_odometry.py --sync > $OUT/bench_odometry_sync.json 2> $OUT/odo_sync.err || { echo odometry sync failed; exit 1; }
for f in bench_odometry_staged bench_odometry_staged_copy bench_odometry_sync; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['frames_per_s'],1),'fps setup',round(d['setup_ms_per_frame'],3),'align',round(d['align_ms_per_frame'],3))"; done
timeout -k 10 300 python3 bench.py --n 100000 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/c2.err || { echo c2 failed; exit 1; }
timeout -k 10 300 python3 bench.py --shard-sim 8 --no-cpu-baseline > $OUT/bench_shard_sim8.json 2> $OUT/sim8.err || { echo sim8 failed; exit 1; }
for f in bench_c2 bench_shard_sim8; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),'conv',round(d['passes']['converged_pass_us'],1))"; done
