#!/bin/bash
# Baseline benches + the k_corr tail breakdown (GICP_TAIL build).  Output: gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tail}
mkdir -p $OUT
if [ "${SKIP_BENCH:-0}" != 1 ]; then
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench20.json 2> $OUT/bench20.err || { echo bench failed; tail $OUT/bench20.err; exit 1; }
timeout -k 10 300 python3 bench.py --n 100000 --no-cpu-baseline > $OUT/c2.json 2> $OUT/c2.err || { echo c2 failed; tail $OUT/c2.err; exit 1; }
timeout -k 10 300 python3 bench.py --shard-sim 8 --no-cpu-baseline > $OUT/sim8.json 2> $OUT/sim8.err || { echo sim8 failed; tail $OUT/sim8.err; exit 1; }
timeout -k 10 300 python3 bench.py --n 20000 --shard-sim 2 --steps 100 --no-cpu-baseline > $OUT/sim2_20k.json 2> $OUT/sim2_20k.err || { echo sim2 failed; tail $OUT/sim2_20k.err; exit 1; }
for f in bench20 c2 sim8 sim2_20k; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),d['unit'],'corr_ms',round(d['roofline']['kernel_avg_ms'],4), 'mov',round(d['passes']['moving_pass_us'],1), 'conv',round(d['passes']['converged_pass_us'],1))"; done
fi
[ "${SKIP_TAIL:-0}" = 1 ] && exit 0
V=${TAIL_VARIANT:-tail}
GICP_LIB_VARIANT=$V timeout -k 10 200 python3 scripts/tail_run.py --n 1000000 > $OUT/tail_1m.txt 2>&1 || { echo tail1m failed; tail $OUT/tail_1m.txt; exit 1; }
GICP_LIB_VARIANT=$V timeout -k 10 200 python3 scripts/tail_run.py --n 1000000 --shard-sim 8 > $OUT/tail_sim8.txt 2>&1 || { echo tailsim8 failed; tail $OUT/tail_sim8.txt; exit 1; }
GICP_LIB_VARIANT=$V timeout -k 10 200 python3 scripts/tail_run.py --n 100000 > $OUT/tail_c2.txt 2>&1 || { echo tailc2 failed; tail $OUT/tail_c2.txt; exit 1; }
GICP_LIB_VARIANT=$V timeout -k 10 200 python3 scripts/tail_run.py --n 20000 --shard-sim 2 --steps 60 > $OUT/tail_20k.txt 2>&1 || { echo tail20k failed; tail $OUT/tail_20k.txt; exit 1; }
for f in tail_1m tail_sim8 tail_c2 tail_20k; do echo "== $f"; tail -3 $OUT/$f.txt; done
