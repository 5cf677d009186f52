#!/bin/bash
# Quick GPU pass: parity tests, smoke, the driver's bench command (20 steps), the 30-step bench, the
# 8-GPU shard stand-in, and bench.py --gpus 2 (must refuse on a 1-GPU box).  Output: gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
echo smoke ok
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || { echo bench failed; tail $OUT/bench20.err; exit 1; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench30.json 2> $OUT/bench30.err || { echo bench30 failed; tail $OUT/bench30.err; exit 1; }
timeout -k 10 300 python3 bench.py --shard-sim 8 --no-cpu-baseline > $OUT/sim8.json 2> $OUT/sim8.err || { echo sim8 failed; tail $OUT/sim8.err; exit 1; }
timeout -k 10 120 python3 bench.py --gpus 2 > $OUT/gpus2.out 2> $OUT/gpus2.err; echo "gpus2 rc=$? $(cat $OUT/gpus2.err | tail -1)"
for f in bench20 bench30 sim8; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),d['unit'],'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'frac',round(d['roofline']['frac'],4), 'mov',round(d['passes']['moving_pass_us'],1), 'conv',round(d['passes']['converged_pass_us'],1), d['passes']['k_corr_us_per_iteration'])"; done
