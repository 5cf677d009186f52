#!/bin/bash
# Round-2 GPU pass: parity tests, smoke, the default bench (C3, cold start), C2 (100k) and a kernel
# trace of the default bench.  Output: gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
timeout -k 10 300 python bench.py --n 100000 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo bench c2 failed; tail $OUT/bench_c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o t --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/trace.err || { echo trace failed; exit 1; }
python3 scripts/trace_iters.py $OUT/trace 30 > $OUT/iterations.txt
for f in bench bench_c2; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),d['unit'],'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'frac',round(d['roofline']['frac'],4), d['passes']['moving_pass_us'], d['passes']['converged_pass_us'], d.get('warm_start'))"; done
cat $OUT/iterations.txt
