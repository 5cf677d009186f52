# Round-end GPU pass: parity tests, smoke, the profile set (bench, trace, PMC), 200-step and
# no-certificate benches, the C5 odometry bench.  Output: gpurun_out/$1/.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
echo smoke ok
bash scripts/profile_round.sh ${1:-final} || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > $OUT/bench200.json 2> $OUT/bench200.err || { echo bench200 failed; exit 1; }
GICP_NO_CERTS=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_nocerts.json 2> $OUT/bench_nocerts.err || { echo nocerts failed; exit 1; }
timeout -k 10 300 python bench_odometry.py > $OUT/odo.json 2> $OUT/odo.err || { echo odo failed; tail $OUT/odo.err; exit 1; }
for f in bench bench200 bench_nocerts; do python -c "import json;d=json.load(open('$OUT/$f.json'));print('$f',round(d['value'],1),d['unit'],'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'frac',round(d['roofline']['frac'],4))"; done
cat $OUT/odo.json; cat $OUT/iterations.txt
