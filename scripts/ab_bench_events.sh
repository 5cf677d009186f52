set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/ab_events
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -5 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2 3; do
  GICP_BENCH_EVENTS=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/old$r.json 2>$OUT/old$r.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/new$r.json 2>$OUT/new$r.err || exit 1
  python -c "import json;a=json.load(open('$OUT/old$r.json'));b=json.load(open('$OUT/new$r.json'));print('events',round(a['value'],1),'none',round(b['value'],1),'corr',round(a['roofline']['kernel_avg_ms']*1e3,1),round(b['roofline']['kernel_avg_ms']*1e3,1))"
done
