set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for env in "GICP_NO_CERTS=0" "GICP_NO_CERTS=1"; do
  export $env
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$env.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$env.json'));print('$env','it/s',round(d['value'],1),'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'pairs',d['valu']['pairs_per_launch'],'err',d['final_error'])"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/bench200_$env.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench200_$env.json'));print('$env 200','it/s',round(d['value'],1),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
done
export GICP_NO_CERTS=0
timeout -k 10 300 python bench_odometry.py > gpurun_out/odo.json 2> gpurun_out/odo.err || { echo odo failed; tail gpurun_out/odo.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/odo.json'));print('odo it/s',round(d['value'],1),'fps',round(d['frames_per_s'],1),d['frame_error'])"
