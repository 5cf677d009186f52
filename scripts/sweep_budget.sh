set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in 1.35 1.6 2.0 2.5; do
  export GICP_TILE_BUDGET=$b
  timeout -k 10 300 python bench_odometry.py --frames 300 > gpurun_out/o.json 2> gpurun_out/o.err || { echo odo failed; tail gpurun_out/o.err; exit 1; }
  a=$(python -c "import json;d=json.load(open('gpurun_out/o.json'));print(round(d['value'],1), round(d['frames_per_s'],1), round(d['setup_ms_per_frame'],3), round(d['align_ms_per_frame'],3))")
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/k.json 2> gpurun_out/k.err || { echo bench failed; tail gpurun_out/k.err; exit 1; }
  c=$(python -c "import json;d=json.load(open('gpurun_out/k.json'));print(round(d['value'],1))")
  echo "budget $b: odo it/s fps setup align = $a ; 1M 30-step $c"
done
