set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 2 4 8; do
timeout -k 10 300 python bench.py --shard-sim $s --steps 200 --no-cpu-baseline > gpurun_out/sim$s.json 2> gpurun_out/sim$s.err || { echo fail; tail gpurun_out/sim$s.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/sim$s.json'));print($s,'it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
done
timeout -k 10 300 python bench.py --steps 200 --no-cpu-baseline > gpurun_out/sim1.json 2> gpurun_out/sim1.err
python -c "import json;d=json.load(open('gpurun_out/sim1.json'));print(1,'it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
