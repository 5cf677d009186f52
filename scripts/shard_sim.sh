# One rank of a G-GPU job timed on one GPU (shard 0 of G, no collective), G = 1, 2, 4, 8.
# STEPS (default 30, the bench default) iterations from the identity.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-30}
for s in 1 2 4 8; do
timeout -k 10 300 python bench.py --shard-sim $s --steps $STEPS --no-cpu-baseline > gpurun_out/sim$s.json 2> gpurun_out/sim$s.err || { echo fail; tail gpurun_out/sim$s.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/sim$s.json'));print($s,'it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
done
