# k_corr time of every shard of an 8-GPU job, each timed alone on one GPU (no collective).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
S=${S:-8}
for i in $(seq 0 $((S-1))); do
timeout -k 10 300 python bench.py --shard-sim $S --shard-index $i --no-cpu-baseline > gpurun_out/bal$i.json 2> gpurun_out/bal$i.err || { echo fail; tail gpurun_out/bal$i.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bal$i.json'));print($i,'it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
done
