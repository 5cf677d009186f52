set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
for n in 100000 1000000; do
  for st in 30 200; do
    timeout -k 10 300 python bench.py --n $n --steps $st --no-cpu-baseline > gpurun_out/cfg/b_${n}_${st}.json 2> gpurun_out/cfg/err || { echo fail; tail gpurun_out/cfg/err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/cfg/b_${n}_${st}.json'));print($n,$st,'it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4))"
  done
done
