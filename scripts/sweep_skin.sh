set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in ${SKINS:-0.2 0.8 1.2 1.6 2.4}; do
  export GICP_SKIN=$k
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/k.json 2> gpurun_out/k.err || { echo bench failed; tail gpurun_out/k.err; exit 1; }
  a=$(python -c "import json;d=json.load(open('gpurun_out/k.json'));print(round(d['value'],1))")
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/k.json 2> gpurun_out/k.err || { echo bench failed; tail gpurun_out/k.err; exit 1; }
  b=$(python -c "import json;d=json.load(open('gpurun_out/k.json'));print(round(d['value'],1))")
  echo "skin $k: 30-step $a it/s 200-step $b"
done
