set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0.002 0.005 0.01 0.02 0.05; do
  export GICP_CERT_KAPPA=$k
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/k.json 2> gpurun_out/k.err || { echo bench failed; tail gpurun_out/k.err; exit 1; }
  a=$(python -c "import json;d=json.load(open('gpurun_out/k.json'));print(round(d['value'],1))")
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 > gpurun_out/k.json 2> gpurun_out/k.err || { echo bench failed; tail gpurun_out/k.err; exit 1; }
  b=$(python -c "import json;d=json.load(open('gpurun_out/k.json'));print(round(d['value'],1))")
  echo "kappa $k: 30-step $a it/s, 200-step $b it/s"
done
