#!/bin/bash
# GPU iteration loop: parity tests, then 1M bench, then (optional) PMC passes 1-2.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest failed rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print('it/s',round(d['value'],1),'ms',round(d['ms_per_step'],4),'corr_ms',round(d['roofline']['kernel_avg_ms'],4),'pairs',d['valu']['pairs_per_launch'],'amb',d['ambiguous_last_pass'])"
if [ "$1" == "pmc" ]; then
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $set -d gpurun_out/pmc/p$i -o pmc --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_p$i.log 2>&1 || { echo pmc failed; exit 1; }
  done
  python scripts/pmc_summary.py gpurun_out/pmc
fi
