#!/bin/bash
# Separate rocprofv3 --pmc passes (no tracing combined) over a short 1M bench run.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
ARGS=${2:---n 1000000 --steps 5 --warmup 1 --no-cpu-baseline}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" \
           "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/p$i -o pmc --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
