#!/bin/bash
# GPU tests, then an interleaved A/B of the default build against variant $2 (libgicp_hip_$2.so), then a
# per-pass instruction-count PMC run of the default build.  Output: gpurun_out/$1/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-abr}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash scripts/bench_variants.sh ${1:-abr}/ab 2 "GICP_LIB_VARIANT=${2:-base}" "X=0" || exit 1
mkdir -p $OUT/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVE_CYCLES -d $OUT/pmc/p1 -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/pmc/p1.log 2>&1 || { echo pmc failed; exit 1; }
python3 scripts/pmc_passes.py $OUT/pmc/p1 > $OUT/pmc_passes.txt
head -6 $OUT/pmc_passes.txt; tail -2 $OUT/pmc_passes.txt
