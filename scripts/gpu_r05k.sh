#!/bin/bash
# round 5: sparse-wave certificate kappa (GICP_CERT_KAPPA_SPARSE x d_c for waves with <= GICP_SPARSE_LANES walking lanes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p $OUT
bash scripts/bench_variants.sh r05k 2 "X=0" "GICP_CERT_KAPPA_SPARSE=0.01" "GICP_CERT_KAPPA_SPARSE=0.02" "GICP_CERT_KAPPA_SPARSE=0.05" "GICP_CERT_KAPPA_SPARSE=0.02 GICP_SPARSE_LANES=16" || exit 1
for v in 0 0.02; do
  GICP_CERT_KAPPA_SPARSE=$v GICP_LIB_VARIANT=tail timeout -k 10 300 python3 scripts/tail_run.py --steps 20 --reps 1 > $OUT/tail_1m_$v.txt 2> $OUT/tail.err || { echo tail failed; tail $OUT/tail.err; exit 1; }
done
tail -21 $OUT/tail_1m_0.02.txt
