#!/bin/bash
# round 5: descent's first row half requested with the last match's coordinates (main) vs HEAD (base)
set -o pipefail
export TMPDIR=/tmp
bash scripts/bench_variants.sh r05i 3 "X=0" "GICP_LIB_VARIANT=base" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05i_c2 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
