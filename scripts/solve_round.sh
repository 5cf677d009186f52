#!/bin/bash
# k_solve probe (stamped + plain) and a kernel trace of the default bench.  Output: gpurun_out/$1/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sv}
mkdir -p $OUT
D=scripts/probes/data
timeout -k 10 60 scripts/probes/solve_bench_plain $D/st_1m.bin $D/T_1m.bin > $OUT/plain.txt 2>&1 || { echo plain failed; exit 1; }
timeout -k 10 60 scripts/probes/solve_bench $D/st_1m.bin $D/T_1m.bin > $OUT/stamped.txt 2>&1 || { echo stamped failed; exit 1; }
cat $OUT/plain.txt; tail -31 $OUT/stamped.txt
bash scripts/trace_run.sh ${1:-sv}/tr
