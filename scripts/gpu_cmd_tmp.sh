set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03n
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc = 0 ] || { grep -E "FAIL|Error" $OUT/pytest_gpu.log | head; exit 1; }
bash scripts/bench_variants.sh r03n/ab 3 "GICP_LIB_VARIANT=nores" "X=0" > $OUT/ab.txt 2>&1 || { tail $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
BENCH_ARGS="--shard-sim 8" bash scripts/bench_variants.sh r03n/ab8 2 "GICP_LIB_VARIANT=nores" "X=0" > $OUT/ab8.txt 2>&1 || { tail $OUT/ab8.txt; exit 1; }
cat $OUT/ab8.txt
timeout -k 10 400 python scripts/twod_1m_vs_oracle.py > $OUT/twod_1m.json 2> $OUT/twod.err || { tail $OUT/twod.err; exit 1; }
cat $OUT/twod_1m.json
