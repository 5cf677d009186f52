#!/bin/bash
# round 5: lanes without a last match start their descent at the seed tile's nearest point (main, default) vs
# GICP_NO_SEED_DESCENT=1 (same build) vs the revision before (base); parity tests of the pass first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05p
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu > gpurun_out/r05p/tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05p/tests.log; exit 1; }
tail -1 gpurun_out/r05p/tests.log
BENCH_ARGS="--steps 20" bash scripts/bench_variants.sh r05p_1m 2 "X=0" "GICP_NO_SEED_DESCENT=1" "GICP_LIB_VARIANT=base" || exit 1
BENCH_ARGS="--n 100000" bash scripts/bench_variants.sh r05p_c2 2 "X=0" "GICP_LIB_VARIANT=base" || exit 1
for v in main base; do
  if [ $v = main ]; then unset GICP_LIB_VARIANT; else export GICP_LIB_VARIANT=$v; fi
  timeout -k 10 300 python3 bench_odometry.py > gpurun_out/r05p/odo_$v.json 2> gpurun_out/r05p/odo_$v.err || { echo odo failed; tail gpurun_out/r05p/odo_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r05p/odo_$v.json'));print('C5 $v',round(d['frames_per_s'],1),'fps align',round(d['align_ms_per_frame'],3),'it/frame',round(d['iterations_per_frame'],2))"
done
