#!/bin/bash
# Round-4 working GPU call: grid parity, A/B against the variants built beside the library, stamps, side lines.
#   scripts/gpu_r04.sh OUT "VARIANT_ENVS..."      (OUT under gpurun_out/)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { echo tests failed; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
if [ $# -gt 0 ]; then
  BENCH_ARGS="--steps 20" timeout -k 10 700 bash scripts/bench_variants.sh ${O#gpurun_out/}/ab 3 "$@" > $O/ab.txt 2>&1 || { echo ab failed; tail $O/ab.txt; exit 1; }
  grep -v "^ *$" $O/ab.txt
fi
if [ -f generalized-icp_amd/gicp/libgicp_hip_stamps.so ]; then
  GICP_LIB_VARIANT=stamps timeout -k 10 200 python scripts/pass_diag.py 1000000 12 > $O/stamps_diag.txt 2> $O/stamps.txt || { echo stamps failed; exit 1; }
  grep -E "all  |slowest" $O/stamps.txt | head -12
fi
timeout -k 10 300 python bench.py --n 100000 --no-cpu-baseline > $O/bench_c2.json 2> $O/c2.err || { echo c2 failed; exit 1; }
timeout -k 10 400 python bench_odometry.py > $O/bench_odometry_staged.json 2> $O/odo.err || { echo odometry failed; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 2 --share-gpu --no-cpu-baseline --steps 20 > $O/share2.json 2> $O/share2.err || { echo share failed; tail -3 $O/share2.err; exit 1; }
timeout -k 10 300 python3 bench.py --shard-sim 8 --no-cpu-baseline > $O/sim8.json 2> $O/sim8.err || { echo sim8 failed; exit 1; }
for f in bench_c2 share2 sim8; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',round(d['value'],1),d['unit'],'k_corr',round(d['roofline']['kernel_avg_ms']*1e3,1),'us', d['passes']['k_corr_us_per_iteration'])"; done
head -c 400 $O/bench_odometry_staged.json; echo
