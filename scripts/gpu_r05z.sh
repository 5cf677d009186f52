#!/bin/bash
# round 5 end, second call: the side lines, the tail breakdowns (tail build) and the launch-gap probe
set -o pipefail
export TMPDIR=/tmp
bash scripts/round_extras.sh r05z_extras || exit 1
SKIP_BENCH=1 bash scripts/gpu_tail.sh r05z_tail || exit 1
# where the setup's time goes (cloud build stages, GICP_VERBOSE=1), the 1M/1M bench's clouds
GICP_VERBOSE=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r05z_tail/setup_verbose.json 2> gpurun_out/r05z_tail/setup_verbose.txt || { echo verbose failed; tail gpurun_out/r05z_tail/setup_verbose.txt; exit 1; }
grep "\[gicp\]" gpurun_out/r05z_tail/setup_verbose.txt | head -8
