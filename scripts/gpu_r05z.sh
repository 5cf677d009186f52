#!/bin/bash
# round 5 end, second call: the side lines, the tail breakdowns (tail build) and the launch-gap probe
set -o pipefail
export TMPDIR=/tmp
bash scripts/round_extras.sh r05z_extras || exit 1
SKIP_BENCH=1 bash scripts/gpu_tail.sh r05z_tail || exit 1
