#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z2
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_extensions.py -m gpu -k "smaller_source_tiles" > gpurun_out/r05z2/tests.log 2>&1 || { tail -40 gpurun_out/r05z2/tests.log; exit 1; }
tail -4 gpurun_out/r05z2/tests.log
