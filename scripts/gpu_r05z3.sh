#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r05z3
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py -m gpu -k "2d_1m" > gpurun_out/r05z3/tests.log 2>&1 || { tail -40 gpurun_out/r05z3/tests.log; exit 1; }
tail -3 gpurun_out/r05z3/tests.log
