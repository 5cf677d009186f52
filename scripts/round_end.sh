#!/bin/bash
# Round-end GPU call: parity tests + smoke, the profile set of the default bench, the side lines.
#   scripts/round_end.sh TAG   -> gpurun_out/TAG_{tests,prof,extras}/   (SKIP_EXTRAS=1: no side lines)
set -o pipefail
export TMPDIR=/tmp
T=${1:-r05}
PD=${PD:-profiles/r05}
mkdir -p gpurun_out/${T}_tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/${T}_tests/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_tests/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_tests/smoke.log 2>&1 || { echo smoke failed; exit 1; }
bash scripts/profile_round.sh ${T}_prof $PD || exit 1
[ "${SKIP_EXTRAS:-0}" = 1 ] || bash scripts/round_extras.sh ${T}_extras || exit 1
cat gpurun_out/${T}_prof/iterations.txt
