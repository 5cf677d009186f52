#!/bin/bash
# round 5: the one-wave solve's stage stamps on the driver workload's captured statistics (30 passes)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 300 python3 scripts/capture_stats.py $OUT/st.npz 1000000 3 30 > $OUT/capture.log 2>&1 || { echo capture failed; tail $OUT/capture.log; exit 1; }
python3 -c "
import numpy as np; z=np.load('$OUT/st.npz'); s=z['stats'][:, :74]; p=z['poses']
np.ascontiguousarray(s, dtype=np.float64).tofile('$OUT/stats.bin'); np.ascontiguousarray(p.reshape(len(p), -1), dtype=np.float64).tofile('$OUT/poses.bin')"
for b in ${PROBES:-solve_bench}; do
  echo "== $b"
  timeout -k 10 60 scripts/probes/$b $OUT/stats.bin $OUT/poses.bin | tee $OUT/$b.txt
done
