#!/bin/bash
# The one-wave solve alone on the driver workload's captured pass statistics: k_solve<3> back to back and its
# stage stamps (scripts/probes/solve_bench[_plain], built by scripts/probes/build_solve_bench.sh).
#   scripts/solve_probe.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/solve}
mkdir -p $OUT
timeout -k 10 300 python3 scripts/capture_stats.py $OUT/st.npz 1000000 3 30 > $OUT/capture.log 2>&1 || { echo capture failed; tail $OUT/capture.log; exit 1; }
python3 -c "
import numpy as np; z=np.load('$OUT/st.npz'); s=z['stats'][:, :74]; p=z['poses']
np.ascontiguousarray(s, dtype=np.float64).tofile('$OUT/stats.bin'); np.ascontiguousarray(p.reshape(len(p), -1), dtype=np.float64).tofile('$OUT/poses.bin')" || exit 1
for b in solve_bench_plain solve_bench; do
  echo "== $b"
  timeout -k 10 60 scripts/probes/$b $OUT/stats.bin $OUT/poses.bin | tee $OUT/$b.txt || exit 1
done
