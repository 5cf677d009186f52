"""Capture the per-iteration statistics of a registration (for solver experiments on the host).

    python scripts/capture_stats.py OUT.npz [N] [DIM] [ITERS]

Runs the bench workload from the identity with the host solve between passes (gicp_iterate +
gicp_solve_pose: the same iterates as gicp_align's device loop up to 1e-12) and saves the statistics
and poses of every pass.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generalized-icp_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import gicp  # noqa: E402

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
dim = int(sys.argv[3]) if len(sys.argv) > 3 else 3
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 30
src, tgt, Tgt, kw, name = bench.workload(n, dim)
p = gicp.default_params(dim, fixed_iterations=1, **kw)
eng = gicp.Engine(0)
eng.set_target(tgt, p)
eng.set_source(src, p)
T = np.eye(dim + 1)
stats, poses = [], []
for it in range(iters):
    st = eng.iterate(T)
    stats.append(st.copy())
    poses.append(T.copy())
    T, loss = gicp.solve_pose(st, T)
np.savez(out, stats=np.array(stats), poses=np.array(poses), workload=name)
print("saved", out, len(stats))
