"""Diagnostic: per-wave phase cycles and event counters of k_corr (libgicp_hip_stamps.so).

    GICP_LIB_VARIANT=stamps python scripts/stamps_run.py [--n 1000000] [--iters 10]

Prints the [stamps] lines of one pass at identity (first iteration) and one at the pose
reached after --iters fixed iterations (steady state, candidate lists warm)."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generalized-icp_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import bench  # noqa: E402
import gicp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
src, tgt, Tgt, kw, name = bench.workload(a.n, 3)
eng = gicp.Engine(0)
p = gicp.default_params(3, fixed_iterations=1, max_iterations=a.iters, **kw)
eng.set_target(tgt, p)
eng.set_source(src, p)
print("== first pass (identity)", file=sys.stderr, flush=True)
eng.iterate(np.eye(4))
T, res = eng.align(None, p)
print("== steady state (after %d iterations)" % a.iters, file=sys.stderr, flush=True)
eng.iterate(T)
eng.iterate(T)
print("== early (after 2 iterations from identity, fresh lists)", file=sys.stderr, flush=True)
p.max_iterations = int(os.environ.get("EARLY_ITERS", "2"))
T2, _ = eng.align(None, p)
eng.iterate(T2)
