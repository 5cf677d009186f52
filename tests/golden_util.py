"""Helpers for the golden fixtures captured from the reference (tests/golden/make_golden.py)."""
import glob
import math
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# fixtures whose reference run diverges (vis seed 4): per-iteration vectors only
DIVERGENT = {"vis_s4"}


def names():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def kwargs(fx):
    return dict(max_iterations=int(fx["max_iterations"]), tolerance=float(fx["tolerance"]),
                max_distance_correspondence=float(fx["max_distance_correspondence"]),
                max_distance_nearest_neighbors=float(fx["max_distance_nearest_neighbors"]))


def pose_err(Ta, Tb):
    d = Ta.shape[0] - 1
    if d == 2:
        ang = abs(math.remainder(math.atan2(Ta[1, 0], Ta[0, 0]) - math.atan2(Tb[1, 0], Tb[0, 0]), 2 * math.pi))
    else:
        c = (np.trace(Ta[:3, :3].T @ Tb[:3, :3]) - 1) / 2
        ang = math.acos(max(-1.0, min(1.0, c)))
    return ang, float(np.linalg.norm(Ta[:d, d] - Tb[:d, d]))


def in_ensemble(T, ens, rot_tol=1e-4, trans_tol=1e-3):
    """SURVEY.md §8(c) grading rule: within 1e-4 rad and 1e-3 units of ANY ensemble member."""
    best = min(pose_err(T, E) for E in ens)
    ok = any(a <= rot_tol and t <= trans_tol for a, t in (pose_err(T, E) for E in ens))
    return ok, best
