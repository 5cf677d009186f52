"""C1 latency line: the drop-in gicp() on the reference's own
2-D scan pairs -- the robot demo's raycast pairs (robot-visualization.py:157-162, 90 and 360 rays) and the
static demo's pairs (visualization.py:169-196) -- as committed fixtures (tests/golden/*.npz, captured from
gicp.py itself by tests/golden/make_golden.py).

    python bench_small.py [--reps 7] [--warmup 2]

For each pair and mode ('faithful': the GPU recomputes the transformed source's covariances, then
correspondences + W, and scipy's fmin_cg minimises the reference's own per-point loss on the host every
iteration, gicp.py:119-154; 'fast': one GPU reduction to the sufficient statistics per iteration + fmin_cg
on the closed form) it times whole calls (median of --reps after --warmup), the iterations they ran, the
host fmin_cg time inside them (the inner solve, gicp.py:148-154), and checks the endpoint against the
reference's endpoint ensemble (1e-4 rad / 1e-3 px).  The reference's own time per pair
(gicp.py on one core of the build container) is printed beside it as context.
Prints one JSON line.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "generalized-icp_amd"), ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

PAIRS = ["robot_p0_r360", "robot_p1_r360", "robot_p2_r360", "robot_p0_r90", "robot_p1_r90", "robot_p2_r90",
         "vis_s0", "vis_s1", "vis_s2", "vis_s3", "vis_s5"]
# gicp.py, 1 core of the build container: robot pairs 35-175 ms per call (2-3 iterations),
# visualization.py pairs ~40 ms per iteration (13-17 iterations)
REFERENCE = {"robot_pair_ms_per_call": [35.0, 175.0], "vis_pair_ms_per_iteration": 40.0,
             "source": "BASELINE.md §3 (gicp.py imported unchanged, taskset -c 0, build container)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    import gicp
    from golden_util import DIVERGENT, in_ensemble, kwargs, load

    # time spent in the host inner solves (wrapped, same functions gicp() calls)
    spent = {"cg": 0.0}
    real = {"faithful": gicp._cg_inner_faithful, "fast": gicp._cg_inner}

    def timed(fn):
        def w(*args, **kw):
            t0 = time.perf_counter()
            try:
                return fn(*args, **kw)
            finally:
                spent["cg"] += time.perf_counter() - t0
        return w

    gicp._cg_inner_faithful = timed(real["faithful"])
    gicp._cg_inner = timed(real["fast"])
    rows = []
    for name in PAIRS:
        fx = load(name)
        kw = kwargs(fx)
        for mode in ("faithful", "fast"):
            def call():
                return gicp.gicp(fx["source"], fx["target"], mode=mode, full_output=True, verbose=False, **kw)
            for _ in range(a.warmup):
                call()
            walls, cgs = [], []
            for _ in range(a.reps):
                spent["cg"] = 0.0
                t0 = time.perf_counter()
                out = call()
                walls.append((time.perf_counter() - t0) * 1e3)
                cgs.append(spent["cg"] * 1e3)
            T = out[0]
            iters = len(out[1]) - 1   # poses after T0: the updates applied
            ok, (rot, tr) = in_ensemble(T, fx["ens_T"])
            ms = statistics.median(walls)
            cg = statistics.median(cgs)
            # iterations the loop ran: the updates applied, plus the converged one (its update is not applied)
            ran = iters + (1 if iters < int(fx["max_iterations"]) else 0)
            rows.append({"pair": name, "mode": mode, "points": [len(fx["source"]), len(fx["target"])],
                         "ms_per_call": round(ms, 3), "ms_per_call_min_max": [round(min(walls), 3), round(max(walls), 3)],
                         "iterations": ran, "ms_per_iteration": round(ms / max(1, ran), 3),
                         "host_cg_ms_per_call": round(cg, 3), "host_cg_share": round(cg / ms, 3),
                         "reference_iterations": int(fx["n_iter"]),
                         "in_reference_ensemble": bool(ok) if name not in DIVERGENT else None,
                         "ensemble_distance": [float(rot), float(tr)]})
    gicp._cg_inner_faithful, gicp._cg_inner = real["faithful"], real["fast"]
    summ = {}
    for mode in ("faithful", "fast"):
        rs = [r for r in rows if r["mode"] == mode]
        robot = [r for r in rs if r["pair"].startswith("robot_")]
        summ[mode] = {"median_ms_per_call_robot": statistics.median(r["ms_per_call"] for r in robot),
                      "median_ms_per_iteration": statistics.median(r["ms_per_iteration"] for r in rs),
                      "median_host_cg_share": statistics.median(r["host_cg_share"] for r in rs),
                      "in_ensemble": f"{sum(1 for r in rs if r['in_reference_ensemble'])}/"
                                     f"{sum(1 for r in rs if r['in_reference_ensemble'] is not None)}"}
    print(json.dumps({"metric": "C1 drop-in gicp() latency on the reference's 2-D scan pairs", "unit": "ms",
                      "higher_is_better": False, "reps": a.reps, "warmup": a.warmup, "summary": summ,
                      "reference_gicp_py": REFERENCE, "pairs": rows,
                      "note": "whole drop-in calls incl. uploads, covariances and the 7-tuple; faithful = the "
                              "reference's trajectory (host fmin_cg on its per-point loss every iteration)"}))


if __name__ == "__main__":
    main()
