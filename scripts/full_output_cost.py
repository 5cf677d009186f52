"""Per-iteration cost of the drop-in gicp() at 1M/1M with full_output=True (the 7-tuple: poses, top-5
det(W) per iteration recorded on the device, lazy rotated covariances) vs full_output=False (VERDICT
r01/r02: ratio < 2, plain <= 0.095 ms).  The marginal cost of an iteration is measured directly:
(wall of a 30-iteration call - wall of the adjacent 0-iteration call) / 30, tolerance 0 (no early stop),
median over 7 such pairs per mode, modes interleaved -- the cloud setup (~20 ms, jittery) and the 7-tuple's
covariance copies are the same in both calls of a pair and cancel (best-of-N of each call kind separately left
the ratio within +-0.9 on the same code).
Prints one JSON line."""
import json, os, sys, time
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "generalized-icp_amd"), os.path.join(os.path.dirname(__file__), "..")]
import gicp
from gicp import synthetic as S

src, tgt, _ = S.scene_pair_3d(1_000_000)
kw = dict(tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0, verbose=False)
gicp.gicp(src, tgt, max_iterations=3, full_output=True, **kw)   # warm-up (library, first allocations)


K, REPS = 30, 7
diffs = {False: [], True: []}
calls = {False: [], True: []}
for _ in range(REPS):
    for full in (False, True):
        t = []
        for iters in (0, K):
            t0 = time.perf_counter()
            out = gicp.gicp(src, tgt, max_iterations=iters, full_output=full, **kw)
            t.append(time.perf_counter() - t0)
            assert len(out[1]) == iters + 1
        diffs[full].append((t[1] - t[0]) / K * 1e3)   # one adjacent pair: setup jitter of this pair only
        calls[full].append(t[1] * 1e3)
res = {}
for full in (False, True):
    key = "full_output" if full else "plain"
    res[key] = float(np.median(diffs[full]))
    res[key + "_pairs"] = [round(x, 4) for x in diffs[full]]
    res[key + f"_call_{K}_ms"] = float(np.median(calls[full]))
res["ratio"] = res["full_output"] / res["plain"]
res["unit"] = ("ms per iteration (drop-in gicp(), 1M/1M 3-D room: median over 7 adjacent pairs of (wall of a 30-iteration "
               "call - wall of a 0-iteration call) / 30; *_call_30_ms = median whole 30-iteration call incl. setup and the "
               "7-tuple's covariance copies; compare Engine.align's device-resident loop in bench.json)")
print(json.dumps(res))
