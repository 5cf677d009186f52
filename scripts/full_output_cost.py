"""Per-iteration cost of the drop-in gicp() at 1M/1M with full_output=True (the 7-tuple: poses, top-5
det(W) per iteration recorded on the device, lazy rotated covariances) vs full_output=False (VERDICT
r01/r02: ratio < 2, plain <= 0.095 ms).  The marginal cost of an iteration is measured directly:
(wall of a K-iteration call - wall of a 0-iteration call) / K, K = 60, tolerance 0 (no early stop), best of
5 each, the four call kinds interleaved -- the cloud setup and the 7-tuple's covariance copies are the same in
both calls and cancel (with K = 30 and best of 3 the ~20 ms setup's jitter left the ratio within +-0.9).
Prints one JSON line."""
import json, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "generalized-icp_amd"), os.path.join(os.path.dirname(__file__), "..")]
import gicp
from gicp import synthetic as S

src, tgt, _ = S.scene_pair_3d(1_000_000)
kw = dict(tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0, verbose=False)
gicp.gicp(src, tgt, max_iterations=3, full_output=True, **kw)   # warm-up (library, first allocations)


K, REPS = 60, 5
best = {}
for _ in range(REPS):
    for full in (False, True):
        for iters in (0, K):
            t0 = time.perf_counter()
            out = gicp.gicp(src, tgt, max_iterations=iters, full_output=full, **kw)
            dt = time.perf_counter() - t0
            assert len(out[1]) == iters + 1
            best[(full, iters)] = min(best.get((full, iters), 1e30), dt)
res = {}
for full in (False, True):
    key = "full_output" if full else "plain"
    res[key] = (best[(full, K)] - best[(full, 0)]) / K * 1e3
    res[key + f"_call_{K}_ms"] = best[(full, K)] * 1e3
res["ratio"] = res["full_output"] / res["plain"]
res["unit"] = ("ms per iteration (drop-in gicp(), 1M/1M 3-D room: (wall of a 60-iteration call - wall of a "
               "0-iteration call) / 60, best of 5, interleaved; *_call_60_ms = a whole 60-iteration call incl. setup and the "
               "7-tuple's covariance copies; compare Engine.align's device-resident loop in bench.json)")
print(json.dumps(res))
