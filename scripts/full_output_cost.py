"""Per-iteration cost of the drop-in gicp() at 1M/1M with full_output=True (the 7-tuple: poses, top-5
det(W) per iteration recorded on the device, lazy rotated covariances) vs full_output=False (VERDICT
r01/r02: ratio < 2, plain <= 0.095 ms).  The marginal cost of an iteration is measured directly:
(wall of a 30-iteration call - wall of a 0-iteration call) / 30, tolerance 0 (no early stop), best
of 3 each -- the cloud setup and the 7-tuple's covariance copies are the same in both calls and cancel.
Prints one JSON line."""
import json, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "generalized-icp_amd"), os.path.join(os.path.dirname(__file__), "..")]
import gicp
from gicp import synthetic as S

src, tgt, _ = S.scene_pair_3d(1_000_000)
kw = dict(tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0, verbose=False)
gicp.gicp(src, tgt, max_iterations=3, full_output=True, **kw)   # warm-up (library, first allocations)


def wall(iters, full):
    best = 1e30
    for _ in range(3):
        t0 = time.perf_counter()
        out = gicp.gicp(src, tgt, max_iterations=iters, full_output=full, **kw)
        best = min(best, time.perf_counter() - t0)
        assert len(out[1]) == iters + 1
    return best


res = {}
for full in (False, True):
    t0, t30 = wall(0, full), wall(30, full)
    key = "full_output" if full else "plain"
    res[key] = (t30 - t0) / 30 * 1e3
    res[key + "_call_30_ms"] = t30 * 1e3
res["ratio"] = res["full_output"] / res["plain"]
res["unit"] = ("ms per iteration (drop-in gicp(), 1M/1M 3-D room: (wall of a 30-iteration call - wall of a "
               "0-iteration call) / 30, best of 3; *_call_30_ms = a whole 30-iteration call incl. setup and the "
               "7-tuple's covariance copies; compare Engine.align's device-resident loop in bench.json)")
print(json.dumps(res))
