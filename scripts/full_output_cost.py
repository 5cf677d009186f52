"""Per-iteration cost of the drop-in gicp() at 1M/1M with full_output=True (the 7-tuple: poses, top-5 det(W)
per iteration on the device, lazy rotated covariances) vs full_output=False (< 2x).
Each call runs 30 iterations (tolerance 0: no early stop); the time spent in the cloud setup calls
(Engine.set_target / set_source / covariances, synchronous) is measured and subtracted; best of 3.
Prints one JSON line."""
import json, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "generalized-icp_amd"), os.path.join(os.path.dirname(__file__), "..")]
import gicp
from gicp import synthetic as S

setup = [0.0]
for name in ("set_target", "set_source", "covariances"):
    f = getattr(gicp.Engine, name)

    def timed(self, *a, _f=f, **k):
        t0 = time.perf_counter()
        try:
            return _f(self, *a, **k)
        finally:
            setup[0] += time.perf_counter() - t0
    setattr(gicp.Engine, name, timed)

src, tgt, _ = S.scene_pair_3d(1_000_000)
kw = dict(tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0, verbose=False)
ITERS = 30
gicp.gicp(src, tgt, max_iterations=3, full_output=False, **kw)   # warm-up (library, first allocations)
res = {}
for full in (False, True):
    best = 1e30
    for _ in range(3):
        setup[0] = 0.0
        t0 = time.perf_counter()
        out = gicp.gicp(src, tgt, max_iterations=ITERS, full_output=full, **kw)
        best = min(best, time.perf_counter() - t0 - setup[0])
        assert len(out[1]) == ITERS + 1
    res["full_output" if full else "plain"] = best / ITERS * 1e3
res["ratio"] = res["full_output"] / res["plain"]
res["unit"] = ("ms per iteration (drop-in gicp(), 1M/1M 3-D room, 30 iterations, host wall clock minus the cloud "
               "setup calls; compare Engine.align's device-resident loop in bench.json)")
print(json.dumps(res))
