"""Per-iteration cost of the drop-in gicp() at 1M/1M: the library's own wall time
of the registration loop (gicp_result.wall_ms of the gicp_align_trace call gicp() makes, read back with
gicp.last_result(); cloud setup and the 7-tuple's assembly are outside it) divided by the iterations, for
full_output=False (poses + losses recorded per iteration) and full_output=True (plus the top-5 det(W)
rows), against Engine.align's wall_ms on the same clouds (the bench's loop, nothing recorded).  Every
loop starts cold (fresh clouds in gicp(); reset_cache before Engine.align), 30 iterations, tolerance 0
(no early stop).  REPS calls of each kind, interleaved; median and spread reported.  One JSON line."""
import json, os, sys
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "generalized-icp_amd"), os.path.join(os.path.dirname(__file__), "..")]
import gicp
from gicp import synthetic as S

K, REPS = 30, 7
src, tgt, _ = S.scene_pair_3d(1_000_000)
kw = dict(tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0, verbose=False)
gicp.gicp(src, tgt, max_iterations=3, full_output=True, **kw)   # warm-up (library, first allocations)
eng = gicp.Engine(0)
p = gicp.default_params(3, max_iterations=K, tolerance=0.0, max_distance_correspondence=0.5,
                        max_distance_nearest_neighbors=1.0)
eng.set_target(tgt, p)
eng.set_source(src, p)
eng.align(None, p)
per = {"plain": [], "full_output": [], "engine_align": []}
for _ in range(REPS):
    for key in per:
        if key == "engine_align":
            eng.reset_cache()
            _, r = eng.align(None, p)
        else:
            out = gicp.gicp(src, tgt, max_iterations=K, full_output=(key == "full_output"), **kw)
            r = gicp.last_result()
            assert len(out[1]) == K + 1
        assert int(r["iterations"]) == K
        per[key].append(r["wall_ms"] / K)
eng.close()
res = {k: float(np.median(v)) for k, v in per.items()}
for k, v in per.items():
    res[k + "_samples"] = [round(x, 4) for x in v]
    res[k + "_spread"] = round(float(np.max(v) - np.min(v)), 4)
res["plain_vs_engine"] = res["plain"] / res["engine_align"]
res["full_vs_plain"] = res["full_output"] / res["plain"]
res["unit"] = ("ms per iteration: gicp_result.wall_ms / 30 of each call (the library's wall time of its 30-iteration "
               "loop, cold start, 1M/1M 3-D room); median over %d calls per kind, interleaved" % REPS)
print(json.dumps(res))
