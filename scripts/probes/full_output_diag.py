"""Where the drop-in's 7-tuple time goes at 1M/1M: Engine.align with and without the trace / top-k,
timed on the host (best of 3), after a warm-up."""
import json, os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "generalized-icp_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import numpy as np
import gicp
from gicp import synthetic as S

src, tgt, _ = S.scene_pair_3d(1_000_000)
p = gicp.default_params(3, max_iterations=30, tolerance=0.0, max_distance_correspondence=0.5,
                        max_distance_nearest_neighbors=1.0)
eng = gicp.Engine(0)
eng.set_target(tgt, p)
eng.set_source(src, p)
res = {}
for name, kw in (("align", {}), ("trace", dict(trace=True)), ("trace_top5", dict(trace=True, top_k=5)),
                 ("align_again", {})):
    best = 1e9
    for _ in range(3):
        eng.reset_cache()
        t0 = time.perf_counter()
        eng.align(None, p, **kw)
        best = min(best, time.perf_counter() - t0)
    res[name] = best / 30 * 1e3
print(json.dumps(res))
