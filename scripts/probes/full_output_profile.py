"""cProfile of the drop-in gicp() at 1M/1M, full_output=True vs False (30 iterations)."""
import cProfile, io, os, pstats, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "generalized-icp_amd"),
                os.path.join(os.path.dirname(__file__), "..", "..")]
import gicp
from gicp import synthetic as S

src, tgt, _ = S.scene_pair_3d(1_000_000)
kw = dict(tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0, verbose=False)
gicp.gicp(src, tgt, max_iterations=3, **kw)
for full in (False, True):
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    gicp.gicp(src, tgt, max_iterations=30, full_output=full, **kw)
    pr.disable()
    print(f"full_output={full}: {time.perf_counter() - t0:.4f} s")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(22)
    print(s.getvalue())
