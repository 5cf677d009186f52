"""Where a C5 frame's time goes: per-stage cloud-build timings (GICP_VERBOSE=1
stderr lines), then the frame loop's pieces timed on the host: build alone, align alone, align with a
staged build running beside it, and the commit wait."""
import os, sys, time
os.environ.setdefault("GICP_VERBOSE", "0")
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "generalized-icp_amd")]
import numpy as np
import gicp
from gicp import synthetic as S

frames = [f for f, _ in S.lidar_stream(14)]
p = gicp.default_params(3, max_iterations=30, tolerance=1e-6, max_distance_correspondence=0.5,
                        max_distance_nearest_neighbors=1.0)
eng = gicp.Engine(0)
eng.set_target(frames[0], p)
eng.target_to_source()
eng.set_target(frames[1], p)
eng.align(None, p)
t_build, t_align, t_align_staged, t_commit, t_stage = [], [], [], [], []
for k in range(2, 13):
    # build alone (synchronous set_target)
    eng.target_to_source()
    t0 = time.perf_counter(); eng.set_target(frames[k], p); t_build.append(time.perf_counter() - t0)
    t0 = time.perf_counter(); T, r = eng.align(None, p); t_align.append(time.perf_counter() - t0)
    # align with the next frame's build staged beside it
    t0 = time.perf_counter(); eng.stage_target(frames[k + 1], p); t_stage.append(time.perf_counter() - t0)
    eng.reset_cache()
    t0 = time.perf_counter(); T2, r2 = eng.align(None, p); t_align_staged.append(time.perf_counter() - t0)
    t0 = time.perf_counter(); eng.commit_target(); t_commit.append(time.perf_counter() - t0)
    assert np.array_equal(T, T2)
    eng.set_source(frames[k], p)   # undo the promotion: keep the loop's pairing simple
ms = lambda v: f"{np.median(v) * 1e3:.3f}"
print(f"build alone {ms(t_build)} ms | align alone {ms(t_align)} ms ({r['iterations']} it) | stage call {ms(t_stage)} ms"
      f" | align beside staged build {ms(t_align_staged)} ms | commit wait {ms(t_commit)} ms")
