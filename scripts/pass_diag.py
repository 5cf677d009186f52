"""Per-pass diagnostics of the 1M/1M registration (bench workload): pass k runs at the pose the host
solve of pass k-1 gave (the same sequence gicp_align runs), printing the pass's wall time (host, incl.
launch + sync), pairs screened, list rebuilds, graph-proved lanes and walking tiles.
    python scripts/pass_diag.py [n] [passes]          (GICP_NO_GRAPH=1 etc. select variants)"""
import os, sys, time
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "generalized-icp_amd"), os.path.join(os.path.dirname(__file__), "..")]
import gicp
from gicp import synthetic as S

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 30
src, tgt, Tgt = S.scene_pair_3d(n)
p = gicp.default_params(3, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
e = gicp.Engine(0)
e.set_target(tgt, p)
e.set_source(src, p)
T = np.eye(4)
for rep in range(2):
    e.reset_cache()
    T = np.eye(4)
    rows = []
    for k in range(passes):
        t0 = time.perf_counter()
        st = e.iterate(T)
        dt = time.perf_counter() - t0
        inf = e.pass_info()
        Tn, _ = gicp.solve_pose(st, T)
        step = np.linalg.norm(Tn[:3, 3] - T[:3, 3])
        rows.append(f"pass {k:2d} {dt*1e6:7.0f} us  step {step*100:7.3f} cm  pairs/pt {inf['pairs']/n:7.1f}  "
                    f"rebuilds {int(inf['list_rebuilds']):6d}  graph {int(inf['graph_proved']):8d}  "
                    f"walked {int(inf['walked_tiles']):6d}  amb {int(inf['ambiguous'])}  acc {int(st[73])}")
        T = Tn
    if rep == 1:
        print("\n".join(rows))
print("final error", S.rotation_angle_error(T, Tgt), S.translation_error(T, Tgt))
