import os, sys, time
sys.path.insert(0, "generalized-icp_amd")
import numpy as np
import gicp
from gicp import synthetic as S
frames = list(S.lidar_stream(6))
p = gicp.default_params(3, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
e = gicp.Engine(0)
for k, (scan, pose) in enumerate(frames):
    t0 = time.perf_counter()
    e.set_target(scan, p)
    t1 = time.perf_counter()
    print(f"frame {k}: set_target {1e3*(t1-t0):.2f} ms", flush=True)
