"""CPU simulation (round 3): share of source lanes with no target within d_c (rejected, gicp.py:136) per
pose between identity and ground truth on the 1M/1M bench scene, the share of 64-point waves holding one,
and the mean wave search radius with and without them.  python scripts/sim/rejected_lanes.py"""
import sys, time, numpy as np
from scipy.spatial import cKDTree
sys.path[:0] = ["generalized-icp_amd", "."]
from gicp import synthetic as S
n = 1_000_000
src, tgt, Tgt = S.scene_pair_3d(n)
tree = cKDTree(tgt)
def spread(x):
    x = x.astype(np.uint64) & 0x3FF
    x = (x | (x << 16)) & 0x30000FF; x = (x | (x << 8)) & 0x300F00F
    x = (x | (x << 4)) & 0x30C30C3; x = (x | (x << 2)) & 0x9249249
    return x
lo = src.min(0); sc = 1023 / (src.max(0) - lo).max()
g = np.clip(((src - lo) * sc), 0, 1023).astype(np.uint64)
order = np.argsort(spread(g[:,0]) | (spread(g[:,1]) << 1) | (spread(g[:,2]) << 2), kind="stable")
src = src[order]
from scipy.spatial.transform import Rotation as Rot
for frac in (0.0, 0.5, 0.8, 0.95):
    # pose a fraction of the way to ground truth
    rv = Rot.from_matrix(Tgt[:3,:3]).as_rotvec() * frac
    T = np.eye(4); T[:3,:3] = Rot.from_rotvec(rv).as_matrix(); T[:3,3] = Tgt[:3,3]*frac
    p = src @ T[:3,:3].T + T[:3,3]
    d1, _ = tree.query(p, workers=8, distance_upper_bound=2.0)
    rej = d1 > 0.5
    nw = len(p)//64
    rw = rej[:nw*64].reshape(nw,64)
    dd = np.minimum(d1[:nw*64].reshape(nw,64), 0.5)
    wmax_all = dd.max(1)
    acc = np.where(rw, 0, dd)
    wmax_acc = acc.max(1)
    print(f"pose {frac:.2f}: rejected lanes {rej.mean()*100:5.1f}%  waves with a rejected lane {rw.any(1).mean()*100:5.1f}%  "
          f"mean wave radius {wmax_all.mean():.3f} m -> {wmax_acc.mean():.3f} m w/o rejected; mean accepted d1 {d1[~rej].mean():.3f}", flush=True)
