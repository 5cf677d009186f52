"""CPU simulation: how many source lanes / waves would a target-kNN-graph certificate settle in
the moving passes of the 1M/1M registration, on top of the gap certificates?

Graph certificate of a lane with last match jp (the previous pass's nearest): candidates
{jp} + N_K(jp) (jp's K nearest targets), j* = the nearest candidate.  Any target t closer to p'
than j* has d(jp, t) <= d(jp, p') + d(p', t) < d(p', jp) + d(p', j*); if that is < r_K(jp) (the
K-th neighbour distance) t is a candidate, so j* is the exact nearest.
"""
import sys, time
import numpy as np
from scipy.spatial import cKDTree
sys.path[:0] = ["generalized-icp_amd", "."]
import gicp
from gicp import synthetic as S
from oracle import gicp_oracle as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 12
dc, dn = 0.5, 1.0
src, tgt, Tgt = S.scene_pair_3d(n)
t0 = time.time()
tree = cKDTree(tgt)
Cs, _ = O.covariances(src, dn, workers=8)
Ct, _ = O.covariances(tgt, dn, workers=8)
# source order: Morton-ish via the target tiles is not available here; sort the source by a 3-D Morton code
lo = src.min(0); sc = 1023 / (src.max(0) - lo).max()
g = ((src - lo) * sc).astype(np.uint64)
def spread(x):
    x &= 0x3FF
    x = (x | (x << 16)) & 0x30000FF
    x = (x | (x << 8)) & 0x300F00F
    x = (x | (x << 4)) & 0x30C30C3
    x = (x | (x << 2)) & 0x9249249
    return x
code = spread(g[:, 0]) | (spread(g[:, 1]) << 1) | (spread(g[:, 2]) << 2)
order = np.argsort(code, kind="stable")
src, Cs = src[order], Cs[order]
Ks = (8, 12, 16, 20)
dK, iK = tree.query(tgt, k=max(Ks) + 1, workers=8)   # self first
print(f"setup {time.time()-t0:.1f}s", flush=True)
T = np.eye(4)
prev = None
for it in range(iters):
    moved = S.transform_points(src, T)
    d2, j2 = tree.query(moved, k=2, workers=8)
    j, d1, dsec = j2[:, 0], d2[:, 0], d2[:, 1]
    idx = np.where(d1 <= dc, j, -1)
    if prev is not None:
        Tp, jp, gap_p = prev
        disp = np.linalg.norm(moved - S.transform_points(src, Tp), axis=1)
        gapc = (jp >= 0) & (2 * disp < gap_p)
        emptyc = (jp < 0) & (gap_p - disp > dc)       # stays rejected
        row = [f"it {it:2d} disp med {np.median(disp)*100:.2f} cm p90 {np.percentile(disp,90)*100:.2f} cm | gap {gapc.mean():.3f} empty {emptyc.mean():.3f}"]
        base = gapc | emptyc
        nw = len(src) // 64
        wave_all = lambda c: np.all(c[:nw * 64].reshape(nw, 64), axis=1).mean()
        row.append(f"waves-all {wave_all(base):.3f}")
        for K in Ks:
            ok = jp >= 0
            jj = np.where(ok, jp, 0)
            cand = np.concatenate([jj[:, None], iK[jj, 1:K + 1]], axis=1)
            dd = np.linalg.norm(moved[:, None, :] - tgt[cand], axis=2)
            best = np.argmin(dd, axis=1)
            dstar = dd[np.arange(len(dd)), best]
            jstar = cand[np.arange(len(dd)), best]
            rK = dK[jj, K]
            gc = ok & (dd[:, 0] + dstar < rK * (1 - 1e-6))
            wrong = gc & (jstar != j) & ~np.isclose(dstar, d1)
            assert not wrong.any(), wrong.sum()
            allc = base | gc
            row.append(f"K{K}: lanes {allc.mean():.3f} waves-all {wave_all(allc):.3f}")
        print(" | ".join(row), flush=True)
    # certificate for the next pass (exact gap among all targets; rejected: empty radius = d1)
    gap = np.where(d1 <= dc + 0.001, dsec - d1, 0.0)
    jp_next = np.where(d1 <= dc + 0.001, j, -1)
    gap = np.where(jp_next < 0, d1, gap)
    prev = (T, jp_next, gap)
    R = T[:3, :3]
    W = O.weights(np.einsum("ab,nbc,dc->nad", R, Cs, R), Ct, idx)
    q = np.zeros_like(src); q[idx >= 0] = tgt[idx[idx >= 0]]
    st = O.stats(src, q, W, idx, T)
    T, _ = gicp.solve_pose(st, T)
print(f"total {time.time()-t0:.1f}s")
