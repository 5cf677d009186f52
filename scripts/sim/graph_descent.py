"""CPU simulation of kNN-graph descent certificates (see graph_cert.py): from the last match jp,
hop to the nearest candidate of the current node's list until a proof holds:
  best == node:   2 d(p', node) < r_K(node)
  best != node:   d(p', node) + d(p', best) < r_K(node)
Reports the fraction of lanes settled by gap certificates or by the descent within H hops, and of
waves (64 Morton-consecutive source points) with every lane settled."""
import sys, time
import numpy as np
from scipy.spatial import cKDTree
sys.path[:0] = ["generalized-icp_amd", "."]
import gicp
from gicp import synthetic as S
from oracle import gicp_oracle as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 12
Ks = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "12,16,20").split(",")]
H = 4
dc, dn = 0.5, 1.0
src, tgt, Tgt = S.scene_pair_3d(n)
t0 = time.time()
tree = cKDTree(tgt)
Cs, _ = O.covariances(src, dn, workers=8)
Ct, _ = O.covariances(tgt, dn, workers=8)
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
dK, iK = tree.query(tgt, k=max(Ks) + 1, workers=8)
print(f"setup {time.time()-t0:.1f}s", flush=True)
nw = len(src) // 64
wave_all = lambda c: np.all(c[:nw * 64].reshape(nw, 64), axis=1).mean()
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
        row = [f"it {it:2d} disp med {np.median(disp)*100:.2f} cm | gap lanes {gapc.mean():.3f} waves {wave_all(gapc):.3f}"]
        for K in Ks:
            ok = (jp >= 0) & ~gapc
            node = np.where(jp >= 0, jp, 0)
            done = gapc.copy()
            hops_used = np.zeros(len(src), int)
            for h in range(H):
                act = ok & ~done
                if not act.any():
                    break
                a = np.nonzero(act)[0]
                cand = np.concatenate([node[a, None], iK[node[a], 1:K + 1]], axis=1)
                dd = np.linalg.norm(moved[a, None, :] - tgt[cand], axis=2)
                b = np.argmin(dd, axis=1)
                db = dd[np.arange(len(a)), b]
                d0 = dd[:, 0]
                rK = dK[node[a], K]
                proof = np.where(b == 0, 2 * d0 < rK, d0 + db < rK)
                winner = cand[np.arange(len(a)), b]
                wrong = proof & (winner != j[a]) & ~np.isclose(db, d1[a])
                assert not wrong.any()
                done[a[proof]] = True
                hops_used[a[proof]] = h + 1
                stuck = (b == 0) & ~proof
                ok[a[stuck]] = False
                node[a] = winner
            row.append(f"K{K}: lanes {done.mean():.4f} waves {wave_all(done):.3f} hops>1 {(hops_used > 1).mean():.3f}")
        print(" | ".join(row), flush=True)
    gap = np.where(d1 <= dc + 0.001, dsec - d1, 0.0)
    jp_next = np.where(d1 <= dc + 0.001, j, -1)
    prev = (T, jp_next, gap)
    R = T[:3, :3]
    W = O.weights(np.einsum("ab,nbc,dc->nad", R, Cs, R), Ct, idx)
    q = np.zeros_like(src); q[idx >= 0] = tgt[idx[idx >= 0]]
    st = O.stats(src, q, W, idx, T)
    T, _ = gicp.solve_pose(st, T)
print(f"total {time.time()-t0:.1f}s")
