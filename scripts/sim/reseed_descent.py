"""CPU simulation for the pass-0 / large-move descent start: per pass, the fraction
of source lanes the K=20 graph descent proves within H hops when it starts from
  jp   : the lane's last match (what k_corr does today; none in pass 0),
  seed : the lane's nearest target point within the wave's Morton seed tile at the current pose
         (tiles approximated by aligned runs of 64 Morton-sorted target points),
  mix  : seed when jp is missing or the lane moved more than THR since its last match, else jp.
Lanes not proved walk in k_corr (the expensive part of the moving passes)."""
import sys, time
import numpy as np
from scipy.spatial import cKDTree
sys.path[:0] = ["generalized-icp_amd", "."]
import gicp
from gicp import synthetic as S
from oracle import gicp_oracle as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 6
H = int(sys.argv[3]) if len(sys.argv) > 3 else 4
THRS = [float(x) for x in (sys.argv[4] if len(sys.argv) > 4 else "0.05,0.1,0.2").split(",")]
LEVELS = [int(x) for x in (sys.argv[5] if len(sys.argv) > 5 else "7,8").split(",")]   # grid bits per axis
K = int(__import__("os").environ.get("SIM_K", "20"))
dc, dn = 0.5, 1.0
src, tgt, Tgt = S.scene_pair_3d(n)
t0 = time.time()
tree = cKDTree(tgt)
Cs, _ = O.covariances(src, dn, workers=8)
Ct, _ = O.covariances(tgt, dn, workers=8)


def spread(x):
    x = x.astype(np.uint64) & 0x3FF
    x = (x | (x << 16)) & 0x30000FF
    x = (x | (x << 8)) & 0x300F00F
    x = (x | (x << 4)) & 0x30C30C3
    x = (x | (x << 2)) & 0x9249249
    return x


def codes(p, lo, sc):
    g = np.clip(((p - lo) * sc), 0, 1023).astype(np.uint64)
    return spread(g[:, 0]) | (spread(g[:, 1]) << 1) | (spread(g[:, 2]) << 2)


slo = src.min(0); ssc = 1023 / (src.max(0) - slo).max()
order = np.argsort(codes(src, slo, ssc), kind="stable")
src, Cs = src[order], Cs[order]
tlo = tgt.min(0); tsc = 1023 / (tgt.max(0) - tlo).max()
tcode = codes(tgt, tlo, tsc)
torder = np.argsort(tcode, kind="stable")
tcode_s = tcode[torder]
dK, iK = tree.query(tgt, k=K + 1, workers=8)
print(f"setup {time.time()-t0:.1f}s", flush=True)
nw = len(src) // 64


def descend(moved, start, act0, jtrue, d1):
    node = start.copy()
    done = np.zeros(len(moved), bool)
    ok = act0.copy()
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
        done[a[proof]] = True
        stuck = (b == 0) & ~proof
        ok[a[stuck]] = False
        node[a] = cand[np.arange(len(a)), b]
    return done


def wave_frac(done, need):
    w = (done | ~need)[:nw * 64].reshape(nw, 64).all(axis=1)
    return w.mean()


T = np.eye(4)
prev = None
for it in range(iters):
    moved = S.transform_points(src, T)
    d2, j2 = tree.query(moved, k=2, workers=8)
    j, d1 = j2[:, 0], d2[:, 0]
    need = np.ones(len(src), bool)
    # Morton seed per wave: the wave centre's code -> aligned 64-run of the sorted target
    cen = moved[:nw * 64].reshape(nw, 64, 3).mean(axis=1)
    pos = np.searchsorted(tcode_s, codes(cen, tlo, tsc), side="right") - 1
    t0_ = np.clip(pos // 64 * 64, 0, len(tgt) - 64)
    rows = torder[t0_[:, None] + np.arange(64)[None, :]]          # [nw, 64] target ids
    dd = np.linalg.norm(moved[:nw * 64].reshape(nw, 64, 1, 3) - tgt[rows][:, None, :, :], axis=3)
    seed = np.zeros(len(src), np.int64)
    seed[:nw * 64] = rows[np.arange(nw)[:, None], np.argmin(dd, axis=2)].ravel()
    sd = np.linalg.norm(moved - tgt[seed], axis=1)
    has = np.zeros(len(src), bool); has[:nw * 64] = True
    res = [f"it {it}"]
    ds = descend(moved, seed, has, j, d1)
    res.append(f"seed: lanes {ds.mean():.3f} waves {wave_frac(ds, need):.3f} (seed dist med {np.median(sd)*100:.1f} cm p90 {np.percentile(sd,90)*100:.1f})")
    # per-lane grid seed: the first Morton-sorted target point in the lane's cell of 2^L per axis
    lane_code = codes(moved, tlo, tsc)
    for L in LEVELS:
        sh = np.uint64(3 * (10 - L))
        tp = tcode_s >> sh
        lp = lane_code >> sh
        k = np.searchsorted(tp, lp, side="left")
        kk = np.minimum(k, len(tp) - 1)
        hit = tp[kk] == lp
        gseed = np.where(hit, torder[kk], seed)
        gd = np.linalg.norm(moved - tgt[gseed], axis=1)
        dg = descend(moved, gseed, has | hit, j, d1)
        res.append(f"grid{L}: lanes {dg.mean():.3f} waves {wave_frac(dg, need):.3f} hit {hit.mean():.2f} (dist med {np.median(gd)*100:.1f} cm)")
        if it == 0:
            ds_best = dg
    if prev is not None:
        Tp, jp = prev
        disp = np.linalg.norm(moved - S.transform_points(src, Tp), axis=1)
        dj = descend(moved, np.maximum(jp, 0), jp >= 0, j, d1)
        res.append(f"disp med {np.median(disp)*100:.1f} cm p90 {np.percentile(disp,90)*100:.1f} | jp: lanes {dj.mean():.3f} waves {wave_frac(dj, need):.3f}")
        for thr in THRS:
            use_seed = (jp < 0) | (disp > thr)
            dm = np.where(use_seed, ds, dj)
            res.append(f"mix{thr}: lanes {dm.mean():.3f} waves {wave_frac(dm, need):.3f} (seeded {use_seed.mean():.2f})")
        both = ds | dj
        res.append(f"either: lanes {both.mean():.3f} waves {wave_frac(both, need):.3f}")
    print(" | ".join(res), flush=True)
    prev = (T, np.where(d1 <= dc, j, -1))
    R = T[:3, :3]
    idx = np.where(d1 <= dc, j, -1)
    W = O.weights(np.einsum("ab,nbc,dc->nad", R, Cs, R), Ct, idx)
    q = np.zeros_like(src); q[idx >= 0] = tgt[idx[idx >= 0]]
    st = O.stats(src, q, W, idx, T)
    T, _ = gicp.solve_pose(st, T)
print(f"total {time.time()-t0:.1f}s")
