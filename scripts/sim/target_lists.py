"""CPU simulation (round 3): target-side tile lists (every target tile within R of tile S, <= 64 kept)
keyed by a pass-0 wave's Morton seed tile: the share of pass-0 waves whose search region (box excess over
S + final radius) the list would certify, for R = 0.5 .. 1.2 m (tiles approximated by aligned 64-runs of
Morton-sorted points).  python scripts/sim/target_lists.py"""
import sys, time, numpy as np
from scipy.spatial import cKDTree
sys.path[:0] = ["generalized-icp_amd", "."]
from gicp import synthetic as S
n = 1_000_000
src, tgt, Tgt = S.scene_pair_3d(n)
def spread(x):
    x = x.astype(np.uint64) & 0x3FF
    x = (x | (x << 16)) & 0x30000FF; x = (x | (x << 8)) & 0x300F00F
    x = (x | (x << 4)) & 0x30C30C3; x = (x | (x << 2)) & 0x9249249
    return x
def codes(p, lo, sc):
    g = np.clip(((p - lo) * sc), 0, 1023).astype(np.uint64)
    return spread(g[:, 0]) | (spread(g[:, 1]) << 1) | (spread(g[:, 2]) << 2)
def tiles(p):
    lo = p.min(0); sc = 1023 / (p.max(0) - lo).max()
    c = codes(p, lo, sc); o = np.argsort(c, kind="stable"); p = p[o]; c = c[o]
    nt = len(p) // 64; q = p[:nt*64].reshape(nt, 64, 3)
    mn, mx = q.min(1), q.max(1)
    return p[:nt*64], (mn + mx) / 2, (mx - mn) / 2, c[:nt*64:64], lo, sc
sp, sC, sH, _, _, _ = tiles(src)
tp, tC, tH, tcode, tlo, tsc = tiles(tgt)
tree = cKDTree(tgt)
d1, _ = tree.query(sp, workers=8, distance_upper_bound=0.5)
d1 = np.minimum(d1, 0.5)
rho = d1.reshape(-1, 64).max(1) * 1.02 + 0.003
ctree = cKDTree(tC)
hd = np.linalg.norm(tH, axis=1).max()
def gap(c1, h1, c2, h2):
    g = np.maximum(np.abs(c1 - c2) - h1 - h2, 0)
    return np.linalg.norm(g, axis=-1)
Rmax = 1.2
t0 = time.time()
nb = ctree.query_ball_point(tC, Rmax + 2 * hd, workers=8)
Ravail = {}
sizes = {}
for R in (0.5, 0.75, 1.0, 1.2):
    ra = np.empty(len(tC)); sz = np.empty(len(tC), int)
    for s in range(len(tC)):
        js = np.asarray(nb[s]); g = gap(tC[s], tH[s], tC[js], tH[js])
        g.sort()
        inr = g[g <= R]
        if len(inr) <= 64: ra[s] = R; sz[s] = len(inr)
        else: ra[s] = g[64] - 1e-6; sz[s] = 64
    Ravail[R] = ra; sizes[R] = sz
print("lists built", time.time() - t0, flush=True)
# seed tile of each source wave: last target tile whose first code <= centre code
scode = codes(sC, tlo, tsc)
seed = np.clip(np.searchsorted(tcode, scode, side="right") - 1, 0, len(tC) - 1)
def excess(cq, hq, cs, hs):   # max distance from a point of box q to box s
    e = np.maximum(np.abs(cq - cs) + hq - hs, 0)
    return np.linalg.norm(e, axis=-1)
h = excess(sC, sH, tC[seed], tH[seed])
for R in (0.5, 0.75, 1.0, 1.2):
    cov = h + rho <= Ravail[R][seed]
    print(f"R {R}: list size mean {sizes[R].mean():.1f} p90 {np.percentile(sizes[R],90):.0f} full {np.mean(sizes[R]==64)*100:.1f}%  | pass-0 waves covered {cov.mean()*100:.1f}%  (h med {np.median(h):.2f} p90 {np.percentile(h,90):.2f}, rho med {np.median(rho):.2f})")
# better seed: the target tile nearest the wave centre (what a hint would give after one pass)
_, near = ctree.query(sC)
h2 = excess(sC, sH, tC[near], tH[near])
for R in (0.5, 0.75, 1.0, 1.2):
    cov = h2 + rho <= Ravail[R][near]
    print(f"R {R}: nearest-centre seed covered {cov.mean()*100:.1f}% (h med {np.median(h2):.2f})")
