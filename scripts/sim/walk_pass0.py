"""CPU simulation (round 4): the first pass's full walk (k_corr walk_c, identity pose, no hints / lists /
certificates) against alternative candidate generators, counted per wave in memory round trips, tile visits,
tiles scanned and rows scanned.  Tiles are aligned 64-runs of Morton-sorted points cut into 4 sub-tiles of 16
(the real build caps tile extents; the comparison between strategies is what this is for).

  hier   : the shipped order -- seed tile, then super-blocks (64 blocks) -> blocks (64 tiles) -> tiles, in index
           order, pruned by the wave box and the wave's current bound (max over lanes)
  grid   : seed tile, then a uniform grid of cells (tiles listed by the cell holding their centre): one request
           for the cells' tile ranges around the wave box, one for those tiles' boxes, then the candidates
           nearest-first

    python scripts/sim/walk_pass0.py [waves] [cell_m]
"""
import sys
import time

import numpy as np

sys.path[:0] = ["generalized-icp_amd", "."]
from gicp import synthetic as S  # noqa: E402

NW = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
CELL = float(sys.argv[2]) if len(sys.argv) > 2 else 0.25
DC = 0.5
R0 = DC * 1.002          # the screen radius (d_c + kappa)
rng = np.random.default_rng(5)
n = 1_000_000
src, tgt, _ = S.scene_pair_3d(n)


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


def cut(g, E):
    """build_tile_table's greedy cut: runs of <= 64 sorted points whose grid box stays within E cells"""
    starts = [0]
    lo = g[0].copy(); hi = g[0].copy(); i0 = 0
    for i in range(1, len(g)):
        v = g[i]
        nlo = np.minimum(lo, v); nhi = np.maximum(hi, v)
        if i - i0 < 64 and (nhi - nlo).max() <= E:
            lo, hi = nlo, nhi
            continue
        starts.append(i); i0 = i; lo = v.copy(); hi = v.copy()
    return np.array(starts)


def tiles(p):
    lo = p.min(0)
    sc = 1023 / (p.max(0) - lo).max()
    c = codes(p, lo, sc)
    o = np.argsort(c, kind="stable")
    p = p[o]
    c = c[o]
    g = np.clip(((p - lo) * sc), 0, 1023).astype(np.int32)
    # the smallest cap (2 2^(k/4) cells) with at most 1.35 x the minimum tile count (as build_tile_table)
    target = int(1.35 * np.ceil(len(p) / 64)) + 2
    best = None
    for k in range(8, 40):
        E = int(2.0 * 2 ** (k / 4))
        st = cut(g[::1], E) if best is None or True else None
        if len(st) <= target:
            best = st
            break
    st = np.append(best, len(p))
    nt = len(best)
    q = np.full((nt, 64, 3), np.nan)
    for t in range(nt):
        q[t, :st[t + 1] - st[t]] = p[st[t]:st[t + 1]]
    qm = np.where(np.isnan(q), np.inf, q); qx = np.where(np.isnan(q), -np.inf, q)
    mn, mx = qm.min(1), qx.max(1)
    sub = q.reshape(nt, 4, 16, 3)
    smn = np.where(np.isnan(sub), np.inf, sub).min(2); smx = np.where(np.isnan(sub), -np.inf, sub).max(2)
    empty = ~np.isfinite(smn)
    smn[empty] = 1e9; smx[empty] = 1e9
    q = np.where(np.isnan(q), 1e9, q)
    print(f"tiles {nt} ({nt / np.ceil(len(p) / 64):.2f}x), cap {E} cells = {E / sc:.2f} m", flush=True)
    return q, (mn + mx) / 2, (mx - mn) / 2, (smn + smx) / 2, (smx - smn) / 2, c[best], lo, sc


sq, sC, sH, _, _, _, _, _ = tiles(src)
tq, tC, tH, tsC, tsH, tcode, tlo, tsc = tiles(tgt)
NT = len(tC)
# hierarchy: blocks of 64 tiles, super-blocks of 64 blocks
NB = (NT + 63) // 64
bC = np.zeros((NB, 3)); bH = np.zeros((NB, 3))
for b in range(NB):
    lo = (tC[64 * b:64 * b + 64] - tH[64 * b:64 * b + 64]).min(0)
    hi = (tC[64 * b:64 * b + 64] + tH[64 * b:64 * b + 64]).max(0)
    bC[b], bH[b] = (lo + hi) / 2, (hi - lo) / 2
NS = (NB + 63) // 64
sbC = np.zeros((NS, 3)); sbH = np.zeros((NS, 3))
for s in range(NS):
    lo = (bC[64 * s:64 * s + 64] - bH[64 * s:64 * s + 64]).min(0)
    hi = (bC[64 * s:64 * s + 64] + bH[64 * s:64 * s + 64]).max(0)
    sbC[s], sbH[s] = (lo + hi) / 2, (hi - lo) / 2
# grid: tiles by the cell of their centre
glo = tgt.min(0) - 1e-6
gdim = np.ceil((tgt.max(0) - glo) / CELL).astype(int) + 1
cell_of = np.floor((tC - glo) / CELL).astype(int)
cid = (cell_of[:, 0] * gdim[1] + cell_of[:, 1]) * gdim[2] + cell_of[:, 2]
order = np.argsort(cid, kind="stable")
cid_sorted = cid[order]
hmax = tH.max(0)          # the largest tile half-extent per axis: a tile's box lies within its cell +- hmax


def gap2(c1, h1, c2, h2):
    g = np.maximum(np.abs(c1 - c2) - h1 - h2, 0)
    return (g * g).sum(-1)


class Wave:
    def __init__(self, w):
        p = sq[w]
        self.p = p[p[:, 0] < 1e8]          # the tile's points (padding rows excluded, as k_corr's invalid lanes)
        self.c, self.h = sC[w], sH[w]
        self.best = np.full(len(self.p), R0 * R0)
        self.rt = self.visits = self.scanned = self.rows = 0

    def wb(self):
        return self.best.max()

    def visit(self, t):
        """k_corr visit_pre: one round trip (metadata + coordinates), the per-lane box test, the sub-tile
        scan of the lanes that need it"""
        self.rt += 1
        self.visits += 1
        g = gap2(self.p, 0, tC[t], tH[t])
        need = g <= self.best
        if not need.any():
            return
        gs = gap2(self.p[:, None, :], 0, tsC[t][None], tsH[t][None])       # lanes x sub-tiles
        subs = (gs <= self.best[:, None]).any(0)
        self.scanned += 1
        self.rows += 16 * subs.sum()
        d = ((self.p[:, None, :] - tq[t][None]) ** 2).sum(-1)
        self.best = np.minimum(self.best, d.min(1))


def seed_of(wv):
    cc = codes(wv.c[None], tlo, tsc)[0]
    return int(np.clip(np.searchsorted(tcode, cc, side="right") - 1, 0, NT - 1))


def hier(w):
    wv = Wave(w)
    seed = seed_of(wv)
    wv.rt += 3          # Morton seed table + binary steps
    wv.visit(seed)
    for s0 in range(0, NS, 64):
        wv.rt += 1      # a round of 64 super-block tests
        sgap = gap2(wv.c, wv.h, sbC[s0:s0 + 64], sbH[s0:s0 + 64])
        for s in np.nonzero(sgap <= wv.wb())[0] + s0:
            if gap2(wv.c, wv.h, sbC[s], sbH[s]) > wv.wb():
                continue
            wv.rt += 1  # the super-block's 64 block tests
            bl = np.arange(64 * s, min(NB, 64 * s + 64))
            for b in bl[gap2(wv.c, wv.h, bC[bl], bH[bl]) <= wv.wb()]:
                if gap2(wv.c, wv.h, bC[b], bH[b]) > wv.wb():
                    continue
                wv.rt += 1  # the block's 64 TileBox tests
                tl = np.arange(64 * b, min(NT, 64 * b + 64))
                cand = tl[(gap2(wv.c, wv.h, tC[tl], tH[tl]) <= wv.wb()) & (tl != seed)]
                for t in cand:
                    if gap2(wv.c, wv.h, tC[t], tH[t]) <= wv.wb():
                        wv.visit(t)
    return wv


def hier2(w, frac=0.5):
    """hier with a two-box candidate test: after the seed visit the lanes whose bound reaches past frac x the
    largest radius form a 'far' box; a block / tile is a candidate if it is within the near lanes' bound of
    the wave box or within the far lanes' bound of the far box (bounds per class, updated as they shrink)"""
    wv = Wave(w)
    seed = seed_of(wv)
    wv.rt += 3
    wv.visit(seed)
    rmax = np.sqrt(wv.wb())
    big = wv.best > (frac * rmax) ** 2
    if big.any():
        pb = wv.p[big]
        fc, fh = (pb.min(0) + pb.max(0)) / 2, (pb.max(0) - pb.min(0)) / 2
    else:
        fc, fh = wv.c, wv.h

    def cand(c, h):
        near = wv.best[~big].max() if (~big).any() else -1.0
        far = wv.best[big].max() if big.any() else -1.0
        return (gap2(wv.c, wv.h, c, h) <= near) | (gap2(fc, fh, c, h) <= far)

    for s0 in range(0, NS, 64):
        wv.rt += 1
        sl = np.arange(s0, min(NS, s0 + 64))
        for s in sl[cand(sbC[sl], sbH[sl])]:
            if not cand(sbC[s], sbH[s]):
                continue
            wv.rt += 1
            bl = np.arange(64 * s, min(NB, 64 * s + 64))
            for b in bl[cand(bC[bl], bH[bl])]:
                if not cand(bC[b], bH[b]):
                    continue
                wv.rt += 1
                tl = np.arange(64 * b, min(NT, 64 * b + 64))
                for t in tl[cand(tC[tl], tH[tl]) & (tl != seed)]:
                    if cand(tC[t], tH[t]):
                        wv.visit(t)
    return wv


def hier4(w):
    """hier with the candidate test against the source tile's 4 sub-boxes (16 lanes each), each with its own
    lanes' bound: a tile / block is a candidate if it is within reach of any sub-box"""
    wv = Wave(w)
    seed = seed_of(wv)
    wv.rt += 3
    wv.visit(seed)
    n = len(wv.p)
    groups = [np.arange(g * 16, min(n, g * 16 + 16)) for g in range(4) if g * 16 < n]
    boxes = [((wv.p[gi].min(0) + wv.p[gi].max(0)) / 2, (wv.p[gi].max(0) - wv.p[gi].min(0)) / 2) for gi in groups]

    def cand(c, h):
        ok = False
        for gi, (bc, bh) in zip(groups, boxes):
            ok = ok | (gap2(bc, bh, c, h) <= wv.best[gi].max())
        return ok

    for s0 in range(0, NS, 64):
        wv.rt += 1
        sl = np.arange(s0, min(NS, s0 + 64))
        for s in sl[cand(sbC[sl], sbH[sl])]:
            if not cand(sbC[s], sbH[s]):
                continue
            wv.rt += 1
            bl = np.arange(64 * s, min(NB, 64 * s + 64))
            for b in bl[cand(bC[bl], bH[bl])]:
                if not cand(bC[b], bH[b]):
                    continue
                wv.rt += 1
                tl = np.arange(64 * b, min(NT, 64 * b + 64))
                for t in tl[cand(tC[tl], tH[tl]) & (tl != seed)]:
                    if cand(tC[t], tH[t]):
                        wv.visit(t)
    return wv


def grid(w, seeded=True, skin=0.0):
    wv = Wave(w)
    seed = -1
    if seeded:
        seed = seed_of(wv)
        wv.rt += 3
        wv.visit(seed)
    r = np.sqrt(wv.wb()) + skin   # the candidates also cover the list's skin (k_corr lists)
    lo = np.floor((wv.c - wv.h - r - hmax - glo) / CELL).astype(int)
    hi = np.floor((wv.c + wv.h + r + hmax - glo) / CELL).astype(int)
    lo = np.maximum(lo, 0)
    hi = np.minimum(hi, gdim - 1)
    xs, ys, zs = [np.arange(lo[a], hi[a] + 1) for a in range(3)]
    cells = ((xs[:, None, None] * gdim[1] + ys[None, :, None]) * gdim[2] + zs[None, None, :]).ravel()
    wv.rt += int(np.ceil(len(cells) / 64))      # cell ranges, 64 cells per request
    a = np.searchsorted(cid_sorted, cells, side="left")
    b = np.searchsorted(cid_sorted, cells, side="right")
    cand = np.concatenate([order[x:y] for x, y in zip(a, b)]) if len(cells) else np.zeros(0, int)
    cand = cand[cand != seed]
    wv.rt += int(np.ceil(len(cand) / 64))       # the candidates' boxes, 64 per request
    wv.ncand = len(cand)
    wv.ncells = len(cells)
    key = gap2(wv.c, wv.h, tC[cand], tH[cand])
    for t in cand[np.argsort(key, kind="stable")]:
        if gap2(wv.c, wv.h, tC[t], tH[t]) <= wv.wb():
            wv.visit(t)
    return wv


waves = rng.choice(len(sC), size=NW, replace=False)
for name, fn in (("hier", hier), ("hier4", hier4)):
    t0 = time.time()
    res = [fn(int(w)) for w in waves]
    rt = np.array([x.rt for x in res]); vi = np.array([x.visits for x in res])
    scn = np.array([x.scanned for x in res]); rows = np.array([x.rows for x in res])
    print(f"{name:7s} cell {CELL:.2f}: round trips {rt.mean():6.1f} (p90 {np.percentile(rt, 90):4.0f}, p99 {np.percentile(rt, 99):4.0f})  visits {vi.mean():5.1f} (p99 {np.percentile(vi, 99):4.0f})"
          f"  scanned {scn.mean():5.1f}  rows {rows.mean():6.1f}   [{time.time() - t0:.0f} s]", flush=True)
    if hasattr(res[0], "ncand"):
        nc = np.array([x.ncand for x in res]); ncl = np.array([x.ncells for x in res])
        print(f"        cells {ncl.mean():5.1f} (max {ncl.max()})  candidates {nc.mean():5.1f} (p90 {np.percentile(nc, 90):.0f}, max {nc.max()})")
