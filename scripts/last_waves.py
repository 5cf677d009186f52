"""Which waves end each pass of the driver's registration (attribute the long pole).

    make -C generalized-icp_amd/csrc VARIANT=tl VDEFS=-DGICP_TIMELINE
    GICP_LIB_VARIANT=tl python scripts/last_waves.py [--n 1000000] [--passes 20] [--shard-sim 1]

The bench's clouds, a cold registration from the identity: pass k runs at the pose the solve of pass k-1 gave
(gicp_iterate + the host solve, the sequence gicp_align runs), each launch's per-wave record dumped by the
timeline build (gicp_kernels.hip GICP_TIMELINE: wave start and end, the end of its certificate + descent
phase, the end of its walk, the walk's kind, lanes that descended / walked, tile visits, tiles scanned, list
use, block tests).  Per pass it prints the span and, for the last 1 % of waves to finish (and the last 10),
what they did: the phase that took their time, the walk's kind, visits, walking lanes, start time.
"""
import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "generalized-icp_amd"), ROOT]

KIND = {0: "none", 1: "list", 2: "list+full", 3: "full", 4: "sparse"}


PH = ("batch", "certs", "descent", "walk", "epi_ld", "gemm", "store")


def waves(path):
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 20).astype(np.int64)
    live = a[:, 17] > 0
    a = a[live]
    base = a[:, 16].min()
    us = lambda x: (x - base) / 100.0   # noqa: E731  (100 MHz realtime)
    has_tile = a[:, 3] > 0
    start, end = us(a[:, 16]), us(a[:, 17])
    ta = np.where(has_tile, us(a[:, 6]), start)
    tb = np.where(has_tile, us(a[:, 7]), ta)
    td = np.where(has_tile, us(a[:, 3]), tb)
    tw = np.where(has_tile, us(a[:, 4]), td)
    te = np.where(a[:, 10] > 0, us(a[:, 10]), tw)
    tf = np.where(a[:, 12] > 0, us(a[:, 12]), te)
    w = dict(
        tile=a[:, 0], start=start, end=end,
        kind=a[:, 5] & 0xFF, ndesc=(a[:, 5] >> 8) & 0xFF, nwalk=(a[:, 5] >> 16) & 0xFF, nwalk_jp=(a[:, 5] >> 24) & 0xFF,
        visits=a[:, 8], scanned=a[:, 9], list_used=a[:, 11], blk=a[:, 13],
        wb0=a[:, 14].astype(np.uint32).view(np.float32), fb=a[:, 15], xcc=a[:, 19] & 7)
    w["ph"] = np.stack([ta - start, tb - ta, td - tb, tw - td, te - tw, tf - te, end - tf])
    return w


def describe(w, sel, label):
    k = np.bincount(w["kind"][sel], minlength=5)
    ph = w["ph"][:, sel]
    top = np.bincount(np.argmax(ph, axis=0), minlength=len(PH))
    phs = " ".join(f"{n} {np.mean(ph[i]):5.1f}" for i, n in enumerate(PH))
    tops = "/".join(str(x) for x in top)
    return (f"  {label:8s} n {sel.sum():5d} start {np.mean(w['start'][sel]):6.1f} dur {np.mean((w['end'] - w['start'])[sel]):5.1f}"
            f" [{phs}] longest {tops}  walk none/list/l+f/full/sparse {k[0]}/{k[1]}/{k[2]}/{k[3]}/{k[4]}"
            f" visits {np.mean(w['visits'][sel]):4.1f} walkers {np.mean(w['nwalk'][sel]):4.1f} (jp {np.mean(w['nwalk_jp'][sel]):4.1f})"
            f" desc {np.mean(w['ndesc'][sel]):4.1f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--passes", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--shard-sim", type=int, default=1)
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="gicp_tl_")
    os.environ["GICP_STAMPS_DUMP"] = os.path.join(tmp, "st")
    import gicp
    from gicp import _lib
    from gicp import synthetic as S
    assert _lib.LIB_PATH.endswith("libgicp_hip_tl.so"), "run with GICP_LIB_VARIANT=tl (the timeline build)"
    src, tgt, _ = S.scene_pair_3d(a.n)
    p = gicp.default_params(3, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    e = gicp.Engine(0)
    e.set_target(tgt, p)
    e.set_source(src, p, shard=0, nshards=a.shard_sim)
    T = np.eye(4)
    for _ in range(a.warmup):   # as bench.py: a warmup registration, then the caches are dropped
        st = e.iterate(T)
        T, _ = gicp.solve_pose(st, T)
    e.reset_cache()
    first = len([f for f in os.listdir(tmp) if f.startswith("st.")])
    T = np.eye(4)
    for _ in range(a.passes):
        st = e.iterate(T)
        T, _ = gicp.solve_pose(st, T)
    e.close()
    print(f"n {a.n}  shard 1/{a.shard_sim}  passes {a.passes} (cold, from the identity; gicp_iterate + host solve)")
    print("per pass: span of the waves (first start -> last end, us) and the waves ending it; phases (us): batch = the"
          " prologue's scalar batch, certs = certificate + point loads, descent = graph descent, walk = list / full walk,"
          " epi_ld = the epilogue's gathers, gemm = W + statistics GEMM, store = partials + wave end")
    for k in range(a.passes):
        w = waves(os.path.join(tmp, f"st.{first + k}"))
        end = w["end"]
        span = end.max()
        n1 = max(1, len(end) // 100)
        order = np.argsort(-end)
        last1 = np.zeros(len(end), bool)
        last1[order[:n1]] = True
        walkers = w["nwalk"] > 0
        print(f"pass {k:2d}: span {span:6.1f} us  waves {len(end)}  walking waves {walkers.sum()}"
              f" (<= 8 walkers: {(walkers & (w['nwalk'] <= 8)).sum()})  p50 end {np.median(end):6.1f}  p99 end {np.percentile(end, 99):6.1f}")
        one = (w["ndesc"] == 1) & (w["nwalk"] == 0)   # waves whose only search was one lane's graph descent
        many = (w["ndesc"] >= 16) & (w["nwalk"] == 0)
        if one.any() or many.any():
            print(f"  descent phase: waves with 1 descending lane (no walk) n {one.sum()} mean"
                  f" {np.mean(w['ph'][2][one]) if one.any() else float('nan'):5.2f} us; >= 16 lanes n {many.sum()} mean"
                  f" {np.mean(w['ph'][2][many]) if many.any() else float('nan'):5.2f} us")
        print(describe(w, np.ones(len(end), bool), "all"))
        if walkers.any():
            print(describe(w, walkers, "walking"))
        sp = w["kind"] == 4
        if sp.any():
            print(f"  sparse waves n {sp.sum()}: walk {np.mean(w['ph'][3][sp]):5.2f} us, walkers covered by the list"
                  f" {np.mean(w['list_used'][sp]):4.2f} / wave, candidate super-blocks {np.mean(w['blk'][sp]):4.2f} / wave,"
                  f" tiles screened {np.mean(w['visits'][sp]):5.1f} / wave")
        fb = w["fb"] > 0   # waves with an fp64 re-resolution (its visits are inside epi_ld)
        if fb.any():
            epi = w["ph"][4]
            # what-if bounds (queueing ignored): the pass's span with each such wave's epi_ld cut to 3 us, and
            # with each walk of > 10 visits halved
            cut = np.where(fb, np.maximum(epi - 3.0, 0.0), 0.0)
            half = np.where(w["visits"] > 10, 0.5 * w["ph"][3], 0.0)
            print(f"  fp64 re-resolution: waves {fb.sum()} (last 1%: {(fb & last1).sum()}), epi_ld {np.mean(epi[fb]):5.1f} us"
                  f" (others {np.mean(epi[~fb]):4.1f}), fp64 visits {np.mean(w['fb'][fb]):4.1f} / wave;"
                  f" span if <= 3 us {np.max(end - cut):6.1f}, if long walks halved {np.max(end - half):6.1f},"
                  f" both {np.max(end - cut - half):6.1f}")
        print(describe(w, last1, "last 1%"))
        for i in order[:6]:
            phs = " ".join(f"{w['ph'][j, i]:4.1f}" for j in range(len(PH)))
            print(f"    tile {w['tile'][i]:6d} xcc {w['xcc'][i]} start {w['start'][i]:6.1f} end {w['end'][i]:6.1f} [{phs}]"
                  f" {KIND[int(w['kind'][i])]}: {w['visits'][i]} visits, {w['scanned'][i]} scanned, {w['nwalk'][i]} walkers"
                  f" ({w['nwalk_jp'][i]} with a last match), radius {w['wb0'][i]:.3f}, {w['ndesc'][i]} descended,"
                  f" {w['fb'][i]} fp64 visits")
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)


if __name__ == "__main__":
    main()
