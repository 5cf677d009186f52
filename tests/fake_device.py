"""A pure-NumPy stand-in for libgicp_hip.so's DEVICE entry points — TEST INFRASTRUCTURE ONLY.

SURVEY.md §4 (last row): a fake backend implementing the C-ABI semantics so the Python wrapper
(``gicp.gicp`` and its 7-tuple assembly, ``devices=``, the device-loop trace, ``Odometry``'s staged
ring) runs in a container without a GPU.  It is installed only by tests (``install(monkeypatch)``
replaces the loaded library object inside ``gicp._lib``); nothing in the product imports it, and the
product still fails loudly when the real library or the GPU is missing.

Every computation is the oracle's (``oracle/gicp_oracle.py``: cKDTree correspondences, the reference's
covariance rule, the DESIGN.md §4 statistics); the pose solve is the real library's host entry point
``gicp_solve_pose`` and ``gicp_cg_inner_2d`` (pure host code, callable without a GPU).  Shards are contiguous point ranges
(the real library deals Morton tiles round-robin; only the sum over shards is specified).
"""
from __future__ import annotations

import ctypes as C
import itertools

import numpy as np

from oracle import gicp_oracle as O

OK, E_INVALID, E_STATE, E_COMM = 0, -1, -3, -4
PASS_INFO = 6


def _arr(ptr, shape, dtype=np.float64):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=shape)


class _Ctx:
    def __init__(self, device):
        self.device = device
        self.err = b""
        self.tgt = self.src = None
        self.ptgt = self.psrc = None
        self.shard, self.nshards = 0, 1
        self.hook = None
        self.hook_ranks = (1, 0)
        self.staged = []          # (points, params) in staging order
        self.last_info = np.zeros(PASS_INFO)
        self.top = None           # (src, tgt, det) of the last pass with want_top_weights


class FakeLib:
    """The subset of include/gicp_hip.h the Python package calls, on NumPy."""

    def __init__(self, real, ndev=2):
        self._real = real         # the real library (host-only entry points: default params, solve)
        self.ndev = ndev
        self._ctx = {}
        self._ids = itertools.count(1)

    # ---- library -----------------------------------------------------------------------------
    def gicp_default_params(self, dim, p):
        return self._real.gicp_default_params(dim, p)

    def gicp_strerror(self, code):
        return self._real.gicp_strerror(code)

    def gicp_solve_pose(self, *a):
        return self._real.gicp_solve_pose(*a)

    def gicp_cg_inner_2d(self, *a):
        return self._real.gicp_cg_inner_2d(*a)

    def gicp_stats_size(self, dim):
        return O.stats_size(dim)

    # ---- context -----------------------------------------------------------------------------
    def gicp_create(self, out, device):
        if not 0 <= device < self.ndev:
            return E_INVALID
        h = next(self._ids)
        self._ctx[h] = _Ctx(device)
        out._obj.value = h
        return OK

    def _c(self, ctx):
        return self._ctx[ctx.value if isinstance(ctx, C.c_void_p) else ctx]

    def gicp_destroy(self, ctx):
        self._ctx.pop(ctx.value if isinstance(ctx, C.c_void_p) else ctx, None)

    def gicp_last_error(self, ctx):
        return self._c(ctx).err

    def _fail(self, c, code, msg):
        c.err = msg.encode()
        return code

    # ---- clouds ------------------------------------------------------------------------------
    def _cloud(self, ptr, n, dim, p):
        pts = _arr(ptr, (int(n), int(dim))).copy()
        par = p._obj if hasattr(p, "_obj") else p
        cov, cnt = O.covariances(pts, par.max_distance_nearest_neighbors, par.k_neighbors or None)
        return dict(pts=pts, cov=cov, cnt=cnt, p=par)

    def gicp_set_target(self, ctx, ptr, n, dim, p):
        c = self._c(ctx)
        c.tgt = self._cloud(ptr, n, dim, p)
        return OK

    def gicp_set_source(self, ctx, ptr, n, dim, p, shard, nshards):
        c = self._c(ctx)
        if not 0 <= shard < nshards:
            return self._fail(c, E_INVALID, "bad shard / nshards")
        c.src = self._cloud(ptr, n, dim, p)
        c.psrc = c.src["p"]
        c.shard, c.nshards = shard, nshards
        return OK

    def gicp_target_to_source(self, ctx, shard, nshards):
        c = self._c(ctx)
        c.src, c.tgt = c.tgt, None
        c.psrc = c.src["p"]
        c.shard, c.nshards = shard, nshards
        return OK

    def gicp_stage_target(self, ctx, ptr, n, dim, p):
        c = self._c(ctx)
        if len(c.staged) >= 2:
            return self._fail(c, E_STATE, "GICP_MAX_STAGED staged targets are pending")
        c.staged.append(self._cloud(ptr, n, dim, p))
        return OK

    def gicp_stage_target_ex(self, ctx, ptr, n, dim, p, flags):   # the copy (flags 0) and borrow are alike here
        if flags & ~1:
            return self._fail(self._c(ctx), E_INVALID, "unknown gicp_stage_target_ex flags")
        return self.gicp_stage_target(ctx, ptr, n, dim, p)

    def gicp_commit_target(self, ctx, shard, nshards):
        c = self._c(ctx)
        if not c.staged:
            return self._fail(c, E_STATE, "no staged target")
        nxt = c.staged.pop(0)      # the slot is consumed even when its build failed (as the library does)
        if nxt is None:            # a test marked this build as failed
            return self._fail(c, E_INVALID, "staged build: injected failure")
        if c.tgt is not None:
            c.src = c.tgt
            c.psrc = c.src["p"]
        c.tgt = nxt
        c.shard, c.nshards = shard, nshards
        return OK

    def gicp_cancel_stage(self, ctx):
        self._c(ctx).staged = []
        return OK

    def gicp_get_covariances(self, ctx, which, out):
        c = self._c(ctx)
        cl = c.tgt if which == 0 else c.src
        _arr(out, cl["cov"].shape)[:] = cl["cov"]
        return OK

    def gicp_get_neighbor_counts(self, ctx, which, out):
        c = self._c(ctx)
        cl = c.tgt if which == 0 else c.src
        _arr(out, cl["cnt"].shape, np.int32)[:] = cl["cnt"]
        return OK

    def gicp_reset_cache(self, ctx):
        return OK

    def gicp_comm_ranks(self, ctx, n, r, k):
        c = self._c(ctx)
        for ptr, v in ((n, c.hook_ranks[0] if c.hook else 1), (r, c.hook_ranks[1] if c.hook else 0),
                       (k, 2 if c.hook else 0)):
            if ptr:
                ptr._obj.value = v
        return OK

    def gicp_set_allreduce(self, ctx, fn, user):
        return self.gicp_set_allreduce_ranks(ctx, fn, user, 1, 0)

    def gicp_set_allreduce_ranks(self, ctx, fn, user, nranks, rank):
        c = self._c(ctx)
        c.hook = None if not fn else C.cast(fn, C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int, C.c_void_p))
        c.hook_ranks = (nranks, rank) if fn else (1, 0)
        return OK

    def gicp_pass_info(self, ctx, out):
        _arr(out, (PASS_INFO,))[:] = self._c(ctx).last_info
        return OK

    # ---- the pass ----------------------------------------------------------------------------
    def _pass(self, c, T):
        """This shard's statistics at pose T (+ per-point index / W / det of the shard)."""
        s, t = c.src, c.tgt
        n, d = s["pts"].shape
        lo, hi = n * c.shard // c.nshards, n * (c.shard + 1) // c.nshards
        mine = np.zeros(n, bool)
        mine[lo:hi] = True
        R = T[:d, :d]
        moved = O.apply_transformation(s["pts"], T)
        idx, dist = O.correspondences(moved, t["pts"], c.psrc.max_distance_correspondence)
        W = O.weights_model(np.einsum("ab,nbc,dc->nad", R, s["cov"], R), t["cov"], idx,
                            {0: "plane_to_plane", 1: "point_to_point", 2: "point_to_plane"}[c.psrc.cov_model], t["cnt"])
        q = np.zeros_like(s["pts"])
        q[idx >= 0] = t["pts"][idx[idx >= 0]]
        sidx = np.where(mine, idx, -1)
        st = O.stats(s["pts"], q, W, sidx, T)
        ok = sidx >= 0
        r = q - moved
        info = np.zeros(PASS_INFO)
        info[3] = float(np.sum(np.where(ok, np.sum(r * r, axis=1), 0.0)))
        det = np.where(ok, np.linalg.det(W), 0.0)
        return np.concatenate([st, info]), dict(idx=idx, dist=dist, W=W, det=det, mine=mine)

    def _exchange(self, c, ext):
        if c.hook is None:
            return ext
        buf = (C.c_double * len(ext))(*ext)
        if c.hook(buf, len(ext), None) != 0:
            raise RuntimeError("host all-reduce hook failed")
        return np.array(buf[:], dtype=np.float64)

    @staticmethod
    def _top(det, mine, idx, k):
        cand = np.nonzero(mine)[0]
        order = np.lexsort((cand, det[cand]))[-k:]   # np.argsort(det)[-k:] order, ties: larger index last
        sel = cand[order]
        return sel, np.where(idx[sel] >= 0, idx[sel], -1), det[sel]

    def gicp_iterate(self, ctx, T_ptr, stats_ptr, dbg):
        c = self._c(ctx)
        if c.src is None or c.tgt is None:
            return self._fail(c, E_STATE, "set_target and set_source first")
        d = c.src["pts"].shape[1]
        T = _arr(T_ptr, (d + 1, d + 1)).copy()
        ext, per = self._pass(c, T)
        ext = self._exchange(c, ext)
        ns = O.stats_size(d)
        _arr(stats_ptr, (ns,))[:] = ext[:ns]
        c.last_info = ext[ns:]
        c.top = None
        if dbg:
            g = dbg._obj if hasattr(dbg, "_obj") else dbg
            n = len(per["idx"])
            if g.index:
                _arr(g.index, (n,), np.int64)[per["mine"]] = per["idx"][per["mine"]]
            if g.weight:
                _arr(g.weight, (n, d, d))[per["mine"]] = np.where((per["idx"] >= 0)[:, None, None], per["W"], 0.0)[per["mine"]]
            if g.distance:
                _arr(g.distance, (n,))[per["mine"]] = per["dist"][per["mine"]]
            if g.want_top_weights:
                c.top = per
        return OK

    def gicp_top_weights(self, ctx, k, src_out, tgt_out, det_out):
        c = self._c(ctx)
        if c.top is None:
            return self._fail(c, E_STATE, "no pass with want_top_weights")
        si, ti, dt = self._top(c.top["det"], c.top["mine"], c.top["idx"], k)
        for ptr, v, ty in ((src_out, si, np.int64), (tgt_out, ti, np.int64), (det_out, dt, np.float64)):
            if ptr:
                out = _arr(ptr, (k,), ty)
                out[:] = -1 if ty is np.int64 else 0.0
                out[k - len(v):] = v
        return OK

    # ---- the loop ----------------------------------------------------------------------------
    def gicp_align(self, ctx, T0, p, T_out, res):
        return self.gicp_align_trace(ctx, T0, p, T_out, res, None)

    def gicp_align_trace(self, ctx, T0_ptr, p, T_out, res, trace):
        c = self._c(ctx)
        if c.src is None or c.tgt is None:
            return self._fail(c, E_STATE, "set_target and set_source first")
        par = p._obj if hasattr(p, "_obj") else p
        c.psrc = par
        d = c.src["pts"].shape[1]
        nt = (d + 1) * (d + 1)
        tr = trace._obj if (trace is not None and hasattr(trace, "_obj")) else trace
        if tr is not None and tr.capacity < par.max_iterations:
            return self._fail(c, E_INVALID, "gicp_trace.capacity < max_iterations")
        T = _arr(T0_ptr, (d + 1, d + 1)).copy()
        last, loss, it, conv, at = np.inf, 0.0, 0, 0, -1
        ns = O.stats_size(d)
        for it in range(par.max_iterations):
            ext, per = self._pass(c, T)
            ext = self._exchange(c, ext)
            Tn = np.empty_like(T)
            lo = C.c_double()
            self._real.gicp_solve_pose(d, ext[:ns].ctypes.data_as(C.POINTER(C.c_double)),
                                       T.ctypes.data_as(C.POINTER(C.c_double)),
                                       Tn.ctypes.data_as(C.POINTER(C.c_double)), C.byref(lo))
            loss = lo.value
            if tr is not None:
                if tr.poses:
                    _arr(tr.poses, (tr.capacity, nt))[it] = T.ravel()
                if tr.losses:
                    _arr(tr.losses, (tr.capacity,))[it] = loss
                if tr.top_k:
                    si, ti, dt = self._top(per["det"], per["mine"], per["idx"], tr.top_k)
                    _arr(tr.top_src, (tr.capacity, tr.top_k), np.int64)[it, -len(si):] = si
                    _arr(tr.top_tgt, (tr.capacity, tr.top_k), np.int64)[it, -len(ti):] = ti
                    _arr(tr.top_det, (tr.capacity, tr.top_k))[it, -len(dt):] = dt
            c.last_info = ext[ns:]
            if not par.fixed_iterations and abs(last - loss) < par.tolerance:
                conv, at = 1, it
                break
            last = loss
            T = Tn
        iters = it + 1 if par.max_iterations > 0 else 0
        _arr(T_out, (d + 1, d + 1))[:] = T
        if res:
            r = res._obj if hasattr(res, "_obj") else res
            r.iterations, r.converged, r.converged_at = iters, conv, at
            r.final_loss = loss
            r.stop_reason = 1 if conv else 0
        return OK


def install(monkeypatch, ndev=2):
    """Load the real library (host entry points only) and put the fake in its place for the test."""
    from gicp import _lib
    real = _lib.load()
    fake = FakeLib(real, ndev)
    monkeypatch.setattr(_lib, "_lib", fake)
    import gicp
    monkeypatch.setattr(gicp, "_ENGINES", {})
    return fake
