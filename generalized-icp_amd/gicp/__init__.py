"""MI355X-native GICP — drop-in for msi-se/generalized-icp's ``gicp.py``.

``from gicp import gicp, apply_transformation`` works as with the reference
(python-implementation/gicp.py:78, :176; imported that way by
visualization.py:7 and robot-visualization.py:6).  The per-iteration hot path
(correspondences, Mahalanobis weights, normal-equation statistics) and the
per-point surface covariances run in hand-written HIP kernels for gfx950
behind the C-ABI of ``libgicp_hip.so``; this module is the thin host layer.

There is no CPU fallback: without the built library or a GPU the engine
raises.  HIP is initialised on the first call, not at import (the reference
calls gicp() from a forked worker, robot-visualization.py:199).
"""
from __future__ import annotations

import ctypes as C
from collections.abc import Sequence

import numpy as np

from . import _lib
from ._lib import Debug, Params, Result, Trace, check, dptr

__all__ = ["gicp", "apply_transformation", "Engine", "RotatedCovariances", "expand_stats", "stats_size",
           "default_params", "last_result"]


def stats_size(dim):
    ns = dim * (dim + 1) // 2
    return ns * ns + ns * dim + ns + dim * dim + dim + 2


def default_params(dim, **kw):
    """gicp_params with the reference defaults (gicp.py:5, :11, :24, :78), overridden by kw."""
    p = Params()
    _lib.load().gicp_default_params(dim, C.byref(p))
    for k, v in kw.items():
        if v is not None:
            setattr(p, k, v)
    return p


def _sym_pairs(d):
    return [(a, b) for a in range(d) for b in range(a, d)]


def expand_stats(st, d):
    """(H, g, c0, count) of  f(z) = c0 - 2 g.(z - z_k) + (z - z_k)^T H (z - z_k),  z = (vec R, t).

    Layout of ``st``: A[ab][ij] = sum W_ab s_i s_j, B[ab][i] = sum W_ab s_i,
    C[ab] = sum W_ab, gR[a][i] = sum (W r_k)_a s_i, gt[a] = sum (W r_k)_a, c0, count."""
    st = np.asarray(st, dtype=np.float64)
    P = _sym_pairs(d)
    ns = len(P)
    pos = {}
    for k, (a, b) in enumerate(P):
        pos[(a, b)] = pos[(b, a)] = k
    o = 0
    A = st[o:o + ns * ns].reshape(ns, ns); o += ns * ns
    B = st[o:o + ns * d].reshape(ns, d); o += ns * d
    Cc = st[o:o + ns]; o += ns
    gR = st[o:o + d * d].reshape(d, d); o += d * d
    gt = st[o:o + d]; o += d
    nz = d * d + d
    H = np.zeros((nz, nz))
    for a in range(d):
        for i in range(d):
            for b in range(d):
                for j in range(d):
                    H[a * d + i, b * d + j] = A[pos[(a, b)], pos[(i, j)]]
                H[a * d + i, d * d + b] = H[d * d + b, a * d + i] = B[pos[(a, b)], i]
        for b in range(d):
            H[d * d + a, d * d + b] = Cc[pos[(a, b)]]
    return H, np.concatenate([gR.ravel(), gt]), float(st[o]), float(st[o + 1])


# 2-D: z6 = (R00, R01, R10, R11, tx, ty) = L (tx, ty, cos th, sin th)
_L2 = np.array([[0, 0, 1, 0], [0, 0, 0, -1], [0, 0, 0, 1], [0, 0, 1, 0], [1, 0, 0, 0], [0, 1, 0, 0]], dtype=np.float64)


def _rot2(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s], [s, c]])


def _offset_to_T(x):
    """gicp.py:42-50."""
    T = np.eye(3)
    T[:2, :2] = _rot2(x[2])
    T[:2, 2] = x[:2]
    return T


def apply_transformation(cloud, T):
    """gicp.py:176-177 (any dimension: x -> R x + t)."""
    T = np.asarray(T)
    d = T.shape[0] - 1
    return np.dot(np.asarray(cloud)[:, :d], T[:d, :d].T) + T[:d, d]


class Engine:
    """One GPU context of libgicp_hip.so (clouds stay resident between calls)."""

    def __init__(self, device=0):
        self._lib = _lib.load()
        self._ctx = C.c_void_p()
        rc = self._lib.gicp_create(C.byref(self._ctx), int(device))
        if rc == _lib.GICP_E_INVALID:
            raise ValueError(f"gicp_create(device={device}): no such GPU")
        if rc != _lib.GICP_OK:
            raise _lib.GicpError(rc, f"gicp_create(device={device}): {self._lib.gicp_strerror(rc).decode()}")
        self.device = device
        self.dim = None
        self.n_src = self.n_tgt = 0
        self.generation = 0        # bumped whenever the source cloud changes (lazy covariance views)
        self._staged = []          # (shape, params, borrowed array or None) of the staged targets, oldest first
        self._hook = None          # keeps the ctypes callback of set_allreduce alive
        self._hook_fn = None       # (fn, nranks, rank) of that hook, to restore it after a gicp() call

    def close(self):
        if self._ctx:
            self._lib.gicp_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _cloud(pts):
        a = np.ascontiguousarray(np.asarray(pts, dtype=np.float64))
        if a.ndim != 2 or a.shape[1] not in (2, 3) or a.shape[0] < 1:
            raise ValueError(f"point cloud must be a non-empty N x 2 or N x 3 array, got shape {a.shape}")
        return a

    def comm_init(self, nranks, rank, uid: bytes):
        check(self._lib.gicp_comm_init(self._ctx, nranks, rank, uid), self._ctx, "gicp_comm_init")

    def comm_ranks(self):
        """(nranks, rank, kind) of the statistics exchange, read back from the RCCL communicator
        (gicp_comm_ranks); kind is 'none', 'rccl' or 'hook'."""
        n, r, k = C.c_int(), C.c_int(), C.c_int()
        check(self._lib.gicp_comm_ranks(self._ctx, C.byref(n), C.byref(r), C.byref(k)), self._ctx, "gicp_comm_ranks")
        return n.value, r.value, {0: "none", 1: "rccl", 2: "hook", 3: "peer"}[k.value]

    def peer_export(self) -> bytes:
        """This rank's exchange area as an IPC handle (gicp_peer_export): all-gather it, then peer_init."""
        buf = C.create_string_buffer(_lib.PEER_HANDLE_BYTES)
        check(self._lib.gicp_peer_export(self._ctx, buf), self._ctx, "gicp_peer_export")
        return buf.raw

    def peer_init(self, nranks, rank, handles, timeout=10.0):
        """Map the peers' exchange areas (handles in rank order) and prove the path with one probe
        exchange (gicp_peer_init, collective): from then on every pass sums the statistics over the
        ranks inside its own launch.  Raises GicpError (code GICP_E_COMM) when the path does not work."""
        if len(handles) != nranks or any(len(h) != _lib.PEER_HANDLE_BYTES for h in handles):
            raise ValueError(f"need {nranks} handles of {_lib.PEER_HANDLE_BYTES} bytes")
        blob = b"".join(handles)
        check(self._lib.gicp_peer_init(self._ctx, int(nranks), int(rank), blob, float(timeout)), self._ctx,
              "gicp_peer_init")

    def peer_close(self):
        check(self._lib.gicp_peer_close(self._ctx), self._ctx, "gicp_peer_close")

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(_lib.COMM_ID_BYTES)
        check(_lib.load().gicp_comm_unique_id(buf), None, "gicp_comm_unique_id")
        return buf.raw

    def set_target(self, pts, params=None):
        a = self._cloud(pts)
        p = params or default_params(a.shape[1])
        check(self._lib.gicp_set_target(self._ctx, dptr(a), a.shape[0], a.shape[1], C.byref(p)), self._ctx,
              "gicp_set_target")
        self.n_tgt, self.dim = a.shape

    def set_source(self, pts, params=None, shard=0, nshards=1):
        a = self._cloud(pts)
        p = params or default_params(a.shape[1])
        check(self._lib.gicp_set_source(self._ctx, dptr(a), a.shape[0], a.shape[1], C.byref(p), shard, nshards),
              self._ctx, "gicp_set_source")
        self.n_src, self.dim = a.shape
        self.generation += 1

    def target_to_source(self, shard=0, nshards=1):
        check(self._lib.gicp_target_to_source(self._ctx, shard, nshards), self._ctx, "gicp_target_to_source")
        self.n_src = self.n_tgt
        self.n_tgt = 0
        self.generation += 1

    MAX_STAGED = 2   # GICP_MAX_STAGED

    def stage_target(self, pts, params=None, borrow=False):
        """Build `pts` as a coming target on its own stream while the current one is registered
        (gicp_stage_target; up to MAX_STAGED pending); commit_target makes the oldest current.  The
        library copies `pts` before this call returns, so the caller may reuse the array at once --
        unless borrow=True (GICP_STAGE_BORROW): then the build reads the array itself (no copy on this
        thread) and the caller must not modify it until commit_target / cancel_stage (this object keeps
        a reference until then)."""
        a = self._cloud(pts)
        p = params or default_params(a.shape[1])
        check(self._lib.gicp_stage_target_ex(self._ctx, dptr(a), a.shape[0], a.shape[1], C.byref(p),
                                             _lib.GICP_STAGE_BORROW if borrow else 0), self._ctx, "gicp_stage_target")
        self._staged.append((a.shape, p, a if borrow else None))

    def commit_target(self, shard=0, nshards=1):
        """Wait for the oldest staged target; the current target becomes the source, the staged one the target."""
        rc = self._lib.gicp_commit_target(self._ctx, shard, nshards)
        staged = self._staged.pop(0) if (self._staged and rc != _lib.GICP_E_STATE) else None   # slot consumed
        check(rc, self._ctx, "gicp_commit_target")
        if self.n_tgt:
            self.n_src = self.n_tgt
            self.generation += 1
        self.n_tgt, self.dim = staged[0]

    def cancel_stage(self):
        """Wait for and drop every staged target."""
        self._lib.gicp_cancel_stage(self._ctx)
        self._staged = []

    def covariances(self, which="target"):
        w = 0 if which == "target" else 1
        n = self.n_tgt if w == 0 else self.n_src
        out = np.empty((n, self.dim, self.dim))
        check(self._lib.gicp_get_covariances(self._ctx, w, dptr(out)), self._ctx, "gicp_get_covariances")
        return out

    def rotated_covariances(self, R, which="source"):
        """R C Rᵀ of every point on the device (gicp_rotated_covariances), original order."""
        w = 0 if which == "target" else 1
        n = self.n_tgt if w == 0 else self.n_src
        R = np.ascontiguousarray(np.asarray(R, dtype=np.float64))
        if R.shape != (self.dim, self.dim):
            raise ValueError(f"R must be {self.dim} x {self.dim}")
        out = np.empty((n, self.dim, self.dim))
        check(self._lib.gicp_rotated_covariances(self._ctx, w, dptr(R), dptr(out)), self._ctx,
              "gicp_rotated_covariances")
        return out

    def graph(self):
        """The target neighbour graph (gicp_get_graph): (index [M, 20] original ids with -1 pads,
        radius [M]: every target nearer than radius[i] to point i is in row i)."""
        idx = np.empty((self.n_tgt, _lib.GRAPH_K), dtype=np.int64)
        rad = np.empty(self.n_tgt)
        check(self._lib.gicp_get_graph(self._ctx, idx.ctypes.data_as(C.POINTER(C.c_int64)), dptr(rad)), self._ctx,
              "gicp_get_graph")
        return idx, rad

    def reset_cache(self):
        """Forget the pose-dependent caches (lists, certificates, last matches): the next pass starts cold."""
        check(self._lib.gicp_reset_cache(self._ctx), self._ctx, "gicp_reset_cache")

    def iteration_times(self):
        """Sampled k_corr time (ms) per iteration of the last align; NaN where not sampled."""
        buf = (C.c_float * 4096)()
        m = self._lib.gicp_iteration_times(self._ctx, buf, 4096)
        check(min(m, 0), self._ctx, "gicp_iteration_times")
        t = np.array(buf[:m], dtype=np.float64)
        t[t < 0] = np.nan
        return t

    def set_allreduce(self, fn, nranks=1, rank=0):
        """Host statistics exchange (gicp_set_allreduce_ranks): fn(buf) gets this rank's statistics as a
        float64 array and must return (or write in place) the sum over ranks; (nranks, rank) is what
        comm_ranks() then reports.  None removes it."""
        if fn is None:
            check(self._lib.gicp_set_allreduce(self._ctx, None, None), self._ctx, "gicp_set_allreduce")
            self._hook = None
            self._hook_fn = None
            return

        def _cb(buf, n, _user):
            try:
                a = np.ctypeslib.as_array(buf, shape=(n,))
                r = fn(a)
                if r is not None and r is not a:
                    a[:] = np.asarray(r, dtype=np.float64)
                return 0
            except Exception:   # an exception must not cross the C boundary
                import traceback
                traceback.print_exc()
                return -1

        cb = _lib.ALLREDUCE_FN(_cb)
        check(self._lib.gicp_set_allreduce_ranks(self._ctx, C.cast(cb, C.c_void_p), None, int(nranks), int(rank)),
              self._ctx, "gicp_set_allreduce")
        self._hook = cb
        self._hook_fn = (fn, int(nranks), int(rank))

    def neighbor_counts(self, which="target"):
        w = 0 if which == "target" else 1
        n = self.n_tgt if w == 0 else self.n_src
        out = np.empty(n, dtype=np.int32)
        check(self._lib.gicp_get_neighbor_counts(self._ctx, w, out.ctypes.data_as(C.POINTER(C.c_int32))), self._ctx,
              "gicp_get_neighbor_counts")
        return out

    def iterate(self, T, debug=False):
        """One pass at pose T -> statistics (and per-point index / W / distance if debug)."""
        T = np.ascontiguousarray(np.asarray(T, dtype=np.float64))
        st = np.empty(stats_size(self.dim))
        dbg = None
        out = None
        if debug:
            n, d = self.n_src, self.dim
            out = dict(index=np.empty(n, dtype=np.int64), weight=np.empty((n, d, d)), distance=np.empty(n))
            dbg = Debug(out["index"].ctypes.data_as(C.POINTER(C.c_int64)), dptr(out["weight"]), dptr(out["distance"]))
        check(self._lib.gicp_iterate(self._ctx, dptr(T), dptr(st), C.byref(dbg) if dbg else None), self._ctx,
              "gicp_iterate")
        return (st, out) if debug else st

    def pass_info(self):
        """Diagnostics of the last pass: ambiguous lanes, pairs screened, list rebuilds, sum |r|^2,
        lanes proved by the graph descent, source tiles that walked."""
        out = np.empty(_lib.PASS_INFO)
        check(self._lib.gicp_pass_info(self._ctx, dptr(out)), self._ctx, "gicp_pass_info")
        return dict(ambiguous=out[0], pairs=out[1], list_rebuilds=out[2], sum_sq=out[3], graph_proved=out[4],
                    walked_tiles=out[5])

    def iterate_top(self, T, k=5):
        """One pass at pose T keeping det(W) on the device, then its top-k on the device
        (gicp.py:170 `np.argsort(det(W))[-k:]`): (statistics, src_idx[k], tgt_idx[k], det[k])."""
        T = np.ascontiguousarray(np.asarray(T, dtype=np.float64))
        st = np.empty(stats_size(self.dim))
        dbg = Debug(None, None, None, 1)
        check(self._lib.gicp_iterate(self._ctx, dptr(T), dptr(st), C.byref(dbg)), self._ctx, "gicp_iterate")
        si = np.empty(k, dtype=np.int64)
        ti = np.empty(k, dtype=np.int64)
        dt = np.empty(k)
        p64 = C.POINTER(C.c_int64)
        check(self._lib.gicp_top_weights(self._ctx, k, si.ctypes.data_as(p64), ti.ctypes.data_as(p64), dptr(dt)),
              self._ctx, "gicp_top_weights")
        return st, si, ti, dt

    def align(self, T0=None, params=None, trace=False, top_k=0):
        """The whole outer loop (gicp.py:116-167) natively; returns (T, result dict), plus with
        trace=True a dict of per-iteration rows recorded on the device (gicp_align_trace): 'poses'
        [iters, d+1, d+1] (the pose each pass ran at), 'losses' [iters], and with top_k > 0 the
        pass's top_k largest det(W): 'top_src', 'top_tgt' [iters, top_k] original indices, 'top_det'."""
        d = self.dim
        T0 = np.eye(d + 1) if T0 is None else np.ascontiguousarray(np.asarray(T0, dtype=np.float64))
        Tout = np.empty((d + 1, d + 1))
        res = Result()
        p = params or default_params(d)
        if trace:
            cap = max(1, int(p.max_iterations))
            rows = dict(poses=np.zeros((cap, d + 1, d + 1)), losses=np.zeros(cap),
                        top_src=np.full((cap, max(top_k, 1)), -1, dtype=np.int64),
                        top_tgt=np.full((cap, max(top_k, 1)), -1, dtype=np.int64),
                        top_det=np.zeros((cap, max(top_k, 1))))
            p64 = C.POINTER(C.c_int64)
            tr = Trace(cap, int(top_k), dptr(rows["poses"]), dptr(rows["losses"]),
                       rows["top_src"].ctypes.data_as(p64), rows["top_tgt"].ctypes.data_as(p64), dptr(rows["top_det"]))
            check(self._lib.gicp_align_trace(self._ctx, dptr(T0), C.byref(p), dptr(Tout), C.byref(res), C.byref(tr)),
                  self._ctx, "gicp_align_trace")
        else:
            check(self._lib.gicp_align(self._ctx, dptr(T0), C.byref(p), dptr(Tout), C.byref(res)), self._ctx,
                  "gicp_align")
        r = res.as_dict()
        r.pop("pad", None)
        r.pop("pad2", None)
        r["stop_reason"] = _lib.STOP_REASONS.get(r["stop_reason"], r["stop_reason"])
        if not trace:
            return Tout, r
        n = min(int(r["iterations"]), int(p.max_iterations))
        out = {k: v[:n] for k, v in rows.items()}
        if not top_k:
            for k in ("top_src", "top_tgt", "top_det"):
                out.pop(k)
        return Tout, r, out


def solve_pose(stats, T_k):
    """Host minimiser of the inner problem from the statistics (gicp_solve_pose)."""
    T_k = np.ascontiguousarray(np.asarray(T_k, dtype=np.float64))
    d = T_k.shape[0] - 1
    st = np.ascontiguousarray(np.asarray(stats, dtype=np.float64))
    out = np.empty_like(T_k)
    loss = C.c_double()
    check(_lib.load().gicp_solve_pose(d, dptr(st), dptr(T_k), dptr(out), C.byref(loss)), None, "gicp_solve_pose")
    return out, loss.value


def _cg_inner(stats, offset, T_k):
    """2-D reference inner solve (gicp.py:148-154): fmin_cg's algorithm (SciPy 1.15.3, restated natively in
    gicp_cg_inner_2d, bit-identical to scipy's own on the same objective: tests/test_cg_native.py) on the
    closed form of the loss from the pass's 26 statistics.  Returns (xopt, fopt)."""
    st = np.ascontiguousarray(stats, dtype=np.float64)
    Tk = np.ascontiguousarray(T_k, dtype=np.float64)
    x0 = np.ascontiguousarray(offset, dtype=np.float64)
    if st.shape != (stats_size(2),) or Tk.shape != (3, 3) or x0.shape != (3,):
        raise ValueError("2-D statistics (26), a 3x3 pose and a 3-vector offset expected")
    x = np.zeros(3)
    fopt = C.c_double()
    check(_lib.load().gicp_cg_inner_2d(dptr(st), dptr(Tk), dptr(x0), dptr(x), C.byref(fopt), None), None,
          "gicp_cg_inner_2d")
    return x, fopt.value


def _loss_2d(x, s, q, W):
    """The reference's loss (gicp.py:52-58) on GPU-produced correspondences q and weights W."""
    r = q - s @ _rot2(x[2]).T - x[:2]
    wr = np.sum(W * r[:, None, :], axis=2)
    return np.sum(r * wr)


def _grad_2d(x, s, q, W):
    """The reference's gradient (gicp.py:60-76)."""
    r = q - s @ _rot2(x[2]).T - x[:2]
    wr = np.sum(W * r[:, None, :], axis=2)
    g = np.zeros(3)
    g[:2] = -2 * np.sum(wr, axis=0)
    dR = np.array([[-np.sin(x[2]), -np.cos(x[2])], [np.cos(x[2]), -np.sin(x[2])]])
    g[2] = np.sum(-2 * (wr.T @ s) * dR)
    return g


def _cg_inner_faithful(src, q, W, offset):
    """fmin_cg on the per-point loss exactly as gicp.py:148-154 evaluates it."""
    from scipy.optimize import fmin_cg

    out = fmin_cg(f=lambda x: _loss_2d(x, src, q, W), x0=offset, fprime=lambda x: _grad_2d(x, src, q, W),
                  disp=False, full_output=True)
    return out[0], out[1]


_ENGINES = {}
_LAST_RESULT = None


def last_result():
    """The gicp_result of the last gicp() call that ran its loop on the device (mode='fast',
    inner='newton'; the first device's): iterations, wall_ms (the library's own wall time of the loop,
    without the clouds' setup and the 7-tuple's assembly), stop reason, ...  None before such a call."""
    return None if _LAST_RESULT is None else dict(_LAST_RESULT)

# 2-D clouds up to this size default to mode='faithful' (scipy fmin_cg on the reference's per-point
# loss, which copies N x 2 x 2 weights to the host every iteration); larger ones to mode='fast'
FAITHFUL_MAX_POINTS = 5000


class RotatedCovariances(Sequence):
    """all_source_cov_matrices of the fast path (gicp.py:120-121,174), held lazily: element k is
    R_k C_s,i R_kᵀ for every source point (rigid invariance), R_k the rotation of
    iteration k.  Only the initial covariances and the rotations are stored; an element is computed
    on the host when read (always the same formula, so a re-read is bit-identical whatever the engine
    did meanwhile), and the last two elements read are kept, so the reference's per-point access
    `all_source_cov_matrices[step][i]` (visualization.py:158) costs one computation per step.  Holds no
    engine: picklable (e.g. through the multiprocessing Queue of robot-visualization.py:153,166).
    Behaves as the reference's list for len / indexing / iteration."""

    _CACHE = 2

    def __init__(self, init_cov, rotations=()):
        self._init = init_cov
        self._R = [np.array(R, dtype=np.float64) for R in rotations]
        self._cache = {}
        self.computed = 0   # elements materialised so far (a test bounds it)

    def append_rotation(self, R):
        self._R.append(np.array(R, dtype=np.float64))

    def __len__(self):
        return len(self._R)

    def _one(self, k):
        hit = self._cache.get(k)
        if hit is not None:
            return hit
        R = self._R[k]
        out = np.matmul(np.matmul(R, self._init), R.T)
        self.computed += 1
        if len(self._cache) >= self._CACHE:
            self._cache.pop(next(iter(self._cache)))
        self._cache[k] = out
        return out

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self._one(i) for i in range(len(self._R))[k]]
        k = range(len(self._R))[k]   # negative indices, IndexError as a list
        return self._one(k)

    def __getstate__(self):
        return {"init": self._init, "R": self._R}

    def __setstate__(self, st):
        self._init = st["init"]
        self._R = st["R"]
        self._cache = {}
        self.computed = 0

    def __repr__(self):
        return f"RotatedCovariances({len(self)} iterations x {len(self._init)} points)"


def _engine(device):
    eng = _ENGINES.get(device)
    if eng is None:
        eng = _ENGINES[device] = Engine(device)
    return eng


def _devices(device, devices):
    """The GPUs a gicp() call runs on: [device], or the distinct entries of `devices`."""
    if devices is None:
        return [int(device)]
    devs = [int(x) for x in devices]
    if not devs:
        raise ValueError("devices must name at least one GPU")
    if len(set(devs)) != len(devs):
        raise ValueError(f"devices lists a GPU more than once: {devs}")
    return devs


class _ThreadSum:
    """Statistics exchange of a multi-device gicp() call (one host thread per GPU): every rank's
    buffer in, the sum in rank order out -- the same bits on every rank, so every device's solve and
    convergence test agree.  A failing rank aborts the barrier and the others raise instead of waiting."""

    def __init__(self, world, timeout=300.0):
        import threading
        self.world = world
        self.slots = [None] * world
        self.bar = threading.Barrier(world, timeout=timeout)

    def __call__(self, rank, buf):
        self.slots[rank] = np.array(buf, dtype=np.float64)
        self.bar.wait()
        total = self.slots[0].copy()
        for r in range(1, self.world):
            total += self.slots[r]
        self.bar.wait()
        return total

    def abort(self):
        self.bar.abort()


def _run_ranks(engines, fn):
    """fn(rank, engine) on one thread per engine (ctypes releases the GIL inside the library);
    returns the results in rank order, re-raising the first failure."""
    if len(engines) == 1:
        return [fn(0, engines[0])]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(engines)) as ex:
        futs = [ex.submit(fn, r, e) for r, e in enumerate(engines)]
        return [f.result() for f in futs]


def _merge_top(rows, k=5):
    """The k largest det(W) over the ranks' top-k rows, ascending as np.argsort(det)[-k:] orders them
    (equal dets: larger original index last).  rows: [(src, tgt, det), ...] per rank."""
    src = np.concatenate([r[0] for r in rows])
    tgt = np.concatenate([r[1] for r in rows])
    det = np.concatenate([r[2] for r in rows])
    ok = src >= 0
    src, tgt, det = src[ok], tgt[ok], det[ok]
    order = np.lexsort((src, det))[-k:]
    return src[order], tgt[order], det[order]


def pcl_stop(T_old, T_new, mse, prev_mse, transformation_epsilon=0.0, rotation_epsilon=0.0,
             euclidean_fitness_epsilon=0.0, mse_relative_epsilon=0.0):
    """PCL-style stopping test after an update (the criteria the reference's ROS experiment set,
    presentation/main.typ:773-776; same order and semantics as k_solve): the increment
    dT = T_new T_old^-1 with |dt|^2 <= transformation_epsilon and cos(angle) >= rotation threshold
    (1 - transformation_epsilon when rotation_epsilon is 0), else |mse - prev| < euclidean_fitness_epsilon,
    else |mse - prev| / prev < mse_relative_epsilon.  Returns 'transform' / 'abs_mse' / 'rel_mse' / None."""
    d = T_old.shape[0] - 1
    dR = T_new[:d, :d] @ T_old[:d, :d].T
    dt = T_new[:d, d] - dR @ T_old[:d, d]
    tr = float(np.trace(dR))
    cosang = 0.5 * (tr - 1.0) if d == 3 else 0.5 * tr
    rot_cos = rotation_epsilon if rotation_epsilon > 0 else 1.0 - transformation_epsilon
    dm = abs(mse - prev_mse)
    if transformation_epsilon > 0 and cosang >= rot_cos and float(dt @ dt) <= transformation_epsilon:
        return "transform"
    if euclidean_fitness_epsilon > 0 and dm < euclidean_fitness_epsilon:
        return "abs_mse"
    if mse_relative_epsilon > 0 and np.isfinite(prev_mse) and dm / prev_mse < mse_relative_epsilon:
        return "rel_mse"
    return None


def gicp(source_points, target_points, max_iterations=100, tolerance=1e-6, max_distance_correspondence=150,
         max_distance_nearest_neighbors=50, *, full_output=True, mode=None, inner=None, k_neighbors=None, device=0,
         devices=None, verbose=True, T0=None, method="plane_to_plane", transformation_epsilon=0.0,
         rotation_epsilon=0.0, euclidean_fitness_epsilon=0.0, mse_relative_epsilon=0.0):
    """Drop-in for gicp.py:78 — returns the same 7-tuple (gicp.py:174):

    (T, all_transformations, initial_source_cov_matrices, target_cov_matrices,
     highest_weight_points_source, highest_weight_points_target, all_source_cov_matrices)

    2-D and 3-D clouds (T is 3x3 or 4x4).

    mode='faithful' (default for 2-D clouds of <= FAITHFUL_MAX_POINTS source points): every
      iteration the GPU recomputes the source covariances on the transformed source
      (gicp.py:120) and produces the correspondences and weights; scipy's fmin_cg then
      minimises the reference's own per-point loss on them (gicp.py:148-154), so the
      inexact inner stop follows the reference's trajectory.
    mode='fast' (3-D default, and larger 2-D clouds): source covariances are
      rotated (rigid invariance), the GPU reduces the loss to its sufficient
      statistics in one pass, and the inner problem is solved from them -- exactly by
      Newton on SO(d) (inner='newton', the 3-D default: the whole loop then runs on the
      device in one gicp_align_trace call, the 7-tuple's per-iteration rows recorded there),
      or by conjugate gradients on the closed form (inner='cg', the 2-D default, host loop): the
      native gicp_cg_inner_2d, a C++ restatement of SciPy 1.15.3's fmin_cg pinned bit for bit
      against scipy's own on the same closed form (tests/test_cg_native.py).
    full_output=False skips the per-point visualisation extras (the three
    lists come back empty), which is what large clouds want.  In 'fast' mode the
    top-5 det(W) points are selected on the GPU (no per-point copy) and
    all_source_cov_matrices is a RotatedCovariances view (computed when read).

    device / devices: the GPU, or a list of distinct GPUs; with several, every GPU holds
      both clouds and reduces its shard of the source, one host thread drives each, and the
      statistics are summed over them every iteration in device order (the same sum on every
      GPU, so all take the same step).  mode='faithful' runs on the first listed GPU.
    method: 'plane_to_plane' (GICP, the reference), 'point_to_point' (ICP: C_s = 0,
      C_t = I) or 'point_to_plane' (C_s = 0, C_t = P^-1), presentation/main.typ:446-455.
    transformation_epsilon / rotation_epsilon / euclidean_fitness_epsilon /
      mse_relative_epsilon: optional PCL-style stopping criteria (see pcl_stop), tested
      after the update; 0 disables each.  tolerance=0 disables the reference's rule.
    """
    src = Engine._cloud(source_points)
    tgt = Engine._cloud(target_points)
    d = src.shape[1]
    if tgt.shape[1] != d:
        raise ValueError("source and target must have the same dimension")
    if mode is None:
        mode = "faithful" if d == 2 and len(src) <= FAITHFUL_MAX_POINTS else "fast"
    if mode not in ("faithful", "fast") or (mode == "faithful" and d != 2):
        raise ValueError("mode must be 'fast', or 'faithful' for 2-D clouds")
    inner = ("cg" if d == 2 else "newton") if inner is None else inner
    if inner not in ("cg", "newton") or (inner == "cg" and d != 2):
        raise ValueError("inner must be 'newton', or 'cg' for 2-D clouds")
    if method not in _lib.COV_MODELS:
        raise ValueError(f"method must be one of {sorted(set(_lib.COV_MODELS))}")
    devs = _devices(device, devices)
    if mode == "faithful":
        devs = devs[:1]
    engines = [_engine(x) for x in devs]
    G = len(engines)
    p = default_params(d, max_iterations=int(max_iterations), tolerance=float(tolerance),
                       max_distance_correspondence=float(max_distance_correspondence),
                       max_distance_nearest_neighbors=float(max_distance_nearest_neighbors), k_neighbors=k_neighbors,
                       cov_model=_lib.COV_MODELS[method])
    pcl = dict(transformation_epsilon=float(transformation_epsilon), rotation_epsilon=float(rotation_epsilon),
               euclidean_fitness_epsilon=float(euclidean_fitness_epsilon),
               mse_relative_epsilon=float(mse_relative_epsilon))

    def build(r, e):
        e.set_target(tgt, p)
        e.set_source(src, p, shard=r, nshards=G)

    _run_ranks(engines, build)
    eng = engines[0]
    target_cov = eng.covariances("target")
    init_src_cov = eng.covariances("source")
    for e in engines[1:]:   # each device computed its own shard's source covariances (NaN elsewhere)
        other = e.covariances("source")
        miss = np.isnan(init_src_cov[:, 0, 0])
        init_src_cov[miss] = other[miss]
    T = np.eye(d + 1) if T0 is None else np.array(T0, dtype=np.float64)
    if mode == "fast" and inner == "newton":
        for k, v in pcl.items():
            setattr(p, k, v)
        return _device_loop(engines, src, tgt, T, p, full_output, verbose, init_src_cov, target_cov)
    return _host_loop(engines, src, tgt, T, T0, p, pcl, mode, inner, full_output, verbose, init_src_cov, target_cov)


def _device_loop(engines, src, tgt, T, p, full_output, verbose, init_src_cov, target_cov):
    """gicp.py:116-172 as ONE gicp_align_trace call per GPU: the loop, the solve and the convergence
    test run on the device; the per-iteration rows the 7-tuple needs (poses, top-5 det(W)) are recorded
    there and copied out once."""
    d = src.shape[1]
    G = len(engines)
    k = 5 if full_output else 0
    xchg = _ThreadSum(G) if G > 1 else None
    if xchg is not None:   # installing this call's hook would tear down an RCCL communicator or peer exchange
        own = [e.comm_ranks()[2] for e in engines]
        if any(k in ("rccl", "peer") for k in own):
            raise ValueError(f"gicp(devices=...): the cached engines carry their own statistics exchange ({own}); "
                             "a multi-device call needs engines without one (close it, or use distributed.align)")
    prev = [e._hook_fn for e in engines]   # a hook the caller installed on the cached engines
    if xchg is not None:
        for r, e in enumerate(engines):
            e.set_allreduce(lambda buf, r=r: xchg(r, buf), nranks=G, rank=r)

    def run(r, e):
        try:
            return e.align(T, p, trace=True, top_k=k)
        except BaseException:
            if xchg is not None:
                xchg.abort()
            raise

    try:
        outs = _run_ranks(engines, run)
    finally:
        if xchg is not None:   # restore what was there before this call
            for e, h in zip(engines, prev):
                e.set_allreduce(*h) if h is not None else e.set_allreduce(None)
    T_fin, res, tr = outs[0]
    global _LAST_RESULT
    _LAST_RESULT = dict(res)
    iters = int(res["iterations"])
    poses = tr["poses"]
    loss_stop = bool(res["converged"]) and res["stop_reason"] == "loss"
    if res["converged"] and verbose:
        if loss_stop:
            print("Converged at iteration", res["converged_at"])                 # gicp.py:161
        else:
            print("Converged at iteration", res["converged_at"], f"({res['stop_reason']})")
    all_T = [T] + [poses[i].copy() for i in range(1, iters)]
    if iters > 0 and not loss_stop:                                            # gicp.py:166-167
        all_T.append(T_fin)
    hw_s, hw_t = [], []
    all_src_cov = []
    if full_output:
        all_src_cov = RotatedCovariances(init_src_cov, [poses[i][:d, :d] for i in range(iters)])   # gicp.py:121
        for i in range(iters - 1 if loss_stop else iters):                      # gicp.py:169-172
            rows = [(o[2]["top_src"][i], o[2]["top_tgt"][i], o[2]["top_det"][i]) for o in outs]
            top_s, top_t, _ = _merge_top(rows) if G > 1 else rows[0]
            hw_s.append(apply_transformation(src[top_s[top_s >= 0]], poses[i]))
            hw_t.append(_targets(tgt, top_s, top_t, d))
    return T_fin, all_T, init_src_cov, target_cov, hw_s, hw_t, all_src_cov


def _targets(tgt, top_s, top_t, d):
    """corresponding_target_points rows of the selected points (gicp.py:140; zeros where rejected)."""
    ok = top_s >= 0
    qt = np.zeros((int(ok.sum()), d))
    m = top_t[ok] >= 0
    qt[m] = tgt[top_t[ok][m]]
    return qt


def _host_loop(engines, src, tgt, T, T0, p, pcl, mode, inner, full_output, verbose, init_src_cov, target_cov):
    """gicp.py:116-172 with the inner solve on the host: faithful mode, and fast mode with inner='cg'."""
    d = src.shape[1]
    G = len(engines)
    eng = engines[0]
    use_pcl = any(v > 0 for k, v in pcl.items() if k != "rotation_epsilon")
    prev_mse = np.inf
    all_T = [T]
    offset = np.array([T[0, 2], T[1, 2], np.arctan2(T[1, 0], T[0, 0])]) if d == 2 else None
    last = np.inf
    hw_s, hw_t = [], []
    all_src_cov = [] if (mode == "faithful" or not full_output) else RotatedCovariances(init_src_cov)
    eye = np.eye(d + 1)
    moved_source = False   # faithful mode: the engine holds a transformed copy of the source
    for it in range(int(p.max_iterations)):
        if mode == "faithful":
            moved = apply_transformation(src, T)                   # gicp.py:119
            if it > 0 or T0 is not None:
                eng.set_source(moved, p)                           # gicp.py:120, on the GPU
                moved_source = True
            cs = eng.covariances("source") if moved_source else init_src_cov
            if full_output:
                all_src_cov.append(cs)
            _, dbg = eng.iterate(eye, debug=True)                  # gicp.py:124-145 on the moved cloud
            idx = dbg["index"]
            q = np.zeros_like(src)
            q[idx >= 0] = tgt[idx[idx >= 0]]
            if inner == "cg":
                new_offset, min_loss = _cg_inner_faithful(src, q, dbg["weight"], offset)
                T_new = _offset_to_T(new_offset)
            else:
                T_new, min_loss = _newton_from_points(src, q, dbg["weight"], idx, T)
                new_offset = None
        else:
            if full_output:                                        # gicp.py:170 on the device
                outs = _run_ranks(engines, lambda r, e: e.iterate_top(T, 5))
                top_s, top_t, _ = _merge_top([o[1:] for o in outs]) if G > 1 else outs[0][1:]
                all_src_cov.append_rotation(T[:d, :d])            # gicp.py:120-121, read lazily
            else:
                outs = [(o,) for o in _run_ranks(engines, lambda r, e: e.iterate(T))]
            st = outs[0][0].copy()
            for o in outs[1:]:                                     # rank order: deterministic
                st += o[0]
            if inner == "cg":
                new_offset, min_loss = _cg_inner(st, offset, T)
                T_new = _offset_to_T(new_offset)
            else:
                T_new, min_loss = solve_pose(st, T)
                new_offset = None
        if abs(last - min_loss) < p.tolerance:                     # gicp.py:155-162
            if verbose:
                print("Converged at iteration", it)
            break
        last = min_loss
        if full_output:                                            # gicp.py:169-172
            if mode == "faithful":
                idx = dbg["index"]
                q = np.zeros_like(src)
                q[idx >= 0] = tgt[idx[idx >= 0]]
                top = np.argsort(np.linalg.det(dbg["weight"]))[-5:]
                hw_s.append(moved[top])
                hw_t.append(q[top])
            else:
                hw_s.append(apply_transformation(src[top_s[top_s >= 0]], T))   # gicp.py:119,171: the 5 rows only
                hw_t.append(_targets(tgt, top_s, top_t, d))
        offset = new_offset
        stop = None
        if use_pcl:                                                # PCL-style criteria, after the update
            sum_sq = sum(e.pass_info()["sum_sq"] for e in engines)
            cnt = float(np.sum(dbg["index"] >= 0)) if mode == "faithful" else float(st[-1])
            mse = sum_sq / cnt if cnt > 0 else 0.0
            stop = pcl_stop(T, T_new, mse, prev_mse, **pcl)
            prev_mse = mse
        T = T_new
        all_T.append(T)
        if stop is not None:
            if verbose:
                print("Converged at iteration", it, f"({stop})")
            break
    if moved_source:
        eng.set_source(src, p)   # leave the engine holding the untransformed source
    return T, all_T, init_src_cov, target_cov, hw_s, hw_t, all_src_cov


def _newton_from_points(src, q, W, idx, T):
    """Exact inner minimiser for the faithful path: statistics of the given (q, W) at T, then the host solve."""
    d = src.shape[1]
    ok = idx >= 0
    s, qq, WW = src[ok], q[ok], W[ok]
    r = qq - s @ T[:d, :d].T - T[:d, d]
    wr = np.einsum("nab,nb->na", WW, r)
    P = _sym_pairs(d)
    ws = np.stack([WW[:, a, b] for a, b in P], axis=1)
    ss = np.stack([s[:, i] * s[:, j] for i, j in P], axis=1)
    st = np.concatenate([np.einsum("np,nq->pq", ws, ss).ravel(), np.einsum("np,ni->pi", ws, s).ravel(), ws.sum(0),
                         np.einsum("na,ni->ai", wr, s).ravel(), wr.sum(0), [np.sum(r * wr)], [float(ok.sum())]])
    return solve_pose(st, T)
