"""GICP oracle — TEST INFRASTRUCTURE ONLY.

A CPU (NumPy/SciPy) restatement of the reference GICP
(/root/reference/python-implementation/gicp.py) used as the CHECKER of the
MI355X engine.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it; the product path (``generalized-icp_amd``)
never does and fails loudly when its HIP library is missing.

Parity pinning: the 2-D instantiation is checked against golden vectors
captured from the reference itself (``tests/golden/*.npz``, made by
``tests/golden/make_golden.py`` in the build container, NumPy 2.2.6 /
SciPy 1.15.3) — covariances, correspondence indices, weight matrices, the
loss at the reference's own optimum, and the final transform against the
reference's endpoint ensemble (``tests/test_oracle_golden.py``).  The 3-D
rules are the build's own (the reference is 2-D only); they
reduce to gicp.py in 2-D and are pinned by ground-truth recovery.

Third-party arithmetic the reference relies on (not vendored, versions pinned
by the fixtures): ``scipy.spatial.KDTree`` (exact k-NN, ``distance_upper_bound``
strict) and ``scipy.optimize.fmin_cg`` (Polak-Ribiere CG, gtol 1e-5,
maxiter 200 * len(x0)).
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import fmin_cg
from scipy.spatial import cKDTree

EPSILON = 100.0   # gicp.py:5
RATIO = 0.1       # gicp.py:11


def default_k(dim):
    return 6 if dim == 2 else 20   # gicp.py:24 (2-D); paper's 20 for 3-D


# ---------------------------------------------------------------------------
# covariances: gicp.py:5-35
# ---------------------------------------------------------------------------
def neighbourhoods(points, d_n, k=None, workers=1):
    """k nearest (self included) with distance strictly < d_n — gicp.py:21-25."""
    pts = np.asarray(points, dtype=np.float64)
    k = default_k(pts.shape[1]) if k is None else k
    tree = cKDTree(pts)
    dist, idx = tree.query(pts, k=min(k, len(pts)), distance_upper_bound=d_n, workers=workers)
    if idx.ndim == 1:
        dist, idx = dist[:, None], idx[:, None]
    valid = idx < len(pts)                      # gicp.py:25 drops index == len(points)
    return idx, valid, dist


def covariance_single_2d(neigh, epsilon=EPSILON, ratio=RATIO):
    """gicp.py:5-17 restated: principal eigenvector of np.cov -> R_v diag(eps, ratio*eps) R_v^T."""
    ground = np.array([[epsilon, 0.0], [0.0, epsilon * ratio]])
    cov = np.cov(neigh, rowvar=False)
    w, v = np.linalg.eig(cov)
    e = v[:, np.argmax(w)]                      # first index on ties (gicp.py:14)
    rv = np.array([[e[0], -e[1]], [e[1], e[0]]])
    return rv @ ground @ rv.T


def covariances(points, d_n, k=None, epsilon=EPSILON, ratio=RATIO, min_neighbors=None, faithful=None, workers=1):
    """Per-point surface covariances (gicp.py:19-35).

    2-D: > 1 neighbour -> ``covariance_single_2d`` else identity (gicp.py:27-34).
    3-D: >= 3 neighbours -> eps (I - n n^T) + ratio eps n n^T
    with n the eigenvector of the smallest eigenvalue of the sample
    covariance; else identity.
    ``faithful`` (default: 2-D with N <= 5000) calls np.cov / np.linalg.eig
    per point exactly like the reference; otherwise a batched equivalent.
    Returns (C [N,d,d], count [N]).
    """
    pts = np.asarray(points, dtype=np.float64)
    n, dim = pts.shape
    min_neighbors = (2 if dim == 2 else 3) if min_neighbors is None else min_neighbors
    idx, valid, _ = neighbourhoods(pts, d_n, k, workers)
    count = valid.sum(axis=1)
    out = np.empty((n, dim, dim))
    out[:] = np.eye(dim)
    faithful = (dim == 2 and n <= 5000) if faithful is None else faithful
    if faithful and dim == 2:
        for i in range(n):
            if count[i] >= min_neighbors:
                try:
                    out[i] = covariance_single_2d(pts[idx[i][valid[i]]], epsilon, ratio)
                except np.linalg.LinAlgError:   # gicp.py:31-32
                    out[i] = np.eye(2)
        return out, count
    ok = count >= min_neighbors
    safe = np.where(valid, idx, 0)
    nb = pts[safe]                                            # [n, k, d]
    w = valid[..., None].astype(np.float64)
    mean = (nb * w).sum(1) / np.maximum(count, 1)[:, None]
    c = (nb - mean[:, None, :]) * w
    cov = np.matmul(c.transpose(0, 2, 1), c) / np.maximum(count - 1, 1)[:, None, None]
    if dim == 2:
        ev, evec = np.linalg.eig(cov[ok])
        e = evec[np.arange(ok.sum()), :, np.argmax(ev, axis=1)]
        nrm = np.stack([-e[:, 1], e[:, 0]], axis=1)           # thin direction = principal rotated 90 deg
    else:
        ev, evec = np.linalg.eigh(cov[ok])
        nrm = evec[:, :, 0]                                   # smallest eigenvalue (ascending)
    out[ok] = epsilon * np.eye(dim) - epsilon * (1 - ratio) * np.einsum("ni,nj->nij", nrm, nrm)
    return out, count


# ---------------------------------------------------------------------------
# correspondences + weights: gicp.py:124-145
# ---------------------------------------------------------------------------
def apply_transformation(cloud, T):
    """gicp.py:176-177, any dimension."""
    d = T.shape[0] - 1
    return np.dot(np.asarray(cloud)[:, :d], T[:d, :d].T) + T[:d, d]


def correspondences(points, target, d_c, tree=None, workers=1):
    """Exact 1-NN in the target (gicp.py:127-133); accepted if d <= d_c (gicp.py:136)."""
    tree = cKDTree(target) if tree is None else tree
    dist, idx = tree.query(points, k=1, workers=workers)
    ok = dist <= d_c
    return np.where(ok, idx, -1), dist


def weights(cov_src, cov_tgt, idx):
    """W_i = inv(C_s,i + C_t,j) for accepted points, zeros otherwise (gicp.py:136-145)."""
    n, d, _ = cov_src.shape
    W = np.zeros((n, d, d))
    ok = idx >= 0
    W[ok] = np.linalg.inv(cov_src[ok] + cov_tgt[idx[ok]])
    return W


def weights_model(cov_src, cov_tgt, idx, model="plane_to_plane", tgt_count=None, min_neighbors=None):
    """The GICP paper's three covariance choices (reference slides presentation/main.typ:446-455):
    plane_to_plane = gicp.py:143-145; point_to_point (standard ICP): C_s = 0, C_t = I -> W = I;
    point_to_plane: C_s = 0, C_t = P^-1 -> W = P = n n^T, n the target's surface normal (eigenvector
    of the smallest eigenvalue of its covariance), W = 0 where the target point has no surface
    (fewer than min_neighbors neighbours: identity covariance, gicp.py:33-34)."""
    if model in ("plane_to_plane", "gicp"):
        return weights(cov_src, cov_tgt, idx)
    n, d, _ = cov_src.shape
    W = np.zeros((n, d, d))
    ok = idx >= 0
    if model in ("point_to_point", "icp"):
        W[ok] = np.eye(d)
        return W
    if model != "point_to_plane":
        raise ValueError(model)
    _, vec = np.linalg.eigh(cov_tgt[idx[ok]])
    nrm = vec[:, :, 0]
    Wok = np.einsum("ni,nj->nij", nrm, nrm)
    if tgt_count is not None:
        mn = d if min_neighbors is None else min_neighbors
        Wok[np.asarray(tgt_count)[idx[ok]] < mn] = 0.0
    W[ok] = Wok
    return W


def mse(s, q, idx, T):
    """Mean squared correspondence distance |q - (R s + t)|^2 over accepted points (PCL's
    calculateMSE over the pass's correspondences; the euclidean-fitness criterion of the
    reference's ROS experiment, presentation/main.typ:776)."""
    d = s.shape[1]
    ok = idx >= 0
    if not ok.any():
        return 0.0
    r = q[ok] - s[ok] @ T[:d, :d].T - T[:d, d]
    return float(np.mean(np.sum(r * r, axis=1)))


def pcl_stop(T_old, T_new, mse_cur, mse_prev, transformation_epsilon=0.0, rotation_epsilon=0.0,
             euclidean_fitness_epsilon=0.0, mse_relative_epsilon=0.0):
    """PCL DefaultConvergenceCriteria restated (transformation / absolute MSE / relative MSE, in that
    order, max similar iterations 0), on the increment T_new T_old^-1; rotation threshold
    1 - transformation_epsilon when unset.  The reference names these parameters
    (presentation/main.typ:773-776, 802-805) but ships no implementation: parity unpinned by it."""
    d = T_old.shape[0] - 1
    inc = T_new @ np.linalg.inv(T_old)
    cos_angle = 0.5 * (np.trace(inc[:d, :d]) - 1.0) if d == 3 else 0.5 * np.trace(inc[:d, :d])
    tsq = float(np.sum(inc[:d, d] ** 2))
    rot_thr = rotation_epsilon if rotation_epsilon > 0 else 1.0 - transformation_epsilon
    if transformation_epsilon > 0 and cos_angle >= rot_thr and tsq <= transformation_epsilon:
        return "transform"
    if euclidean_fitness_epsilon > 0 and abs(mse_cur - mse_prev) < euclidean_fitness_epsilon:
        return "abs_mse"
    if mse_relative_epsilon > 0 and np.isfinite(mse_prev) and abs(mse_cur - mse_prev) / mse_prev < mse_relative_epsilon:
        return "rel_mse"
    return None


# ---------------------------------------------------------------------------
# loss and its sufficient statistics: gicp.py:52-76
# ---------------------------------------------------------------------------
def rot2(theta):
    c, s = np.cos(theta), np.sin(theta)
    return np.array([[c, -s], [s, c]])


def loss_2d(x, s, q, W):
    """gicp.py:52-58 restated (vectorised over points)."""
    r = q - s @ rot2(x[2]).T - x[:2]
    wr = np.sum(W * r[:, None, :], axis=2)
    return np.sum(r * wr)


def grad_2d(x, s, q, W):
    """gicp.py:60-76 restated."""
    r = q - s @ rot2(x[2]).T - x[:2]
    wr = np.sum(W * r[:, None, :], axis=2)
    g = np.zeros(3)
    g[:2] = -2 * np.sum(wr, axis=0)
    dR = np.array([[-np.sin(x[2]), -np.cos(x[2])], [np.cos(x[2]), -np.sin(x[2])]])
    g[2] = np.sum(-2 * (wr.T @ s) * dR)
    return g


def sym_pairs(d):
    return [(a, b) for a in range(d) for b in range(a, d)]


def stats_size(d):
    ns = d * (d + 1) // 2
    return ns * ns + ns * d + ns + d * d + d + 2


def stats(s, q, W, idx, T_k):
    """Sufficient statistics of the loss around pose T_k (DESIGN.md §4 layout).

    With z = (vec R row-major, t) and r_i = q_i - R s_i - t:
      sum r^T W r = c0 - 2 g^T (z - z_k) + (z - z_k)^T H (z - z_k)
    A[ab][ij] = sum W_ab s_i s_j, B[ab][i] = sum W_ab s_i, C[ab] = sum W_ab,
    gR[a][i] = sum (W r_k)_a s_i, gt[a] = sum (W r_k)_a, c0 = sum r_k^T W r_k, count.
    Only accepted points (idx >= 0) contribute (W = 0 otherwise, gicp.py:137).
    """
    d = s.shape[1]
    ok = idx >= 0
    s, q, W = s[ok], q[ok], W[ok]
    r = q - s @ T_k[:d, :d].T - T_k[:d, d]
    wr = np.einsum("nab,nb->na", W, r)
    P = sym_pairs(d)
    ws = np.stack([W[:, a, b] for a, b in P], axis=1)           # [n, ns]
    ss = np.stack([s[:, i] * s[:, j] for i, j in P], axis=1)    # [n, ns]
    out = [np.einsum("np,nq->pq", ws, ss).ravel(), np.einsum("np,ni->pi", ws, s).ravel(), ws.sum(0),
           np.einsum("na,ni->ai", wr, s).ravel(), wr.sum(0), [np.sum(r * wr)], [float(ok.sum())]]
    return np.concatenate([np.asarray(o, dtype=np.float64).ravel() for o in out])


def expand_stats(st, d):
    """(H, g, c0, count) in z = (vec R, t) from the structured statistics."""
    P = sym_pairs(d)
    ns = len(P)
    pos = {}
    for k, (a, b) in enumerate(P):
        pos[(a, b)] = pos[(b, a)] = k
    o = 0
    A = st[o:o + ns * ns].reshape(ns, ns); o += ns * ns
    B = st[o:o + ns * d].reshape(ns, d); o += ns * d
    C = st[o:o + ns]; o += ns
    gR = st[o:o + d * d].reshape(d, d); o += d * d
    gt = st[o:o + d]; o += d
    c0, cnt = st[o], st[o + 1]
    nz = d * d + d
    H = np.zeros((nz, nz))
    for a in range(d):
        for i in range(d):
            for b in range(d):
                for j in range(d):
                    H[a * d + i, b * d + j] = A[pos[(a, b)], pos[(i, j)]]
                H[a * d + i, d * d + b] = H[d * d + b, a * d + i] = B[pos[(a, b)], i]
        for b in range(d):
            H[d * d + a, d * d + b] = C[pos[(a, b)]]
    g = np.concatenate([gR.ravel(), gt])
    return H, g, c0, cnt


def pose_vector(T):
    d = T.shape[0] - 1
    return np.concatenate([T[:d, :d].ravel(), T[:d, d]])


def quad_loss(T, H, g, c0, T_k):
    dz = pose_vector(T) - pose_vector(T_k)
    return c0 - 2 * g @ dz + dz @ H @ dz


# ---------------------------------------------------------------------------
# inner solvers (gicp.py:148-154)
# ---------------------------------------------------------------------------
def offset_to_T(x):
    """gicp.py:42-50."""
    T = np.eye(3)
    T[:2, :2] = rot2(x[2])
    T[:2, 2] = x[:2]
    return T


def skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def so3_exp(w):
    th = np.linalg.norm(w)
    K = skew(w)
    if th < 1e-12:
        return np.eye(3) + K + 0.5 * K @ K
    return np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K


def inner_gn(s, q, W, idx, T0, max_iter=100, tol=1e-14):
    """Exact minimiser of sum r^T W r over SE(d) by per-point Gauss-Newton
    (residuals recomputed every step, no closed form) — the 3-D inner solve
    of SURVEY.md §8.A, independent of the statistics path it checks."""
    d = s.shape[1]
    ok = idx >= 0
    s, q, W = s[ok], q[ok], W[ok]
    T = T0.copy()

    def f(T):
        r = q - s @ T[:d, :d].T - T[:d, d]
        return float(np.sum(r * np.matmul(W, r[:, :, None])[:, :, 0]))

    if len(s) == 0:
        return T, 0.0
    cur = f(T)
    lam = 0.0
    for _ in range(max_iter):
        R, t = T[:d, :d], T[:d, d]
        p = s @ R.T + t
        r = q - p
        # left perturbation T' = [exp(w), dt] o T: r' = q - exp(w) p - dt
        if d == 2:
            J = np.zeros((len(s), 2, 3))          # d r / d(theta, tx, ty)
            J[:, 0, 0], J[:, 1, 0] = p[:, 1], -p[:, 0]
            J[:, :, 1:] = -np.eye(2)
        else:
            J = np.zeros((len(s), 3, 6))          # d r / d(omega, dt)
            J[:, 0, 1], J[:, 0, 2] = -p[:, 2], p[:, 1]       # -[w]x p = [p]x w (skew(p), row by row)
            J[:, 1, 0], J[:, 1, 2] = p[:, 2], -p[:, 0]
            J[:, 2, 0], J[:, 2, 1] = -p[:, 1], p[:, 0]
            J[:, :, 3:] = -np.eye(3)
        JW = np.matmul(J.transpose(0, 2, 1), W)                       # J^T W per point
        na = JW.shape[1]
        JWf = JW.transpose(1, 0, 2).reshape(na, -1)                  # sums over points as one GEMM each
        Hm = JWf @ J.reshape(-1, na)
        gv = JWf @ r.reshape(-1)
        while True:
            step = -np.linalg.solve(Hm + lam * np.diag(np.diag(Hm)), gv)
            Tn = np.eye(d + 1)
            if d == 2:
                Rn = rot2(step[0]) @ R
            else:
                Rn = so3_exp(step[:3]) @ R
            Tn[:d, :d] = Rn
            Tn[:d, d] = rot2(step[0]) @ t + step[1:] if d == 2 else so3_exp(step[:3]) @ t + step[3:]
            new = f(Tn)
            if new <= cur or np.max(np.abs(step)) < tol:
                break
            lam = max(1e-9, lam * 10)
            if lam > 1e9:
                return T, cur
        T, cur = Tn, new
        lam = lam / 10 if lam > 1e-9 else 0.0
        if np.max(np.abs(step)) < tol:
            break
    if d == 2:   # keep a clean SO(2)
        th = np.arctan2(T[1, 0], T[0, 0])
        T[:2, :2] = rot2(th)
    return T, cur


# ---------------------------------------------------------------------------
# the outer loop: gicp.py:78-174
# ---------------------------------------------------------------------------
def gicp(source_points, target_points, max_iterations=100, tolerance=1e-6, max_distance_correspondence=150,
         max_distance_nearest_neighbors=50, inner=None, k=None, source_cov="auto", fixed_iterations=False,
         record=False, T0=None, method="plane_to_plane", transformation_epsilon=0.0, rotation_epsilon=0.0,
         euclidean_fitness_epsilon=0.0, mse_relative_epsilon=0.0, workers=1):
    """Oracle of gicp() returning the reference's 7-tuple (+ records if asked).

    workers: cKDTree query threads (the neighbourhoods and the correspondences; results are the same).

    method / the PCL-style epsilons: the §8(f) extensions (weights_model, pcl_stop); defaults are the
    reference's behaviour.

    inner: 'cg' (2-D default: scipy fmin_cg on the restated loss, reproducing
    the reference's inexact stopping), 'gn' (exact minimiser; 3-D default).
    source_cov: 'recompute' (gicp.py:120, 2-D default) or 'rotate'
    (R C_s,0 R^T, rigid-invariant; 3-D default).
    """
    src = np.asarray(source_points, dtype=np.float64)
    tgt = np.asarray(target_points, dtype=np.float64)
    d = src.shape[1]
    if tgt.shape[1] != d or d not in (2, 3):
        raise ValueError("source and target must both be N x 2 or N x 3")
    inner = ("cg" if d == 2 else "gn") if inner is None else inner
    if inner == "cg" and d != 2:
        raise ValueError("inner='cg' is the 2-D reference mode")
    if source_cov == "auto":
        source_cov = "recompute" if d == 2 else "rotate"
    d_c, d_n = max_distance_correspondence, max_distance_nearest_neighbors
    tgt_cov, tgt_cnt = covariances(tgt, d_n, k, workers=workers)
    pcl = dict(transformation_epsilon=transformation_epsilon, rotation_epsilon=rotation_epsilon,
               euclidean_fitness_epsilon=euclidean_fitness_epsilon, mse_relative_epsilon=mse_relative_epsilon)
    use_pcl = transformation_epsilon > 0 or euclidean_fitness_epsilon > 0 or mse_relative_epsilon > 0
    prev_mse = np.inf
    stop_reason = None
    tree = cKDTree(tgt)
    T = np.eye(d + 1) if T0 is None else np.array(T0, dtype=np.float64)
    all_T = [T]
    offset = np.array([T[0, 2], T[1, 2], np.arctan2(T[1, 0], T[0, 0])]) if d == 2 else None
    last = np.inf
    init_src_cov, _ = covariances(src, d_n, k, workers=workers)
    hw_s, hw_t, all_src_cov, recs = [], [], [], []
    converged_at = -1
    for it in range(max_iterations):
        moved = apply_transformation(src, T)
        if source_cov == "recompute":
            cs, _ = covariances(moved, d_n, k, workers=workers)
        else:
            R = T[:d, :d]
            cs = np.matmul(np.matmul(R, init_src_cov), R.T)
        all_src_cov.append(cs)
        idx, dist = correspondences(moved, tgt, d_c, tree, workers=workers)
        q = np.zeros_like(src)
        q[idx >= 0] = tgt[idx[idx >= 0]]
        W = weights_model(cs, tgt_cov, idx, method, tgt_cnt)
        if inner == "cg":
            out = fmin_cg(f=lambda x: loss_2d(x, src, q, W), x0=offset,
                          fprime=lambda x: grad_2d(x, src, q, W), disp=False, full_output=True)
            new_offset, min_loss = out[0], out[1]
            T_new = offset_to_T(new_offset)
        else:
            T_new, min_loss = inner_gn(src, q, W, idx, T)
            new_offset = None
        if record:
            recs.append(dict(T=T, idx=idx, dist=dist, q=q, W=W, T_new=T_new, loss=min_loss,
                             stats=stats(src, q, W, idx, T)))
        if not fixed_iterations and abs(last - min_loss) < tolerance:   # gicp.py:155-162
            converged_at = it
            break
        last = min_loss
        offset = new_offset
        if use_pcl and not fixed_iterations:
            m = mse(src, q, idx, T)
            stop_reason = pcl_stop(T, T_new, m, prev_mse, **pcl)
            prev_mse = m
        T = T_new
        all_T.append(T)
        top = np.argsort(np.linalg.det(W))[-5:]                       # gicp.py:170-172
        hw_s.append(moved[top])
        hw_t.append(q[top])
        if stop_reason is not None:
            converged_at = it
            break
    out = (T, all_T, init_src_cov, tgt_cov, hw_s, hw_t, all_src_cov)
    if record:
        return out, dict(iterations=recs, converged_at=converged_at, stop_reason=stop_reason)
    return out
