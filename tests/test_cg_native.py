"""The native 2-D inner solve (gicp_cg_inner_2d, csrc/gicp_cg.cpp) against scipy.optimize.fmin_cg itself.

The reference's inner solve is fmin_cg (gicp.py:152).  The fast mode runs the same algorithm natively on the
closed form of the loss; here scipy's fmin_cg minimises the very same closed form (written below in plain
Python floats, operation for operation as the C++ evaluates it), so any difference is the CG / line-search
restatement's: xopt, fopt, nfev, ngev and warnflag must agree BIT FOR BIT.  Statistics: the oracle's on
the reference's own per-iteration q / W / T_k of every golden fixture, plus random and degenerate ones.
Pure host code: runs without a GPU."""
import ctypes as C
import math
import warnings

import numpy as np
import pytest

from golden_util import load, names
from oracle import gicp_oracle as O

gicp = pytest.importorskip("gicp")
from gicp import _lib  # noqa: E402

L2 = [[0, 0, 1, 0], [0, 0, 0, -1], [0, 0, 0, 1], [0, 0, 1, 0], [1, 0, 0, 0], [0, 1, 0, 0]]


def closed_form(st, Tk):
    """f, g of the loss on 26 statistics, Python floats in the C++'s operation order."""
    st = [float(v) for v in st]

    def pos(a, b):
        return (0 if a == 0 else 2) if a == b else 1
    A, B, Cc, gR, gt = st[0:9], st[9:15], st[15:18], st[18:22], st[22:24]
    H = [[0.0] * 6 for _ in range(6)]
    for a in range(2):
        for i in range(2):
            for b in range(2):
                for j in range(2):
                    H[a * 2 + i][b * 2 + j] = A[pos(a, b) * 3 + pos(i, j)]
                H[a * 2 + i][4 + b] = H[4 + b][a * 2 + i] = B[pos(a, b) * 2 + i]
    for a in range(2):
        for b in range(2):
            H[4 + a][4 + b] = Cc[pos(a, b)]
    g6 = gR + gt
    g4 = []
    H4 = [[0.0] * 4 for _ in range(4)]
    for p in range(4):
        s = 0.0
        for i in range(6):
            s += L2[i][p] * g6[i]
        g4.append(s)
        for q in range(4):
            s = 0.0
            for i in range(6):
                for j in range(6):
                    s += L2[i][p] * H[i][j] * L2[j][q]
            H4[p][q] = s
    c0 = st[24]
    zk = [float(Tk[0, 2]), float(Tk[1, 2]), float(Tk[0, 0]), float(Tk[1, 0])]

    def terms(x):
        c, s = math.cos(float(x[2])), math.sin(float(x[2]))
        dz = [float(x[0]) - zk[0], float(x[1]) - zk[1], c - zk[2], s - zk[3]]
        Hd = []
        for p in range(4):
            h = 0.0
            for q in range(4):
                h += H4[p][q] * dz[q]
            Hd.append(h)
        return dz, Hd, c, s

    def f(x):
        dz, Hd, _, _ = terms(x)
        gz = q = 0.0
        for p in range(4):
            gz += g4[p] * dz[p]
        for p in range(4):
            q += dz[p] * Hd[p]
        return (c0 - 2.0 * gz) + q

    def g(x):
        dz, Hd, c, s = terms(x)
        v = [-2.0 * g4[p] + 2.0 * Hd[p] for p in range(4)]
        return np.array([v[0], v[1], -s * v[2] + c * v[3]])
    return f, g


def native(st, Tk, x0):
    lib = _lib.load()
    st = np.ascontiguousarray(st, dtype=np.float64)
    Tk = np.ascontiguousarray(Tk, dtype=np.float64)
    x0 = np.ascontiguousarray(x0, dtype=np.float64)
    x = np.zeros(3)
    fo = C.c_double()
    cnt = (C.c_int32 * 4)()
    rc = lib.gicp_cg_inner_2d(_lib.dptr(st), _lib.dptr(Tk), _lib.dptr(x0), _lib.dptr(x), C.byref(fo), cnt)
    assert rc == 0
    return x, fo.value, list(cnt)


def scipy_cg(st, Tk, x0):
    from scipy.optimize import fmin_cg
    f, g = closed_form(st, Tk)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        xo, fo, nf, ng, wf = fmin_cg(f, np.array(x0, dtype=np.float64), fprime=g, disp=False, full_output=True)
    return xo, fo, [nf, ng, wf]


def check_bitwise(st, Tk, x0):
    xn, fn, cn = native(st, Tk, x0)
    xs, fs, cs = scipy_cg(st, Tk, x0)
    assert cn[:3] == cs, (cn, cs)
    assert np.array_equal(xn, xs), (xn, xs, xn - xs)
    assert fn == fs or (math.isnan(fn) and math.isnan(fs)), (fn, fs)
    return cn


def test_numpy_dot_of_small_vectors_is_an_fma_chain():
    """The restatement's dot() assumption (scipy's np.dot of its 3-vectors): fma(a2, b2, fma(a1, b1, a0 b0))."""
    from fractions import Fraction as F
    rng = np.random.default_rng(3)
    for _ in range(500):
        a = rng.standard_normal(3) * 10.0 ** rng.uniform(-3, 3, 3)
        b = rng.standard_normal(3) * 10.0 ** rng.uniform(-3, 3, 3)
        s = 0.0
        for i in range(3):
            s = float(F(float(a[i])) * F(float(b[i])) + F(s))
        assert np.dot(a, b) == s


@pytest.mark.parametrize("name", names())
def test_bitwise_on_the_reference_iterations(name):
    """Every iteration of every golden fixture: the oracle's statistics of the reference's own q / W at the
    reference's T_k, from the reference's x0 -- native == scipy fmin_cg bit for bit."""
    fx = load(name)
    src = fx["source"]
    n = min(len(fx["x0"]), len(fx["q"]))   # (segment_2k keeps q / W of its first iterations only)
    for k in range(n):
        T_k = fx["all_T"][min(k, len(fx["all_T"]) - 1)]
        st = O.stats(src, fx["q"][k], fx["W"][k], fx["idx"][k], T_k)
        check_bitwise(st, T_k, fx["x0"][k])


def test_bitwise_on_random_and_degenerate_statistics():
    rng = np.random.default_rng(11)
    fx = load("vis_s0")
    src = fx["source"]
    idx = fx["idx"][0]
    used = 0
    for trial in range(40):
        th = rng.uniform(-math.pi, math.pi)
        T_k = np.array([[math.cos(th), -math.sin(th), rng.normal(0, 50)], [math.sin(th), math.cos(th), rng.normal(0, 50)],
                        [0, 0, 1]])
        q = src @ T_k[:2, :2].T + T_k[:2, 2] + rng.normal(0, 3, src.shape)
        W = fx["W"][0] * rng.uniform(0.1, 10)
        st = O.stats(src, q, W, idx, T_k)
        x0 = np.array([T_k[0, 2], T_k[1, 2], th]) + rng.normal(0, [5, 5, 0.3])
        used += check_bitwise(st, T_k, x0)[3] > 0
    assert used > 30
    # no correspondence at all: zero statistics, gradient 0 at once (no iteration)
    z = np.zeros(26)
    assert check_bitwise(z, np.eye(3), np.array([1.0, 2.0, 0.3]))[3] == 0


def test_cg_inner_uses_the_native_solve(monkeypatch):
    """gicp._cg_inner (the fast mode's inner solve) is the native call, not scipy."""
    import scipy.optimize
    fx = load("robot_p0_r360")
    T_k = fx["all_T"][0]
    st = O.stats(fx["source"], fx["q"][0], fx["W"][0], fx["idx"][0], T_k)

    def boom(*a, **k):
        raise AssertionError("scipy fmin_cg called on the product path")
    monkeypatch.setattr(scipy.optimize, "fmin_cg", boom)
    x, fopt = gicp._cg_inner(st, fx["x0"][0], T_k)
    xn, fn, _ = native(st, T_k, fx["x0"][0])
    assert np.array_equal(x, xn) and fopt == fn
