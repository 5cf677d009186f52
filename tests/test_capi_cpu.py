"""CPU-side checks of libgicp_hip.so: it loads, exports every declared entry point, and its
host solver (pure host code) agrees with the oracle.  No GPU compute is called here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from golden_util import load, names
from oracle import gicp_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gicp_hip.h")

gicp = pytest.importorskip("gicp")
from gicp import _lib  # noqa: E402


def declared_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(gicp_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    syms = declared_symbols()
    assert len(syms) >= 16
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_lib.SIGNATURES), "ctypes table out of sync with include/gicp_hip.h"


def test_build_info_matches_the_sources_in_this_tree():
    """gicp_build_info() carries the hash of the sources it was compiled from; it must be the hash of
    the sources beside it (a stale or foreign library fails here)."""
    info = _lib.build_info()
    assert info["arch"] == "gfx950"
    assert info["src"] == _lib.source_hash(), (info, "rebuild: make -C generalized-icp_amd/csrc")


def test_basic_host_entry_points():
    lib = _lib.load()
    assert lib.gicp_version() >= 100
    assert lib.gicp_stats_size(2) == 26 and lib.gicp_stats_size(3) == 74
    assert lib.gicp_stats_size(4) < 0
    p = gicp.default_params(2)
    assert (p.max_iterations, p.k_neighbors, p.tolerance) == (100, 6, 1e-6)          # gicp.py:78, :24
    assert (p.max_distance_correspondence, p.max_distance_nearest_neighbors) == (150, 50)
    assert (p.epsilon, p.ratio) == (100.0, 0.1)                                      # gicp.py:5, :11
    assert gicp.default_params(3).k_neighbors == 20
    assert lib.gicp_strerror(-1) == b"invalid argument"


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = C.c_void_p()
    rc = _lib.load().gicp_create(C.byref(ctx), 0)
    assert rc == _lib.GICP_E_HIP and not ctx.value
    with pytest.raises(_lib.GicpError):
        gicp.Engine(0)


def test_stats_layout_matches_oracle():
    assert gicp.stats_size(2) == O.stats_size(2) == 26
    assert gicp.stats_size(3) == O.stats_size(3) == 74
    rng = np.random.default_rng(0)
    for d in (2, 3):
        st = rng.normal(size=O.stats_size(d))
        H1, g1, c1, n1 = O.expand_stats(st, d)
        H2, g2, c2, n2 = gicp.expand_stats(st, d)
        assert np.array_equal(H1, H2) and np.array_equal(g1, g2) and c1 == c2 and n1 == n2


@pytest.mark.parametrize("name", ["vis_s0", "vis_s3", "robot_p0_r360", "segment_2k"])
def test_host_solver_2d_matches_oracle_gn(name):
    """gicp_solve_pose on oracle statistics == per-point Gauss-Newton of the oracle (same minimiser)."""
    fx = load(name)
    src = fx["source"]
    for k in range(min(3, len(fx["W"]))):
        Tk = fx["all_T"][k]
        st = O.stats(src, fx["q"][k], fx["W"][k], fx["idx"][k], Tk)
        T1, f1 = gicp.solve_pose(st, Tk)
        T2, f2 = O.inner_gn(src, fx["q"][k], fx["W"][k], fx["idx"][k], Tk)
        if abs(f1 - f2) > 1e-6 * max(1, f2):
            # non-convex in theta: both must at least be stationary points not above the start
            assert f1 <= O.loss_2d(fx["x0"][k], src, fx["q"][k], fx["W"][k]) * (1 + 1e-12)
            continue
        np.testing.assert_allclose(T1, T2, atol=1e-7)
        # the loss the solver reports is the true loss at its pose
        x = np.array([T1[0, 2], T1[1, 2], np.arctan2(T1[1, 0], T1[0, 0])])
        assert abs(O.loss_2d(x, src, fx["q"][k], fx["W"][k]) - f1) <= 1e-8 * max(1.0, f1)


def test_host_solver_3d_matches_oracle_gn():
    rng = np.random.default_rng(3)
    n = 400
    s = rng.uniform(-5, 5, (n, 3))
    Tg = np.eye(4)
    Tg[:3, :3] = O.so3_exp(np.array([0.03, -0.02, 0.05]))
    Tg[:3, 3] = [0.2, -0.1, 0.3]
    q = O.apply_transformation(s, Tg) + rng.normal(0, 0.01, (n, 3))
    A = rng.normal(size=(n, 3, 3))
    W = np.einsum("nij,nkj->nik", A, A) + 0.5 * np.eye(3)
    idx = np.arange(n)
    idx[::17] = -1
    Tk = np.eye(4)
    Tk[:3, 3] = [0.1, 0, 0.1]
    st = O.stats(s, q, W, idx, Tk)
    T1, f1 = gicp.solve_pose(st, Tk)
    T2, f2 = O.inner_gn(s, q, W, idx, Tk)
    np.testing.assert_allclose(T1, T2, atol=1e-9)
    assert abs(f1 - f2) <= 1e-8 * f2
    assert np.allclose(T1[:3, :3] @ T1[:3, :3].T, np.eye(3), atol=1e-12)


def test_host_solver_no_correspondences_keeps_pose():
    st = np.zeros(74)
    Tk = np.eye(4)
    Tk[:3, 3] = [1, 2, 3]
    T, f = gicp.solve_pose(st, Tk)
    assert np.array_equal(T, Tk) and f == 0.0


def test_apply_transformation_matches_reference_formula():
    rng = np.random.default_rng(1)
    pts = rng.normal(size=(10, 2))
    T = O.offset_to_T([1.0, -2.0, 0.3])
    np.testing.assert_array_equal(gicp.apply_transformation(pts, T), np.dot(pts[:, :2], T[:2, :2].T) + T[:2, 2])


def test_golden_names_cover_both_demos():
    n = names()
    assert any(x.startswith("robot_") for x in n) and any(x.startswith("vis_") for x in n)
