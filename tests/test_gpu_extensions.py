"""GPU parity of the SURVEY.md §8(f) extensions, through the C-ABI, against the oracle:
row 2 (top-5 det(W) selected on the device, gicp.py:169-172), row 3 (point-to-point / point-to-plane
covariance choices, presentation/main.typ:446-455) and row 4 (PCL-style stopping criteria,
presentation/main.typ:773-776).  The reference implements neither row 3 nor row 4 (its slides and
ROS experiment only name them): those are pinned to the oracle's restatement, not to the reference."""
import numpy as np
import pytest

from oracle import gicp_oracle as O

pytestmark = pytest.mark.gpu

gicp = pytest.importorskip("gicp")
from gicp import synthetic as S  # noqa: E402

P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
MODELS = {"point_to_point": 1, "point_to_plane": 2, "plane_to_plane": 0}


@pytest.fixture(scope="module")
def eng():
    e = gicp.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def scene3d():
    return S.scene_pair_3d(20000)


def _pose():
    T = np.eye(4)
    T[:3, :3] = S.axis_angle([1.0, -2.0, 0.5], np.deg2rad(1.5))
    T[:3, 3] = [0.05, -0.02, 0.01]
    return T


@pytest.mark.parametrize("model", ["point_to_point", "point_to_plane"])
def test_cov_model_pass_vs_oracle(eng, scene3d, model):
    """Indices bit-exact; W = I / n n^T to 1e-9; statistics to 1e-9 of the oracle's on the same q, W."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, cov_model=MODELS[model], **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    C_t = eng.covariances("target")
    cnt_t = eng.neighbor_counts("target")
    T = _pose()
    st, dbg = eng.iterate(T, debug=True)
    moved = O.apply_transformation(src, T)
    idx, _ = O.correspondences(moved, tgt, P3["max_distance_correspondence"])
    assert np.array_equal(dbg["index"], idx)
    W = O.weights_model(np.zeros((len(src), 3, 3)), C_t, idx, model, cnt_t)
    np.testing.assert_allclose(dbg["weight"], W, rtol=1e-9, atol=1e-12)
    q = np.zeros_like(src)
    q[idx >= 0] = tgt[idx[idx >= 0]]
    ref = O.stats(src, q, W, idx, T)
    np.testing.assert_allclose(st, ref, rtol=1e-9, atol=1e-9 * np.max(np.abs(ref)))


def test_pass_info_sum_sq_vs_oracle_mse(eng, scene3d):
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T = _pose()
    st = eng.iterate(T)
    info = eng.pass_info()
    moved = O.apply_transformation(src, T)
    idx, _ = O.correspondences(moved, tgt, P3["max_distance_correspondence"])
    q = np.zeros_like(src)
    q[idx >= 0] = tgt[idx[idx >= 0]]
    assert st[-1] == np.sum(idx >= 0)
    np.testing.assert_allclose(info["sum_sq"] / st[-1], O.mse(src, q, idx, T), rtol=1e-10)


@pytest.mark.parametrize("dim", [2, 3])
def test_top_weights_vs_argsort(eng, scene3d, dim):
    """gicp_top_weights == np.argsort(np.linalg.det(W))[-5:] of the same pass (gicp.py:170): the det
    values to 1e-9 and, where they are distinct, the same source points in the same order."""
    if dim == 3:
        src, tgt, _ = scene3d
        p = gicp.default_params(3, **P3)
        T = _pose()
    else:
        src, tgt, _ = S.segment_scene_2d(5000)
        p = gicp.default_params(2, max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0)
        T = np.eye(3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    _, dbg = eng.iterate(T, debug=True)
    det = np.linalg.det(dbg["weight"])
    ref = np.argsort(det, kind="stable")[-5:]
    st, si, ti, dt = eng.iterate_top(T, 5)
    np.testing.assert_allclose(dt, det[ref], rtol=1e-9)
    np.testing.assert_allclose(det[si], det[ref], rtol=1e-9)
    if len(np.unique(np.round(det[ref], 6))) == 5:
        assert np.array_equal(si, ref)
    assert np.array_equal(ti, dbg["index"][si])
    # k = 1 and k = 16, and the fallback when the shard is smaller than k
    _, si1, _, _ = eng.iterate_top(T, 1)
    assert si1[0] == si[-1]
    _, si16, _, dt16 = eng.iterate_top(T, 16)
    assert np.all(np.diff(dt16) >= 0) and si16[-1] == si[-1]


def test_top_weights_small_cloud(eng):
    rng = np.random.default_rng(3)
    tgt = rng.random((40, 3))
    src = tgt[:3] + 1e-3
    p = gicp.default_params(3, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    _, si, ti, dt = eng.iterate_top(np.eye(4), 5)
    assert np.array_equal(si[:2], [-1, -1]) and sorted(si[2:]) == [0, 1, 2]


def test_top_weights_requires_pass(eng, scene3d):
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    with pytest.raises(gicp._lib.GicpError):
        gicp._lib.check(eng._lib.gicp_top_weights(eng._ctx, 5, None, None, None), eng._ctx, "gicp_top_weights")


@pytest.mark.parametrize("crit", [dict(transformation_epsilon=1e-8), dict(euclidean_fitness_epsilon=1e-7),
                                  dict(mse_relative_epsilon=1e-4)])
def test_pcl_criteria_device_matches_host_loop(eng, scene3d, crit):
    """k_solve's PCL-style test (device loop, gicp_align) stops at the same iteration, for the same
    reason and with the same pose as the host loop over the same passes (gicp.pcl_stop), whose
    rule is the oracle's pcl_stop."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, max_iterations=40, tolerance=0.0, **P3, **crit)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    Tdev, res = eng.align(None, p)
    T = np.eye(4)
    prev = np.inf
    reason = None
    its = 0
    for it in range(40):
        st = eng.iterate(T)
        mse = eng.pass_info()["sum_sq"] / st[-1]
        Tn, _ = gicp.solve_pose(st, T)
        its += 1
        reason = gicp.pcl_stop(T, Tn, mse, prev, **crit)
        assert reason == O.pcl_stop(T, Tn, mse, prev, **crit)
        prev = mse
        T = Tn
        if reason:
            break
    assert reason is not None and res["stop_reason"] == reason
    assert res["iterations"] == its and res["converged"] == 1
    np.testing.assert_allclose(Tdev, T, rtol=0, atol=1e-10)
    np.testing.assert_allclose(res["mse"], mse, rtol=1e-12)


@pytest.mark.parametrize("method", ["point_to_point", "point_to_plane"])
def test_gicp_methods_end_to_end_vs_oracle(scene3d, method):
    """The drop-in with method= against the oracle's outer loop (exact Gauss-Newton inner solve both
    sides): same endpoint to 1e-6 rad / 1e-6 m, and the ground truth recovered to the noise level."""
    src, tgt, Tgt = S.scene_pair_3d(8000)
    kw = dict(max_iterations=40, tolerance=1e-10, **P3)
    T, all_T, *_ = gicp.gicp(src, tgt, method=method, full_output=False, verbose=False, **kw)
    To, *_ = O.gicp(src, tgt, method=method, **kw)
    assert S.rotation_angle_error(T, To) < 1e-6 and S.translation_error(T, To) < 1e-6
    # point-to-point ICP on independently sampled surfaces is biased by the sampling (~2.5 cm here)
    tol_r, tol_t = (3e-3, 5e-2) if method == "point_to_point" else (2e-3, 2e-2)
    assert S.rotation_angle_error(T, Tgt) < tol_r and S.translation_error(T, Tgt) < tol_t


def test_gicp_full_output_top5_vs_oracle():
    """The 7-tuple's highest-weight lists (gicp.py:169-172) from the device top-k: per iteration the
    5 selected source points carry the 5 largest det(W) of the oracle's pass (to 1e-9; which of
    several exactly tied points -- e.g. isolated ones, W = I/2 -- is taken is the sort's choice,
    np.argsort's default is not stable), and their targets are the oracle's correspondences."""
    from scipy.spatial import cKDTree
    src, tgt, _ = S.scene_pair_3d(4000)
    kw = dict(max_iterations=3, tolerance=0.0, **P3)
    out = gicp.gicp(src, tgt, verbose=False, **kw)
    _, rec = O.gicp(src, tgt, fixed_iterations=True, record=True, **kw)
    assert len(out[4]) == len(out[5]) == 3
    for it in range(3):
        r = rec["iterations"][it]
        det = np.linalg.det(r["W"])
        moved = O.apply_transformation(src, r["T"])
        d, sel = cKDTree(moved).query(out[4][it])
        assert np.all(d < 1e-6)
        np.testing.assert_allclose(np.sort(det[sel]), np.sort(det)[-5:], rtol=1e-9)
        np.testing.assert_allclose(out[5][it], r["q"][sel], atol=1e-9)


def test_align_without_timing_events_is_identical(eng, scene3d):
    """timing_stride < 0 (bench.py's timed run) records no HIP events: the same pose and statistics,
    no sampled kernel time; the default stride samples every 8th launch."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=12, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T_ev, r_ev = eng.align(None, p)
    p.timing_stride = -1
    T_no, r_no = eng.align(None, p)
    assert np.array_equal(T_ev, T_no)
    assert r_no["final_loss"] == r_ev["final_loss"] and r_no["iterations"] == r_ev["iterations"] == 12
    assert r_no["corr_samples"] == 0 and r_no["corr_kernel_ms"] == 0.0
    assert r_ev["corr_samples"] == 2 and r_ev["corr_kernel_ms"] > 0.0


@pytest.mark.parametrize("dim", [2, 3])
def test_rotated_covariances_vs_host_einsum(eng, scene3d, dim):
    """gicp_rotated_covariances (device, a I - (R m)(R m)^T) == R C R^T of the copied covariances
    (the host einsum gicp.py:120-121 is restated by), original order, to 1e-12 of the entries."""
    if dim == 3:
        src, tgt, _ = scene3d
        p = gicp.default_params(3, **P3)
        R = _pose()[:3, :3]
    else:
        src, tgt, _ = S.segment_scene_2d(5000)
        p = gicp.default_params(2, max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0)
        R = O.rot2(0.3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    for which in ("source", "target"):
        C0 = eng.covariances(which)
        ref = np.einsum("ab,nbc,dc->nad", R, C0, R)
        got = eng.rotated_covariances(R, which)
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-12 * np.abs(ref).max())


def test_gicp_full_output_rotated_covariances_lazy(scene3d):
    """all_source_cov_matrices of the fast path (gicp.py:121) is a lazy view: one element per executed
    iteration, each == R_k C_s R_k^T of that iteration's pose (host einsum, 1e-12), computed from the
    initial covariances on the host whatever the engine holds."""
    src, tgt, _ = scene3d
    kw = dict(max_iterations=4, tolerance=0.0, **P3)
    T, all_T, init_cov, _, _, _, all_cov = gicp.gicp(src, tgt, verbose=False, **kw)
    assert isinstance(all_cov, gicp.RotatedCovariances) and len(all_cov) == 4
    refs = [np.einsum("ab,nbc,dc->nad", Tk[:3, :3], init_cov, Tk[:3, :3]) for Tk in all_T[:4]]
    for k in range(4):
        np.testing.assert_allclose(all_cov[k], refs[k], rtol=0, atol=1e-12 * np.abs(refs[k]).max())
    gicp.gicp(src[:5000], tgt[:5000], verbose=False, full_output=False, **kw)   # the engine's source changes
    np.testing.assert_allclose(all_cov[-1], refs[-1], rtol=0, atol=1e-12 * np.abs(refs[-1]).max())
    assert len(list(all_cov)) == 4 and len(all_cov[1:3]) == 2


def test_gicp_2d_large_cloud_defaults_to_fast_mode(monkeypatch):
    """A 2-D 100k call takes mode='fast' (no per-point W / index copied back: every pass is a
    statistics-only gicp_iterate or the device top-k), and agrees with an explicit mode='fast' call."""
    src, tgt, _ = S.segment_scene_2d(100_000)
    kw = dict(max_iterations=6, tolerance=0.0, max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0)
    seen = []
    orig = gicp.Engine.iterate

    def spy(self, T, debug=False):
        seen.append(debug)
        return orig(self, T, debug=debug)

    monkeypatch.setattr(gicp.Engine, "iterate", spy)
    T, all_T, *_ = gicp.gicp(src, tgt, verbose=False, full_output=False, **kw)
    assert seen and not any(seen), "a large 2-D call copied per-point weights to the host"
    n_full = len(seen)
    seen.clear()
    out = gicp.gicp(src, tgt, verbose=False, **kw)   # full_output: top-5 on the device, lazy covariances
    assert not any(seen) and isinstance(out[6], gicp.RotatedCovariances)
    monkeypatch.undo()
    T2, *_ = gicp.gicp(src, tgt, verbose=False, full_output=False, mode="fast", **kw)
    np.testing.assert_array_equal(T, T2)
    assert n_full == len(all_T) - 1


@pytest.mark.parametrize("name", ["vis_s3", "robot_p0_r360"])
def test_gicp_2d_faithful_with_initial_pose_vs_oracle(name):
    """mode='faithful' with a non-identity T0: the first pass runs on the source moved by T0
    (gicp.py:119-120), as the oracle does; same endpoint as the oracle's loop, and all_src_cov[0] is
    the covariance set of the moved cloud."""
    from golden_util import kwargs, load
    fx = load(name)
    T0 = O.offset_to_T(np.array([1.5, -0.8, 0.01]))
    kw = kwargs(fx)
    out = gicp.gicp(fx["source"], fx["target"], T0=T0, verbose=False, **kw)
    ref = O.gicp(fx["source"], fx["target"], T0=T0, **kw)
    moved0 = O.apply_transformation(fx["source"], T0)
    cov0, _ = O.covariances(moved0, kw["max_distance_nearest_neighbors"])
    np.testing.assert_allclose(out[6][0], cov0, atol=1e-10)
    assert np.allclose(out[1][0], T0)
    th = lambda T: np.arctan2(T[1, 0], T[0, 0])  # noqa: E731
    assert abs(th(out[0]) - th(ref[0])) < 1e-4 and np.max(np.abs(out[0][:2, 2] - ref[0][:2, 2])) < 1e-3


def test_reset_cache_changes_no_result(eng, scene3d):
    """gicp_reset_cache drops lists / certificates / last matches: a cold align gives the bit-identical
    pose and loss of a warm one, and per-iteration kernel times cover every launch over 8 offsets."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=16, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T_a, r_a = eng.align(None, p)
    T_w, r_w = eng.align(None, p)        # warm: caches from the first call
    eng.reset_cache()
    T_c, r_c = eng.align(None, p)        # cold again
    assert np.array_equal(T_a, T_w) and np.array_equal(T_a, T_c)
    assert r_a["final_loss"] == r_w["final_loss"] == r_c["final_loss"]
    times = np.full(16, np.nan)
    for off in range(8):
        p.timing_offset = off
        eng.reset_cache()
        eng.align(None, p)
        t = eng.iteration_times()
        assert len(t) == 16 and np.sum(~np.isnan(t)) == 2
        times[~np.isnan(t)] = t[~np.isnan(t)]
    assert np.all(times > 0)


def test_native_library_built_from_these_sources(eng):
    """Build provenance on the GPU box: the library this process runs was compiled
    from exactly the sources in this tree (gicp_build_info's hash = the tree's), and it is the in-tree
    build (not a copy elsewhere)."""
    import os

    from gicp import _lib
    info = _lib.build_info()
    assert info["src"] == _lib.source_hash(), info
    assert os.path.dirname(_lib.LIB_PATH) == os.path.dirname(os.path.abspath(gicp.__file__))
    print(f"gicp_build_info: {info}")


@pytest.mark.parametrize("tile", ["32", "16"])
def test_smaller_source_tiles_same_correspondences(monkeypatch, scene3d, tile):
    """GICP_SRC_TILE (source tiles of at most 32 / 16 points): the same exact nearest neighbours
    as the oracle's KD-tree (indices bit-exact), statistics within 1e-11 of the 64-point tiling's (the per-unit
    partial sums group the points differently), and the same registration to 1e-9."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=8, **P3)
    T = _pose()
    moved = O.apply_transformation(src, T)
    idx, _ = O.correspondences(moved, tgt, P3["max_distance_correspondence"])
    out = {}
    for t in ("64", tile):
        monkeypatch.setenv("GICP_SRC_TILE", t)
        e = gicp.Engine(0)
        try:
            e.set_target(tgt, p)
            e.set_source(src, p)
            st, dbg = e.iterate(T, debug=True)
            Tr, _ = e.align(None, p)
        finally:
            e.close()
        out[t] = (st, dbg["index"], Tr)
    assert np.array_equal(out[tile][1], idx)
    ref = out["64"][0]
    np.testing.assert_allclose(out[tile][0], ref, rtol=1e-11, atol=1e-11 * np.max(np.abs(ref)))
    np.testing.assert_allclose(out[tile][2], out["64"][2], rtol=0, atol=1e-9)
