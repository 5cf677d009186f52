"""GPU parity: the HIP path (through the C-ABI) against the reference's golden vectors (2-D)
and the oracle (3-D).  Bit-exact for correspondence indices; fp64 tolerances stated per test."""
import numpy as np
import pytest

from golden_util import DIVERGENT, in_ensemble, kwargs, load, names
from oracle import gicp_oracle as O

pytestmark = pytest.mark.gpu

gicp = pytest.importorskip("gicp")
from gicp import synthetic as S  # noqa: E402

NAMES = names()


@pytest.fixture(scope="module")
def eng():
    e = gicp.Engine(0)
    yield e
    e.close()


def _params(fx):
    kw = kwargs(fx)
    return gicp.default_params(2, **kw)


# ----------------------------------------------------------------------------- 2-D golden
@pytest.mark.parametrize("name", NAMES)
def test_covariances_2d_vs_reference(eng, name):
    """k_knn_cov vs gicp.py:104/:111 outputs captured from the reference (atol 1e-10 on entries ~100)."""
    fx = load(name)
    p = _params(fx)
    eng.set_target(fx["target"], p)
    eng.set_source(fx["source"], p)
    np.testing.assert_allclose(eng.covariances("target"), fx["tgt_cov"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(eng.covariances("source"), fx["init_src_cov"], rtol=0, atol=1e-10)


@pytest.mark.parametrize("name", NAMES)
def test_iteration_2d_vs_reference(eng, name):
    """Given the reference's T_k: indices bit-exact, W to 1e-8 rel (rotated vs recomputed source
    covariances), statistics == oracle statistics of the reference's q/W (1e-8 rel)."""
    fx = load(name)
    p = _params(fx)
    eng.set_target(fx["target"], p)
    eng.set_source(fx["source"], p)
    for k in range(len(fx["W"])):
        Tk = fx["all_T"][k]
        st, dbg = eng.iterate(Tk, debug=True)
        assert np.array_equal(dbg["index"], fx["idx"][k]), f"iteration {k}"
        np.testing.assert_allclose(dbg["weight"], fx["W"][k], rtol=1e-8, atol=1e-14)
        ref = O.stats(fx["source"], fx["q"][k], fx["W"][k], fx["idx"][k], Tk)
        scale = np.maximum(np.abs(ref), 1e-12 * np.max(np.abs(ref)))
        assert np.max(np.abs(st - ref) / scale) < 1e-7, k


STABLE = ["vis_s3", "robot_p0_r90", "robot_p2_r90", "robot_p0_r360", "robot_p2_r360", "segment_2k"]


@pytest.mark.parametrize("name", STABLE)
def test_gicp_2d_fast_mode_in_reference_ensemble(name):
    """The closed-form path (one GPU reduction per iteration + fmin_cg on the statistics) on the
    fixtures where the reference endpoint is stable under input perturbation."""
    fx = load(name)
    T, *_ = gicp.gicp(fx["source"], fx["target"], mode="fast", full_output=False, verbose=False, **kwargs(fx))
    ok, best = in_ensemble(T, fx["ens_T"])
    assert ok, best


@pytest.mark.parametrize("name", [n for n in NAMES if n not in DIVERGENT])
def test_gicp_2d_end_to_end_in_reference_ensemble(name, capsys):
    """Drop-in gicp() on the GPU lands within 1e-4 rad / 1e-3 px of the reference's endpoint ensemble."""
    fx = load(name)
    out = gicp.gicp(fx["source"], fx["target"], **kwargs(fx))
    assert len(out) == 7
    T, all_T, init_cov, tgt_cov, hw_s, hw_t, all_cov = out
    ok, best = in_ensemble(T, fx["ens_T"])
    assert ok, best
    # gicp.py:121,167: one covariance set per executed iteration; all_T grows only when not converged
    n_exec = len(all_cov)
    assert len(all_T) == (n_exec + 1 if n_exec == int(fx["max_iterations"]) and len(all_T) > n_exec else n_exec)
    assert len(hw_s) == len(all_T) - 1 and hw_s[0].shape == (5, 2)
    np.testing.assert_allclose(tgt_cov, fx["tgt_cov"], atol=1e-10)
    np.testing.assert_allclose(init_cov, fx["init_src_cov"], atol=1e-10)
    k = min(len(all_cov), len(fx["all_src_cov"]))
    np.testing.assert_allclose(all_cov[0], fx["all_src_cov"][0], atol=1e-10)
    if np.allclose(T, fx["T"], atol=1e-6):
        # |delta loss| < 1e-6 on losses ~1e3 decides at the 1e-9 relative level, below the rounding
        # difference of any two evaluations of the loss: the stop may come one iteration apart
        assert abs(len(all_T) - len(fx["all_T"])) <= 1
        assert ("Converged at iteration" in capsys.readouterr().out) == bool(fx["converged"])


# ----------------------------------------------------------------------------- 3-D vs oracle
@pytest.fixture(scope="module")
def scene3d():
    src, tgt, Tgt = S.scene_pair_3d(20000)
    return src, tgt, Tgt


P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)


def test_covariances_3d_vs_oracle(eng, scene3d):
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    C_gpu = eng.covariances("target")
    cnt_gpu = eng.neighbor_counts("target")
    C_or, cnt_or = O.covariances(tgt, P3["max_distance_nearest_neighbors"])
    assert np.array_equal(cnt_gpu, np.minimum(cnt_or, 20))
    err = np.max(np.abs(C_gpu - C_or), axis=(1, 2))
    # the normal of a near-isotropic neighbourhood is ill-conditioned; everything else to 1e-8
    assert np.quantile(err, 0.999) < 1e-8, np.quantile(err, 0.999)
    assert np.mean(err > 1e-6) < 1e-3


def test_iteration_3d_vs_oracle(eng, scene3d):
    src, tgt, Tgt = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    C_t = eng.covariances("target")
    C_s = eng.covariances("source")
    T = np.eye(4)
    T[:3, 3] = [0.05, -0.02, 0.01]
    st, dbg = eng.iterate(T, debug=True)
    moved = O.apply_transformation(src, T)
    idx, dist = O.correspondences(moved, tgt, P3["max_distance_correspondence"])
    assert np.array_equal(dbg["index"], idx)
    # distances are exact where a target point lies inside the screen bound (~d_c); beyond it the
    # kernel reports inf (the point is rejected either way, gicp.py:136)
    fin = np.isfinite(dbg["distance"])
    assert np.all(fin[idx >= 0]) and np.all(dist[~fin] > P3["max_distance_correspondence"])
    np.testing.assert_allclose(dbg["distance"][fin], dist[fin], rtol=1e-12)
    R = T[:3, :3]
    W = O.weights(np.einsum("ab,nbc,dc->nad", R, C_s, R), C_t, idx)
    np.testing.assert_allclose(dbg["weight"], W, rtol=1e-9, atol=1e-15)
    q = np.zeros_like(src)
    q[idx >= 0] = tgt[idx[idx >= 0]]
    ref = O.stats(src, q, W, idx, T)
    np.testing.assert_allclose(st, ref, rtol=1e-9, atol=1e-9 * np.max(np.abs(ref)))


def test_align_3d_vs_oracle_and_ground_truth(eng, scene3d):
    src, tgt, Tgt = scene3d
    p = gicp.default_params(3, max_iterations=30, tolerance=1e-9, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T, res = eng.align(None, p)
    To, all_T, *_ = O.gicp(src, tgt, max_iterations=30, tolerance=1e-9, **P3)
    from golden_util import pose_err
    a, t = pose_err(T, To)
    assert a < 1e-6 and t < 1e-6, (a, t)
    a, t = pose_err(T, Tgt)
    assert a < 2e-4 and t < 2e-3, (a, t)   # recovers 2 deg / 19 cm to noise level
    assert res["iterations"] == len(all_T) or res["converged"]


def test_sharded_statistics_sum_to_full(eng, scene3d):
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    T = np.eye(4)
    eng.set_source(src, p)
    full = eng.iterate(T)
    parts = []
    for s in range(3):
        eng.set_source(src, p, shard=s, nshards=3)
        parts.append(eng.iterate(T))
    np.testing.assert_allclose(np.sum(parts, axis=0), full, rtol=1e-12, atol=1e-12 * np.max(np.abs(full)))


def test_sharded_source_computes_its_own_covariances(eng, scene3d):
    """a sharded source builds the covariances of its own tiles only -- those rows equal
    the unsharded build's bit for bit, the other rows are NaN, and the shards' rows partition the cloud."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    full = eng.covariances("source")
    assert not np.isnan(full).any()
    owner = np.full(len(src), -1)
    for s in range(3):
        eng.set_source(src, p, shard=s, nshards=3)
        c = eng.covariances("source")
        mine = ~np.isnan(c[:, 0, 0])
        assert np.isnan(c[~mine]).all() and not np.isnan(c[mine]).any()
        assert np.array_equal(c[mine], full[mine])
        assert np.all(owner[mine] == -1)
        owner[mine] = s
    assert np.all(owner >= 0)


def test_iterate_is_deterministic(eng, scene3d):
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T = np.eye(4)
    a = eng.iterate(T)
    b = eng.iterate(T)
    assert np.array_equal(a, b)


def test_device_solve_matches_host_solve(eng, scene3d):
    """k_solve (one wave, lane-parallel Newton) reaches the same pose as the host solver on the
    statistics of the same pass, for two successive iterations (2-D and 3-D)."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, fixed_iterations=1, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T = np.eye(4)
    for n in (1, 2):
        p.max_iterations = n
        Tdev, _ = eng.align(None, p)
        st = eng.iterate(T)
        T, loss = gicp.solve_pose(st, T)
        np.testing.assert_allclose(Tdev, T, rtol=0, atol=1e-12)
    fx = load("robot_p0_r90")
    kw = kwargs(fx)
    p2 = gicp.default_params(2, fixed_iterations=1, max_iterations=1,
                             max_distance_correspondence=float(kw["max_distance_correspondence"]),
                             max_distance_nearest_neighbors=float(kw["max_distance_nearest_neighbors"]))
    eng.set_target(fx["target"], p2)
    eng.set_source(fx["source"], p2)
    Tdev, _ = eng.align(None, p2)
    Th, _ = gicp.solve_pose(eng.iterate(np.eye(3)), np.eye(3))
    np.testing.assert_allclose(Tdev, Th, rtol=0, atol=1e-11)


# ----------------------------------------------------------------------------- edge cases
def test_duplicates_and_ties_2d(eng):
    """Exact duplicate target points (ties) and a point on the d_c boundary."""
    rng = np.random.default_rng(5)
    tgt = rng.uniform(0, 100, (300, 2))
    tgt = np.concatenate([tgt, tgt[:50]])           # 50 exact duplicates
    src = tgt[:200] + rng.normal(0, 0.5, (200, 2))
    p = gicp.default_params(2, max_distance_correspondence=3.0, max_distance_nearest_neighbors=10.0)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    C_or, _ = O.covariances(tgt, 10.0)
    np.testing.assert_allclose(eng.covariances("target"), C_or, atol=1e-9)
    st, dbg = eng.iterate(np.eye(3), debug=True)
    idx, dist = O.correspondences(src, tgt, 3.0)
    same = dbg["index"] == idx
    # where indices differ they must be exact duplicates (identical coordinates)
    assert np.all(same | np.all(tgt[np.maximum(dbg["index"], 0)] == tgt[np.maximum(idx, 0)], axis=1))
    np.testing.assert_allclose(dbg["distance"], dist, rtol=1e-13)


def test_tiny_and_disjoint_clouds(eng):
    p = gicp.default_params(2, max_distance_correspondence=1.0, max_distance_nearest_neighbors=5.0)
    eng.set_target(np.array([[0.0, 0.0]]), p)
    eng.set_source(np.array([[0.5, 0.0], [10.0, 10.0]]), p)
    np.testing.assert_array_equal(eng.covariances("target"), np.eye(2)[None])   # isolated -> I
    st, dbg = eng.iterate(np.eye(3), debug=True)
    assert list(dbg["index"]) == [0, -1]
    assert st[-1] == 1.0
    eng.set_source(np.array([[50.0, 50.0]]), p)
    st = eng.iterate(np.eye(3))
    assert np.all(st == 0)
    T, f = gicp.solve_pose(st, np.eye(3))
    assert np.array_equal(T, np.eye(3)) and f == 0.0


def test_boundary_distances_exact(eng):
    """d_c inclusive (gicp.py:136) and d_n strict (KDTree distance_upper_bound) at exact distances."""
    tgt = np.array([[0.0, 0.0], [3.0, 0.0], [10.0, 0.0], [0.0, 4.0]])
    p = gicp.default_params(2, max_distance_correspondence=3.0, max_distance_nearest_neighbors=4.0)
    eng.set_target(tgt, p)
    eng.set_source(np.array([[-3.0, 0.0], [13.0000001, 0.0]]), p)
    st, dbg = eng.iterate(np.eye(3), debug=True)
    assert list(dbg["index"]) == [0, -1]            # distance exactly 3 accepted, 3.0000001 rejected
    cnt = eng.neighbor_counts("target")
    _, cnt_or = O.covariances(tgt, 4.0)
    assert list(cnt) == list(cnt_or)                # (0,0)-(0,4) at exactly 4: excluded


def test_one_rank_rccl_allreduce_is_identity(scene3d):
    """The RCCL all-reduce inside gicp_align/gicp_iterate (the multi-GPU exchange)
    on a one-rank communicator: the library's stream path with the collective enqueued between
    k_corr and k_solve must give bit-identical statistics and poses to the path without it."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=6, **P3)
    res = []
    for with_comm in (False, True):
        e = gicp.Engine(0)
        try:
            if with_comm:
                e.comm_init(1, 0, gicp.Engine.comm_unique_id())
            e.set_target(tgt, p)
            e.set_source(src, p)
            st = e.iterate(np.eye(4))
            T, r = e.align(None, p)
            res.append((st, T, r["iterations"]))
        finally:
            e.close()
    assert np.array_equal(res[0][0], res[1][0])
    assert np.array_equal(res[0][1], res[1][1]) and res[0][2] == res[1][2] == 6


def test_nn_certificates_do_not_change_results(scene3d, monkeypatch):
    """Per-point nearest-neighbour certificates and the per-lane search cap from the last match
     skip or shorten walks for lanes whose nearest target is provably unchanged; the
    candidate lists (adaptive skin) and the super-block level only change which tiles a walk tests.
    A 60-iteration fixed run and single passes around its endpoint must be bit-identical across the
    default engine, one without certificates (GICP_NO_CERTS=1, no cap either) and one without
    certificates or lists (plain full walks), one without the target graph's descent, the sparse-wave
    search off and on for every walking wave, and the lane-parallel fp64 re-resolution
    (GICP_SPARSE_AMB) off and on for every wave with an ambiguous lane, while the certified passes evaluate
    far fewer pairs."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=60, **P3)
    out = {}
    for flag in ("0", "1", "plain", "nograph", "sparse_off", "sparse_all", "sparse_all_plain", "amb_off", "amb_all"):
        monkeypatch.setenv("GICP_NO_GRAPH", "1" if flag == "nograph" else "0")
        monkeypatch.setenv("GICP_SPARSE_AMB", "0" if flag == "amb_off" else "64" if flag == "amb_all" else "2")
        monkeypatch.setenv("GICP_NO_CERTS", "1" if flag in ("1", "plain", "sparse_all_plain") else "0")
        monkeypatch.setenv("GICP_NO_LISTS", "1" if flag in ("plain", "sparse_all_plain") else "0")
        monkeypatch.setenv("GICP_SPARSE_WALK", "0" if flag == "sparse_off" else "64" if flag.startswith("sparse_all") else "2")
        e = gicp.Engine(0)
        try:
            e.set_target(tgt, p)
            e.set_source(src, p)
            T, r = e.align(None, p)
            sts = [e.iterate(T), e.iterate(T)]
            Tn = T.copy()
            Tn[:3, 3] += [1e-4, -2e-4, 5e-5]          # a small move: most certificates still hold
            sts.append(e.iterate(Tn))
            Tf = T.copy()
            Tf[:3, 3] += [0.2, 0.0, 0.0]              # a large one: they must not
            sts.append(e.iterate(Tf))
            out[flag] = (T, sts, e.pass_info()["pairs"], r["pairs_evaluated"])
        finally:
            e.close()
    for other in ("1", "plain", "nograph", "sparse_off", "sparse_all", "sparse_all_plain", "amb_off", "amb_all"):
        assert np.array_equal(out["0"][0], out[other][0]), other
        for a, b in zip(out["0"][1], out[other][1]):
            assert np.array_equal(a, b)
    assert out["0"][3] < 0.05 * out["1"][3]            # the converged pass walked almost nothing


def test_target_graph_rows_cover_their_radius(eng, scene3d):
    """The target neighbour graph: every target nearer than radius[i] to point i is in
    row i (cKDTree ball query, fp64), rows hold distinct other points, and the radius is the distance
    of a neighbour the row does not hold (so rows are the nearest ones, up to the screen's error)."""
    from scipy.spatial import cKDTree
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    idx, rad = eng.graph()
    assert idx.shape == (len(tgt), 20) and np.all(rad > 0)
    tree = cKDTree(tgt)
    d21, _ = tree.query(tgt, k=22)
    assert np.all(rad <= d21[:, 21] * (1 + 1e-5))            # at most the 21st other neighbour's distance
    # ... and not much below the 20th's, or the neighbourhood cap d_n when fewer lie within it
    assert np.all(rad >= np.minimum(d21[:, 20], P3["max_distance_nearest_neighbors"]) * (1 - 1e-3) - 1e-6)
    for i in range(0, len(tgt), 97):
        row = idx[i][idx[i] >= 0]
        assert i not in row and len(set(row)) == len(row)
        assert np.all(idx[i][len(row):] < 0)                   # real entries first, then the -1 pads
        d = np.linalg.norm(tgt[row] - tgt[i], axis=1)          # nearest-first (the descent's early exit)
        assert np.all(np.diff(d) >= -1e-6 * (1.0 + d[1:])), (i, d)
        ball = [t for t in tree.query_ball_point(tgt[i], rad[i]) if t != i and np.linalg.norm(tgt[t] - tgt[i]) < rad[i]]
        assert set(ball) <= set(row), i


def test_graph_descent_along_a_moving_pose(scene3d, monkeypatch):
    """Graph descent proves nearest neighbours while the pose still moves by centimetres to decimetres:
    a sequence of passes with growing steps gives bit-identical statistics and correspondence indices with
    and without the graph (GICP_NO_GRAPH=1) and with every walking wave searched lane-parallel
    (GICP_SPARSE_WALK=64) or every ambiguous lane re-resolved wave-wide (GICP_SPARSE_AMB=0),
    and with the graph the moving passes screen fewer pairs."""
    src, tgt, _ = scene3d
    p = gicp.default_params(3, **P3)
    poses = []
    for k, step in enumerate([0.0, 0.002, 0.01, 0.03, 0.08, 0.15, 0.01, 0.001]):
        T = np.eye(4)
        T[:3, :3] = S.axis_angle([1.0, 0.5 * k, -0.3], step * 0.2)
        T[:3, 3] = [step, -0.5 * step, 0.25 * step]
        poses.append(T)
    out = {}
    for flag in ("0", "1", "sparse_all", "amb_off"):
        monkeypatch.setenv("GICP_NO_GRAPH", "1" if flag == "1" else "0")
        monkeypatch.setenv("GICP_SPARSE_WALK", "64" if flag == "sparse_all" else "2")
        monkeypatch.setenv("GICP_SPARSE_AMB", "0" if flag == "amb_off" else "2")
        e = gicp.Engine(0)
        try:
            e.set_target(tgt, p)
            e.set_source(src, p)
            sts, pairs = [], []
            for T in poses:
                st, dbg = e.iterate(T, debug=True)
                sts.append((st, dbg["index"]))
                pairs.append(e.pass_info()["pairs"])
            out[flag] = (sts, pairs)
        finally:
            e.close()
    for other in ("1", "sparse_all", "amb_off"):
        for (a, ia), (b, ib) in zip(out["0"][0], out[other][0]):
            assert np.array_equal(ia, ib) and np.array_equal(a, b), other
    assert sum(out["0"][1][1:]) < sum(out["1"][1][1:])


def test_large_coordinate_offsets(eng):
    """Clouds in map coordinates (UTM-like offsets of ~5e6 m): the screen works tile-relative, so the
    correspondences stay bit-exact and W exact, and the loop still recovers the ground truth."""
    src, tgt, Tgt = S.scene_pair_3d(20000)
    off = np.array([451234.5, 5402187.25, 123.0])
    so, to = src + off, tgt + off
    p = gicp.default_params(3, **P3)
    eng.set_target(to, p)
    eng.set_source(so, p)
    C_t = eng.covariances("target")
    C_s = eng.covariances("source")
    st, dbg = eng.iterate(np.eye(4), debug=True)
    idx, _ = O.correspondences(so, to, P3["max_distance_correspondence"])
    assert np.array_equal(dbg["index"], idx)
    np.testing.assert_allclose(dbg["weight"], O.weights(C_s, C_t, idx), rtol=1e-9, atol=1e-15)
    p = gicp.default_params(3, max_iterations=40, tolerance=1e-12, **P3)
    T, _ = eng.align(None, p)
    Oo = np.eye(4)
    Oo[:3, 3] = off
    Tgt_o = Oo @ Tgt @ np.linalg.inv(Oo)          # the same motion expressed in the offset frame
    # statistics about the far-away origin lose ~8 digits (s s^T ~ 1e13): the pose is judged where it
    # acts, on the cloud (max point displacement vs the true motion), not by its lever-arm translation
    disp = np.max(np.linalg.norm(O.apply_transformation(so, T) - O.apply_transformation(so, Tgt_o), axis=1))
    assert S.rotation_angle_error(T, Tgt_o) < 1e-4 and disp < 5e-3, disp


def test_non_finite_input_is_rejected(eng):
    pts = np.random.default_rng(0).random((100, 3))
    pts[17, 1] = np.nan
    with pytest.raises(ValueError):
        eng.set_target(pts, gicp.default_params(3))
    pts[17, 1] = np.inf
    with pytest.raises(ValueError):
        eng.set_source(pts, gicp.default_params(3))


def test_foreign_hip_error_does_not_fail_the_next_call(eng, scene3d):
    """HIP's last error is per thread and shared with every HIP user on it.  A failed call of
    another user (here hipSetDevice on a device that does not exist, through the HIP runtime directly) left
    on this thread must not make the library's next launch check report GICP_E_HIP."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipSetDevice(ctypes.c_int(4096)) != 0   # the foreign failure, left unread
    src, tgt, _ = scene3d
    p = gicp.default_params(3, max_iterations=3, fixed_iterations=1, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    assert hip.hipSetDevice(ctypes.c_int(4096)) != 0
    T, res = eng.align(None, p)
    assert res["iterations"] == 3 and np.all(np.isfinite(T))
    assert hip.hipSetDevice(ctypes.c_int(4096)) != 0
    st = eng.iterate(np.eye(4))
    assert st[-1] > 0
