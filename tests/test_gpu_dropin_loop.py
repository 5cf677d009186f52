"""The drop-in gicp() on the device-resident loop (gicp_align_trace) and on several devices.

gicp.py:116-172 returns the pose plus per-iteration lists (all_transformations, the top-5 det(W)
points, the per-iteration source covariances).  In fast mode with the Newton inner solve, gicp()
now runs the whole loop in ONE gicp_align_trace call and gets those rows from the device; these
tests hold it to a host-driven loop over the same engine (gicp_iterate + gicp_solve_pose +
gicp_top_weights at every pose: the loop gicp() ran before), and hold devices= to device=."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

gicp = pytest.importorskip("gicp")
from gicp import synthetic as S  # noqa: E402

P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)


@pytest.fixture(scope="module")
def scene():
    return S.scene_pair_3d(20000)


def _host_loop(src, tgt, max_iterations, tolerance, k=5):
    """gicp.py:116-172 driven from the host over the C-ABI (one pass, one host solve per iteration)."""
    eng = gicp.Engine(0)
    try:
        p = gicp.default_params(3, **P3)
        eng.set_target(tgt, p)
        eng.set_source(src, p)
        T = np.eye(4)
        all_T, tops, poses, losses = [T], [], [], []
        last = np.inf
        for it in range(max_iterations):
            st, si, ti, _ = eng.iterate_top(T, k)
            poses.append(T)
            Tn, loss = gicp.solve_pose(st, T)
            losses.append(loss)
            if abs(last - loss) < tolerance:
                return T, all_T, tops, poses, losses, it
            last = loss
            tops.append((si, ti))
            T = Tn
            all_T.append(T)
        return T, all_T, tops, poses, losses, None
    finally:
        eng.close()


@pytest.mark.parametrize("tol", [0.0, 1e-6])
def test_trace_rows_match_host_loop(scene, tol):
    """Engine.align(trace=True): every row (pose the pass ran at, min_loss, top-5 source / target
    indices) equals the host loop's at the same iteration to 1e-9 (indices exactly)."""
    src, tgt, _ = scene
    n = 12
    T_h, all_T, tops, poses, losses, conv = _host_loop(src, tgt, n, tol)
    eng = gicp.Engine(0)
    try:
        p = gicp.default_params(3, max_iterations=n, tolerance=tol, **P3)
        eng.set_target(tgt, p)
        eng.set_source(src, p)
        T, res, tr = eng.align(None, p, trace=True, top_k=5)
    finally:
        eng.close()
    np.testing.assert_allclose(T, T_h, atol=1e-9)
    assert res["iterations"] == len(poses) == len(tr["poses"])
    assert (res["converged_at"] if res["converged"] else None) == conv
    for k in range(len(poses)):
        np.testing.assert_allclose(tr["poses"][k], poses[k], atol=1e-9)
        np.testing.assert_allclose(tr["losses"][k], losses[k], rtol=1e-9)
    for k, (si, ti) in enumerate(tops):
        assert np.array_equal(tr["top_src"][k], si) and np.array_equal(tr["top_tgt"][k], ti)


def test_trace_without_top_k_and_bad_capacity(scene):
    src, tgt, _ = scene
    eng = gicp.Engine(0)
    try:
        p = gicp.default_params(3, max_iterations=5, **P3)
        eng.set_target(tgt, p)
        eng.set_source(src, p)
        T1, r1 = eng.align(None, p)
        T2, r2, tr = eng.align(None, p, trace=True)
        assert np.array_equal(T1, T2) and r1["iterations"] == r2["iterations"] == len(tr["poses"])
        assert "top_src" not in tr
        np.testing.assert_array_equal(tr["poses"][0], np.eye(4))
        import ctypes as C
        from gicp import _lib
        poses = np.zeros((4, 4, 4))
        bad = _lib.Trace(4, 0, _lib.dptr(poses), None, None, None, None)   # capacity 4 < max_iterations 5
        Tout = np.empty((4, 4))
        rc = _lib.load().gicp_align_trace(eng._ctx, _lib.dptr(np.eye(4)), C.byref(p), _lib.dptr(Tout), None,
                                          C.byref(bad))
        assert rc == _lib.GICP_E_INVALID and b"capacity" in _lib.load().gicp_last_error(eng._ctx)
        bad = _lib.Trace(8, 17, _lib.dptr(np.zeros((8, 4, 4))), None, None, None, None)
        rc = _lib.load().gicp_align_trace(eng._ctx, _lib.dptr(np.eye(4)), C.byref(p), _lib.dptr(Tout), None,
                                          C.byref(bad))
        assert rc == _lib.GICP_E_INVALID
    finally:
        eng.close()


def test_dropin_device_loop_matches_host_loop(scene, capsys):
    """gicp() 3-D (fast, Newton): the 7-tuple equals the host loop's -- pose and all_transformations to
    1e-9, the top-5 rows' points exactly, one rotated covariance set per executed iteration, and the
    reference's print (gicp.py:161) on convergence."""
    src, tgt, _ = scene
    T_h, all_T_h, tops, poses, _, conv = _host_loop(src, tgt, 40, 1e-6)
    assert conv is not None, "the scene converges within 40 iterations"
    out = gicp.gicp(src, tgt, max_iterations=40, tolerance=1e-6, **P3)
    assert capsys.readouterr().out.strip() == f"Converged at iteration {conv}"
    T, all_T, init_cov, tgt_cov, hw_s, hw_t, all_cov = out
    np.testing.assert_allclose(T, T_h, atol=1e-9)
    assert len(all_T) == len(all_T_h) == conv + 1
    for a, b in zip(all_T, all_T_h):
        np.testing.assert_allclose(a, b, atol=1e-9)
    assert len(hw_s) == len(hw_t) == len(tops) == conv
    for k, (si, ti) in enumerate(tops):
        np.testing.assert_allclose(hw_s[k], gicp.apply_transformation(src[si], poses[k]), atol=1e-9)
        q = np.zeros((len(si), 3))
        q[ti >= 0] = tgt[ti[ti >= 0]]
        np.testing.assert_array_equal(hw_t[k], q)
    assert isinstance(all_cov, gicp.RotatedCovariances) and len(all_cov) == conv + 1
    R = poses[-1][:3, :3]
    np.testing.assert_allclose(all_cov[-1], np.einsum("ab,nbc,dc->nad", R, init_cov, R), atol=1e-12 * 100)


def test_dropin_max_iterations_keeps_last_update(scene):
    """No convergence: max_iterations + 1 transformations (gicp.py:108,167), the last one the result."""
    src, tgt, _ = scene
    T, all_T, *_ , hw_s, hw_t, all_cov = gicp.gicp(src, tgt, max_iterations=3, tolerance=0.0, verbose=False, **P3)
    assert len(all_T) == 4 and np.array_equal(all_T[-1], T)
    assert len(hw_s) == len(hw_t) == 3 and len(all_cov) == 3


def test_rotated_covariances_cached_and_picklable(scene):
    """the reference reads all_source_cov_matrices[step][i] per point (visualization.py:158);
    each step is computed once (two cached), re-reads are bit-identical whatever the engine did since,
    and the list pickles (robot-visualization.py's worker returns results through a Queue)."""
    import pickle
    src, tgt, _ = scene
    out = gicp.gicp(src, tgt, max_iterations=4, tolerance=0.0, verbose=False, **P3)
    acm = out[6]
    first = acm[2].copy()
    for i in range(200):
        _ = acm[2][i]
        _ = acm[3][i]
    assert acm.computed == 2
    gicp.gicp(src[:3000], tgt[:3000], max_iterations=2, tolerance=0.0, verbose=False, **P3)   # engine changes
    acm._cache.clear()
    assert np.array_equal(acm[2], first)
    back = pickle.loads(pickle.dumps(acm))
    assert len(back) == len(acm) and np.array_equal(back[2], first)


def test_devices_list_of_one_is_device(scene):
    """devices=[0] is the device=0 call bit for bit; duplicates and absent GPUs are refused."""
    src, tgt, _ = scene
    kw = dict(max_iterations=8, tolerance=0.0, verbose=False, **P3)
    a = gicp.gicp(src, tgt, device=0, **kw)
    b = gicp.gicp(src, tgt, devices=[0], **kw)
    assert np.array_equal(a[0], b[0]) and all(np.array_equal(x, y) for x, y in zip(a[1], b[1]))
    with pytest.raises(ValueError, match="more than once"):
        gicp.gicp(src, tgt, devices=[0, 0], **kw)
    with pytest.raises(ValueError, match="no such GPU"):
        gicp.gicp(src, tgt, devices=[0, 4096], **kw)
    with pytest.raises(ValueError):
        gicp.gicp(src, tgt, devices=[], **kw)


@pytest.mark.parametrize("loop", ["device", "host"])
def test_two_contexts_one_gpu_as_two_devices(scene, loop):
    """The multi-device path of gicp() (one thread per GPU, statistics summed in device order every
    iteration) run on two contexts of the one GPU, shards 0 and 1 of 2: pose within 1e-9 of the
    one-device call, the top-5 rows merged across the shards equal to the one-device rows."""
    src, tgt, _ = scene
    kw = dict(max_iterations=10, tolerance=0.0, verbose=False, **P3)
    ref = gicp.gicp(src, tgt, **kw)
    engines = [gicp.Engine(0), gicp.Engine(0)]
    try:
        p = gicp.default_params(3, max_iterations=10, tolerance=0.0, **P3)
        for r, e in enumerate(engines):
            e.set_target(tgt, p)
            e.set_source(src, p, shard=r, nshards=2)
        init = engines[0].covariances("source")
        tcov = engines[0].covariances("target")
        if loop == "device":
            out = gicp._device_loop(engines, src, tgt, np.eye(4), p, True, False, init, tcov)
        else:
            pcl = dict(transformation_epsilon=0.0, rotation_epsilon=0.0, euclidean_fitness_epsilon=0.0,
                       mse_relative_epsilon=0.0)
            out = gicp._host_loop(engines, src, tgt, np.eye(4), None, p, pcl, "fast", "newton", True, False, init,
                                  tcov)
    finally:
        for e in engines:
            e.close()
    np.testing.assert_allclose(out[0], ref[0], atol=1e-9)
    assert len(out[1]) == len(ref[1]) and len(out[4]) == len(ref[4])
    for a, b in zip(out[4], ref[4]):
        np.testing.assert_allclose(a, b, atol=1e-6)
    for a, b in zip(out[5], ref[5]):
        np.testing.assert_array_equal(a, b)
