"""GPU parity at BASELINE.json's full sizes (configs[1] 100k/100k, configs[2] 1M/1M, configs[4] one
100k-point LiDAR frame pair): the oracle's cKDTree on the GPU box's host cores checks every
correspondence of a 1M pass bit-exactly and its statistics to 1e-9, and size-independent properties
cover the rest (shard additivity, certificates on/off bit-identity, ground-truth recovery)."""
import os

import numpy as np
import pytest

from oracle import gicp_oracle as O

pytestmark = pytest.mark.gpu

gicp = pytest.importorskip("gicp")
from gicp import synthetic as S  # noqa: E402

P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
WORKERS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def eng():
    e = gicp.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def scene1m():
    return S.scene_pair_3d(1_000_000)


def _pose(deg=1.0, t=(0.06, -0.03, 0.02)):
    T = np.eye(4)
    T[:3, :3] = S.axis_angle([0.3, -1.0, 0.7], np.deg2rad(deg))
    T[:3, 3] = t
    return T


def test_pass_1m_vs_oracle(eng, scene1m):
    """configs[2]: every one of the 1M correspondence indices equals the oracle's cKDTree answer,
    W to 1e-9 relative, the 74 statistics to 1e-9 of the oracle's on the same q and W."""
    src, tgt, _ = scene1m
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    C_s = eng.covariances("source")
    C_t = eng.covariances("target")
    T = _pose()
    st, dbg = eng.iterate(T, debug=True)
    moved = O.apply_transformation(src, T)
    idx, _ = O.correspondences(moved, tgt, P3["max_distance_correspondence"], workers=WORKERS)
    assert np.array_equal(dbg["index"], idx)
    R = T[:3, :3]
    W = O.weights(np.einsum("ab,nbc,dc->nad", R, C_s, R), C_t, idx)
    np.testing.assert_allclose(dbg["weight"], W, rtol=1e-9, atol=1e-15)
    q = np.zeros_like(src)
    q[idx >= 0] = tgt[idx[idx >= 0]]
    ref = O.stats(src, q, W, idx, T)
    np.testing.assert_allclose(st, ref, rtol=1e-9, atol=1e-9 * np.max(np.abs(ref)))


def test_covariances_1m_vs_oracle(eng, scene1m):
    _, tgt, _ = scene1m
    p = gicp.default_params(3, **P3)
    eng.set_target(tgt, p)
    C_gpu = eng.covariances("target")
    cnt_gpu = eng.neighbor_counts("target")
    C_or, cnt_or = O.covariances(tgt, P3["max_distance_nearest_neighbors"], workers=WORKERS)
    assert np.array_equal(cnt_gpu, np.minimum(cnt_or, 20))
    err = np.max(np.abs(C_gpu - C_or), axis=(1, 2))
    assert np.quantile(err, 0.999) < 1e-8, np.quantile(err, 0.999)
    assert np.mean(err > 1e-6) < 1e-3


def test_align_1m_properties(eng, scene1m):
    """30 fixed iterations at 1M (the bench workload): ground truth recovered; 8 shards' statistics
    sum to the full pass; graph descent / certificates / lists on or off, and every workgroup -> unit map
    (XCD stripes throughout, chunk-interleaved throughout), give bit-identical poses."""
    src, tgt, Tgt = scene1m
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=30, **P3)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    T, res = eng.align(None, p)
    assert S.rotation_angle_error(T, Tgt) < 2e-5 and S.translation_error(T, Tgt) < 2e-4
    assert res["iterations"] == 30 and res["correspondences"] > 990_000
    full = eng.iterate(T)
    parts = []
    for s in range(8):
        eng.set_source(src, p, shard=s, nshards=8)
        parts.append(eng.iterate(T))
    np.testing.assert_allclose(np.sum(parts, axis=0), full, rtol=1e-11, atol=1e-11 * np.max(np.abs(full)))
    # without certificates (and their search cap), then also without candidate lists: same poses, bit for bit
    for env in ({"GICP_NO_GRAPH": "1"}, {"GICP_NO_CERTS": "1"}, {"GICP_NO_CERTS": "1", "GICP_NO_LISTS": "1"},
                {"GICP_MOVING_ITERS": "0"}, {"GICP_MOVING_ITERS": "0", "GICP_UNIT_MAP": "1"},
                {"GICP_MOVING_ITERS": "30", "GICP_MOVING_MAP": "3"}, {"GICP_SPARSE_WALK": "0"}, {"GICP_SPARSE_WALK": "8"},
                {"GICP_SPARSE_AMB": "0"}, {"GICP_SPARSE_AMB": "64"}):
        os.environ.update(env)
        try:
            e2 = gicp.Engine(0)
        finally:
            for k in env:
                del os.environ[k]
        try:
            e2.set_target(tgt, p)
            e2.set_source(src, p)
            T2, _ = e2.align(None, p)
        finally:
            e2.close()
        assert np.array_equal(T, T2), env


def test_align_1m_vs_oracle_loop(scene1m):
    """configs[2] itself (the bench's 1M/1M clouds) through the drop-in's whole outer loop against the
    oracle's loop, iteration by iteration: the driver's 20 fixed iterations from the identity (bench.py
    --steps 20: the moving passes and the settling ones), all 21 poses element-wise within 1e-9."""
    src, tgt, Tgt = scene1m
    kw = dict(max_iterations=20, tolerance=0.0, **P3)   # tolerance 0: the rule never fires, 20 iterations
    out = gicp.gicp(src, tgt, full_output=True, verbose=False, **kw)
    ref = O.gicp(src, tgt, workers=16, **kw)
    assert len(out[1]) == len(ref[1]) == 21
    for k, (Tg, To) in enumerate(zip(out[1], ref[1])):
        # element-wise (an angle from arccos cannot resolve below ~1.5e-8 rad)
        err = np.max(np.abs(Tg - To))
        assert err < 1e-9, (k, err)
    assert S.rotation_angle_error(out[0], Tgt) < S.rotation_angle_error(np.eye(4), Tgt)


def test_align_100k_vs_oracle(eng):
    """configs[1]: the whole outer loop at 100k/100k against the oracle's (exact inner solves both)."""
    src, tgt, Tgt = S.scene_pair_3d(100_000)
    kw = dict(max_iterations=12, tolerance=1e-9, **P3)
    T, *_ = gicp.gicp(src, tgt, full_output=False, verbose=False, **kw)
    To, *_ = O.gicp(src, tgt, **kw)
    assert S.rotation_angle_error(T, To) < 1e-7 and S.translation_error(T, To) < 1e-6
    assert S.rotation_angle_error(T, Tgt) < 1e-4 and S.translation_error(T, Tgt) < 1e-3


def test_lidar_frame_pair_vs_oracle():
    """configs[4]: one 100k-point spinning-LiDAR frame pair (the odometry step's registration) against
    the oracle; many source points have no target within d_c here (rejected lanes, certificates of
    empty neighbourhoods)."""
    frames = list(S.lidar_stream(3))
    prev, cur = frames[1][0], frames[2][0]
    kw = dict(max_iterations=15, tolerance=1e-9, **P3)
    T, *_ = gicp.gicp(prev, cur, full_output=False, verbose=False, **kw)
    To, *_ = O.gicp(prev, cur, **kw)
    assert S.rotation_angle_error(T, To) < 1e-6 and S.translation_error(T, To) < 1e-5


def test_2d_100k_fast_mode_vs_oracle(eng):
    """VERDICT r02 missing 3: 2-D parity at scale.  The BASELINE.md §3 segment scene at 100k/100k
    (gicp.py:5-35,116-167 in 2-D, k = 6): first pass's correspondences bit-exact against cKDTree, and
    10 fixed iterations of the fast path (rotated covariances, exact Newton inner solve, on the device)
    within 1e-6 of the oracle's loop with the same semantics (rotated covariances, exact inner solve)."""
    src, tgt, Tgt = S.segment_scene_2d(100_000)
    kw = dict(max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0)
    p = gicp.default_params(2, **kw)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    _, dbg = eng.iterate(np.eye(3), debug=True)
    idx, _ = O.correspondences(src, tgt, kw["max_distance_correspondence"], workers=WORKERS)
    assert np.array_equal(dbg["index"], idx)
    T, all_T, *_ = gicp.gicp(src, tgt, max_iterations=10, tolerance=0.0, mode="fast", inner="newton",
                             full_output=False, verbose=False, **kw)
    To, all_To, *_ = O.gicp(src, tgt, max_iterations=10, tolerance=0.0, inner="gn", source_cov="rotate",
                            fixed_iterations=True, **kw)
    assert len(all_T) == len(all_To) == 11
    for a, b in zip(all_T, all_To):
        th = np.arctan2(a[1, 0], a[0, 0]) - np.arctan2(b[1, 0], b[0, 0])
        assert abs(th) < 1e-6 and np.max(np.abs(a[:2, 2] - b[:2, 2])) < 1e-4, (th, a, b)   # px, box 1000


def test_2d_1m_fast_mode_vs_oracle(eng):
    """The 2-D bench size (BASELINE.md §3's segment scene at 1M/1M, k = 6): the first pass's 1M correspondence
    indices bit-exact against cKDTree, and 5 fixed iterations of the fast path within 1e-8 rad / 1e-6 px of
    the oracle's loop with the same semantics (rotated covariances, exact inner solve) at every iteration."""
    src, tgt, _ = S.segment_scene_2d(1_000_000)
    kw = dict(max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0)
    p = gicp.default_params(2, **kw)
    eng.set_target(tgt, p)
    eng.set_source(src, p)
    _, dbg = eng.iterate(np.eye(3), debug=True)
    idx, _ = O.correspondences(src, tgt, kw["max_distance_correspondence"], workers=WORKERS)
    assert np.array_equal(dbg["index"], idx)
    T, all_T, *_ = gicp.gicp(src, tgt, max_iterations=5, tolerance=0.0, mode="fast", inner="newton",
                             full_output=False, verbose=False, **kw)
    To, all_To, *_ = O.gicp(src, tgt, max_iterations=5, tolerance=0.0, inner="gn", source_cov="rotate",
                            fixed_iterations=True, workers=WORKERS, **kw)
    assert len(all_T) == len(all_To) == 6
    for a, b in zip(all_T, all_To):
        th = np.arctan2(a[1, 0], a[0, 0]) - np.arctan2(b[1, 0], b[0, 0])
        assert abs(th) < 1e-8 and np.max(np.abs(a[:2, 2] - b[:2, 2])) < 1e-6, (th, a, b)


def test_2d_default_above_faithful_limit_vs_oracle():
    """a 2-D call just above FAITHFUL_MAX_POINTS takes mode='fast' (rotated covariances,
    fmin_cg on the closed-form loss); its endpoint is within the parity tolerance (1e-4 rad, 1e-3 px)
    of the oracle's reference-semantics loop (covariances recomputed per iteration, gicp.py:120, and
    fmin_cg on the per-point loss, gicp.py:148-154)."""
    n = gicp.FAITHFUL_MAX_POINTS + 1000
    src, tgt, _ = S.segment_scene_2d(n)
    kw = dict(max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0)
    out = gicp.gicp(src, tgt, verbose=False, **kw)
    assert isinstance(out[6], gicp.RotatedCovariances), "default above the limit is the fast path"
    To, *_ = O.gicp(src, tgt, **kw)
    th = np.arctan2(out[0][1, 0], out[0][0, 0]) - np.arctan2(To[1, 0], To[0, 0])
    assert abs(th) < 1e-4 and np.max(np.abs(out[0][:2, 2] - To[:2, 2])) < 1e-3
