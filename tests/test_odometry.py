"""C5 odometry stream: pose composition on the CPU, the device stream
against the oracle and the generating poses on the GPU."""
import math

import numpy as np
import pytest

from gicp import synthetic as S
from gicp.odometry import compose


def _planar(x, y, yaw, d=2):
    P = np.eye(d + 1)
    P[0, 0], P[0, 1], P[1, 0], P[1, 1] = math.cos(yaw), -math.sin(yaw), math.sin(yaw), math.cos(yaw)
    P[0, d], P[1, d] = x, y
    return P


def test_compose_se3_recovers_trajectory():
    poses = S.lidar_trajectory(20)
    pose = poses[0].copy()
    for k in range(1, 20):
        T = np.linalg.inv(poses[k]) @ poses[k - 1]          # p_cur = T p_prev
        pose, _ = compose(pose, T, "se3")
        np.testing.assert_allclose(pose, poses[k], atol=1e-9)


def test_compose_reference_formula():
    """robot-visualization.py:257-265 literally: delta = -T[:2, 2], dyaw = -atan2(T10, T00), the
    delta rotated by the previous yaw."""
    rng = np.random.default_rng(3)
    state = (0.0, 0.0, 0.0)
    x, y, yaw = state
    for _ in range(10):
        T = _planar(*rng.normal(0, [2.0, 2.0, 0.05]))
        P, state = compose(np.eye(3), T, "reference", state)
        dx, dy, dyaw = -T[0, 2], -T[1, 2], -math.atan2(T[1, 0], T[0, 0])
        x, y, yaw = x + dx * math.cos(yaw) - dy * math.sin(yaw), y + dx * math.sin(yaw) + dy * math.cos(yaw), yaw + dyaw
        np.testing.assert_allclose(state, (x, y, yaw), atol=1e-12)
        np.testing.assert_allclose(P, _planar(x, y, yaw), atol=1e-12)


def _bare_odometry(composition, dim=2):
    """An Odometry without a device context: pose bookkeeping (_integrate / pose / poses) never calls it."""
    from gicp.odometry import Odometry
    o = Odometry.__new__(Odometry)
    o.dim, o.composition, o._staged = dim, composition, []
    o.reset()
    return o


@pytest.mark.parametrize("composition", ["se3", "reference"])
def test_pose_setter_continues_either_composition(composition):
    """setting `pose` replaces the latest pose and the reference formula's planar state, so the
    next registration composes from it under either composition."""
    o = _bare_odometry(composition)
    start = _planar(1.0, -2.0, 0.3)
    o.pose = start
    np.testing.assert_allclose(o.poses[-1], start)
    np.testing.assert_allclose(o.yaw_xy, (1.0, -2.0, 0.3), atol=1e-15)
    T = _planar(0.2, 0.1, 0.05)
    o._integrate(T)
    want, _ = compose(start, T, composition, (1.0, -2.0, 0.3))
    np.testing.assert_allclose(o.pose, want, atol=1e-12)
    assert len(o.poses) == 2
    o.poses = [np.eye(3)]
    assert len(o.poses) == 1
    o.yaw_xy = (0.5, 0.5, 0.0)
    assert o.yaw_xy == (0.5, 0.5, 0.0)


def test_lidar_scan_hits_and_noise():
    scene = S.lidar_scene()
    pose = S.lidar_trajectory(1)[0]
    dirs = S.lidar_dirs(8, 90)
    pts = S.lidar_scan(scene, pose, dirs, np.random.default_rng(0), noise=0.0)
    assert len(pts) == len(dirs)                           # closed room: every ray hits
    # noiseless hits lie on the scene: the world point is on some rectangle plane or sphere
    w = pts @ pose[:3, :3].T + pose[:3, 3]
    d_best = np.full(len(w), np.inf)
    for p0, e1, e2 in scene.rects:
        n = np.cross(e1, e2)
        n /= np.linalg.norm(n)
        d_best = np.minimum(d_best, np.abs((w - p0) @ n))
    for cx, cy, cz, r in scene.spheres:
        d_best = np.minimum(d_best, np.abs(np.linalg.norm(w - [cx, cy, cz], axis=1) - r))
    assert np.max(d_best) < 1e-9


def test_trajectory_follows_the_c5_spec():
    """~0.5 m and ~0.5 deg of yaw per frame (+-10 % jitter)."""
    P = S.lidar_trajectory(200)
    for k in range(1, 200):
        d = np.linalg.inv(P[k - 1]) @ P[k]
        assert 0.44 < np.linalg.norm(d[:3, 3]) < 0.56
        assert math.radians(0.44) < S.rotation_angle_error(d, np.eye(4)) < math.radians(0.56)


@pytest.mark.gpu
def test_staged_stream_equals_synchronous_stream():
    """The double-buffered stream (next scan built on a second stream during the registration,
    gicp_stage_target / gicp_commit_target) gives bit-identical registrations to building each scan
    when it is needed, on the C5 trajectory (0.5 m / 0.5 deg frames, constant-velocity start)."""
    import gicp
    from gicp.odometry import Odometry
    kw = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    frames = [f for f, _ in S.lidar_stream(6, beams=32, azimuths=900)]
    out = {}
    for mode in ("sync", "staged1", "staged2"):
        odo = Odometry(3, params=gicp.default_params(3, max_iterations=30, tolerance=1e-9, **kw))
        if mode == "sync":
            Ts = [odo.step(f)[0] for f in frames]
        else:   # builds started one or two registrations ahead (GICP_MAX_STAGED pending)
            Ts = [T for T, _ in odo.run(frames, depth=int(mode[-1]))]
        out[mode] = (Ts, odo.pose.copy())
        odo.eng.close()
    for mode in ("staged1", "staged2"):
        assert len(out[mode][0]) == len(frames)
        for a, b in zip(out["sync"][0][1:], out[mode][0][1:]):
            assert np.array_equal(a, b)
        assert np.array_equal(out["sync"][1], out[mode][1])


@pytest.mark.gpu
def test_odometry_stream_vs_oracle_and_truth():
    from oracle import gicp_oracle as O
    from gicp.odometry import Odometry
    kw = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    frames = list(S.lidar_stream(4, beams=16, azimuths=600, step=0.15, along_path=True))
    import gicp
    odo = Odometry(3, params=gicp.default_params(3, max_iterations=40, tolerance=1e-10, **kw), init="identity")
    pose_oracle = np.eye(4)
    for k, (scan, pose) in enumerate(frames):
        T, res = odo.step(scan)
        if T is None:
            continue
        prev = frames[k - 1][0]
        To, *_ = O.gicp(prev, scan, max_iterations=40, tolerance=1e-10, **kw)
        from golden_util import pose_err
        a, t = pose_err(T, To)
        assert a < 1e-6 and t < 1e-5, (k, a, t)              # same engine semantics as the oracle
        pose_oracle = pose_oracle @ np.linalg.inv(To)
        # against the generating motion (0.15 m, 0.6 deg): the reference's covariance model (in-plane
        # to normal variance 10:1) under-registers the sliding direction of ring-pattern
        # scans; both engines agree on that (above), so this is a sanity bound only
        Ttrue = np.linalg.inv(pose) @ frames[k - 1][1]
        assert S.rotation_angle_error(T, Ttrue) < 2e-3 and S.translation_error(T, Ttrue) < 0.1
    np.testing.assert_allclose(odo.pose, pose_oracle, atol=1e-5)


@pytest.mark.gpu
def test_full_size_stream_per_frame_vs_oracle():
    """VERDICT r02 missing 4: eleven full C5 frames (64 x 1563 rays, ~100k points each), streamed with
    the staged builds and constant-velocity starts (robot-visualization.py:239-265); every frame's
    registration within 1e-6 rad / 1e-5 m of the oracle's from the same start pose."""
    import gicp
    from oracle import gicp_oracle as O
    from gicp.odometry import Odometry
    from golden_util import pose_err
    kw = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    frames = [f for f, _ in S.lidar_stream(11)]
    assert min(len(f) for f in frames) > 80_000
    odo = Odometry(3, params=gicp.default_params(3, max_iterations=30, tolerance=1e-9, **kw))
    T_prev = None
    checked = 0
    for k, (T, res) in enumerate(odo.run(frames)):
        if T is None:
            continue
        To, *_ = O.gicp(frames[k - 1], frames[k], max_iterations=30, tolerance=1e-9, T0=T_prev, **kw)
        a, t = pose_err(T, To)
        assert a < 1e-6 and t < 1e-5, (k, a, t)
        T_prev = T
        checked += 1
    odo.eng.close()
    assert checked == 10


@pytest.mark.gpu
def test_stage_ring_limits_and_order():
    """gicp_stage_target keeps up to GICP_MAX_STAGED builds pending and commits them in staging order;
    one more is refused (GICP_E_STATE), a commit with none pending too, cancel drops them all."""
    import gicp
    from gicp import _lib
    kw = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    f = [s for s, _ in S.lidar_stream(5, beams=16, azimuths=400)]
    p = gicp.default_params(3, **kw)
    eng = gicp.Engine(0)
    try:
        eng.set_target(f[0], p)
        eng.stage_target(f[1], p)
        eng.stage_target(f[2], p)
        with pytest.raises(_lib.GicpError):
            eng.stage_target(f[3], p)
        eng.commit_target()
        assert eng.n_tgt == len(f[1]) and eng.n_src == len(f[0])
        eng.commit_target()
        assert eng.n_tgt == len(f[2]) and eng.n_src == len(f[1])
        with pytest.raises(_lib.GicpError):
            eng.commit_target()
        eng.stage_target(f[3], p)
        eng.stage_target(f[4], p)
        eng.cancel_stage()
        with pytest.raises(_lib.GicpError):
            eng.commit_target()
        T, res = eng.align(None, gicp.default_params(3, max_iterations=5, **kw))
        assert np.all(np.isfinite(T))
    finally:
        eng.close()


@pytest.mark.gpu
def test_staged_scan_buffer_may_be_refilled_at_once():
    """gicp_stage_target copies the caller's scan before it returns, so a sensor
    buffer refilled right after staging still registers the scan it held -- bit-identical to building
    that scan synchronously."""
    import gicp
    kw = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    f = [s for s, _ in S.lidar_stream(2)]
    p = gicp.default_params(3, max_iterations=20, tolerance=1e-9, **kw)
    a, b = gicp.Engine(0), gicp.Engine(0)
    try:
        a.set_target(f[0], p)
        buf = np.ascontiguousarray(f[1].copy())
        a.stage_target(buf, p)
        buf[:] = buf[::-1] + 7.0            # the sensor overwrites its buffer at once
        a.commit_target()
        Ta, ra = a.align(None, p)
        b.set_target(f[0], p)
        b.target_to_source()
        b.set_target(f[1], p)
        Tb, rb = b.align(None, p)
    finally:
        a.close()
        b.close()
    assert np.array_equal(Ta, Tb) and ra["iterations"] == rb["iterations"]


@pytest.mark.gpu
def test_borrowed_staging_equals_copied_staging():
    """GICP_STAGE_BORROW (no copy: the build reads the caller's buffer in place, the caller leaves it alone
    until the commit) registers exactly what the copying stage does, through a whole staged stream; the
    persistent per-slot build threads serve both."""
    from gicp.odometry import Odometry
    kw = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    scans = [s for s, _ in S.lidar_stream(6)]
    out = {}
    for borrow in (False, True):
        import gicp
        odo = Odometry(3, params=gicp.default_params(3, max_iterations=30, tolerance=1e-9, **kw), borrow=borrow)
        try:
            out[borrow] = [(T, r["iterations"]) for T, r in odo.run(scans) if T is not None]
        finally:
            odo.eng.close()
    assert len(out[True]) == len(out[False]) == 5
    for (Ta, ia), (Tb, ib) in zip(out[False], out[True]):
        assert np.array_equal(Ta, Tb) and ia == ib
