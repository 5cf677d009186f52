"""The Python wrapper on a NumPy fake of the device entry points (tests/fake_device.py, SURVEY.md §4
last row): gicp()'s 7-tuple assembly on the device-loop trace, devices=, the host loop's shard sums,
and Odometry's staged ring, exercised in a container without a GPU.  The fake computes with the oracle;
the pose solve is the real library's host entry point."""
import numpy as np
import pytest

from gicp import synthetic as S
from oracle import gicp_oracle as O

gicp = pytest.importorskip("gicp")
from fake_device import install  # noqa: E402

P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)


@pytest.fixture
def fake(monkeypatch):
    return install(monkeypatch, ndev=2)


@pytest.fixture(scope="module")
def scene():
    return S.scene_pair_3d(3000)


def test_dropin_3d_device_loop_vs_oracle(fake, scene, capsys):
    """gicp() 3-D takes the device loop (gicp_align_trace): the pose and every all_transformations entry
    equal the oracle's loop with the same semantics; the top-5 rows are the transformed source points of
    the 5 largest det(W); one rotated covariance set per executed iteration; the reference's print."""
    src, tgt, _ = scene
    out = gicp.gicp(src, tgt, max_iterations=40, tolerance=1e-6, **P3)
    ref, rec = O.gicp(src, tgt, max_iterations=40, tolerance=1e-6, record=True, **P3)
    printed = capsys.readouterr().out.strip()
    assert rec["converged_at"] >= 0, "the scene converges within 40 iterations"
    assert printed == f"Converged at iteration {rec['converged_at']}"
    T, all_T, init_cov, tgt_cov, hw_s, hw_t, all_cov = out
    assert len(all_T) == len(ref[1])
    for a, b in zip(all_T, ref[1]):   # exact inner solves both (statistics Newton vs per-point Gauss-Newton)
        np.testing.assert_allclose(a, b, atol=2e-6)
    assert len(hw_s) == len(ref[4]) and len(all_cov) == len(ref[6])
    for k in range(len(hw_s)):
        W = rec["iterations"][k]["W"]
        det = np.where(rec["iterations"][k]["idx"] >= 0, np.linalg.det(W), 0.0)
        top = np.lexsort((np.arange(len(det)), det))[-5:]
        np.testing.assert_allclose(hw_s[k], O.apply_transformation(src[top], all_T[k]), atol=1e-9)
    np.testing.assert_allclose(all_cov[-1], ref[6][-1], atol=1e-3)   # rotated by poses within 2e-6


def test_devices_two_equal_one(fake, scene):
    """devices=[0, 1]: two engines, shards 0 and 1, the statistics summed in device order through the
    host hook every iteration -- the pose within 1e-9 of one device, the merged top rows equal."""
    src, tgt, _ = scene
    kw = dict(max_iterations=8, tolerance=0.0, verbose=False, **P3)
    one = gicp.gicp(src, tgt, devices=[0], **kw)
    two = gicp.gicp(src, tgt, devices=[0, 1], **kw)
    np.testing.assert_allclose(two[0], one[0], atol=1e-9)
    assert len(two[4]) == len(one[4])
    for a, b in zip(two[4], one[4]):
        np.testing.assert_allclose(a, b, atol=1e-9)
    for a, b in zip(two[5], one[5]):
        np.testing.assert_array_equal(a, b)


def test_devices_refused(fake, scene):
    src, tgt, _ = scene
    with pytest.raises(ValueError, match="more than once"):
        gicp.gicp(src, tgt, devices=[1, 1], verbose=False, **P3)
    with pytest.raises(ValueError, match="no such GPU"):
        gicp.gicp(src, tgt, devices=[0, 2], verbose=False, **P3)


def test_2d_fast_cg_two_devices(fake):
    """2-D fast mode with the fmin_cg inner solve (host loop): shard statistics summed on the host."""
    src, tgt, _ = S.segment_scene_2d(6000)
    kw = dict(max_iterations=5, tolerance=0.0, verbose=False, max_distance_correspondence=20.0,
              max_distance_nearest_neighbors=25.0)
    one = gicp.gicp(src, tgt, devices=[0], **kw)
    two = gicp.gicp(src, tgt, devices=[0, 1], **kw)
    assert isinstance(one[6], gicp.RotatedCovariances)
    # fmin_cg stops inexactly (|grad|_inf <= gtol = 1e-5, gicp.py:152): statistics summed over two shards
    # round differently from one device's, so the two stopping points differ by ~gtol / curvature
    np.testing.assert_allclose(two[0], one[0], atol=1e-5)


def test_odometry_ring_depths_agree(fake):
    """Odometry.run with builds one or two scans ahead equals building each scan when needed."""
    from gicp.odometry import Odometry
    frames = [f for f, _ in S.lidar_stream(5, beams=8, azimuths=200)]
    out = []
    for depth in (0, 1, 2):
        odo = Odometry(3, params=gicp.default_params(3, max_iterations=10, tolerance=1e-9, **P3))
        Ts = [odo.step(f)[0] for f in frames] if depth == 0 else [T for T, _ in odo.run(frames, depth=depth)]
        out.append(Ts)
        assert not odo._staged
    for Ts in out[1:]:
        for a, b in zip(out[0][1:], Ts[1:]):
            np.testing.assert_array_equal(a, b)


def test_commit_without_stage_is_an_error(fake):
    from gicp import _lib
    eng = gicp.Engine(0)
    with pytest.raises(_lib.GicpError):
        eng.commit_target()


def test_devices_hook_reports_ranks_and_restores_callers_hook(fake, scene):
    """gicp(devices=[0, 1]) installs its thread-barrier hook with (nranks, rank) = (2, r), so comm_ranks
    reports the job while it runs, and puts back the hook a caller had on the cached engines after."""
    src, tgt, _ = scene
    kw = dict(max_iterations=3, tolerance=0.0, verbose=False, **P3)
    eng0 = gicp._engine(0)
    mine = lambda buf: buf   # noqa: E731 -- an identity hook of the caller's
    eng0.set_allreduce(mine, nranks=1, rank=0)
    seen = {}
    real_align = gicp.Engine.align

    def spy(self, *a, **k):
        seen[self.device] = self.comm_ranks()
        return real_align(self, *a, **k)

    import unittest.mock as um
    with um.patch.object(gicp.Engine, "align", spy):
        gicp.gicp(src, tgt, devices=[0, 1], **kw)
    assert seen == {0: (2, 0, "hook"), 1: (2, 1, "hook")}
    assert eng0._hook_fn[0] is mine and eng0.comm_ranks() == (1, 0, "hook")
    assert gicp._engine(1).comm_ranks() == (1, 0, "none")


def test_odometry_failed_staged_build_then_retry(fake):
    """A staged build that fails: the step raises, its ring slot is consumed on both sides (the wrapper's
    list stays in step with the library's), and retrying the same scan registers it correctly (the
    synchronous path) instead of promoting the next slot's build."""
    from gicp.odometry import Odometry
    frames = [f for f, _ in S.lidar_stream(4, beams=8, azimuths=200)]
    params = gicp.default_params(3, max_iterations=10, tolerance=1e-9, **P3)
    ref = Odometry(3, params=params)
    Tref = [ref.step(f)[0] for f in frames]
    odo = Odometry(3, params=params)
    odo.step(frames[0], next_scans=frames[1:3])
    assert odo._staged == [frames[1], frames[2]] or [id(x) for x in odo._staged] == [id(frames[1]), id(frames[2])]
    fake._c(odo.eng._ctx).staged[0] = None          # frames[1]'s build fails
    with pytest.raises(ValueError, match="injected"):
        odo.step(frames[1], next_scans=frames[2:4])
    assert len(odo._staged) == 1 and odo._staged[0] is frames[2]
    T1, _ = odo.step(frames[1], next_scans=frames[2:4])   # the retry: built synchronously
    np.testing.assert_array_equal(T1, Tref[1])
    T2, _ = odo.step(frames[2])
    np.testing.assert_array_equal(T2, Tref[2])


def test_odometry_restages_whole_lookahead_on_mismatch(fake):
    """When the coming scans differ from what is staged, every staged build is dropped and the whole
    look-ahead is staged again (a valid head is not lost); a staged list longer than the look-ahead with
    a matching prefix is kept."""
    from gicp.odometry import Odometry
    frames = [f for f, _ in S.lidar_stream(5, beams=8, azimuths=200)]
    odo = Odometry(3, params=gicp.default_params(3, max_iterations=5, tolerance=1e-9, **P3))
    odo.step(frames[0], next_scans=[frames[1], frames[2]])
    odo.step(frames[1], next_scans=[frames[2], frames[4]])     # head frames[2] still staged: frames[4] added
    assert [x is y for x, y in zip(odo._staged, [frames[2], frames[4]])] == [True, True]
    odo.step(frames[2], next_scans=[frames[3], frames[4]])     # staged [4] != coming [3, 4]: restage both
    assert len(odo._staged) == 2 and odo._staged[0] is frames[3] and odo._staged[1] is frames[4]
    assert len(fake._c(odo.eng._ctx).staged) == 2
    odo.step(frames[3], next_scans=[])                        # shorter look-ahead: the staged [4] is kept
    assert len(odo._staged) == 1 and odo._staged[0] is frames[4]
    odo.step(frames[4])
    assert not odo._staged
