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
    np.testing.assert_allclose(two[0], one[0], atol=1e-6)


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
