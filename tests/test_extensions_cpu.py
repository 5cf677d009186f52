"""CPU checks of the §8(f) extension rules: the oracle's covariance choices (presentation/main.typ:
446-455) and the PCL-style stopping test (presentation/main.typ:773-776), and the drop-in's host
restatement of that test (gicp.pcl_stop, the rule k_solve applies on the device)."""
import numpy as np
import pytest

from oracle import gicp_oracle as O


def _gicp():
    return pytest.importorskip("gicp")


def _rand_T(rng, d, ang, trans):
    T = np.eye(d + 1)
    if d == 3:
        w = rng.normal(size=3)
        w *= ang / np.linalg.norm(w)
        T[:3, :3] = O.so3_exp(w)
    else:
        T[:2, :2] = O.rot2(ang)
    T[:d, d] = rng.normal(size=d) * trans
    return T


@pytest.mark.parametrize("d", [2, 3])
def test_pcl_stop_host_equals_oracle(d):
    g = _gicp()
    rng = np.random.default_rng(0)
    kinds = [dict(transformation_epsilon=1e-6), dict(transformation_epsilon=1e-6, rotation_epsilon=0.9999),
             dict(euclidean_fitness_epsilon=1e-3), dict(mse_relative_epsilon=1e-2),
             dict(transformation_epsilon=1e-4, euclidean_fitness_epsilon=1e-5, mse_relative_epsilon=1e-3)]
    seen = set()
    for _ in range(400):
        Ta = _rand_T(rng, d, rng.uniform(0, 0.5), 1.0)
        inc = _rand_T(rng, d, 10 ** rng.uniform(-6, -1), 10 ** rng.uniform(-5, -1))
        Tb = inc @ Ta
        m0 = 10 ** rng.uniform(-3, 0)
        m1 = m0 * (1 + 10 ** rng.uniform(-5, -1) * rng.choice([-1, 1]))
        prev = np.inf if rng.random() < 0.1 else m0
        for kw in kinds:
            a = g.pcl_stop(Ta, Tb, m1, prev, **kw)
            b = O.pcl_stop(Ta, Tb, m1, prev, **kw)
            assert a == b
            seen.add(a)
    assert {"transform", "abs_mse", "rel_mse", None} <= seen


def test_pcl_stop_first_iteration_never_stops_on_mse():
    T = np.eye(4)
    T2 = T.copy()
    T2[0, 3] = 1.0
    assert O.pcl_stop(T, T2, 1.0, np.inf, euclidean_fitness_epsilon=1e9, mse_relative_epsilon=1e9) is None


def test_weights_models_3d():
    from gicp import synthetic as S
    src, tgt, _ = S.scene_pair_3d(3000)
    Ct, cnt = O.covariances(tgt, 1.0)
    idx, _ = O.correspondences(src, tgt, 0.5)
    Cs = np.zeros((len(src), 3, 3))
    ok = idx >= 0
    Wi = O.weights_model(Cs, Ct, idx, "point_to_point", cnt)
    assert np.array_equal(Wi[ok], np.broadcast_to(np.eye(3), (ok.sum(), 3, 3))) and not Wi[~ok].any()
    Wp = O.weights_model(Cs, Ct, idx, "point_to_plane", cnt)
    surf = ok & (cnt[np.maximum(idx, 0)] >= 3)
    # projector onto the target normal: symmetric, idempotent, trace 1; zero without a surface
    P = Wp[surf]
    np.testing.assert_allclose(np.einsum("nab,nbc->nac", P, P), P, atol=1e-12)
    np.testing.assert_allclose(np.trace(P, axis1=1, axis2=2), 1.0, atol=1e-12)
    # its normal is the direction of the smallest covariance eigenvalue (0.1 eps)
    Ctj = Ct[idx[surf]]
    np.testing.assert_allclose(np.einsum("nab,nbc->nac", Ctj, P), 10.0 * P, atol=1e-9)
    assert not Wp[ok & ~surf].any() and not Wp[~ok].any()
    Wg = O.weights_model(O.covariances(src, 1.0)[0], Ct, idx, "plane_to_plane")
    np.testing.assert_array_equal(Wg, O.weights(O.covariances(src, 1.0)[0], Ct, idx))


def test_oracle_methods_recover_ground_truth():
    from gicp import synthetic as S
    src, tgt, Tgt = S.scene_pair_3d(6000)
    for m in ("point_to_point", "point_to_plane"):
        T, *_ = O.gicp(src, tgt, max_iterations=40, tolerance=1e-10, max_distance_correspondence=0.5,
                       max_distance_nearest_neighbors=1.0, method=m)
        tol_r, tol_t = (3e-3, 5e-2) if m == "point_to_point" else (2e-3, 2e-2)   # ICP: sampling bias
        assert S.rotation_angle_error(T, Tgt) < tol_r and S.translation_error(T, Tgt) < tol_t, m


def test_oracle_pcl_transform_stop_applies_update():
    from gicp import synthetic as S
    src, tgt, _ = S.scene_pair_3d(4000)
    kw = dict(max_iterations=50, tolerance=0.0, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    out, rec = O.gicp(src, tgt, record=True, transformation_epsilon=1e-8, **kw)
    assert rec["stop_reason"] == "transform"
    k = rec["converged_at"]
    assert k < 49 and len(out[1]) == k + 2          # the stopping iteration's update is applied (PCL)
    assert np.array_equal(out[0], rec["iterations"][k]["T_new"])
