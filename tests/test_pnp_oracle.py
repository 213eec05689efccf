"""Pin the PnP oracle (oracle/pnp.py) -- CPU only.

The reference's PnP stage cannot run here (Ceres, cv2 and the cffi library
are absent), so the oracle is pinned by the reference's own
known-answer self-test (lib/utils/extend_utils/src/uncertainty_pnp.cpp:98-156:
random pose rt ~ U[0,1]^6, eight points ~ U[0,1]^3, fx = fy = 400,
px = py = 128, identity weights, start perturbed by U[0, 0.1] -> the pose is
recovered), by exact-data P3P recovery, and by scipy for the weights."""
import numpy as np
import scipy.linalg

from oracle import pnp as P

K_SELF = np.array([[400.0, 0, 128.0], [0, 400.0, 128.0], [0, 0, 1]])
# LINEMOD camera (lib/utils/base_utils.py:241-243)
K_LM = np.array([[572.4114, 0.0, 325.2611], [0.0, 573.57043, 242.04899], [0.0, 0.0, 1.0]])


def project(R, t, p3, K):
    X = p3 @ R.T + t
    return np.stack([K[0, 0] * X[:, 0] / X[:, 2] + K[0, 2], K[1, 1] * X[:, 1] / X[:, 2] + K[1, 2]], 1)


def test_known_answer_selftest_of_the_reference():
    """uncertainty_pnp.cpp:98-156 (z shifted by +2 so that every point is in
    front of the camera for every seed; the reference's single draw was)."""
    rng = np.random.default_rng(0)
    for _ in range(50):
        rt = rng.uniform(0, 1, 6)
        rt[5] += 2.0
        p3 = rng.uniform(0, 1, (8, 3))
        p2 = project(P.rodrigues_vec_to_mat(rt[:3]), rt[3:], p3, K_SELF)
        x0 = rt + rng.uniform(0, 0.1, 6)
        d = {}
        x = P.ceres_lm(x0, p2, p3, np.tile([1.0, 0.0, 1.0], (8, 1)), K_SELF, diag=d)
        np.testing.assert_allclose(x, rt, atol=1e-6)
        assert d["status"] in ("function", "parameter", "gradient") and d["iterations"] <= 50


def test_p3p_recovers_exact_pose():
    rng = np.random.default_rng(1)
    for _ in range(100):
        r = rng.normal(size=3)
        R = P.rodrigues_vec_to_mat(r)
        t = np.array([0.0, 0.0, 1.0]) + rng.uniform(-0.1, 0.1, 3)
        p3 = rng.uniform(-0.1, 0.1, (4, 3))
        p2 = project(R, t, p3, K_LM)
        ok, rv, tt = P.p3p_pose(p3, p2, K_LM)
        assert ok
        np.testing.assert_allclose(P.rodrigues_vec_to_mat(rv), R, atol=1e-5)
        np.testing.assert_allclose(tt, t, atol=1e-5)


def test_rodrigues_round_trip():
    rng = np.random.default_rng(2)
    for _ in range(200):
        r = rng.normal(size=3)
        r *= rng.uniform(0, np.pi * 0.999) / np.linalg.norm(r)
        np.testing.assert_allclose(P.rodrigues_mat_to_vec(P.rodrigues_vec_to_mat(r)), r, atol=1e-9)
    # theta = pi: either axis sign is the same rotation
    for r in ([np.pi, 0, 0], [0, 0, np.pi], [np.pi / np.sqrt(2), np.pi / np.sqrt(2), 0]):
        R = P.rodrigues_vec_to_mat(np.array(r))
        np.testing.assert_allclose(P.rodrigues_vec_to_mat(P.rodrigues_mat_to_vec(R)), R, atol=1e-7)   # acos near -1: ~sqrt(eps)


def test_weights_match_scipy_sqrtm():
    rng = np.random.default_rng(3)
    cov = []
    for _ in range(20):
        a = rng.normal(size=(2, 2))
        cov.append(a @ a.T + 1e-3 * np.eye(2))
    cov = np.array(cov)
    cov[3, 0, 0] = 1e-7           # below the 1e-6 gate -> zero weights
    cov[5, 1, 0] = np.nan         # NaN -> zero weights
    w = P.weights_from_cov(cov)
    for i in range(20):
        if i in (3, 5):
            assert np.all(w[i] == 0)
            continue
        ref = np.linalg.inv(scipy.linalg.sqrtm(cov[i]).real)
        np.testing.assert_allclose(w[i], [ref[0, 0], ref[0, 1], ref[1, 1]], rtol=1e-9)
    w2 = P.weights_v2(cov)
    for i in range(20):
        if cov[i, 0, 0] < 1e-5:
            assert np.all(w2[i] == 0)
        elif not np.isnan(cov[i]).any():
            np.testing.assert_allclose(w2[i, 0], 1.0 / np.linalg.eigvalsh(cov[i]).max(), rtol=1e-12)


def box_keypoints():
    """LINEMOD-style 9 keypoints: the 8 corners of a 10 cm box + its centre."""
    c = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], np.float64) * 0.05
    return np.concatenate([c, np.zeros((1, 3))], 0)


def noisy_case(seed, noise=1.0):
    rng = np.random.default_rng(seed)
    p3 = box_keypoints()
    R = P.rodrigues_vec_to_mat(rng.normal(size=3))
    t = np.array([rng.uniform(-0.1, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(0.6, 1.0)])
    p2 = project(R, t, p3, K_LM)
    cov = []
    for _ in range(9):
        a = rng.normal(size=(2, 2)) * noise
        cov.append(a @ a.T + 0.05 * np.eye(2))
    cov = np.array(cov)
    p2n = p2 + np.array([rng.multivariate_normal([0, 0], c) for c in cov])
    return p2n.astype(np.float32), cov.astype(np.float32), p3, R, t


def test_uncertainty_pnp_noisy_is_a_stationary_point_near_truth():
    for seed in range(10):
        p2, cov, p3, R, t = noisy_case(seed)
        w = P.weights_from_cov(cov)
        d = {}
        Rt = P.uncertainty_pnp(p2, w, p3, K_LM, diag=d)
        assert d["p3p_ok"]
        np.testing.assert_allclose(Rt[:, :3] @ Rt[:, :3].T, np.eye(3), atol=1e-12)
        assert np.linalg.norm(Rt[:, 3] - t) < 0.02
        # the least squares' gradient at the solution is ~0 relative to its scale
        x = np.concatenate([P.rodrigues_mat_to_vec(Rt[:, :3]), Rt[:, 3]])
        cost, r, J = P.evaluate(x, p2.astype(np.float64), p3, w, K_LM)
        assert np.abs(J.T @ r).max() <= 1e-3 * max(1.0, np.abs(J).max() * np.abs(r).max())


def test_four_points_is_the_p3p_pose():
    """pn == 4: the P3P pose is returned without refinement (extend_utils.py:90-94)."""
    _, _, p3, R, t = noisy_case(7)
    p2 = project(R, t, p3, K_LM)
    w = np.tile([1.0, 0.0, 1.0], (4, 1))
    Rt = P.uncertainty_pnp(p2[:4], w, p3[:4], K_LM)
    np.testing.assert_allclose(Rt[:, :3], R, atol=1e-6)
    np.testing.assert_allclose(Rt[:, 3], t, atol=1e-6)


def test_demo_cat_pose_from_the_references_evd():
    """Known answer from the reference's own data: its EVD-with-mean output on
    the demo cat (tests/golden/cat_evdm.npz, made by ransac_voting_gpu.py) with
    the demo's 3-D keypoints -> the demo's ground-truth pose (data/demo
    cat_pose.npy).  The first keypoint's covariance is below the 1e-6 gate
    (zero weight, evaluation_utils.py:171)."""
    from tests import golden_io as G
    g = G.load("cat_evdm")
    mean, cov = g["mean"][0], g["cov"][0]
    assert cov[0, 0, 0] < 1e-6
    d = {}
    Rt = P.uncertainty_pnp(mean, P.weights_from_cov(cov), g["points_3d"], K_LM, diag=d)
    assert d["p3p_ok"]
    np.testing.assert_allclose(Rt, g["pose"], atol=2e-5)
    np.testing.assert_allclose(P.uncertainty_pnp_v2(mean, cov, g["points_3d"], K_LM), g["pose"], atol=2e-5)
