"""Parity of the device uncertainty PnP (pv_uncertainty_pnp, through the C ABI)
with the CPU oracle (oracle/pnp.py: cv2 P3P + Ceres 2.0 LM restated).

Both sides are fp64; they differ only in summation order (J^T J column sums
vs BLAS) and in the quartic root finder (Ferrari + Newton vs numpy.roots +
Newton), so poses agree to ~1e-9 and the tests use 1e-7 (rotation entries,
metres).  Edge cases the reference has: zero weights (cov[0,0] < 1e-6 or
NaN, evaluation_utils.py:171), pn == 4 (P3P only, extend_utils.py:90-94),
the refine-only C entry (uncertainty_pnp.cpp:58-92)."""
import numpy as np
import pytest
import torch

from oracle import pnp as P
from tests.test_pnp_oracle import K_LM, K_SELF, box_keypoints, noisy_case, project

pytestmark = pytest.mark.gpu

TOL = 1e-7


@pytest.fixture(scope="module")
def eu():
    from pvnet_amd import extend_utils
    return extend_utils


def test_refine_matches_oracle_known_answer(device, eu):
    """uncertainty_pnp.cpp:98-156 on the device: the same start -> the same pose."""
    rng = np.random.default_rng(0)
    B = 32
    p3s, p2s, x0s, rts = [], [], [], []
    for _ in range(B):
        rt = rng.uniform(0, 1, 6)
        rt[5] += 2.0
        p3 = rng.uniform(0, 1, (8, 3))
        p2s.append(project(P.rodrigues_vec_to_mat(rt[:3]), rt[3:], p3, K_SELF))
        p3s.append(p3)
        x0s.append(rt + rng.uniform(0, 0.1, 6))
        rts.append(rt)
    w = np.tile([1.0, 0.0, 1.0], (B, 8, 1))
    # float32 image points on both sides (the device API takes the voting's f32 keypoints)
    p2 = np.array(p2s, np.float32)
    out = eu.uncertainty_pnp_batch(torch.from_numpy(p2).to(device), torch.from_numpy(w).to(device),
                                   np.array(p3s), K_SELF, mode="weights",
                                   init_rt=torch.from_numpy(np.array(x0s)).to(device)).cpu().numpy()
    for i in range(B):
        ref = P.ceres_lm(x0s[i], p2[i].astype(np.float64), p3s[i], w[i], K_SELF)
        np.testing.assert_allclose(out[i], ref, atol=TOL)
        np.testing.assert_allclose(out[i], rts[i], atol=1e-3)   # f32 image points: ~1e-5 px of noise


def _batch(seeds, pn=9):
    cases = [noisy_case(s) for s in seeds]
    p2 = np.stack([c[0] for c in cases])[:, :pn]
    cov = np.stack([c[1] for c in cases])[:, :pn]
    p3 = box_keypoints()[:pn]
    return p2, cov, p3, cases


@pytest.mark.parametrize("mode", ["cov", "cov_v2"])
def test_full_pnp_matches_oracle(mode, device, eu):
    p2, cov, p3, cases = _batch(range(64))
    cov[3, 2] = np.float32(1e-7) * np.eye(2, dtype=np.float32)     # gated -> zero weight
    cov[5, 4, 1, 0] = np.nan                                          # NaN -> zero weight (mode cov)
    if mode == "cov_v2":
        cov[5, 4, 1, 0] = 0.0
    diag = {}
    Rt = eu.uncertainty_pnp_batch(torch.from_numpy(p2).to(device), torch.from_numpy(cov).to(device), p3, K_LM,
                                  mode=mode, diag=diag).cpu().numpy()
    for i in range(len(cases)):
        d = {}
        if mode == "cov":
            ref = P.uncertainty_pnp(p2[i], P.weights_from_cov(cov[i]), p3, K_LM, diag=d)
        else:
            ref = P.uncertainty_pnp_v2(p2[i], cov[i], p3, K_LM, diag=d)
        np.testing.assert_allclose(diag["init_rt"][i].cpu().numpy(), d["init"], atol=1e-6, err_msg=f"init {i}")
        assert bool(diag["p3p_ok"][i]) == bool(d["p3p_ok"])
        # (no P3P solution: the reference's cv2 path has no pose to start from;
        # both sides then start from zero and may end non-finite alike)
        np.testing.assert_allclose(Rt[i], ref, atol=TOL, err_msg=f"image {i}", equal_nan=True)
    assert (diag["status"].cpu().numpy() > 0).all()
    assert diag["p3p_ok"].cpu().numpy().mean() > 0.9


def test_numpy_api_matches_batch_and_reference_signature(device, eu):
    p2, cov, p3, _ = _batch([11])
    w = P.weights_from_cov(cov[0])
    Rt = eu.uncertainty_pnp(p2[0], w, p3, K_LM)
    assert Rt.shape == (3, 4) and Rt.dtype == np.float64
    np.testing.assert_allclose(Rt, P.uncertainty_pnp(p2[0], w, p3, K_LM), atol=TOL)
    Rt2 = eu.uncertainty_pnp_v2(p2[0], cov[0], p3, K_LM)
    np.testing.assert_allclose(Rt2, P.uncertainty_pnp_v2(p2[0], cov[0], p3, K_LM), atol=TOL)


def test_four_points_p3p_only(device, eu):
    _, _, p3, R, t = noisy_case(7)
    p2 = project(R, t, p3, K_LM)[:4].astype(np.float32)
    w = np.tile([1.0, 0.0, 1.0], (4, 1))
    Rt = eu.uncertainty_pnp(p2, w, p3[:4], K_LM)
    np.testing.assert_allclose(Rt, P.uncertainty_pnp(p2, w, p3[:4], K_LM), atol=1e-6)
    np.testing.assert_allclose(Rt[:, :3], R, atol=1e-4)


def test_per_image_cameras_and_models(device, eu):
    """[b, pn, 3] model points and [b, 3, 3] cameras (YCB-style mixed objects)."""
    rng = np.random.default_rng(5)
    B = 16
    p2, cov, p3, _ = _batch(range(100, 100 + B))
    p3b = np.stack([p3 * rng.uniform(0.8, 1.2) for _ in range(B)])
    Kb = np.stack([K_LM * np.array([[rng.uniform(0.95, 1.05)] * 3, [rng.uniform(0.95, 1.05)] * 3, [1, 1, 1]])
                   for _ in range(B)])
    Rt = eu.uncertainty_pnp_batch(torch.from_numpy(p2).to(device), torch.from_numpy(cov).to(device), p3b, Kb,
                                  mode="cov").cpu().numpy()
    for i in range(B):
        ref = P.uncertainty_pnp(p2[i], P.weights_from_cov(cov[i]), p3b[i], Kb[i])
        np.testing.assert_allclose(Rt[i], ref, atol=TOL)


def test_pose_from_voting_end_to_end(device, eu):
    """EVD (mean, cov) of the HIP voting path -> device PnP, against the oracle
    PnP on the same (mean, cov)."""
    from pvnet_amd import ransac_voting_gpu as rvg
    from pvnet_amd import synth
    R = P.rodrigues_vec_to_mat(np.array([0.3, -0.5, 0.2]))
    t = np.array([0.0, 0.0, 0.8])
    kp = project(R, t, box_keypoints(), K_LM)
    f = synth.synthetic_field(21, keypoints=kp, center=(325.0, 242.0))
    seg = torch.from_numpy(f["seg"]).to(device)
    ver = torch.from_numpy(f["vertex"]).to(device)
    b, c, h, w = ver.shape
    vertex = ver.permute(0, 2, 3, 1).view(b, h, w, c // 2, 2)
    mask = seg.argmax(1)
    mean = rvg.ransac_voting_layer_v3(mask, vertex, 512)
    mean, cov = rvg.estimate_voting_distribution_with_mean(mask, vertex, mean)
    p3 = box_keypoints()
    Rt = eu.pose_from_voting(mean, cov, p3, K_LM).cpu().numpy()
    m, cv = mean.cpu().numpy()[0], cov.cpu().numpy()[0]
    ref = P.uncertainty_pnp(m, P.weights_from_cov(cv), p3, K_LM)
    np.testing.assert_allclose(Rt[0], ref, atol=1e-6)
    np.testing.assert_allclose(Rt[0, :, 3], t, atol=0.02)       # the pose behind the noisy field


def test_input_checks(device, eu):
    p2 = torch.zeros((2, 3, 2), device=device)
    with pytest.raises(RuntimeError, match="4 <= pn"):
        eu.uncertainty_pnp_batch(p2, torch.zeros((2, 3, 2, 2), device=device), np.zeros((3, 3)), K_LM)
    p2 = torch.zeros((2, 9, 2), device=device)
    with pytest.raises(RuntimeError, match="covariances"):
        eu.uncertainty_pnp_batch(p2, torch.zeros((2, 9, 3), device=device), box_keypoints(), K_LM)
    with pytest.raises(RuntimeError, match="init_rt needs"):
        eu.uncertainty_pnp_batch(p2, torch.zeros((2, 9, 2, 2), device=device), box_keypoints(), K_LM,
                                 init_rt=torch.zeros((2, 6), device=device))


def test_demo_cat_pose_from_the_references_evd(device, eu):
    """The reference's EVD output on the demo cat (golden) -> device PnP ->
    the demo's ground-truth pose; and the same from the device's own EVD
    with the golden idxs injected (v3 mean from the golden keypoints)."""
    from pvnet_amd import ransac_voting_gpu as rvg
    from tests import golden_io as G
    g = G.load("cat_evdm")
    mean = torch.from_numpy(g["mean"]).to(device)
    cov = torch.from_numpy(g["cov"]).to(device)
    Rt = eu.pose_from_voting(mean, cov, g["points_3d"], K_LM).cpu().numpy()[0]
    np.testing.assert_allclose(Rt, P.uncertainty_pnp(g["mean"][0], P.weights_from_cov(g["cov"][0]), g["points_3d"],
                                                     K_LM), atol=TOL)
    np.testing.assert_allclose(Rt, g["pose"], atol=2e-5)
    mask, vertex, _ = G.cat_inputs(g)
    idxs = g["idxs"][0].reshape(1, -1, 9, 2)
    m2, c2 = rvg.estimate_voting_distribution_with_mean(torch.from_numpy(mask).to(device),
                                                        torch.from_numpy(vertex).to(device), mean, _idxs=idxs)
    Rt2 = eu.pose_from_voting(m2, c2, g["points_3d"], K_LM).cpu().numpy()[0]
    np.testing.assert_allclose(Rt2, g["pose"], atol=2e-5)


def test_ycb21_pose_from_voting(device, eu):
    """configs[4] on the device: 21 keypoints, YCB camera, v3 -> EVD with
    mean -> uncertainty PnP, with the reference's idxs injected.  The
    reference's own covariances (golden) give the same pose through the
    device PnP as through the oracle PnP, and the device's voting gives the
    pose the field was generated from."""
    from pvnet_amd import ransac_voting_gpu as rvg
    from tests import golden_io as G
    g = G.load("ycb21_cases")
    K, p3 = g["camera"], g["points_3d"]
    mean = torch.from_numpy(g["v3_keypoints"]).to(device)
    Rt = eu.pose_from_voting(mean, torch.from_numpy(g["evdm_cov"]).to(device), p3, K).cpu().numpy()[0]
    ref = P.uncertainty_pnp(g["v3_keypoints"][0], P.weights_from_cov(g["evdm_cov"][0]), p3, K)
    np.testing.assert_allclose(Rt, ref, atol=1e-6)
    # noisy field (0.05 rad, 20 % outliers): 0.2 mrad / 6 mm (z at 1 m) from the generating pose
    np.testing.assert_allclose(Rt, g["pose"], atol=1e-2)
    mask, vertex, _ = G.ycb_inputs(g)
    m, v = torch.from_numpy(mask).to(device), torch.from_numpy(vertex).to(device)
    kp = rvg.ransac_voting_layer_v3(m, v, 512, _idxs=g["v3_idxs"].astype(np.int32))
    _, cov = rvg.estimate_voting_distribution_with_mean(m, v, kp, _idxs=g["evdm_idxs"].astype(np.int32)
                                                        .reshape(1, -1, 21, 2))
    # device keypoints within 1e-2 px and covariances within 1e-4 (of scale) of the reference's
    np.testing.assert_allclose(kp.cpu().numpy(), g["v3_keypoints"], atol=1e-2, rtol=0)
    np.testing.assert_allclose(cov.cpu().numpy(), g["evdm_cov"], rtol=1e-4, atol=1e-4 * np.abs(g["evdm_cov"]).max())
    Rt2 = eu.pose_from_voting(kp, cov, p3, K).cpu().numpy()[0]
    np.testing.assert_allclose(Rt2, ref, atol=1e-4)


def test_float64_image_points_keep_full_precision(device, eu):
    """The single-image drop-ins take float64 points like the reference's cffi
    path (extend_utils.py:80): sub-f32 detail reaches the LM, the batched
    form takes float64 tensors the same way, and float32 still works."""
    p2, cov, p3, _ = _batch([13])
    x = p2[0].astype(np.float64) + np.random.default_rng(1).uniform(-3e-5, 3e-5, p2[0].shape)
    w = P.weights_from_cov(cov[0])
    Rt = eu.uncertainty_pnp(x, w, p3, K_LM)
    np.testing.assert_allclose(Rt, P.uncertainty_pnp(x, w, p3, K_LM), atol=TOL)
    Rb = eu.uncertainty_pnp_batch(torch.from_numpy(x[None]).to(device), torch.from_numpy(w[None]).to(device), p3, K_LM,
                                  mode="weights").cpu().numpy()[0]
    np.testing.assert_allclose(Rb, Rt, atol=1e-12)
    R32 = eu.uncertainty_pnp_batch(torch.from_numpy(x[None].astype(np.float32)).to(device),
                                   torch.from_numpy(w[None]).to(device), p3, K_LM, mode="weights").cpu().numpy()[0]
    np.testing.assert_allclose(R32, P.uncertainty_pnp(x.astype(np.float32), w, p3, K_LM), atol=TOL)
