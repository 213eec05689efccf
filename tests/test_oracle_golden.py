"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.npz,
made by tests/golden/make_golden.py from ransac_voting_gpu.py).

Bit-exact: hypotheses, per-(h,v) inlier counts, winner indices, refine inlier
counts, masks.  Tolerance: keypoints (fp32 least squares whose summation order
differs between torch and numpy) and covariances (fp32 matmul order)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_io as G

KP_TOL = 1e-2      # px: fp32 LS sums (torch order vs correctly rounded); north star allows 0.5 px
COV_RTOL = 1e-4    # relative, per BASELINE.json


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def check_v3(mask, vertex, g, prefix="", hn=None, keep=None, **kw):
    idxs = list(g[prefix + "idxs"])
    fg = [int(O.fg_mask_v3(m).sum()) for m in mask]
    voted = [i for i, n in enumerate(fg) if n >= kw.get("min_num", 100)]
    idx_full = [None] * len(mask)
    for k, i in enumerate(voted):
        idx_full[i] = idxs[k]
    diag = []
    kp = O.ransac_voting_layer_v3(mask, vertex, hn or idxs[0].shape[0], idxs=idx_full, keep=keep, diag=diag, **kw)
    dv = [d for d in diag if not d.get("skipped")]
    assert len(dv) == len(voted)
    for k, d in enumerate(dv):
        np.testing.assert_array_equal(bits(d["hyp"]), bits(g[prefix + "hyp"][k]))
        np.testing.assert_array_equal(d["counts"], g[prefix + "counts"][k])
        ref_inl = np.zeros(d["hyp"].shape[1], np.int64)
        inl = np.zeros((1, d["hyp"].shape[1], d["tn"]), np.uint8)
        O.voting_for_hypothesis(d["direct"], d["coords"], d["win_pts"][None], inl, kw.get("inlier_thresh", 0.99))
        ref_inl[:] = inl[0].sum(1)
        np.testing.assert_array_equal(ref_inl, g[prefix + "refine_counts"][k])
    np.testing.assert_allclose(kp, g[prefix + "keypoints"], atol=KP_TOL, rtol=0)
    return kp, diag


def test_cat_v3_512_known_answer():
    g = G.load("cat_v3_512")
    mask, vertex, _ = G.cat_inputs(g)
    kp, diag = check_v3(mask, vertex, g)
    # the ground-truth field's keypoints are recovered (1.8e-4 px)
    assert np.abs(kp[0] - g["points_2d"]).max() < 1e-3
    assert diag[0]["iters"] == int(g["iters"])


def test_cat_v3_128_downsampled():
    g = G.load("cat_v3_128_maxnum100")
    mask, vertex, _ = G.cat_inputs(g)
    keep = np.unpackbits(g["keep_bits"][0])[: 480 * 640].reshape(1, 480, 640).astype(bool)
    check_v3(mask, vertex, g, keep=keep, max_num=100)


@pytest.mark.parametrize("hn", [512, 128])
def test_synth_v3(hn):
    g = G.load(f"synth_v3_{hn}")
    mask, vertex, _ = G.synth_inputs(g)
    assert int(mask.sum()) == 29861
    _, diag = check_v3(mask, vertex, g)
    assert diag[0]["iters"] == int(g["iters"])


@pytest.mark.parametrize("case", ["cat_evdm", "synth_evdm"])
def test_evd_with_mean(case):
    g = G.load(case)
    mask, vertex = (G.cat_inputs(g) if case.startswith("cat") else G.synth_inputs(g))[:2]
    _, cov = O.estimate_voting_distribution_with_mean(mask, vertex, g["mean"], idxs=[list(g["idxs"][0])])
    np.testing.assert_allclose(cov, g["cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["cov"]).max())


def test_evd_topk_all():
    g = G.load("synth_evd_top4096")
    mask, vertex, _ = G.synth_inputs(g)
    mu, cov = O.estimate_voting_distribution(mask, vertex, topk=4096, idxs=[list(g["idxs"][0])])
    np.testing.assert_allclose(mu, g["mean"], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(cov, g["cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["cov"]).max())


def test_evd_topk128_tie_invariants():
    """topk(sorted=False) leaves ties at the k-th value unspecified (RV:320):
    compare only what does not depend on which tied hypothesis was kept."""
    g = G.load("synth_evd_top128")
    mask, vertex, _ = G.synth_inputs(g)
    mu, cov = O.estimate_voting_distribution(mask, vertex, topk=128, idxs=[list(g["idxs"][0])])
    # the selected hypotheses all sit near the keypoint: means agree to well under a pixel
    np.testing.assert_allclose(mu, g["mean"], atol=0.05)
    np.testing.assert_allclose(cov, g["cov"], rtol=0.5, atol=0.05)


def test_edge_batch_mixed():
    g = G.load("edge_cases")
    check_v3(g["a_mask"], g["a_vertex"], g, prefix="a_")
    _, cov = O.estimate_voting_distribution_with_mean(
        g["a_mask"], g["a_vertex"], g["a_keypoints"], round_hyp_num=32, min_hyp_num=100,
        idxs=[list(g["a_evdm_idxs"][0:4]), list(g["a_evdm_idxs"][4:8]), list(g["a_evdm_idxs"][8:12])])
    np.testing.assert_allclose(cov, g["a_evdm_cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["a_evdm_cov"]).max())


def test_edge_singular_identity_fallback():
    g = G.load("edge_cases")
    kp, diag = check_v3(g["b_mask"], g["b_vertex"], g, prefix="b_")
    assert diag[0]["iters"] == int(g["b_iters"]) == 101
    # identity fallback: keypoints are ATb, not the LS solution
    np.testing.assert_allclose(kp[0], diag[0]["ATb"], rtol=1e-6)


def test_edge_forced_pairs():
    g = G.load("edge_cases")
    kp, diag = check_v3(g["c_mask"], g["c_vertex"], g, prefix="c_")
    hyp = diag[0]["hyp"]
    assert tuple(hyp[0, 0]) == (30.0, 20.0)          # exactly on a pixel centre
    assert tuple(hyp[1, 0]) == (0.0, 0.0)            # t0 == t1
    assert tuple(hyp[3, 0]) == (0.0, 0.0)            # zero direction
    np.testing.assert_array_equal(hyp[4], hyp[5])


def test_edge_downsample_and_jitter():
    g = G.load("edge_cases")
    check_v3(g["d_mask"], g["d_vertex"], g, prefix="d_", keep=g["d_keep"], max_num=300)
    check_v3(g["e_mask"], g["e_vertex"], g, prefix="e_", inlier_thresh=0.999)


def test_vp_kernels():
    g = G.load("vp_kernels")
    hyp = O.generate_hypothesis_vanishing_point(g["direct"], g["coords"], g["idxs"])
    np.testing.assert_array_equal(bits(hyp), bits(g["hyp"]))
    inl = np.zeros(g["inliers"].shape, np.uint8)
    O.voting_for_hypothesis_vanishing_point(g["direct"], g["coords"], hyp, inl, 0.99)
    np.testing.assert_array_equal(inl, g["inliers"])


def test_b_inv_semantics():
    A = np.array([[[2, 1], [1, 3]], [[4, 0], [0, 5]]], np.float32)
    np.testing.assert_allclose(O.b_inv(A), np.linalg.inv(A), rtol=1e-6)
    A[1] = 0                                          # one singular -> identity for all (RV:514-517)
    np.testing.assert_array_equal(O.b_inv(A), np.broadcast_to(np.eye(2, dtype=np.float32), A.shape))


def test_v5_matches_reference_golden():
    """ransac_voting_layer_v5 (RV:769-864, called as TRAIN:123): keypoints and
    the 0.999 confidence, with the reference's idxs and downsampling keep-mask."""
    g = G.load("v5_cases")
    mask, vertex = G.cat_inputs(g)[:2]
    keep = np.unpackbits(g["cat_keep_bits"])[: 480 * 640].reshape(1, 480, 640).astype(bool)
    dg = []
    kp, conf = O.ransac_voting_layer_v5(mask, vertex, 128, inlier_thresh=0.99, max_num=100, idxs=g["cat_idxs"],
                                        keep=keep, diag=dg)
    np.testing.assert_array_equal(dg[0]["counts"], g["cat_counts"][0])
    np.testing.assert_array_equal(dg[0]["conf_counts"], g["cat_conf_counts"][0])
    np.testing.assert_allclose(kp, g["cat_keypoints"], atol=KP_TOL)
    np.testing.assert_array_equal(conf, g["cat_conf"])
    dg = []
    kp, conf = O.ransac_voting_layer_v5(g["s_mask"], g["s_vertex"], 32, inlier_thresh=0.99, max_num=100,
                                        idxs=[g["s_idxs"][0], None], keep=g["s_keep"], diag=dg)
    np.testing.assert_array_equal(dg[0]["counts"], g["s_counts"][0])
    np.testing.assert_array_equal(dg[0]["conf_counts"], g["s_conf_counts"][0])
    np.testing.assert_allclose(kp, g["s_keypoints"], atol=KP_TOL)
    np.testing.assert_array_equal(conf, g["s_conf"])


def test_motion_voting_matches_reference_golden():
    g = G.load("motion_cases")
    np.testing.assert_allclose(O.ransac_motion_voting(g["mask"], g["vertex"]), g["points"], atol=1e-3, rtol=0)


def test_ycb21_v3_and_evd_with_mean():
    """configs[4] shapes (21 keypoints, YCB camera): v3 bit-exact counts and
    hypotheses, keypoints; EVD with mean (16 x 256 hypotheses) covariances."""
    g = G.load("ycb21_cases")
    mask, vertex, _ = G.ycb_inputs(g)
    gg = {k[3:]: (g[k].astype(np.int32) if k in ("v3_idxs", "v3_counts") else g[k])
          for k in g if k.startswith("v3_")}
    _, diag = check_v3(mask, vertex, gg)
    assert diag[0]["iters"] == int(g["v3_iters"])
    _, cov = O.estimate_voting_distribution_with_mean(mask, vertex, g["v3_keypoints"],
                                                      idxs=[list(g["evdm_idxs"][0].astype(np.int32))])
    np.testing.assert_allclose(cov, g["evdm_cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["evdm_cov"]).max())


def test_ycb21_evd_branches():
    """RV:343-348 (foreground < min_num: zero hypotheses, ratio 1 -> the
    covariance of the origin about the mean) and RV:351-355 (downsampled,
    foreground re-counted) in one batch, both EVD variants."""
    g = G.load("ycb21_cases")
    keep = lambda name: np.stack([np.ones((40, 48), bool), np.ones((40, 48), bool), g[f"br_{name}_keep2"]])
    ix = g["br_mean_idxs"]
    _, cov = O.estimate_voting_distribution_with_mean(
        g["br_mask"], g["br_vertex"], g["br_mean"], round_hyp_num=32, min_hyp_num=128, max_num=300,
        idxs=[list(ix[0]), None, list(ix[1])], keep=keep("mean"))
    np.testing.assert_allclose(cov, g["br_mean_cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["br_mean_cov"]).max())
    assert np.abs(g["br_mean_cov"][1]).max() > 0          # the skipped image's covariance is not zero
    ix = g["br_topk_idxs"]
    mu, cov = O.estimate_voting_distribution(
        g["br_mask"], g["br_vertex"], round_hyp_num=64, min_hyp_num=64, topk=64, min_num=20, max_num=300,
        idxs=[list(ix[0]), None, list(ix[1])], keep=keep("topk"))
    np.testing.assert_allclose(mu, g["br_topk_mean"], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(cov, g["br_topk_cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["br_topk_cov"]).max())
