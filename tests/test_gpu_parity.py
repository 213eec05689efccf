"""Parity of the HIP path (through the C ABI of libpvvote.so) with the CPU
oracle and the reference's golden vectors.  Bit-exact for hypotheses, inlier
bytes, counts, winners; tolerances for the fp32 least squares / covariances."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle as O
from pvnet_amd import _lib
from tests import golden_io as G

pytestmark = pytest.mark.gpu

KP_TOL = 1e-2
COV_RTOL = 1e-4


@pytest.fixture(scope="module")
def rv():
    from pvnet_amd import ransac_voting
    return ransac_voting


@pytest.fixture(scope="module")
def rvg():
    from pvnet_amd import ransac_voting_gpu
    return ransac_voting_gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def cu(x, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    return t.to(dev) if dtype is None else t.to(device=dev, dtype=dtype)


def test_native_library_is_the_gfx950_build(device):
    from pvnet_amd import _lib
    import ctypes
    L = _lib.load()
    buf = ctypes.create_string_buffer(64)
    assert L.pv_device_arch(buf, 64) == 0
    assert buf.value.decode().startswith("gfx950"), buf.value


def test_wave_min_max_reduction(device):
    """The DPP / permlane wave reduction the vote kernels' guard bands rest on
    (debug export, not in pvvote.h): every lane gets the min and max."""
    import ctypes
    from pvnet_amd import _lib
    L = _lib.load()
    fn = L.pv_debug_wave_minmax
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    rng = np.random.default_rng(7)
    x = rng.standard_normal((256, 64)).astype(np.float32) * 100
    for k in range(64):                  # the extreme in every lane position
        x[k, k] = 1e6
        x[64 + k, k] = -1e6
    x[128, 5] = np.nan                   # fminf / fmaxf skip NaN
    x[129, :] = 3.0
    xd = cu(x, device)
    out = torch.empty((256, 2), dtype=torch.float32, device=device)
    assert fn(xd.data_ptr(), out.data_ptr(), 256, torch.cuda.current_stream(device).cuda_stream) == 0
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[:, 0], np.nanmin(x, 1))
    np.testing.assert_array_equal(got[:, 1], np.nanmax(x, 1))


# ---------------------------------------------------------------- kernels
@pytest.mark.parametrize("case", ["cat_v3_512", "synth_v3_512"])
def test_generate_and_vote_kernels_bit_exact(case, device, rv):
    g = G.load(case)
    mask, vertex = (G.cat_inputs(g) if case.startswith("cat") else G.synth_inputs(g))[:2]
    coords, direct = O.compact(O.fg_mask_v3(mask[0]), vertex[0])
    idxs = g["idxs"][0]
    hyp = rv.generate_hypothesis(cu(direct, device), cu(coords, device), cu(idxs, device)).cpu().numpy()
    np.testing.assert_array_equal(bits(hyp), bits(g["hyp"][0]))
    cnt = rv.vote_counts(cu(direct, device), cu(coords, device), cu(hyp, device), 0.99).cpu().numpy()
    np.testing.assert_array_equal(cnt, g["counts"][0])
    # byte outputs on a slice of hypotheses (the full mask is 137 MB at the synthetic size)
    hs = slice(0, 64)
    ref = np.zeros((64, hyp.shape[1], coords.shape[0]), np.uint8)
    O.voting_for_hypothesis(direct, coords, hyp[hs], ref, 0.99)
    for dense in (False, True):
        out = torch.zeros(ref.shape, dtype=torch.uint8, device=device)
        fn = rv.voting_for_hypothesis_dense if dense else rv.voting_for_hypothesis
        fn(cu(direct, device), cu(coords, device), cu(hyp[hs], device), out, 0.99)
        np.testing.assert_array_equal(out.cpu().numpy(), ref)
        np.testing.assert_array_equal(out.cpu().numpy().sum(2), g["counts"][0][hs])


def test_vote_bytes_full_size(device, rv):
    """The bench's U1 call (hn=512, tn=29,861: the CU-balanced grid of full
    and quarter blocks): every row's inliers sum to the golden counts, and
    sampled rows -- in full blocks and in quarter blocks -- equal the
    oracle's bytes, in both modes."""
    g = G.load("synth_v3_512")
    mask, vertex = G.synth_inputs(g)[:2]
    coords, direct = O.compact(O.fg_mask_v3(mask[0]), vertex[0])
    hyp = g["hyp"][0]
    rows = np.array([0, 63, 64, 200, 255, 256, 300, 447, 448, 460, 497, 511])
    ref = np.zeros((len(rows), hyp.shape[1], coords.shape[0]), np.uint8)
    O.voting_for_hypothesis(direct, coords, hyp[rows], ref, 0.99)
    for dense in (False, True):
        out = torch.zeros((hyp.shape[0], hyp.shape[1], coords.shape[0]), dtype=torch.uint8, device=device)
        fn = rv.voting_for_hypothesis_dense if dense else rv.voting_for_hypothesis
        fn(cu(direct, device), cu(coords, device), cu(hyp, device), out, 0.99)
        np.testing.assert_array_equal(out.sum(2, dtype=torch.int32).cpu().numpy(), g["counts"][0])
        np.testing.assert_array_equal(out[torch.from_numpy(rows).to(device)].cpu().numpy(), ref)


def test_vote_bytes_balanced_grid_other_shape(device, rv):
    """hn=256, tn=15,000 (270 units on 256 CUs: 256 full + 56 quarter blocks,
    a different split of the CU-balanced grid): row sums equal the fused
    vote-count kernel's counts, sampled rows equal the oracle's bytes."""
    g = G.load("synth_v3_512")
    mask, vertex = G.synth_inputs(g)[:2]
    coords, direct = O.compact(O.fg_mask_v3(mask[0]), vertex[0])
    sel = np.sort(np.random.default_rng(11).choice(coords.shape[0], 15000, replace=False))
    coords, direct = np.ascontiguousarray(coords[sel]), np.ascontiguousarray(direct[sel])
    idxs = np.random.default_rng(12).integers(0, 15000, (256, 9, 2)).astype(np.int32)
    hyp = rv.generate_hypothesis(cu(direct, device), cu(coords, device), cu(idxs, device))
    cnt = rv.vote_counts(cu(direct, device), cu(coords, device), hyp, 0.99).cpu().numpy()
    out = torch.empty((256, 9, 15000), dtype=torch.uint8, device=device)
    rv.voting_for_hypothesis_dense(cu(direct, device), cu(coords, device), hyp, out, 0.99)
    np.testing.assert_array_equal(out.sum(2, dtype=torch.int32).cpu().numpy(), cnt)
    rows = np.array([0, 60, 64, 130, 192, 200, 240, 255])
    ref = np.zeros((len(rows), 9, 15000), np.uint8)
    O.voting_for_hypothesis(direct, coords, hyp.cpu().numpy()[rows], ref, 0.99)
    np.testing.assert_array_equal(out[torch.from_numpy(rows).to(device)].cpu().numpy(), ref)


def test_voting_or_semantics_keeps_existing_bytes(device, rv):
    g = G.load("edge_cases")
    coords, direct = O.compact(O.fg_mask_v3(g["c_mask"][0]), g["c_vertex"][0])
    hyp = g["c_hyp"][0]
    init = (np.random.default_rng(0).random((hyp.shape[0], hyp.shape[1], coords.shape[0])) < 0.3).astype(np.uint8) * 7
    ref = init.copy()
    O.voting_for_hypothesis(direct, coords, hyp, ref, 0.99)
    out = cu(init, device)
    rv.voting_for_hypothesis(cu(direct, device), cu(coords, device), cu(hyp, device), out, 0.99)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_guard_band_stress(seed, device, rv):
    """Thresholds placed exactly on reference cosines, degenerate pixels and
    hypotheses: every byte must still equal the exact reference decision."""
    rng = np.random.default_rng(seed)
    tn, vn, hn = 3000, 3, 200
    coords = np.stack([rng.integers(0, 640, tn), rng.integers(0, 480, tn)], 1).astype(np.float32)
    ang = rng.uniform(-np.pi, np.pi, (tn, vn))
    scale = rng.choice([1.0, 1e-7, 3e-7, 0.0, 1e5, 2e19], size=(tn, vn), p=[0.9, 0.02, 0.02, 0.02, 0.02, 0.02])
    direct = np.stack([np.cos(ang) * scale, np.sin(ang) * scale], -1).astype(np.float32)
    hyp = np.stack([rng.uniform(-100, 700, (hn, vn)), rng.uniform(-100, 600, (hn, vn))], -1).astype(np.float32)
    hyp[:10] = np.round(hyp[:10])                      # exactly on pixel centres / lattice
    hyp[10:12] = coords[rng.integers(0, tn, (2, vn))]  # exactly on foreground pixels
    hyp[12, :, 0] = 1e20                               # outside the fast domain
    hyp[13] = np.nan
    # thresholds equal to actual reference cosines (pairs land exactly on them)
    d = hyp[20, 0] - coords[5]
    for thr in (0.99, float(np.float32(np.dot(d, direct[5, 0]) / (np.linalg.norm(d) * np.linalg.norm(direct[5, 0])))),
                0.0, -0.5, 0.999999):
        ref = np.zeros((hn, vn, tn), np.uint8)
        O.voting_for_hypothesis(direct, coords, hyp, ref, thr)
        out = torch.zeros(ref.shape, dtype=torch.uint8, device=device)
        rv.voting_for_hypothesis_dense(cu(direct, device), cu(coords, device), cu(hyp, device), out, thr)
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"thr={thr}")
        cnt = rv.vote_counts(cu(direct, device), cu(coords, device), cu(hyp, device), thr).cpu().numpy()
        np.testing.assert_array_equal(cnt, ref.sum(2), err_msg=f"thr={thr}")


@pytest.mark.parametrize("span", [5000.0, 40000.0])
def test_vote_bytes_wide_frames(span, device, rv):
    """API coordinates spread over thousands of pixels at low thresholds: the
    matrix-core kernel's fp16 operands (b = tau u.c' up to tau R) must stay in
    range, or the window takes the exact sequence; fractional coordinates,
    a partial last window and a partial hypothesis set (hn = 80)."""
    rng = np.random.default_rng(int(span))
    tn, vn, hn = 1500, 2, 80
    coords = (rng.random((tn, 2)) * span).astype(np.float32)
    coords[::3] = np.round(coords[::3])
    ang = rng.uniform(-np.pi, np.pi, (tn, vn))
    direct = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)
    hyp = (rng.random((hn, vn, 2)) * span * 1.2 - span * 0.1).astype(np.float32)
    for thr in (0.3, 0.9, 0.99):
        ref = np.zeros((hn, vn, tn), np.uint8)
        O.voting_for_hypothesis(direct, coords, hyp, ref, thr)
        assert 0 < ref.sum() < ref.size
        out = torch.full(ref.shape, 9, dtype=torch.uint8, device=device)
        rv.voting_for_hypothesis_dense(cu(direct, device), cu(coords, device), cu(hyp, device), out, thr)
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"thr={thr}")
    # the counts at hn = 512 (k_vote_mfma's grid), same frames and thresholds
    hyp5 = (rng.random((512, vn, 2)) * span * 1.2 - span * 0.1).astype(np.float32)
    for thr in (0.3, 0.9):
        cnt = rv.vote_counts(cu(direct, device), cu(coords, device), cu(hyp5, device), thr).cpu().numpy()
        np.testing.assert_array_equal(cnt, O.vote_counts(direct, coords, hyp5, thr), err_msg=f"counts thr={thr}")


@pytest.mark.parametrize("full_queue", [False, True])
def test_band_pairs_both_modes(full_queue, device, rv):
    """Band pairs go through k_fix_bytes' queue (or, with the queue full, the
    in-kernel exact pass): dense and OR modes, thresholds on reference cosines."""
    L = _lib.load()
    prev = L.pv_debug_set_bytes_mode(4 if full_queue else 0)    # (test-only export, not in the header)
    try:
        _band_pairs_both_modes(device, rv)
    finally:
        L.pv_debug_set_bytes_mode(prev)


def _band_pairs_both_modes(device, rv):
    rng = np.random.default_rng(7)
    tn, vn, hn = 2500, 2, 96
    coords = np.stack([rng.integers(0, 640, tn), rng.integers(0, 480, tn)], 1).astype(np.float32)
    ang = rng.uniform(-np.pi, np.pi, (tn, vn))
    direct = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)
    hyp = np.stack([rng.uniform(-50, 690, (hn, vn)), rng.uniform(-50, 530, (hn, vn))], -1).astype(np.float32)
    hyp[5:9] = coords[rng.integers(0, tn, (4, vn))]
    d = hyp[20, 0] - coords[11]
    thr = float(np.float32(np.dot(d, direct[11, 0]) / (np.linalg.norm(d) * np.linalg.norm(direct[11, 0]))))
    init = (rng.random((hn, vn, tn)) < 0.2).astype(np.uint8) * 3
    for dense in (True, False):
        ref = np.zeros((hn, vn, tn), np.uint8) if dense else init.copy()
        O.voting_for_hypothesis(direct, coords, hyp, ref, thr)
        out = torch.zeros(ref.shape, dtype=torch.uint8, device=device) if dense else cu(init, device)
        fn = rv.voting_for_hypothesis_dense if dense else rv.voting_for_hypothesis
        fn(cu(direct, device), cu(coords, device), cu(hyp, device), out, thr)
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"dense={dense}")


def test_vp_kernels(device, rv):
    g = G.load("vp_kernels")
    hyp = rv.generate_hypothesis_vanishing_point(cu(g["direct"], device), cu(g["coords"], device),
                                                 cu(g["idxs"], device))
    np.testing.assert_array_equal(bits(hyp.cpu().numpy()), bits(g["hyp"]))
    inl = torch.zeros(g["inliers"].shape, dtype=torch.uint8, device=device)
    rv.voting_for_hypothesis_vanishing_point(cu(g["direct"], device), cu(g["coords"], device), hyp, inl, 0.99)
    np.testing.assert_array_equal(inl.cpu().numpy(), g["inliers"])


def test_input_checks(device, rv):
    d = torch.zeros(10, 3, 2, device=device)
    c = torch.zeros(10, 2, device=device)
    i = torch.zeros(4, 3, 2, dtype=torch.int32, device=device)
    with pytest.raises(RuntimeError, match="CUDA"):
        rv.generate_hypothesis(d.cpu(), c, i)
    with pytest.raises(RuntimeError, match="contiguous"):
        rv.generate_hypothesis(d.transpose(0, 1), c, i)


# ---------------------------------------------------------------- v3 pipeline
def run_v3(rvg, mask, vertex, g, prefix, device, hn=None, keep=None, **kw):
    idxs_g = g[prefix + "idxs"]
    b = mask.shape[0]
    fg = [int(O.fg_mask_v3(m).sum()) for m in mask]
    voted = [i for i, n in enumerate(fg) if n >= kw.get("min_num", 100)]
    hn = hn or idxs_g.shape[1]
    idxs = np.zeros((b, hn) + idxs_g.shape[2:], np.int32)
    for k, i in enumerate(voted):
        idxs[i] = idxs_g[k]
    diag = {}
    kp = rvg.ransac_voting_layer_v3(cu(mask, device), cu(vertex, device), hn, _idxs=idxs, _keep=keep,
                                    _diag=diag, **kw).cpu().numpy()
    diag = {k: v.cpu().numpy() for k, v in diag.items()}
    for k, i in enumerate(voted):
        np.testing.assert_array_equal(bits(diag["hyp"][i]), bits(g[prefix + "hyp"][k]))
        np.testing.assert_array_equal(diag["counts"][i].T, g[prefix + "counts"][k])
        np.testing.assert_array_equal(diag["win_idx"][i], np.argmax(g[prefix + "counts"][k], 0))
    for i in range(b):
        if i not in voted:
            assert diag["tn"][i] == 0 and np.all(kp[i] == 0)
    np.testing.assert_allclose(kp, g[prefix + "keypoints"], atol=KP_TOL, rtol=0)
    return kp, diag


def test_v3_cat_known_answer(device, rvg):
    g = G.load("cat_v3_512")
    mask, vertex, _ = G.cat_inputs(g)
    kp, diag = run_v3(rvg, mask, vertex, g, "", device)
    assert np.abs(kp[0] - g["points_2d"]).max() < 1e-3
    assert int(diag["iters"][0]) == int(g["iters"])


def test_v3_cat_downsampled(device, rvg):
    g = G.load("cat_v3_128_maxnum100")
    mask, vertex, _ = G.cat_inputs(g)
    keep = np.unpackbits(g["keep_bits"][0])[: 480 * 640].reshape(1, 480, 640)
    run_v3(rvg, mask, vertex, g, "", device, keep=keep, max_num=100)


@pytest.mark.parametrize("hn", [512, 128])
def test_v3_synth_full_size(hn, device, rvg):
    g = G.load(f"synth_v3_{hn}")
    mask, vertex, _ = G.synth_inputs(g)
    kp, diag = run_v3(rvg, mask, vertex, g, "", device)
    assert int(diag["tn"][0]) == 29861
    assert int(diag["iters"][0]) == int(g["iters"])


def _angles_f32(direct, coords, hyp):
    """KU:107-125's per-pixel sequence in float32 (numpy rounds each op like
    the kernel): the angle of each pixel's direction to the hypothesis, NaN
    where a norm guard rejects it.  direct/coords [tn,2], hyp [2]."""
    F = np.float32
    dx = F(hyp[0]) - coords[:, 0]
    dy = F(hyp[1]) - coords[:, 1]
    nx, ny = direct[:, 0], direct[:, 1]
    n1 = np.sqrt(nx * nx + ny * ny)
    n2 = np.sqrt(dx * dx + dy * dy)
    with np.errstate(all="ignore"):
        a = (dx * nx + dy * ny) / (n1 * n2)
    a[(n1 <= F(1e-6)) | (n2 <= F(1e-6))] = np.nan
    return a


@pytest.mark.parametrize("case", ["cat_v3_512", "synth_v3_512"])
@pytest.mark.parametrize("thr_mode", ["default", "boundary"])
def test_v3_refine_sums_match_oracle(case, thr_mode, device, rvg):
    """K6's least-squares sums (diag ata / atb) equal the oracle's (RV:584-599,
    correctly rounded) over the winner's inlier set -- one pixel in or out
    would move them by ~1/tn.  "boundary": the threshold is set to the exact
    float32 angle of some pixels to the first keypoint's winner, so those
    pixels sit exactly on the cone's edge (angle == thr: outliers) and the
    kernel's squared pre-test must hand them to the exact sequence."""
    g = G.load(case)
    mask, vertex = (G.cat_inputs(g) if case.startswith("cat") else G.synth_inputs(g))[:2]
    coords, direct = O.compact(O.fg_mask_v3(mask[0]), vertex[0])
    idxs = g["idxs"]
    thr = 0.99
    if thr_mode == "boundary":
        d0 = {}
        rvg.ransac_voting_layer_v3(cu(mask, device), cu(vertex, device), 512, _idxs=idxs, _diag=d0)
        w0 = int(d0["win_idx"].cpu().numpy()[0, 0])
        hyp0 = d0["hyp"].cpu().numpy()[0, w0, 0]
        a = _angles_f32(direct[:, 0], coords, hyp0)
        cand = np.sort(a[np.isfinite(a) & (a > 0.9) & (a < 1.0)])
        thr = float(cand[len(cand) // 2])
        assert np.count_nonzero(a == np.float32(thr)) >= 1
    diag = {}
    rvg.ransac_voting_layer_v3(cu(mask, device), cu(vertex, device), 512, inlier_thresh=thr, _idxs=idxs,
                               _diag=diag)
    diag = {k: v.cpu().numpy() for k, v in diag.items()}
    vn = vertex.shape[3]
    win_pts = diag["hyp"][0][diag["win_idx"][0], np.arange(vn)]
    win_pts[diag["win_ratio"][0] <= 0] = 0
    _, ata, atb = O.refine(direct, coords, win_pts.astype(np.float32), np.float32(thr))
    np.testing.assert_allclose(diag["ata"][0].reshape(vn, 2, 2), ata, rtol=1e-6, atol=1e-7 * np.abs(ata).max())
    np.testing.assert_allclose(diag["atb"][0].reshape(vn, 2), atb, rtol=1e-6, atol=1e-7 * np.abs(atb).max())


def test_v3_many_hypotheses(device, rvg):
    """round_hyp_num 2048 (> 1024: k_refine_solve's instantiation that keeps the
    hypotheses in memory and reads the counts past the first 1024 in a loop)
    on a cropped synthetic frame, against the oracle with the same pixel
    pairs: counts bit-exact, the winners, the fp64 sums, the keypoints."""
    g = G.load("synth_v3_512")
    mask, vertex, _ = G.synth_inputs(g)
    crop = np.zeros_like(mask)
    crop[:, 190:250, 280:340] = mask[:, 190:250, 280:340]      # a few thousand foreground pixels
    tn = int(O.fg_mask_v3(crop[0]).sum())
    assert 1000 < tn < 4000
    hn = 2048
    idxs = np.random.default_rng(5).integers(0, tn, size=(1, hn, vertex.shape[3], 2), dtype=np.int32)
    diag = {}
    kp = rvg.ransac_voting_layer_v3(cu(crop, device), cu(vertex, device), hn, _idxs=idxs, _diag=diag).cpu().numpy()
    diag = {k: v.cpu().numpy() for k, v in diag.items()}
    dg = []
    ko = O.ransac_voting_layer_v3(crop, vertex, hn, idxs=[idxs[0]], diag=dg)
    np.testing.assert_array_equal(diag["counts"][0].T, dg[0]["counts"])
    np.testing.assert_array_equal(diag["win_idx"][0], dg[0]["win_idx"])
    vn = vertex.shape[3]
    np.testing.assert_allclose(diag["ata"][0].reshape(vn, 2, 2), dg[0]["ATA"], rtol=1e-6,
                               atol=1e-7 * np.abs(dg[0]["ATA"]).max())
    np.testing.assert_allclose(diag["atb"][0].reshape(vn, 2), dg[0]["ATb"], rtol=1e-6,
                               atol=1e-7 * np.abs(dg[0]["ATb"]).max())
    np.testing.assert_allclose(kp, ko, atol=KP_TOL, rtol=0)


def test_v3_from_network_fused(device, rvg):
    """seg_pred/vertex_pred straight from the network layout (argmax fused)."""
    g = G.load("synth_v3_512")
    _, _, f = G.synth_inputs(g)
    idxs = g["idxs"]
    for dt in (torch.float32, torch.float16):
        seg = cu(f["seg"], device, dt)
        ver = cu(f["vertex"], device, dt)
        diag = {}
        kp = rvg.ransac_voting_layer_v3_from_network(seg, ver, 512, _idxs=idxs, _diag=diag).cpu().numpy()
        if dt == torch.float32:
            np.testing.assert_array_equal(bits(diag["hyp"].cpu().numpy()[0]), bits(g["hyp"][0]))
            np.testing.assert_array_equal(diag["counts"].cpu().numpy()[0].T, g["counts"][0])
            np.testing.assert_allclose(kp, g["keypoints"], atol=KP_TOL, rtol=0)
        else:
            # fp16 network outputs: compare with the oracle on the same (rounded) field
            v16 = f["vertex"].astype(np.float16).astype(np.float32)
            vv = np.ascontiguousarray(v16.transpose(0, 2, 3, 1).reshape(1, 480, 640, 9, 2))
            dg = []
            ko = O.ransac_voting_layer_v3(np.argmax(f["seg"], 1), vv, 512, idxs=[idxs[0]], diag=dg)
            np.testing.assert_array_equal(diag["counts"].cpu().numpy()[0].T, dg[0]["counts"])
            np.testing.assert_allclose(kp, ko, atol=KP_TOL, rtol=0)


def test_v3_edge_cases(device, rvg):
    g = G.load("edge_cases")
    run_v3(rvg, g["a_mask"], g["a_vertex"], g, "a_", device)
    kp, diag = run_v3(rvg, g["b_mask"], g["b_vertex"], g, "b_", device)
    assert int(diag["iters"][0]) == int(g["b_iters"]) == 101
    np.testing.assert_allclose(kp[0], diag["atb"][0], rtol=1e-6)     # b_inv identity fallback
    run_v3(rvg, g["c_mask"], g["c_vertex"], g, "c_", device)
    run_v3(rvg, g["d_mask"], g["d_vertex"], g, "d_", device, keep=g["d_keep"].astype(np.uint8), max_num=300)
    run_v3(rvg, g["e_mask"], g["e_vertex"], g, "e_", device, inlier_thresh=0.999)


def test_v3_mask_dtypes_and_contiguous_vertex(device, rvg):
    g = G.load("edge_cases")
    m = g["a_mask"]
    base, _ = run_v3(rvg, m, g["a_vertex"], g, "a_", device)
    for conv in (lambda x: x.astype(np.int32), lambda x: (x & 0xFF).astype(np.uint8)):
        kp, _ = run_v3(rvg, conv(m), g["a_vertex"], g, "a_", device)
        np.testing.assert_array_equal(kp, base)


def test_v3_rng_path_statistical(device, rvg):
    """Device RNG instead of injected idxs: results agree with the oracle's
    (different random draws) within the north star's 0.5 px."""
    g = G.load("synth_v3_512")
    mask, vertex, f = G.synth_inputs(g)
    torch.manual_seed(0)
    kp = rvg.ransac_voting_layer_v3(cu(mask, device), cu(vertex, device), 512).cpu().numpy()
    np.testing.assert_allclose(kp, g["keypoints"], atol=0.5)
    gc = G.load("cat_v3_512")
    mc, vc, _ = G.cat_inputs(gc)
    kc = rvg.ransac_voting_layer_v3(cu(mc, device), cu(vc, device), 512).cpu().numpy()
    assert np.abs(kc[0] - gc["points_2d"]).max() < 1e-3


def test_v3_batch_matches_single(device, rvg):
    """8 synthetic images in one batched call == 8 single calls (same idxs)."""
    from pvnet_amd import synth
    fb = synth.synthetic_batch(4, seed=100)
    mask = np.argmax(fb["seg"], 1)
    vertex = np.ascontiguousarray(fb["vertex"].transpose(0, 2, 3, 1).reshape(4, 480, 640, 9, 2))
    idxs = np.random.default_rng(3).integers(0, 29861, (4, 128, 9, 2)).astype(np.int32)
    kb = rvg.ransac_voting_layer_v3(cu(mask, device), cu(vertex, device), 128, _idxs=idxs).cpu().numpy()
    for i in range(4):
        k1 = rvg.ransac_voting_layer_v3(cu(mask[i:i + 1], device), cu(vertex[i:i + 1], device), 128,
                                        _idxs=idxs[i:i + 1]).cpu().numpy()
        np.testing.assert_array_equal(kb[i], k1[0])
        ko = O.ransac_voting_layer_v3(mask[i:i + 1], vertex[i:i + 1], 128, idxs=[idxs[i]])
        np.testing.assert_allclose(kb[i], ko[0], atol=KP_TOL)
        np.testing.assert_allclose(kb[i], fb["keypoints"][i], atol=5.0)   # noisy field vs generator truth


def test_v3_batch_wide_compaction(device, rvg):
    """A batch large enough for the multi-chunk compaction (k_compact_wide:
    more than 4,096 one-chunk blocks) -- five full frames, one of them below
    min_num and one empty -- with and without downsampling (an injected
    keep-mask at max_num 20,000; the chunks then go one by one through the
    look-back).  Every image equals its own single call (the one-chunk
    kernels) bit for bit, and the oracle's keypoints."""
    from pvnet_amd import synth
    b, hn = 5, 128
    fb = synth.synthetic_batch(b, seed=300)
    mask = np.argmax(fb["seg"], 1).astype(np.int64)
    mask[3] = 0
    mask[3, 100:105, 200:210] = 1          # 50 pixels: below min_num
    mask[4] = 0                            # empty
    vertex = np.ascontiguousarray(fb["vertex"].transpose(0, 2, 3, 1).reshape(b, 480, 640, 9, 2))
    rng = np.random.default_rng(31)
    keep = (rng.random((b, 480, 640)) < 0.6).astype(np.uint8)
    for max_num, kp_keep in ((30000, None), (20000, keep)):
        tn = [int(((mask[i] != 0) & (kp_keep[i] != 0 if kp_keep is not None else True)).sum()) for i in range(b)]
        fg = [int((mask[i] != 0).sum()) for i in range(b)]
        n_idx = [t if f > max_num else f for t, f in zip(tn, fg)]
        idxs = np.stack([rng.integers(0, max(n, 1), (hn, 9, 2)) for n in n_idx]).astype(np.int32)
        diag = {}
        kb = rvg.ransac_voting_layer_v3(cu(mask, device), cu(vertex, device), hn, max_num=max_num, _idxs=idxs,
                                        _keep=kp_keep, _diag=diag).cpu().numpy()
        for i in range(b):
            d1 = {}
            k1 = rvg.ransac_voting_layer_v3(cu(mask[i:i + 1], device), cu(vertex[i:i + 1], device), hn,
                                            max_num=max_num, _idxs=idxs[i:i + 1],
                                            _keep=None if kp_keep is None else kp_keep[i:i + 1],
                                            _diag=d1).cpu().numpy()
            assert int(diag["tn"][i]) == int(d1["tn"][0]), (max_num, i)
            np.testing.assert_array_equal(diag["counts"][i].cpu().numpy(), d1["counts"][0].cpu().numpy())
            np.testing.assert_array_equal(kb[i], k1[0])
            ko = O.ransac_voting_layer_v3(mask[i:i + 1], vertex[i:i + 1], hn, max_num=max_num, idxs=[idxs[i]],
                                          keep=None if kp_keep is None else [kp_keep[i]])
            np.testing.assert_allclose(kb[i], ko[0], atol=KP_TOL)
        assert int(diag["tn"][3]) == 0 and int(diag["tn"][4]) == 0
        assert int(diag["tn"][0]) == (n_idx[0] if max_num == 20000 else fg[0])


# ---------------------------------------------------------------- EVD
@pytest.mark.parametrize("case", ["cat_evdm", "synth_evdm"])
def test_evd_with_mean(case, device, rvg):
    g = G.load(case)
    mask, vertex = (G.cat_inputs(g) if case.startswith("cat") else G.synth_inputs(g))[:2]
    idxs = g["idxs"][0].reshape(1, -1, 9, 2)
    _, cov = rvg.estimate_voting_distribution_with_mean(cu(mask, device), cu(vertex, device), cu(g["mean"], device),
                                                        _idxs=idxs)
    cov = cov.cpu().numpy()
    np.testing.assert_allclose(cov, g["cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["cov"]).max())


def test_evd_edge_batch(device, rvg):
    g = G.load("edge_cases")
    idx = g["a_evdm_idxs"]
    idxs = np.stack([idx[0:4].reshape(-1, 3, 2), idx[4:8].reshape(-1, 3, 2), idx[8:12].reshape(-1, 3, 2)])
    _, cov = rvg.estimate_voting_distribution_with_mean(cu(g["a_mask"], device), cu(g["a_vertex"], device),
                                                        cu(g["a_keypoints"], device), round_hyp_num=32,
                                                        min_hyp_num=100, _idxs=idxs)
    np.testing.assert_allclose(cov.cpu().numpy(), g["a_evdm_cov"], rtol=COV_RTOL,
                               atol=1e-4 * np.abs(g["a_evdm_cov"]).max())


def test_evd_topk(device, rvg):
    g = G.load("synth_evd_top4096")
    mask, vertex, _ = G.synth_inputs(g)
    idxs = g["idxs"][0].reshape(1, -1, 9, 2)
    mu, cov = rvg.estimate_voting_distribution(cu(mask, device), cu(vertex, device), topk=4096, _idxs=idxs)
    np.testing.assert_allclose(mu.cpu().numpy(), g["mean"], atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(cov.cpu().numpy(), g["cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["cov"]).max())
    g = G.load("synth_evd_top128")
    idxs = g["idxs"][0].reshape(1, -1, 9, 2)
    mu, cov = rvg.estimate_voting_distribution(cu(mask, device), cu(vertex, device), topk=128, _idxs=idxs)
    mo, co = O.estimate_voting_distribution(mask, vertex, topk=128, idxs=[list(g["idxs"][0])])
    np.testing.assert_allclose(mu.cpu().numpy(), mo, atol=1e-3, rtol=1e-5)
    np.testing.assert_allclose(cov.cpu().numpy(), co, rtol=COV_RTOL, atol=1e-4 * np.abs(co).max())


def test_graph_capture(device, rvg):
    """The whole v3 pipeline is capturable in a hipGraph and replays exactly."""
    from pvnet_amd import synth
    f = synth.synthetic_field(7)
    seg = cu(f["seg"], device)
    ver = cu(f["vertex"], device)
    ws = rvg.VotingWorkspace()
    out = torch.empty((1, 9, 2), device=device)
    rvg.ransac_voting_layer_v3_from_network(seg, ver, 128, _seed=5, _workspace=ws, out=out)
    ref = out.clone()
    torch.cuda.synchronize()
    gph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(gph, stream=s):
            rvg.ransac_voting_layer_v3_from_network(seg, ver, 128, _seed=5, _workspace=ws, out=out)
    out.zero_()
    gph.replay()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref.cpu().numpy())


def test_fractional_coordinates_and_ragged_rows(device, rv):
    """API inputs with non-integer coordinates (c - o is rounded in the fast
    test) and row lengths that are not multiples of 8 (every byte-row start
    alignment); bytes and counts equal the reference decisions."""
    rng = np.random.default_rng(7)
    for tn in (1, 7, 513, 1029):
        vn, hn = 2, 37
        coords = (np.stack([rng.uniform(0, 640, tn), rng.uniform(0, 480, tn)], 1)).astype(np.float32)
        kp = np.array([[300.3, 200.7], [100.1, 400.9]], np.float32)
        d = kp[None] - coords[:, None]
        ang = np.arctan2(d[..., 1], d[..., 0]) + rng.normal(0, 0.1, (tn, vn))
        direct = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32) * rng.uniform(0.5, 2, (tn, vn, 1)).astype(np.float32)
        hyp = (kp[None] + rng.normal(0, 20, (hn, vn, 2))).astype(np.float32)
        ref = np.zeros((hn, vn, tn), np.uint8)
        O.voting_for_hypothesis(direct, coords, hyp, ref, 0.99)
        out = torch.full(ref.shape, 9, dtype=torch.uint8, device=device)
        rv.voting_for_hypothesis_dense(cu(direct, device), cu(coords, device), cu(hyp, device), out, 0.99)
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"tn={tn}")
        cnt = rv.vote_counts(cu(direct, device), cu(coords, device), cu(hyp, device), 0.99).cpu().numpy()
        np.testing.assert_array_equal(cnt, ref.sum(2), err_msg=f"tn={tn}")


def test_v5_confidence_matches_reference(device, rvg):
    """ransac_voting_layer_v5 as TRAIN:123 calls it (hn=128, 0.99, max_num=100):
    hypotheses and counts bit-exact, keypoints within tolerance, and the 0.999
    confidence equal to the reference's."""
    g = G.load("v5_cases")
    mask, vertex, _ = G.cat_inputs(g)
    keep = np.unpackbits(g["cat_keep_bits"][0])[: 480 * 640].reshape(1, 480, 640)
    diag = {}
    kp, conf = rvg.ransac_voting_layer_v5(cu(mask, device), cu(vertex, device), 128, inlier_thresh=0.99,
                                          max_num=100, _idxs=g["cat_idxs"], _keep=keep, _diag=diag)
    np.testing.assert_array_equal(diag["counts"].cpu().numpy()[0].T, g["cat_counts"][0])
    np.testing.assert_allclose(kp.cpu().numpy(), g["cat_keypoints"], atol=KP_TOL, rtol=0)
    np.testing.assert_array_equal(conf.cpu().numpy(), g["cat_conf"])
    # batch: a downsampled small field and one below min_num (zeros)
    idxs = np.zeros((2,) + g["s_idxs"].shape[1:], np.int32)
    idxs[0] = g["s_idxs"][0]
    diag = {}
    kp, conf = rvg.ransac_voting_layer_v5(cu(g["s_mask"], device), cu(g["s_vertex"], device), 32,
                                          inlier_thresh=0.99, max_num=100, _idxs=idxs,
                                          _keep=g["s_keep"].astype(np.uint8), _diag=diag)
    np.testing.assert_array_equal(diag["counts"].cpu().numpy()[0].T, g["s_counts"][0])
    np.testing.assert_allclose(kp.cpu().numpy(), g["s_keypoints"], atol=KP_TOL, rtol=0)
    np.testing.assert_array_equal(conf.cpu().numpy(), g["s_conf"])


def test_motion_voting(device, rvg):
    """ransac_motion_voting (RV:966-987): the reference's own outputs (fp32
    torch.mean) within 1e-3 px, the oracle's fp64 mean within 1e-4 px."""
    g = G.load("motion_cases")
    got = rvg.ransac_motion_voting(cu(g["mask"], device), cu(g["vertex"], device)).cpu().numpy()
    np.testing.assert_allclose(got, g["points"], atol=1e-3, rtol=0)
    np.testing.assert_allclose(got, O.ransac_motion_voting(g["mask"], g["vertex"]), atol=1e-4, rtol=0)
    assert np.all(got[2] == 0)


# ---------------------------------------------------------------- configs[2]
@pytest.mark.parametrize("half", [False, True])
def test_v3_config2_batch32_mixed(half, device, rvg):
    """configs[2]'s voting call: one batch of 32 network-layout fields whose
    foreground spans ~2k..30k pixels (13 disk radii, cycling), hn=512, with
    injected pixel pairs; fp16 network outputs (the fp16 backbone's) are voted
    in fp32.  Every image's counts equal the oracle's bit for bit (the oracle
    votes the same fp16-rounded directions) and its keypoints agree."""
    from pvnet_amd import synth
    b, hn = 32, 512
    fs = [synth.synthetic_field(5000 + i, radius=25.0 + 72.5 * (i % 13) / 12.0) for i in range(b)]
    dt = np.float16 if half else np.float32
    seg = np.concatenate([f["seg"] for f in fs]).astype(dt)
    ver = np.concatenate([f["vertex"] for f in fs]).astype(dt)
    rng = np.random.default_rng(32)
    idxs = np.stack([rng.integers(0, f["tn"], (hn, 9, 2)) for f in fs]).astype(np.int32)
    diag = {}
    kp = rvg.ransac_voting_layer_v3_from_network(cu(seg, device), cu(ver, device), hn, _idxs=idxs,
                                                 _diag=diag).cpu().numpy()
    counts = diag["counts"].cpu().numpy()
    assert sorted(int(f["tn"]) for f in fs)[0] < 2500 and max(int(f["tn"]) for f in fs) == 29861
    for i in range(b):
        vv = np.ascontiguousarray(ver[i:i + 1].astype(np.float32).transpose(0, 2, 3, 1).reshape(1, 480, 640, 9, 2))
        dg = []
        ko = O.ransac_voting_layer_v3(np.argmax(seg[i:i + 1].astype(np.float32), 1), vv, hn, idxs=[idxs[i]], diag=dg)
        np.testing.assert_array_equal(counts[i].T, dg[0]["counts"], err_msg=f"image {i}")
        np.testing.assert_allclose(kp[i], ko[0], atol=KP_TOL, err_msg=f"image {i}")


def test_default_workspace_two_streams(device, rvg):
    """Calls without _workspace on two streams at once: the default
    workspace keeps one buffer per (device, stream), so concurrent calls do not
    overwrite each other's scratch; results equal the sequential ones."""
    from pvnet_amd import synth
    fa, fb = synth.synthetic_field(41), synth.synthetic_field(42)
    ia = np.random.default_rng(1).integers(0, fa["tn"], (1, 256, 9, 2)).astype(np.int32)
    ib = np.random.default_rng(2).integers(0, fb["tn"], (1, 256, 9, 2)).astype(np.int32)
    sa, va, sb, vb = (cu(fa["seg"], device), cu(fa["vertex"], device), cu(fb["seg"], device), cu(fb["vertex"], device))
    ra = rvg.ransac_voting_layer_v3_from_network(sa, va, 256, _idxs=ia).cpu().numpy()
    rb = rvg.ransac_voting_layer_v3_from_network(sb, vb, 256, _idxs=ib).cpu().numpy()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for _ in range(3):
        s1.wait_stream(torch.cuda.current_stream())
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s1):
            oa = rvg.ransac_voting_layer_v3_from_network(sa, va, 256, _idxs=ia)
        with torch.cuda.stream(s2):
            ob = rvg.ransac_voting_layer_v3_from_network(sb, vb, 256, _idxs=ib)
        torch.cuda.current_stream().wait_stream(s1)
        torch.cuda.current_stream().wait_stream(s2)
        outs.append((oa, ob))
    torch.cuda.synchronize()
    for oa, ob in outs:
        np.testing.assert_array_equal(oa.cpu().numpy(), ra)
        np.testing.assert_array_equal(ob.cpu().numpy(), rb)


def test_workspace_growth_inside_capture_raises(device, rvg):
    """A workspace that would allocate inside a graph capture raises (warm it up first)."""
    from pvnet_amd import synth
    f = synth.synthetic_field(43, H=96, W=128, radius=30.5, center=(64.0, 48.0))
    seg, ver = cu(f["seg"], device), cu(f["vertex"], device)
    g = torch.cuda.CUDAGraph()
    with pytest.raises(RuntimeError, match="graph capture"):
        with torch.cuda.graph(g):
            rvg.ransac_voting_layer_v3_from_network(seg, ver, 64, _workspace=rvg.VotingWorkspace(), _seed=1)


# ---------------------------------------------------------------- configs[4]: 21 keypoints
def test_ycb21_v3_and_evd_with_mean(device, rvg):
    """vn = 21 (YCB, configs[4]) through v3 (hn 512, bit-exact counts and
    hypotheses vs the reference's) and EVD with mean (16 x 256 hypotheses)."""
    g = G.load("ycb21_cases")
    mask, vertex, _ = G.ycb_inputs(g)
    gg = {k[3:]: (g[k].astype(np.int32) if k in ("v3_idxs", "v3_counts") else g[k])
          for k in g if k.startswith("v3_")}
    kp, diag = run_v3(rvg, mask, vertex, gg, "", device)
    assert int(diag["iters"][0]) == int(g["v3_iters"])
    idxs = g["evdm_idxs"][0].astype(np.int32).reshape(1, -1, 21, 2)
    _, cov = rvg.estimate_voting_distribution_with_mean(cu(mask, device), cu(vertex, device),
                                                        cu(g["v3_keypoints"], device), _idxs=idxs)
    np.testing.assert_allclose(cov.cpu().numpy(), g["evdm_cov"], rtol=COV_RTOL,
                               atol=1e-4 * np.abs(g["evdm_cov"]).max())


def test_ycb21_evd_branches(device, rvg):
    """One batch with a normal image, one below min_num (RV:343-348) and one
    above max_num (RV:351-355, the reference's keep-mask injected), both EVD
    variants, against the reference's covariances."""
    g = G.load("ycb21_cases")
    m, v = cu(g["br_mask"], device), cu(g["br_vertex"], device)
    for name in ("mean", "topk"):
        ix = g[f"br_{name}_idxs"]
        idxs = np.zeros((3, ix.shape[1] * ix.shape[2], 21, 2), np.int32)
        idxs[0] = ix[0].reshape(-1, 21, 2)
        idxs[2] = ix[1].reshape(-1, 21, 2)
        keep = np.ones((3, 40, 48), np.uint8)
        keep[2] = g[f"br_{name}_keep2"]
        if name == "mean":
            _, cov = rvg.estimate_voting_distribution_with_mean(m, v, cu(g["br_mean"], device), round_hyp_num=32,
                                                                min_hyp_num=128, max_num=300, _idxs=idxs, _keep=keep)
        else:
            mu, cov = rvg.estimate_voting_distribution(m, v, round_hyp_num=64, min_hyp_num=64, topk=64, min_num=20,
                                                       max_num=300, _idxs=idxs, _keep=keep)
            np.testing.assert_allclose(mu.cpu().numpy(), g["br_topk_mean"], atol=1e-3, rtol=1e-5)
        ref = g[f"br_{name}_cov"]
        np.testing.assert_allclose(cov.cpu().numpy(), ref, rtol=COV_RTOL, atol=1e-4 * np.abs(ref).max())


# ---------------------------------------------------------------- both vote kernels
@pytest.mark.parametrize("kernel", [0, 1], ids=["k_vote_mfma", "k_vote_count"])
def test_both_vote_kernels_bit_exact(kernel, device, rvg):
    """The matrix-core vote kernel (default) and the VALU one give the
    reference's counts bit for bit: full-size synthetic and cat fields, the
    edge batch, 21 keypoints, and the EVD rounds (hn 4096) -- selected per
    call through pv_debug_set_vote_kernel."""
    import ctypes
    L = _lib.load()
    L.pv_debug_set_vote_kernel.argtypes = [ctypes.c_int32]
    L.pv_debug_set_vote_kernel.restype = ctypes.c_int32
    prev = L.pv_debug_set_vote_kernel(kernel)
    try:
        for name in ("synth_v3_512", "cat_v3_512"):
            g = G.load(name)
            mask, vertex = (G.synth_inputs(g) if name.startswith("synth") else G.cat_inputs(g))[:2]
            run_v3(rvg, mask, vertex, g, "", device)
        g = G.load("edge_cases")
        run_v3(rvg, g["c_mask"], g["c_vertex"], g, "c_", device)
        g = G.load("ycb21_cases")
        mask, vertex, _ = G.ycb_inputs(g)
        gg = {k[3:]: (g[k].astype(np.int32) if k in ("v3_idxs", "v3_counts") else g[k])
              for k in g if k.startswith("v3_")}
        run_v3(rvg, mask, vertex, gg, "", device)
        g = G.load("synth_evdm")
        mask, vertex, _ = G.synth_inputs(g)
        _, cov = rvg.estimate_voting_distribution_with_mean(cu(mask, device), cu(vertex, device),
                                                            cu(g["mean"], device), _idxs=g["idxs"][0].reshape(1, -1, 9, 2))
        np.testing.assert_allclose(cov.cpu().numpy(), g["cov"], rtol=COV_RTOL, atol=1e-4 * np.abs(g["cov"]).max())
    finally:
        L.pv_debug_set_vote_kernel(prev)


def test_compaction_lookback_self_count_fallback(device, rvg):
    """The downsampling look-back of k_compact with every earlier block's kept
    count worked out by the waiting thread itself -- the path a block takes
    when a predecessor has not been scheduled within the spin limit -- gives
    the golden results (downsampled cat, the downsampled edge case)."""
    L = _lib.load()
    L.pv_debug_lookback_self.argtypes = [ctypes.c_int32]
    L.pv_debug_lookback_self.restype = ctypes.c_int32
    assert L.pv_debug_lookback_self(1) == 0
    try:
        g = G.load("cat_v3_128_maxnum100")
        mask, vertex, _ = G.cat_inputs(g)
        keep = np.unpackbits(g["keep_bits"][0])[: 480 * 640].reshape(1, 480, 640)
        run_v3(rvg, mask, vertex, g, "", device, keep=keep, max_num=100)
        g = G.load("edge_cases")
        run_v3(rvg, g["d_mask"], g["d_vertex"], g, "d_", device, keep=g["d_keep"].astype(np.uint8), max_num=300)
    finally:
        L.pv_debug_lookback_self(0)


def test_workspace_reused_across_shapes(device, rvg):
    """One workspace through calls of different shapes, downsampled and not:
    each call matches its golden results (no state carried between calls)."""
    ws = rvg.VotingWorkspace()
    gs = G.load("synth_v3_512")
    ms, vs, _ = G.synth_inputs(gs)
    ge = G.load("edge_cases")
    gd = G.load("cat_v3_128_maxnum100")
    md, vd, _ = G.cat_inputs(gd)
    keep = np.unpackbits(gd["keep_bits"][0])[: 480 * 640].reshape(1, 480, 640)
    for _ in range(2):
        run_v3(rvg, ge["a_mask"], ge["a_vertex"], ge, "a_", device, _workspace=ws)
        run_v3(rvg, ms, vs, gs, "", device, _workspace=ws)
        run_v3(rvg, ge["b_mask"], ge["b_vertex"], ge, "b_", device, _workspace=ws)
        run_v3(rvg, md, vd, gd, "", device, keep=keep, max_num=100, _workspace=ws)
        run_v3(rvg, ge["d_mask"], ge["d_vertex"], ge, "d_", device, keep=ge["d_keep"].astype(np.uint8), max_num=300,
               _workspace=ws)


def test_random_api_votes_match_oracle(device, rv):
    """A slice of tools/fuzz_votes.py (which ran 15,448 such cases on the GPU
    box, profiles/r02_fuzz_votes.txt): random tn / vn / hn / thresholds /
    coordinate spans with degenerate pixels and hypotheses; dense bytes, OR
    bytes and counts all equal the oracle's."""
    for case in range(1000, 1024):
        rng = np.random.default_rng(case)
        tn, vn = int(rng.integers(1, 3000)), int(rng.integers(1, 4))
        hn = int(rng.choice([1, 7, 100, 200, 512]))
        span = float(rng.choice([8.0, 640.0, 5000.0, 50000.0]))
        thr = float(rng.choice([0.99, 0.9, 0.5, 0.3, 0.999]))
        coords = (rng.random((tn, 2)) * span).astype(np.float32)
        ang = rng.uniform(-np.pi, np.pi, (tn, vn))
        scale = rng.choice([1.0, 1e-7, 0.0, 2e19], size=(tn, vn), p=[0.97, 0.01, 0.01, 0.01])
        direct = np.stack([np.cos(ang) * scale, np.sin(ang) * scale], -1).astype(np.float32)
        hyp = (rng.random((hn, vn, 2)) * span * 1.4 - span * 0.2).astype(np.float32)
        hyp[rng.random((hn, vn)) < 0.03] = 3e7
        ref = np.zeros((hn, vn, tn), np.uint8)
        O.voting_for_hypothesis(direct, coords, hyp, ref, thr)
        dd, cc, hh = cu(direct, device), cu(coords, device), cu(hyp, device)
        out = torch.zeros(ref.shape, dtype=torch.uint8, device=device)
        rv.voting_for_hypothesis_dense(dd, cc, hh, out, thr)
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"case {case} dense")
        init = (rng.random(ref.shape) < 0.1).astype(np.uint8) * 5
        out = cu(init, device)
        rv.voting_for_hypothesis(dd, cc, hh, out, thr)
        np.testing.assert_array_equal(out.cpu().numpy(), np.where(ref == 1, 1, init), err_msg=f"case {case} OR")
        np.testing.assert_array_equal(rv.vote_counts(dd, cc, hh, thr).cpu().numpy(), ref.sum(2), err_msg=f"case {case}")


@pytest.mark.parametrize("case", ["stress0", "stress1", "wide5000", "wide40000", "tiny17", "ragged1000"])
def test_vote_bytes_dense_512(case, device, rv):
    """Dense voting_for_hypothesis at hn = 512 (the bench's U1 shape, the
    CU-balanced byte grid): every byte equals the oracle's (KU:116-125) --
    thresholds on reference cosines and outside the
    fast range, degenerate / huge / zero directions, hypotheses on pixel
    centres, on the integer lattice, huge and NaN, fractional and wide-spread
    coordinates, windows and batches cut short -- and over a byte pattern
    left in the output (dense: every byte rewritten)."""
    rng = np.random.default_rng(sum(map(ord, case)))
    hn = 512
    if case.startswith("stress"):
        tn, vn = 3000, 2
        coords = np.stack([rng.integers(0, 640, tn), rng.integers(0, 480, tn)], 1).astype(np.float32)
        ang = rng.uniform(-np.pi, np.pi, (tn, vn))
        scale = rng.choice([1.0, 1e-7, 3e-7, 0.0, 1e5, 2e19], size=(tn, vn), p=[0.9, 0.02, 0.02, 0.02, 0.02, 0.02])
        direct = np.stack([np.cos(ang) * scale, np.sin(ang) * scale], -1).astype(np.float32)
        hyp = np.stack([rng.uniform(-100, 700, (hn, vn)), rng.uniform(-100, 600, (hn, vn))], -1).astype(np.float32)
        hyp[:10] = np.round(hyp[:10])
        hyp[10:12] = coords[rng.integers(0, tn, (2, vn))]
        hyp[12, :, 0] = 1e20
        hyp[13] = np.nan
        hyp[300:310] = coords[rng.integers(0, tn, (10, vn))]
        d = hyp[20, 0] - coords[5]
        thrs = (0.99, float(np.float32(np.dot(d, direct[5, 0]) / (np.linalg.norm(d) * np.linalg.norm(direct[5, 0])))),
                0.0, 0.999999)
    elif case.startswith("wide"):
        span = float(case[4:])
        tn, vn = 1500, 2
        coords = (rng.random((tn, 2)) * span).astype(np.float32)
        coords[::3] = np.round(coords[::3])
        ang = rng.uniform(-np.pi, np.pi, (tn, vn))
        direct = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)
        hyp = (rng.random((hn, vn, 2)) * span * 1.2 - span * 0.1).astype(np.float32)
        thrs = (0.3, 0.9, 0.99)
    else:
        tn = 17 if case == "tiny17" else 1000
        vn = 3
        coords = np.stack([rng.integers(200, 440, tn), rng.integers(120, 360, tn)], 1).astype(np.float32)
        kp = np.array([320.0, 240.0], np.float32)
        d0 = kp - coords
        ang = np.arctan2(d0[:, 1], d0[:, 0])[:, None] + rng.normal(0, 0.05, (tn, vn))
        direct = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)
        hyp = (kp + rng.normal(0, 30, (hn, vn, 2))).astype(np.float32)
        thrs = (0.99, 0.9)
    for thr in thrs:
        ref = np.zeros((hn, vn, tn), np.uint8)
        O.voting_for_hypothesis(direct, coords, hyp, ref, thr)
        out = torch.full(ref.shape, 5, dtype=torch.uint8, device=device)
        rv.voting_for_hypothesis_dense(cu(direct, device), cu(coords, device), cu(hyp, device), out, thr)
        np.testing.assert_array_equal(out.cpu().numpy(), ref, err_msg=f"{case} thr={thr}")
