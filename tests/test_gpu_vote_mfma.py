"""Adversarial parity of the product vote/count kernel, k_vote_mfma, and the
matrix-core arithmetic its exactness argument rests on.

k_vote_mfma decides a (hypothesis, pixel) pair by the sign of z = X - |Y|,
X and Y evaluated on the matrix cores from hi/lo-split fp16 operands; a pair
whose |z| is inside the guard band gzm*B + gzr*D is re-decided by the
reference's IEEE sequence (ransac_voting_kernel.cu:116-125).  These tests
(1) measure the matrix core's f32 sum of 8 exact fp16 products on crafted
cancellation sums against the 16 u * sum|terms| the band assumes, and
(2) run k_vote_mfma -- the kernel pv_vote_counts and the pipeline launch for
hn a multiple of 512 -- on inputs built to land on the threshold: thresholds
equal to reference cosines, degenerate direction scales, NaN / 1e20 / 3e7
hypotheses and hypotheses on pixel centres.  Counts must equal the oracle's
bit for bit."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import oracle as O
from pvnet_amd import _lib

pytestmark = pytest.mark.gpu

U = 2.0 ** -24
MFMA_SUM_BOUND = 16.0      # u * sum|terms| (pvvote.hip mfma_gz)


def cu(x, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(x))
    return t.to(dev) if dtype is None else t.to(device=dev, dtype=dtype)


def mfma_sums(A, B, device):
    """D[i] = A[i] (32 x 8 fp16) @ B[i] (8 x 32 fp16) on v_mfma_f32_32x32x8_f16."""
    L = _lib.load()
    fn = L.pv_debug_mfma_sums
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
    T = A.shape[0]
    a = torch.from_numpy(A.view(np.int16).copy()).to(device)
    b = torch.from_numpy(B.view(np.int16).copy()).to(device)
    d = torch.empty((T, 32, 32), dtype=torch.float32, device=device)
    assert fn(a.data_ptr(), b.data_ptr(), d.data_ptr(), T, torch.cuda.current_stream(device).cuda_stream) == 0
    return d.cpu().numpy()


def crafted_tiles(rng, T):
    """Tiles whose sums maximise accumulated rounding: per tile one position p
    holds a product near 1 (random mantissa and sign), the other seven
    products sit near one f32 ulp of it (2^-25 .. 2^-21, signs all equal to the
    big one's, all opposite, or mixed), so every addition of a sequential,
    truncating or aligned-and-truncated sum loses up to a full ulp; plus
    near-cancelling pairs of big products, fp16 subnormal operands and
    random wide-range operands."""
    A = np.zeros((T, 32, 8), np.float16)
    B = np.zeros((T, 8, 32), np.float16)
    for i in range(T):
        fam = i % 4
        p = (i // 4) % 8
        if fam == 0 or fam == 1:
            sm = -11 - (i // 32) % 3                      # small B scale 2^-11 .. 2^-13
            ma = 1 + rng.integers(0, 1024, (32, 8)) / 1024.0
            mb = 1 + rng.integers(0, 1024, (8, 32)) / 1024.0
            sa = np.ones((32, 8))
            sb = rng.choice([-1.0, 1.0], (8, 32))
            if fam == 1:                                  # smalls share the big product's sign (or oppose it)
                sb = np.broadcast_to(rng.choice([-1.0, 1.0], (1, 32)), (8, 32)).copy()
                sb[p] = rng.choice([-1.0, 1.0], 32)
            A[i] = (ma * sa * 2.0 ** -12).astype(np.float16)
            A[i, :, p] = (ma[:, p] / 2).astype(np.float16)  # big A in [0.5, 1)
            B[i] = (mb * sb * 2.0 ** sm).astype(np.float16)
            B[i, p] = (mb[p] * sb[p]).astype(np.float16)
        elif fam == 2:                                    # near-cancelling big pair + smalls
            q = (p + 1 + (i // 32) % 7) % 8
            x = 1 + rng.integers(0, 1024, 32) / 1024.0
            A[i] = (rng.choice([-1.0, 1.0], (32, 8)) * 2.0 ** -12 * (1 + rng.integers(0, 1024, (32, 8)) / 1024.0)
                    ).astype(np.float16)
            A[i, :, p] = x.astype(np.float16)
            A[i, :, q] = (-x * (1 - rng.integers(1, 64, 32) * 2.0 ** -11)).astype(np.float16)
            B[i] = (2.0 ** -11 * (1 + rng.integers(0, 1024, (8, 32)) / 1024.0)).astype(np.float16)
            B[i, p] = 1.0
            B[i, q] = 1.0
        else:                                             # subnormal fp16 operands / wide random range
            ea = rng.integers(-24, 6, (32, 8)).astype(np.float64)
            eb = rng.integers(-14, 6, (8, 32)).astype(np.float64)
            A[i] = (rng.uniform(-1, 1, (32, 8)) * 2.0 ** ea).astype(np.float16)
            B[i] = (rng.uniform(-1, 1, (8, 32)) * 2.0 ** eb).astype(np.float16)
    return A, B


def nominal(x):
    """|x| with fp16 subnormals counted at 2^-14: the matrix core aligns the
    8 products to the largest product exponent taken from the operands'
    exponent fields (a subnormal operand has exponent -14 there), so a sum
    whose largest nominal product is a subnormal one with leading zeros keeps
    fewer bits of the actual values (tools/mfma_sub_probe.py: every single
    product, subnormal operands included, is exact; a normal product beside a
    subnormal one stays within 2 u of the sum)."""
    a = np.abs(x.astype(np.float64))
    return np.where((a > 0) & (a < 2.0 ** -14), 2.0 ** -14, a)


def test_mfma_sum_error_bound(device):
    """The matrix core's f32 sum of 8 exact fp16 products stays within
    16 u of the sum of the products' nominal magnitudes (= sum|terms| when
    no operand is an fp16 subnormal) -- the constant k_vote_mfma's guard band
    (mfma_gz) is derived with, DESIGN.md 5a -- on crafted worst cases: one
    product near 1 with seven near one f32 ulp of it (every addition of a
    sequential, truncating or aligned sum loses up to an ulp), near-cancelling
    pairs, and random operands over the whole fp16 range including
    subnormals."""
    rng = np.random.default_rng(2024)
    T = 512
    A, B = crafted_tiles(rng, T)
    D = mfma_sums(A, B, device).astype(np.float64)
    t = A.astype(np.float64)[:, :, :, None] * B.astype(np.float64)[:, None, :, :]   # exact products [T,32,8,32]
    exact = t.astype(np.longdouble).sum(axis=2)       # 22-bit products, < 50-bit spread: exact in 64-bit mantissa
    mag = np.abs(t).sum(axis=2)
    nom = (nominal(A)[:, :, :, None] * nominal(B)[:, None, :, :]).sum(axis=2)
    err = np.abs(D.astype(np.longdouble) - exact).astype(np.float64)
    ok = mag > 0
    assert np.all(err[~ok] == 0)
    ratio = np.zeros_like(mag)
    ratio[ok] = err[ok] / (nom[ok] * U)
    plain = np.zeros_like(mag)
    plain[ok] = err[ok] / (mag[ok] * U)
    fam = [round(float(ratio[f::4].max()), 3) for f in range(4)]
    print(f"matrix-core sum error: max {ratio.max():.3f} u * nominal sum over {ok.sum()} sums (families {fam}); "
          f"normal-operand families {max(plain[f::4].max() for f in range(3)):.3f} "
          f"u * sum|terms|; with subnormal operands up to {plain[3::4].max():.1f} u * sum|terms|")
    assert ratio.max() <= MFMA_SUM_BOUND, ratio.max()
    assert max(plain[f::4].max() for f in range(3)) <= MFMA_SUM_BOUND
    # every single product is exact (fp16 x fp16 fits f32), subnormal operands included
    A1 = np.zeros((1, 32, 8), np.float16)
    B1 = np.zeros((1, 8, 32), np.float16)
    A1[0, :, 3] = (rng.uniform(-1, 1, 32) * 2.0 ** rng.integers(-24, 8, 32)).astype(np.float16)
    B1[0, 3, :] = (rng.uniform(-1, 1, 32) * 2.0 ** rng.integers(-24, 8, 32)).astype(np.float16)
    D1 = mfma_sums(A1, B1, device)
    np.testing.assert_array_equal(D1[0], (A1[0, :, 3:4].astype(np.float32) * B1[0, 3:4, :].astype(np.float32)))


def _stress_inputs(seed, tn=3000, vn=3, hn=512, fractional=False):
    rng = np.random.default_rng(seed)
    coords = np.stack([rng.integers(0, 640, tn), rng.integers(0, 480, tn)], 1).astype(np.float32)
    if fractional:
        coords[::2] += rng.random((coords[::2].shape[0], 2)).astype(np.float32)
    ang = rng.uniform(-np.pi, np.pi, (tn, vn))
    scale = rng.choice([1.0, 1e-7, 3e-7, 0.0, 1e5, 2e19], size=(tn, vn), p=[0.9, 0.02, 0.02, 0.02, 0.02, 0.02])
    direct = np.stack([np.cos(ang) * scale, np.sin(ang) * scale], -1).astype(np.float32)
    hyp = np.stack([rng.uniform(-100, 700, (hn, vn)), rng.uniform(-100, 600, (hn, vn))], -1).astype(np.float32)
    hyp[:10] = np.round(hyp[:10])                           # on the integer lattice
    hyp[10:14] = coords[rng.integers(0, tn, (4, vn))]       # exactly on foreground pixels
    hyp[14, :, 0] = 1e20                                    # outside the fast domain
    hyp[15] = np.nan
    hyp[16:24] = rng.uniform(-3e7, 3e7, (8, vn, 2)).astype(np.float32)   # |h| >= 8e6: exact-only in k_vote_mfma
    hyp[24] = np.float32(3e7)
    hyp[25:28] = np.inf * rng.choice([-1, 1], (3, vn, 2))
    hyp[28:40] = (coords[rng.integers(0, tn, (12, vn))] + rng.normal(0, 1e-3, (12, vn, 2))).astype(np.float32)
    return coords, direct, hyp


def _ref_cosines(coords, direct, hyp, rng, k=3):
    """Thresholds equal to the cosines of actual (hypothesis, pixel) pairs, in
    the reference's fp32 arithmetic (KU:116-123 with contraction off)."""
    out = []
    tn, vn = direct.shape[:2]
    while len(out) < k:
        h, v, t = int(rng.integers(40, hyp.shape[0])), int(rng.integers(0, vn)), int(rng.integers(0, tn))
        n = direct[t, v]
        d = (hyp[h, v] - coords[t]).astype(np.float32)
        n1 = np.sqrt(np.float32(n[0] * n[0]) + np.float32(n[1] * n[1]), dtype=np.float32)
        n2 = np.sqrt(np.float32(d[0] * d[0]) + np.float32(d[1] * d[1]), dtype=np.float32)
        if not (n1 > 1e-6 and n2 > 1e-6):
            continue
        c = np.float32(np.float32(np.float32(d[0] * n[0]) + np.float32(d[1] * n[1])) / np.float32(n1 * n2))
        if 0.05 <= c <= 0.999999:
            out.append(float(c))
    return out


@pytest.mark.parametrize("seed, fractional", [(0, False), (1, False), (2, True), (3, True)])
def test_vote_mfma_guard_band_stress(seed, fractional, device):
    """k_vote_mfma through pv_vote_counts at hn=512 on threshold-hugging
    inputs: thresholds on reference cosines (and the fast domain's edges),
    degenerate scales, NaN / inf / 1e20 / 3e7 hypotheses, hypotheses on and
    within 1e-3 px of pixel centres; fractional API coordinates in two cases.
    Counts equal the oracle's; the VALU kernel (k_vote_count) is run on the
    same inputs through the pipeline hook for comparison."""
    from pvnet_amd import ransac_voting as rv
    coords, direct, hyp = _stress_inputs(seed, fractional=fractional)
    rng = np.random.default_rng(100 + seed)
    thrs = [0.99, 0.05, 0.999999, 0.3] + _ref_cosines(coords, direct, hyp, rng)
    dd, cc, hh = cu(direct, device), cu(coords, device), cu(hyp, device)
    for thr in thrs:
        want = O.vote_counts(direct, coords, hyp, thr)
        got = rv.vote_counts(dd, cc, hh, thr).cpu().numpy()
        np.testing.assert_array_equal(got, want, err_msg=f"seed {seed} thr={thr!r}")


def test_vote_mfma_pipeline_threshold_on_cosines(device):
    """The pipeline (k_vote_mfma on compacted pixel records) with inlier_thresh
    equal to reference cosines of its own hypotheses, a direction field with
    degenerate scales (0, 1e-7, 1e5, 2e19) and injected pairs that include
    t0 == t1 and zero-direction pixels: counts equal the oracle's."""
    from pvnet_amd import ransac_voting_gpu as rvg
    from pvnet_amd import synth
    f = synth.synthetic_field(77, scale_jitter=True)
    vv = np.ascontiguousarray(f["vertex"].transpose(0, 2, 3, 1).reshape(1, 480, 640, 9, 2))
    rng = np.random.default_rng(5)
    rows, cols = np.nonzero(f["mask"])
    pick = rng.random(rows.shape[0]) < 0.05
    sc = rng.choice([0.0, 1e-7, 1e5, 2e19], size=(int(pick.sum()), 9, 1)).astype(np.float32)
    vv[0, rows[pick], cols[pick]] *= sc
    mask = f["mask"][None].astype(np.int64)
    tn = int(f["tn"])
    idxs = rng.integers(0, tn, (1, 512, 9, 2)).astype(np.int32)
    idxs[0, :16, :, 1] = idxs[0, :16, :, 0]                  # t0 == t1: the (0, 0) hypothesis
    coords, direct = O.compact(O.fg_mask_v3(mask[0]), vv[0])
    hyp = O.generate_hypothesis(direct, coords, idxs[0])
    thrs = [0.99] + _ref_cosines(coords, direct, hyp, rng, k=2)
    for thr in thrs:
        dg = []
        ko = O.ransac_voting_layer_v3(mask, vv, 512, inlier_thresh=thr, idxs=[idxs[0]], diag=dg)
        diag = {}
        kp = rvg.ransac_voting_layer_v3(cu(mask, device), cu(vv, device), 512, inlier_thresh=thr, _idxs=idxs,
                                        _diag=diag).cpu().numpy()
        np.testing.assert_array_equal(diag["counts"].cpu().numpy()[0].T, dg[0]["counts"], err_msg=f"thr={thr!r}")
        np.testing.assert_allclose(kp, ko, atol=1e-2, rtol=0, err_msg=f"thr={thr!r}")


# ---------------------------------------------------------------- the kernel's own forms
def _f16_split(x):
    """hi + lo fp16 split of f32 x (form_row / the B fragments: lo = x - hi in f32, rounded)."""
    x = np.asarray(x, np.float32)
    hi = x.astype(np.float16)
    lo = (x - hi.astype(np.float32)).astype(np.float32).astype(np.float16)
    return hi, lo


def _fmaf(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(np.float32)


def kernel_forms(u, cq, hq, tau):
    """A / B operands exactly as k_vote_mfma builds them (form_row, the B
    fragments; pvvote.hip), for pixels with unit directions u [P,2] (f32),
    offsets c' [P,2] from the origin (f32, integers for pixel centres) and
    hypotheses h' [H,2] (f32) -- P = 16 pixels and H = 32 hypotheses per
    tile.  Returns (A [32, 8], B [8, 32], s [32])."""
    tau = np.float32(tau)
    A = np.zeros((32, 8), np.float16)
    for p in range(16):
        ux, uy = np.float32(u[p, 0]), np.float32(u[p, 1])
        cx, cy = np.float32(cq[p, 0]), np.float32(cq[p, 1])
        axX, ayX = np.float32(tau * ux), np.float32(tau * uy)
        for r, (ax, ay, b) in enumerate(((axX, ayX, _fmaf(axX, cx, np.float32(ayX * cy))),
                                         (np.float32(-uy), ux, _fmaf(-uy, cx, np.float32(ux * cy))))):
            axh, axl = _f16_split(ax)
            ayh, ayl = _f16_split(ay)
            bh, bl = _f16_split(np.float32(-b))
            A[2 * p + r] = [axh, axh, axl, ayh, ayh, ayl, bh, bl]
    B = np.zeros((8, 32), np.float16)
    s = np.zeros(32, np.float64)
    for j in range(32):
        hx, hy = np.float32(hq[j, 0]), np.float32(hq[j, 1])
        mag = max(abs(hx), abs(hy))
        e = int(np.frexp(mag)[1]) if mag > 0 else 0           # mag < 2^e
        k = max(0, e - 14)
        sj = np.float32(2.0 ** -k)
        xh, xl = _f16_split(np.float32(hx * sj))
        yh, yl = _f16_split(np.float32(hy * sj))
        B[:, j] = [xh, xl, xh, yh, yl, yh, np.float16(sj), np.float16(sj)]
        s[j] = float(sj)
    return A, B, s


@pytest.mark.parametrize("thr", [0.99, 0.9, 0.5, 0.05, 0.999999])
def test_mfma_forms_error_bound(thr, device):
    """The forms k_vote_mfma evaluates, X = tau u.(h'-c') and Y = u x (h'-c')
    on the matrix cores from its own hi/lo fp16 operands, give z = X - |Y|
    within (41.5 tau + 38.7) u B s of the exact z (B = |h'| + |c'| + 1) -- the
    error budget of DESIGN.md 5a (pvvote.hip mfma_gz, before its 2x margin)
    -- on realistic and adversarial operands: random and near-axis unit
    directions (split parts in the fp16 subnormal range), offsets up to the
    fp16 range limit of b (30000 / max(tau, 1)), hypotheses from 1e-4 px to
    8e6 px away (s down to 2^-9) and hypotheses placed on the threshold cone."""
    rng = np.random.default_rng(int(thr * 1e6))
    tau64 = np.sqrt(1.0 - np.float64(np.float32(thr)) ** 2) / np.float64(np.float32(thr))
    tau = np.float32(tau64)
    Rmax = 30000.0 / max(float(tau), 1.0)
    T = 192
    As, Bs, S, U_, C_, H_ = [], [], [], [], [], []
    for i in range(T):
        reg = i % 6
        ang = rng.uniform(-np.pi, np.pi, 16)
        if reg == 1:                                   # near-axis directions: tiny components
            ang = rng.choice([0, np.pi / 2, np.pi, -np.pi / 2], 16) + rng.uniform(-1e-4, 1e-4, 16)
        u = np.stack([np.cos(ang), np.sin(ang)], 1).astype(np.float32)
        R = [300.0, 5.0, Rmax * 0.99, 1000.0, 50.0, 200.0][reg]
        cq = np.round(rng.uniform(-R, R, (16, 2)) / np.sqrt(2)).astype(np.float32)
        dist = [rng.uniform(0, 800, 32), 10.0 ** rng.uniform(-4, 1, 32), rng.uniform(0, 3e4, 32),
                10.0 ** rng.uniform(3, 6.9, 32), rng.uniform(0, 2, 32), rng.uniform(0, 600, 32)][reg]
        ha = rng.uniform(-np.pi, np.pi, 32)
        hq = np.stack([np.cos(ha), np.sin(ha)], 1) * dist[:, None]
        if reg == 5:                                   # on the threshold cone of pixel j % 16
            th = np.arccos(np.float64(np.float32(thr))) * rng.choice([-1, 1], 32)
            p = np.arange(32) % 16
            base = np.arctan2(u[p, 1], u[p, 0]) + th
            hq = cq[p] + np.stack([np.cos(base), np.sin(base)], 1) * rng.uniform(1, 600, (32, 1))
        hq = hq.astype(np.float32)
        A, B, s = kernel_forms(u, cq, hq, tau)
        As.append(A)
        Bs.append(B)
        S.append(s)
        U_.append(u)
        C_.append(cq)
        H_.append(hq)
    D = mfma_sums(np.stack(As), np.stack(Bs), device)                  # [T, 32, 32]
    worst = 0.0
    for i in range(T):
        u, cq, hq, s = U_[i].astype(np.float64), C_[i].astype(np.float64), H_[i].astype(np.float64), S[i]
        X, Y = D[i, 0::2, :], D[i, 1::2, :]                             # [16 pixels, 32 hypotheses]
        z = (X - np.abs(Y)).astype(np.float32).astype(np.float64)        # the kernel's f32 z
        d = hq[None, :, :] - cq[:, None, :]                              # exact h' - c'
        xp = u[:, None, 0] * d[..., 0] + u[:, None, 1] * d[..., 1]
        yp = u[:, None, 0] * d[..., 1] - u[:, None, 1] * d[..., 0]
        zt = (tau64 * xp - np.abs(yp)) * s[None, :]
        Bb = (np.hypot(hq[:, 0], hq[:, 1])[None, :] + np.hypot(cq[:, 0], cq[:, 1])[:, None] + 1.0) * s[None, :]
        bound = (41.5 * float(tau) + 38.7) * U * Bb
        r = np.abs(z - zt) / bound
        worst = max(worst, float(r.max()))
        assert np.all(np.abs(z - zt) <= bound), (i, float(r.max()))
    print(f"thr {thr}: matrix-core forms within {worst:.3f} of the error budget (41.5 tau + 38.7) u B s")
