"""CPU oracle for the uncertainty-weighted PnP stage -- TEST INFRASTRUCTURE ONLY.

Only ``tests/`` (and ``bench.py``'s ``cpu_baseline`` leg) may import this
module, and only as the checker / a timed CPU baseline.  The product package
``pvnet_amd`` never imports it.

What it restates (the consumer of the EVD covariances):

* ``weights_from_cov``   -- lib/utils/evaluation_utils.py:168-178
  (W = inv(sqrtm(C)) per keypoint, zero when C[0,0] < 1e-6 or C has a NaN);
* ``weights_v2``         -- lib/utils/extend_utils/extend_utils.py:131-139
  (isotropic 1 / max eigenvalue, zero when C[0,0] < 1e-5);
* ``uncertainty_pnp``    -- extend_utils.py:63-114: P3P initial pose on the
  four highest-weight points (``cv2.solvePnP(..., SOLVEPNP_P3P)``), then the
  weighted reprojection least squares of
  lib/utils/extend_utils/src/uncertainty_pnp.cpp:7-92 solved by Ceres;
* ``uncertainty_pnp_v2`` -- extend_utils.py:116-166.

Third-party algorithms restated here (neither library is importable or
buildable in this image):

* OpenCV ``SOLVEPNP_P3P`` (opencv 3.4 / 4.x, ``modules/calib3d/src/p3p.cpp``):
  the P3P problem on points 0..2 of the four, the candidate whose
  reprojection of point 3 is closest wins.  Any exact P3P solver yields the
  same candidate set; here Grunert's quartic (Haralick et al., IJCV 1994,
  eqs. 9-13; verified numerically) with real roots from ``numpy.roots``
  polished by Newton steps, and each candidate's pose from the two
  congruent triangles' orthonormal frames.
* ``cv2.Rodrigues`` (rotation vector <-> matrix).
* Ceres Solver 2.0 (``ceres/rotation.h`` AngleAxisRotatePoint, ``Jet``
  forward-mode autodiff, ``TrustRegionMinimizer`` with the
  ``LevenbergMarquardtStrategy`` and the default ``Solver::Options``:
  Jacobi column scaling fixed at iteration 0, initial trust region radius
  1e4, max radius 1e16, min relative decrease 1e-3, diagonal clamped to
  [1e-6, 1e32], function / gradient / parameter tolerances 1e-6 / 1e-10 /
  1e-8, 50 iterations).

Parity: unpinned by reference outputs (Ceres, cv2 and the cffi library are
absent); pinned by the reference's own known-answer self-test
(uncertainty_pnp.cpp:98-156: exact correspondences, a perturbed start, the
pose recovered) and by exact-data P3P recovery -- tests/test_pnp_oracle.py.
"""
from __future__ import annotations

import numpy as np

EPS = np.finfo(np.float64).eps


# ---------------------------------------------------------------- weights
def sqrtm_spd2(c):
    """Principal square root of a symmetric 2x2 PSD matrix (the value
    scipy.linalg.sqrtm returns for one): (C + s I) / sqrt(tr C + 2 s), s = sqrt(det C)."""
    c = np.asarray(c, np.float64)
    det = max(c[0, 0] * c[1, 1] - c[0, 1] * c[1, 0], 0.0)
    s = np.sqrt(det)
    t = np.sqrt(c[0, 0] + c[1, 1] + 2.0 * s)
    return (c + s * np.eye(2)) / t


def weights_from_cov(cov):
    """evaluation_utils.py:168-178 -> [pn, 3] (wxx, wxy, wyy) of inv(sqrtm(C))."""
    cov = np.asarray(cov, np.float64)
    out = np.zeros((cov.shape[0], 3), np.float64)
    for i in range(cov.shape[0]):
        c = cov[i]
        if c[0, 0] < 1e-6 or np.isnan(c).any():
            continue
        w = np.linalg.inv(sqrtm_spd2(c))
        out[i] = (w[0, 0], w[0, 1], w[1, 1])
    return out


def weights_v2(cov):
    """extend_utils.py:131-139, 157-159 -> [pn, 3] (w, 0, w), w = 1 / max eig(C)."""
    cov = np.asarray(cov, np.float64)
    w = np.zeros(cov.shape[0], np.float64)
    for i in range(cov.shape[0]):
        if cov[i, 0, 0] < 1e-5:
            continue
        if np.isnan(cov[i]).any():      # the reference's eigvals raises here; the device gives NaN
            w[i] = np.nan
            continue
        w[i] = 1.0 / np.max(np.linalg.eigvals(cov[i]).real)
    return np.stack([w, np.zeros_like(w), w], 1)


# ---------------------------------------------------------------- rotations
def rodrigues_vec_to_mat(r):
    """cv2.Rodrigues(rvec) -> R."""
    r = np.asarray(r, np.float64).reshape(3)
    th = np.sqrt(r @ r)
    if th < EPS:
        return np.eye(3)
    k = r / th
    c, s = np.cos(th), np.sin(th)
    kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return c * np.eye(3) + (1 - c) * np.outer(k, k) + s * kx


def rodrigues_mat_to_vec(R):
    """cv2.Rodrigues(R) -> rvec for an orthonormal R: the axis from the skew
    part, theta = acos((tr R - 1) / 2); near theta = pi (skew part < 1e-5) the
    axis from R = 2 k k^T - I (either sign is the same rotation)."""
    R = np.asarray(R, np.float64)
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = np.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = np.clip((R[0, 0] + R[1, 1] + R[2, 2] - 1) * 0.5, -1.0, 1.0)
    th = np.arccos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros(3)
        # theta ~ pi: R = 2 k k^T - I; the axis from the largest diagonal entry
        m = int(np.argmax(np.diag(R)))
        k = np.zeros(3)
        k[m] = np.sqrt(max((R[m, m] + 1.0) * 0.5, 0.0))
        for i in range(3):
            if i != m:
                k[i] = (R[m, i] + R[i, m]) * 0.25 / k[m]
        return k / np.sqrt(k @ k) * th
    vth = 1.0 / (2.0 * s) * th
    return np.array([rx, ry, rz]) * vth


# ---------------------------------------------------------------- P3P
def _real_roots4(a):
    """Real roots of a4 x^4 + ... + a0 (numpy.roots), each polished by Newton."""
    a = np.asarray(a, np.float64)
    nz = np.nonzero(np.abs(a) > 0)[0]
    if len(nz) == 0:
        return []
    r = np.roots(a[nz[0]:])
    out = []
    scale = np.max(np.abs(r)) if len(r) else 1.0
    for z in r:
        if abs(z.imag) > 1e-8 * max(1.0, abs(z)) and abs(z.imag) > 1e-10 * scale:
            continue
        x = z.real
        for _ in range(3):
            p = np.polyval(a, x)
            dp = np.polyval(np.polyder(a), x)
            if dp == 0:
                break
            x = x - p / dp
        out.append(x)
    return out


def p3p_candidates(P, rays):
    """Grunert's P3P on world points P[0..2] and unit rays[0..2] -> list of (R, t)."""
    P = np.asarray(P, np.float64)
    j = np.asarray(rays, np.float64)
    a = np.linalg.norm(P[1] - P[2])
    b = np.linalg.norm(P[0] - P[2])
    c = np.linalg.norm(P[0] - P[1])
    ca, cb, cg = j[1] @ j[2], j[0] @ j[2], j[0] @ j[1]
    a2, b2, c2 = a * a, b * b, c * c
    if b2 == 0:
        return []
    amc, apc = (a2 - c2) / b2, (a2 + c2) / b2
    A4 = (amc - 1) ** 2 - 4 * c2 / b2 * ca ** 2
    A3 = 4 * (amc * (1 - amc) * cb - (1 - apc) * ca * cg + 2 * c2 / b2 * ca ** 2 * cb)
    A2 = 2 * (amc ** 2 - 1 + 2 * amc ** 2 * cb ** 2 + 2 * (b2 - c2) / b2 * ca ** 2 - 4 * apc * ca * cb * cg
              + 2 * (b2 - a2) / b2 * cg ** 2)
    A1 = 4 * (-amc * (1 + amc) * cb + 2 * a2 / b2 * cg ** 2 * cb - (1 - apc) * ca * cg)
    A0 = (1 + amc) ** 2 - 4 * a2 / b2 * cg ** 2
    out = []
    for v in _real_roots4([A4, A3, A2, A1, A0]):
        if v <= 0:
            continue
        den = 2 * (cg - v * ca)
        if den == 0:
            continue
        u = ((-1 + amc) * v * v - 2 * amc * cb * v + 1 + amc) / den
        q = 1 + v * v - 2 * v * cb
        if u <= 0 or q <= 0:
            continue
        s1 = np.sqrt(b2 / q)
        C = np.stack([s1 * j[0], u * s1 * j[1], v * s1 * j[2]])
        R, t = _frames_pose(P[:3], C)
        if R is not None:
            out.append((R, t))
    return out


def _frame(X):
    e1 = X[1] - X[0]
    n1 = np.linalg.norm(e1)
    e3 = np.cross(e1, X[2] - X[0])
    n3 = np.linalg.norm(e3)
    if n1 == 0 or n3 == 0:
        return None
    e1, e3 = e1 / n1, e3 / n3
    return np.stack([e1, np.cross(e3, e1), e3], 1)


def _frames_pose(P, C):
    """R, t with C_i = R P_i + t for two congruent triangles (orthonormal frames)."""
    FP, FC = _frame(P), _frame(C)
    if FP is None or FC is None:
        return None, None
    R = FC @ FP.T
    t = C[0] - R @ P[0]
    return R, t


def p3p_pose(P4, x4, K):
    """cv2.solvePnP(P4, x4, K, 0, flags=SOLVEPNP_P3P): candidates from points
    0..2, the one reprojecting point 3 closest (squared pixels) wins.
    Returns (ok, rvec, t)."""
    P4 = np.asarray(P4, np.float64)
    x4 = np.asarray(x4, np.float64)
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    mu = (x4[:, 0] - cx) / fx
    mv = (x4[:, 1] - cy) / fy
    rays = np.stack([mu, mv, np.ones(4)], 1)
    rays /= np.linalg.norm(rays, axis=1, keepdims=True)
    best, best_e = None, None
    for R, t in p3p_candidates(P4[:3], rays[:3]):
        X = R @ P4[3] + t
        if X[2] == 0:
            continue
        e = (cx + fx * X[0] / X[2] - x4[3, 0]) ** 2 + (cy + fy * X[1] / X[2] - x4[3, 1]) ** 2
        if best is None or e < best_e:
            best, best_e = (R, t), e
    if best is None:
        return False, np.zeros(3), np.zeros(3)
    return True, rodrigues_mat_to_vec(best[0]), best[1]


# ---------------------------------------------------------------- jets (Ceres Jet<double, 6>)
class Jet:
    __slots__ = ("a", "v")

    def __init__(self, a, v=None):
        self.a = np.float64(a)        # numpy semantics: x / 0 -> inf, like the device
        self.v = np.zeros(6) if v is None else v

    def __add__(self, o):
        return Jet(self.a + o.a, self.v + o.v) if isinstance(o, Jet) else Jet(self.a + o, self.v)

    __radd__ = __add__

    def __sub__(self, o):
        return Jet(self.a - o.a, self.v - o.v) if isinstance(o, Jet) else Jet(self.a - o, self.v)

    def __rsub__(self, o):
        return Jet(o - self.a, -self.v)

    def __mul__(self, o):
        if isinstance(o, Jet):
            return Jet(self.a * o.a, self.a * o.v + self.v * o.a)
        return Jet(self.a * o, self.v * o)

    __rmul__ = __mul__

    def __truediv__(self, o):
        if isinstance(o, Jet):
            inv = 1.0 / o.a
            f_over_g = self.a * inv
            return Jet(self.a * inv, (self.v - f_over_g * o.v) * inv)
        return Jet(self.a / o, self.v / o)

    def __rtruediv__(self, o):
        return Jet(o) / self


def jsqrt(x):
    s = np.sqrt(x.a)
    return Jet(s, x.v * (1.0 / (2.0 * s)))


def jcos(x):
    return Jet(np.cos(x.a), -np.sin(x.a) * x.v)


def jsin(x):
    return Jet(np.sin(x.a), np.cos(x.a) * x.v)


def angle_axis_rotate_point(aa, pt):
    """ceres/rotation.h AngleAxisRotatePoint (jets in aa, constants in pt)."""
    theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2]
    if theta2.a > EPS:
        theta = jsqrt(theta2)
        costheta, sintheta = jcos(theta), jsin(theta)
        theta_inverse = 1.0 / theta
        w = [aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse]
        wx = [w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]]
        tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (1.0 - costheta)
        return [pt[i] * costheta + wx[i] * sintheta + w[i] * tmp for i in range(3)]
    wx = [aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]]
    return [wx[i] + pt[i] for i in range(3)]


def residual_jets(x, p2, p3, w, K):
    """uncertainty_pnp.cpp:17-33 with the pose as Jet<6>: -> (r [2], J [2, 6])."""
    pose = [Jet(x[k], np.eye(6)[k].copy()) for k in range(6)]
    tp = angle_axis_rotate_point(pose[:3], p3)
    tp = [tp[0] + pose[3], tp[1] + pose[4], tp[2] + pose[5]]
    fx, fy, px, py = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    proj_x = fx * tp[0] / tp[2] + px
    proj_y = fy * tp[1] / tp[2] + py
    dx, dy = proj_x - p2[0], proj_y - p2[1]
    r0 = w[0] * dx + w[1] * dy
    r1 = w[1] * dx + w[2] * dy
    return np.array([r0.a, r1.a]), np.stack([r0.v, r1.v])


def evaluate(x, pts2d, pts3d, wgt, K, jac=True):
    with np.errstate(all="ignore"):
        return _evaluate(x, pts2d, pts3d, wgt, K, jac)


def _evaluate(x, pts2d, pts3d, wgt, K, jac):
    r, J = [], []
    for i in range(pts2d.shape[0]):
        ri, Ji = residual_jets(x, pts2d[i], pts3d[i], wgt[i], K)
        r.append(ri)
        J.append(Ji)
    r = np.concatenate(r)
    return 0.5 * float(r @ r), r, (np.concatenate(J) if jac else None)


# ---------------------------------------------------------------- Ceres 2.0 LM (restated)
def ceres_lm(x0, pts2d, pts3d, wgt, K, max_iter=50, diag=None):
    """TrustRegionMinimizer + LevenbergMarquardtStrategy with the default
    Solver::Options (see the module docstring); returns the final x (6)."""
    x = np.array(x0, np.float64)
    cost, r, J = evaluate(x, pts2d, pts3d, wgt, K)
    if not np.isfinite(cost):            # (e.g. the zero pose after a failed P3P): nothing to minimise
        if diag is not None:
            diag.update(iterations=0, cost=cost, status="max_iterations")
        return x
    scale = 1.0 / (1.0 + np.sqrt((J * J).sum(0)))          # jacobi scaling, fixed at iteration 0
    radius, decrease = 1e4, 2.0
    it = 0
    status = "max_iterations"
    while True:
        g = J.T @ r
        if np.max(np.abs(g)) <= 1e-10:
            status = "gradient"
            break
        if it >= max_iter:
            break
        it += 1
        Js = J * scale
        d = np.clip((Js * Js).sum(0), 1e-6, 1e32)
        A = Js.T @ Js + np.diag(d / radius)
        try:
            L = np.linalg.cholesky(A)
            step = -np.linalg.solve(L.T, np.linalg.solve(L, Js.T @ r))
            ok = np.all(np.isfinite(step))
        except np.linalg.LinAlgError:
            ok = False
        if not ok:
            radius /= decrease
            decrease *= 2.0
            if radius < 1e-32:
                status = "radius"
                break
            continue
        mr = Js @ step
        model_change = -float(mr @ (r + mr / 2.0))
        delta = step * scale
        if np.linalg.norm(delta) <= 1e-8 * (np.linalg.norm(x) + 1e-8):
            status = "parameter"
            break
        xc = x + delta
        cc, rc, _ = evaluate(xc, pts2d, pts3d, wgt, K, jac=False)
        if np.isfinite(cc) and abs(cost - cc) <= 1e-6 * cost:
            status = "function"
            break
        rho = (cost - cc) / model_change if (np.isfinite(cc) and model_change > 0) else -np.inf
        if rho > 1e-3:
            x = xc
            cost, r, J = evaluate(x, pts2d, pts3d, wgt, K)
            radius = min(1e16, radius / max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3))
            decrease = 2.0
        else:
            radius /= decrease
            decrease *= 2.0
            if radius < 1e-32:
                status = "radius"
                break
    if diag is not None:
        diag.update(iterations=it, cost=cost, status=status)
    return x


# ---------------------------------------------------------------- the wrappers
def _rt(rvec, t):
    return np.concatenate([rodrigues_vec_to_mat(rvec), np.asarray(t, np.float64).reshape(3, 1)], 1)


def pnp_from_weights(points_2d, weights_2d, points_3d, K, order_key, diag=None):
    pn = points_2d.shape[0]
    assert points_3d.shape[0] == pn and pn >= 4
    p2 = np.asarray(points_2d, np.float64)
    p3 = np.asarray(points_3d, np.float64)
    w = np.asarray(weights_2d, np.float64)
    K = np.asarray(K, np.float64)
    # argsort(...)[-4:]: ascending, the four largest; ties by index (stable)
    idxs = np.argsort(order_key, kind="stable")[-4:]
    ok, rvec, t = p3p_pose(p3[idxs], p2[idxs], K)
    if diag is not None:
        diag.update(p3p_ok=ok, init=np.concatenate([rvec, t]), idxs=idxs)
    if pn == 4:
        return _rt(rvec, t)
    x = ceres_lm(np.concatenate([rvec, t]), p2, p3, w, K, diag=diag)
    return _rt(x[:3], x[3:])


def uncertainty_pnp(points_2d, weights_2d, points_3d, camera_matrix, diag=None):
    """extend_utils.py:63-114 -> Rt [3, 4]."""
    w = np.asarray(weights_2d, np.float64)
    return pnp_from_weights(points_2d, w, points_3d, camera_matrix, w[:, 0] + w[:, 1], diag)


def uncertainty_pnp_v2(points_2d, covars, points_3d, camera_matrix, diag=None):
    """extend_utils.py:116-166 -> Rt [3, 4]."""
    w = weights_v2(covars)
    return pnp_from_weights(points_2d, w, points_3d, camera_matrix, w[:, 0], diag)
