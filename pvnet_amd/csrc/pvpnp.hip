// pvpnp.hip -- MI355X (gfx950) batched uncertainty-weighted PnP, the stage
// after the voting: EVD covariances -> weights -> P3P initial pose -> the
// weighted reprojection least squares.  Exported through include/pvvote.h.
//
// Reference (kennege/pvnet):
//   EU  lib/utils/extend_utils/extend_utils.py        (uncertainty_pnp[_v2], :63-166)
//   UP  lib/utils/extend_utils/src/uncertainty_pnp.cpp (cost functor + Ceres solve, :7-92)
//   EV  lib/utils/evaluation_utils.py                 (weights from covariances, :168-178)
// Third-party algorithms restated (absent from the image; DESIGN.md "PnP"):
//   OpenCV SOLVEPNP_P3P (candidates from points 0..2, point 3 picks),
//   cv2.Rodrigues, Ceres 2.0 AngleAxisRotatePoint / Jet autodiff /
//   TrustRegionMinimizer + LevenbergMarquardtStrategy with default options.
//
// Layout: one wave (one 64-thread block) per image, lane = model point
// (pn <= 64).  Residuals and Jacobians are per lane (forward-mode jets, as
// Ceres' AutoDiffCostFunction evaluates them); J^T J, J^T r and the cost are
// column sums over the lanes through LDS; the 6x6 trust-region solve runs
// redundantly in every lane (uniform values, no divergence).  All fp64, as the
// reference.  The P3P initial pose runs in lane 0 (a few hundred flops).
#include <hip/hip_runtime.h>

#include <float.h>
#include <math.h>
#include <stdint.h>

#include "../../include/pvvote.h"

namespace {

constexpr int kMaxPts = 64;
constexpr int kSums = 28;   // 21 (upper J^T J) + 6 (J^T r) + 1 (r^T r)

// ---------------------------------------------------------------- jets
// Ceres' Jet<double, 6>: value + derivative w.r.t. the 6 pose parameters.
struct Jet {
    double a;
    double v[6];
};
__device__ __forceinline__ Jet jconst(double a) {
    Jet r;
    r.a = a;
    for (int k = 0; k < 6; ++k) r.v[k] = 0.0;
    return r;
}
__device__ __forceinline__ Jet operator+(const Jet &x, const Jet &y) {
    Jet r;
    r.a = x.a + y.a;
    for (int k = 0; k < 6; ++k) r.v[k] = x.v[k] + y.v[k];
    return r;
}
__device__ __forceinline__ Jet operator-(const Jet &x, const Jet &y) {
    Jet r;
    r.a = x.a - y.a;
    for (int k = 0; k < 6; ++k) r.v[k] = x.v[k] - y.v[k];
    return r;
}
__device__ __forceinline__ Jet operator*(const Jet &x, const Jet &y) {
    Jet r;
    r.a = x.a * y.a;
    for (int k = 0; k < 6; ++k) r.v[k] = x.a * y.v[k] + x.v[k] * y.a;
    return r;
}
__device__ __forceinline__ Jet operator*(const Jet &x, double s) {
    Jet r;
    r.a = x.a * s;
    for (int k = 0; k < 6; ++k) r.v[k] = x.v[k] * s;
    return r;
}
__device__ __forceinline__ Jet operator*(double s, const Jet &x) { return x * s; }
__device__ __forceinline__ Jet operator+(const Jet &x, double s) {
    Jet r = x;
    r.a = x.a + s;
    return r;
}
__device__ __forceinline__ Jet operator-(const Jet &x, double s) {
    Jet r = x;
    r.a = x.a - s;
    return r;
}
__device__ __forceinline__ Jet operator-(double s, const Jet &x) {
    Jet r;
    r.a = s - x.a;
    for (int k = 0; k < 6; ++k) r.v[k] = -x.v[k];
    return r;
}
// Ceres: f / g = (f.a / g.a, (f.v - (f.a / g.a) g.v) / g.a)
__device__ __forceinline__ Jet operator/(const Jet &f, const Jet &g) {
    const double inv = 1.0 / g.a, fg = f.a * inv;
    Jet r;
    r.a = f.a * inv;
    for (int k = 0; k < 6; ++k) r.v[k] = (f.v[k] - fg * g.v[k]) * inv;
    return r;
}
__device__ __forceinline__ Jet operator/(double s, const Jet &g) { return jconst(s) / g; }
__device__ __forceinline__ Jet jsqrt(const Jet &x) {
    const double s = sqrt(x.a), d = 1.0 / (2.0 * s);
    Jet r;
    r.a = s;
    for (int k = 0; k < 6; ++k) r.v[k] = x.v[k] * d;
    return r;
}
__device__ __forceinline__ Jet jcos(const Jet &x) {
    const double s = -sin(x.a);
    Jet r;
    r.a = cos(x.a);
    for (int k = 0; k < 6; ++k) r.v[k] = s * x.v[k];
    return r;
}
__device__ __forceinline__ Jet jsin(const Jet &x) {
    const double c = cos(x.a);
    Jet r;
    r.a = sin(x.a);
    for (int k = 0; k < 6; ++k) r.v[k] = c * x.v[k];
    return r;
}
// plain doubles through the same code
__device__ __forceinline__ double jsqrt(double x) { return sqrt(x); }
__device__ __forceinline__ double jcos(double x) { return cos(x); }
__device__ __forceinline__ double jsin(double x) { return sin(x); }
__device__ __forceinline__ double val(double x) { return x; }
__device__ __forceinline__ double val(const Jet &x) { return x.a; }

// ceres/rotation.h AngleAxisRotatePoint (pose T, point constants)
template <typename T>
__device__ __forceinline__ void angle_axis_rotate_point(const T aa[3], const double pt[3], T out[3]) {
    const T theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
    if (val(theta2) > DBL_EPSILON) {
        const T theta = jsqrt(theta2);
        const T costheta = jcos(theta), sintheta = jsin(theta);
        const T theta_inverse = 1.0 / theta;
        const T w[3] = {aa[0] * theta_inverse, aa[1] * theta_inverse, aa[2] * theta_inverse};
        const T wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2], w[0] * pt[1] - w[1] * pt[0]};
        const T tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (1.0 - costheta);
        for (int i = 0; i < 3; ++i) out[i] = pt[i] * costheta + wx[i] * sintheta + w[i] * tmp;
    } else {
        const T wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2], aa[0] * pt[1] - aa[1] * pt[0]};
        for (int i = 0; i < 3; ++i) out[i] = wx[i] + pt[i];
    }
}

// UP:17-33, ReprojectionErrorArray::operator()
struct PointData {
    double x2d, y2d, x3d, y3d, z3d, wxx, wxy, wyy;
};
struct Cam {
    double fx, fy, px, py;
};
template <typename T>
__device__ __forceinline__ void residual(const T pose[6], const PointData &p, const Cam &c, T res[2]) {
    const double pts3d[3] = {p.x3d, p.y3d, p.z3d};
    T t3[3];
    angle_axis_rotate_point(pose, pts3d, t3);
    t3[0] = t3[0] + pose[3];
    t3[1] = t3[1] + pose[4];
    t3[2] = t3[2] + pose[5];
    const T proj_x = c.fx * t3[0] / t3[2] + c.px;
    const T proj_y = c.fy * t3[1] / t3[2] + c.py;
    const T dx = proj_x - p.x2d, dy = proj_y - p.y2d;
    res[0] = p.wxx * dx + p.wxy * dy;
    res[1] = p.wxy * dx + p.wyy * dy;
}
// ---------------------------------------------------------------- weights (EV:168-178, EU:131-139)
__device__ __forceinline__ void weights_from_cov(const float *c4, int mode, double w[3]) {
    const double c00 = c4[0], c01 = c4[1], c10 = c4[2], c11 = c4[3];
    w[0] = w[1] = w[2] = 0.0;
    if (mode == PV_PNP_COV) {
        // inv(sqrtm(C)), sqrtm(C) = (C + s I) / t, s = sqrt(det C), t = sqrt(tr C + 2 s)
        if (c00 < 1e-6 || c00 != c00 || c01 != c01 || c10 != c10 || c11 != c11) return;
        const double s = sqrt(fmax(c00 * c11 - c01 * c10, 0.0));
        const double t = sqrt(c00 + c11 + 2.0 * s);
        const double a = (c00 + s) / t, b = c01 / t, cc = c10 / t, d = (c11 + s) / t;
        const double det = a * d - b * cc;
        w[0] = d / det;
        w[1] = -b / det;
        w[2] = a / det;
    } else {
        // 1 / max eigenvalue of the symmetric 2x2
        if (!(c00 >= 1e-5)) return;
        const double m = 0.5 * (c00 + c11), q = sqrt(0.25 * (c00 - c11) * (c00 - c11) + c01 * c10);
        const double lam = m + q;
        w[0] = w[2] = 1.0 / lam;
    }
}

// ---------------------------------------------------------------- small dense algebra
__device__ __forceinline__ void cross3(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ double norm3(const double a[3]) { return sqrt(dot3(a, a)); }

// orthonormal frame of a triangle (columns e1, e3 x e1, e3); false if degenerate
__device__ bool tri_frame(const double X[3][3], double F[3][3]) {
    double e1[3] = {X[1][0] - X[0][0], X[1][1] - X[0][1], X[1][2] - X[0][2]};
    const double e2r[3] = {X[2][0] - X[0][0], X[2][1] - X[0][1], X[2][2] - X[0][2]};
    double e3[3];
    cross3(e1, e2r, e3);
    const double n1 = norm3(e1), n3 = norm3(e3);
    if (n1 == 0.0 || n3 == 0.0) return false;
    for (int i = 0; i < 3; ++i) { e1[i] /= n1; e3[i] /= n3; }
    double e2[3];
    cross3(e3, e1, e2);
    for (int i = 0; i < 3; ++i) { F[i][0] = e1[i]; F[i][1] = e2[i]; F[i][2] = e3[i]; }
    return true;
}

// cv2.Rodrigues(rvec) -> R
__device__ void rodrigues_to_mat(const double r[3], double R[3][3]) {
    const double th = sqrt(dot3(r, r));
    if (th < DBL_EPSILON) {
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) R[i][j] = i == j ? 1.0 : 0.0;
        return;
    }
    const double k[3] = {r[0] / th, r[1] / th, r[2] / th};
    const double c = cos(th), s = sin(th);
    const double kx[3][3] = {{0.0, -k[2], k[1]}, {k[2], 0.0, -k[0]}, {-k[1], k[0], 0.0}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = (i == j ? c : 0.0) + (1.0 - c) * k[i] * k[j] + s * kx[i][j];
}

// cv2.Rodrigues(R) -> rvec (orthonormal R; theta ~ pi from R = 2 k k^T - I)
__device__ void rodrigues_to_vec(const double R[3][3], double r[3]) {
    double rx = R[2][1] - R[1][2], ry = R[0][2] - R[2][0], rz = R[1][0] - R[0][1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    const double c = fmin(fmax((R[0][0] + R[1][1] + R[2][2] - 1.0) * 0.5, -1.0), 1.0);
    const double th = acos(c);
    if (s < 1e-5) {
        if (c > 0) { r[0] = r[1] = r[2] = 0.0; return; }
        int m = 0;
        if (R[1][1] > R[m][m]) m = 1;
        if (R[2][2] > R[m][m]) m = 2;
        double k[3];
        k[m] = sqrt(fmax((R[m][m] + 1.0) * 0.5, 0.0));
        for (int i = 0; i < 3; ++i)
            if (i != m) k[i] = (R[m][i] + R[i][m]) * 0.25 / k[m];
        const double n = sqrt(dot3(k, k));
        for (int i = 0; i < 3; ++i) r[i] = k[i] / n * th;
        return;
    }
    const double vth = 1.0 / (2.0 * s) * th;
    r[0] = rx * vth;
    r[1] = ry * vth;
    r[2] = rz * vth;
}

// ---------------------------------------------------------------- polynomial roots
__device__ double polish(const double *a, int deg, double x) {   // a[0] x^deg + ... (Newton, 3 steps)
    for (int it = 0; it < 3; ++it) {
        double p = a[0], dp = 0.0;
        for (int i = 1; i <= deg; ++i) { dp = dp * x + p; p = p * x + a[i]; }
        if (dp == 0.0 || !isfinite(p / dp)) break;
        x -= p / dp;
    }
    return x;
}

// the largest real root of m^3 + B m^2 + C m + D
__device__ double cubic_largest(double B, double C, double D) {
    const double P = C - B * B / 3.0, Q = 2.0 * B * B * B / 27.0 - B * C / 3.0 + D;
    const double disc = 0.25 * Q * Q + P * P * P / 27.0;
    double t;
    if (disc > 0.0) {
        const double sq = sqrt(disc);
        t = cbrt(-0.5 * Q + sq) + cbrt(-0.5 * Q - sq);
    } else if (P == 0.0) {
        t = cbrt(-Q);
    } else {
        const double rr = sqrt(-P / 3.0);
        const double arg = fmin(fmax(-0.5 * Q / (rr * rr * rr), -1.0), 1.0);
        t = 2.0 * rr * cos(acos(arg) / 3.0);
    }
    const double a[4] = {1.0, B, C, D};
    return polish(a, 3, t - B / 3.0);
}

// real roots of a4 x^4 + a3 x^3 + a2 x^2 + a1 x + a0 (Ferrari: the resolvent
// cubic's largest root splits the depressed quartic into two quadratics),
// each polished by Newton steps on the original polynomial
__device__ int quartic_real_roots(const double a[5], double out[4]) {
    if (a[0] == 0.0) return 0;
    const double b = a[1] / a[0], c = a[2] / a[0], d = a[3] / a[0], e = a[4] / a[0];
    const double b2 = b * b;
    const double p = c - 3.0 * b2 / 8.0;
    const double q = d - 0.5 * b * c + b2 * b / 8.0;
    const double r = e - 0.25 * b * d + b2 * c / 16.0 - 3.0 * b2 * b2 / 256.0;
    double y[4];
    int n = 0;
    auto quad = [&](double B1, double C1) {   // y^2 + B1 y + C1
        double disc = B1 * B1 - 4.0 * C1;
        const double tol = 1e-12 * fmax(1.0, B1 * B1 + fabs(C1));
        if (disc < 0.0 && disc > -tol) disc = 0.0;
        if (disc < 0.0) return;
        const double s = sqrt(disc);
        y[n++] = 0.5 * (-B1 + s);
        y[n++] = 0.5 * (-B1 - s);
    };
    const double scale = fmax(1.0, fmax(fabs(p), fmax(fabs(q), fabs(r))));
    if (fabs(q) <= 1e-14 * scale) {
        // biquadratic: z^2 + p z + r, y = +-sqrt(z)
        double z[2];
        double disc = p * p - 4.0 * r;
        if (disc < 0.0 && disc > -1e-12 * fmax(1.0, p * p)) disc = 0.0;
        if (disc >= 0.0) {
            const double s = sqrt(disc);
            z[0] = 0.5 * (-p + s);
            z[1] = 0.5 * (-p - s);
            for (int k = 0; k < 2; ++k) {
                if (z[k] >= 0.0) {
                    y[n++] = sqrt(z[k]);
                    y[n++] = -sqrt(z[k]);
                }
            }
        }
    } else {
        const double m = cubic_largest(p, 0.25 * p * p - r, -q * q / 8.0);
        if (m > 0.0) {
            const double s = sqrt(2.0 * m);
            quad(s, 0.5 * p + m - q / (2.0 * s));
            quad(-s, 0.5 * p + m + q / (2.0 * s));
        }
    }
    for (int k = 0; k < n; ++k) out[k] = polish(a, 4, y[k] - 0.25 * b);
    return n;
}

// ---------------------------------------------------------------- P3P (cv2 SOLVEPNP_P3P restated)
// World points P[4], image points x[4] (pixels): candidates from points
// 0..2 (Grunert's quartic, Haralick et al. 1994), the one reprojecting point 3
// closest wins.  Returns false if there is no candidate.
__device__ bool p3p_pose(const double P[4][3], const double x[4][2], const Cam &cam, double rvec[3],
                         double t[3]) {
    double j[4][3];
    for (int i = 0; i < 4; ++i) {
        const double mu = (x[i][0] - cam.px) / cam.fx, mv = (x[i][1] - cam.py) / cam.fy;
        const double nn = sqrt(mu * mu + mv * mv + 1.0);
        j[i][0] = mu / nn;
        j[i][1] = mv / nn;
        j[i][2] = 1.0 / nn;
    }
    double d12[3], d02[3], d01[3];
    for (int k = 0; k < 3; ++k) {
        d12[k] = P[1][k] - P[2][k];
        d02[k] = P[0][k] - P[2][k];
        d01[k] = P[0][k] - P[1][k];
    }
    const double a2 = dot3(d12, d12), b2 = dot3(d02, d02), c2 = dot3(d01, d01);
    if (b2 == 0.0) return false;
    const double ca = dot3(j[1], j[2]), cb = dot3(j[0], j[2]), cg = dot3(j[0], j[1]);
    const double amc = (a2 - c2) / b2, apc = (a2 + c2) / b2;
    double A[5];
    A[0] = (amc - 1.0) * (amc - 1.0) - 4.0 * c2 / b2 * ca * ca;
    A[1] = 4.0 * (amc * (1.0 - amc) * cb - (1.0 - apc) * ca * cg + 2.0 * c2 / b2 * ca * ca * cb);
    A[2] = 2.0 * (amc * amc - 1.0 + 2.0 * amc * amc * cb * cb + 2.0 * (b2 - c2) / b2 * ca * ca -
                  4.0 * apc * ca * cb * cg + 2.0 * (b2 - a2) / b2 * cg * cg);
    A[3] = 4.0 * (-amc * (1.0 + amc) * cb + 2.0 * a2 / b2 * cg * cg * cb - (1.0 - apc) * ca * cg);
    A[4] = (1.0 + amc) * (1.0 + amc) - 4.0 * a2 / b2 * cg * cg;
    double roots[4];
    const int nr = quartic_real_roots(A, roots);
    double FP[3][3];
    const double P3[3][3] = {{P[0][0], P[0][1], P[0][2]}, {P[1][0], P[1][1], P[1][2]}, {P[2][0], P[2][1], P[2][2]}};
    if (!tri_frame(P3, FP)) return false;
    bool found = false;
    double best = 0.0;
    for (int k = 0; k < nr; ++k) {
        const double v = roots[k];
        if (!(v > 0.0)) continue;
        const double den = 2.0 * (cg - v * ca);
        if (den == 0.0) continue;
        const double u = ((-1.0 + amc) * v * v - 2.0 * amc * cb * v + 1.0 + amc) / den;
        const double qq = 1.0 + v * v - 2.0 * v * cb;
        if (!(u > 0.0) || !(qq > 0.0)) continue;
        const double s1 = sqrt(b2 / qq), s2 = u * s1, s3 = v * s1;
        double C[3][3];
        for (int i = 0; i < 3; ++i) {
            C[0][i] = s1 * j[0][i];
            C[1][i] = s2 * j[1][i];
            C[2][i] = s3 * j[2][i];
        }
        double FC[3][3];
        if (!tri_frame(C, FC)) continue;
        double R[3][3];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) R[r][c] = FC[r][0] * FP[c][0] + FC[r][1] * FP[c][1] + FC[r][2] * FP[c][2];
        double tt[3];
        for (int r = 0; r < 3; ++r) tt[r] = C[0][r] - (R[r][0] * P[0][0] + R[r][1] * P[0][1] + R[r][2] * P[0][2]);
        double X[3];
        for (int r = 0; r < 3; ++r) X[r] = R[r][0] * P[3][0] + R[r][1] * P[3][1] + R[r][2] * P[3][2] + tt[r];
        if (X[2] == 0.0) continue;
        const double ex = cam.px + cam.fx * X[0] / X[2] - x[3][0], ey = cam.py + cam.fy * X[1] / X[2] - x[3][1];
        const double e = ex * ex + ey * ey;
        if (!found || e < best) {
            found = true;
            best = e;
            rodrigues_to_vec(R, rvec);
            for (int r = 0; r < 3; ++r) t[r] = tt[r];
        }
    }
    if (!found) {
        rvec[0] = rvec[1] = rvec[2] = 0.0;
        t[0] = t[1] = t[2] = 0.0;
    }
    return found;
}

// ---------------------------------------------------------------- the trust-region LM (Ceres 2.0, restated)
struct Shared {
    double part[kMaxPts][kSums + 1];   // per-lane contributions (+1: no bank-aligned rows)
    double sums[kSums];
    double cost_part[kMaxPts];
    double cost;
    double x0[6];                      // initial pose (lane 0 -> all)
    int ok;
    int sel[4];
};

// column sums of part[0..pn) -> sums (lanes 0..27), then visible to the wave
__device__ __forceinline__ void reduce_sums(Shared &S, int pn) {
    const int lane = threadIdx.x;
    __syncthreads();
    if (lane < kSums) {
        double s = 0.0;
        for (int i = 0; i < pn; ++i) s += S.part[i][lane];
        S.sums[lane] = s;
    }
    __syncthreads();
}
__device__ __forceinline__ double reduce_cost(Shared &S, int pn) {
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int i = 0; i < pn; ++i) s += S.cost_part[i];
        S.cost = 0.5 * s;
    }
    __syncthreads();
    return S.cost;
}

// evaluate at x: cost, g = J^T r, H = J^T J (6x6, full) -- every lane gets them
__device__ void eval_full(Shared &S, const PointData &pd, const Cam &cam, bool active, int pn, const double x[6],
                          double *cost, double H[6][6], double g[6]) {
    const int lane = threadIdx.x;
    if (active) {
        Jet pose[6];
        for (int k = 0; k < 6; ++k) {
            pose[k] = jconst(x[k]);
            pose[k].v[k] = 1.0;
        }
        Jet r[2];
        residual(pose, pd, cam, r);
        int q = 0;
        for (int i = 0; i < 6; ++i)
            for (int jj = i; jj < 6; ++jj) S.part[lane][q++] = r[0].v[i] * r[0].v[jj] + r[1].v[i] * r[1].v[jj];
        for (int i = 0; i < 6; ++i) S.part[lane][21 + i] = r[0].v[i] * r[0].a + r[1].v[i] * r[1].a;
        S.part[lane][27] = r[0].a * r[0].a + r[1].a * r[1].a;
    }
    reduce_sums(S, pn);
    int q = 0;
    for (int i = 0; i < 6; ++i)
        for (int jj = i; jj < 6; ++jj) { H[i][jj] = S.sums[q]; H[jj][i] = S.sums[q]; ++q; }
    for (int i = 0; i < 6; ++i) g[i] = S.sums[21 + i];
    *cost = 0.5 * S.sums[27];
}

__device__ double eval_cost(Shared &S, const PointData &pd, const Cam &cam, bool active, int pn, const double x[6]) {
    if (active) {
        double r[2];
        residual(x, pd, cam, r);
        S.cost_part[threadIdx.x] = r[0] * r[0] + r[1] * r[1];
    }
    return reduce_cost(S, pn);
}

// Cholesky solve of the SPD 6x6 A y = b; false if not positive definite
__device__ bool chol_solve6(double A[6][6], const double b[6], double y[6]) {
    double L[6][6];
    for (int i = 0; i < 6; ++i) {
        for (int jj = 0; jj <= i; ++jj) {
            double s = A[i][jj];
            for (int k = 0; k < jj; ++k) s -= L[i][k] * L[jj][k];
            if (i == jj) {
                if (!(s > 0.0)) return false;
                L[i][i] = sqrt(s);
            } else {
                L[i][jj] = s / L[jj][jj];
            }
        }
    }
    double z[6];
    for (int i = 0; i < 6; ++i) {
        double s = b[i];
        for (int k = 0; k < i; ++k) s -= L[i][k] * z[k];
        z[i] = s / L[i][i];
    }
    for (int i = 5; i >= 0; --i) {
        double s = z[i];
        for (int k = i + 1; k < 6; ++k) s -= L[k][i] * y[k];
        y[i] = s / L[i][i];
    }
    for (int i = 0; i < 6; ++i)
        if (!isfinite(y[i])) return false;
    return true;
}

// TrustRegionMinimizer::Minimize with LevenbergMarquardtStrategy, default
// Solver::Options (see the header comment); x in/out, returns the status
__device__ int trust_region_lm(Shared &S, const PointData &pd, const Cam &cam, bool active, int pn, double x[6],
                               int *iters, double *final_cost) {
    double cost, H[6][6], g[6];
    eval_full(S, pd, cam, active, pn, x, &cost, H, g);
    *iters = 0;
    *final_cost = cost;
    if (!isfinite(cost)) return PV_PNP_STOP_MAX_ITER;
    double scale[6];
    for (int i = 0; i < 6; ++i) scale[i] = 1.0 / (1.0 + sqrt(H[i][i]));   // jacobi scaling, fixed at iteration 0
    double radius = 1e4, decrease = 2.0;
    int it = 0;
    int status = PV_PNP_STOP_MAX_ITER;
    for (;;) {
        double gmax = 0.0;
        for (int i = 0; i < 6; ++i) gmax = fmax(gmax, fabs(g[i]));
        if (gmax <= 1e-10) { status = PV_PNP_STOP_GRADIENT; break; }
        if (it >= 50) break;
        ++it;
        // scaled system: (S H S + diag(clamp(s_j^2 H_jj) / radius)) step = -S g
        double A[6][6], rhs[6], step[6];
        for (int i = 0; i < 6; ++i) {
            for (int jj = 0; jj < 6; ++jj) A[i][jj] = scale[i] * H[i][jj] * scale[jj];
            const double dg = fmin(fmax(A[i][i], 1e-6), 1e32);
            A[i][i] += dg / radius;
            rhs[i] = -scale[i] * g[i];
        }
        if (!chol_solve6(A, rhs, step)) {
            radius /= decrease;
            decrease *= 2.0;
            if (radius < 1e-32) { status = PV_PNP_STOP_RADIUS; break; }
            continue;
        }
        // model cost change -(Js step)^T (r + Js step / 2) = -(step^T S g + step^T S H S step / 2)
        double sg = 0.0, shs = 0.0;
        for (int i = 0; i < 6; ++i) {
            sg += step[i] * scale[i] * g[i];
            double hs = 0.0;
            for (int jj = 0; jj < 6; ++jj) hs += scale[i] * H[i][jj] * scale[jj] * step[jj];
            shs += step[i] * hs;
        }
        const double model_change = -(sg + 0.5 * shs);
        double delta[6], xc[6], dn = 0.0, xn = 0.0;
        for (int i = 0; i < 6; ++i) {
            delta[i] = step[i] * scale[i];
            xc[i] = x[i] + delta[i];
            dn += delta[i] * delta[i];
            xn += x[i] * x[i];
        }
        if (sqrt(dn) <= 1e-8 * (sqrt(xn) + 1e-8)) { status = PV_PNP_STOP_PARAMETER; break; }
        const double cc = eval_cost(S, pd, cam, active, pn, xc);
        if (isfinite(cc) && fabs(cost - cc) <= 1e-6 * cost) { status = PV_PNP_STOP_FUNCTION; break; }
        const double rho = (isfinite(cc) && model_change > 0.0) ? (cost - cc) / model_change : -INFINITY;
        if (rho > 1e-3) {
            for (int i = 0; i < 6; ++i) x[i] = xc[i];
            eval_full(S, pd, cam, active, pn, x, &cost, H, g);
            const double q = 2.0 * rho - 1.0;
            radius = fmin(1e16, radius / fmax(1.0 / 3.0, 1.0 - q * q * q));
            decrease = 2.0;
        } else {
            radius /= decrease;
            decrease *= 2.0;
            if (radius < 1e-32) { status = PV_PNP_STOP_RADIUS; break; }
        }
    }
    *iters = it;
    *final_cost = cost;
    return status;
}

// ordering key of point i (EU:84 wxx + wxy, EU:146 the v2 weight); NaN sorts last
__device__ __forceinline__ bool key_less(double a, double b) {
    if (a != a) return false;
    if (b != b) return true;
    return a < b;
}

// One block (64 threads) per image.
__global__ __launch_bounds__(64) void k_uncertainty_pnp(pv_pnp_batch bt, const double *init_rt, double *Rt,
                                                         double *result_rt, pv_pnp_diag dg) {
    __shared__ Shared S;
    const int img = blockIdx.x, lane = threadIdx.x, pn = bt.pn;
    const bool active = lane < pn;
    const double *K = bt.K + (int64_t)img * bt.K_stride;
    const Cam cam{K[0], K[4], K[2], K[5]};
    const double *P3 = bt.pts3d + (int64_t)img * bt.pts3d_stride;
    PointData pd{};
    double key = 0.0;
    if (active) {
        const int64_t pi = (int64_t)img * pn + lane;
        pd.x2d = bt.pts2d64 ? bt.pts2d64[pi * 2] : (double)bt.pts2d[pi * 2];
        pd.y2d = bt.pts2d64 ? bt.pts2d64[pi * 2 + 1] : (double)bt.pts2d[pi * 2 + 1];
        pd.x3d = P3[lane * 3];
        pd.y3d = P3[lane * 3 + 1];
        pd.z3d = P3[lane * 3 + 2];
        double w[3];
        if (bt.mode == PV_PNP_WEIGHTS) {
            const double *wp = (const double *)bt.wgt + pi * 3;
            w[0] = wp[0]; w[1] = wp[1]; w[2] = wp[2];
        } else {
            weights_from_cov((const float *)bt.wgt + pi * 4, bt.mode, w);
        }
        pd.wxx = w[0]; pd.wxy = w[1]; pd.wyy = w[2];
        key = bt.mode == PV_PNP_COV_V2 ? w[0] : w[0] + w[1];
    }
    double x[6];
    int p3p_ok = 1;
    if (init_rt) {
        for (int k = 0; k < 6; ++k) x[k] = init_rt[(int64_t)img * 6 + k];
    } else {
        // the four highest keys in ascending order, ties by index: np.argsort(key, kind="stable")[-4:]
        S.part[lane][0] = key;
        __syncthreads();
        if (active) {
            int pos = 0;
            for (int jj = 0; jj < pn; ++jj) {
                const double kj = S.part[jj][0];
                pos += key_less(kj, key) || (jj < lane && !key_less(key, kj) && !key_less(kj, key)) ? 1 : 0;
            }
            if (pos >= pn - 4) S.sel[pos - (pn - 4)] = lane;
        }
        __syncthreads();
        if (lane == 0) {
            double P[4][3], xx[4][2];
            for (int k = 0; k < 4; ++k) {
                const int s = S.sel[k];
                for (int c = 0; c < 3; ++c) P[k][c] = P3[s * 3 + c];
                const int64_t o = ((int64_t)img * pn + s) * 2;
                xx[k][0] = bt.pts2d64 ? bt.pts2d64[o] : (double)bt.pts2d[o];
                xx[k][1] = bt.pts2d64 ? bt.pts2d64[o + 1] : (double)bt.pts2d[o + 1];
            }
            double rv[3], tt[3];
            S.ok = p3p_pose(P, xx, cam, rv, tt) ? 1 : 0;
            for (int k = 0; k < 3; ++k) { S.x0[k] = rv[k]; S.x0[3 + k] = tt[k]; }
        }
        __syncthreads();
        for (int k = 0; k < 6; ++k) x[k] = S.x0[k];
        p3p_ok = S.ok;
    }
    int iters = 0, status = PV_PNP_STOP_P3P_ONLY;
    double cost = 0.0;
    if (dg.init_rt && lane < 6) dg.init_rt[(int64_t)img * 6 + lane] = x[lane];
    if (init_rt || pn > 4) {
        status = trust_region_lm(S, pd, cam, active, pn, x, &iters, &cost);
    } else {
        cost = eval_cost(S, pd, cam, active, pn, x);
    }
    if (lane == 0) {
        if (result_rt)
            for (int k = 0; k < 6; ++k) result_rt[(int64_t)img * 6 + k] = x[k];
        if (Rt) {
            double R[3][3];
            rodrigues_to_mat(x, R);
            double *o = Rt + (int64_t)img * 12;
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) o[r * 4 + c] = R[r][c];
                o[r * 4 + 3] = x[3 + r];
            }
        }
        if (dg.p3p_ok) dg.p3p_ok[img] = p3p_ok;
        if (dg.iterations) dg.iterations[img] = iters;
        if (dg.status) dg.status[img] = status;
        if (dg.cost) dg.cost[img] = cost;
    }
}

int check_batch(const pv_pnp_batch *bt) {
    if (!bt || bt->b < 0 || bt->pn < 4 || bt->pn > kMaxPts) return PV_EINVAL;
    if (bt->mode != PV_PNP_WEIGHTS && bt->mode != PV_PNP_COV && bt->mode != PV_PNP_COV_V2) return PV_EINVAL;
    if (bt->b > 0 && ((!bt->pts2d && !bt->pts2d64) || !bt->wgt || !bt->pts3d || !bt->K)) return PV_EINVAL;
    if (bt->pts3d_stride < 0 || bt->K_stride < 0) return PV_EINVAL;
    return PV_OK;
}

}  // namespace

extern "C" {

int pv_uncertainty_pnp(const pv_pnp_batch *batch, double *Rt, const pv_pnp_diag *diag, pv_stream_t stream) {
    int r = check_batch(batch);
    if (r) return r;
    if (!Rt) return PV_EINVAL;
    if (batch->b == 0) return PV_OK;
    pv_pnp_diag dg{};
    if (diag) dg = *diag;
    k_uncertainty_pnp<<<batch->b, 64, 0, (hipStream_t)stream>>>(*batch, nullptr, Rt, nullptr, dg);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

int pv_uncertainty_pnp_refine(const pv_pnp_batch *batch, const double *init_rt, double *result_rt,
                              const pv_pnp_diag *diag, pv_stream_t stream) {
    int r = check_batch(batch);
    if (r) return r;
    if (!init_rt || !result_rt || batch->mode != PV_PNP_WEIGHTS) return PV_EINVAL;
    if (batch->b == 0) return PV_OK;
    pv_pnp_diag dg{};
    if (diag) dg = *diag;
    k_uncertainty_pnp<<<batch->b, 64, 0, (hipStream_t)stream>>>(*batch, init_rt, nullptr, result_rt, dg);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? PV_OK : (int)e;
}

}  // extern "C"
