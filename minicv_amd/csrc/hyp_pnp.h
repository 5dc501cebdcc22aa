// hyp_pnp.h — per-hypothesis code of the PnP-RANSAC path behind
// cvSolvePnPRansac / cvSolvePnP / solveAp3p (MiniCVNative.cpp:48-139, ap3p.cpp:282-317).
// Compiled for gfx950 (ransac_pnp.hip) and for the host (mcvHostPnP* test hooks) with
// -ffp-contract=off: +,-,*,/ and sqrt round identically on both sides.
//
// Restated behaviour:
//  * AP3P (Ke & Roumeliotis, CVPR 2017) exactly as the reference's computePoses
//    (ap3p.cpp:123-255): bearing vectors, the f1i / f2i / g1..g7 terms, the quartic in
//    cos(theta1'), C13, R = Ck1nl C13 Cb1k3tz^T, t = sin(theta1') b3' - R^T w3. The quartic by the
//    reference's own solveQuartic (Ferrari through complex arithmetic) + polishQuarticRoots
//    (ap3p.cpp:10-77), real parts of complex roots kept as candidates — the RANSAC default; its
//    transcendentals are the device's (ocml) on the GPU and glibc's on the host, so a root can
//    differ in its last bits between the two. MCV_FLAG_FAST_MINIMAL: the real roots
//    from e_poly_real_roots (derivative-interval bisection, bit-identical host / GPU).
//  * Camera-from-world rotation of a solution is R^T (OpenCV's ap3p stores the transpose;
//    the reference's solveAp3p export returns R itself, ap3p.cpp:245-250 — kept for that export).
//  * OpenCV 4.x solvePnPRansac / PnPRansacCallback [ext]: 4-point minimal sets for P3P / AP3P
//    (the first three solve, the fourth picks the solution of least reprojection error), image
//    points undistorted first (undistortPoints, 5 fixed iterations), error = squared pixel
//    distance between the observed point and projectPoints (k1, k2, p1, p2 model, fp64 inside,
//    fp32 output), inlier iff err <= (float)thr^2 (thr is a float: the reference's
//    reprojectionError argument).
#pragma once

#include "mcv_common.h"
#include "hyp_essential.h"   // e_poly_real_roots
#include "epnp.h"   // EPnP; kDblMin
#include "glibc_math.h"   // glibc's cbrt / hypot / clog branches (the reference's libm)

namespace mcv {

static const int kPnpMaxSolutions = 4;
static const int kUndistortIters = 5;

// Camera: K (fx, fy, cx, cy; skew ignored as projectPoints does) + distortion (k1, k2, p1, p2).
struct PnpCamera { double fx, fy, cx, cy, k1, k2, p1, p2; };

// Pose: X_cam = R X_world + t (row-major R).
struct PnpPose { double R[9]; double t[3]; };

// undistortPoints (OpenCV cvUndistortPointsInternal, fixed 5 iterations) -> normalised (x, y);
// x0 = (u - cx) * (1 / fx) as that function scales by ifx = 1./fx.
MCV_HD void pnp_undistort(const PnpCamera& c, double u, double v, double& x, double& y) {
    const double ifx = 1. / c.fx, ify = 1. / c.fy;
    const double x0 = (u - c.cx) * ifx, y0 = (v - c.cy) * ify;
    x = x0;
    y = y0;
    for (int it = 0; it < kUndistortIters; ++it) {
        const double r2 = x * x + y * y;
        const double icdist = 1.0 / (1.0 + (c.k2 * r2 + c.k1) * r2);
        if (icdist < 0) { x = x0; y = y0; break; }
        const double dx = 2.0 * c.p1 * x * y + c.p2 * (r2 + 2.0 * x * x);
        const double dy = c.p1 * (r2 + 2.0 * y * y) + 2.0 * c.p2 * x * y;
        x = (x0 - dx) * icdist;
        y = (y0 - dy) * icdist;
    }
}

// projectPoints for one point (k1, k2, p1, p2): pixel (u, v) in fp64, returned as float like the
// CV_32F projpoints of PnPRansacCallback::computeError. Returns false if Zc == 0 (OpenCV then
// divides by 1; here the point is an outlier).
MCV_HD void pnp_project(const PnpCamera& c, const double* R, const double* t, double X, double Y, double Z,
                        double& u, double& v) {
    const double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    const double Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    const double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
#if defined(__HIP_DEVICE_COMPILE__)
    // 1 / Zc bit for bit for |Zc| in [2^-64, 2^64]: the refined reciprocal followed by the quotient
    // correction of the IEEE sequence (div_f64_refined with n = 1, mcvTestDivF64 mode 1); the two
    // Newton steps alone are not a correctly rounded reciprocal for every significand
    double iz = div_f64_refined(1.0, Zc, rcp_f64_refined(Zc));
    if (!div_f64_refined_domain(Zc)) iz = 1.0 / (Zc != 0 ? Zc : 1.0);   // = (Zc != 0 ? 1 / Zc : 1)
#else
    const double iz = 1.0 / (Zc != 0 ? Zc : 1.0);   // = (Zc != 0 ? 1 / Zc : 1)
#endif
    const double x = Xc * iz, y = Yc * iz;
    const double r2 = x * x + y * y, r4 = r2 * r2;
    const double a1 = 2.0 * x * y, a2 = r2 + 2.0 * x * x, a3 = r2 + 2.0 * y * y;
    const double cdist = 1.0 + c.k1 * r2 + c.k2 * r4;
    const double xd = x * cdist + c.p1 * a1 + c.p2 * a2;
    const double yd = y * cdist + c.p1 * a3 + c.p2 * a1;
    u = xd * c.fx + c.cx;
    v = yd * c.fy + c.cy;
}

// Reprojection error: float observed point minus the float projection, squared norm in fp32
// (fused: fmaf(dx, dx, dy * dy); unfused: dx * dx + dy * dy).
MCV_HD float pnp_error(const PnpCamera& c, const double* R, const double* t, float X, float Y, float Z, float uo,
                       float vo, bool fused) {
    double u, v;
    pnp_project(c, R, t, X, Y, Z, u, v);
    const float dx = uo - (float)u, dy = vo - (float)v;
#if defined(__HIP_DEVICE_COMPILE__)
    return fused ? __builtin_fmaf(dx, dx, dy * dy) : dx * dx + dy * dy;
#else
    return fused ? fmaf(dx, dx, dy * dy) : dx * dx + dy * dy;
#endif
}

// ---- AP3P (reference computePoses, restated) --------------------------------------------------
MCV_HD void v3_cross(const double* a, const double* b, double* r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = -(a[0] * b[2] - a[2] * b[0]);
    r[2] = a[0] * b[1] - a[1] * b[0];
}
MCV_HD double v3_dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
MCV_HD double v3_norm(const double* a) { return sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }

// Everything computePoses derives before the quartic (ap3p.cpp:133-211): the frames k1 / nl /
// k3 / tz, b3' and the g1..g7 terms; c = quartic coefficients ascending (c[4] s^4 + ... + c[0]).
struct Ap3pSetup {
    double k1[3], nl[3], temp[3], k3[3], tz[3], b1[3], b3p[3], w3[3];
    double g1, g2, g3, g4, g5, g6, g7, k3b3;
    double c[5];
    bool ok;   // finite coefficients and non-degenerate frames
};

MCV_HD void ap3p_setup(const double (*b)[3], const double (*w)[3], Ap3pSetup& S) {
    const double* w1 = w[0];
    const double* w2 = w[1];
    const double* w3 = w[2];
    const double* b1 = b[0];
    const double* b2 = b[1];
    const double* b3 = b[2];
    double u0[3] = {w1[0] - w2[0], w1[1] - w2[1], w1[2] - w2[2]};
    const double nu0 = v3_norm(u0);
    double* k1 = S.k1;
    k1[0] = u0[0] / nu0; k1[1] = u0[1] / nu0; k1[2] = u0[2] / nu0;
    double* k3 = S.k3;
    v3_cross(b1, b2, k3);
    const double nk3 = v3_norm(k3);
    k3[0] = k3[0] / nk3; k3[1] = k3[1] / nk3; k3[2] = k3[2] / nk3;
    double v1[3], v2[3];
    v3_cross(b1, k3, S.tz);
    v3_cross(b1, b3, v1);
    v3_cross(b2, b3, v2);
    double u1[3] = {w1[0] - w3[0], w1[1] - w3[1], w1[2] - w3[2]};
    const double u1k1 = v3_dot(u1, k1);
    const double k3b3 = v3_dot(k3, b3);
    double f11 = k3b3;
    double f13 = v3_dot(k3, v1);
    const double f15 = -u1k1 * f11;
    double* nl = S.nl;
    v3_cross(u1, k1, nl);
    const double delta = v3_norm(nl);
    nl[0] = nl[0] / delta; nl[1] = nl[1] / delta; nl[2] = nl[2] / delta;
    f11 = f11 * delta;
    f13 = f13 * delta;
    const double u2k1 = u1k1 - nu0;
    double f21 = v3_dot(S.tz, v2);
    double f22 = nk3 * k3b3;
    double f23 = v3_dot(k3, v2);
    const double f24 = u2k1 * f22;
    const double f25 = -u2k1 * f21;
    f21 = f21 * delta;
    f22 = f22 * delta;
    f23 = f23 * delta;
    S.g1 = f13 * f22;
    S.g2 = f13 * f25 - f15 * f23;
    S.g3 = f11 * f23 - f13 * f21;
    S.g4 = -f13 * f24;
    S.g5 = f11 * f22;
    S.g6 = f11 * f25 - f15 * f21;
    S.g7 = -f15 * f24;
    const double g1 = S.g1, g2 = S.g2, g3 = S.g3, g4 = S.g4, g5 = S.g5, g6 = S.g6, g7 = S.g7;
    double* c = S.c;
    c[4] = g5 * g5 + g1 * g1 + g3 * g3;
    c[3] = 2 * (g5 * g6 + g1 * g2 + g3 * g4);
    c[2] = g6 * g6 + 2 * g5 * g7 + g2 * g2 + g4 * g4 - g1 * g1 - g3 * g3;
    c[1] = 2 * (g6 * g7 - g1 * g2 - g3 * g4);
    c[0] = g7 * g7 - g2 * g2 - g4 * g4;
    bool finite = true;
    for (int k = 0; k < 5; ++k) finite = finite && isfinite(c[k]);
    S.ok = finite && isfinite(delta) && isfinite(k3b3) && nk3 > 0 && nu0 > 0 && delta > 0;
    v3_cross(k1, nl, S.temp);
    for (int k = 0; k < 3; ++k) { S.b1[k] = b1[k]; S.w3[k] = w3[k]; }
    const double sc = delta / k3b3;
    S.b3p[0] = b3[0] * sc; S.b3p[1] = b3[1] * sc; S.b3p[2] = b3[2] * sc;
    S.k3b3 = k3b3;
}

// One root cos(theta1') -> (R, t) (ap3p.cpp:220-255). Returns whether every value is finite.
MCV_HD bool ap3p_pose(const Ap3pSetup& S, double ct1, double* R, double* tv) {
    const double Ck1nl[9] = {S.k1[0], S.nl[0], S.temp[0], S.k1[1], S.nl[1], S.temp[1], S.k1[2], S.nl[2], S.temp[2]};
    const double Cb1k3tzT[9] = {S.b1[0], S.b1[1], S.b1[2], S.k3[0], S.k3[1], S.k3[2], S.tz[0], S.tz[1], S.tz[2]};
    double st1 = sqrt(1 - ct1 * ct1);
    st1 = (S.k3b3 > 0) ? st1 : -st1;
    double ct3 = S.g1 * ct1 + S.g2;
    double st3 = S.g3 * ct1 + S.g4;
    const double nt3 = st1 / ((S.g5 * ct1 + S.g6) * ct1 + S.g7);
    ct3 = ct3 * nt3;
    st3 = st3 * nt3;
    const double C13[9] = {ct3, 0, -st3, st1 * st3, ct1, st1 * ct3, ct1 * st3, -st1, ct1 * ct3};
    double T[9];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            T[3 * r + q] = Ck1nl[3 * r] * C13[q] + Ck1nl[3 * r + 1] * C13[3 + q] + Ck1nl[3 * r + 2] * C13[6 + q];
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q)
            R[3 * r + q] = T[3 * r] * Cb1k3tzT[q] + T[3 * r + 1] * Cb1k3tzT[3 + q] + T[3 * r + 2] * Cb1k3tzT[6 + q];
    const double* w3 = S.w3;
    const double rp3[3] = {w3[0] * R[0] + w3[1] * R[3] + w3[2] * R[6], w3[0] * R[1] + w3[1] * R[4] + w3[2] * R[7],
                           w3[0] * R[2] + w3[1] * R[5] + w3[2] * R[8]};
    bool ok = isfinite(nt3);
    for (int k = 0; k < 9; ++k) ok = ok && isfinite(R[k]);
    for (int k = 0; k < 3; ++k) { tv[k] = st1 * S.b3p[k] - rp3[k]; ok = ok && isfinite(tv[k]); }
    return ok;
}

// b[3][3]: bearing vectors (unit) b1, b2, b3; w[3][3]: world points. Outputs up to 4 solutions
// (Rr = the reference's R, row-major; tr = translation). Returns the count. The RANSAC form: the
// real roots of the quartic from e_poly_real_roots (bit-reproducible), non-finite poses dropped.
MCV_HD int ap3p_compute_poses(const double (*b)[3], const double (*w)[3], double (*Rr)[9], double (*tr)[3]) {
    Ap3pSetup S;
    ap3p_setup(b, w, S);
    if (!S.ok) return 0;
    double s[4];
    const int ns = e_poly_real_roots_fixed<4>(S.c, s);   // = e_poly_real_roots(c, 4, s), register-resident
    int n = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // ns <= 4 = kPnpMaxSolutions: no solution is ever cut off
        if (i >= ns) break;
        const double ct1 = s[i];
        if (fabs(ct1) > 1) continue;
        double R[9], tv[3];
        const bool ok = ap3p_pose(S, ct1, R, tv);
        // append to slot n as selects (a dynamically indexed store would put Rr / tr in scratch)
#pragma unroll
        for (int slot = 0; slot < kPnpMaxSolutions; ++slot) {
            const bool wr = ok && slot == n;
#pragma unroll
            for (int k = 0; k < 9; ++k) Rr[slot][k] = wr ? R[k] : Rr[slot][k];
#pragma unroll
            for (int k = 0; k < 3; ++k) tr[slot][k] = wr ? tv[k] : tr[slot][k];
        }
        if (ok) ++n;
    }
    return n;
}

// ---- the reference's own quartic path for the solveAp3p export ----------------------------------
// solveQuartic (ap3p.cpp:10-59): Ferrari through std::complex<double> as libstdc++ evaluates it
// (csqrt of glibc, pow(complex, 1/3) = polar(exp(log|w| / 3), arg(w) / 3), real / complex by
// Smith's division as libgcc's __divdc3), every root's real part kept; polishQuarticRoots
// (ap3p.cpp:61-74): two Newton passes over the four roots. Transcendentals (cbrt, log, exp, cos,
// atan2, hypot) are the device's (ocml) vs glibc on the host: agreement to ~1e-15, not bit for bit.
struct Cplx { double re, im; };

MCV_HD Cplx cplx_sqrt(double x, double y) {
    if (!isfinite(x) || !isfinite(y)) {
        const double n = x + y;
        return {n, n};
    }
    if (y == 0) {
        if (x < 0) return {0.0, copysign(sqrt(-x), y)};
        return {fabs(sqrt(x)), copysign(0.0, y)};
    }
    if (x == 0) {
        const double r = fabs(y) >= 2 * kDblMin ? sqrt(0.5 * fabs(y)) : 0.5 * sqrt(2 * fabs(y));
        return {r, copysign(r, y)};
    }
    const double d = glibc_hypot(x, y);   // glibc's csqrt calls glibc's hypot (glibc_math.h)
    double r, s;
    if (x > 0) {
        r = sqrt(0.5 * (d + x));
        s = 0.5 * (y / r);
    } else {
        s = sqrt(0.5 * (d - x));
        r = fabs(0.5 * (y / s));
    }
    return {r, copysign(s, y)};
}

MCV_HD Cplx cplx_div(Cplx a, Cplx b) {
    double ratio, denom;
    if (fabs(b.re) < fabs(b.im)) {
        ratio = b.re / b.im;
        denom = (b.re * ratio) + b.im;
        return {((a.re * ratio) + a.im) / denom, ((a.im * ratio) - a.re) / denom};
    }
    ratio = b.im / b.re;
    denom = (b.im * ratio) + b.re;
    return {((a.im * ratio) + a.re) / denom, (a.im - (a.re * ratio)) / denom};
}

// factors: a4, a3, a2, a1, a0 (descending, as solveQuartic reads them). cplx (optional) is set when the
// resolvent's w is complex: pow(w, 1/3) then runs glibc's clog / exp / cos / atan2 through libstdc++,
// restated with glibc's tables and its FMA build's operation order in glibc_math.h (as are cbrt and
// csqrt's hypot on the real branch), so every step is glibc's bit for bit on the device too.
MCV_HD void ap3p_solve_quartic(const double* f, double* roots, bool* cplx = nullptr) {
    const double a4 = f[0], a3 = f[1], a2 = f[2], a1 = f[3], a0 = f[4];
    const double a4_2 = a4 * a4, a3_2 = a3 * a3, a4_3 = a4_2 * a4, a2a4 = a2 * a4;
    const double p4 = (8 * a2a4 - 3 * a3_2) / (8 * a4_2);
    const double q4 = (a3_2 * a3 - 4 * a2a4 * a3 + 8 * a1 * a4_2) / (8 * a4_3);
    const double r4 = (256 * a0 * a4_3 - 3 * (a3_2 * a3_2) - 64 * a1 * a3 * a4_2 + 16 * a2a4 * a3_2) / (256 * (a4_3 * a4));
    const double p3 = ((p4 * p4) / 12 + r4) / 3;
    const double q3 = (72 * r4 * p4 - 2 * p4 * p4 * p4 - 27 * q4 * q4) / 432;
    const Cplx sd = cplx_sqrt(q3 * q3 - p3 * p3 * p3, 0.0);
    Cplx w;
    if (q3 >= 0) w = {-sd.re - q3, -sd.im};
    else w = {sd.re - q3, sd.im};
    double t;
    if (cplx) *cplx = w.im != 0.0;
    if (w.im == 0.0) {
        const double wr = glibc_cbrt(w.re);   // glibc's bits (glibc_math.h)
        t = 2.0 * (wr + p3 / wr);
    } else {
        // pow(w, 1 / 3) = polar(exp(log|w| / 3), arg(w) / 3) (libstdc++): clog's real part (glibc's
        // branches, log / log1p / hypot), its imaginary part atan2, then exp and cos (glibc_math.h)
        const double third = 1.0 / 3;
        const double lr = glibc_clog_re(w.re, w.im), li = glibc_atan2(w.im, w.re);
        t = 4.0 * (glibc_exp(third * lr) * glibc_cos(third * li));
    }
    const Cplx sqrt_2m = cplx_sqrt(-2 * p4 / 3 + t, 0.0);
    const double B_4A = -a3 / (4 * a4);
    const double complex1 = 4 * p4 / 3 + t;
    const Cplx complex2 = cplx_div({2 * q4, 0.0}, sqrt_2m);
    const double sqrt_2m_rh = sqrt_2m.re / 2;
    const double sqrt1 = cplx_sqrt(-(complex1 + complex2.re), -complex2.im).re / 2;
    roots[0] = B_4A + sqrt_2m_rh + sqrt1;
    roots[1] = B_4A + sqrt_2m_rh - sqrt1;
    const double sqrt2 = cplx_sqrt(-(complex1 - complex2.re), complex2.im).re / 2;
    roots[2] = B_4A - sqrt_2m_rh + sqrt2;
    roots[3] = B_4A - sqrt_2m_rh - sqrt2;
}

MCV_HD void ap3p_polish(const double* c, double* roots) {
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 4; ++j) {
            const double error = (((c[0] * roots[j] + c[1]) * roots[j] + c[2]) * roots[j] + c[3]) * roots[j] + c[4];
            const double derivative = ((4 * c[0] * roots[j] + 3 * c[1]) * roots[j] + 2 * c[2]) * roots[j] + c[3];
            roots[j] -= error / derivative;
        }
}

// computePoses exactly as the export runs it: the four polished Ferrari roots in order, |cos| > 1
// skipped, nothing else filtered (non-finite poses of degenerate input are returned as they come).
MCV_HD int ap3p_compute_poses_ref(const double (*b)[3], const double (*w)[3], double (*Rr)[9], double (*tr)[3],
                                  bool* cplx = nullptr) {
    Ap3pSetup S;
    ap3p_setup(b, w, S);
    const double f[5] = {S.c[4], S.c[3], S.c[2], S.c[1], S.c[0]};
    double s[4];
    ap3p_solve_quartic(f, s, cplx);
    ap3p_polish(f, s);
    int n = 0;
    for (int i = 0; i < 4; ++i) {
        const double ct1 = s[i];
        if (fabs(ct1) > 1) continue;
        ap3p_pose(S, ct1, Rr[n], tr[n]);
        ++n;
    }
    return n;
}

// computePoses with the reference's own quartic path (solveQuartic + polishQuarticRoots, ap3p.cpp:203-204):
// the four polished Ferrari roots in order, |cos| > 1 skipped (a NaN root is not: as in the reference,
// it yields a NaN pose, which counts no inliers), poses appended through selects (register-resident).
// The RANSAC kernel's default; its transcendentals (cbrt, log, log1p, atan2, exp, cos, hypot) are glibc's
// restated (glibc_math.h), on the GPU and in the host twin alike.
MCV_HD int ap3p_compute_poses_ferrari(const double (*b)[3], const double (*w)[3], double (*Rr)[9], double (*tr)[3],
                                      bool* cplx = nullptr) {
    Ap3pSetup S;
    ap3p_setup(b, w, S);
    const double f[5] = {S.c[4], S.c[3], S.c[2], S.c[1], S.c[0]};
    double s[4];
    ap3p_solve_quartic(f, s, cplx);
    ap3p_polish(f, s);
    int n = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const double ct1 = s[i];
        if (fabs(ct1) > 1) continue;
        double R[9], tv[3];
        (void)ap3p_pose(S, ct1, R, tv);
#pragma unroll
        for (int slot = 0; slot < kPnpMaxSolutions; ++slot) {
            const bool wr = slot == n;
#pragma unroll
            for (int k = 0; k < 9; ++k) Rr[slot][k] = wr ? R[k] : Rr[slot][k];
#pragma unroll
            for (int k = 0; k < 3; ++k) tr[slot][k] = wr ? tv[k] : tr[slot][k];
        }
        ++n;
    }
    return n;
}

// Bearing vector of a normalised image point (x, y): (x, y, 1) / |(x, y, 1)| as the reference
// builds it (ap3p.cpp:285-301: mk = 1 / norm, then mu *= mk, mv *= mk).
MCV_HD void pnp_bearing(double x, double y, double* b) {
    const double nrm = sqrt(x * x + y * y + 1);
    const double mk = 1. / nrm;
    b[0] = x * mk;
    b[1] = y * mk;
    b[2] = mk;
}

// Four-point AP3P pose: points 0..2 solve, point 3 (pixel reprojection error, distortion-free on
// the undistorted point) picks the solution; first minimum on ties. x/y: undistorted normalised
// image coordinates; W: world points. Returns 1 and the camera-from-world pose, or 0.
MCV_HD int pnp_ap3p4(const PnpCamera& c, const double* x, const double* y, const double (*W)[3], PnpPose& pose) {
    double b[3][3], w[3][3];
    for (int i = 0; i < 3; ++i) {
        pnp_bearing(x[i], y[i], b[i]);
        for (int k = 0; k < 3; ++k) w[i][k] = W[i][k];
    }
    double Rr[kPnpMaxSolutions][9], tr[kPnpMaxSolutions][3];
    for (int i = 0; i < kPnpMaxSolutions; ++i) {
        for (int k = 0; k < 9; ++k) Rr[i][k] = 0.0;
        for (int k = 0; k < 3; ++k) tr[i][k] = 0.0;
    }
    const int n = ap3p_compute_poses(b, w, Rr, tr);
    if (n == 0) return 0;
    double bestErr = 0, bR[9], bt[3];
#pragma unroll
    for (int i = 0; i < kPnpMaxSolutions; ++i) {
        if (i >= n) break;
        // camera-from-world rotation = Rr^T
        const double* R = Rr[i];
        const double X = R[0] * W[3][0] + R[3] * W[3][1] + R[6] * W[3][2] + tr[i][0];
        const double Y = R[1] * W[3][0] + R[4] * W[3][1] + R[7] * W[3][2] + tr[i][1];
        const double Z = R[2] * W[3][0] + R[5] * W[3][1] + R[8] * W[3][2] + tr[i][2];
        const double du = c.fx * (X / Z - x[3]);
        const double dv = c.fy * (Y / Z - y[3]);
        const double e = du * du + dv * dv;
        const bool take = i == 0 || bestErr > e;   // first minimum
        bestErr = take ? e : bestErr;
        for (int k = 0; k < 9; ++k) bR[k] = take ? R[k] : bR[k];
        for (int k = 0; k < 3; ++k) bt[k] = take ? tr[i][k] : bt[k];
    }
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) pose.R[3 * r + q] = bR[3 * q + r];
    for (int k = 0; k < 3; ++k) pose.t[k] = bt[k];
    return 1;
}

// Packed PnP correspondence on the device: float4 {X, Y, Z, u} + float4 {v, 0, 0, 0} (32 B),
// fp32 as solvePnPRansac's convertTo(CV_32F).
struct PnpPoint { float X, Y, Z, u, v, pad0, pad1, pad2; };

// OpenCV 4.x's AP3P minimal solve as PnPRansacCallback runs it on a 4-point subset [ext: calib3d
// solvePnP -> solveP3P -> ap3p::solve(Rs, ts, opoints, undistortedPoints)]: undistortPoints writes the
// normalised points into a CV_32F result (xf = (float)x), extract_points maps them back to pixels
// (mu = xf fx + cx in double), ap3p::solve normalises again (inv_fx mu - cx_fx, inv_fx = 1 / fx,
// cx_fx = cx / fx) and builds the bearings (ap3p.cpp:285-301's form), computePoses with the Ferrari
// quartic, and the fourth point picks the solution of least pixel reprojection error
// ((cx + fx X3p / Z3p - mu3)^2 + ..., first minimum). Returns 1 and the camera-from-world pose, or 0.
MCV_HD int pnp_ap3p4_cv(const PnpCamera& c, const double* x, const double* y, const double (*W)[3], PnpPose& pose,
                        bool* cplx = nullptr) {
    const double inv_fx = 1. / c.fx, inv_fy = 1. / c.fy, cx_fx = c.cx / c.fx, cy_fy = c.cy / c.fy;
    double mu[4], mv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        mu[i] = (double)(float)x[i] * c.fx + c.cx;
        mv[i] = (double)(float)y[i] * c.fy + c.cy;
    }
    double b[3][3], w[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        pnp_bearing(inv_fx * mu[i] - cx_fx, inv_fy * mv[i] - cy_fy, b[i]);
#pragma unroll
        for (int k = 0; k < 3; ++k) w[i][k] = W[i][k];
    }
    double Rr[kPnpMaxSolutions][9], tr[kPnpMaxSolutions][3];
#pragma unroll
    for (int i = 0; i < kPnpMaxSolutions; ++i) {
#pragma unroll
        for (int k = 0; k < 9; ++k) Rr[i][k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) tr[i][k] = 0.0;
    }
    const int n = ap3p_compute_poses_ferrari(b, w, Rr, tr, cplx);
    if (n == 0) return 0;
    double bestErr = 0, bR[9], bt[3];
#pragma unroll
    for (int i = 0; i < kPnpMaxSolutions; ++i) {
        if (i >= n) break;
        const double* R = Rr[i];   // camera-from-world rotation = Rr^T
        const double X = R[0] * W[3][0] + R[3] * W[3][1] + R[6] * W[3][2] + tr[i][0];
        const double Y = R[1] * W[3][0] + R[4] * W[3][1] + R[7] * W[3][2] + tr[i][1];
        const double Z = R[2] * W[3][0] + R[5] * W[3][1] + R[8] * W[3][2] + tr[i][2];
        const double mu3p = c.cx + c.fx * X / Z;
        const double mv3p = c.cy + c.fy * Y / Z;
        const double e = (mu3p - mu[3]) * (mu3p - mu[3]) + (mv3p - mv[3]) * (mv3p - mv[3]);
        const bool take = i == 0 || bestErr > e;   // first minimum
        bestErr = take ? e : bestErr;
#pragma unroll
        for (int k = 0; k < 9; ++k) bR[k] = take ? R[k] : bR[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) bt[k] = take ? tr[i][k] : bt[k];
    }
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) pose.R[3 * r + q] = bR[3 * q + r];
    for (int k = 0; k < 3; ++k) pose.t[k] = bt[k];
    return 1;
}

// One hypothesis: 4 distinct indices, undistort, AP3P + 4th-point selection: OpenCV's chain
// (pnp_ap3p4_cv, default) or, with fast (MCV_FLAG_FAST_MINIMAL), the real-root-finder form (pnp_ap3p4).
// Returns 1 (model), kStatusNoModel or kStatusNoSample.
MCV_HD int pnp_hypothesis(const PnpPoint* pts, int N, const PnpCamera& c, const Sampler& smp, uint64_t hyp,
                          PnpPose& pose, int* idx_out, bool fast = false) {
    SubsetSrc<4> src(smp, hyp);
    int idx[4];
    bool found = false;   // search and solve apart (h_hypothesis): one solve pass per wave
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, idx);
        if (got < 0) break;
        if (got == 0) continue;
        found = true;
        break;
    }
    if (!found) return kStatusNoSample;
    double x[4], y[4], W[4][3];
    for (int i = 0; i < 4; ++i) {
        const PnpPoint p = pts[idx[i]];
        pnp_undistort(c, (double)p.u, (double)p.v, x[i], y[i]);
        W[i][0] = p.X; W[i][1] = p.Y; W[i][2] = p.Z;
    }
    if (idx_out) for (int i = 0; i < 4; ++i) idx_out[i] = idx[i];
    const int ok = fast ? pnp_ap3p4(c, x, y, W, pose) : pnp_ap3p4_cv(c, x, y, W, pose);
    return ok ? 1 : kStatusNoModel;
}

// PnP solver kinds (the reference's solverKind, MiniCVNative.cpp:99-116): 0 ITERATIVE, 1 EPNP,
// 2 P3P, 3 DLS, 4 UPNP, 5 AP3P; other values select ITERATIVE there (kind stays 0).
MCV_HD int pnp_kind(int solverKind) { return solverKind >= 0 && solverKind <= 5 ? solverKind : 0; }
// solvePnPRansac's minimal-set solver: P3P / AP3P keep their 4-point kernel (AP3P here for both),
// every other kind samples 5 points for EPnP.
MCV_HD bool pnp_kind_epnp(int kind) { return kind != 2 && kind != 5; }

// EPnP on 5 float correspondences as PnPRansacCallback::runKernel feeds it: the float subset's
// image points go through undistortPoints with a CV_32F result (the normalised coordinates are
// rounded to float), epnp::init_points maps them back to pixels (x * fu + uc in double), world
// points are the float coordinates.
MCV_HD void pnp_epnp5_points(const PnpCamera& c, const PnpPoint* p5, double (&pw)[5][3], double (&us)[5][2]) {
    for (int i = 0; i < 5; ++i) {
        const PnpPoint p = p5[i];
        double x, y;
        pnp_undistort(c, (double)p.u, (double)p.v, x, y);
        us[i][0] = (double)(float)x * c.fx + c.cx;
        us[i][1] = (double)(float)y * c.fy + c.cy;
        pw[i][0] = p.X; pw[i][1] = p.Y; pw[i][2] = p.Z;
    }
}
MCV_HD void pnp_epnp5(const PnpCamera& c, const PnpPoint* p5, PnpPose& pose, EpnpWs& ws) {
    double pw[5][3], us[5][2];
    pnp_epnp5_points(c, p5, pw, us);
    const EpnpCam ec{c.fx, c.fy, c.cx, c.cy};
    double R[3][3], t[3];
    epnp_solve_small<5>(pw, us, ec, R, t, ws);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) pose.R[3 * i + j] = R[i][j];
        pose.t[i] = t[i];
    }
}
MCV_HD void pnp_epnp5(const PnpCamera& c, const PnpPoint* p5, PnpPose& pose) {
    EpnpWs ws;
    pnp_epnp5(c, p5, pose, ws);
}

// One EPnP hypothesis: 5 distinct indices (Philox stream) -> pnp_epnp5. EPnP always yields a
// model (possibly non-finite, which then counts no inliers), as solvePnP(EPNP) returns true.
MCV_HD bool pnp_sample5(int N, const Sampler& smp, uint64_t hyp, int (&idx)[5]) {
    SubsetSrc<5> src(smp, hyp);
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {   // search and solve apart (h_hypothesis)
        const int got = src.next(N, idx);
        if (got < 0) return false;
        if (got > 0) return true;
    }
    return false;
}
MCV_HD int pnp_hypothesis_epnp(const PnpPoint* pts, int N, const PnpCamera& c, const Sampler& smp, uint64_t hyp,
                               PnpPose& pose, int* idx_out, EpnpWs& ws) {
    int idx[5];
    if (!pnp_sample5(N, smp, hyp, idx)) return kStatusNoSample;
    PnpPoint p5[5];
    for (int i = 0; i < 5; ++i) p5[i] = pts[idx[i]];
    if (idx_out) for (int i = 0; i < 5; ++i) idx_out[i] = idx[i];
    pnp_epnp5(c, p5, pose, ws);
    return 1;
}
MCV_HD int pnp_hypothesis_epnp(const PnpPoint* pts, int N, const PnpCamera& c, const Sampler& smp, uint64_t hyp,
                               PnpPose& pose, int* idx_out) {
    EpnpWs ws;
    return pnp_hypothesis_epnp(pts, N, c, smp, hyp, pose, idx_out, ws);
}

// The split device generate: pnp_hypothesis_epnp as three kernels over a launch's hypotheses, which
// pass their state through structure-of-arrays scratch (value e of hypothesis i at base[e * s + i]).
// Kernel 1: sample, control points, alphas, M^T M. Kernel 2: the SVD's Jacobi sweeps, the only part
// that needs a per-lane working matrix in LDS (jacobi12_sweeps_split: half of it in LDS, half in
// registers, four waves per CU). Kernel 3: the SVD's tail (norms, sort, null-row completion) on the
// matrix in global scratch and L_6x10. Kernel 4: the betas of the three approximations with their
// Gauss-Newton steps (L_6x10 and rho copied to a per-lane LDS slice: Gauss-Newton re-reads them every
// iteration). Kernel 5: the three poses and compute_pose's pick. Every value crosses the kernels as the
// same double and every operation keeps its order, so the composition computes pnp_hypothesis_epnp's
// bits. Split by register footprint: one kernel held 422 registers (one wave per SIMD) and 3.97 ms per
// 2^20 hypotheses for kernels 3-5, which take 0.80 + 1.64 + 0.58 ms.
static const int kEpnpCtx = 57;   // pw (15), us (10), al (20), cws (12)
struct EpnpSplit {
    double* mtm;   // kMtmSums x s
    double* ctx;   // kEpnpCtx x s
    double* A;     // 144 x s: the working matrix after the sweeps (EpnpWsSoA)
    double* W;     // 12 x s: its squared row norms after the sweeps
    int64_t s;
};
static const int kEpnpSplitDoubles = kMtmSums + kEpnpCtx + 144 + 12;
static const int kEpnpLoStride = 74;   // doubles per lane of kernel 2's LDS (6 x 12 + pad, 16-byte rows)

// Kernel 1: sample, points, control points, alphas and M^T M. Returns 1 or kStatusNoSample.
MCV_HD int pnp_epnp_split_mtm(const PnpPoint* pts, int N, const PnpCamera& c, const Sampler& smp, uint64_t hyp,
                              const EpnpSplit& X, int64_t i) {
    int idx[5];
    if (!pnp_sample5(N, smp, hyp, idx)) return kStatusNoSample;
    PnpPoint p5[5];
    for (int k = 0; k < 5; ++k) p5[k] = pts[idx[k]];
    double pw[5][3], us[5][2], al[5][4], mtm[kMtmSums];
    pnp_epnp5_points(c, p5, pw, us);
    EpnpCtrl C;
    epnp_small_mtm<5>(pw, us, EpnpCam{c.fx, c.fy, c.cx, c.cy}, C, al, mtm);
    double* q = X.ctx + i;
    int e = 0;
    for (int k = 0; k < 5; ++k)
        for (int j = 0; j < 3; ++j) q[(e++) * X.s] = pw[k][j];
    for (int k = 0; k < 5; ++k)
        for (int j = 0; j < 2; ++j) q[(e++) * X.s] = us[k][j];
    for (int k = 0; k < 5; ++k)
        for (int j = 0; j < 4; ++j) q[(e++) * X.s] = al[k][j];
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 3; ++j) q[(e++) * X.s] = C.cws[k][j];
    for (int k = 0; k < kMtmSums; ++k) X.mtm[k * X.s + i] = mtm[k];
    return 1;
}

// Kernel 2: M^T M into the split working matrix (lo: the lane's LDS slice), jacobi_svd_core's initial
// squared norms and its sweeps; the matrix and the norms out.
MCV_HD void pnp_epnp_split_sweeps(const EpnpSplit& X, int64_t i, double* lo) {
    double hi[12][6], W[12];
    MCV_SMALL_UNROLL
    for (int a = 0; a < 12; ++a)
        MCV_SMALL_UNROLL
        for (int b = 0; b < 12; ++b) {
            const double v = X.mtm[mtm_index(a < b ? a : b, a < b ? b : a) * X.s + i];
            if (b < 6) lo[6 * a + b] = v;
            else hi[a][b - 6] = v;
        }
    MCV_SMALL_UNROLL
    for (int a = 0; a < 12; ++a) {
        double sd = 0;
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) sd += lo[6 * a + k] * lo[6 * a + k];
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) sd += hi[a][k] * hi[a][k];
        W[a] = sd;
    }
    jacobi12_sweeps_split(lo, hi, W);
    const EpnpWsSoA o{X.A + i, X.s};
    MCV_SMALL_UNROLL
    for (int a = 0; a < 12; ++a) {
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) o(a, k) = lo[6 * a + k];
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) o(a, 6 + k) = hi[a][k];
        X.W[a * X.s + i] = W[a];
    }
}

// Kernel 3: the SVD's tail and L_6x10 on the matrix in scratch. Kernel 4: the betas of the three
// approximations (Gauss-Newton included) into the M^T M slots, which kernel 2 has consumed.
MCV_HD void pnp_epnp_split_tail(const EpnpSplit& X, int64_t i) {
    const EpnpWsSoA A{X.A + i, X.s};
    double W[12], cws[4][3];
    for (int a = 0; a < 12; ++a) W[a] = X.W[a * X.s + i];
    jacobi12_tail(A, W);
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 3; ++j) cws[k][j] = X.ctx[(45 + 3 * k + j) * X.s + i];
    epnp_l_rows(cws, A);
}
MCV_HD void pnp_epnp_split_betas(const EpnpSplit& X, int64_t i, double* lds66) {
    const EpnpWsSoA A{X.A + i, X.s};
    const EpnpLRef L{lds66};
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 11; ++c) L(r, c) = A(r, c);
    double betas[4][4];
    epnp_betas_from_l(betas, L);
    for (int n = 1; n < 4; ++n)
        for (int k = 0; k < 4; ++k) X.mtm[(4 * (n - 1) + k) * X.s + i] = betas[n][k];
}

// Kernel 5: the three poses from the betas and the null-space vectors, and compute_pose's pick.
MCV_HD void pnp_epnp_split_pose(const PnpCamera& c, const EpnpSplit& X, int64_t i, PnpPose& pose) {
    const EpnpWsSoA A{X.A + i, X.s};
    double betas[4][4];
    for (int k = 0; k < 4; ++k) betas[0][k] = 0;
    for (int n = 1; n < 4; ++n)
        for (int k = 0; k < 4; ++k) betas[n][k] = X.mtm[(4 * (n - 1) + k) * X.s + i];
    double pw[5][3], us[5][2], al[5][4];
    const double* q = X.ctx + i;
    int e = 0;
    for (int k = 0; k < 5; ++k)
        for (int j = 0; j < 3; ++j) pw[k][j] = q[(e++) * X.s];
    for (int k = 0; k < 5; ++k)
        for (int j = 0; j < 2; ++j) us[k][j] = q[(e++) * X.s];
    for (int k = 0; k < 5; ++k)
        for (int j = 0; j < 4; ++j) al[k][j] = q[(e++) * X.s];
    double R[3][3], t[3];
    epnp_small_pick<5>(pw, us, EpnpCam{c.fx, c.fy, c.cx, c.cy}, al, A, betas, R, t);
    for (int r = 0; r < 3; ++r) {
        for (int j = 0; j < 3; ++j) pose.R[3 * r + j] = R[r][j];
        pose.t[r] = t[r];
    }
}

}  // namespace mcv
