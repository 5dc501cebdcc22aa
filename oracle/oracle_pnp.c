/*
 * oracle_pnp.c — CPU restatement of the PnP-RANSAC path. TEST
 * INFRASTRUCTURE ONLY (rules and parity status: oracle.c header).
 *
 * Follows the reference's AP3P solver /root/reference/src/MiniCVNative/ap3p.cpp:123-255
 * (computePoses: bearing/world geometry, f1i/f2i/g1..g7 terms :150-195, quartic :196-201, C13 and
 * R = Ck1nl C13 Cb1k3tz^T :214-236, t = sin(theta1') b3' - R^T w3 :238-243) and its bearing
 * construction :285-301, with the real quartic roots taken by the shared Rolle-bisection root
 * finder (orc_poly_real_roots) instead of solveQuartic's complex Ferrari formulas; the export
 * semantics of MiniCVNative.cpp:93-139 (cvSolvePnPRansac) with OpenCV 4.x solvePnPRansac /
 * PnPRansacCallback / projectPoints / undistortPoints restated [ext]. Same operation order as
 * minicv_amd/csrc/hyp_pnp.h (bit-exact hypotheses, counts, masks); the LM refit's sums run in
 * another order on the GPU, so refined poses agree to a tolerance.
 *
 * Pinned by exact synthetic geometry: noise-free correspondences of a known pose must give that
 * pose back (AP3P to ~1e-9, RANSAC + LM to ~1e-9), and the 3-point export equals the transposed
 * rotation convention of the reference (ap3p.cpp:245-250).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <complex.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle_int.h"

typedef struct { double fx, fy, cx, cy, k1, k2, p1, p2; } Cam;

static Cam cam_of(const double* c8) {
    Cam c = {c8[0], c8[1], c8[2], c8[3], c8[4], c8[5], c8[6], c8[7]};
    return c;
}

/* cvUndistortPointsInternal: x0 = (u - cx) * ifx with ifx = 1./fx, 5 fixed iterations */
static void undistort(const Cam* c, double u, double v, double* xo, double* yo) {
    double ifx = 1. / c->fx, ify = 1. / c->fy;
    double x0 = (u - c->cx) * ifx, y0 = (v - c->cy) * ify, x = x0, y = y0;
    for (int it = 0; it < 5; ++it) {
        double r2 = x * x + y * y;
        double ic = 1.0 / (1.0 + (c->k2 * r2 + c->k1) * r2);
        if (ic < 0) { x = x0; y = y0; break; }
        double dx = 2.0 * c->p1 * x * y + c->p2 * (r2 + 2.0 * x * x);
        double dy = c->p1 * (r2 + 2.0 * y * y) + 2.0 * c->p2 * x * y;
        x = (x0 - dx) * ic;
        y = (y0 - dy) * ic;
    }
    *xo = x;
    *yo = y;
}

void orc_undistort(const double* cam8, double u, double v, double* x, double* y) {
    Cam c = cam_of(cam8);
    undistort(&c, u, v, x, y);
}

static void project(const Cam* c, const double* R, const double* t, double X, double Y, double Z, double* u, double* v) {
    double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    double iz = Zc != 0 ? 1.0 / Zc : 1.0;
    double x = Xc * iz, y = Yc * iz;
    double r2 = x * x + y * y, r4 = r2 * r2;
    double a1 = 2.0 * x * y, a2 = r2 + 2.0 * x * x, a3 = r2 + 2.0 * y * y;
    double cd = 1.0 + c->k1 * r2 + c->k2 * r4;
    double xd = x * cd + c->p1 * a1 + c->p2 * a2;
    double yd = y * cd + c->p1 * a3 + c->p2 * a1;
    *u = xd * c->fx + c->cx;
    *v = yd * c->fy + c->cy;
}

static float reproj_err(const Cam* c, const double* R, const double* t, const float* p, int fused) {
    double u, v;
    project(c, R, t, p[0], p[1], p[2], &u, &v);
    float dx = p[3] - (float)u, dy = p[4] - (float)v;
    return fused ? fmaf(dx, dx, dy * dy) : dx * dx + dy * dy;
}

static void cross(const double* a, const double* b, double* r) {
    r[0] = a[1] * b[2] - a[2] * b[1];
    r[1] = -(a[0] * b[2] - a[2] * b[0]);
    r[2] = a[0] * b[1] - a[1] * b[0];
}
static double dot(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static double nrm(const double* a) { return sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }

/* solveQuartic (ap3p.cpp:10-59) as libstdc++ evaluates its std::complex<double> expressions on
 * Linux: C99 complex with glibc's csqrt / clog, pow(complex, double) = polar(exp(y log|w|), y arg w)
 * (libstdc++'s non-real branch), real / complex through libgcc's __divdc3; then
 * polishQuarticRoots (ap3p.cpp:61-74). f: descending coefficients a4..a0. */
static _Thread_local int orc_last_branch = -1;   /* the last ferrari_ref's branch: 0 cbrt, 1 complex pow */
int orc_ap3p_last_branch(void) { return orc_last_branch; }

/* glibc's own functions over arrays (the reference for glibc_math.h's restatements):
 * fn 0 cbrt(a), 1 hypot(a, b), 2 creal(clog(a + i b)), 4 exp(a), 5 log(a), 6 log1p(a), 7 cos(a),
 * 8 atan2(a, b). */
int orc_libm(int fn, const double* a, const double* b, int n, double* out) {
    for (int i = 0; i < n; ++i) {
        switch (fn) {
            case 0: out[i] = cbrt(a[i]); break;
            case 1: out[i] = hypot(a[i], b[i]); break;
            case 2: out[i] = creal(clog(CMPLX(a[i], b[i]))); break;
            case 4: out[i] = exp(a[i]); break;
            case 5: out[i] = log(a[i]); break;
            case 6: out[i] = log1p(a[i]); break;
            case 7: out[i] = cos(a[i]); break;
            case 8: out[i] = atan2(a[i], b[i]); break;
            default: return -1;
        }
    }
    return n;
}

static void ferrari_ref(const double* f, double* roots) {
    double a4 = f[0], a3 = f[1], a2 = f[2], a1 = f[3], a0 = f[4];
    double a4_2 = a4 * a4, a3_2 = a3 * a3, a4_3 = a4_2 * a4, a2a4 = a2 * a4;
    double p4 = (8 * a2a4 - 3 * a3_2) / (8 * a4_2);
    double q4 = (a3_2 * a3 - 4 * a2a4 * a3 + 8 * a1 * a4_2) / (8 * a4_3);
    double r4 = (256 * a0 * a4_3 - 3 * (a3_2 * a3_2) - 64 * a1 * a3 * a4_2 + 16 * a2a4 * a3_2) / (256 * (a4_3 * a4));
    double p3 = ((p4 * p4) / 12 + r4) / 3;
    double q3 = (72 * r4 * p4 - 2 * p4 * p4 * p4 - 27 * q4 * q4) / 432;
    double t;
    double complex w;
    double complex sd = csqrt(CMPLX(q3 * q3 - p3 * p3 * p3, 0.0));
    if (q3 >= 0)
        w = -sd - q3;
    else
        w = sd - q3;
    orc_last_branch = cimag(w) == 0.0 ? 0 : 1;
    if (cimag(w) == 0.0) {
        double wr = cbrt(creal(w));
        t = 2.0 * (wr + p3 / wr);
    } else {
        double third = 1.0 / 3;
        double complex lw = clog(w);
        t = 4.0 * (exp(third * creal(lw)) * cos(third * cimag(lw)));
    }
    double complex sqrt_2m = csqrt(CMPLX(-2 * p4 / 3 + t, 0.0));
    double B_4A = -a3 / (4 * a4);
    double complex1 = 4 * p4 / 3 + t;
    double complex complex2 = CMPLX(2 * q4, 0.0) / sqrt_2m;
    double sqrt_2m_rh = creal(sqrt_2m) / 2;
    double sqrt1 = creal(csqrt(-(complex1 + complex2))) / 2;
    roots[0] = B_4A + sqrt_2m_rh + sqrt1;
    roots[1] = B_4A + sqrt_2m_rh - sqrt1;
    double sqrt2 = creal(csqrt(-(complex1 - complex2))) / 2;
    roots[2] = B_4A - sqrt_2m_rh + sqrt2;
    roots[3] = B_4A - sqrt_2m_rh - sqrt2;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 4; ++j) {
            double error = (((f[0] * roots[j] + f[1]) * roots[j] + f[2]) * roots[j] + f[3]) * roots[j] + f[4];
            double derivative = ((4 * f[0] * roots[j] + 3 * f[1]) * roots[j] + 2 * f[2]) * roots[j] + f[3];
            roots[j] -= error / derivative;
        }
}

/* computePoses; Rr/tr as the reference stores them. Returns the count (<= 4).
 * ref = 0: the RANSAC form (bit-reproducible real roots, non-finite poses dropped);
 * ref = 1: the reference's own path (ferrari_ref, all four roots in order, nothing filtered). */
static int ap3p_poses_impl(const double* b, const double* w, double* Rr, double* tr, int ref);

int orc_ap3p_poses(const double* b /*3x3 rows = b1,b2,b3*/, const double* w /*rows = w1,w2,w3*/, double* Rr,
                   double* tr) {
    return ap3p_poses_impl(b, w, Rr, tr, 0);
}

static int ap3p_poses_impl(const double* b, const double* w, double* Rr, double* tr, int ref) {
    const double *w1 = w, *w2 = w + 3, *w3 = w + 6, *b1 = b, *b2 = b + 3, *b3 = b + 6;
    double u0[3] = {w1[0] - w2[0], w1[1] - w2[1], w1[2] - w2[2]};
    double nu0 = nrm(u0);
    double k1[3] = {u0[0] / nu0, u0[1] / nu0, u0[2] / nu0};
    double k3[3], tz[3], v1[3], v2[3], nl[3];
    cross(b1, b2, k3);
    double nk3 = nrm(k3);
    for (int i = 0; i < 3; ++i) k3[i] = k3[i] / nk3;
    cross(b1, k3, tz);
    cross(b1, b3, v1);
    cross(b2, b3, v2);
    double u1[3] = {w1[0] - w3[0], w1[1] - w3[1], w1[2] - w3[2]};
    double u1k1 = dot(u1, k1), k3b3 = dot(k3, b3);
    double f11 = k3b3, f13 = dot(k3, v1), f15 = -u1k1 * f11;
    cross(u1, k1, nl);
    double delta = nrm(nl);
    for (int i = 0; i < 3; ++i) nl[i] = nl[i] / delta;
    f11 = f11 * delta;
    f13 = f13 * delta;
    double u2k1 = u1k1 - nu0;
    double f21 = dot(tz, v2), f22 = nk3 * k3b3, f23 = dot(k3, v2);
    double f24 = u2k1 * f22, f25 = -u2k1 * f21;
    f21 = f21 * delta;
    f22 = f22 * delta;
    f23 = f23 * delta;
    double g1 = f13 * f22, g2 = f13 * f25 - f15 * f23, g3 = f11 * f23 - f13 * f21, g4 = -f13 * f24;
    double g5 = f11 * f22, g6 = f11 * f25 - f15 * f21, g7 = -f15 * f24;
    double c[5];
    c[4] = g5 * g5 + g1 * g1 + g3 * g3;
    c[3] = 2 * (g5 * g6 + g1 * g2 + g3 * g4);
    c[2] = g6 * g6 + 2 * g5 * g7 + g2 * g2 + g4 * g4 - g1 * g1 - g3 * g3;
    c[1] = 2 * (g6 * g7 - g1 * g2 - g3 * g4);
    c[0] = g7 * g7 - g2 * g2 - g4 * g4;
    int fin = 1;
    for (int k = 0; k < 5; ++k) fin = fin && isfinite(c[k]);
    if (!ref && (!fin || !isfinite(delta) || !isfinite(k3b3) || !(nk3 > 0) || !(nu0 > 0) || !(delta > 0))) return 0;
    double s[10];
    int ns;
    if (ref) {
        double f[5] = {c[4], c[3], c[2], c[1], c[0]};
        ferrari_ref(f, s);
        ns = 4;
    } else {
        ns = orc_poly_real_roots(c, 4, s);
    }
    double tmp[3];
    cross(k1, nl, tmp);
    double A[9] = {k1[0], nl[0], tmp[0], k1[1], nl[1], tmp[1], k1[2], nl[2], tmp[2]};
    double B[9] = {b1[0], b1[1], b1[2], k3[0], k3[1], k3[2], tz[0], tz[1], tz[2]};
    double sc = delta / k3b3;
    double b3p[3] = {b3[0] * sc, b3[1] * sc, b3[2] * sc};
    int n = 0;
    for (int i = 0; i < ns && n < 4; ++i) {
        double ct1 = s[i];
        if (fabs(ct1) > 1) continue;
        double st1 = sqrt(1 - ct1 * ct1);
        st1 = (k3b3 > 0) ? st1 : -st1;
        double ct3 = g1 * ct1 + g2, st3 = g3 * ct1 + g4;
        double nt3 = st1 / ((g5 * ct1 + g6) * ct1 + g7);
        ct3 = ct3 * nt3;
        st3 = st3 * nt3;
        double C[9] = {ct3, 0, -st3, st1 * st3, ct1, st1 * ct3, ct1 * st3, -st1, ct1 * ct3};
        double T[9], R[9];
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) T[3 * r + q] = A[3 * r] * C[q] + A[3 * r + 1] * C[3 + q] + A[3 * r + 2] * C[6 + q];
        for (int r = 0; r < 3; ++r)
            for (int q = 0; q < 3; ++q) R[3 * r + q] = T[3 * r] * B[q] + T[3 * r + 1] * B[3 + q] + T[3 * r + 2] * B[6 + q];
        double rp3[3] = {w3[0] * R[0] + w3[1] * R[3] + w3[2] * R[6], w3[0] * R[1] + w3[1] * R[4] + w3[2] * R[7],
                         w3[0] * R[2] + w3[1] * R[5] + w3[2] * R[8]};
        int ok = isfinite(nt3);
        for (int k = 0; k < 9; ++k) { Rr[9 * n + k] = R[k]; ok = ok && isfinite(R[k]); }
        for (int k = 0; k < 3; ++k) { tr[3 * n + k] = st1 * b3p[k] - rp3[k]; ok = ok && isfinite(tr[3 * n + k]); }
        if (ok || ref) ++n;
    }
    return n;
}

static void bearing(double x, double y, double* b) {
    double nr = sqrt(x * x + y * y + 1), mk = 1. / nr;
    b[0] = x * mk;
    b[1] = y * mk;
    b[2] = mk;
}

/* solveAp3p export semantics (3 points, pixel inputs through inv_fx etc.) */
int orc_solve_ap3p(const double* mu, const double* mv, const double* W9, double inv_fx, double inv_fy, double cx_fx,
                   double cy_fy, double* Rs, double* ts) {
    double b[9];
    for (int i = 0; i < 3; ++i) {
        double u = inv_fx * mu[i] - cx_fx, v = inv_fy * mv[i] - cy_fy;
        double nr = sqrt(u * u + v * v + 1), mk = 1. / nr;
        b[3 * i] = u * mk;
        b[3 * i + 1] = v * mk;
        b[3 * i + 2] = mk;
    }
    return ap3p_poses_impl(b, W9, Rs, ts, 1);
}

/* AP3P on 3 points + the 4th picks (pixel error, first minimum); camera-from-world pose out. */
static int ap3p4(const Cam* c, const double* x, const double* y, const double* W /*4x3*/, double* R, double* t) {
    double b[9], Rr[36], tr[12];
    for (int i = 0; i < 3; ++i) bearing(x[i], y[i], b + 3 * i);
    int n = orc_ap3p_poses(b, W, Rr, tr);
    if (n == 0) return 0;
    int best = 0;
    double be = 0;
    for (int i = 0; i < n; ++i) {
        const double* Q = Rr + 9 * i;
        const double* w4 = W + 9;
        double X = Q[0] * w4[0] + Q[3] * w4[1] + Q[6] * w4[2] + tr[3 * i];
        double Y = Q[1] * w4[0] + Q[4] * w4[1] + Q[7] * w4[2] + tr[3 * i + 1];
        double Z = Q[2] * w4[0] + Q[5] * w4[1] + Q[8] * w4[2] + tr[3 * i + 2];
        double du = c->fx * (X / Z - x[3]), dv = c->fy * (Y / Z - y[3]);
        double e = du * du + dv * dv;
        if (i == 0 || be > e) { best = i; be = e; }
    }
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) R[3 * r + q] = Rr[9 * best + 3 * q + r];
    memcpy(t, tr + 3 * best, sizeof(double) * 3);
    return 1;
}

/* OpenCV 4.x's AP3P on a 4-point subset (solvePnP -> solveP3P -> ap3p::solve [ext]): undistortPoints into
 * a CV_32F result, extract_points' pixels (xf fx + cx), ap3p's normalisation (inv_fx mu - cx_fx), the
 * reference's computePoses with its Ferrari quartic + polish (glibc's transcendentals: the reference's own
 * arithmetic on Linux), the fourth point's pixel reprojection error picks (first minimum). */
static int ap3p4_cv(const Cam* c, const double* x, const double* y, const double* W /*4x3*/, double* R, double* t) {
    const double inv_fx = 1. / c->fx, inv_fy = 1. / c->fy, cx_fx = c->cx / c->fx, cy_fy = c->cy / c->fy;
    double mu[4], mv[4], b[9], Rr[36], tr[12];
    for (int i = 0; i < 4; ++i) {
        mu[i] = (double)(float)x[i] * c->fx + c->cx;
        mv[i] = (double)(float)y[i] * c->fy + c->cy;
    }
    for (int i = 0; i < 3; ++i) bearing(inv_fx * mu[i] - cx_fx, inv_fy * mv[i] - cy_fy, b + 3 * i);
    int n = ap3p_poses_impl(b, W, Rr, tr, 1);
    if (n == 0) return 0;
    int best = 0;
    double be = 0;
    for (int i = 0; i < n; ++i) {
        const double* Q = Rr + 9 * i;
        const double* w4 = W + 9;
        double X = Q[0] * w4[0] + Q[3] * w4[1] + Q[6] * w4[2] + tr[3 * i];
        double Y = Q[1] * w4[0] + Q[4] * w4[1] + Q[7] * w4[2] + tr[3 * i + 1];
        double Z = Q[2] * w4[0] + Q[5] * w4[1] + Q[8] * w4[2] + tr[3 * i + 2];
        double mu3p = c->cx + c->fx * X / Z, mv3p = c->cy + c->fy * Y / Z;
        double e = (mu3p - mu[3]) * (mu3p - mu[3]) + (mv3p - mv[3]) * (mv3p - mv[3]);
        if (i == 0 || be > e) { best = i; be = e; }
    }
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 3; ++q) R[3 * r + q] = Rr[9 * best + 3 * q + r];
    memcpy(t, tr + 3 * best, sizeof(double) * 3);
    return 1;
}

/* the RANSAC form of the 4-point solve: OpenCV's chain (default) or the real-root-finder form */
static int ap3p4_sel(const Cam* c, const double* x, const double* y, const double* W, double* R, double* t) {
    return orc_get_fast_minimal() ? ap3p4(c, x, y, W, R, t) : ap3p4_cv(c, x, y, W, R, t);
}

/* pts: N x 8 floats {X, Y, Z, u, v, 0, 0, 0} (the device PnpPoint layout). */
int orc_pnp_hypothesis(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R, double* t,
                       int* idx_out) {
    Cam c = cam_of(cam8);
    orc_last_branch = -1;
    Stream st;
    st.seed = seed; st.hyp = (uint64_t)hyp; st.pos = 0;
    int idx[4];
    for (int a = 0; a < ORC_MAX_ATTEMPTS; ++a) {
        if (!draw_distinct(&st, N, 4, idx)) continue;
        double x[4], y[4], W[12];
        for (int i = 0; i < 4; ++i) {
            const float* p = pts + 8 * (size_t)idx[i];
            undistort(&c, (double)p[3], (double)p[4], &x[i], &y[i]);
            W[3 * i] = p[0]; W[3 * i + 1] = p[1]; W[3 * i + 2] = p[2];
        }
        if (idx_out) memcpy(idx_out, idx, sizeof(idx));
        return ap3p4_sel(&c, x, y, W, R, t) ? 1 : ORC_NO_MODEL;
    }
    return ORC_NO_SAMPLE;
}

int orc_pnp_count(const float* pts, int N, const double* cam8, const double* R, const double* t, float thr2, int fused,
                  uint8_t* mask) {
    Cam c = cam_of(cam8);
    int n = 0;
    for (int i = 0; i < N; ++i) {
        int in = reproj_err(&c, R, t, pts + 8 * (size_t)i, fused) <= thr2;
        if (mask) mask[i] = (uint8_t)in;
        n += in;
    }
    return n;
}

void orc_pnp_counts(const float* pts, int N, const double* cam8, uint64_t seed, int64_t begin, int64_t count,
                    float thr2, int fused, int* out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t h = 0; h < count; ++h) {
        double R[9], t[3];
        int st = orc_pnp_hypothesis(pts, N, cam8, seed, begin + h, R, t, NULL);
        out[h] = st == 1 ? orc_pnp_count(pts, N, cam8, R, t, thr2, fused, NULL) : st;
    }
}

/* counts with the minimal solver of solverKind `kind` (EPnP on 5 points unless 2 / 5) */
static int kind_epnp(int kind) {
    if (kind < 0 || kind > 5) kind = 0;
    return kind != 2 && kind != 5;
}

void orc_pnp_counts_k(const float* pts, int N, const double* cam8, uint64_t seed, int64_t begin, int64_t count,
                      float thr2, int fused, int kind, int* out, int nthreads) {
    const int ep = kind_epnp(kind);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t h = 0; h < count; ++h) {
        double R[9], t[3];
        int st = ep ? orc_pnp_hypothesis_epnp(pts, N, cam8, seed, begin + h, R, t, NULL)
                    : orc_pnp_hypothesis(pts, N, cam8, seed, begin + h, R, t, NULL);
        out[h] = st == 1 ? orc_pnp_count(pts, N, cam8, R, t, thr2, fused, NULL) : st;
    }
}

/* ---- rotation algebra + LM (independent restatement of pnp_host.cpp's definition) -------- */
static void skew3(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1]; S[3] = v[2]; S[4] = 0; S[5] = -v[0]; S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
static void mm3(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

void orc_rodrigues(const double* r, double* R, double* dR) {
    double th2 = dot(r, r), th = sqrt(th2), S[9], S2[9];
    skew3(r, S);
    if (th < 1e-12) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) + S[k];
        if (dR)
            for (int j = 0; j < 3; ++j) {
                double e[3] = {0, 0, 0};
                e[j] = 1;
                skew3(e, dR + 9 * j);
            }
        return;
    }
    double s = sin(th), c = cos(th);
    mm3(S, S, S2);
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0) + (s / th) * S[k] + ((1 - c) / th2) * S2[k];
    if (!dR) return;
    for (int j = 0; j < 3; ++j) {
        double w[3], rx[3], A[9];
        for (int i = 0; i < 3; ++i) w[i] = (i == j) - R[3 * i + j];
        rx[0] = r[1] * w[2] - r[2] * w[1];
        rx[1] = r[2] * w[0] - r[0] * w[2];
        rx[2] = r[0] * w[1] - r[1] * w[0];
        skew3(rx, A);
        for (int k = 0; k < 9; ++k) A[k] = (r[j] * S[k] + A[k]) / th2;
        mm3(A, R, dR + 9 * j);
    }
}

void orc_rodrigues_inv(const double* R, double* r) {
    double w[3] = {(R[7] - R[5]) * 0.5, (R[2] - R[6]) * 0.5, (R[3] - R[1]) * 0.5};
    double s = nrm(w), c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c < -1 ? -1 : (c > 1 ? 1 : c);
    if (s > 1e-7) {
        double th = atan2(s, c);
        for (int k = 0; k < 3; ++k) r[k] = w[k] * (th / s);
        return;
    }
    if (c > 0) {
        memcpy(r, w, sizeof(w));
        return;
    }
    int m = 0;
    for (int k = 1; k < 3; ++k)
        if (R[4 * k] > R[4 * m]) m = k;
    double ax[3];
    for (int k = 0; k < 3; ++k) ax[k] = (R[3 * m + k] + R[3 * k + m]) * 0.25 + (k == m ? 0.5 : 0.0);
    double n = nrm(ax);
    for (int k = 0; k < 3; ++k) ax[k] /= n;
    if (dot(ax, w) < 0)
        for (int k = 0; k < 3; ++k) ax[k] = -ax[k];
    double th = atan2(s, c);
    for (int k = 0; k < 3; ++k) r[k] = ax[k] * th;
}

/* sums over masked points: J^T J (6x6 full), J^T r, |r|^2 */
static double lm_sums(const float* pts, int N, const uint8_t* mask, const Cam* c, const double* q, int wantJ, double* A,
                      double* g) {
    double R[9], dR[27], S = 0;
    orc_rodrigues(q, R, wantJ ? dR : NULL);
    const double* t = q + 3;
    if (wantJ) { memset(A, 0, sizeof(double) * 36); memset(g, 0, sizeof(double) * 6); }
    for (int i = 0; i < N; ++i) {
        if (mask && !mask[i]) continue;
        const float* p = pts + 8 * (size_t)i;
        double X = p[0], Y = p[1], Z = p[2];
        double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0], Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        double iz = Zc != 0 ? 1.0 / Zc : 1.0, x = Xc * iz, y = Yc * iz;
        double r2 = x * x + y * y, r4 = r2 * r2, cd = 1.0 + c->k1 * r2 + c->k2 * r4;
        double xd = x * cd + c->p1 * (2.0 * x * y) + c->p2 * (r2 + 2.0 * x * x);
        double yd = y * cd + c->p1 * (r2 + 2.0 * y * y) + c->p2 * (2.0 * x * y);
        double ru = xd * c->fx + c->cx - (double)p[3], rv = yd * c->fy + c->cy - (double)p[4];
        S += ru * ru + rv * rv;
        if (!wantJ) continue;
        double dcr = c->k1 + 2.0 * c->k2 * r2;
        double dxdx = cd + x * dcr * 2.0 * x + 2.0 * c->p1 * y + 6.0 * c->p2 * x;
        double dxdy = x * dcr * 2.0 * y + 2.0 * c->p1 * x + 2.0 * c->p2 * y;
        double dydx = y * dcr * 2.0 * x + 2.0 * c->p1 * x + 2.0 * c->p2 * y;
        double dydy = cd + y * dcr * 2.0 * y + 6.0 * c->p1 * y + 2.0 * c->p2 * x;
        double du[3] = {c->fx * dxdx * iz, c->fx * dxdy * iz, c->fx * (-dxdx * x - dxdy * y) * iz};
        double dv[3] = {c->fy * dydx * iz, c->fy * dydy * iz, c->fy * (-dydx * x - dydy * y) * iz};
        double Ju[6], Jv[6];
        for (int j = 0; j < 3; ++j) {
            const double* d = dR + 9 * j;
            double gx = d[0] * X + d[1] * Y + d[2] * Z, gy = d[3] * X + d[4] * Y + d[5] * Z;
            double gz = d[6] * X + d[7] * Y + d[8] * Z;
            Ju[j] = du[0] * gx + du[1] * gy + du[2] * gz;
            Jv[j] = dv[0] * gx + dv[1] * gy + dv[2] * gz;
            Ju[3 + j] = du[j];
            Jv[3 + j] = dv[j];
        }
        for (int j = 0; j < 6; ++j) {
            for (int k = 0; k < 6; ++k) A[6 * j + k] += Ju[j] * Ju[k] + Jv[j] * Jv[k];
            g[j] += Ju[j] * ru + Jv[j] * rv;
        }
    }
    return S;
}

void orc_pnp_lm(const float* pts, int N, const uint8_t* mask, const double* cam8, double* rvec, double* t,
                int maxIters) {
    Cam c = cam_of(cam8);
    double p[6] = {rvec[0], rvec[1], rvec[2], t[0], t[1], t[2]}, A[36], g[6];
    double S = lm_sums(pts, N, mask, &c, p, 1, A, g), lambda = 1e-3;
    for (int it = 0; it < maxIters; ++it) {
        double M[36], rhs[6], d[6], q[6], dn = 0, pn = 0;
        memcpy(M, A, sizeof(M));
        for (int k = 0; k < 6; ++k) {
            M[7 * k] = A[7 * k] + lambda * (A[7 * k] > DBL_EPSILON ? A[7 * k] : DBL_EPSILON);
            rhs[k] = -g[k];
        }
        eig_pinv_apply(M, 6, rhs, d, NULL);
        for (int k = 0; k < 6; ++k) {
            q[k] = p[k] + d[k];
            dn = fabs(d[k]) > dn ? fabs(d[k]) : dn;
            pn = fabs(p[k]) > pn ? fabs(p[k]) : pn;
        }
        double Sq = lm_sums(pts, N, mask, &c, q, 0, NULL, NULL);
        if (Sq < S) {
            int stall = (S - Sq) <= FLT_EPSILON * S;
            memcpy(p, q, sizeof(p));
            lambda = lambda * 0.1 > 1e-12 ? lambda * 0.1 : 1e-12;
            S = lm_sums(pts, N, mask, &c, p, 1, A, g);
            if (stall || dn <= FLT_EPSILON * (pn + FLT_EPSILON)) break;
        } else {
            lambda *= 10;
            if (dn <= FLT_EPSILON * (pn + FLT_EPSILON) || lambda > 1e16) break;
        }
    }
    for (int k = 0; k < 3; ++k) { rvec[k] = p[k]; t[k] = p[3 + k]; }
}

/* Virtual visual servoing refinement, restating pnp_host.cpp's pnp_vvs definition
 * (solvePnPRefineVVS [ext]): normalised-plane error e = projection - undistorted observation,
 * interaction matrix L (camera twist (v, w)), v = -lambda pinv(L^T L) L^T e, cMo <- exp(v)^-1 cMo,
 * at most maxIters steps or |v| < FLT_EPSILON; sums in point order. */
void orc_pnp_vvs(const float* pts, int N, const double* cam8, double* rvec, double* t, int maxIters, double lambda) {
    Cam c = cam_of(cam8);
    double R[9];
    orc_rodrigues(rvec, R, NULL);
    for (int it = 0; it < maxIters; ++it) {
        double A[36], g[6], v[6];
        memset(A, 0, sizeof(A));
        memset(g, 0, sizeof(g));
        for (int i = 0; i < N; ++i) {
            const float* p = pts + 8 * (size_t)i;
            double X = p[0], Y = p[1], Z = p[2];
            double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0], Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
            double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
            double iz = Zc != 0 ? 1.0 / Zc : 1.0, x = Xc * iz, y = Yc * iz, xo, yo;
            undistort(&c, (double)p[3], (double)p[4], &xo, &yo);
            double ex = x - xo, ey = y - yo;
            double Lx[6] = {-iz, 0.0, x * iz, x * y, -(1.0 + x * x), y};
            double Ly[6] = {0.0, -iz, y * iz, 1.0 + y * y, -x * y, -x};
            for (int j = 0; j < 6; ++j) {
                for (int k = 0; k < 6; ++k) A[6 * j + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
                g[j] += Lx[j] * ex + Ly[j] * ey;
            }
        }
        eig_pinv_apply(A, 6, g, v, NULL);
        double vn = 0;
        for (int k = 0; k < 6; ++k) { v[k] = -lambda * v[k]; vn += v[k] * v[k]; }
        const double *u = v, *w = v + 3;
        double Rw[9], S[9], S2[9], V[9], tt[3], Rn[9], tn[3];
        orc_rodrigues(w, Rw, NULL);
        skew3(w, S);
        mm3(S, S, S2);
        double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2], th = sqrt(th2);
        double a = th < 1e-8 ? 0.5 : (1 - cos(th)) / th2;
        double b = th < 1e-8 ? 1.0 / 6.0 : (th - sin(th)) / (th2 * th);
        for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0 ? 1.0 : 0.0) + a * S[k] + b * S2[k];
        for (int i = 0; i < 3; ++i) tt[i] = V[3 * i] * u[0] + V[3 * i + 1] * u[1] + V[3 * i + 2] * u[2];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Rn[3 * i + j] = Rw[i] * R[j] + Rw[3 + i] * R[3 + j] + Rw[6 + i] * R[6 + j];
        for (int i = 0; i < 3; ++i)
            tn[i] = Rw[i] * (t[0] - tt[0]) + Rw[3 + i] * (t[1] - tt[1]) + Rw[6 + i] * (t[2] - tt[2]);
        memcpy(R, Rn, sizeof(R));
        memcpy(t, tn, sizeof(tn));
        if (sqrt(vn) < FLT_EPSILON) break;
    }
    orc_rodrigues_inv(R, rvec);
}

/* cvSolvePnPRansac semantics (seeded), solverKind `kind` (OpenCV solvePnPRansac):
 * P3P / AP3P (2, 5): AP3P on 4-point sets; every other kind EPnP on 5-point sets; npoints ==
 * model_points: one solve on all points; final pose: LM from the RANSAC pose for ITERATIVE (0),
 * EPnP on the inliers (float points as doubles) for the others.
 * Returns the inlier count (0 on failure); mask, rvec, tvec out. */
static int solve_pnp_ransac_impl(const double* img, const double* world, int N, const double* K9, const double* dist4,
                                 double thr, double conf, int maxIters, uint64_t seed, int flags, int kind,
                                 double* rvec, double* tvec, uint8_t* mask, int64_t* bestOut, int nthreads);

/* flags & ORC_FLAG_FAST_MINIMAL: the AP3P kinds take the real-root-finder quartic for the call */
int orc_solve_pnp_ransac_k(const double* img, const double* world, int N, const double* K9, const double* dist4,
                           double thr, double conf, int maxIters, uint64_t seed, int flags, int kind, double* rvec,
                           double* tvec, uint8_t* mask, int64_t* bestOut, int nthreads) {
    const int fast0 = orc_get_fast_minimal();
    if (flags & ORC_FLAG_FAST_MINIMAL) orc_set_fast_minimal(1);
    int r = solve_pnp_ransac_impl(img, world, N, K9, dist4, thr, conf, maxIters, seed, flags, kind, rvec, tvec, mask,
                                  bestOut, nthreads);
    orc_set_fast_minimal(fast0);
    return r;
}

static int solve_pnp_ransac_impl(const double* img, const double* world, int N, const double* K9, const double* dist4,
                                 double thr, double conf, int maxIters, uint64_t seed, int flags, int kind,
                                 double* rvec, double* tvec, uint8_t* mask, int64_t* bestOut, int nthreads) {
    if (bestOut) *bestOut = -1;
    if (N < 4) return 0;
    if (kind < 0 || kind > 5) kind = 0;
    const int ep = kind_epnp(kind);
    double cam8[8] = {K9[0], K9[4], K9[2], K9[5], dist4 ? dist4[0] : 0, dist4 ? dist4[1] : 0, dist4 ? dist4[2] : 0,
                      dist4 ? dist4[3] : 0};
    float* pts = (float*)calloc((size_t)N * 8, sizeof(float));
    for (int i = 0; i < N; ++i) {
        float* p = pts + 8 * (size_t)i;
        p[0] = (float)world[3 * i]; p[1] = (float)world[3 * i + 1]; p[2] = (float)world[3 * i + 2];
        p[3] = (float)img[2 * i]; p[4] = (float)img[2 * i + 1];
    }
    Cam c = cam_of(cam8);
    int fused = (flags & ORC_FLAG_FUSED_ERROR) != 0, result = 0;
    float thr2 = (float)(thr * thr);
    double R[9], t[3];
    if (N == 4 || (ep && N == 5)) {
        int ok = 1;
        if (N == 4) {
            double x[4], y[4], W[12];
            for (int i = 0; i < 4; ++i) {
                undistort(&c, (double)pts[8 * i + 3], (double)pts[8 * i + 4], &x[i], &y[i]);
                W[3 * i] = pts[8 * i]; W[3 * i + 1] = pts[8 * i + 1]; W[3 * i + 2] = pts[8 * i + 2];
            }
            ok = ap3p4_sel(&c, x, y, W, R, t);
        } else {
            orc_epnp5_f32(pts, cam8, R, t);
        }
        if (ok) {
            orc_rodrigues_inv(R, rvec);
            memcpy(tvec, t, sizeof(t));
            if (mask) memset(mask, 1, (size_t)N);
            result = N;
        }
        free(pts);
        return result;
    }
    int64_t niters = maxIters > 1 ? maxIters : 1;
    int* cnt = (int*)malloc(sizeof(int) * (size_t)niters);
    int* cvt = orc_cv_begin(flags, 0, NULL, N, ep ? 5 : 4, niters);
    orc_pnp_counts_k(pts, N, cam8, seed, 0, niters, thr2, fused, kind, cnt, nthreads);
    int bc = 0;
    int64_t best = orc_ransac_replay(cnt, niters, N, ep ? 5 : 4, conf, maxIters, (flags & ORC_FLAG_FIXED_ITERS) != 0,
                                     &bc);
    free(cnt);
    int st = best < 0 ? 0
             : ep     ? orc_pnp_hypothesis_epnp(pts, N, cam8, seed, best, R, t, NULL)
                      : orc_pnp_hypothesis(pts, N, cam8, seed, best, R, t, NULL);
    orc_cv_end(cvt);
    if (st == 1) {
        uint8_t* m = (uint8_t*)malloc((size_t)N);
        result = orc_pnp_count(pts, N, cam8, R, t, thr2, fused, m);
        orc_rodrigues_inv(R, rvec);
        memcpy(tvec, t, sizeof(t));
        if (!(flags & ORC_FLAG_NO_REFINE) && result > 0) {
            if (kind == 0) {
                orc_pnp_lm(pts, N, m, cam8, rvec, tvec, 20);
            } else {
                double* ii = (double*)malloc(sizeof(double) * 2 * (size_t)result);
                double* ww = (double*)malloc(sizeof(double) * 3 * (size_t)result);
                int k = 0;
                for (int i = 0; i < N; ++i)
                    if (m[i]) {
                        const float* p = pts + 8 * (size_t)i;
                        ii[2 * k] = p[3]; ii[2 * k + 1] = p[4];
                        ww[3 * k] = p[0]; ww[3 * k + 1] = p[1]; ww[3 * k + 2] = p[2];
                        ++k;
                    }
                double R2[9];
                orc_epnp_points(ii, ww, result, cam8, R2, tvec);
                orc_rodrigues_inv(R2, rvec);
                free(ii);
                free(ww);
            }
        }
        if (mask) memcpy(mask, m, (size_t)N);
        free(m);
        if (bestOut) *bestOut = best;
    }
    free(pts);
    return result;
}

int orc_solve_pnp_ransac(const double* img, const double* world, int N, const double* K9, const double* dist4,
                         double thr, double conf, int maxIters, uint64_t seed, int flags, double* rvec, double* tvec,
                         uint8_t* mask, int64_t* bestOut, int nthreads) {
    return orc_solve_pnp_ransac_k(img, world, N, K9, dist4, thr, conf, maxIters, seed, flags, 5, rvec, tvec, mask,
                                  bestOut, nthreads);
}

/* cvSolvePnP for the EPnP family (1, 3, 4: EPnP on all double points), ITERATIVE (0 and unknown
 * kinds: that pose, then LM over all points as float PnpPoints) and SQPNP (6: oracle_sqpnp.c).
 * Returns 1, or 0 for a non-finite pose / no SQPnP solution. */
int orc_solve_pnp(const double* img, const double* world, int N, const double* K9, const double* dist4, int kind,
                  double* rvec, double* tvec) {
    double cam8[8] = {K9[0], K9[4], K9[2], K9[5], dist4 ? dist4[0] : 0, dist4 ? dist4[1] : 0, dist4 ? dist4[2] : 0,
                      dist4 ? dist4[3] : 0};
    if (kind == 6) return orc_sqpnp(img, world, N, cam8, rvec, tvec) > 0;
    double R[9];
    orc_epnp_points(img, world, N, cam8, R, tvec);
    orc_rodrigues_inv(R, rvec);
    for (int k = 0; k < 3; ++k)
        if (!isfinite(rvec[k]) || !isfinite(tvec[k])) return 0;
    if (kind == 0 || kind < 0 || kind > 6) {
        float* pts = (float*)calloc((size_t)N * 8, sizeof(float));
        for (int i = 0; i < N; ++i) {
            float* p = pts + 8 * (size_t)i;
            p[0] = (float)world[3 * i]; p[1] = (float)world[3 * i + 1]; p[2] = (float)world[3 * i + 2];
            p[3] = (float)img[2 * i]; p[4] = (float)img[2 * i + 1];
        }
        orc_pnp_lm(pts, N, NULL, cam8, rvec, tvec, 20);
        free(pts);
    }
    return 1;
}
