// hyp_fundamental.h — one RANSAC fundamental-matrix hypothesis (8-point minimal sets, north_star)
// and the fp64 epipolar errors of the inlier sweep. Compiled for gfx950 (mcv_f_generate /
// mcv_f_verify) and for the host (mcvHostHypothesis), with -ffp-contract=off: both sides round
// every operation identically (fp64 division and sqrt are IEEE correctly rounded on both).
//
// Semantics restated from OpenCV 4.x calib3d [ext, unverifiable here; SURVEY.md §8a row a9]:
//   run8Point: centre + scale each point set, linear system (x2,1)^T F (x1,1) = 0, null vector,
//   rank 2 by zeroing the smallest singular value, de-normalise, F *= 1/F22 if |F22| > FLT_EPSILON.
// Restated as run8Point: centroid + sqrt(2) / mean Euclidean distance normalisation, A = sum r r^T,
// cv::eigen (JacobiImpl_, jacobi_eig.h) with its eigenvalue check, rank 2 through SVD::compute
// (JacobiSVDImpl_) with w[2] = 0, T2^T F0 T1, F *= 1/F22.
// Errors: MCV_FERR_SAMPSON = first-order geometric error x2'Fx1^2 / (|Fx1|_12^2 + |F'x2|_12^2)
// (OpenCV EMEstimatorCallback::computeError's formula), MCV_FERR_EPIPOLAR = OpenCV
// FMEstimatorCallback::computeError (max of the two squared point-to-epipolar-line distances);
// both in fp64, cast to float, inlier iff err <= (float)thr^2.
#pragma once

#include "mcv_common.h"
#include "hyp_homography.h"   // det3, mat3_mul, have_collinear (point-set checks)
#include "epnp.h"             // jacobi_svd (JacobiSVDImpl_)
#include "jacobi_eig.h"       // eig9_jacobi (JacobiImpl_)

namespace mcv {

struct FModelD { double f[9]; };   // row-major F, x2^T F x1 = 0

// haveCollinearPoints(ms, count): last point against the lines through earlier pairs.
template <int M>
MCV_HD bool have_collinear_last(const float* px, const float* py) {
    const int i = M - 1;
#pragma unroll
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)(px[j] - px[i]);
        const double dy1 = (double)(py[j] - py[i]);
        for (int k = 0; k < j; ++k) {
            const double dx2 = (double)(px[k] - px[i]);
            const double dy2 = (double)(py[k] - py[i]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= (double)kFltEpsilon * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

// Cyclic Jacobi on a symmetric 3x3 (row-major, destroyed); V columns = eigenvectors. Fixed rotation
// order (0,1), (0,2), (1,2); at most 16 sweeps; stops when the off-diagonal part vanishes relative
// to the diagonal. Identical operation sequence on host and device (sqrt and division are IEEE).
MCV_HD void jacobi3(double* A, double* V) {
    for (int i = 0; i < 9; ++i) V[i] = (i == 0 || i == 4 || i == 8) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 16; ++sweep) {
        const double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        const double dg = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (!(off > dg * 1e-32)) break;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int p = r == 2 ? 1 : 0;
            const int q = r == 0 ? 1 : 2;
            const double apq = A[3 * p + q];
            if (apq == 0) continue;
            const double theta = (A[3 * q + q] - A[3 * p + p]) / (2 * apq);
            const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; ++k) {   // A <- A J
                const double akp = A[3 * k + p], akq = A[3 * k + q];
                A[3 * k + p] = c * akp - s * akq;
                A[3 * k + q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; ++k) {   // A <- J^T A
                const double apk = A[3 * p + k], aqk = A[3 * q + k];
                A[3 * p + k] = c * apk - s * aqk;
                A[3 * q + k] = s * apk + c * aqk;
            }
            for (int k = 0; k < 3; ++k) {   // V <- V J
                const double vkp = V[3 * k + p], vkq = V[3 * k + q];
                V[3 * k + p] = c * vkp - s * vkq;
                V[3 * k + q] = s * vkp + c * vkq;
            }
        }
    }
}

// run8Point's rank-2 step: SVD::compute(F0, w, U, Vt) — JacobiSVDImpl_ on F0^T (jacobi_svd, epnp.h),
// U = the transposed left-vector rows — then w[2] = 0 and F0 = U * diag(w) * Vt as two Matx products
// (s = 0; s += a(i,k) b(k,j) in k order).
MCV_HD void f_rank2(double* F) {
    double At[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) At[i][j] = F[3 * j + i];
    double w[3], Vt[3][3];
    jacobi_svd<3, 3>(At, w, Vt);
    w[2] = 0.;
    double UD[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0;
            for (int k = 0; k < 3; ++k) acc += At[k][i] * (k == j ? w[j] : 0.0);   // U(i, k) = At[k][i]
            UD[i][j] = acc;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0;
            for (int k = 0; k < 3; ++k) acc += UD[i][k] * Vt[k][j];
            F[3 * i + j] = acc;
        }
}

// run8Point's normalising transform of a point set: centroid (the sum times t = 1 / count), mean
// Euclidean distance to it (norm(Point2d) summed, times t), scale = sqrt(2) / that distance, the same
// for both axes. T = [[s, 0, -s cx], [0, s, -s cy], [0, 0, 1]]. false when the distance is below
// FLT_EPSILON (run8Point returns 0).
template <int M>
MCV_HD bool f_norm(const float* x, const float* y, double* cx, double* cy, double* sx, double* sy) {
    double mx = 0, my = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) { mx += (double)x[i]; my += (double)y[i]; }
    const double t = 1. / M;
    mx *= t;
    my *= t;
    double sc = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        const double dx = (double)x[i] - mx, dy = (double)y[i] - my;
        sc += sqrt(dx * dx + dy * dy);
    }
    sc *= t;
    if (sc < (double)kFltEpsilon) return false;
    sc = sqrt(2.) / sc;
    *cx = mx; *cy = my;
    *sx = sc; *sy = sc;
    return true;
}

// De-normalise F = T2^T F0 T1 and scale F22 to 1 when |F22| > FLT_EPSILON (run8Point).
MCV_HD bool f_denormalize(const double* F0, double c1x, double c1y, double s1x, double s1y, double c2x, double c2y,
                          double s2x, double s2y, double* F) {
    const double T1[9] = {s1x, 0, -s1x * c1x, 0, s1y, -s1y * c1y, 0, 0, 1};
    const double T2t[9] = {s2x, 0, 0, 0, s2y, 0, -s2x * c2x, -s2y * c2y, 1};
    double T[9];
    mat3_mul(T2t, F0, T);
    mat3_mul(T, T1, F);
    if (fabs(F[8]) > (double)kFltEpsilon) {
        const double s = 1. / F[8];
        for (int i = 0; i < 9; ++i) F[i] = F[i] * s;
    }
    bool ok = true;
    for (int i = 0; i < 9; ++i) ok = ok && isfinite(F[i]);
    return ok;
}

// MCV_FLAG_FAST_MINIMAL (opt-in): the 8x9 system's null vector with f22 = 1 by Gaussian elimination
// (partial pivoting) instead of the eigen-solve of A^T A (no eigenvalue check), then rank 2 and
// de-normalisation as below.
MCV_HD bool f_solve8_elim(const float* x1, const float* y1, const float* x2, const float* y2, double* F) {
    double c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y;
    if (!f_norm<8>(x1, y1, &c1x, &c1y, &s1x, &s1y) || !f_norm<8>(x2, y2, &c2x, &c2y, &s2x, &s2y)) return false;
    double a[8][9];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double X1 = ((double)x1[i] - c1x) * s1x, Y1 = ((double)y1[i] - c1y) * s1y;
        const double X2 = ((double)x2[i] - c2x) * s2x, Y2 = ((double)y2[i] - c2y) * s2y;
        a[i][0] = X2 * X1; a[i][1] = X2 * Y1; a[i][2] = X2;
        a[i][3] = Y2 * X1; a[i][4] = Y2 * Y1; a[i][5] = Y2;
        a[i][6] = X1; a[i][7] = Y1; a[i][8] = -1.0;   // f22 = 1 moved to the right-hand side
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int c = 0; c < 8; ++c) {
        int p = c;
        double best = fabs(a[c][c]);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int r = c + 1; r < 8; ++r) {
            const double v = fabs(a[r][c]);
            if (v > best) { best = v; p = r; }
        }
        if (!(best > 0)) return false;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int r = c + 1; r < 8; ++r) {
            const bool sw = (r == p);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int k = c; k < 9; ++k) {
                const double t = a[c][k];
                a[c][k] = sw ? a[r][k] : t;
                a[r][k] = sw ? t : a[r][k];
            }
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int r = c + 1; r < 8; ++r) {
            const double f = a[r][c] / a[c][c];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int k = c + 1; k < 9; ++k) a[r][k] = a[r][k] - f * a[c][k];
        }
    }
    double h[8];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 7; i >= 0; --i) {
        double s = a[i][8];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int k = i + 1; k < 8; ++k) s = s - a[i][k] * h[k];
        h[i] = s / a[i][i];
    }
    double F0[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
    f_rank2(F0);
    return f_denormalize(F0, c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y, F);
}

// Minimal 8-point solve = run8Point on the sample; a = image-1 points (x1, y1), b = image-2 points
// (x2, y2): normalisation, A += r r^T (points in order, upper triangle: A is symmetric exactly),
// cv::eigen (eig9_jacobi), the eigenvalue check (the first 8 sorted eigenvalues must not fall below
// DBL_EPSILON in magnitude, else run8Point returns 0), F0 = the last eigenvector, rank 2,
// de-normalisation.
template <class WS>
MCV_HD bool f_solve8(const float* x1, const float* y1, const float* x2, const float* y2, double* F, WS& ws,
                     bool fast = false) {
    if (fast) return f_solve8_elim(x1, y1, x2, y2, F);
    double c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y;
    if (!f_norm<8>(x1, y1, &c1x, &c1y, &s1x, &s1y) || !f_norm<8>(x2, y2, &c2x, &c2y, &s2x, &s2y)) return false;
    double dg[9], up[36];
#pragma unroll
    for (int e = 0; e < 36; ++e) up[e] = 0.0;
#pragma unroll
    for (int e = 0; e < 9; ++e) dg[e] = 0.0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const double X1 = ((double)x1[i] - c1x) * s1x, Y1 = ((double)y1[i] - c1y) * s1y;
        const double X2 = ((double)x2[i] - c2x) * s2x, Y2 = ((double)y2[i] - c2y) * s2y;
        const double r[9] = {X2 * X1, X2 * Y1, X2, Y2 * X1, Y2 * Y1, Y2, X1, Y1, 1.0};
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            dg[j] += r[j] * r[j];
#pragma unroll
            for (int k = j + 1; k < 9; ++k) up[eig_tri(j, k)] += r[j] * r[k];
        }
    }
    bool fin = true;
#pragma unroll
    for (int e = 0; e < 36; ++e) {
        fin = fin && isfinite(up[e]);
        ws[kEigA + e] = up[e];
    }
#pragma unroll
    for (int e = 0; e < 9; ++e) {
        fin = fin && isfinite(dg[e]);
        ws[kEigW + e] = dg[e];
    }
    if (!fin) return false;
    double w[9];
    const int r = eig9_jacobi(ws, w, 8);
    bool rank8 = true;
#pragma unroll
    for (int i = 0; i < 8; ++i) rank8 = rank8 && !(fabs(w[i]) < kDblEpsilon);
    if (!rank8) return false;
    double F0[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) F0[j] = ws[kEigV + 9 * r + j];
    f_rank2(F0);
    return f_denormalize(F0, c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y, F);
}

// One hypothesis: 1 (model), kStatusNoModel, kStatusNoSample.
template <class WS>
MCV_HD int f_hypothesis(const float* pts4, int N, const Sampler& smp, uint64_t hyp, double* F, int* idx_out, WS& ws,
                        bool fast = false) {
    SubsetSrc<8> src(smp, hyp);
    float x1[8], y1[8], x2[8], y2[8];
    int idx[8];
    bool found = false;
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, idx);
        if (got < 0) break;
        if (got == 0) continue;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float* p = pts4 + 4 * (int64_t)idx[i];
            x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
        }
        if (!src.tabled() && (have_collinear_last<8>(x1, y1) || have_collinear_last<8>(x2, y2))) continue;
        found = true;   // search and solve apart (h_hypothesis): one solve pass per wave
        break;
    }
    if (!found) return kStatusNoSample;
    if (idx_out) for (int i = 0; i < 8; ++i) idx_out[i] = idx[i];
    return f_solve8(x1, y1, x2, y2, F, ws, fast) ? 1 : kStatusNoModel;
}

// ---- errors (fp64, cast to float) ----------------------------------------------------------
// Sampson numerator c^2 and denominator, fused (default): Fx1 = (fma(f0,x1,fma(f1,y1,f2)), ...),
// F^T x2 likewise, c = fma(x2, Fx1_0, fma(y2, Fx1_1, Fx1_2)), den = fma(a,a,fma(b,b,fma(g,g,h*h))).
MCV_HD void f_sampson_parts_fused(const double* F, double x1, double y1, double x2, double y2, double& c2,
                                  double& den) {
    const double ax = fma(F[0], x1, fma(F[1], y1, F[2]));
    const double ay = fma(F[3], x1, fma(F[4], y1, F[5]));
    const double az = fma(F[6], x1, fma(F[7], y1, F[8]));
    const double bx = fma(F[0], x2, fma(F[3], y2, F[6]));
    const double by = fma(F[1], x2, fma(F[4], y2, F[7]));
    const double c = fma(x2, ax, fma(y2, ay, az));
    den = fma(ax, ax, fma(ay, ay, fma(bx, bx, by * by)));
    c2 = c * c;
}

// Sampson parts, op by op (OpenCV Matx*Vec / dot order).
MCV_HD void f_sampson_parts(const double* F, double x1, double y1, double x2, double y2, double& c2, double& den) {
    const double ax = F[0] * x1 + F[1] * y1 + F[2] * 1.;
    const double ay = F[3] * x1 + F[4] * y1 + F[5] * 1.;
    const double az = F[6] * x1 + F[7] * y1 + F[8] * 1.;
    const double bx = F[0] * x2 + F[3] * y2 + F[6] * 1.;
    const double by = F[1] * x2 + F[4] * y2 + F[7] * 1.;
    const double c = x2 * ax + y2 * ay + 1. * az;
    const double a2 = ax * ax, b2 = ay * ay, c2_ = bx * bx, d2 = by * by;
    den = a2 + b2 + c2_ + d2;
    c2 = c * c;
}

// Certified inlier test of a Sampson error without the fp64 division (the sweep's hot path):
// err = (float)(c2 / den) <= thr2  is decided exactly by
//   c2 < den * lo  -> inlier,   c2 > den * hi  -> outlier,   otherwise (or den < 2^-960) undecided,
// with mid = the double midpoint between thr2 and the next float up, lo = mid (1 - 2^-49),
// hi = mid (1 + 2^-49): a correctly rounded quotient below mid(1 - 2^-50) rounds (to double, then
// to float) to <= thr2, one above mid(1 + 2^-50) to > thr2, and the products' rounding (2^-53
// relative while den * lo stays normal) cannot cross those margins. Undecided lanes (probability
// ~1e-14 per evaluation) take the exact division.
struct SampsonCut { double lo, hi; };
static const double kSampsonDenMin = 0x1p-960;

MCV_HD SampsonCut sampson_cut(float thr2) {
    SampsonCut c;
    c.lo = -1.0;              // disabled: nothing certified inside ...
    c.hi = __builtin_inf();   // ... or outside -> every evaluation divides
    if (!(thr2 >= 0.0f) || !(thr2 <= 1e30f)) return c;
    const float nx = nextafterf(thr2, __builtin_inff());
    const double mid = ((double)thr2 + (double)nx) * 0.5;   // exact in fp64
    if (!(mid >= 0x1p-60)) return c;
    c.lo = mid * (1.0 - 0x1p-49);
    c.hi = mid * (1.0 + 0x1p-49);
    return c;
}

// Sampson, fused (default): e = (float)(c*c/den).
MCV_HD float f_err_sampson_fused(const double* F, double x1, double y1, double x2, double y2) {
    const double ax = fma(F[0], x1, fma(F[1], y1, F[2]));
    const double ay = fma(F[3], x1, fma(F[4], y1, F[5]));
    const double az = fma(F[6], x1, fma(F[7], y1, F[8]));
    const double bx = fma(F[0], x2, fma(F[3], y2, F[6]));
    const double by = fma(F[1], x2, fma(F[4], y2, F[7]));
    const double c = fma(x2, ax, fma(y2, ay, az));
    const double den = fma(ax, ax, fma(ay, ay, fma(bx, bx, by * by)));
    return (float)(c * c / den);
}

// Sampson, op by op (OpenCV Matx*Vec / dot order).
MCV_HD float f_err_sampson(const double* F, double x1, double y1, double x2, double y2) {
    const double ax = F[0] * x1 + F[1] * y1 + F[2] * 1.;
    const double ay = F[3] * x1 + F[4] * y1 + F[5] * 1.;
    const double az = F[6] * x1 + F[7] * y1 + F[8] * 1.;
    const double bx = F[0] * x2 + F[3] * y2 + F[6] * 1.;
    const double by = F[1] * x2 + F[4] * y2 + F[7] * 1.;
    const double c = x2 * ax + y2 * ay + 1. * az;
    const double a2 = ax * ax, b2 = ay * ay, c2 = bx * bx, d2 = by * by;
    return (float)(c * c / (a2 + b2 + c2 + d2));
}

// OpenCV FMEstimatorCallback::computeError, fused.
MCV_HD float f_err_epipolar_fused(const double* F, double x1, double y1, double x2, double y2) {
    double a = fma(F[0], x1, fma(F[1], y1, F[2]));
    double b = fma(F[3], x1, fma(F[4], y1, F[5]));
    double c = fma(F[6], x1, fma(F[7], y1, F[8]));
    const double s2 = 1. / fma(a, a, b * b);
    const double d2 = fma(x2, a, fma(y2, b, c));
    a = fma(F[0], x2, fma(F[3], y2, F[6]));
    b = fma(F[1], x2, fma(F[4], y2, F[7]));
    c = fma(F[2], x2, fma(F[5], y2, F[8]));
    const double s1 = 1. / fma(a, a, b * b);
    const double d1 = fma(x1, a, fma(y1, b, c));
    const double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
    return (float)(e1 < e2 ? e2 : e1);
}

// OpenCV FMEstimatorCallback::computeError, op by op.
MCV_HD float f_err_epipolar(const double* F, double x1, double y1, double x2, double y2) {
    double a = F[0] * x1 + F[1] * y1 + F[2];
    double b = F[3] * x1 + F[4] * y1 + F[5];
    double c = F[6] * x1 + F[7] * y1 + F[8];
    const double s2 = 1. / (a * a + b * b);
    const double d2 = x2 * a + y2 * b + c;
    a = F[0] * x2 + F[3] * y2 + F[6];
    b = F[1] * x2 + F[4] * y2 + F[7];
    c = F[2] * x2 + F[5] * y2 + F[8];
    const double s1 = 1. / (a * a + b * b);
    const double d1 = x1 * a + y1 * b + c;
    const double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
    return (float)(e1 < e2 ? e2 : e1);   // std::max(d1*d1*s1, d2*d2*s2)
}

// Dummy model for padded / invalid sweep slots: den = 1, c^2 >= 1e20 -> certified outlier everywhere.
MCV_HD double f_dummy_model(int j) { return j == 2 ? 1.0 : (j == 8 ? 1e10 : 0.0); }


// Error selector: kind = errorKind * 2 + unfused.
MCV_HD float f_error(int kind, const double* F, double x1, double y1, double x2, double y2) {
    switch (kind) {
        case 0: return f_err_sampson_fused(F, x1, y1, x2, y2);
        case 1: return f_err_sampson(F, x1, y1, x2, y2);
        case 2: return f_err_epipolar_fused(F, x1, y1, x2, y2);
        default: return f_err_epipolar(F, x1, y1, x2, y2);
    }
}

#if defined(__HIPCC__)
// One sweep step for K models at one correspondence per lane: inlier ballots into cnt[k].
// KIND 0/1 (Sampson) use the certified division-free test: per model two lane masks (certified
// inliers, undecided lanes) straight from the fp64 compares, and ONE wave-uniform branch for the
// whole step into the exact division of the undecided lanes (rare). Keeping the fallback out of
// the per-model path leaves the common case as compares + scalar mask logic, with no exec-mask
// round trips through VGPRs. KIND 2/3 (epipolar) evaluate f_error directly.
template <int K, int KIND>
__device__ __forceinline__ void f_sweep_point(const double (&fm)[K][9], double x1, double y1, double x2, double y2,
                                              bool v, float thr2, double lo, double hi, uint32_t (&cnt)[K]) {
    if constexpr (KIND <= 1) {
        // each compare straight into a lane mask (v_cmp -> SGPR pair), combined by scalar ops
        const uint64_t vm = __builtin_amdgcn_ballot_w64(v);
        uint64_t inm[K], amb[K], anyAmb = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double c2, den;
            if constexpr (KIND == 0) f_sampson_parts_fused(fm[k], x1, y1, x2, y2, c2, den);
            else f_sampson_parts(fm[k], x1, y1, x2, y2, c2, den);
            const uint64_t ok = __builtin_amdgcn_ballot_w64(den >= kSampsonDenMin);
            const uint64_t in = ok & __builtin_amdgcn_ballot_w64(c2 < den * lo);
            const uint64_t out = ok & __builtin_amdgcn_ballot_w64(c2 > den * hi);
            inm[k] = vm & in;
            amb[k] = vm & ~(in | out);
            anyAmb |= amb[k];
        }
        if (__builtin_expect(anyAmb != 0, 0)) {
            const uint64_t me = 1ull << (__lane_id() & 63);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (amb[k] == 0) continue;
                double c2, den;
                if constexpr (KIND == 0) f_sampson_parts_fused(fm[k], x1, y1, x2, y2, c2, den);
                else f_sampson_parts(fm[k], x1, y1, x2, y2, c2, den);
                inm[k] |= __builtin_amdgcn_ballot_w64((amb[k] & me) != 0 && (float)(c2 / den) <= thr2);
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) cnt[k] += (uint32_t)__popcll(inm[k]);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k)
            cnt[k] += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(v && f_error(KIND, fm[k], x1, y1, x2, y2) <= thr2));
    }
}
#endif

}  // namespace mcv
