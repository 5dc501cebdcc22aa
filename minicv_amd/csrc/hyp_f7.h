// hyp_f7.h — OpenCV FM_RANSAC's minimal solver (run7Point, calib3d fundam.cpp [ext]) for the
// MCV_FLAG_SEVEN_POINT mode of cvFindFundamentalMat: 7-point samples, up to 3 models each.
// Compiled for gfx950 (mcv_f7_generate) and the host (mcvHostF7 twin) with -ffp-contract=off.
//
// Restated: checkSubset = haveCollinearPoints on both 7-point sets (FMEstimatorCallback); the 7 x 9
// system (x2 x1, x2 y1, x2, y2 x1, y2 y1, y2, x1, y1, 1) in fp64 from the float points;
// SVDecomp(A, FULL_UV) = JacobiSVD with the two null-space rows completed by cv::RNG(0x12345678)
// (epnp.h jacobi_svd<9, 7, 9>), f1 = Vt row 7, f2 = Vt row 8, f1 -= f2; the cubic det(l f1 + f2)
// with run7Point's cofactor expansion; for each real root l: s = f1[8] l + f2[8], F = l f1 + f2
// scaled by 1/s (F[8] = 1) when |s| > DBL_EPSILON, else F[8] = 0.
// Deviation: cv::solveCubic's closed form (acos / cos / pow — not bit-reproducible between libm and
// the GPU) is replaced by the bracketed real-root finder of hyp_essential.h, whose roots agree to
// the last bits; the three-root case keeps solveCubic's order (x0 = -2 sqrt(Q) cos(theta / 3) is the
// smallest, x1 the largest, x2 the middle root), fewer roots come out ascending.
#pragma once

#include "hyp_fundamental.h"
#include "hyp_essential.h"   // e_poly_real_roots, epnp.h (jacobi_svd)

namespace mcv {

// run7Point on float points (image 1: x1, y1; image 2: x2, y2). Writes n <= 3 models to F, returns n.
MCV_HD int f_solve7(const float* x1, const float* y1, const float* x2, const float* y2, double (*F)[9]) {
    double A[9][9];
    for (int i = 0; i < 9; ++i)
        for (int k = 0; k < 9; ++k) A[i][k] = 0.0;
    for (int i = 0; i < 7; ++i) {
        const double X0 = x1[i], Y0 = y1[i], X1 = x2[i], Y1 = y2[i];
        A[i][0] = X1 * X0; A[i][1] = X1 * Y0; A[i][2] = X1;
        A[i][3] = Y1 * X0; A[i][4] = Y1 * Y0; A[i][5] = Y1;
        A[i][6] = X0; A[i][7] = Y0; A[i][8] = 1;
    }
    double w[7];
    jacobi_svd<9, 7, 9>(A, w, nullptr);
    double f1[9], f2[9];
    for (int i = 0; i < 9; ++i) {
        f2[i] = A[8][i];
        f1[i] = A[7][i] - f2[i];
    }
    double c[4];
    double t0 = f2[4] * f2[8] - f2[5] * f2[7];
    double t1 = f2[3] * f2[8] - f2[5] * f2[6];
    double t2 = f2[3] * f2[7] - f2[4] * f2[6];
    c[3] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2;
    c[2] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2 - f1[3] * (f2[1] * f2[8] - f2[2] * f2[7]) +
           f1[4] * (f2[0] * f2[8] - f2[2] * f2[6]) - f1[5] * (f2[0] * f2[7] - f2[1] * f2[6]) +
           f1[6] * (f2[1] * f2[5] - f2[2] * f2[4]) - f1[7] * (f2[0] * f2[5] - f2[2] * f2[3]) +
           f1[8] * (f2[0] * f2[4] - f2[1] * f2[3]);
    t0 = f1[4] * f1[8] - f1[5] * f1[7];
    t1 = f1[3] * f1[8] - f1[5] * f1[6];
    t2 = f1[3] * f1[7] - f1[4] * f1[6];
    c[1] = f2[0] * t0 - f2[1] * t1 + f2[2] * t2 - f2[3] * (f1[1] * f1[8] - f1[2] * f1[7]) +
           f2[4] * (f1[0] * f1[8] - f1[2] * f1[6]) - f2[5] * (f1[0] * f1[7] - f1[1] * f1[6]) +
           f2[6] * (f1[1] * f1[5] - f1[2] * f1[4]) - f2[7] * (f1[0] * f1[5] - f1[2] * f1[3]) +
           f2[8] * (f1[0] * f1[4] - f1[1] * f1[3]);
    c[0] = f1[0] * t0 - f1[1] * t1 + f1[2] * t2;
    bool finite = true;
    for (int k = 0; k < 4; ++k) finite = finite && isfinite(c[k]);
    if (!finite) return 0;
    const double asc[4] = {c[3], c[2], c[1], c[0]};   // l^0 .. l^3
    double r[10];
    const int n = e_poly_real_roots(asc, 3, r);
    if (n < 1 || n > 3) return 0;
    double roots[3] = {r[0], n > 1 ? r[1] : 0.0, n > 2 ? r[2] : 0.0};
    if (n == 3) { roots[1] = r[2]; roots[2] = r[1]; }   // solveCubic order: smallest, largest, middle
    for (int k = 0; k < n; ++k) {
        double lambda = roots[k], mu = 1.;
        const double s = f1[8] * roots[k] + f2[8];
        if (fabs(s) > kDblEpsilon) {
            mu = 1. / s;
            lambda *= mu;
            F[k][8] = 1.;
        } else {
            F[k][8] = 0.;
        }
        for (int i = 0; i < 8; ++i) F[k][i] = f1[i] * lambda + f2[i] * mu;
    }
    return n;
}

// One 7-point hypothesis: the number of models (0 = kStatusNoModel) or kStatusNoSample.
MCV_HD int f7_hypothesis(const float* pts4, int N, const Sampler& smp, uint64_t hyp, double (*F)[9], int* idx_out) {
    SubsetSrc<7> src(smp, hyp);
    float x1[7], y1[7], x2[7], y2[7];
    int idx[7];
    bool found = false;
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, idx);
        if (got < 0) break;
        if (got == 0) continue;
        for (int i = 0; i < 7; ++i) {
            const float* p = pts4 + 4 * (int64_t)idx[i];
            x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
        }
        if (!src.tabled() && (have_collinear_last<7>(x1, y1) || have_collinear_last<7>(x2, y2))) continue;
        found = true;   // search and solve apart (h_hypothesis): one solve pass per wave
        break;
    }
    if (!found) return kStatusNoSample;
    if (idx_out) for (int i = 0; i < 7; ++i) idx_out[i] = idx[i];
    return f_solve7(x1, y1, x2, y2, F);
}

}  // namespace mcv
