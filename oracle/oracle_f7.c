/*
 * oracle_f7.c — CPU restatement of OpenCV FM_RANSAC's 7-point path (calib3d fundam.cpp
 * run7Point + FMEstimatorCallback, RANSACPointSetRegistrator with up to 3 models per sample) for
 * the MCV_FLAG_SEVEN_POINT mode of cvFindFundamentalMat. TEST INFRASTRUCTURE ONLY (rules: oracle.c
 * header). OpenCV is absent here [ext]: parity with it is unpinned; the solver is pinned by exact
 * two-view geometry (tests/test_oracle.py: the true F is among the models of noise-free samples).
 * The null space comes from JacobiSVD with the cv::RNG completion rows (orc_jsvd), the cubic's
 * real roots from orc_poly_real_roots in solveCubic's order (smallest, largest, middle) — the
 * device code (minicv_amd/csrc/hyp_f7.h) must equal this file bit for bit.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "oracle_int.h"

#define F7_SLOTS 3

static int collinear7(const float* x, const float* y) {
    int i = 6;
    for (int j = 0; j < i; ++j) {
        double dx1 = (float)(x[j] - x[i]), dy1 = (float)(y[j] - y[i]);
        for (int k = 0; k < j; ++k) {
            double dx2 = (float)(x[k] - x[i]), dy2 = (float)(y[k] - y[i]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= (double)FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return 1;
        }
    }
    return 0;
}

/* run7Point: up to 3 models (F27 = 3 x 9, row-major each), returns their number. */
int orc_f7_solve(const float* x1, const float* y1, const float* x2, const float* y2, double* F27) {
    double U[81], w[7];
    memset(U, 0, sizeof(U));
    for (int i = 0; i < 7; ++i) {
        double X0 = x1[i], Y0 = y1[i], X1 = x2[i], Y1 = y2[i];
        double* a = U + 9 * i;
        a[0] = X1 * X0; a[1] = X1 * Y0; a[2] = X1;
        a[3] = Y1 * X0; a[4] = Y1 * Y0; a[5] = Y1;
        a[6] = X0; a[7] = Y0; a[8] = 1;
    }
    orc_jsvd(U, w, NULL, 9, 7, 9);
    double f1[9], f2[9];
    for (int i = 0; i < 9; ++i) {
        f2[i] = U[72 + i];
        f1[i] = U[63 + i] - f2[i];
    }
    double c[4], t0, t1, t2;
    t0 = f2[4] * f2[8] - f2[5] * f2[7];
    t1 = f2[3] * f2[8] - f2[5] * f2[6];
    t2 = f2[3] * f2[7] - f2[4] * f2[6];
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
    for (int k = 0; k < 4; ++k)
        if (!isfinite(c[k])) return 0;
    double asc[4] = {c[3], c[2], c[1], c[0]}, r[10];
    int n = orc_poly_real_roots(asc, 3, r);
    if (n < 1 || n > 3) return 0;
    double roots[3] = {r[0], n > 1 ? r[1] : 0.0, n > 2 ? r[2] : 0.0};
    if (n == 3) { roots[1] = r[2]; roots[2] = r[1]; }
    for (int k = 0; k < n; ++k) {
        double lambda = roots[k], mu = 1.;
        double s = f1[8] * roots[k] + f2[8];
        double* F = F27 + 9 * k;
        if (fabs(s) > DBL_EPSILON) {
            mu = 1. / s;
            lambda *= mu;
            F[8] = 1.;
        } else {
            F[8] = 0.;
        }
        for (int i = 0; i < 8; ++i) F[i] = f1[i] * lambda + f2[i] * mu;
    }
    return n;
}

int orc_f7_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F27, int* idx_out) {
    Stream st;
    st.seed = seed; st.hyp = (uint64_t)hyp; st.pos = 0;
    int idx[7];
    float x1[7], y1[7], x2[7], y2[7];
    for (int a = 0; a < ORC_MAX_ATTEMPTS; ++a) {
        if (!draw_distinct(&st, N, 7, idx)) continue;
        for (int i = 0; i < 7; ++i) {
            const float* p = pts4 + 4 * (size_t)idx[i];
            x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
        }
        if (collinear7(x1, y1) || collinear7(x2, y2)) continue;
        if (idx_out) memcpy(idx_out, idx, sizeof(idx));
        return orc_f7_solve(x1, y1, x2, y2, F27);
    }
    return ORC_NO_SAMPLE;
}

/* counts[3h + s]: inliers of model s of hypothesis begin + h, -1 no model, -2 (slot 0) sampler failure */
void orc_f7_counts(const float* pts4, int N, uint64_t seed, int64_t begin, int64_t count, float thr2, int kind,
                   int* out, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t h = 0; h < count; ++h) {
        double F[27];
        int n = orc_f7_hypothesis(pts4, N, seed, begin + h, F, NULL);
        for (int s = 0; s < F7_SLOTS; ++s)
            out[F7_SLOTS * h + s] = n > s ? orc_f_count(pts4, N, F + 9 * s, thr2, kind, NULL)
                                          : (s == 0 && n == ORC_NO_SAMPLE ? ORC_NO_SAMPLE : ORC_NO_MODEL);
    }
}

/* cvFindFundamentalMat with MCV_FLAG_SEVEN_POINT: N == 7 -> run7Point (first model); N >= 15 ->
   RANSAC over 7-point samples with the per-slot replay; F = the winning slot's model (no refit). */
int orc_find_fundamental7(const double* a, const double* b, int N, double thr, double conf, int maxIters,
                          uint64_t seed, int flags, int errorKind, double* F, uint8_t* mask, int64_t* bestSlotOut,
                          int nthreads) {
    if (mask) memset(mask, 0, (size_t)(N > 0 ? N : 0));
    if (bestSlotOut) *bestSlotOut = -1;
    if (N < 7 || (N != 7 && N < 15)) return 0;
    if (thr <= 0) thr = 3;
    float* pts = (float*)malloc(sizeof(float) * 4 * (size_t)N);
    for (int i = 0; i < N; ++i) {
        pts[4 * i] = (float)a[2 * i]; pts[4 * i + 1] = (float)a[2 * i + 1];
        pts[4 * i + 2] = (float)b[2 * i]; pts[4 * i + 3] = (float)b[2 * i + 1];
    }
    int count = 0;
    if (N == 7) {
        float x1[7], y1[7], x2[7], y2[7];
        double F27[27];
        for (int i = 0; i < 7; ++i) { x1[i] = pts[4 * i]; y1[i] = pts[4 * i + 1]; x2[i] = pts[4 * i + 2]; y2[i] = pts[4 * i + 3]; }
        if (orc_f7_solve(x1, y1, x2, y2, F27) > 0) {
            memcpy(F, F27, sizeof(double) * 9);
            count = 7;
            if (mask) memset(mask, 1, 7);
        }
    } else {
        const float thr2 = (float)(thr * thr);
        const int kind = (errorKind == 1 ? 2 : 0) + ((flags & ORC_FLAG_FUSED_ERROR) ? 0 : 1);
        int64_t niters = maxIters > 1 ? maxIters : 1;
        int* cnts = (int*)malloc(sizeof(int) * F7_SLOTS * (size_t)niters);
        int* cvt = orc_cv_begin(flags, 2, pts, N, 7, niters);
        orc_f7_counts(pts, N, seed, 0, niters, thr2, kind, cnts, nthreads);
        int bc = 0;
        int64_t best = orc_ransac_replay_slots(cnts, niters, F7_SLOTS, N, 7, conf, maxIters,
                                               (flags & ORC_FLAG_FIXED_ITERS) != 0, &bc);
        free(cnts);
        if (best >= 0) {
            double F27[27];
            orc_f7_hypothesis(pts, N, seed, best / F7_SLOTS, F27, NULL);
            memcpy(F, F27 + 9 * (best % F7_SLOTS), sizeof(double) * 9);
            count = orc_f_count(pts, N, F, thr2, kind, mask);
            if (bestSlotOut) *bestSlotOut = best;
        }
        orc_cv_end(cvt);
    }
    free(pts);
    return count;
}
