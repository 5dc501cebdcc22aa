/*
 * oracle.c — CPU restatement of MiniCV's matching + RANSAC hot path. TEST INFRASTRUCTURE ONLY:
 * imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
 * product (libMiniCVNative.so has no CPU fallback).
 *
 * PARITY STATUS: "parity unpinned" with respect to OpenCV. The reference delegates every
 * computation of this path to third-party OpenCV (calib3d / features2d; call sites
 * /root/reference/src/MiniCVNative/MiniCVNative.cpp:125,177,204), which is not installed in this
 * container, is version-unpinned (vcpkg HEAD, /root/reference/buildnative.sh:15,48) and cannot be
 * built offline; the reference ships no test that pins a number (/root/reference/src/Test/
 * Program.fs:57-97 only prints detector counts). This file restates the OpenCV 4.x algorithms
 * [ext, from the published source, unverifiable here] and is pinned instead by: Random123's
 * Philox4x32-10 known-answer vectors, analytic known-answer problems (exact homographies /
 * fundamental matrices, including the cvTest matrix MiniCVNative.cpp:506), cross-checks against
 * independent numpy/scipy algebra, and committed golden fixtures (tests/golden/).
 *
 * It is written independently of minicv_amd/csrc (no shared header) but to the same definition,
 * operation by operation, so that per-hypothesis models and inlier masks agree bit for bit.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off: no FMA contraction, IEEE double/float).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include <limits.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------
 * Philox4x32-10 (Salmon, Moraes, Dror, Shaw — "Parallel random numbers: as easy as 1, 2, 3").
 * ---------------------------------------------------------------------------------------- */
void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#include "oracle_int.h"

uint32_t stream_next(Stream* st) {
    if ((st->pos & 3) == 0) {
        uint32_t c[4] = {(uint32_t)(st->pos >> 2), (uint32_t)st->hyp, (uint32_t)(st->hyp >> 32), 0x4D435631u};
        uint32_t k[2] = {(uint32_t)st->seed, (uint32_t)(st->seed >> 32)};
        orc_philox(c, k, st->buf);
    }
    return st->buf[st->pos++ & 3];
}

int stream_uniform(Stream* st, int n) { return (int)(((uint64_t)stream_next(st) * (uint32_t)n) >> 32); }


/* MCV_FLAG_CV_SAMPLER: while a table is installed (orc_cv_begin), every hypothesis takes its sample
 * from row `hyp` of OpenCV's own getSubset stream (orc_cv_subsets below) instead of Philox. A row
 * with -1 in column 0 (getSubset gave up) makes draw_distinct fail, so the attempt loop ends in
 * ORC_NO_SAMPLE; an accepted row passes the callers' subset checks again (the builder ran them). */
static const int* g_cv_table = NULL;

/* getSubset's inner loop: m distinct indices, duplicates redrawn (bounded). */
int draw_distinct(Stream* st, int N, int m, int* idx) {
    if (g_cv_table) {
        const int* row = g_cv_table + (size_t)m * st->hyp;
        for (int i = 0; i < m; ++i) idx[i] = row[i];
        return row[0] >= 0;
    }
    for (int i = 0; i < m; ++i) {
        int v = stream_uniform(st, N), tries = 0;
        for (;;) {
            int dup = 0;
            for (int j = 0; j < i; ++j) dup |= (idx[j] == v);
            if (!dup) break;
            if (++tries >= ORC_MAX_REDRAW) return 0;
            v = stream_uniform(st, N);
        }
        idx[i] = v;
    }
    return 1;
}

/* ------------------------------------------------------------------------------------------
 * Homography. OpenCV 4.x calib3d/src/fundam.cpp HomographyEstimatorCallback [ext].
 * ---------------------------------------------------------------------------------------- */
static double det3(double a00, double a01, double a02, double a10, double a11, double a12, double a20, double a21,
                   double a22) {
    return a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
}

/* haveCollinearPoints(m, count=4): last point vs lines through earlier pairs. */
static int collinear_last(const float* x, const float* y, int count) {
    int i = count - 1;
    for (int j = 0; j < i; ++j) {
        double dx1 = (double)(float)(x[j] - x[i]), dy1 = (double)(float)(y[j] - y[i]);
        for (int k = 0; k < j; ++k) {
            double dx2 = (double)(float)(x[k] - x[i]), dy2 = (double)(float)(y[k] - y[i]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= (double)FLT_EPSILON * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return 1;
        }
    }
    return 0;
}

static int h_subset_ok(const float* sx, const float* sy, const float* dx, const float* dy) {
    static const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    if (collinear_last(sx, sy, 4) || collinear_last(dx, dy, 4)) return 0;
    int negative = 0;
    for (int i = 0; i < 4; ++i) {
        int a = tt[i][0], b = tt[i][1], c = tt[i][2];
        double dA = det3(sx[a], sy[a], 1., sx[b], sy[b], 1., sx[c], sy[c], 1.);
        double dB = det3(dx[a], dy[a], 1., dx[b], dy[b], 1., dx[c], dy[c], 1.);
        negative += dA * dB < 0;
    }
    return negative == 0 || negative == 4;
}

/* ------------------------------------------------------------------------------------------
 * OpenCV's sample stream [ext: OpenCV 4.x core cv::RNG, calib3d ptsetreg.cpp
 * RANSACPointSetRegistrator::run / getSubset], restated independently of minicv_amd/csrc/cv_sampler.cpp:
 * one RNG((uint64)-1) per run; per hypothesis up to 10000 attempts, each drawing m indices with
 * rng.uniform(0, N) and redrawing an index equal to an earlier one of the same attempt, then the
 * callback's checkSubset (check 1: the homography callback's collinearity + orientation test,
 * 2: the fundamental callbacks' collinearity test on both point sets, 0: none — EM / PnP).
 * out[m*h .. m*h+m) = the accepted subset of hypothesis h; -1 from the first hypothesis whose
 * getSubset failed on. Returns the number of rows filled with accepted subsets.
 * ---------------------------------------------------------------------------------------- */
static uint32_t cvrng_next(uint64_t* s) {
    *s = (uint64_t)(uint32_t)*s * 4164903690u + (*s >> 32);
    return (uint32_t)*s;
}

int64_t orc_cv_subsets(int check, const float* pts4, int N, int m, int64_t rows, int* out) {
    uint64_t state = ~(uint64_t)0;
    int64_t h = 0;
    for (; h < rows; ++h) {
        int* idx = out + (size_t)m * h;
        int ok = 0;
        for (int attempt = 0; attempt < ORC_MAX_ATTEMPTS && !ok; ++attempt) {
            for (int i = 0; i < m; ++i) {
                int dup;
                do {
                    idx[i] = (int)(cvrng_next(&state) % (uint32_t)N);
                    dup = 0;
                    for (int j = 0; j < i; ++j) dup |= idx[j] == idx[i];
                } while (dup);
            }
            if (check == 0) { ok = 1; break; }
            float x1[8], y1[8], x2[8], y2[8];
            for (int i = 0; i < m; ++i) {
                const float* p = pts4 + 4 * (size_t)idx[i];
                x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
            }
            ok = check == 1 ? h_subset_ok(x1, y1, x2, y2) : !(collinear_last(x1, y1, m) || collinear_last(x2, y2, m));
        }
        if (!ok) break;
    }
    for (int64_t r = h; r < rows; ++r)
        for (int i = 0; i < m; ++i) out[(size_t)m * r + i] = -1;
    return h;
}

/* Install OpenCV's stream for a run when flags ask for it (NULL otherwise); orc_cv_end removes it. */
int* orc_cv_begin(int flags, int check, const float* pts4, int N, int m, int64_t rows) {
    if (!(flags & ORC_FLAG_CV_SAMPLER) || rows <= 0) return NULL;
    int* t = (int*)malloc(sizeof(int) * (size_t)m * (size_t)rows);
    orc_cv_subsets(check, pts4, N, m, rows, t);
    g_cv_table = t;
    return t;
}
void orc_cv_end(int* t) {
    if (!t) return;
    g_cv_table = NULL;
    free(t);
}

static void mul33(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

/* The minimal solver of the H / 8-point F hypotheses: 0 = OpenCV's eigen path (default), 1 = the
 * MCV_FLAG_FAST_MINIMAL elimination. Test infrastructure: set before the (OpenMP) calls. */
static int g_fast_minimal = 0;
void orc_set_fast_minimal(int v) { g_fast_minimal = v; }
int orc_get_fast_minimal(void) { return g_fast_minimal; }

/* MCV_FLAG_FAST_MINIMAL (opt-in): runKernel's normalisation, then the 8x8 system (h22 = 1) by Gaussian
 * elimination with partial pivoting (first maximum), back substitution, de-normalisation,
 * H *= 1/H22. Returns 0 when degenerate. */
static int h_solve4_elim(const float* sx, const float* sy, const float* dx, const float* dy, double* H) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, smx = 0, smy = 0, sMx = 0, sMy = 0;
    for (int i = 0; i < 4; ++i) { cmx += dx[i]; cmy += dy[i]; cMx += sx[i]; cMy += sy[i]; }
    cmx /= 4; cmy /= 4; cMx /= 4; cMy /= 4;
    for (int i = 0; i < 4; ++i) {
        smx += fabs(dx[i] - cmx); smy += fabs(dy[i] - cmy);
        sMx += fabs(sx[i] - cMx); sMy += fabs(sy[i] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return 0;
    smx = 4 / smx; smy = 4 / smy; sMx = 4 / sMx; sMy = 4 / sMy;
    double a[8][9];
    for (int i = 0; i < 4; ++i) {
        double x = (dx[i] - cmx) * smx, y = (dy[i] - cmy) * smy;
        double X = (sx[i] - cMx) * sMx, Y = (sy[i] - cMy) * sMy;
        double r0[9] = {X, Y, 1, 0, 0, 0, -(x * X), -(x * Y), x};
        double r1[9] = {0, 0, 0, X, Y, 1, -(y * X), -(y * Y), y};
        memcpy(a[2 * i], r0, sizeof(r0));
        memcpy(a[2 * i + 1], r1, sizeof(r1));
    }
    for (int c = 0; c < 8; ++c) {
        int p = c;
        double best = fabs(a[c][c]);
        for (int r = c + 1; r < 8; ++r)
            if (fabs(a[r][c]) > best) { best = fabs(a[r][c]); p = r; }
        if (!(best > 0)) return 0;
        if (p != c)
            for (int k = c; k < 9; ++k) { double t = a[c][k]; a[c][k] = a[p][k]; a[p][k] = t; }
        for (int r = c + 1; r < 8; ++r) {
            double f = a[r][c] / a[c][c];
            for (int k = c + 1; k < 9; ++k) a[r][k] = a[r][k] - f * a[c][k];
        }
    }
    double h[8];
    for (int i = 7; i >= 0; --i) {
        double s = a[i][8];
        for (int k = i + 1; k < 8; ++k) s = s - a[i][k] * h[k];
        h[i] = s / a[i][i];
    }
    double Hn[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
    double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9];
    mul33(invHnorm, Hn, T);
    mul33(T, Hnorm2, H);
    double s = 1. / H[8];
    for (int i = 0; i < 9; ++i) {
        H[i] = H[i] * s;
        if (!isfinite(H[i])) return 0;
    }
    return 1;
}

/* Minimal 4-point solve = HomographyEstimatorCallback::runKernel on the sample (h_run_kernel_xy,
 * below: LtL, cv::eigen, de-normalisation, 1/H22). 0 when the scales vanish or H is not finite. */
static int h_run_kernel_xy(const float* sx, const float* sy, const float* dx, const float* dy, int count, double* H);
static int h_solve4(const float* sx, const float* sy, const float* dx, const float* dy, double* H) {
    if (g_fast_minimal) return h_solve4_elim(sx, sy, dx, dy, H);
    if (!h_run_kernel_xy(sx, sy, dx, dy, 4, H)) return 0;
    for (int i = 0; i < 9; ++i)
        if (!isfinite(H[i])) return 0;
    return 1;
}

/* One hypothesis: 1 = model, ORC_NO_MODEL, ORC_NO_SAMPLE. */
int orc_h_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* H, float* hf, int* idx_out) {
    Stream st;
    st.seed = seed; st.hyp = (uint64_t)hyp; st.pos = 0;
    int idx[4];
    float sx[4], sy[4], dx[4], dy[4];
    for (int attempt = 0; attempt < ORC_MAX_ATTEMPTS; ++attempt) {
        if (!draw_distinct(&st, N, 4, idx)) continue;
        for (int i = 0; i < 4; ++i) {
            const float* p = pts4 + 4 * (size_t)idx[i];
            sx[i] = p[0]; sy[i] = p[1]; dx[i] = p[2]; dy[i] = p[3];
        }
        if (!h_subset_ok(sx, sy, dx, dy)) continue;
        if (idx_out) memcpy(idx_out, idx, sizeof(idx));
        if (!h_solve4(sx, sy, dx, dy, H)) return ORC_NO_MODEL;
        for (int i = 0; i < 8; ++i) {
            hf[i] = (float)H[i];
            if (!isfinite(hf[i])) return ORC_NO_MODEL;
        }
        return 1;
    }
    return ORC_NO_SAMPLE;
}

/* computeError + findInliers for one fp32 model. mask may be NULL.
 * fused = 1 (default definition): w = fma(h6,x,fma(h7,y,1)); ww = 1/w (IEEE);
 *   ex = fma(fma(h0,x,fma(h1,y,h2)), ww, -mx); ey likewise; e = fma(ex,ex,ey*ey)
 * fused = 0: OpenCV's expression evaluated op by op (x86 SSE-baseline arithmetic). */
int orc_h_count(const float* pts4, int N, const float* h, float thr2, uint8_t* mask, int fused) {
    int n = 0;
    for (int i = 0; i < N; ++i) {
        const float* p = pts4 + 4 * (size_t)i;
        float x = p[0], y = p[1], e;
        if (fused) {
            float ww = 1.f / fmaf(h[6], x, fmaf(h[7], y, 1.f));
            float ex = fmaf(fmaf(h[0], x, fmaf(h[1], y, h[2])), ww, -p[2]);
            float ey = fmaf(fmaf(h[3], x, fmaf(h[4], y, h[5])), ww, -p[3]);
            e = fmaf(ex, ex, ey * ey);
        } else {
            float ww = 1.f / (h[6] * x + h[7] * y + 1.f);
            float ex = (h[0] * x + h[1] * y + h[2]) * ww - p[2];
            float ey = (h[3] * x + h[4] * y + h[5]) * ww - p[3];
            e = ex * ex + ey * ey;
        }
        int in = e <= thr2;
        if (mask) mask[i] = (uint8_t)in;
        n += in;
    }
    return n;
}

/* Status-or-count per hypothesis over [hypBegin, hypBegin+hypCount), threads over hypotheses. */
void orc_h_counts(const float* pts4, int N, uint64_t seed, int64_t hypBegin, int64_t hypCount, float thr2,
                  int fused, int* counts, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t i = 0; i < hypCount; ++i) {
        double H[9];
        float hf[8];
        int st = orc_h_hypothesis(pts4, N, seed, hypBegin + i, H, hf, NULL);
        counts[i] = st == 1 ? orc_h_count(pts4, N, hf, thr2, NULL, fused) : st;
    }
}

/* RANSACUpdateNumIters [ext: OpenCV ptsetreg.cpp]. */
int orc_update_num_iters(double p, double ep, int modelPoints, int maxIters) {
    p = p > 0 ? p : 0.; p = p < 1 ? p : 1.;
    ep = ep > 0 ? ep : 0.; ep = ep < 1 ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= (double)maxIters * (-denom)) ? maxIters : (int)lrint(num / denom);
}

/* cv::eigen of a symmetric double matrix: JacobiImpl_<double> of OpenCV 4.x core lapack.cpp [ext],
 * restated — classical Jacobi, pivot = the largest strict-upper element found through the per-row
 * (indR) and per-column (indC) maxima (first maximum on ties), stop at |pivot| <= DBL_EPSILON or after
 * n*n*30 rotations, lapack.cpp's hypot, eigenvalues sorted descending by selection with the rows of V
 * (the eigenvectors) swapped along. A (n <= 9, row-major) is destroyed. */
static double lp_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a > b) { b /= a; return a * sqrt(1 + b * b); }
    if (b > 0) { a /= b; return b * sqrt(1 + a * a); }
    return 0;
}

static int row_argmax(const double* A, int n, int r) {   /* argmax_{c > r} |A[r][c]| */
    int m = r + 1;
    double mv = fabs(A[n * r + m]);
    for (int c = r + 2; c < n; ++c)
        if (mv < fabs(A[n * r + c])) { mv = fabs(A[n * r + c]); m = c; }
    return m;
}

static int col_argmax(const double* A, int n, int c) {   /* argmax_{r < c} |A[r][c]| */
    int m = 0;
    double mv = fabs(A[c]);
    for (int r = 1; r < c; ++r)
        if (mv < fabs(A[n * r + c])) { mv = fabs(A[n * r + c]); m = r; }
    return m;
}

static void jacobi(double* A, int n, double* w, double* V) {
    int indR[9], indC[9];
    for (int i = 0; i < n * n; ++i) V[i] = (i / n == i % n);
    for (int k = 0; k < n; ++k) {
        w[k] = A[(n + 1) * k];
        if (k < n - 1) indR[k] = row_argmax(A, n, k);
        if (k > 0) indC[k] = col_argmax(A, n, k);
    }
    for (int it = 0; n > 1 && it < n * n * 30; ++it) {
        int k = 0, l;
        double mv = fabs(A[indR[0]]);
        for (int i = 1; i < n - 1; ++i)
            if (mv < fabs(A[n * i + indR[i]])) { mv = fabs(A[n * i + indR[i]]); k = i; }
        l = indR[k];
        for (int i = 1; i < n; ++i)
            if (mv < fabs(A[n * indC[i] + i])) { mv = fabs(A[n * indC[i] + i]); k = indC[i]; l = i; }
        double p = A[n * k + l];
        if (fabs(p) <= DBL_EPSILON) break;
        double y = (w[l] - w[k]) * 0.5;
        double t = fabs(y) + lp_hypot(p, y);
        double s = lp_hypot(p, t);
        double c = t / s;
        s = p / s;
        t = (p / t) * p;
        if (y < 0) { s = -s; t = -t; }
        A[n * k + l] = 0;
        w[k] -= t;
        w[l] += t;
#define ORC_ROT(v0, v1) do { double a0_ = (v0), b0_ = (v1); (v0) = a0_ * c - b0_ * s; (v1) = a0_ * s + b0_ * c; } while (0)
        for (int i = 0; i < k; ++i) ORC_ROT(A[n * i + k], A[n * i + l]);
        for (int i = k + 1; i < l; ++i) ORC_ROT(A[n * k + i], A[n * i + l]);
        for (int i = l + 1; i < n; ++i) ORC_ROT(A[n * k + i], A[n * l + i]);
        for (int i = 0; i < n; ++i) ORC_ROT(V[n * k + i], V[n * l + i]);
#undef ORC_ROT
        for (int j = 0; j < 2; ++j) {
            int idx = j == 0 ? k : l;
            if (idx < n - 1) indR[idx] = row_argmax(A, n, idx);
            if (idx > 0) indC[idx] = col_argmax(A, n, idx);
        }
    }
    for (int k = 0; k < n - 1; ++k) {
        int m = k;
        for (int i = k + 1; i < n; ++i)
            if (w[m] < w[i]) m = i;
        if (m != k) {
            double t = w[k]; w[k] = w[m]; w[m] = t;
            for (int i = 0; i < n; ++i) { t = V[n * k + i]; V[n * k + i] = V[n * m + i]; V[n * m + i] = t; }
        }
    }
}

/* cv::solve / cv::invert with DECOMP_EIG: eigen (above) then SVBkSb (u = v = eigenvector rows,
 * threshold 2 DBL_EPSILON x sum of the signed w). */
void eig_pinv_apply(const double* A, int n, const double* b, double* x, double* Ainv) {
    double M[81], w[9], V[81], thr = 0;
    memcpy(M, A, sizeof(double) * n * n);
    jacobi(M, n, w, V);
    for (int i = 0; i < n; ++i) thr += w[i];
    thr *= DBL_EPSILON * 2;
    if (x) for (int j = 0; j < n; ++j) x[j] = 0;
    if (Ainv) for (int j = 0; j < n * n; ++j) Ainv[j] = 0;
    for (int e = 0; e < n; ++e) {
        if (fabs(w[e]) <= thr) continue;
        double wi = 1 / w[e];
        if (x) {
            double d = 0;
            for (int k = 0; k < n; ++k) d += V[e * n + k] * b[k];
            d *= wi;
            for (int j = 0; j < n; ++j) x[j] = x[j] + d * V[e * n + j];
        }
        if (Ainv) {
            double buf[9];
            for (int j = 0; j < n; ++j) buf[j] = V[e * n + j] * wi;
            for (int i = 0; i < n; ++i)
                for (int j = 0; j < n; ++j) Ainv[i * n + j] = Ainv[i * n + j] + V[e * n + i] * buf[j];
        }
    }
}

/* HomographyEstimatorCallback::runKernel [ext: OpenCV fundam.cpp] on count correspondences
 * M = (sx, sy) -> m = (dx, dy), sequential sums: centroids, mean |deviation| scales (0 when one
 * vanishes), LtL[j][k] += Lx[j] Lx[k] + Ly[j] Ly[k] (k >= j) then completeSymm, cv::eigen, H0 = the
 * last eigenvector row, invHnorm H0 Hnorm2, times 1/H22 (convertTo). */
static int h_run_kernel_xy(const float* sx, const float* sy, const float* dx, const float* dy, int count, double* H) {
    double cmx = 0, cmy = 0, cMx = 0, cMy = 0, smx = 0, smy = 0, sMx = 0, sMy = 0;
    for (int t = 0; t < count; ++t) { cmx += dx[t]; cmy += dy[t]; cMx += sx[t]; cMy += sy[t]; }
    cmx /= count; cmy /= count; cMx /= count; cMy /= count;
    for (int t = 0; t < count; ++t) {
        smx += fabs(dx[t] - cmx); smy += fabs(dy[t] - cmy); sMx += fabs(sx[t] - cMx); sMy += fabs(sy[t] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return 0;
    smx = count / smx; smy = count / smy; sMx = count / sMx; sMy = count / sMy;
    double L[81] = {0};
    for (int t = 0; t < count; ++t) {
        double x = (dx[t] - cmx) * smx, y = (dy[t] - cmy) * smy, X = (sx[t] - cMx) * sMx, Y = (sy[t] - cMy) * sMy;
        double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; ++j)
            for (int k = j; k < 9; ++k) L[j * 9 + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; ++j)
        for (int k = 0; k < j; ++k) L[j * 9 + k] = L[k * 9 + j];
    for (int j = 0; j < 81; ++j)
        if (!isfinite(L[j])) return 0;   /* NaN input: OpenCV's NaN model counts no inlier either */
    double w[9], V[81];
    jacobi(L, 9, w, V);
    double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9], R[9];
    mul33(invHnorm, V + 72, T);
    mul33(T, Hnorm2, R);
    double sc = 1. / R[8];
    for (int k = 0; k < 9; ++k) H[k] = R[k] * sc;
    return 1;
}

/* The same over listed correspondences of a float4 set (refit over the inliers). */
static int h_run_kernel(const float* pts4, const int* list, int count, double* H) {
    float* b = (float*)malloc(sizeof(float) * 4 * (size_t)(count > 0 ? count : 1));
    for (int t = 0; t < count; ++t) {
        const float* p = pts4 + 4 * (size_t)list[t];
        b[t] = p[0]; b[count + t] = p[1]; b[2 * (size_t)count + t] = p[2]; b[3 * (size_t)count + t] = p[3];
    }
    int r = h_run_kernel_xy(b, b + count, b + 2 * (size_t)count, b + 3 * (size_t)count, count, H);
    free(b);
    return r;
}

/* HomographyRefineCallback::compute: returns |r|^2; A (8x8) and v (8) when non-NULL. */
static double h_lm_compute(const float* pts4, const int* list, int count, const double* h, double* A, double* v) {
    double S = 0;
    if (A) { memset(A, 0, 64 * sizeof(double)); memset(v, 0, 8 * sizeof(double)); }
    for (int t = 0; t < count; ++t) {
        const float* p = pts4 + 4 * (size_t)list[t];
        double Mx = p[0], My = p[1];
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
        double xi = (h[0] * Mx + h[1] * My + h[2]) * ww, yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        double rx = xi - p[2], ry = yi - p[3];
        S += rx * rx + ry * ry;
        if (A) {
            double Jx[8] = {Mx * ww, My * ww, ww, 0, 0, 0, -Mx * ww * xi, -My * ww * xi};
            double Jy[8] = {0, 0, 0, Mx * ww, My * ww, ww, -Mx * ww * yi, -My * ww * yi};
            for (int j = 0; j < 8; ++j) {
                for (int k = 0; k < 8; ++k) A[j * 8 + k] += Jx[j] * Jx[k] + Jy[j] * Jy[k];
                v[j] += Jx[j] * rx + Jy[j] * ry;
            }
        }
    }
    return S;
}

/* LMSolverImpl::run [ext: OpenCV levmarq.cpp, classic version], maxIters, eps = FLT_EPSILON. */
static void h_lm(const float* pts4, const int* list, int count, double* H, int maxIters) {
    double x[8], xd[8], d[8], v[8], A[64], Ap[64], D[8];
    memcpy(x, H, sizeof(x));
    double S = h_lm_compute(pts4, list, count, x, A, v);
    for (int i = 0; i < 8; ++i) D[i] = A[i * 9];
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        memcpy(Ap, A, sizeof(A));
        for (int i = 0; i < 8; ++i) Ap[i * 9] += lambda * D[i];
        eig_pinv_apply(Ap, 8, v, d, NULL);
        for (int i = 0; i < 8; ++i) xd[i] = x[i] - d[i];
        double Sd = h_lm_compute(pts4, list, count, xd, NULL, NULL);
        double dS = 0;
        for (int i = 0; i < 8; ++i) {
            double ad = 0;
            for (int k = 0; k < 8; ++k) ad += A[i * 8 + k] * d[k];
            dS += d[i] * (-ad + 2 * v[i]);
        }
        double R = (S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > 0.75) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < 0.25) {
            double t = 0;
            for (int i = 0; i < 8; ++i) t += d[i] * v[i];
            double nu = (Sd - S) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = nu < 2 ? 2 : (nu > 10 ? 10 : nu);
            if (lambda == 0) {
                eig_pinv_apply(A, 8, NULL, NULL, Ap);
                double mx = DBL_EPSILON;
                for (int i = 0; i < 8; ++i) mx = fabs(Ap[i * 9]) > mx ? fabs(Ap[i * 9]) : mx;
                lambda = lc = 1. / mx;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            memcpy(x, xd, sizeof(x));
            S = h_lm_compute(pts4, list, count, x, A, v);
        }
        ++iter;
        double dn = 0;
        for (int i = 0; i < 8; ++i) dn = fabs(d[i]) > dn ? fabs(d[i]) : dn;
        if (!(iter < maxIters && dn >= FLT_EPSILON && S >= (double)FLT_EPSILON * FLT_EPSILON)) break;
    }
    memcpy(H, x, sizeof(x));
}

/* Sequential RANSAC replay over precomputed per-hypothesis statuses/counts (the loop of
 * RANSACPointSetRegistrator::run). Returns best hypothesis index or -1. */
int64_t orc_ransac_replay(const int* counts, int64_t ncounts, int N, int m, double conf, int maxIters, int fixed,
                          int* bestCount) {
    int64_t niters = maxIters > 1 ? maxIters : 1, best = -1;
    int bc = 0;
    for (int64_t it = 0; it < niters && it < ncounts; ++it) {
        int c = counts[it];
        if (c == ORC_NO_SAMPLE) break;
        if (c < 0) continue;
        if (c > (bc > m - 1 ? bc : m - 1)) {
            bc = c; best = it;
            if (!fixed) niters = orc_update_num_iters(conf, (double)(N - c) / N, m, (int)niters);
        }
    }
    if (bestCount) *bestCount = bc;
    return best;
}


/* cv::findHomography(src, dst, method, thr, mask, maxIters, conf) with the counter-based sampler.
 * pts as fp64 AoS (converted to float as convertTo(CV_32F)). Returns inlier count, 0 on failure. */
int orc_find_homography(const double* src, const double* dst, int N, double thr, double conf, int maxIters,
                        int method, uint64_t seed, int flags, double* H, uint8_t* mask, int64_t* bestHypOut,
                        int nthreads) {
    if (mask) memset(mask, 0, (size_t)(N > 0 ? N : 0));
    if (bestHypOut) *bestHypOut = -1;
    if (N < 4) return 0;
    if (thr <= 0) thr = 3;
    float* pts = (float*)malloc(sizeof(float) * 4 * (size_t)N);
    int* list = (int*)malloc(sizeof(int) * (size_t)N);
    uint8_t* m8 = (uint8_t*)malloc((size_t)N);
    for (int i = 0; i < N; ++i) {
        pts[4 * i] = (float)src[2 * i]; pts[4 * i + 1] = (float)src[2 * i + 1];
        pts[4 * i + 2] = (float)dst[2 * i]; pts[4 * i + 3] = (float)dst[2 * i + 1];
    }
    int result = 0, count = 0;
    if (method == 0 || N == 4) {
        for (int i = 0; i < N; ++i) { list[i] = i; m8[i] = 1; }
        result = h_run_kernel(pts, list, N, H);
        if (result && N > 4) h_lm(pts, list, N, H, 10);
        count = N;
    } else {
        const float thr2 = (float)(thr * thr);
        int64_t niters = maxIters > 1 ? maxIters : 1, best = -1;
        int bc = 0;
        int* cnts = (int*)malloc(sizeof(int) * (size_t)niters);
        int* cvt = orc_cv_begin(flags, 1, pts, N, 4, niters);
        /* counts for every hypothesis up front (parallel), replay sequentially */
        const int fused = (flags & ORC_FLAG_FUSED_ERROR) != 0;
        orc_h_counts(pts, N, seed, 0, niters, thr2, fused, cnts, nthreads);
        best = orc_ransac_replay(cnts, niters, N, 4, conf, maxIters, (flags & ORC_FLAG_FIXED_ITERS) != 0, &bc);
        free(cnts);
        if (best >= 0) {
            double Hb[9];
            float hf[8];
            orc_h_hypothesis(pts, N, seed, best, Hb, hf, NULL);
            count = orc_h_count(pts, N, hf, thr2, m8, fused);
            memcpy(H, Hb, sizeof(Hb));
            result = 1;
            if (!(flags & ORC_FLAG_NO_REFINE)) {
                int k = 0;
                for (int i = 0; i < N; ++i)
                    if (m8[i]) list[k++] = i;
                if (k > 0) {
                    double Hr[9];
                    if (h_run_kernel(pts, list, k, Hr)) memcpy(H, Hr, sizeof(Hr));
                    h_lm(pts, list, k, H, 10);
                }
            }
            if (bestHypOut) *bestHypOut = best;
        }
        orc_cv_end(cvt);
    }
    if (result && mask) memcpy(mask, m8, (size_t)N);
    free(pts); free(list); free(m8);
    return result ? count : 0;
}

/* ------------------------------------------------------------------------------------------
 * Fundamental matrix, 8-point minimal sets (north_star). OpenCV 4.x run8Point / FMEstimatorCallback
 * and EMEstimatorCallback::computeError (Sampson) [ext]; same definition as
 * minicv_amd/csrc/hyp_fundamental.h (run8Point's sqrt(2) / mean-distance normalisation, f22 = 1
 * elimination for the null vector, rank 2 through JacobiSVD with w[2] = 0).
 * ---------------------------------------------------------------------------------------- */
void jacobi3_orc(double* A, double* V) {
    for (int i = 0; i < 9; ++i) V[i] = (i == 0 || i == 4 || i == 8) ? 1.0 : 0.0;
    static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
    for (int sweep = 0; sweep < 16; ++sweep) {
        double off = A[1] * A[1] + A[2] * A[2] + A[5] * A[5];
        double dg = A[0] * A[0] + A[4] * A[4] + A[8] * A[8];
        if (!(off > dg * 1e-32)) break;
        for (int r = 0; r < 3; ++r) {
            int p = P[r], q = Q[r];
            double apq = A[3 * p + q];
            if (apq == 0) continue;
            double theta = (A[3 * q + q] - A[3 * p + p]) / (2 * apq);
            double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; ++k) {
                double x = A[3 * k + p], y = A[3 * k + q];
                A[3 * k + p] = c * x - s * y; A[3 * k + q] = s * x + c * y;
            }
            for (int k = 0; k < 3; ++k) {
                double x = A[3 * p + k], y = A[3 * q + k];
                A[3 * p + k] = c * x - s * y; A[3 * q + k] = s * x + c * y;
            }
            for (int k = 0; k < 3; ++k) {
                double x = V[3 * k + p], y = V[3 * k + q];
                V[3 * k + p] = c * x - s * y; V[3 * k + q] = s * x + c * y;
            }
        }
    }
}

/* run8Point's rank-2 step: cv::SVD::compute(F0) = JacobiSVDImpl_ on F0^T (orc_jsvd), w[2] = 0,
 * F0 = (U diag(w)) Vt with Matx products (s = 0; s += a b in k order). */
static void f_rank2_orc(double* F) {
    double At[9], w[3], Vt[9], UD[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) At[3 * i + j] = F[3 * j + i];
    orc_jsvd(At, w, Vt, 3, 3, 3);
    w[2] = 0.;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0;
            for (int k = 0; k < 3; ++k) acc += At[3 * k + i] * (k == j ? w[j] : 0.0);
            UD[3 * i + j] = acc;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            double acc = 0;
            for (int k = 0; k < 3; ++k) acc += UD[3 * i + k] * Vt[3 * k + j];
            F[3 * i + j] = acc;
        }
}

static int f_denorm_orc(const double* F0, double c1x, double c1y, double s1x, double s1y, double c2x, double c2y,
                        double s2x, double s2y, double* F) {
    double T1[9] = {s1x, 0, -s1x * c1x, 0, s1y, -s1y * c1y, 0, 0, 1};
    double T2t[9] = {s2x, 0, 0, 0, s2y, 0, -s2x * c2x, -s2y * c2y, 1};
    double T[9];
    mul33(T2t, F0, T);
    mul33(T, T1, F);
    if (fabs(F[8]) > (double)FLT_EPSILON) {
        double s = 1. / F[8];
        for (int i = 0; i < 9; ++i) F[i] = F[i] * s;
    }
    for (int i = 0; i < 9; ++i)
        if (!isfinite(F[i])) return 0;
    return 1;
}

/* run8Point's normalisation: centroid = sum * (1 / m), mean Euclidean distance (times 1 / m),
 * scale = sqrt(2) / distance for both axes; 0 when the distance is below FLT_EPSILON. */
static int f_norm8(const float* x, const float* y, int m, double* cx, double* cy, double* sx, double* sy) {
    double mx = 0, my = 0, d = 0, t = 1. / m;
    for (int i = 0; i < m; ++i) { mx += x[i]; my += y[i]; }
    mx *= t; my *= t;
    for (int i = 0; i < m; ++i) {
        double dx = x[i] - mx, dy = y[i] - my;
        d += sqrt(dx * dx + dy * dy);
    }
    d *= t;
    if (d < FLT_EPSILON) return 0;
    d = sqrt(2.) / d;
    *cx = mx; *cy = my; *sx = d; *sy = d;
    return 1;
}

/* run8Point's eigen step on the accumulated A (upper triangle filled; completed here): cv::eigen, the
 * eigenvalue check (0 when one of the 8 largest is below DBL_EPSILON in magnitude), F0 = the last
 * eigenvector row, rank 2, de-normalisation. */
static int f_from_ata(double* A, double c1x, double c1y, double s1x, double s1y, double c2x, double c2y, double s2x,
                      double s2y, double* F) {
    for (int j = 0; j < 9; ++j)
        for (int k = 0; k < j; ++k) A[j * 9 + k] = A[k * 9 + j];
    for (int j = 0; j < 81; ++j)
        if (!isfinite(A[j])) return 0;
    double w[9], V[81], F0[9];
    jacobi(A, 9, w, V);
    int i = 0;
    for (; i < 9; ++i)
        if (fabs(w[i]) < DBL_EPSILON) break;
    if (i < 8) return 0;
    memcpy(F0, V + 72, sizeof(F0));
    f_rank2_orc(F0);
    return f_denorm_orc(F0, c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y, F);
}

/* MCV_FLAG_FAST_MINIMAL (opt-in): the 8x9 system with f22 = 1 by Gaussian elimination. */
static int f_solve8_elim_orc(const float* x1, const float* y1, const float* x2, const float* y2, double* F) {
    double c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y;
    if (!f_norm8(x1, y1, 8, &c1x, &c1y, &s1x, &s1y) || !f_norm8(x2, y2, 8, &c2x, &c2y, &s2x, &s2y)) return 0;
    double a[8][9];
    for (int i = 0; i < 8; ++i) {
        double X1 = (x1[i] - c1x) * s1x, Y1 = (y1[i] - c1y) * s1y, X2 = (x2[i] - c2x) * s2x, Y2 = (y2[i] - c2y) * s2y;
        double r[9] = {X2 * X1, X2 * Y1, X2, Y2 * X1, Y2 * Y1, Y2, X1, Y1, -1.0};
        memcpy(a[i], r, sizeof(r));
    }
    for (int c = 0; c < 8; ++c) {
        int p = c;
        double best = fabs(a[c][c]);
        for (int r = c + 1; r < 8; ++r)
            if (fabs(a[r][c]) > best) { best = fabs(a[r][c]); p = r; }
        if (!(best > 0)) return 0;
        if (p != c)
            for (int k = c; k < 9; ++k) { double t = a[c][k]; a[c][k] = a[p][k]; a[p][k] = t; }
        for (int r = c + 1; r < 8; ++r) {
            double f = a[r][c] / a[c][c];
            for (int k = c + 1; k < 9; ++k) a[r][k] = a[r][k] - f * a[c][k];
        }
    }
    double h[8];
    for (int i = 7; i >= 0; --i) {
        double s = a[i][8];
        for (int k = i + 1; k < 8; ++k) s = s - a[i][k] * h[k];
        h[i] = s / a[i][i];
    }
    double F0[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
    f_rank2_orc(F0);
    return f_denorm_orc(F0, c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y, F);
}

/* run8Point on the 8-point sample: normalisation, A += r r^T, f_from_ata. */
static int f_solve8_orc(const float* x1, const float* y1, const float* x2, const float* y2, double* F) {
    if (g_fast_minimal) return f_solve8_elim_orc(x1, y1, x2, y2, F);
    double c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y;
    if (!f_norm8(x1, y1, 8, &c1x, &c1y, &s1x, &s1y) || !f_norm8(x2, y2, 8, &c2x, &c2y, &s2x, &s2y)) return 0;
    double A[81] = {0};
    for (int i = 0; i < 8; ++i) {
        double X1 = (x1[i] - c1x) * s1x, Y1 = (y1[i] - c1y) * s1y, X2 = (x2[i] - c2x) * s2x, Y2 = (y2[i] - c2y) * s2y;
        double r[9] = {X2 * X1, X2 * Y1, X2, Y2 * X1, Y2 * Y1, Y2, X1, Y1, 1.0};
        for (int j = 0; j < 9; ++j)
            for (int k = j; k < 9; ++k) A[j * 9 + k] += r[j] * r[k];
    }
    return f_from_ata(A, c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y, F);
}

int orc_f_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F, int* idx_out) {
    Stream st;
    st.seed = seed; st.hyp = (uint64_t)hyp; st.pos = 0;
    int idx[8];
    float x1[8], y1[8], x2[8], y2[8];
    for (int attempt = 0; attempt < ORC_MAX_ATTEMPTS; ++attempt) {
        if (!draw_distinct(&st, N, 8, idx)) continue;
        for (int i = 0; i < 8; ++i) {
            const float* p = pts4 + 4 * (size_t)idx[i];
            x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
        }
        if (collinear_last(x1, y1, 8) || collinear_last(x2, y2, 8)) continue;
        if (idx_out) memcpy(idx_out, idx, sizeof(idx));
        return f_solve8_orc(x1, y1, x2, y2, F) ? 1 : ORC_NO_MODEL;
    }
    return ORC_NO_SAMPLE;
}

/* kind = errorKind * 2 + unfused: 0 Sampson fused, 1 Sampson op-by-op, 2 epipolar fused, 3 epipolar. */
float f_err_orc(int kind, const double* F, double x1, double y1, double x2, double y2) {
    if (kind == 0) {
        double ax = fma(F[0], x1, fma(F[1], y1, F[2])), ay = fma(F[3], x1, fma(F[4], y1, F[5]));
        double az = fma(F[6], x1, fma(F[7], y1, F[8]));
        double bx = fma(F[0], x2, fma(F[3], y2, F[6])), by = fma(F[1], x2, fma(F[4], y2, F[7]));
        double c = fma(x2, ax, fma(y2, ay, az));
        double den = fma(ax, ax, fma(ay, ay, fma(bx, bx, by * by)));
        return (float)(c * c / den);
    }
    if (kind == 1) {
        double ax = F[0] * x1 + F[1] * y1 + F[2] * 1., ay = F[3] * x1 + F[4] * y1 + F[5] * 1.;
        double az = F[6] * x1 + F[7] * y1 + F[8] * 1.;
        double bx = F[0] * x2 + F[3] * y2 + F[6] * 1., by = F[1] * x2 + F[4] * y2 + F[7] * 1.;
        double c = x2 * ax + y2 * ay + 1. * az;
        double a2 = ax * ax, b2 = ay * ay, c2 = bx * bx, d2 = by * by;
        return (float)(c * c / (a2 + b2 + c2 + d2));
    }
    double a, b, c, s1, s2, d1, d2;
    if (kind == 2) {
        a = fma(F[0], x1, fma(F[1], y1, F[2])); b = fma(F[3], x1, fma(F[4], y1, F[5]));
        c = fma(F[6], x1, fma(F[7], y1, F[8]));
        s2 = 1. / fma(a, a, b * b); d2 = fma(x2, a, fma(y2, b, c));
        a = fma(F[0], x2, fma(F[3], y2, F[6])); b = fma(F[1], x2, fma(F[4], y2, F[7]));
        c = fma(F[2], x2, fma(F[5], y2, F[8]));
        s1 = 1. / fma(a, a, b * b); d1 = fma(x1, a, fma(y1, b, c));
    } else {
        a = F[0] * x1 + F[1] * y1 + F[2]; b = F[3] * x1 + F[4] * y1 + F[5]; c = F[6] * x1 + F[7] * y1 + F[8];
        s2 = 1. / (a * a + b * b); d2 = x2 * a + y2 * b + c;
        a = F[0] * x2 + F[3] * y2 + F[6]; b = F[1] * x2 + F[4] * y2 + F[7]; c = F[2] * x2 + F[5] * y2 + F[8];
        s1 = 1. / (a * a + b * b); d1 = x1 * a + y1 * b + c;
    }
    double e1 = d1 * d1 * s1, e2 = d2 * d2 * s2;
    return (float)(e1 < e2 ? e2 : e1);
}

int orc_f_count(const float* pts4, int N, const double* F, float thr2, int kind, uint8_t* mask) {
    int n = 0;
    for (int i = 0; i < N; ++i) {
        const float* p = pts4 + 4 * (size_t)i;
        int in = f_err_orc(kind, F, p[0], p[1], p[2], p[3]) <= thr2;
        if (mask) mask[i] = (uint8_t)in;
        n += in;
    }
    return n;
}

void orc_f_counts(const float* pts4, int N, uint64_t seed, int64_t hypBegin, int64_t hypCount, float thr2, int kind,
                  int* counts, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int64_t i = 0; i < hypCount; ++i) {
        double F[9];
        int st = orc_f_hypothesis(pts4, N, seed, hypBegin + i, F, NULL);
        counts[i] = st == 1 ? orc_f_count(pts4, N, F, thr2, kind, NULL) : st;
    }
}

/* run8Point over all points (FM_8POINT / method 0): same normalisation, eigen (JacobiImpl_), the
 * eigenvalue check, rank 2. */
static int f_fit_all_orc(const float* pts4, int N, double* F) {
    double c1x = 0, c1y = 0, c2x = 0, c2y = 0, d1 = 0, d2 = 0, t = 1. / N;
    for (int i = 0; i < N; ++i) { c1x += pts4[4 * i]; c1y += pts4[4 * i + 1]; c2x += pts4[4 * i + 2]; c2y += pts4[4 * i + 3]; }
    c1x *= t; c1y *= t; c2x *= t; c2y *= t;
    for (int i = 0; i < N; ++i) {
        double ax = pts4[4 * i] - c1x, ay = pts4[4 * i + 1] - c1y, bx = pts4[4 * i + 2] - c2x, by = pts4[4 * i + 3] - c2y;
        d1 += sqrt(ax * ax + ay * ay);
        d2 += sqrt(bx * bx + by * by);
    }
    d1 *= t; d2 *= t;
    if (d1 < FLT_EPSILON || d2 < FLT_EPSILON) return 0;
    double s1x = sqrt(2.) / d1, s1y = s1x, s2x = sqrt(2.) / d2, s2y = s2x;
    double A[81] = {0};
    for (int i = 0; i < N; ++i) {
        double X1 = (pts4[4 * i] - c1x) * s1x, Y1 = (pts4[4 * i + 1] - c1y) * s1y;
        double X2 = (pts4[4 * i + 2] - c2x) * s2x, Y2 = (pts4[4 * i + 3] - c2y) * s2y;
        double r[9] = {X2 * X1, X2 * Y1, X2, Y2 * X1, Y2 * Y1, Y2, X1, Y1, 1.0};
        for (int j = 0; j < 9; ++j)
            for (int k = j; k < 9; ++k) A[j * 9 + k] += r[j] * r[k];
    }
    return f_from_ata(A, c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y, F);
}

/* cv::findFundamentalMat(a, b, FM_RANSAC (8-point kernel) | FM_8POINT, thr, conf, maxIters, mask). */
int orc_find_fundamental(const double* a, const double* b, int N, double thr, double conf, int maxIters, int method,
                         uint64_t seed, int flags, int errorKind, double* F, uint8_t* mask, int64_t* bestHypOut,
                         int nthreads) {
    if (mask) memset(mask, 0, (size_t)(N > 0 ? N : 0));
    if (bestHypOut) *bestHypOut = -1;
    if (N < 8) return 0;
    if (thr <= 0) thr = 3;
    float* pts = (float*)malloc(sizeof(float) * 4 * (size_t)N);
    for (int i = 0; i < N; ++i) {
        pts[4 * i] = (float)a[2 * i]; pts[4 * i + 1] = (float)a[2 * i + 1];
        pts[4 * i + 2] = (float)b[2 * i]; pts[4 * i + 3] = (float)b[2 * i + 1];
    }
    int count = 0;
    if (method == 0 || N == 8) {
        if (f_fit_all_orc(pts, N, F)) {
            count = N;
            if (mask) memset(mask, 1, (size_t)N);
        }
    } else {
        const float thr2 = (float)(thr * thr);
        const int kind = (errorKind == 1 ? 2 : 0) + ((flags & ORC_FLAG_FUSED_ERROR) ? 0 : 1);
        int64_t niters = maxIters > 1 ? maxIters : 1;
        int* cnts = (int*)malloc(sizeof(int) * (size_t)niters);
        int* cvt = orc_cv_begin(flags, 2, pts, N, 8, niters);
        orc_f_counts(pts, N, seed, 0, niters, thr2, kind, cnts, nthreads);
        int bc = 0;
        int64_t best = orc_ransac_replay(cnts, niters, N, 8, conf, maxIters, (flags & ORC_FLAG_FIXED_ITERS) != 0, &bc);
        free(cnts);
        if (best >= 0) {
            orc_f_hypothesis(pts, N, seed, best, F, NULL);
            count = orc_f_count(pts, N, F, thr2, kind, mask);
            if (bestHypOut) *bestHypOut = best;
        }
        orc_cv_end(cvt);
    }
    free(pts);
    return count;
}

/* ------------------------------------------------------------------------------------------
 * Brute-force matchers (BFMatcher NORM_HAMMING / NORM_L2, knn k = 2) [ext: OpenCV features2d].
 * Ties: the lower train index wins (strict comparison while scanning trains in order).
 * ---------------------------------------------------------------------------------------- */
void orc_match_hamming(const uint8_t* q, int nq, const uint8_t* t, int nt, int bytes, int* idx, int* dist, int* idx2,
                       int* dist2, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int i = 0; i < nq; ++i) {
        int b1 = INT_MAX, b2 = INT_MAX, i1 = -1, i2 = -1;
        const uint8_t* qi = q + (size_t)i * bytes;
        for (int j = 0; j < nt; ++j) {
            const uint8_t* tj = t + (size_t)j * bytes;
            int d = 0;
            for (int b = 0; b < bytes; ++b) d += __builtin_popcount((unsigned)(qi[b] ^ tj[b]));
            if (d < b1) { b2 = b1; i2 = i1; b1 = d; i1 = j; }
            else if (d < b2) { b2 = d; i2 = j; }
        }
        idx[i] = i1; dist[i] = b1;
        if (idx2) idx2[i] = i2;
        if (dist2) dist2[i] = b2;
    }
}

/* Exact (fp64-accumulated) squared distances; returns sqrt like NORM_L2. */
void orc_match_l2(const float* q, int nq, const float* t, int nt, int dim, int* idx, double* dist, int* idx2,
                  double* dist2, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int i = 0; i < nq; ++i) {
        double b1 = INFINITY, b2 = INFINITY;
        int i1 = -1, i2 = -1;
        const float* qi = q + (size_t)i * dim;
        for (int j = 0; j < nt; ++j) {
            const float* tj = t + (size_t)j * dim;
            double d = 0;
            for (int k = 0; k < dim; ++k) { double e = (double)qi[k] - (double)tj[k]; d += e * e; }
            if (d < b1) { b2 = b1; i2 = i1; b1 = d; i1 = j; }
            else if (d < b2) { b2 = d; i2 = j; }
        }
        idx[i] = i1; dist[i] = sqrt(b1);
        if (idx2) idx2[i] = i2;
        if (dist2) dist2[i] = sqrt(b2);
    }
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
