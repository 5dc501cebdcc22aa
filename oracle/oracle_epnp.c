/*
 * oracle_epnp.c — CPU restatement of EPnP as OpenCV 4.x computes it (calib3d epnp.cpp
 * compute_pose, with cv::SVD / cv::solve / cv::invert(DECOMP_SVD) = JacobiSVDImpl_ + SVBkSb from
 * core lapack.cpp) for the solverKind 0/1/3/4 paths of the reference's cvSolvePnPRansac /
 * cvSolvePnP (/root/reference/src/MiniCVNative/MiniCVNative.cpp:48-139). TEST INFRASTRUCTURE ONLY
 * (rules: oracle.c header).
 *
 * OpenCV is not vendored in /root/reference and not installed here [ext]: this restates the
 * published algorithm and the scalar loop order of those functions; x86 OpenCV builds run some
 * JacobiSVD loops through SIMD helpers (other partial-sum orders), so the last bits of OpenCV's
 * own result are not claimed (parity with OpenCV unpinned; the EPnP solution itself is pinned by
 * exact synthetic geometry: noise-free correspondences of a known pose give that pose back to
 * ~1e-10, tests/test_oracle_pnp.py). The GPU path
 * (minicv_amd/csrc/epnp.h) must equal this file bit for bit.
 *
 * Sums over the points of a large set run in blocks of EPNP_BLOCK consecutive points (each block
 * from 0 in point order, then the block sums in order): the sequential OpenCV order whenever
 * n <= EPNP_BLOCK.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include "oracle_int.h"

#define EPNP_BLOCK 1024

/* core lapack.cpp's hypot template (what JacobiSVDImpl_'s unqualified hypot resolves to). */
static double cv_hypot(double a, double b) {
    a = fabs(a);
    b = fabs(b);
    if (a > b) {
        b /= a;
        return a * sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * sqrt(1 + a * a);
    }
    return 0;
}

/* JacobiSVDImpl_<double>(At, W, Vt, m, n, n1): At is n1 x m row-major (the transposed matrix; rows
 * n .. n1-1 zero on entry, completed by the cv::RNG branch); Vt n x n or NULL. */
void orc_jsvd(double* At, double* Wout, double* Vt, int m, int n, int n1) {
    const double eps = DBL_EPSILON * 10, minval = DBL_MIN;
    double W[16];
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sd;
        if (Vt) {
            for (int k = 0; k < n; k++) Vt[i * n + k] = 0;
            Vt[i * n + i] = 1;
        }
    }
    int max_iter = m > 30 ? m : 30;
    for (int iter = 0; iter < max_iter; iter++) {
        int changed = 0;
        for (int i = 0; i < n - 1; i++)
            for (int j = i + 1; j < n; j++) {
                double *Ai = At + i * m, *Aj = At + j * m;
                double a = W[i], p = 0, b = W[j];
                for (int k = 0; k < m; k++) p += Ai[k] * Aj[k];
                if (fabs(p) <= eps * sqrt(a * b)) continue;
                p *= 2;
                double beta = a - b, gamma = cv_hypot(p, beta), c, s;
                if (beta < 0) {
                    double delta = (gamma - beta) * 0.5;
                    s = sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
                for (int k = 0; k < m; k++) {
                    double t0 = c * Ai[k] + s * Aj[k];
                    double t1 = -s * Ai[k] + c * Aj[k];
                    Ai[k] = t0;
                    Aj[k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = 1;
                if (Vt) {
                    double *Vi = Vt + i * n, *Vj = Vt + j * n;
                    for (int k = 0; k < n; k++) {
                        double t0 = c * Vi[k] + s * Vj[k];
                        double t1 = -s * Vi[k] + c * Vj[k];
                        Vi[k] = t0;
                        Vj[k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
    for (int i = 0; i < n; i++) {
        double sd = 0;
        for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
        W[i] = sqrt(sd);
    }
    for (int i = 0; i < n - 1; i++) {
        int j = i;
        for (int k = i + 1; k < n; k++)
            if (W[j] < W[k]) j = k;
        if (i != j) {
            double t = W[i]; W[i] = W[j]; W[j] = t;
            for (int k = 0; k < m; k++) { t = At[i * m + k]; At[i * m + k] = At[j * m + k]; At[j * m + k] = t; }
            if (Vt)
                for (int k = 0; k < n; k++) { t = Vt[i * n + k]; Vt[i * n + k] = Vt[j * n + k]; Vt[j * n + k] = t; }
        }
    }
    for (int i = 0; i < n; i++) Wout[i] = W[i];
    uint64_t rng = 0x12345678u;
    for (int i = 0; i < n1; i++) {
        double sd = i < n ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ii++) {
            double val0 = 1. / m;
            for (int k = 0; k < m; k++) {
                rng = (uint64_t)(uint32_t)rng * 4164903690u + (uint32_t)(rng >> 32);
                At[i * m + k] = ((uint32_t)rng & 256) != 0 ? val0 : -val0;
            }
            for (int it = 0; it < 2; it++)
                for (int j = 0; j < i; j++) {
                    sd = 0;
                    for (int k = 0; k < m; k++) sd += At[i * m + k] * At[j * m + k];
                    double asum = 0;
                    for (int k = 0; k < m; k++) {
                        double t = At[i * m + k] - sd * At[j * m + k];
                        At[i * m + k] = t;
                        asum += fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    for (int k = 0; k < m; k++) At[i * m + k] *= asum;
                }
            sd = 0;
            for (int k = 0; k < m; k++) sd += At[i * m + k] * At[i * m + k];
            sd = sqrt(sd);
        }
        double s = sd > minval ? 1 / sd : 0.;
        for (int k = 0; k < m; k++) At[i * m + k] *= s;
    }
}

static void jsvd(double* At, double* Wout, double* Vt, int m, int n) { orc_jsvd(At, Wout, Vt, m, n, n); }

/* SVBkSb: rhs b (m) or b == NULL for the inverse (x: n x m). u rows = At rows after jsvd. */
static void svbksb(const double* U, const double* w, const double* Vt, int m, int n, const double* b, double* x) {
    double thr = 0;
    for (int i = 0; i < n; i++) thr += w[i];
    thr *= DBL_EPSILON * 2;
    int nb = b ? 1 : m;
    for (int i = 0; i < n * nb; i++) x[i] = 0;
    for (int i = 0; i < n; i++) {
        double wi = w[i];
        if (fabs(wi) <= thr) continue;
        wi = 1 / wi;
        if (b) {
            double s = 0;
            for (int j = 0; j < m; j++) s += U[i * m + j] * b[j];
            s *= wi;
            for (int j = 0; j < n; j++) x[j] = x[j] + s * Vt[i * n + j];
        } else {
            double buf[16];
            for (int c = 0; c < m; c++) buf[c] = U[i * m + c] * wi;
            for (int r = 0; r < n; r++) {
                double s = Vt[i * n + r];
                for (int c = 0; c < m; c++) x[r * m + c] = x[r * m + c] + s * buf[c];
            }
        }
    }
}

/* cv::solve(A (6 x k), rho, x, DECOMP_SVD) */
static void solve6(const double* A6k, int k, const double* rho, double* x) {
    double At[6 * 6], w[6], Vt[36];
    for (int i = 0; i < k; i++)
        for (int r = 0; r < 6; r++) At[i * 6 + r] = A6k[r * k + i];
    jsvd(At, w, Vt, 6, k);
    svbksb(At, w, Vt, 6, k, rho, x);
}

static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

static void qr_solve(double* A /*6x4*/, double* b, double* X) {
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    for (int k = 0; k < nc; k++) {
        double eta = fabs(A[k * nc + k]);
        /* epnp::qr_solve reads the pivot column one row behind its counter: A[k][k] twice and
           never the last row */
        for (int i = k + 1; i < nr; i++) {
            double elt = fabs(A[(i - 1) * nc + k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) return;
        double sum2 = 0.0, inv_eta = 1. / eta;
        for (int i = k; i < nr; i++) {
            A[i * nc + k] *= inv_eta;
            sum2 += A[i * nc + k] * A[i * nc + k];
        }
        double sigma = sqrt(sum2);
        if (A[k * nc + k] < 0) sigma = -sigma;
        A[k * nc + k] += sigma;
        A1[k] = sigma * A[k * nc + k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; j++) {
            double sum = 0;
            for (int i = k; i < nr; i++) sum += A[i * nc + k] * A[i * nc + j];
            double tau = sum / A1[k];
            for (int i = k; i < nr; i++) A[i * nc + j] -= tau * A[i * nc + k];
        }
    }
    for (int j = 0; j < nc; j++) {
        double tau = 0;
        for (int i = j; i < nr; i++) tau += A[i * nc + j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; i++) b[i] -= tau * A[i * nc + j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        double sum = 0;
        for (int j = i + 1; j < nc; j++) sum += A[i * nc + j] * X[j];
        X[i] = (b[i] - sum) / A2[i];
    }
}

static void gauss_newton(const double* L, const double* rho, double* be) {
    double X[4] = {0, 0, 0, 0};
    for (int it = 0; it < 5; it++) {
        double A[24], b[6];
        for (int i = 0; i < 6; i++) {
            const double* l = L + 10 * i;
            A[4 * i + 0] = 2 * l[0] * be[0] + l[1] * be[1] + l[3] * be[2] + l[6] * be[3];
            A[4 * i + 1] = l[1] * be[0] + 2 * l[2] * be[1] + l[4] * be[2] + l[7] * be[3];
            A[4 * i + 2] = l[3] * be[0] + l[4] * be[1] + 2 * l[5] * be[2] + l[8] * be[3];
            A[4 * i + 3] = l[6] * be[0] + l[7] * be[1] + l[8] * be[2] + 2 * l[9] * be[3];
            b[i] = rho[i] - (l[0] * be[0] * be[0] + l[1] * be[0] * be[1] + l[2] * be[1] * be[1] + l[3] * be[0] * be[2] +
                             l[4] * be[1] * be[2] + l[5] * be[2] * be[2] + l[6] * be[0] * be[3] + l[7] * be[1] * be[3] +
                             l[8] * be[2] * be[3] + l[9] * be[3] * be[3]);
        }
        qr_solve(A, b, X);
        for (int i = 0; i < 4; i++) be[i] += X[i];
    }
}

/* blocked sums: acc[a] over points, term(i, a) produced by the caller per block */
typedef struct {
    const double *pw, *us;
    int n;
    double fu, fv, uc, vc;
    double cws[4][3], ccinv[9];
    double* alphas;
} Ep;

static void alphas_of(const Ep* e, const double* p, double* a) {
    for (int j = 0; j < 3; j++)
        a[1 + j] = e->ccinv[3 * j] * (p[0] - e->cws[0][0]) + e->ccinv[3 * j + 1] * (p[1] - e->cws[0][1]) +
                   e->ccinv[3 * j + 2] * (p[2] - e->cws[0][2]);
    a[0] = 1.0 - a[1] - a[2] - a[3];
}

static void pc_of(const double* a, double ccs[4][3], double* pc) {
    for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
}

/* compute_pose on n points (pw: n x 3, us: n x 2 pixel observations). */
void orc_epnp(const double* pw, const double* us, int n, const double* cam4, double* Rout, double* tout) {
    Ep e;
    e.pw = pw; e.us = us; e.n = n;
    e.fu = cam4[0]; e.fv = cam4[1]; e.uc = cam4[2]; e.vc = cam4[3];
    const int nblk = (n + EPNP_BLOCK - 1) / EPNP_BLOCK;
    /* centroid */
    double sum[3] = {0, 0, 0};
    for (int bk = 0; bk < nblk; bk++) {
        double loc[3] = {0, 0, 0};
        for (int i = bk * EPNP_BLOCK; i < n && i < (bk + 1) * EPNP_BLOCK; i++)
            for (int j = 0; j < 3; j++) loc[j] += pw[3 * i + j];
        for (int j = 0; j < 3; j++) sum[j] += loc[j];
    }
    for (int j = 0; j < 3; j++) e.cws[0][j] = sum[j] / n;
    /* PCA: PW0^T PW0 */
    double P[9];
    {
        double tot[6] = {0, 0, 0, 0, 0, 0};
        for (int bk = 0; bk < nblk; bk++) {
            double loc[6] = {0, 0, 0, 0, 0, 0};
            for (int i = bk * EPNP_BLOCK; i < n && i < (bk + 1) * EPNP_BLOCK; i++) {
                double d[3];
                for (int j = 0; j < 3; j++) d[j] = pw[3 * i + j] - e.cws[0][j];
                int o = 0;
                for (int a = 0; a < 3; a++)
                    for (int b = a; b < 3; b++) loc[o++] += d[a] * d[b];
            }
            for (int o = 0; o < 6; o++) tot[o] += loc[o];
        }
        int o = 0;
        for (int a = 0; a < 3; a++)
            for (int b = a; b < 3; b++, o++) P[3 * a + b] = P[3 * b + a] = tot[o];
    }
    {
        double At[9], dc[3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) At[3 * i + j] = P[3 * j + i];
        jsvd(At, dc, NULL, 3, 3);
        for (int i = 1; i < 4; i++) {
            double k = sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; j++) e.cws[i][j] = e.cws[0][j] + k * At[3 * (i - 1) + j];
        }
        double CCt[9], w[3], Vt[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) CCt[3 * (j - 1) + i] = e.cws[j][i] - e.cws[0][i];
        jsvd(CCt, w, Vt, 3, 3);
        svbksb(CCt, w, Vt, 3, 3, NULL, e.ccinv);
    }
    double* al = (double*)malloc(sizeof(double) * 4 * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) alphas_of(&e, pw + 3 * i, al + 4 * i);
    /* M^T M */
    double mtm[78];
    memset(mtm, 0, sizeof(mtm));
    for (int bk = 0; bk < nblk; bk++) {
        double loc[78];
        memset(loc, 0, sizeof(loc));
        for (int i = bk * EPNP_BLOCK; i < n && i < (bk + 1) * EPNP_BLOCK; i++) {
            double r1[12], r2[12];
            const double* a = al + 4 * i;
            for (int q = 0; q < 4; q++) {
                r1[3 * q] = a[q] * e.fu; r1[3 * q + 1] = 0.0; r1[3 * q + 2] = a[q] * (e.uc - us[2 * i]);
                r2[3 * q] = 0.0; r2[3 * q + 1] = a[q] * e.fv; r2[3 * q + 2] = a[q] * (e.vc - us[2 * i + 1]);
            }
            int o = 0;
            for (int x = 0; x < 12; x++)
                for (int y = x; y < 12; y++, o++) {
                    loc[o] += r1[x] * r1[y];
                    loc[o] += r2[x] * r2[y];
                }
        }
        for (int o = 0; o < 78; o++) mtm[o] += loc[o];
    }
    double ut[144], dw[12];
    {
        int o = 0;
        for (int x = 0; x < 12; x++)
            for (int y = x; y < 12; y++, o++) ut[12 * x + y] = ut[12 * y + x] = mtm[o];
        jsvd(ut, dw, NULL, 12, 12);
    }
    /* L_6x10, rho */
    double L[60], rho[6];
    {
        const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
        double dv[4][6][3];
        for (int i = 0; i < 4; i++) {
            int a = 0, b = 1;
            for (int j = 0; j < 6; j++) {
                for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
                b++;
                if (b > 3) { a++; b = a + 1; }
            }
        }
        for (int i = 0; i < 6; i++) {
            double* row = L + 10 * i;
            row[0] = dot3(dv[0][i], dv[0][i]);
            row[1] = 2.0 * dot3(dv[0][i], dv[1][i]);
            row[2] = dot3(dv[1][i], dv[1][i]);
            row[3] = 2.0 * dot3(dv[0][i], dv[2][i]);
            row[4] = 2.0 * dot3(dv[1][i], dv[2][i]);
            row[5] = dot3(dv[2][i], dv[2][i]);
            row[6] = 2.0 * dot3(dv[0][i], dv[3][i]);
            row[7] = 2.0 * dot3(dv[1][i], dv[3][i]);
            row[8] = 2.0 * dot3(dv[2][i], dv[3][i]);
            row[9] = dot3(dv[3][i], dv[3][i]);
        }
        int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
        for (int i = 0; i < 6; i++) {
            const double *p1 = e.cws[pa[i]], *p2 = e.cws[pb[i]];
            rho[i] = (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) +
                     (p1[2] - p2[2]) * (p1[2] - p2[2]);
        }
    }
    double betas[4][4];
    memset(betas, 0, sizeof(betas));
    {
        double L4[24], b4[4];
        for (int i = 0; i < 6; i++) {
            L4[4 * i] = L[10 * i]; L4[4 * i + 1] = L[10 * i + 1]; L4[4 * i + 2] = L[10 * i + 3]; L4[4 * i + 3] = L[10 * i + 6];
        }
        solve6(L4, 4, rho, b4);
        double* be = betas[1];
        if (b4[0] < 0) {
            be[0] = sqrt(-b4[0]); be[1] = -b4[1] / be[0]; be[2] = -b4[2] / be[0]; be[3] = -b4[3] / be[0];
        } else {
            be[0] = sqrt(b4[0]); be[1] = b4[1] / be[0]; be[2] = b4[2] / be[0]; be[3] = b4[3] / be[0];
        }
        gauss_newton(L, rho, be);
    }
    {
        double L3[18], b3[3];
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < 3; k++) L3[3 * i + k] = L[10 * i + k];
        solve6(L3, 3, rho, b3);
        double* be = betas[2];
        if (b3[0] < 0) {
            be[0] = sqrt(-b3[0]);
            be[1] = (b3[2] < 0) ? sqrt(-b3[2]) : 0.0;
        } else {
            be[0] = sqrt(b3[0]);
            be[1] = (b3[2] > 0) ? sqrt(b3[2]) : 0.0;
        }
        if (b3[1] < 0) be[0] = -be[0];
        be[2] = 0.0; be[3] = 0.0;
        gauss_newton(L, rho, be);
    }
    {
        double L5[30], b5[5];
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < 5; k++) L5[5 * i + k] = L[10 * i + k];
        solve6(L5, 5, rho, b5);
        double* be = betas[3];
        if (b5[0] < 0) {
            be[0] = sqrt(-b5[0]);
            be[1] = (b5[2] < 0) ? sqrt(-b5[2]) : 0.0;
        } else {
            be[0] = sqrt(b5[0]);
            be[1] = (b5[2] > 0) ? sqrt(b5[2]) : 0.0;
        }
        if (b5[1] < 0) be[0] = -be[0];
        be[2] = b5[3] / be[0];
        be[3] = 0.0;
        gauss_newton(L, rho, be);
    }
    double pw0[3];
    for (int j = 0; j < 3; j++) pw0[j] = sum[j] / n;
    double rep[4] = {0, 0, 0, 0}, Rs[4][9], ts[4][3];
    for (int N = 1; N <= 3; N++) {
        double ccs[4][3];
        for (int j = 0; j < 4; j++)
            for (int k = 0; k < 3; k++) ccs[j][k] = 0.0;
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (11 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += betas[N][i] * v[3 * j + k];
        }
        double pcf[3];
        pc_of(al, ccs, pcf);
        if (pcf[2] < 0.0)
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] = -ccs[j][k];
        double pc0[3] = {0, 0, 0};
        for (int bk = 0; bk < nblk; bk++) {
            double loc[3] = {0, 0, 0};
            for (int i = bk * EPNP_BLOCK; i < n && i < (bk + 1) * EPNP_BLOCK; i++) {
                double pc[3];
                pc_of(al + 4 * i, ccs, pc);
                for (int j = 0; j < 3; j++) loc[j] += pc[j];
            }
            for (int j = 0; j < 3; j++) pc0[j] += loc[j];
        }
        for (int j = 0; j < 3; j++) pc0[j] /= n;
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int bk = 0; bk < nblk; bk++) {
            double loc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int i = bk * EPNP_BLOCK; i < n && i < (bk + 1) * EPNP_BLOCK; i++) {
                double pc[3];
                pc_of(al + 4 * i, ccs, pc);
                for (int j = 0; j < 3; j++)
                    for (int k = 0; k < 3; k++) loc[3 * j + k] += (pc[j] - pc0[j]) * (pw[3 * i + k] - pw0[k]);
            }
            for (int o = 0; o < 9; o++) abt[o] += loc[o];
        }
        /* cvSVD(ABt, D, U, V): Jacobi on ABt^T; R = U V^T, U[i][k] = At[k][i], V[j][k] = Vt[k][j] */
        double At[9], w[3], Vt[9], R[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) At[3 * i + j] = abt[3 * j + i];
        jsvd(At, w, Vt, 3, 3);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                R[3 * i + j] = At[i] * Vt[j] + At[3 + i] * Vt[3 + j] + At[6 + i] * Vt[6 + j];
        double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                     R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
        if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
        double t[3];
        for (int i = 0; i < 3; i++) t[i] = pc0[i] - dot3(R + 3 * i, pw0);
        double s = 0;
        for (int bk = 0; bk < nblk; bk++) {
            double loc = 0;
            for (int i = bk * EPNP_BLOCK; i < n && i < (bk + 1) * EPNP_BLOCK; i++) {
                const double* p = pw + 3 * i;
                double Xc = dot3(R, p) + t[0];
                double Yc = dot3(R + 3, p) + t[1];
                double inv_Zc = 1.0 / (dot3(R + 6, p) + t[2]);
                double ue = e.uc + e.fu * Xc * inv_Zc;
                double ve = e.vc + e.fv * Yc * inv_Zc;
                double u = us[2 * i], v = us[2 * i + 1];
                loc += sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
            }
            s += loc;
        }
        rep[N] = s / n;
        memcpy(Rs[N], R, sizeof(R));
        memcpy(ts[N], t, sizeof(t));
    }
    free(al);
    int N = 1;
    if (rep[2] < rep[1]) N = 2;
    if (rep[3] < rep[N]) N = 3;
    memcpy(Rout, Rs[N], sizeof(double) * 9);
    memcpy(tout, ts[N], sizeof(double) * 3);
}

/* A 5-point RANSAC subset as PnPRansacCallback::runKernel feeds EPnP: undistortPoints with a float
   result, pixels x * f + c in double, float world points. */
void orc_epnp5_f32(const float* p5 /* 5 x 8 PnpPoint floats */, const double* cam8, double* R, double* t) {
    double pw[15], us[10];
    for (int i = 0; i < 5; i++) {
        const float* p = p5 + 8 * i;
        double x, y;
        orc_undistort(cam8, (double)p[3], (double)p[4], &x, &y);
        us[2 * i] = (double)(float)x * cam8[0] + cam8[2];
        us[2 * i + 1] = (double)(float)y * cam8[1] + cam8[3];
        pw[3 * i] = p[0]; pw[3 * i + 1] = p[1]; pw[3 * i + 2] = p[2];
    }
    orc_epnp(pw, us, 5, cam8, R, t);
}

int orc_pnp_hypothesis_epnp(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R,
                            double* t, int* idx_out) {
    Stream st;
    st.seed = seed; st.hyp = (uint64_t)hyp; st.pos = 0;
    int idx[5];
    for (int a = 0; a < ORC_MAX_ATTEMPTS; ++a) {
        if (!draw_distinct(&st, N, 5, idx)) continue;
        float p5[40];
        for (int i = 0; i < 5; i++) memcpy(p5 + 8 * i, pts + 8 * (size_t)idx[i], 8 * sizeof(float));
        if (idx_out) memcpy(idx_out, idx, sizeof(idx));
        orc_epnp5_f32(p5, cam8, R, t);
        return 1;
    }
    return ORC_NO_SAMPLE;
}

/* The inlier / all-points EPnP of solvePnP(EPNP) on double inputs: undistortPoints (double
   result) -> x * f + c. img: n x 2, world: n x 3 (doubles). */
void orc_epnp_points(const double* img, const double* world, int n, const double* cam8, double* R, double* t) {
    double* us = (double*)malloc(sizeof(double) * 2 * (size_t)(n > 0 ? n : 1));
    for (int i = 0; i < n; i++) {
        double x, y;
        orc_undistort(cam8, img[2 * i], img[2 * i + 1], &x, &y);
        us[2 * i] = x * cam8[0] + cam8[2];
        us[2 * i + 1] = y * cam8[1] + cam8[3];
    }
    orc_epnp(world, us, n, cam8, R, t);
    free(us);
}
