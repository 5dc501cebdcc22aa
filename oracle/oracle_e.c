/*
 * oracle_e.c — CPU restatement of the essential-matrix path. TEST
 * INFRASTRUCTURE ONLY (see oracle.c's header for the rules and the parity status).
 *
 * Follows the reference's five-point solver /root/reference/src/MiniCVNative/fivepoint.cpp:233-339
 * (runFivepoint: Q rows :239-248, null space :250-256, coefficient matrix :258-260 with the
 * getCoeffMat column order, elimination :262, B(z) :264-297, degree-10 determinant :299-309,
 * real roots + back-substitution :314-335) and the exports MiniCVNative.cpp:165-215 (findEssentialMat
 * -> mask copy -> decomposeEssentialMat / recoverPose), with OpenCV 4.x findEssentialMat /
 * EMEstimatorCallback / recoverPose / triangulatePoints restated [ext]. The deterministic
 * replacements of SVD / Mat::inv / solvePoly are the build's definition; this file
 * implements that definition independently of minicv_amd/csrc/hyp_essential.h, with the same
 * operation order so models and masks agree bit for bit.
 *
 * Pinned by: exact synthetic two-view geometry (an E = [t]x R built from a known pose must be
 * among the solutions; the chosen pose must equal the true one), the algebraic constraints of
 * every returned E (det E = 0, 2 E E^T E - tr(E E^T) E = 0, x2^T E x1 = 0 on the sample), and
 * agreement of the product's GPU path with this restatement. No OpenCV output is available here.
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

#define EMAX 10

/* ---- ordered doubles --------------------------------------------------------------------- */
static int64_t key_of(double x) {
    int64_t i;
    memcpy(&i, &x, 8);
    if (i < 0) i = (int64_t)(0x8000000000000000ull - (uint64_t)i);
    return i;
}
static double val_of(int64_t k) {
    if (k < 0) k = (int64_t)(0x8000000000000000ull - (uint64_t)k);
    double x;
    memcpy(&x, &k, 8);
    return x;
}

/* m! / (m-j)! */
static double falling(int m, int j) {
    double r = 1.0;
    for (int k = 0; k < j; ++k) r = r * (double)(m - k);
    return r;
}

static double horner(const double* q, int d, double x) {
    double f = q[d];
    for (int k = d - 1; k >= 0; --k) f = f * x + q[k];
    return f;
}

/* Illinois regula falsi with bit-pattern bisection safeguards, to a 1-ulp bracket */
static double root_in(const double* q, int d, double lo, double hi, double flo, double fhi) {
    int side = 0, stall = 0;
    for (int it = 0; it < 256; ++it) {
        int64_t a = key_of(lo), b = key_of(hi), mid = (a >> 1) + (b >> 1) + (a & b & 1);
        if (mid == a || mid == b) break;
        double m;
        if (stall >= 2) {
            m = val_of(mid);
            stall = 0;
        } else {
            m = lo - flo * ((hi - lo) / (fhi - flo));
            if (!(m > lo && m < hi)) m = val_of(mid);
        }
        double fm = horner(q, d, m);
        if (fm == 0) return m;
        uint64_t before = (uint64_t)b - (uint64_t)a, after;
        int64_t km = key_of(m);
        if ((fm < 0) == (flo < 0)) {
            after = (uint64_t)b - (uint64_t)km;
            lo = m; flo = fm;
            if (side == -1) fhi = fhi * 0.5;
            side = -1;
        } else {
            after = (uint64_t)km - (uint64_t)a;
            hi = m; fhi = fm;
            if (side == 1) flo = flo * 0.5;
            side = 1;
        }
        stall = after > before / 2 ? stall + 1 : 0;
    }
    return lo;
}

/* real roots ascending of sum cin[k] z^k (deg <= 10): Rolle intervals from the derivatives */
int orc_poly_real_roots(const double* cin, int deg, double* roots) {
    int n = deg;
    while (n > 0 && cin[n] == 0) --n;
    if (n < 1) return 0;
    double c[11], R = 0;
    for (int k = 0; k <= n; ++k) c[k] = cin[k] / cin[n];
    for (int k = 0; k < n; ++k) R = fabs(c[k]) > R ? fabs(c[k]) : R;
    R = 1.0 + R;
    if (!isfinite(R)) return 0;
    double crit[10], cur[10], q[11];
    int ncrit = 0;
    for (int j = n - 1; j >= 0; --j) {
        int d = n - j, nc = 0;
        for (int k = 0; k <= d; ++k) q[k] = c[k + j] * falling(k + j, j);
        double a = -R, fa = horner(q, d, a);
        for (int s = 0; s <= ncrit; ++s) {
            double b = s < ncrit ? crit[s] : R, fb = horner(q, d, b);
            if (fb == 0) {
                if (nc == 0 || cur[nc - 1] != b) cur[nc++] = b;
            } else if (fa != 0 && ((fa < 0) != (fb < 0))) {
                cur[nc++] = root_in(q, d, a, b, fa, fb);
            }
            a = b;
            fa = fb;
        }
        memcpy(crit, cur, sizeof(double) * (size_t)nc);
        ncrit = nc;
    }
    memcpy(roots, crit, sizeof(double) * (size_t)ncrit);
    return ncrit;
}

/* ---- null space of the 5 x 9 epipolar system: Gauss-Jordan, full pivoting, then MGS ------ */
static int null_basis(const double* x1, const double* y1, const double* x2, const double* y2, double nb[4][9]) {
    double M[5][9], scale = 0;
    int col[9];
    for (int i = 0; i < 5; ++i) {
        const double row[9] = {x1[i] * x2[i], y1[i] * x2[i], x2[i], x1[i] * y2[i], y1[i] * y2[i], y2[i],
                               x1[i], y1[i], 1.0};
        for (int k = 0; k < 9; ++k) {
            M[i][k] = row[k];
            if (fabs(row[k]) > scale) scale = fabs(row[k]);
        }
    }
    if (!(scale > 0) || !isfinite(scale)) return 0;
    for (int k = 0; k < 9; ++k) col[k] = k;
    for (int r = 0; r < 5; ++r) {
        double best = -1;
        int bi = r, bj = r;
        for (int i = r; i < 5; ++i)
            for (int j = r; j < 9; ++j)
                if (fabs(M[i][col[j]]) > best) { best = fabs(M[i][col[j]]); bi = i; bj = j; }
        if (!(best > 1e-12 * scale)) return 0;
        double tmp[9];
        memcpy(tmp, M[r], sizeof(tmp)); memcpy(M[r], M[bi], sizeof(tmp)); memcpy(M[bi], tmp, sizeof(tmp));
        int tc = col[r]; col[r] = col[bj]; col[bj] = tc;
        double piv = M[r][col[r]];
        for (int j = r + 1; j < 9; ++j) M[r][col[j]] = M[r][col[j]] / piv;
        M[r][col[r]] = 1.0;
        for (int i = 0; i < 5; ++i) {
            if (i == r) continue;
            double f = M[i][col[r]];
            for (int j = r + 1; j < 9; ++j) M[i][col[j]] = M[i][col[j]] - f * M[r][col[j]];
            M[i][col[r]] = 0.0;
        }
    }
    for (int b = 0; b < 4; ++b) {
        double* v = nb[b];
        memset(v, 0, sizeof(double) * 9);
        v[col[5 + b]] = 1.0;
        for (int r = 0; r < 5; ++r) v[col[r]] = -M[r][col[5 + b]];
        for (int c = 0; c < b; ++c) {
            double d = 0;
            for (int k = 0; k < 9; ++k) d = d + nb[c][k] * v[k];
            for (int k = 0; k < 9; ++k) v[k] = v[k] - d * nb[c][k];
        }
        double s = 0;
        for (int k = 0; k < 9; ++k) s = s + v[k] * v[k];
        double nrm = sqrt(s);
        if (!(nrm > 0)) return 0;
        for (int k = 0; k < 9; ++k) v[k] = v[k] / nrm;
    }
    return 1;
}

/* ---- cubic constraints ---------------------------------------------------------------------
 * Variables (x, y, z, w = 1) = indices 0..3. Quadratics as symmetric Q[a][b] (a <= b used).
 * Cubic column of x^ex y^ey z^ez (ex + ey + ez <= 3), getCoeffMat order:
 * x3 y3 x2y xy2 x2z x2 y2z y2 xyz xy | xz2 xz x yz2 yz y z3 z2 z 1. */
static int cubic_col(int ex, int ey, int ez) {
    static const int tab[4][4][4] = {
        /* ex = 0 */ {{19, 18, 17, 16}, {15, 14, 13, -1}, {7, 6, -1, -1}, {1, -1, -1, -1}},
        /* ex = 1 */ {{12, 11, 10, -1}, {9, 8, -1, -1}, {3, -1, -1, -1}, {-1, -1, -1, -1}},
        /* ex = 2 */ {{5, 4, -1, -1}, {2, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}},
        /* ex = 3 */ {{0, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}, {-1, -1, -1, -1}}};
    return tab[ex][ey][ez];
}

static void qmul(const double* l, const double* m, double Q[4][4]) {
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b) Q[a][b] = a == b ? l[a] * m[a] : l[a] * m[b] + l[b] * m[a];
}

static void cubic_acc(double* row, double Q[4][4], const double* l) {
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b)
            for (int c = 0; c < 4; ++c) {
                int e[4] = {0, 0, 0, 0};
                e[a]++; e[b]++; e[c]++;
                int k = cubic_col(e[0], e[1], e[2]);
                row[k] = row[k] + Q[a][b] * l[c];
            }
}

static void constraint_matrix(double nb[4][9], double A[10][20]) {
    double E[9][4];   /* E[k] = linear form of entry k */
    for (int k = 0; k < 9; ++k)
        for (int v = 0; v < 4; ++v) E[k][v] = nb[v][k];
    memset(A, 0, sizeof(double) * 200);
    /* det */
    static const int co[3][4] = {{4, 8, 5, 7}, {5, 6, 3, 8}, {3, 7, 4, 6}};
    for (int i = 0; i < 3; ++i) {
        double P[4][4], Qm[4][4], D[4][4];
        qmul(E[co[i][0]], E[co[i][1]], P);
        qmul(E[co[i][2]], E[co[i][3]], Qm);
        for (int a = 0; a < 4; ++a)
            for (int b = a; b < 4; ++b) D[a][b] = P[a][b] - Qm[a][b];
        cubic_acc(A[0], D, E[i]);
    }
    /* E E^T, trace */
    double S[3][3][4][4];
    for (int i = 0; i < 3; ++i)
        for (int j = i; j < 3; ++j) {
            qmul(E[3 * i], E[3 * j], S[i][j]);
            for (int k = 1; k < 3; ++k) {
                double P[4][4];
                qmul(E[3 * i + k], E[3 * j + k], P);
                for (int a = 0; a < 4; ++a)
                    for (int b = a; b < 4; ++b) S[i][j][a][b] = S[i][j][a][b] + P[a][b];
            }
        }
    double T[4][4];
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b) T[a][b] = S[0][0][a][b] + S[1][1][a][b] + S[2][2][a][b];
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) {
            double L[4][4];
            for (int a = 0; a < 4; ++a)
                for (int b = a; b < 4; ++b) {
                    double s = i <= k ? S[i][k][a][b] : S[k][i][a][b];
                    L[a][b] = 2.0 * s - (i == k ? T[a][b] : 0.0);
                }
            for (int j = 0; j < 3; ++j) cubic_acc(A[1 + 3 * i + j], L, E[3 * k + j]);
        }
}

static int reduce10(double A[10][20], double C[10][10]) {
    double scale = 0;
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 20; ++c) scale = fabs(A[r][c]) > scale ? fabs(A[r][c]) : scale;
    if (!(scale > 0) || !isfinite(scale)) return 0;
    for (int c = 0; c < 10; ++c) {
        int p = c;
        for (int r = c + 1; r < 10; ++r)
            if (fabs(A[r][c]) > fabs(A[p][c])) p = r;
        if (!(fabs(A[p][c]) > 1e-13 * scale)) return 0;
        if (p != c)
            for (int k = c; k < 20; ++k) { double t = A[c][k]; A[c][k] = A[p][k]; A[p][k] = t; }
        double piv = A[c][c];
        for (int k = c + 1; k < 20; ++k) A[c][k] = A[c][k] / piv;
        for (int r = 0; r < 10; ++r) {
            if (r == c) continue;
            double f = A[r][c];
            for (int k = c + 1; k < 20; ++k) A[r][k] = A[r][k] - f * A[c][k];
        }
    }
    for (int r = 0; r < 10; ++r) memcpy(C[r], &A[r][10], sizeof(double) * 10);
    return 1;
}

static void pmul(const double* a, int da, const double* b, int db, double* r) {
    for (int k = 0; k <= da + db; ++k) r[k] = 0.0;
    for (int i = 0; i <= da; ++i)
        for (int j = 0; j <= db; ++j) r[i + j] = r[i + j] + a[i] * b[j];
}

static double peval(const double* c, int n, double z) {
    double f = c[n];
    for (int k = n - 1; k >= 0; --k) f = f * z + c[k];
    return f;
}

/* Five-point solve; returns the number of unit-norm E written to E[10][9]. */
int orc_e_solve5(const double* x1, const double* y1, const double* x2, const double* y2, double* Eout) {
    double nb[4][9], A[10][20], C[10][10];
    if (!null_basis(x1, y1, x2, y2, nb)) return 0;
    constraint_matrix(nb, A);
    if (!reduce10(A, C)) return 0;
    /* B(z) rows, ascending powers: X (deg 3), Y (deg 3), K (deg 4) */
    double X[3][4], Y[3][4], K[3][5];
    for (int i = 0; i < 3; ++i) {
        const double* e = C[4 + 2 * i];
        const double* f = C[5 + 2 * i];
        X[i][3] = 0.0 - f[0]; X[i][2] = e[0] - f[1]; X[i][1] = e[1] - f[2]; X[i][0] = e[2] - 0.0;
        Y[i][3] = 0.0 - f[3]; Y[i][2] = e[3] - f[4]; Y[i][1] = e[4] - f[5]; Y[i][0] = e[5] - 0.0;
        K[i][4] = 0.0 - f[6]; K[i][3] = e[6] - f[7]; K[i][2] = e[7] - f[8]; K[i][1] = e[8] - f[9];
        K[i][0] = e[9] - 0.0;
    }
    double u[8], v[8], w7[8], P1[11], P2[11], P3[11], a6[7], b6[7], w6[7], det[11];
    pmul(Y[1], 3, K[2], 4, u); pmul(Y[2], 3, K[1], 4, v);
    for (int k = 0; k < 8; ++k) w7[k] = u[k] - v[k];
    pmul(X[0], 3, w7, 7, P1);
    pmul(X[1], 3, K[2], 4, u); pmul(X[2], 3, K[1], 4, v);
    for (int k = 0; k < 8; ++k) w7[k] = u[k] - v[k];
    pmul(Y[0], 3, w7, 7, P2);
    pmul(X[1], 3, Y[2], 3, a6); pmul(X[2], 3, Y[1], 3, b6);
    for (int k = 0; k < 7; ++k) w6[k] = a6[k] - b6[k];
    pmul(K[0], 4, w6, 6, P3);
    for (int k = 0; k < 11; ++k) det[k] = P1[k] - P2[k] + P3[k];
    double zs[10];
    int nz = orc_poly_real_roots(det, 10, zs), count = 0;
    for (int s = 0; s < nz; ++s) {
        double z = zs[s], B[3][3];
        for (int i = 0; i < 3; ++i) { B[i][0] = peval(X[i], 3, z); B[i][1] = peval(Y[i], 3, z); B[i][2] = peval(K[i], 4, z); }
        static const int ra[3] = {0, 0, 1}, rb[3] = {1, 2, 2};
        double nv2 = -1, n[3] = {0, 0, 0};
        for (int q = 0; q < 3; ++q) {
            const double* p = B[ra[q]];
            const double* o = B[rb[q]];
            double c0 = p[1] * o[2] - p[2] * o[1], c1 = p[2] * o[0] - p[0] * o[2], c2 = p[0] * o[1] - p[1] * o[0];
            double m2 = c0 * c0 + c1 * c1 + c2 * c2;
            if (m2 > nv2) { nv2 = m2; n[0] = c0; n[1] = c1; n[2] = c2; }
        }
        double nv = sqrt(nv2);
        if (!(nv > 0) || !(fabs(n[2]) >= 1e-10 * nv)) continue;
        double x = n[0] / n[2], y = n[1] / n[2], e[9], ss = 0;
        for (int k = 0; k < 9; ++k) {
            e[k] = x * nb[0][k] + y * nb[1][k] + z * nb[2][k] + nb[3][k];
            ss = ss + e[k] * e[k];
        }
        double ns = sqrt(ss);
        if (!(ns > 0) || !isfinite(ns)) continue;
        for (int k = 0; k < 9; ++k) Eout[9 * count + k] = e[k] / ns;
        ++count;
    }
    return count;
}

/* ---- the reference's own five-point path (fivepoint.cpp:233-339, runFivepoint) ----------------
 * Default minimal solver of the RANSAC path and the cvFivePoint export. Every step restated in the
 * reference's (and OpenCV 4.x's [ext]) operation order:
 *  - null space: SVD::compute(Q, W, U, Vt, MODIFY_A | FULL_UV) of the 5 x 9 system (:252) = JacobiSVD on
 *    Q's rows with the four completion rows drawn by cv::RNG(0x12345678) (orc_jsvd); EE = Vt rows 5..8;
 *  - the 10 x 20 constraint matrix: getCoeffMat (:10-231), every entry's expression evaluated term by
 *    term in the source's order from fivepoint_terms.inc (generated from the reference's text by
 *    scripts/gen/gen_fivepoint_terms.py), then its column permutation perm[20] (:220-225);
 *  - A = A.colRange(0, 10).inv() * A.colRange(10, 20) (:260): OpenCV evaluates inv(X) * Y as
 *    cv::solve(X, Y, DECOMP_LU) [ext: matop.cpp MatOp_Invert::matmul -> MatOp_Solve] = LUImpl on X with
 *    the ten right-hand sides (eps 100 DBL_EPSILON), not an explicit inverse;
 *  - B (3 x 13) = row1 - row2 from rows 4..9 (:262-277), the degree-10 coefficients c[] (:299-309)
 *    term by term from fivepoint_terms.inc;
 *  - cv::solvePoly (Durand-Kerner, 300 sweeps, OpenCV Complex arithmetic), roots with |Im| <= 1e-10 in
 *    solvePoly's order; Bz rows (:318-323); SVD::solveZ (last row of Vt of the 3 x 3 JacobiSVD);
 *    |xy1[2]| < 1e-10 skips; Evec = ((X x + Y y) + 0) + Z z + W (addWeighted, scaleAdd, add), Evec /= norm
 *    (normL2Sqr's 4-way unrolled sum; convertTo by 1 / norm).
 * Divergences (degenerate samples only): a singular 10 x 10 block (|pivot| < 100 DBL_EPSILON) gives no
 * model here, where cv::solve returns zeros and the reference goes on to NaN / arbitrary models; a
 * leading coefficient |c[10]| <= DBL_EPSILON repeats the last root where solvePoly copies uninitialised
 * buffer entries. */
#include "fivepoint_terms.inc"

static double fp_factor(unsigned char f, const double* v) {
    const int k = f >> 6, i = f & 63;
    if (k == 0) return orc_fp_literals[i];
    if (k == 1) return v[i];
    const double p2 = v[i] * v[i];
    return k == 2 ? p2 : p2 * v[i];
}

static double fp_sum(const OrcFpTerm* t, int n, const double* v) {
    double acc = 0;
    for (int j = 0; j < n; ++j) {
        double p = fp_factor(t[j].f[0], v);
        for (int q = 1; q < 4 && t[j].f[q] != 0xFF; ++q) p = p * fp_factor(t[j].f[q], v);
        if (t[j].neg) p = -p;
        acc = j == 0 ? p : acc + p;
    }
    return acc;
}

/* getCoeffMat(e, A): e = EE^T (4 x 9 row-major), A row-major 10 x 20 after the column permutation */
void orc_fp_coeff_matrix(const double* e, double* A) {
    double Araw[200];
    for (int k = 0; k < 200; ++k)
        Araw[k] = fp_sum(orc_fp_a_terms + orc_fp_a_start[k], orc_fp_a_start[k + 1] - orc_fp_a_start[k], e);
    for (int i = 0; i < 20; ++i)
        for (int j = 0; j < 10; ++j) A[i + 20 * j] = Araw[orc_fp_perm[i] + 20 * j];
}

void orc_fp_det_coeffs(const double* b, double* c) {
    for (int k = 0; k < 11; ++k)
        c[k] = fp_sum(orc_fp_c_terms + orc_fp_c_start[k], orc_fp_c_start[k + 1] - orc_fp_c_start[k], b);
}

/* LUImpl<double>(A, 10, b, 10 right-hand sides), eps = 100 DBL_EPSILON; b <- A^-1 b. */
static int lu_solve10(double A[10][10], double b[10][10]) {
    const double eps = DBL_EPSILON * 100;
    for (int i = 0; i < 10; ++i) {
        int k = i;
        for (int j = i + 1; j < 10; ++j)
            if (fabs(A[j][i]) > fabs(A[k][i])) k = j;
        if (fabs(A[k][i]) < eps) return 0;
        if (k != i) {
            for (int j = i; j < 10; ++j) { double t = A[i][j]; A[i][j] = A[k][j]; A[k][j] = t; }
            for (int j = 0; j < 10; ++j) { double t = b[i][j]; b[i][j] = b[k][j]; b[k][j] = t; }
        }
        double d = -1 / A[i][i];
        for (int j = i + 1; j < 10; ++j) {
            double alpha = A[j][i] * d;
            for (int q = i + 1; q < 10; ++q) A[j][q] += alpha * A[i][q];
            for (int q = 0; q < 10; ++q) b[j][q] += alpha * b[i][q];
        }
        A[i][i] = -d;
    }
    for (int i = 9; i >= 0; --i)
        for (int j = 0; j < 10; ++j) {
            double s = b[i][j];
            for (int q = i + 1; q < 10; ++q) s -= A[i][q] * b[q][j];
            b[i][j] = s * A[i][i];
        }
    return 1;
}

/* cv::solvePoly(c (ascending, degree 10), roots, 300): re[10], im[10] */
void orc_solve_poly10(const double* c, double* rre, double* rim) {
    double cre[11], cim[11];
    for (int i = 0; i <= 10; ++i) { cre[i] = c[i]; cim[i] = 0.0; }
    int n = 10;
    for (; n > 1; --n)
        if (fabs(cre[n]) + fabs(cim[n]) > DBL_EPSILON) break;
    double pre = 1, pim = 0;
    for (int i = 0; i < 10; ++i) { rre[i] = 0; rim[i] = 0; }
    for (int i = 0; i < n; ++i) {
        rre[i] = pre; rim[i] = pim;
        double t = pre * 1 - pim * 1;
        pim = pre * 1 + pim * 1;
        pre = t;
    }
    for (int iter = 0; iter < 300; ++iter) {
        double maxDiff = 0;
        for (int i = 0; i < n; ++i) {
            pre = rre[i]; pim = rim[i];
            double nre = cre[n], nim = cim[n], dre = cre[n], dim = cim[n];
            for (int j = 0; j < n; ++j) {
                double tre = nre * pre - nim * pim + cre[n - j - 1];
                double tim = nre * pim + nim * pre + cim[n - j - 1];
                nre = tre; nim = tim;
                if (j != i) {
                    double ere = pre - rre[j], eim = pim - rim[j];
                    double ure = dre * ere - dim * eim, uim = dre * eim + dim * ere;
                    dre = ure; dim = uim;
                }
            }
            double t = 1. / (dre * dre + dim * dim);
            double qre = (nre * dre + nim * dim) * t, qim = (-nre * dim + nim * dre) * t;
            rre[i] = pre - qre;
            rim[i] = pim - qim;
            double a = sqrt(qre * qre + qim * qim);
            maxDiff = maxDiff < a ? a : maxDiff;   /* std::max(maxDiff, cv::abs(num)) */
        }
        if (maxDiff <= 0) break;
    }
    for (; n < 10; ++n) { rre[n] = rre[n - 1]; rim[n] = rim[n - 1]; }
}

/* B (3 x 13, row-major as fivepoint.cpp's b[39]) from the solved 10 x 10 block C */
static void fp_b_matrix(double C[10][10], double* b) {
    for (int i = 0; i < 3; ++i) {
        const double* r1 = C[2 * i + 4];
        const double* r2 = C[2 * i + 5];
        double row1[13] = {0}, row2[13] = {0};
        for (int k = 0; k < 3; ++k) { row1[1 + k] = r1[k] * 1.0; row1[5 + k] = r1[3 + k] * 1.0; row2[k] = r2[k] * 1.0; row2[4 + k] = r2[3 + k] * 1.0; }
        for (int k = 0; k < 4; ++k) { row1[9 + k] = r1[6 + k] * 1.0; row2[8 + k] = r2[6 + k] * 1.0; }
        for (int k = 0; k < 13; ++k) b[13 * i + k] = row1[k] - row2[k];
    }
}

/* normL2Sqr<double, double>(a, 9) with CV_ENABLE_UNROLLED [ext: OpenCV core/base.hpp] */
static double norm_l2sqr9(const double* a) {
    double s = 0;
    int i = 0;
    for (; i <= 9 - 4; i += 4) s += a[i] * a[i] + a[i + 1] * a[i + 1] + a[i + 2] * a[i + 2] + a[i + 3] * a[i + 3];
    for (; i < 9; ++i) s += a[i] * a[i];
    return s;
}

int orc_e_solve5_ref(const double* x1, const double* y1, const double* x2, const double* y2, double* Eout) {
    double nb[4][9], A[200], C[10][10];
    {
        double U[81], w[5];
        memset(U, 0, sizeof(U));
        for (int i = 0; i < 5; ++i) {
            double* r = U + 9 * i;
            r[0] = x1[i] * x2[i]; r[1] = y1[i] * x2[i]; r[2] = x2[i] * 1.0;
            r[3] = x1[i] * y2[i]; r[4] = y1[i] * y2[i]; r[5] = y2[i] * 1.0;
            r[6] = x1[i] * 1.0; r[7] = y1[i] * 1.0; r[8] = 1.0;
        }
        orc_jsvd(U, w, NULL, 9, 5, 9);
        for (int b = 0; b < 4; ++b) memcpy(nb[b], U + 9 * (5 + b), sizeof(double) * 9);
    }
    orc_fp_coeff_matrix(&nb[0][0], A);
    {
        double L[10][10];
        for (int r = 0; r < 10; ++r)
            for (int k = 0; k < 10; ++k) { L[r][k] = A[20 * r + k]; C[r][k] = A[20 * r + 10 + k]; }
        if (!lu_solve10(L, C)) return 0;
    }
    double b[39], c[11];
    fp_b_matrix(C, b);
    orc_fp_det_coeffs(b, c);
    double rre[10], rim[10];
    orc_solve_poly10(c, rre, rim);
    int count = 0;
    for (int i = 0; i < 10; ++i) {
        if (fabs(rim[i]) > 1e-10) continue;
        double z1 = rre[i], z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
        double At[9], w[3], Vt[9];
        for (int j = 0; j < 3; ++j) {
            const double* br = b + 13 * j;
            At[j] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
            At[3 + j] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
            At[6 + j] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
        }
        orc_jsvd(At, w, Vt, 3, 3, 3);
        const double* xy1 = Vt + 6;
        if (fabs(xy1[2]) < 1e-10) continue;
        double x = xy1[0] / xy1[2], y = xy1[1] / xy1[2], e[9];
        for (int k = 0; k < 9; ++k) e[k] = ((nb[0][k] * x + nb[1][k] * y) + 0.0 + nb[2][k] * z1) + nb[3][k];
        double sc = 1. / sqrt(norm_l2sqr9(e));
        for (int k = 0; k < 9; ++k) Eout[9 * count + k] = e[k] * sc + 0.0;
        ++count;
    }
    return count;
}

/* One hypothesis on double4 normalised points. Returns #models, or ORC_NO_SAMPLE. */
int orc_e_hypothesis(const double* pts4, int N, uint64_t seed, int64_t hyp, double* E90, int* idx_out) {
    Stream st;
    st.seed = seed; st.hyp = (uint64_t)hyp; st.pos = 0;
    int idx[5];
    for (int attempt = 0; attempt < ORC_MAX_ATTEMPTS; ++attempt) {
        if (!draw_distinct(&st, N, 5, idx)) continue;
        double x1[5], y1[5], x2[5], y2[5];
        for (int i = 0; i < 5; ++i) {
            const double* p = pts4 + 4 * (size_t)idx[i];
            x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
        }
        if (idx_out) memcpy(idx_out, idx, sizeof(idx));
        /* default: the reference's own solver; MCV_FLAG_FAST_MINIMAL: the Illinois replacement */
        return orc_get_fast_minimal() ? orc_e_solve5(x1, y1, x2, y2, E90) : orc_e_solve5_ref(x1, y1, x2, y2, E90);
    }
    return ORC_NO_SAMPLE;
}

int orc_e_count(const double* pts4, int N, const double* E, float thr2, int kind, uint8_t* mask) {
    int n = 0;
    for (int i = 0; i < N; ++i) {
        const double* p = pts4 + 4 * (size_t)i;
        int in = f_err_orc(kind, E, p[0], p[1], p[2], p[3]) <= thr2;
        if (mask) mask[i] = (uint8_t)in;
        n += in;
    }
    return n;
}

/* counts[10 h + s]: inliers of model s of hypothesis hypBegin + h; -1 no model; slot 0 = -2 no sample */
void orc_e_counts(const double* pts4, int N, uint64_t seed, int64_t hypBegin, int64_t hypCount, float thr2, int kind,
                  int* counts, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 2)
#endif
    for (int64_t h = 0; h < hypCount; ++h) {
        double E[EMAX * 9];
        int n = orc_e_hypothesis(pts4, N, seed, hypBegin + h, E, NULL);
        int* c = counts + EMAX * h;
        for (int s = 0; s < EMAX; ++s) c[s] = ORC_NO_MODEL;
        if (n == ORC_NO_SAMPLE) { c[0] = ORC_NO_SAMPLE; continue; }
        for (int s = 0; s < n; ++s) c[s] = orc_e_count(pts4, N, E + 9 * s, thr2, kind, NULL);
    }
}

/* RANSACPointSetRegistrator::run over per-slot counts: models tried in slot order, niters
 * checked per hypothesis. Returns the best slot index or -1. */
int64_t orc_ransac_replay_slots(const int* counts, int64_t nhyp, int slots, int N, int m, double conf, int maxIters,
                                int fixed, int* bestCount) {
    int64_t niters = maxIters > 1 ? maxIters : 1, best = -1;
    int bc = 0;
    for (int64_t it = 0; it < niters && it < nhyp; ++it) {
        const int* c = counts + it * slots;
        if (c[0] == ORC_NO_SAMPLE) break;
        for (int s = 0; s < slots; ++s) {
            if (c[s] < 0) continue;
            if (c[s] > (bc > m - 1 ? bc : m - 1)) {
                bc = c[s];
                best = it * slots + s;
                if (!fixed) niters = orc_update_num_iters(conf, (double)(N - c[s]) / N, m, (int)niters);
            }
        }
    }
    if (bestCount) *bestCount = bc;
    return best;
}

/* findEssentialMat(p1, p2, focal, pp, RANSAC, conf, thr, mask) with maxIters / seed / flags.
 * Returns the inlier count (0 on failure); *nmodels = number of models of the N == 5 solve. */
int orc_find_essential(const double* a, const double* b, int N, double focal, double ppx, double ppy, double thr,
                       double conf, int maxIters, uint64_t seed, int flags, double* E, uint8_t* mask,
                       int64_t* bestSlotOut, int nthreads) {
    if (bestSlotOut) *bestSlotOut = -1;
    if (N < 5) return 0;
    double* pts = (double*)malloc(sizeof(double) * 4 * (size_t)N);
    for (int i = 0; i < N; ++i) {
        pts[4 * i] = (a[2 * i] - ppx) / focal; pts[4 * i + 1] = (a[2 * i + 1] - ppy) / focal;
        pts[4 * i + 2] = (b[2 * i] - ppx) / focal; pts[4 * i + 3] = (b[2 * i + 1] - ppy) / focal;
    }
    double t = thr / ((focal + focal) / 2);
    float thr2 = (float)(t * t);
    int kind = (flags & ORC_FLAG_FUSED_ERROR) ? 0 : 1, result = 0;
    if (N == 5) {
        double x1[5], y1[5], x2[5], y2[5], Es[EMAX * 9];
        for (int i = 0; i < 5; ++i) { x1[i] = pts[4 * i]; y1[i] = pts[4 * i + 1]; x2[i] = pts[4 * i + 2]; y2[i] = pts[4 * i + 3]; }
        int n = orc_e_solve5_ref(x1, y1, x2, y2, Es);   /* count == modelPoints: runKernel once */
        if (n == 1) {
            memcpy(E, Es, sizeof(double) * 9);
            if (mask) memset(mask, 1, 5);
            result = 5;
        }
        free(pts);
        return result;
    }
    int64_t niters = maxIters > 1 ? maxIters : 1;
    int* cnt = (int*)malloc(sizeof(int) * EMAX * (size_t)niters);
    int* cvt = orc_cv_begin(flags, 0, NULL, N, 5, niters);
    const int fast0 = orc_get_fast_minimal();
    if (flags & ORC_FLAG_FAST_MINIMAL) orc_set_fast_minimal(1);
    orc_e_counts(pts, N, seed, 0, niters, thr2, kind, cnt, nthreads);
    int bc = 0;
    int64_t best = orc_ransac_replay_slots(cnt, niters, EMAX, N, 5, conf, maxIters, (flags & ORC_FLAG_FIXED_ITERS) != 0, &bc);
    free(cnt);
    if (best >= 0) {
        double Es[EMAX * 9];
        int n = orc_e_hypothesis(pts, N, seed, best / EMAX, Es, NULL);
        if (n > best % EMAX) {
            memcpy(E, Es + 9 * (best % EMAX), sizeof(double) * 9);
            result = orc_e_count(pts, N, E, thr2, kind, mask);
            if (bestSlotOut) *bestSlotOut = best;
        }
    }
    orc_cv_end(cvt);
    orc_set_fast_minimal(fast0);
    free(pts);
    return result;
}

/* ---- pose ------------------------------------------------------------------------------- */
static void cross3(const double* a, const double* b, double* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* decomposeEssentialMat with V from the eigenvectors of E^T E (see hyp_essential.h e_decompose). */
void orc_e_decompose(const double* E, double* R1, double* R2, double* t) {
    double M[9], V[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[3 * i + j] = E[i] * E[j] + E[3 + i] * E[3 + j] + E[6 + i] * E[6 + j];
    jacobi3_orc(M, V);
    double d[3] = {M[0], M[4], M[8]};
    int i0 = 0;
    if (d[1] > d[i0]) i0 = 1;
    if (d[2] > d[i0]) i0 = 2;
    int i1 = -1;
    for (int k = 0; k < 3; ++k)
        if (k != i0 && (i1 < 0 || d[k] > d[i1])) i1 = k;
    double v0[3], v1[3], v2[3], u0[3], u1[3], u2[3], n0 = 0, n1 = 0;
    for (int k = 0; k < 3; ++k) { v0[k] = V[3 * k + i0]; v1[k] = V[3 * k + i1]; }
    cross3(v0, v1, v2);
    for (int k = 0; k < 3; ++k) {
        u0[k] = E[3 * k] * v0[0] + E[3 * k + 1] * v0[1] + E[3 * k + 2] * v0[2];
        u1[k] = E[3 * k] * v1[0] + E[3 * k + 1] * v1[1] + E[3 * k + 2] * v1[2];
        n0 = n0 + u0[k] * u0[k];
        n1 = n1 + u1[k] * u1[k];
    }
    n0 = sqrt(n0); n1 = sqrt(n1);
    for (int k = 0; k < 3; ++k) { u0[k] = u0[k] / n0; u1[k] = u1[k] / n1; }
    cross3(u0, u1, u2);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            R1[3 * i + j] = u0[i] * v1[j] - u1[i] * v0[j] + u2[i] * v2[j];
            R2[3 * i + j] = u1[i] * v0[j] - u0[i] * v1[j] + u2[i] * v2[j];
        }
    memcpy(t, u2, sizeof(u2));
}

static void jacobi4(double* A, double* V) {
    for (int i = 0; i < 16; ++i) V[i] = (i % 5 == 0) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 30; ++sweep) {
        double off = 0, dg = 0;
        for (int p = 0; p < 4; ++p) {
            dg = dg + A[5 * p] * A[5 * p];
            for (int q = p + 1; q < 4; ++q) off = off + A[4 * p + q] * A[4 * p + q];
        }
        if (!(off > dg * 1e-32)) break;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 4; ++q) {
                double apq = A[4 * p + q];
                if (apq == 0) continue;
                double th = (A[5 * q] - A[5 * p]) / (2 * apq);
                double tt = (th >= 0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
                for (int k = 0; k < 4; ++k) {
                    double x = A[4 * k + p], y = A[4 * k + q];
                    A[4 * k + p] = c * x - s * y; A[4 * k + q] = s * x + c * y;
                }
                for (int k = 0; k < 4; ++k) {
                    double x = A[4 * p + k], y = A[4 * q + k];
                    A[4 * p + k] = c * x - s * y; A[4 * q + k] = s * x + c * y;
                }
                for (int k = 0; k < 4; ++k) {
                    double x = V[4 * k + p], y = V[4 * k + q];
                    V[4 * k + p] = c * x - s * y; V[4 * k + q] = s * x + c * y;
                }
            }
    }
}

/* triangulatePoints (DLT null vector) + recoverPose's cheirality test, P = {R (9), t (3)} */
static int cheiral(const double* P, double x1, double y1, double x2, double y2, double dist) {
    double A[4][4] = {{-1.0, 0.0, x1, 0.0}, {0.0, -1.0, y1, 0.0}};
    double r0[4] = {P[0], P[1], P[2], P[9]}, r1[4] = {P[3], P[4], P[5], P[10]}, r2[4] = {P[6], P[7], P[8], P[11]};
    for (int k = 0; k < 4; ++k) { A[2][k] = x2 * r2[k] - r0[k]; A[3][k] = y2 * r2[k] - r1[k]; }
    double M[16], V[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) M[4 * i + j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
    jacobi4(M, V);
    int m = 0;
    for (int k = 1; k < 4; ++k)
        if (M[5 * k] < M[5 * m]) m = k;
    double Q0 = V[m], Q1 = V[4 + m], Q2 = V[8 + m], Q3 = V[12 + m];
    if (!(Q2 * Q3 > 0)) return 0;
    double X = Q0 / Q3, Y = Q1 / Q3, Z = Q2 / Q3;
    if (!(Z < dist)) return 0;
    double z2 = r2[0] * X + r2[1] * Y + r2[2] * Z + r2[3];
    return z2 > 0 && z2 < dist;
}

/* recoverPose(E, p1, p2, R, t, focal, pp, mask): returns the chosen candidate's count; good4 out. */
int orc_recover_pose(const double* a, const double* b, int N, double focal, double ppx, double ppy, const double* E,
                     const uint8_t* mask, double* R, double* t, int* good4) {
    double R1[9], R2[9], t0[3], P[4][12];
    orc_e_decompose(E, R1, R2, t0);
    for (int k = 0; k < 4; ++k) {
        memcpy(P[k], (k & 1) ? R2 : R1, sizeof(R1));
        for (int j = 0; j < 3; ++j) P[k][9 + j] = k < 2 ? t0[j] : -t0[j];
    }
    int g[4] = {0, 0, 0, 0};
    for (int i = 0; i < N; ++i) {
        if (mask && !mask[i]) continue;
        double x1 = (a[2 * i] - ppx) / focal, y1 = (a[2 * i + 1] - ppy) / focal;
        double x2 = (b[2 * i] - ppx) / focal, y2 = (b[2 * i + 1] - ppy) / focal;
        for (int k = 0; k < 4; ++k) g[k] += cheiral(P[k], x1, y1, x2, y2, 50.0);
    }
    int pick = 3;
    if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3]) pick = 0;
    else if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3]) pick = 1;
    else if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3]) pick = 2;
    memcpy(R, P[pick], sizeof(double) * 9);
    memcpy(t, P[pick] + 9, sizeof(double) * 3);
    if (good4) memcpy(good4, g, sizeof(g));
    return g[pick];
}
