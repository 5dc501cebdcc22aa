// hyp_essential.h — per-hypothesis code of the essential-matrix RANSAC path:
// the opt-in replacement five-point solver (MCV_FLAG_FAST_MINIMAL; the default is the reference's own,
// five_point_ref.h), the pose decomposition and the two-view cheirality test.
// Compiled for gfx950 (ransac_e.hip) and for the host (mcvHostEssential test hook) with
// -ffp-contract=off, so both sides round every operation identically (fp64 +,-,*,/ and sqrt are
// IEEE correctly rounded on both; comparisons and integer bisection are exact).
//
// Reference behaviour restated (fivepoint.cpp:233-339, runFivepoint; OpenCV 4.x
// EMEstimatorCallback [ext]): Q (n x 9) rows (x1 x2, y1 x2, x2, x1 y2, y1 y2, y2, x1, y1, 1) of
// x2^T E x1 = 0; a 4-D null-space basis E = x X + y Y + z Z + W; the ten cubic constraints
// det(E) = 0 and 2 E E^T E - tr(E E^T) E = 0 over the 20 monomials
//   [x^3, y^3, x^2y, xy^2, x^2z, x^2, y^2z, y^2, xyz, xy | xz^2, xz, x, yz^2, yz, y, z^3, z^2, z, 1]
// (fivepoint.cpp getCoeffMat's column order); eliminate the first 10 columns; rows 4..9 pair up
// into the 3 x 13 matrix B(z) (fivepoint.cpp:279-296), whose determinant is a degree-10
// polynomial in z (fivepoint.cpp:299-309); each real root gives (x, y) from the null vector of
// B(z) and one E, normalised to unit Frobenius norm (fivepoint.cpp:314-335).
// Deterministic replacements: the null space by Gauss-Jordan with full pivoting
// + modified Gram-Schmidt (not SVD); the coefficient matrix by generic polynomial products (not
// the expanded getCoeffMat formulas); the elimination by Gauss-Jordan with partial pivoting (not
// Mat::inv); the real roots by derivative-interval (Rolle) bracketing and Illinois regula falsi
// to a 1-ulp bracket, safeguarded by bisection over the ordered bit patterns of doubles (not
// solvePoly's complex iteration; tangent double roots are not reported); the null
// vector of B(z) by the largest of the three row cross products (not SVD::solveZ).
#pragma once

#include "mcv_common.h"
#include "hyp_fundamental.h"   // jacobi3

namespace mcv {

static const int kEMaxModels = 10;

struct EModel { double e[9]; };   // row-major E, x2^T E x1 = 0 (normalised camera coordinates)

// ---- ordered bit patterns of doubles (bisection in at most 64 halvings) -------------------
MCV_HD int64_t e_dkey(double x) {
    const int64_t i = __builtin_bit_cast(int64_t, x);
    return i >= 0 ? i : (int64_t)(0x8000000000000000ull - (uint64_t)i);
}
MCV_HD double e_dval(int64_t k) {
    const int64_t i = k >= 0 ? k : (int64_t)(0x8000000000000000ull - (uint64_t)k);
    return __builtin_bit_cast(double, i);
}

// Falling factorials m! / (m - j)! for m, j <= 10 (exact in fp64): coefficient scale of the
// j-th derivative.
MCV_HD double e_falling(int m, int j) {
    double r = 1.0;
    for (int k = 0; k < j; ++k) r = r * (double)(m - k);
    return r;
}

// Horner on ascending coefficients q[0..d].
MCV_HD double e_poly_eval(const double* q, int d, double x) {
    double f = q[d];
    for (int k = d - 1; k >= 0; --k) f = f * x + q[k];
    return f;
}

// Root of q (degree d) in (lo, hi) given opposite signs flo = q(lo), fhi = q(hi), to adjacent
// doubles: Illinois regula falsi (the retained end's value is halved when it is kept twice), a
// bisection step on the ordered bit patterns whenever the point falls outside the bracket or the
// bracket failed to halve (in bit-pattern distance) twice in a row. Returns an exact zero if hit,
// else the lower end of the final 1-ulp bracket.
// Eval is any callable returning q(x) with exactly e_poly_eval's rounding (the wave solver passes
// a fixed-length Horner over zero-padded coefficients, which rounds identically).
template <class Eval>
MCV_HD double e_root_bracketed_f(const Eval& eval, double lo, double hi, double flo, double fhi) {
    int side = 0, stall = 0;
    for (int it = 0; it < 256; ++it) {
        const int64_t klo = e_dkey(lo), khi = e_dkey(hi);
        const int64_t kmid = (klo >> 1) + (khi >> 1) + (klo & khi & 1);
        if (kmid == klo || kmid == khi) break;
        double m;
        if (stall >= 2) {
            m = e_dval(kmid);
            stall = 0;
        } else {
            m = lo - flo * ((hi - lo) / (fhi - flo));
            if (!(m > lo && m < hi)) m = e_dval(kmid);
        }
        const double fm = eval(m);
        if (fm == 0) return m;
        const uint64_t w0 = (uint64_t)khi - (uint64_t)klo;
        const int64_t km = e_dkey(m);
        uint64_t w1;
        if ((fm < 0) == (flo < 0)) {
            w1 = (uint64_t)khi - (uint64_t)km;
            lo = m;
            flo = fm;
            if (side == -1) fhi = fhi * 0.5;
            side = -1;
        } else {
            w1 = (uint64_t)km - (uint64_t)klo;
            hi = m;
            fhi = fm;
            if (side == 1) flo = flo * 0.5;
            side = 1;
        }
        stall = (w1 > w0 / 2) ? stall + 1 : 0;
    }
    return lo;
}

MCV_HD double e_root_bracketed(const double* q, int d, double lo, double hi, double flo, double fhi) {
    return e_root_bracketed_f([q, d](double x) { return e_poly_eval(q, d, x); }, lo, hi, flo, fhi);
}

// Real roots (ascending) of sum_k cin[k] z^k, degree <= 10. The real roots of p^(j) are separated
// by those of p^(j+1) (Rolle), all inside the Cauchy bound R of p (Gauss-Lucas); walk j = n-1..0,
// with p^(j)'s coefficients c[k + j] (k + j)! / k! formed once per level.
MCV_HD int e_poly_real_roots(const double* cin, int deg, double* roots) {
    int n = deg;
    while (n > 0 && cin[n] == 0) --n;
    if (n < 1) return 0;
    double c[11];
    for (int k = 0; k <= n; ++k) c[k] = cin[k] / cin[n];
    double R = 0;
    for (int k = 0; k < n; ++k) {
        const double a = fabs(c[k]);
        R = a > R ? a : R;
    }
    R = 1.0 + R;
    if (!isfinite(R)) return 0;
    double rp[10], rc[10], q[11];
    int np = 0;
    for (int j = n - 1; j >= 0; --j) {
        const int d = n - j;
        for (int k = 0; k <= d; ++k) q[k] = c[k + j] * e_falling(k + j, j);
        int nc = 0;
        double a = -R;
        double fa = e_poly_eval(q, d, a);
        for (int s = 0; s <= np; ++s) {
            const double b = s < np ? rp[s] : R;
            const double fb = e_poly_eval(q, d, b);
            if (fb == 0) {
                if (nc == 0 || rc[nc - 1] != b) rc[nc++] = b;
            } else if (fa != 0 && ((fa < 0) != (fb < 0))) {
                rc[nc++] = e_root_bracketed(q, d, a, b, fa, fb);
            }
            a = b;
            fa = fb;
        }
        for (int k = 0; k < nc; ++k) rp[k] = rc[k];
        np = nc;
    }
    for (int k = 0; k < np; ++k) roots[k] = rp[k];
    return np;
}

// e_poly_real_roots for a fixed maximum degree NMAX with no dynamically indexed arrays (so the
// device keeps everything in registers; the AP3P quartic): levels and intervals unrolled, pushes
// into the root list as select chains, every level's Horner over coefficients zero-padded to
// degree NMAX — +0 * x + (+0) stays +0 and (+-0) + q[d] = q[d], so it rounds exactly like the
// degree-d loop. Bit-identical to e_poly_real_roots(cin, NMAX, roots).
template <int NMAX>
struct EPolyPad {
    double q[NMAX + 1];
    MCV_HD double operator()(double x) const {
        double f = q[NMAX];
        for (int k = NMAX - 1; k >= 0; --k) f = f * x + q[k];
        return f;
    }
};

template <int NMAX>
MCV_HD int e_poly_real_roots_fixed(const double (&cin)[NMAX + 1], double (&roots)[NMAX]) {
    int n = 0;
#pragma unroll
    for (int k = 1; k <= NMAX; ++k) n = cin[k] != 0 ? k : n;   // highest non-zero coefficient
    if (n < 1) return 0;
    double lead = cin[1];
#pragma unroll
    for (int k = 2; k <= NMAX; ++k) lead = n == k ? cin[k] : lead;
    double c[NMAX + 1];
#pragma unroll
    for (int k = 0; k <= NMAX; ++k) c[k] = k <= n ? cin[k] / lead : 0.0;
    double R = 0;
#pragma unroll
    for (int k = 0; k < NMAX; ++k) {
        const double a = fabs(c[k]);
        R = (k < n && a > R) ? a : R;
    }
    R = 1.0 + R;
    if (!isfinite(R)) return 0;
    double rp[NMAX], rc[NMAX];
#pragma unroll
    for (int k = 0; k < NMAX; ++k) rp[k] = rc[k] = 0.0;
    int np = 0;
#pragma unroll
    for (int j = NMAX - 1; j >= 0; --j) {
        if (j > n - 1) continue;
        const int d = n - j;
        EPolyPad<NMAX> P;
#pragma unroll
        for (int k = 0; k <= NMAX; ++k) P.q[k] = (k + j <= NMAX && k <= d) ? c[k + j <= NMAX ? k + j : 0] * e_falling(k + j, j) : 0.0;
        int nc = 0;
        double last = 0.0;
        auto push = [&](double v) {
#pragma unroll
            for (int t = 0; t < NMAX; ++t) rc[t] = t == nc ? v : rc[t];
            last = v;
            ++nc;
        };
        double a = -R;
        double fa = P(a);
#pragma unroll
        for (int s = 0; s < NMAX; ++s) {
            if (s > np) break;
            const double b = s < np ? rp[s] : R;
            const double fb = P(b);
            if (fb == 0) {
                if (nc == 0 || last != b) push(b);
            } else if (fa != 0 && ((fa < 0) != (fb < 0))) {
                push(e_root_bracketed_f(P, a, b, fa, fb));
            }
            a = b;
            fa = fb;
        }
#pragma unroll
        for (int t = 0; t < NMAX; ++t) rp[t] = rc[t];
        np = nc;
    }
#pragma unroll
    for (int t = 0; t < NMAX; ++t) roots[t] = rp[t];
    return np;
}

// ---- polynomial algebra in (x, y, z, w = 1) -------------------------------------------------
// Linear form: 4 coefficients (x, y, z, w). Quadratic: pairs (a <= b) in the order
// (0,0) (0,1) (0,2) (0,3) (1,1) (1,2) (1,3) (2,2) (2,3) (3,3). Cubic: 20 coefficients in the
// column order of the coefficient matrix (header comment).
MCV_HD int e_pair(int a, int b) {   // a <= b
    return a == 0 ? b : (a == 1 ? 3 + b : (a == 2 ? 5 + b : 9));
}
// sorted triple (a <= b <= c) -> cubic column
MCV_HD int e_triple(int a, int b, int c) {
    const int code = a * 16 + b * 4 + c;
    switch (code) {
        case 0 * 16 + 0 * 4 + 0: return 0;    // x^3
        case 1 * 16 + 1 * 4 + 1: return 1;    // y^3
        case 0 * 16 + 0 * 4 + 1: return 2;    // x^2 y
        case 0 * 16 + 1 * 4 + 1: return 3;    // x y^2
        case 0 * 16 + 0 * 4 + 2: return 4;    // x^2 z
        case 0 * 16 + 0 * 4 + 3: return 5;    // x^2
        case 1 * 16 + 1 * 4 + 2: return 6;    // y^2 z
        case 1 * 16 + 1 * 4 + 3: return 7;    // y^2
        case 0 * 16 + 1 * 4 + 2: return 8;    // x y z
        case 0 * 16 + 1 * 4 + 3: return 9;    // x y
        case 0 * 16 + 2 * 4 + 2: return 10;   // x z^2
        case 0 * 16 + 2 * 4 + 3: return 11;   // x z
        case 0 * 16 + 3 * 4 + 3: return 12;   // x
        case 1 * 16 + 2 * 4 + 2: return 13;   // y z^2
        case 1 * 16 + 2 * 4 + 3: return 14;   // y z
        case 1 * 16 + 3 * 4 + 3: return 15;   // y
        case 2 * 16 + 2 * 4 + 2: return 16;   // z^3
        case 2 * 16 + 2 * 4 + 3: return 17;   // z^2
        case 2 * 16 + 3 * 4 + 3: return 18;   // z
        default: return 19;                   // 1
    }
}

// q = l * m
MCV_HD void e_mul11(const double* l, const double* m, double* q) {
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b)
            q[e_pair(a, b)] = a == b ? l[a] * m[a] : l[a] * m[b] + l[b] * m[a];
}

// acc += q * l   (pairs in order, then l's variable 0..3)
MCV_HD void e_acc21(double* acc, const double* q, const double* l) {
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b) {
            const double qv = q[e_pair(a, b)];
            for (int c = 0; c < 4; ++c) {
                const int lo = c < a ? c : a;
                const int hi = c > b ? c : b;
                const int mid = c < a ? a : (c > b ? b : c);
                const int t = e_triple(lo, mid, hi);
                acc[t] = acc[t] + qv * l[c];
            }
        }
}

// ---- five-point solver ----------------------------------------------------------------------
// Orthonormal basis nb[4][9] of the null space of the 5 x 9 epipolar system. False if rank < 5.
MCV_HD bool e_null_basis(const double* x1, const double* y1, const double* x2, const double* y2, double (*nb)[9]) {
    double a[5][9];
    double scale = 0;
    for (int i = 0; i < 5; ++i) {
        a[i][0] = x1[i] * x2[i]; a[i][1] = y1[i] * x2[i]; a[i][2] = x2[i];
        a[i][3] = x1[i] * y2[i]; a[i][4] = y1[i] * y2[i]; a[i][5] = y2[i];
        a[i][6] = x1[i]; a[i][7] = y1[i]; a[i][8] = 1.0;
        for (int k = 0; k < 9; ++k) {
            const double v = fabs(a[i][k]);
            scale = v > scale ? v : scale;
        }
    }
    if (!(scale > 0) || !isfinite(scale)) return false;
    int perm[9];
    for (int k = 0; k < 9; ++k) perm[k] = k;
    for (int r = 0; r < 5; ++r) {
        double best = -1;
        int pr = r, pc = r;
        for (int i = r; i < 5; ++i)
            for (int j = r; j < 9; ++j) {
                const double v = fabs(a[i][perm[j]]);
                if (v > best) { best = v; pr = i; pc = j; }
            }
        if (!(best > 1e-12 * scale)) return false;
        for (int k = 0; k < 9; ++k) {
            const double t = a[r][k];
            a[r][k] = a[pr][k];
            a[pr][k] = t;
        }
        const int tp = perm[r]; perm[r] = perm[pc]; perm[pc] = tp;
        const double piv = a[r][perm[r]];
        for (int j = r + 1; j < 9; ++j) a[r][perm[j]] = a[r][perm[j]] / piv;
        a[r][perm[r]] = 1.0;
        for (int i = 0; i < 5; ++i) {
            if (i == r) continue;
            const double f = a[i][perm[r]];
            for (int j = r + 1; j < 9; ++j) a[i][perm[j]] = a[i][perm[j]] - f * a[r][perm[j]];
            a[i][perm[r]] = 0.0;
        }
    }
    for (int b = 0; b < 4; ++b) {
        double* v = nb[b];
        for (int k = 0; k < 9; ++k) v[k] = 0.0;
        v[perm[5 + b]] = 1.0;
        for (int r = 0; r < 5; ++r) v[perm[r]] = -a[r][perm[5 + b]];
        for (int c = 0; c < b; ++c) {   // modified Gram-Schmidt
            double d = 0;
            for (int k = 0; k < 9; ++k) d = d + nb[c][k] * v[k];
            for (int k = 0; k < 9; ++k) v[k] = v[k] - d * nb[c][k];
        }
        double s = 0;
        for (int k = 0; k < 9; ++k) s = s + v[k] * v[k];
        const double nrm = sqrt(s);
        if (!(nrm > 0)) return false;
        for (int k = 0; k < 9; ++k) v[k] = v[k] / nrm;
    }
    return true;
}

// The 10 x 20 cubic constraint matrix for E = x nb0 + y nb1 + z nb2 + nb3.
// Row 0: det(E); row 1 + 3i + j: (2 E E^T - tr(E E^T) I) E, entry (i, j).
MCV_HD void e_coeffs(const double (*nb)[9], double (*A)[20]) {
    double L[9][4];
    for (int k = 0; k < 9; ++k)
        for (int v = 0; v < 4; ++v) L[k][v] = nb[v][k];
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 20; ++c) A[r][c] = 0.0;
    // det = E00 (E11 E22 - E12 E21) + E01 (E12 E20 - E10 E22) + E02 (E10 E21 - E11 E20)
    {
        double p[10], q[10], m[10];
        const int cof[3][4] = {{4, 8, 5, 7}, {5, 6, 3, 8}, {3, 7, 4, 6}};
        for (int i = 0; i < 3; ++i) {
            e_mul11(L[cof[i][0]], L[cof[i][1]], p);
            e_mul11(L[cof[i][2]], L[cof[i][3]], q);
            for (int k = 0; k < 10; ++k) m[k] = p[k] - q[k];
            e_acc21(A[0], m, L[i]);
        }
    }
    // EEt (symmetric), trace, Lambda = 2 EEt - tr I
    double EEt[3][3][10];
    for (int i = 0; i < 3; ++i)
        for (int j = i; j < 3; ++j) {
            double p[10];
            e_mul11(L[3 * i + 0], L[3 * j + 0], EEt[i][j]);
            for (int k = 1; k < 3; ++k) {
                e_mul11(L[3 * i + k], L[3 * j + k], p);
                for (int t = 0; t < 10; ++t) EEt[i][j][t] = EEt[i][j][t] + p[t];
            }
        }
    double tr[10];
    for (int t = 0; t < 10; ++t) tr[t] = EEt[0][0][t] + EEt[1][1][t] + EEt[2][2][t];
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) {
            double lam[10];
            const double* s = i <= k ? EEt[i][k] : EEt[k][i];
            for (int t = 0; t < 10; ++t) lam[t] = 2.0 * s[t] - (i == k ? tr[t] : 0.0);
            for (int j = 0; j < 3; ++j) e_acc21(A[1 + 3 * i + j], lam, L[3 * k + j]);
        }
}

// Gauss-Jordan on columns 0..9 (partial pivoting); C[r][j] = reduced A[r][10 + j]. False if singular.
MCV_HD bool e_eliminate(double (*A)[20], double (*C)[10]) {
    double scale = 0;
    for (int r = 0; r < 10; ++r)
        for (int c = 0; c < 20; ++c) {
            const double v = fabs(A[r][c]);
            scale = v > scale ? v : scale;
        }
    if (!(scale > 0) || !isfinite(scale)) return false;
    for (int c = 0; c < 10; ++c) {
        int p = c;
        double best = fabs(A[c][c]);
        for (int r = c + 1; r < 10; ++r) {
            const double v = fabs(A[r][c]);
            if (v > best) { best = v; p = r; }
        }
        if (!(best > 1e-13 * scale)) return false;
        if (p != c)
            for (int k = c; k < 20; ++k) {
                const double t = A[c][k];
                A[c][k] = A[p][k];
                A[p][k] = t;
            }
        const double piv = A[c][c];
        for (int k = c + 1; k < 20; ++k) A[c][k] = A[c][k] / piv;
        for (int r = 0; r < 10; ++r) {
            if (r == c) continue;
            const double f = A[r][c];
            for (int k = c + 1; k < 20; ++k) A[r][k] = A[r][k] - f * A[c][k];
        }
    }
    for (int r = 0; r < 10; ++r)
        for (int j = 0; j < 10; ++j) C[r][j] = A[r][10 + j];
    return true;
}

// Ascending polynomial product r = a * b (r zeroed here).
MCV_HD void e_polymul(const double* a, int da, const double* b, int db, double* r) {
    for (int k = 0; k <= da + db; ++k) r[k] = 0.0;
    for (int i = 0; i <= da; ++i)
        for (int j = 0; j <= db; ++j) r[i + j] = r[i + j] + a[i] * b[j];
}

MCV_HD double e_horner(const double* c, int n, double z) {
    double f = c[n];
    for (int k = n - 1; k >= 0; --k) f = f * z + c[k];
    return f;
}

// B(z): per row i, polynomials in z (ascending): bx (deg 3), by (deg 3), bc (deg 4).
// Row = C[4+2i] - z * C[5+2i] over the tail monomials [xz^2, xz, x, yz^2, yz, y, z^3, z^2, z, 1];
// C points at C[0][0], rows `stride` doubles apart.
MCV_HD void e_bz(const double* C, int stride, double (*bx)[4], double (*by)[4], double (*bc)[5]) {
    for (int i = 0; i < 3; ++i) {
        const double* e = C + (4 + 2 * i) * stride;
        const double* f = C + (5 + 2 * i) * stride;
        bx[i][3] = 0.0 - f[0]; bx[i][2] = e[0] - f[1]; bx[i][1] = e[1] - f[2]; bx[i][0] = e[2] - 0.0;
        by[i][3] = 0.0 - f[3]; by[i][2] = e[3] - f[4]; by[i][1] = e[4] - f[5]; by[i][0] = e[5] - 0.0;
        bc[i][4] = 0.0 - f[6]; bc[i][3] = e[6] - f[7]; bc[i][2] = e[7] - f[8]; bc[i][1] = e[8] - f[9];
        bc[i][0] = e[9] - 0.0;
    }
}

// det B = bx0 (by1 bc2 - by2 bc1) - by0 (bx1 bc2 - bx2 bc1) + bc0 (bx1 by2 - bx2 by1)
MCV_HD void e_detpoly(const double (*bx)[4], const double (*by)[4], const double (*bc)[5], double* det) {
    double t1[8], t2[8], m7[8], p1[11], p2[11], q6[7], q6b[7], m6[7], p3[11];
    e_polymul(by[1], 3, bc[2], 4, t1);
    e_polymul(by[2], 3, bc[1], 4, t2);
    for (int k = 0; k < 8; ++k) m7[k] = t1[k] - t2[k];
    e_polymul(bx[0], 3, m7, 7, p1);
    e_polymul(bx[1], 3, bc[2], 4, t1);
    e_polymul(bx[2], 3, bc[1], 4, t2);
    for (int k = 0; k < 8; ++k) m7[k] = t1[k] - t2[k];
    e_polymul(by[0], 3, m7, 7, p2);
    e_polymul(bx[1], 3, by[2], 3, q6);
    e_polymul(bx[2], 3, by[1], 3, q6b);
    for (int k = 0; k < 7; ++k) m6[k] = q6[k] - q6b[k];
    e_polymul(bc[0], 4, m6, 6, p3);
    for (int k = 0; k < 11; ++k) det[k] = p1[k] - p2[k] + p3[k];
}

// Null vector of B(z) for one real root z (the largest of the row-pair cross products, first on
// ties) -> unit-norm E. False if the root gives no model.
MCV_HD bool e_model_at(const double (*bx)[4], const double (*by)[4], const double (*bc)[5], const double* nb0,
                       const double* nb1, const double* nb2, const double* nb3, double z, double* E) {
    double r[3][3];
    for (int i = 0; i < 3; ++i) {
        r[i][0] = e_horner(bx[i], 3, z);
        r[i][1] = e_horner(by[i], 3, z);
        r[i][2] = e_horner(bc[i], 4, z);
    }
    double v[3] = {0, 0, 0}, best = -1;
    const int pa[3] = {0, 0, 1}, pb[3] = {1, 2, 2};
    for (int q = 0; q < 3; ++q) {
        const double* u = r[pa[q]];
        const double* w = r[pb[q]];
        const double c0 = u[1] * w[2] - u[2] * w[1];
        const double c1 = u[2] * w[0] - u[0] * w[2];
        const double c2 = u[0] * w[1] - u[1] * w[0];
        const double n2 = c0 * c0 + c1 * c1 + c2 * c2;
        if (n2 > best) { best = n2; v[0] = c0; v[1] = c1; v[2] = c2; }
    }
    const double nv = sqrt(best);
    if (!(nv > 0) || !(fabs(v[2]) >= 1e-10 * nv)) return false;
    const double x = v[0] / v[2], y = v[1] / v[2];
    double e[9], ss = 0;
    for (int k = 0; k < 9; ++k) {
        e[k] = x * nb0[k] + y * nb1[k] + z * nb2[k] + nb3[k];
        ss = ss + e[k] * e[k];
    }
    const double ns = sqrt(ss);
    if (!(ns > 0) || !isfinite(ns)) return false;
    for (int k = 0; k < 9; ++k) E[k] = e[k] / ns;
    return true;
}

// Five-point solve on normalised coordinates: up to 10 unit-norm E (row-major) in E[10][9].
MCV_HD int e_solve5(const double* x1, const double* y1, const double* x2, const double* y2, double (*E)[9]) {
    double nb[4][9];
    if (!e_null_basis(x1, y1, x2, y2, nb)) return 0;
    double C[10][10];
    {
        double A[10][20];
        e_coeffs(nb, A);
        if (!e_eliminate(A, C)) return 0;
    }
    double bx[3][4], by[3][4], bc[3][5];
    e_bz(&C[0][0], 10, bx, by, bc);
    double det[11];
    e_detpoly(bx, by, bc, det);
    double roots[10];
    const int nr = e_poly_real_roots(det, 10, roots);
    int count = 0;
    for (int s = 0; s < nr; ++s)
        if (e_model_at(bx, by, bc, nb[0], nb[1], nb[2], nb[3], roots[s], E[count])) ++count;
    return count;
}

// The reference's own five-point solver (the default RANSAC path and the cvFivePoint export) lives in
// five_point_ref.h; e_solve5 above is the opt-in replacement (MCV_FLAG_FAST_MINIMAL).

// One hypothesis on packed double4 normalised correspondences {x1, y1, x2, y2}: 5 distinct
// indices from the Philox stream (no subset check: EMEstimatorCallback has none), five-point
// solve. Returns the number of models (0 = kStatusNoModel) or kStatusNoSample.
MCV_HD int e_hypothesis(const double* pts4, int N, const Sampler& smp, uint64_t hyp, double (*E)[9], int* idx_out) {
    SubsetSrc<5> src(smp, hyp);
    int idx[5];
    bool found = false;   // search and solve apart (h_hypothesis): one solve pass per wave
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, idx);
        if (got < 0) break;
        if (got == 0) continue;
        found = true;
        break;
    }
    if (!found) return kStatusNoSample;
    double x1[5], y1[5], x2[5], y2[5];
    for (int i = 0; i < 5; ++i) {
        const double* p = pts4 + 4 * (int64_t)idx[i];
        x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
    }
    if (idx_out) for (int i = 0; i < 5; ++i) idx_out[i] = idx[i];
    return e_solve5(x1, y1, x2, y2, E);
}

// ---- pose ----------------------------------------------------------------------------------
// decomposeEssentialMat (OpenCV 4.x [ext]): E = U diag(s, s, 0) V^T, R1 = U W V^T, R2 = U W^T V^T,
// t = U[:, 2], W = [[0,1,0],[-1,0,0],[0,0,1]], det U = det V = +1. Here V = eigenvectors of E^T E
// (jacobi3, two largest eigenvalues first, first maximum on ties), u_k = E v_k / |E v_k| (k = 0, 1),
// u2 = u0 x u1, v2 = v0 x v1 — so R1 = u0 v1^T - u1 v0^T + u2 v2^T, R2 = u1 v0^T - u0 v1^T + u2 v2^T.
MCV_HD void e_decompose(const double* E, double* R1, double* R2, double* t) {
    double M[9], V[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) M[3 * i + j] = E[i] * E[j] + E[3 + i] * E[3 + j] + E[6 + i] * E[6 + j];
    jacobi3(M, V);
    const double d[3] = {M[0], M[4], M[8]};
    int i0 = 0;
    for (int k = 1; k < 3; ++k)
        if (d[k] > d[i0]) i0 = k;
    int i1 = -1;
    for (int k = 0; k < 3; ++k)
        if (k != i0 && (i1 < 0 || d[k] > d[i1])) i1 = k;
    double v0[3], v1[3], v2[3], u0[3], u1[3], u2[3];
    for (int k = 0; k < 3; ++k) { v0[k] = V[3 * k + i0]; v1[k] = V[3 * k + i1]; }
    v2[0] = v0[1] * v1[2] - v0[2] * v1[1];
    v2[1] = v0[2] * v1[0] - v0[0] * v1[2];
    v2[2] = v0[0] * v1[1] - v0[1] * v1[0];
    double n0 = 0, n1 = 0;
    for (int k = 0; k < 3; ++k) {
        u0[k] = E[3 * k] * v0[0] + E[3 * k + 1] * v0[1] + E[3 * k + 2] * v0[2];
        u1[k] = E[3 * k] * v1[0] + E[3 * k + 1] * v1[1] + E[3 * k + 2] * v1[2];
        n0 = n0 + u0[k] * u0[k];
        n1 = n1 + u1[k] * u1[k];
    }
    n0 = sqrt(n0);
    n1 = sqrt(n1);
    for (int k = 0; k < 3; ++k) { u0[k] = u0[k] / n0; u1[k] = u1[k] / n1; }
    u2[0] = u0[1] * u1[2] - u0[2] * u1[1];
    u2[1] = u0[2] * u1[0] - u0[0] * u1[2];
    u2[2] = u0[0] * u1[1] - u0[1] * u1[0];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            R1[3 * i + j] = u0[i] * v1[j] - u1[i] * v0[j] + u2[i] * v2[j];
            R2[3 * i + j] = u1[i] * v0[j] - u0[i] * v1[j] + u2[i] * v2[j];
        }
    for (int k = 0; k < 3; ++k) t[k] = u2[k];
}

// Cyclic Jacobi on a symmetric 4x4 (row-major, destroyed); V columns = eigenvectors.
MCV_HD void e_jacobi4(double* A, double* V) {
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
                const double apq = A[4 * p + q];
                if (apq == 0) continue;
                const double theta = (A[5 * q] - A[5 * p]) / (2 * apq);
                const double tt = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(tt * tt + 1.0), s = tt * c;
                for (int k = 0; k < 4; ++k) {
                    const double akp = A[4 * k + p], akq = A[4 * k + q];
                    A[4 * k + p] = c * akp - s * akq;
                    A[4 * k + q] = s * akp + c * akq;
                }
                for (int k = 0; k < 4; ++k) {
                    const double apk = A[4 * p + k], aqk = A[4 * q + k];
                    A[4 * p + k] = c * apk - s * aqk;
                    A[4 * q + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < 4; ++k) {
                    const double vkp = V[4 * k + p], vkq = V[4 * k + q];
                    V[4 * k + p] = c * vkp - s * vkq;
                    V[4 * k + q] = s * vkp + c * vkq;
                }
            }
    }
}

// recoverPose's cheirality test of one correspondence against P1 = [I | 0], P2 = [R | t]
// (OpenCV 4.x recoverPose / triangulatePoints [ext]): the homogeneous DLT point Q (null vector of
// the 4x4 system; here the eigenvector of A^T A with the smallest eigenvalue), then
//   Q2 Q3 > 0,  Q2/Q3 < dist,  (P2 Q/Q3)_z > 0,  (P2 Q/Q3)_z < dist.
// P = {R row-major (9), t (3)}.
MCV_HD bool e_cheirality(const double* P, double x1, double y1, double x2, double y2, double dist) {
    double A[4][4];
    A[0][0] = -1.0; A[0][1] = 0.0; A[0][2] = x1; A[0][3] = 0.0;
    A[1][0] = 0.0; A[1][1] = -1.0; A[1][2] = y1; A[1][3] = 0.0;
    const double r0[4] = {P[0], P[1], P[2], P[9]};
    const double r1[4] = {P[3], P[4], P[5], P[10]};
    const double r2[4] = {P[6], P[7], P[8], P[11]};
    for (int k = 0; k < 4; ++k) {
        A[2][k] = x2 * r2[k] - r0[k];
        A[3][k] = y2 * r2[k] - r1[k];
    }
    double M[16], V[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) M[4 * i + j] = A[0][i] * A[0][j] + A[1][i] * A[1][j] + A[2][i] * A[2][j] + A[3][i] * A[3][j];
    e_jacobi4(M, V);
    int m = 0;
    for (int k = 1; k < 4; ++k)
        if (M[5 * k] < M[5 * m]) m = k;
    const double Q0 = V[m], Q1 = V[4 + m], Q2 = V[8 + m], Q3 = V[12 + m];
    if (!(Q2 * Q3 > 0)) return false;
    const double X = Q0 / Q3, Y = Q1 / Q3, Z = Q2 / Q3;
    if (!(Z < dist)) return false;
    const double z2 = r2[0] * X + r2[1] * Y + r2[2] * Z + r2[3];
    return z2 > 0 && z2 < dist;
}

}  // namespace mcv
