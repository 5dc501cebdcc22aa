// five_point_ref.h — the reference's own five-point solver (fivepoint.cpp:233-339, runFivepoint; the
// same arithmetic as OpenCV 4.x EMEstimatorCallback::runKernel [ext], which the reference's
// findEssentialMat calls at MiniCVNative.cpp:177,204), in pieces a GPU lane can run from registers.
// It is the default minimal solver of the essential-matrix RANSAC path and of the cvFivePoint export;
// compiled for gfx950 and for the host (mcvHostFivePointRef) with -ffp-contract=off.
//
// Operation order, step by step (oracle/oracle_e.c orc_e_solve5_ref restates the same):
//  * Q (5 x 9) rows (x1 x2, y1 x2, x2 * 1.0, x1 y2, y1 y2, y2 * 1.0, x1 * 1.0, y1 * 1.0, 1), then
//    SVD::compute(Q, FULL_UV) (:252): JacobiSVDImpl_ on Q's rows with the four null rows completed from
//    cv::RNG(0x12345678) (fpr_jsvd below, epnp.h's jacobi_svd with compile-time row indices); the null
//    basis EE^T = rows 5..8;
//  * getCoeffMat (:10-231): each of the 200 entries is its source expression evaluated term by term
//    (products left to right, the signed terms summed left to right) from fivepoint_terms.h — term data
//    generated from the reference's text by scripts/gen/gen_fivepoint_terms.py — then perm[20];
//  * A.colRange(0, 10).inv() * A.colRange(10, 20) (:260): OpenCV evaluates inv(X) * Y as
//    cv::solve(X, Y, DECOMP_LU) [ext: matop.cpp MatOp_Invert::matmul -> MatOp_Solve], i.e. LUImpl with the
//    ten right-hand sides (partial pivoting, first maximum, eps 100 DBL_EPSILON), no explicit inverse;
//  * B = row1 - row2 (:262-277) and the coefficients c[0..10] of det B(z) (:299-309) term by term;
//  * cv::solvePoly(c, roots) (:297): Durand-Kerner from (1 + i)^k, 300 in-place sweeps with OpenCV's
//    Complex arithmetic (a / b through t = 1 / |b|^2), stop when a whole sweep changes nothing;
//  * per root with |Im| <= 1e-10, in solvePoly's order: Bz (:318-323), SVD::solveZ(Bz) = the last row of
//    Vt of Bz's 3 x 3 JacobiSVD, skipped when |xy1[2]| < 1e-10; Evec = EE.col(0) x + EE.col(1) y
//    (addWeighted: + 0), + EE.col(2) z (scaleAdd), + EE.col(3) (add); Evec /= norm(Evec): normL2Sqr's
//    4-way unrolled sum, then convertTo by 1 / norm (+ 0).
// Degenerate samples only: a singular 10 x 10 block gives no model (cv::solve would return zeros and the
// reference then NaN / arbitrary models, which count no inliers either); a leading coefficient
// |c[10]| <= DBL_EPSILON repeats the last root where solvePoly copies uninitialised buffer entries.
#pragma once

#include "mcv_common.h"
#include "epnp.h"              // cv_hypot, kDblMin
#include "fivepoint_terms.h"
#include <utility>

namespace mcv {

// ---- term tables -> straight-line code ---------------------------------------------------------
// Every table index below is a template argument, so after inlining each factor is a register
// read (v is the caller's register array) and the 5748 + 480 terms are straight-line fp64 code.
template <int F>
MCV_HD double fpr_factor(const double* v) {
    constexpr int kind = F >> 6, i = F & 63;
    if constexpr (kind == 0) return kFpLiterals[i];
    else if constexpr (kind == 1) return v[i];
    else if constexpr (kind == 2) return v[i] * v[i];
    else return (v[i] * v[i]) * v[i];
}

template <bool C, int K>
MCV_HD double fpr_term(const double* v) {
    constexpr FpTerm t = C ? kFpCTerms[K] : kFpATerms[K];
    double p = fpr_factor<t.f[0]>(v);
    if constexpr (t.f[1] != 0xFF) p = p * fpr_factor<t.f[1]>(v);
    if constexpr (t.f[2] != 0xFF) p = p * fpr_factor<t.f[2]>(v);
    if constexpr (t.f[3] != 0xFF) p = p * fpr_factor<t.f[3]>(v);
    if constexpr (t.neg != 0) p = -p;
    return p;
}

template <bool C, int S, int... K>
MCV_HD double fpr_sum(const double* v, std::integer_sequence<int, K...>) {
    double acc = fpr_term<C, S>(v);
    ((acc = acc + fpr_term<C, S + 1 + K>(v)), ...);
    return acc;
}

template <bool C, int E>
MCV_HD double fpr_entry(const double* v) {
    constexpr int s = C ? kFpCStart[E] : kFpAStart[E];
    constexpr int n = (C ? kFpCStart[E + 1] : kFpAStart[E + 1]) - s;
    return fpr_sum<C, s>(v, std::make_integer_sequence<int, n - 1>{});
}

// Column of getCoeffMat's raw entry after the permutation AA[i + 20 j] = A[perm[i] + 20 j].
constexpr int fpr_final_col(int rawCol) {
    int i = 0;
    while (kFpPerm[i] != rawCol) ++i;
    return i;
}

// getCoeffMat(e, A): e = EE^T flattened (e[9 b + k] = null vector b, element k); st(row, col, value)
// receives the 200 entries of the permuted 10 x 20 matrix in the source's statement order.
template <class Store, int... E>
MCV_HD void fpr_coeff_matrix_impl(const double* e, Store& st, std::integer_sequence<int, E...>) {
    (st(E / 20, fpr_final_col(E % 20), fpr_entry<false, E>(e)), ...);
}
template <class Store>
MCV_HD void fpr_coeff_matrix(const double* e, Store& st) {
    fpr_coeff_matrix_impl(e, st, std::make_integer_sequence<int, 200>{});
}

// c[0..10] of det B(z) from b = B (3 x 13, row-major).
template <int... K>
MCV_HD void fpr_det_coeffs_impl(const double* b, double* c, std::integer_sequence<int, K...>) {
    ((c[K] = fpr_entry<true, K>(b)), ...);
}
MCV_HD void fpr_det_coeffs(const double* b, double* c) {
    fpr_det_coeffs_impl(b, c, std::make_integer_sequence<int, 11>{});
}

// ---- JacobiSVDImpl_<double> with compile-time row indices ------------------------------------
// epnp.h's jacobi_svd, the same operations in the same order; the selection sort swaps rows through
// per-candidate selects (no dynamically indexed row), so every array stays in registers.
template <int M, int N, int N1, bool VT>
MCV_HD void fpr_jsvd(double (&A)[N1][M], double (&Wo)[N], double (&Vt)[N][N]) {
    const double eps = kDblEpsilon * 10, minval = kDblMin;
    double W[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) sd += A[i][k] * A[i][k];
        W[i] = sd;
        if constexpr (VT) {
#pragma unroll
            for (int k = 0; k < N; ++k) Vt[i][k] = k == i ? 1.0 : 0.0;
        }
    }
    const int maxIter = M > 30 ? M : 30;
    for (int iter = 0; iter < maxIter; ++iter) {
        bool changed = false;
#pragma unroll
        for (int i = 0; i < N - 1; ++i)
#pragma unroll
            for (int j = i + 1; j < N; ++j) {
                double a = W[i], b = W[j], p = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) p += A[i][k] * A[j][k];
                if (__builtin_fabs(p) <= eps * __builtin_sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = cv_hypot(p, beta);
                double c, s;
                if (beta < 0) {
                    const double delta = (gamma - beta) * 0.5;
                    s = __builtin_sqrt(delta / gamma);
                    c = p / (gamma * s * 2);
                } else {
                    c = __builtin_sqrt((gamma + beta) / (gamma * 2));
                    s = p / (gamma * c * 2);
                }
                a = b = 0;
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    const double t0 = c * A[i][k] + s * A[j][k];
                    const double t1 = -s * A[i][k] + c * A[j][k];
                    A[i][k] = t0;
                    A[j][k] = t1;
                    a += t0 * t0;
                    b += t1 * t1;
                }
                W[i] = a;
                W[j] = b;
                changed = true;
                if constexpr (VT) {
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double t0 = c * Vt[i][k] + s * Vt[j][k];
                        const double t1 = -s * Vt[i][k] + c * Vt[j][k];
                        Vt[i][k] = t0;
                        Vt[j][k] = t1;
                    }
                }
            }
        if (!changed) break;
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double sd = 0;
#pragma unroll
        for (int k = 0; k < M; ++k) sd += A[i][k] * A[i][k];
        W[i] = __builtin_sqrt(sd);
    }
#pragma unroll
    for (int i = 0; i < N - 1; ++i) {
        int j = i;
        double wj = W[i];
#pragma unroll
        for (int k = i + 1; k < N; ++k)
            if (wj < W[k]) { j = k; wj = W[k]; }
#pragma unroll
        for (int k = i + 1; k < N; ++k) {
            if (k != j) continue;
            const double tw = W[i]; W[i] = W[k]; W[k] = tw;
#pragma unroll
            for (int q = 0; q < M; ++q) { const double t = A[i][q]; A[i][q] = A[k][q]; A[k][q] = t; }
            if constexpr (VT) {
#pragma unroll
                for (int q = 0; q < N; ++q) { const double t = Vt[i][q]; Vt[i][q] = Vt[k][q]; Vt[k][q] = t; }
            }
        }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) Wo[i] = W[i];
    CvRng rng{0x12345678u};
#pragma unroll
    for (int i = 0; i < N1; ++i) {
        double sd = i < N ? W[i < N ? i : 0] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ++ii) {
            // null singular value: random +-1/M vector orthogonalised against the previous rows
            const double val0 = 1. / M;
#pragma unroll
            for (int k = 0; k < M; ++k) A[i][k] = (rng.next() & 256) != 0 ? val0 : -val0;
#pragma unroll
            for (int it = 0; it < 2; ++it)
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    sd = 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) sd += A[i][k] * A[j][k];
                    double asum = 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) {
                        const double t = A[i][k] - sd * A[j][k];
                        A[i][k] = t;
                        asum += __builtin_fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
#pragma unroll
                    for (int k = 0; k < M; ++k) A[i][k] *= asum;
                }
            sd = 0;
#pragma unroll
            for (int k = 0; k < M; ++k) sd += A[i][k] * A[i][k];
            sd = __builtin_sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
#pragma unroll
        for (int k = 0; k < M; ++k) A[i][k] *= s;
    }
}

// Null basis e[36] (EE^T rows) of the 5 x 9 system of one sample (fivepoint.cpp:238-254).
MCV_HD void fpr_null_basis(const double* x1, const double* y1, const double* x2, const double* y2, double (&e)[36]) {
    double U[9][9], w[5], vt_unused[5][5];
#pragma unroll
    for (int i = 0; i < 9; ++i)
#pragma unroll
        for (int k = 0; k < 9; ++k) U[i][k] = 0.0;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        U[i][0] = x1[i] * x2[i]; U[i][1] = y1[i] * x2[i]; U[i][2] = x2[i] * 1.0;
        U[i][3] = x1[i] * y2[i]; U[i][4] = y1[i] * y2[i]; U[i][5] = y2[i] * 1.0;
        U[i][6] = x1[i] * 1.0; U[i][7] = y1[i] * 1.0; U[i][8] = 1.0;
    }
    fpr_jsvd<9, 5, 9, false>(U, w, vt_unused);
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int k = 0; k < 9; ++k) e[9 * b + k] = U[5 + b][k];
}

// cv::solve(A(:, 0:10), A(:, 10:20), DECOMP_LU) in place on a 10 x 20 register matrix: LUImpl with the
// right-hand sides in columns 10..19 (eps 100 DBL_EPSILON). Row swaps run as per-candidate selects.
// Afterwards columns 10..19 hold the solution. False when a pivot is below eps.
MCV_HD bool fpr_lu_solve(double (&A)[10][20]) {
    const double eps = kDblEpsilon * 100;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        int k = i;
        double ak = __builtin_fabs(A[i][i]);
#pragma unroll
        for (int j = i + 1; j < 10; ++j)
            if (__builtin_fabs(A[j][i]) > ak) { k = j; ak = __builtin_fabs(A[j][i]); }
        if (ak < eps) return false;
#pragma unroll
        for (int r = i + 1; r < 10; ++r) {
            if (r != k) continue;
#pragma unroll
            for (int j = i; j < 20; ++j) { const double t = A[i][j]; A[i][j] = A[r][j]; A[r][j] = t; }
        }
        const double d = -1 / A[i][i];
#pragma unroll
        for (int j = i + 1; j < 10; ++j) {
            const double alpha = A[j][i] * d;
#pragma unroll
            for (int q = i + 1; q < 20; ++q) A[j][q] += alpha * A[i][q];
        }
        A[i][i] = -d;
    }
#pragma unroll
    for (int i = 9; i >= 0; --i)
#pragma unroll
        for (int j = 10; j < 20; ++j) {
            double s = A[i][j];
#pragma unroll
            for (int q = i + 1; q < 10; ++q) s -= A[i][q] * A[q][j];
            A[i][j] = s * A[i][i];
        }
    return true;
}

// B (3 x 13, fivepoint.cpp's b[39]) from the solved block (columns 10..19 of the LU matrix).
MCV_HD void fpr_b_matrix(const double (&A)[10][20], double (&b)[39]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double* r1 = &A[2 * i + 4][10];
        const double* r2 = &A[2 * i + 5][10];
        double row1[13], row2[13];
#pragma unroll
        for (int k = 0; k < 13; ++k) row1[k] = row2[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            row1[1 + k] = r1[k] * 1.0; row1[5 + k] = r1[3 + k] * 1.0;
            row2[k] = r2[k] * 1.0; row2[4 + k] = r2[3 + k] * 1.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) { row1[9 + k] = r1[6 + k] * 1.0; row2[8 + k] = r2[6 + k] * 1.0; }
#pragma unroll
        for (int k = 0; k < 13; ++k) b[13 * i + k] = row1[k] - row2[k];
    }
}

struct FprCplx { double re, im; };

// One Durand-Kerner sweep body of cv::solvePoly for a polynomial of degree NN: roots updated in place
// in order; returns the largest |num|^2 of the sweep as std::max(maxDiff, abs(num)) forms it (a NaN
// never replaces it), so maxDiff <= 0 iff this is <= 0 (the square root is monotone, zero only at zero).
template <int NN>
MCV_HD double fpr_dk_sweep(const FprCplx (&cc)[11], FprCplx (&rr)[10]) {
    double md2 = 0;
#pragma unroll
    for (int i = 0; i < NN; ++i) {
        const FprCplx p = rr[i];
        FprCplx num = cc[NN], den = cc[NN];
#pragma unroll
        for (int j = 0; j < NN; ++j) {
            num = {num.re * p.re - num.im * p.im + cc[NN - j - 1].re, num.re * p.im + num.im * p.re + cc[NN - j - 1].im};
            if (j != i) {
                const FprCplx d = {p.re - rr[j].re, p.im - rr[j].im};
                den = {den.re * d.re - den.im * d.im, den.re * d.im + den.im * d.re};
            }
        }
        const double q = den.re * den.re + den.im * den.im;
        double t;
        if (div_f64_refined_domain(q)) t = div_f64_refined(1.0, q, rcp_f64_refined(q));   // = 1. / q
        else t = 1. / q;
        num = {(num.re * den.re + num.im * den.im) * t, (-num.re * den.im + num.im * den.re) * t};
        rr[i] = {p.re - num.re, p.im - num.im};
        const double a2 = num.re * num.re + num.im * num.im;
        md2 = md2 < a2 ? a2 : md2;
    }
    return md2;
}

#if defined(__HIP_DEVICE_COMPILE__)
// The same sweep with every 1. / q as the refined reciprocal and no branch: the whole sweep is one basic
// block, so the scheduler overlaps root i + 1's Horner evaluation (independent of this sweep's updates)
// with root i's dependent denominator / division chain. `bad` reports a q outside the refined domain; the
// caller then discards the sweep and reruns it with IEEE = true (the division's own branch-free expansion).
template <int NN, bool IEEE>
__device__ double fpr_dk_sweep_nb(const FprCplx (&cc)[11], FprCplx (&rr)[10], bool& bad) {
    double md2 = 0;
    // root i's numerator depends only on rr[i] as the sweep found it (no earlier step of the sweep
    // writes rr[i]): all ten Horner evaluations are formed first, as independent chains, and only the
    // denominators and updates run in the sweep's order
    FprCplx nums[NN];
#pragma unroll
    for (int i = 0; i < NN; ++i) {
        const FprCplx p = rr[i];
        FprCplx num = cc[NN];
#pragma unroll
        for (int j = 0; j < NN; ++j)
            num = {num.re * p.re - num.im * p.im + cc[NN - j - 1].re, num.re * p.im + num.im * p.re + cc[NN - j - 1].im};
        nums[i] = num;
    }
#pragma unroll
    for (int i = 0; i < NN; ++i) {
        const FprCplx p = rr[i];
        FprCplx num = nums[i], den = cc[NN];
#pragma unroll
        for (int j = 0; j < NN; ++j) {
            if (j != i) {
                const FprCplx d = {p.re - rr[j].re, p.im - rr[j].im};
                den = {den.re * d.re - den.im * d.im, den.re * d.im + den.im * d.re};
            }
        }
        const double q = den.re * den.re + den.im * den.im;
        bad |= !div_f64_refined_domain(q);
        const double t = IEEE ? 1. / q : div_f64_refined(1.0, q, rcp_f64_refined(q));
        num = {(num.re * den.re + num.im * den.im) * t, (-num.re * den.im + num.im * den.re) * t};
        rr[i] = {p.re - num.re, p.im - num.im};
        const double a2 = num.re * num.re + num.im * num.im;
        md2 = md2 < a2 ? a2 : md2;
    }
    return md2;
}
#endif

// cv::solvePoly(c (ascending, degree 10), roots, 300).
MCV_HD void fpr_solve_poly(const double (&c)[11], FprCplx (&roots)[10]) {
    FprCplx co[11];
#pragma unroll
    for (int i = 0; i <= 10; ++i) co[i] = {c[i], 0.0};
    int n = 10;
    for (; n > 1; --n)
        if (__builtin_fabs(c[n]) + 0.0 > kDblEpsilon) break;
    FprCplx p = {1, 0};
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        roots[i] = i < n ? p : FprCplx{0.0, 0.0};
        if (i < n) p = {p.re * 1.0 - p.im * 1.0, p.re * 1.0 + p.im * 1.0};
    }
    if (n == 10) {
        for (int iter = 0; iter < 300; ++iter) {
#if defined(__HIP_DEVICE_COMPILE__)
            FprCplx keep[10];
#pragma unroll
            for (int i = 0; i < 10; ++i) keep[i] = roots[i];
            bool bad = false;
            double md2 = fpr_dk_sweep_nb<10, false>(co, roots, bad);
            if (bad) {   // rare: redo the sweep with the IEEE divisions
#pragma unroll
                for (int i = 0; i < 10; ++i) roots[i] = keep[i];
                md2 = fpr_dk_sweep_nb<10, true>(co, roots, bad);
            }
            if (md2 <= 0) break;
#else
            if (fpr_dk_sweep<10>(co, roots) <= 0) break;
#endif
        }
        return;
    }
    // lower degree (a vanishing leading coefficient): the generic loop, rare. It works on its own copy
    // (dynamically indexed, so in scratch) and hands the roots back by constant indices: `roots` itself
    // is never indexed dynamically and stays in registers on the degree-10 path.
    FprCplx rr[10], cl[11];
#pragma unroll
    for (int i = 0; i < 10; ++i) rr[i] = roots[i];
#pragma unroll
    for (int i = 0; i <= 10; ++i) cl[i] = co[i];
    for (int iter = 0; iter < 300; ++iter) {
        double md2 = 0;
        for (int i = 0; i < n; ++i) {
            const FprCplx pp = rr[i];
            FprCplx num = cl[n], den = cl[n];
            for (int j = 0; j < n; ++j) {
                num = {num.re * pp.re - num.im * pp.im + cl[n - j - 1].re, num.re * pp.im + num.im * pp.re + cl[n - j - 1].im};
                if (j != i) {
                    const FprCplx d = {pp.re - rr[j].re, pp.im - rr[j].im};
                    den = {den.re * d.re - den.im * d.im, den.re * d.im + den.im * d.re};
                }
            }
            const double t = 1. / (den.re * den.re + den.im * den.im);
            num = {(num.re * den.re + num.im * den.im) * t, (-num.re * den.im + num.im * den.re) * t};
            rr[i] = {pp.re - num.re, pp.im - num.im};
            const double a2 = num.re * num.re + num.im * num.im;
            md2 = md2 < a2 ? a2 : md2;
        }
        if (md2 <= 0) break;
    }
    for (int k = n; k < 10; ++k) rr[k] = rr[k - 1];
#pragma unroll
    for (int i = 0; i < 10; ++i) roots[i] = rr[i];
}

// normL2Sqr<double, double>(a, 9) with CV_ENABLE_UNROLLED [ext: OpenCV core/base.hpp].
MCV_HD double fpr_norm_l2sqr9(const double (&a)[9]) {
    double s = 0;
    s += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
    s += a[4] * a[4] + a[5] * a[5] + a[6] * a[6] + a[7] * a[7];
    s += a[8] * a[8];
    return s;
}

// The model of one real root z (fivepoint.cpp:312-335): false when |xy1[2]| < 1e-10.
MCV_HD bool fpr_model(const double (&b)[39], const double* e, double z1, double (&E)[9]) {
    const double z2 = z1 * z1, z3 = z2 * z1, z4 = z3 * z1;
    double At[3][3], w[3], Vt[3][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double* br = b + 13 * j;
        At[0][j] = br[0] * z3 + br[1] * z2 + br[2] * z1 + br[3];
        At[1][j] = br[4] * z3 + br[5] * z2 + br[6] * z1 + br[7];
        At[2][j] = br[8] * z4 + br[9] * z3 + br[10] * z2 + br[11] * z1 + br[12];
    }
    fpr_jsvd<3, 3, 3, true>(At, w, Vt);
    const double* xy1 = Vt[2];
    if (__builtin_fabs(xy1[2]) < 1e-10) return false;
    const double x = xy1[0] / xy1[2], y = xy1[1] / xy1[2];
    double v[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = ((e[k] * x + e[9 + k] * y) + 0.0 + e[18 + k] * z1) + e[27 + k];
    const double sc = 1. / __builtin_sqrt(fpr_norm_l2sqr9(v));
#pragma unroll
    for (int k = 0; k < 9; ++k) E[k] = v[k] * sc + 0.0;
    return true;
}

// Register store of getCoeffMat's entries into a 10 x 20 matrix.
struct FprStoreA {
    double (&A)[10][20];
    MCV_HD void operator()(int r, int c, double v) { A[r][c] = v; }
};

// The whole solve on one lane (host twin, the cvFivePoint export): up to 10 unit-norm E, their count.
MCV_HD int fpr_solve5(const double* x1, const double* y1, const double* x2, const double* y2, double (*Eout)[9]) {
    double e[36];
    fpr_null_basis(x1, y1, x2, y2, e);
    double A[10][20];
    FprStoreA st{A};
    fpr_coeff_matrix(e, st);
    if (!fpr_lu_solve(A)) return 0;
    double b[39], c[11];
    fpr_b_matrix(A, b);
    fpr_det_coeffs(b, c);
    FprCplx roots[10];
    fpr_solve_poly(c, roots);
    int count = 0;
    for (int i = 0; i < 10; ++i) {
        if (__builtin_fabs(roots[i].im) > 1e-10) continue;
        double E[9];
        if (!fpr_model(b, e, roots[i].re, E)) continue;
        for (int k = 0; k < 9; ++k) Eout[count][k] = E[k];
        ++count;
    }
    return count;
}

}  // namespace mcv
