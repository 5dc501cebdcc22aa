// epnp.h — EPnP (Lepetit, Moreno-Noguer, Fua, IJCV 2009) as OpenCV 4.x's epnp.cpp computes it
// [ext: OpenCV calib3d, not vendored in /root/reference], for the solverKind 0/1/3/4 paths of
// cvSolvePnPRansac / cvSolvePnP (reference MiniCVNative.cpp:48-139; SOLVEPNP_DLS / UPNP fall back
// to EPnP in OpenCV 4.x). Compiled for gfx950 (one RANSAC hypothesis per lane, 5 points) and for
// the host (the O(1) dense algebra of the inlier solve) with -ffp-contract=off, so both sides
// round every operation identically; oracle/oracle_epnp.c restates the same algorithm in C.
//
// Restated pieces (operation order as written in the OpenCV sources):
//  * compute_pose: control points (centroid + PCA of the centred world points through cvSVD),
//    barycentric alphas (cvInvert DECOMP_SVD), M^T M (cvMulTransposed), its SVD, L_6x10 / rho,
//    betas of the three approximations (cvSolve DECOMP_SVD), 5 Gauss-Newton steps each
//    (epnp::qr_solve, Householder, including its pivot-scan that skips the last row), then
//    compute_R_and_t (ccs, pcs, solve_for_sign, estimate_R_and_t via the SVD of ABt) and the
//    mean reprojection error picking N = 1, 2 or 3 (first minimum).
//  * cv::SVD / cv::solve / cv::invert: JacobiSVDImpl_<double> (one-sided cyclic Jacobi on the
//    transposed matrix, eps = 10 DBL_EPSILON, at most max(m, 30) sweeps, descending selection
//    sort, cv::RNG(0x12345678) fill of null singular vectors) and SVBkSb (threshold 2 DBL_EPSILON
//    x sum w). The scalar loop order of the generic template is restated; x86 builds may run
//    some of those loops through SIMD helpers (VBLAS) with other partial-sum orders [ext].
//  * hypot is lapack.cpp's own template (cv_hypot below), not libm's.
// Large point sets (the inlier solve) sum per-point terms in blocks of kEpnpBlock consecutive
// points, each block sequentially from 0, the block sums sequentially: for n <= kEpnpBlock this
// is exactly the sequential order of the OpenCV loops.
#pragma once

#include "mcv_common.h"

namespace mcv {

static const double kDblMin = 2.2250738585072014e-308;
static const int kEpnpBlock = 1024;

// The hypot template of OpenCV's core lapack.cpp (the one JacobiSVDImpl_ calls — an unqualified
// hypot inside namespace cv): the larger magnitude times sqrt(1 + ratio^2). Only |.|, /, *, + and
// sqrt, so host and device round it identically.
MCV_HD double cv_hypot(double a, double b) {
    a = __builtin_fabs(a);
    b = __builtin_fabs(b);
    if (a > b) {
        b /= a;
        return a * __builtin_sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * __builtin_sqrt(1 + a * a);
    }
    return 0;
}

// JacobiSVDImpl_'s rotation: with p the doubled dot product and a, b the two rows' squared norms,
//   beta = a - b, gamma = hypot(p, beta) (cv_hypot), and for beta < 0: s = sqrt((gamma - beta) / 2 /
//   gamma), c = p / (gamma s 2); else c = sqrt((gamma + beta) / (gamma 2)), s = p / (gamma c 2).
// Device: when max(|p|, |beta|) is in [2^-63, 2^60] and min(|p|, |beta|) and |p| are 0 or >= 2^-900,
// every quotient takes gfx950's refined-reciprocal form and every sqrt the unscaled expansion
// (arguments in [0.5, 2]), both bit-identical to IEEE there (mcvTestDivF64 modes 0-5); a lane outside
// that domain takes the IEEE operations (a branch no lane takes on EPnP's systems, so the wave skips
// it). The dependent chain of a rotating pair shrinks from ~45 to ~30 fp64 operations. Host: IEEE.
MCV_HD void svd_rotation(double p, double a, double b, double& c, double& s) {
    const double beta = a - b;
#if defined(__HIP_DEVICE_COMPILE__)
    const double ap = __builtin_fabs(p), ab = __builtin_fabs(beta);
    const bool pg = ap > ab;
    const double hi = pg ? ap : ab, lo = pg ? ab : ap;
    if (__builtin_expect(hi <= 0x1p60 && hi >= 0x1p-63 && (lo == 0.0 || lo >= 0x1p-900) && ap >= 0x1p-900, 1)) {
        const double r1 = div_f64_refined(lo, hi, rcp_f64_refined(hi));
        const double gamma = hi * sqrt_f64_1to2(1 + r1 * r1);   // cv_hypot(p, beta): either branch
        if (beta < 0) {
            const double delta = (gamma - beta) * 0.5;
            s = sqrt_f64_1to2(div_f64_refined(delta, gamma, rcp_f64_refined(gamma)));
            const double d2 = gamma * s * 2;
            c = div_f64_refined(p, d2, rcp_f64_refined(d2));
        } else {
            const double g2 = gamma * 2;
            c = sqrt_f64_1to2(div_f64_refined(gamma + beta, g2, rcp_f64_refined(g2)));
            const double d2 = gamma * c * 2;
            s = div_f64_refined(p, d2, rcp_f64_refined(d2));
        }
        return;
    }
#endif
    const double gamma = cv_hypot(p, beta);
    if (beta < 0) {
        const double delta = (gamma - beta) * 0.5;
        s = __builtin_sqrt(delta / gamma);
        c = p / (gamma * s * 2);
    } else {
        c = __builtin_sqrt((gamma + beta) / (gamma * 2));
        s = p / (gamma * c * 2);
    }
}

// JacobiSVDImpl_<double>: A holds the N rows of length M of the TRANSPOSED input (At). On return
// A's rows are the left singular vectors (normalised), Wo the singular values (descending), and
// Vt (if non-null) the right singular vectors as rows. The A result does not depend on Vt.
// N1 > N (SVD::FULL_UV with more columns than rows): rows N .. N1-1 of A start at zero and are
// completed to an orthonormal basis by the cv::RNG branch.
// Device: the small decompositions (N <= 6: the 3 x 3 control-point / ABt SVDs, cv::solve's 6 x K)
// unroll their pair and element loops, so A, W and Vt stay in registers (rolled, their data-dependent
// row indices put them in scratch); the 12 x 12 keeps its rolled loops over the caller's LDS slice.
// Unrolling changes no operation or its order.
#if defined(__HIP_DEVICE_COMPILE__)
#define MCV_SVD_UNROLL _Pragma("unroll SU")
#define MCV_SMALL_UNROLL _Pragma("unroll")
#else
#define MCV_SVD_UNROLL
#define MCV_SMALL_UNROLL
#endif
template <int M, int N, int N1, bool HASV>
MCV_HD void jacobi_svd_core(double (&A)[N1][M], double (&Wo)[N], double (*Vt)[N]) {
    constexpr int SU = N <= 6 ? 16 : 1;
    const double eps = kDblEpsilon * 10, minval = kDblMin;
    double W[N];
    MCV_SVD_UNROLL
    for (int i = 0; i < N; ++i) {
        double sd = 0;
        MCV_SMALL_UNROLL
        for (int k = 0; k < M; ++k) sd += A[i][k] * A[i][k];
        W[i] = sd;
        if constexpr (HASV)
            MCV_SMALL_UNROLL
            for (int k = 0; k < N; ++k) Vt[i][k] = k == i ? 1.0 : 0.0;
    }
    {
        const int maxIter = M > 30 ? M : 30;
        for (int iter = 0; iter < maxIter; ++iter) {
            bool changed = false;
            MCV_SVD_UNROLL
            for (int i = 0; i < N - 1; ++i)
                MCV_SVD_UNROLL
                for (int j = i + 1; j < N; ++j) {
                    double a = W[i], b = W[j], p = 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < M; ++k) p += A[i][k] * A[j][k];
                    if (__builtin_fabs(p) <= eps * __builtin_sqrt(a * b)) continue;
                    p *= 2;
                    double c, s;
                    svd_rotation(p, a, b, c, s);
                    a = b = 0;
                    MCV_SMALL_UNROLL
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
                    if constexpr (HASV)
                        MCV_SMALL_UNROLL
                        for (int k = 0; k < N; ++k) {
                            const double t0 = c * Vt[i][k] + s * Vt[j][k];
                            const double t1 = -s * Vt[i][k] + c * Vt[j][k];
                            Vt[i][k] = t0;
                            Vt[j][k] = t1;
                        }
                }
            if (!changed) break;
        }
    }
    MCV_SVD_UNROLL
    for (int i = 0; i < N; ++i) {
        double sd = 0;
        MCV_SMALL_UNROLL
        for (int k = 0; k < M; ++k) sd += A[i][k] * A[i][k];
        W[i] = __builtin_sqrt(sd);
    }
    MCV_SVD_UNROLL
    for (int i = 0; i < N - 1; ++i) {
        int j = i;
        double wj = W[i];
        MCV_SMALL_UNROLL
        for (int k = i + 1; k < N; ++k)
            if (wj < W[k]) j = k, wj = W[k];
        // the swap with row j, as a compile-time row index per candidate (no dynamic indexing)
        MCV_SVD_UNROLL
        for (int jj = i + 1; jj < N; ++jj) {
            if (jj != j) continue;
            const double tw = W[i]; W[i] = W[jj]; W[jj] = tw;
            MCV_SMALL_UNROLL
            for (int k = 0; k < M; ++k) { const double t = A[i][k]; A[i][k] = A[jj][k]; A[jj][k] = t; }
            if constexpr (HASV)
                MCV_SMALL_UNROLL
                for (int k = 0; k < N; ++k) { const double t = Vt[i][k]; Vt[i][k] = Vt[jj][k]; Vt[jj][k] = t; }
        }
    }
    MCV_SVD_UNROLL
    for (int i = 0; i < N; ++i) Wo[i] = W[i];
    CvRng rng{0x12345678u};
    MCV_SVD_UNROLL
    for (int i = 0; i < N1; ++i) {
        double sd = i < N ? W[i] : 0;
        for (int ii = 0; ii < 100 && sd <= minval; ++ii) {
            // null singular value: random +-1/M vector orthogonalised against the previous rows
            const double val0 = 1. / M;
            MCV_SMALL_UNROLL
            for (int k = 0; k < M; ++k) A[i][k] = (rng.next() & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; ++it)
                MCV_SVD_UNROLL
                for (int j = 0; j < i; ++j) {
                    sd = 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < M; ++k) sd += A[i][k] * A[j][k];
                    double asum = 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < M; ++k) {
                        const double t = A[i][k] - sd * A[j][k];
                        A[i][k] = t;
                        asum += __builtin_fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < M; ++k) A[i][k] *= asum;
                }
            sd = 0;
            MCV_SMALL_UNROLL
            for (int k = 0; k < M; ++k) sd += A[i][k] * A[i][k];
            sd = __builtin_sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        MCV_SMALL_UNROLL
        for (int k = 0; k < M; ++k) A[i][k] *= s;
    }
}

// With Vt (rows: the right singular vectors) / without (a compile-time choice: a runtime null test of
// a private array's address kept that array out of registers on the GPU).
template <int M, int N, int N1 = N>
MCV_HD void jacobi_svd(double (&A)[N1][M], double (&Wo)[N], double (&Vt)[N][N]) {
    jacobi_svd_core<M, N, N1, true>(A, Wo, Vt);
}
template <int M, int N, int N1 = N>
MCV_HD void jacobi_svd(double (&A)[N1][M], double (&Wo)[N], decltype(nullptr)) {
    jacobi_svd_core<M, N, N1, false>(A, Wo, nullptr);
}

// SVBkSb for one right-hand side: x = sum_i [|w_i| > 2 eps sum w] (u_i . b / w_i) v_i, with
// u_i = U[i] (rows of the jacobi_svd A result) and v_i = Vt[i].
template <int M, int N>
MCV_HD void svd_backsubst(const double (&U)[N][M], const double (&w)[N], const double (&Vt)[N][N],
                          const double (&b)[M], double (&x)[N]) {
    double thr = 0;
    MCV_SMALL_UNROLL
    for (int i = 0; i < N; ++i) thr += w[i];
    thr *= kDblEpsilon * 2;
    MCV_SMALL_UNROLL
    for (int j = 0; j < N; ++j) x[j] = 0;
    MCV_SMALL_UNROLL
    for (int i = 0; i < N; ++i) {
        double wi = w[i];
        if (__builtin_fabs(wi) <= thr) continue;
        wi = 1 / wi;
        double s = 0;
        MCV_SMALL_UNROLL
        for (int j = 0; j < M; ++j) s += U[i][j] * b[j];
        s *= wi;
        MCV_SMALL_UNROLL
        for (int j = 0; j < N; ++j) x[j] = x[j] + s * Vt[i][j];
    }
}

// cv::invert(DECOMP_SVD) of a square matrix given its decomposition (SVBkSb with b = I).
template <int N>
MCV_HD void svd_pinv(const double (&U)[N][N], const double (&w)[N], const double (&Vt)[N][N], double (&X)[N][N]) {
    double thr = 0;
    MCV_SMALL_UNROLL
    for (int i = 0; i < N; ++i) thr += w[i];
    thr *= kDblEpsilon * 2;
    MCV_SMALL_UNROLL
    for (int r = 0; r < N; ++r)
        MCV_SMALL_UNROLL
        for (int c = 0; c < N; ++c) X[r][c] = 0;
    MCV_SMALL_UNROLL
    for (int i = 0; i < N; ++i) {
        double wi = w[i];
        if (__builtin_fabs(wi) <= thr) continue;
        wi = 1 / wi;
        double buf[N];
        MCV_SMALL_UNROLL
        for (int c = 0; c < N; ++c) buf[c] = U[i][c] * wi;
        MCV_SMALL_UNROLL
        for (int r = 0; r < N; ++r) {
            const double s = Vt[i][r];
            MCV_SMALL_UNROLL
            for (int c = 0; c < N; ++c) X[r][c] = X[r][c] + s * buf[c];
        }
    }
}

// cv::solve(L, rho, x, DECOMP_SVD) for a 6 x K system.
template <int K>
MCV_HD void svd_solve6(const double (&L)[6][K], const double (&rho)[6], double (&x)[K]) {
    double A[K][6], w[K], Vt[K][K];
    MCV_SMALL_UNROLL
    for (int i = 0; i < K; ++i)
        MCV_SMALL_UNROLL
        for (int r = 0; r < 6; ++r) A[i][r] = L[r][i];
    jacobi_svd<6, K>(A, w, Vt);
    svd_backsubst<6, K>(A, w, Vt, rho, x);
}

MCV_HD double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

struct EpnpCam { double fu, fv, uc, vc; };

// Control points and the inverse of their difference matrix (choose_control_points +
// compute_barycentric_coordinates' cvInvert).
struct EpnpCtrl {
    double cws[4][3];
    double ccinv[3][3];
};

// cws[0] = sum / n; PCA of the centred points: PW0^T PW0 (symmetric, full) -> cvSVD(U^T).
MCV_HD void epnp_control(const double (&sum)[3], const double (&pw0tpw0)[3][3], int n, EpnpCtrl& C) {
    for (int j = 0; j < 3; ++j) C.cws[0][j] = sum[j] / n;
    double A[3][3], dc[3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = pw0tpw0[j][i];
    jacobi_svd<3, 3>(A, dc, nullptr);   // A = U^T (uct)
    for (int i = 1; i < 4; ++i) {
        const double k = __builtin_sqrt(dc[i - 1] / n);
        for (int j = 0; j < 3; ++j) C.cws[i][j] = C.cws[0][j] + k * A[i - 1][j];
    }
    double B[3][3], w[3], Vt[3][3];
    for (int i = 0; i < 3; ++i)            // B = CC^T; CC[i][j - 1] = cws[j][i] - cws[0][i]
        for (int j = 1; j < 4; ++j) B[j - 1][i] = C.cws[j][i] - C.cws[0][i];
    jacobi_svd<3, 3>(B, w, Vt);
    svd_pinv<3>(B, w, Vt, C.ccinv);
}

MCV_HD void epnp_alphas(const EpnpCtrl& C, const double* p, double (&a)[4]) {
    for (int j = 0; j < 3; ++j)
        a[1 + j] = C.ccinv[j][0] * (p[0] - C.cws[0][0]) + C.ccinv[j][1] * (p[1] - C.cws[0][1]) +
                   C.ccinv[j][2] * (p[2] - C.cws[0][2]);
    a[0] = 1.0 - a[1] - a[2] - a[3];
}

// The two rows of M for one point (fill_M).
MCV_HD void epnp_m_rows(const double (&a)[4], double u, double v, const EpnpCam& c, double (&r1)[12],
                        double (&r2)[12]) {
    for (int i = 0; i < 4; ++i) {
        r1[3 * i] = a[i] * c.fu;
        r1[3 * i + 1] = 0.0;
        r1[3 * i + 2] = a[i] * (c.uc - u);
        r2[3 * i] = 0.0;
        r2[3 * i + 1] = a[i] * c.fv;
        r2[3 * i + 2] = a[i] * (c.vc - v);
    }
}

// Upper triangle of M^T M, row-major (a <= b): 78 sums.
static const int kMtmSums = 78;
MCV_HD int mtm_index(int a, int b) { return a * 12 - a * (a - 1) / 2 + (b - a); }

// The four null-space vectors (rows 11, 10, 9, 8 of U^T of M^T M) and everything that depends
// only on them and the control points: L_6x10, rho and the betas of the three approximations
// after Gauss-Newton.
struct EpnpBetas {
    double v[4][12];
    double betas[4][4];   // [N][.] for N = 1, 2, 3 (index 0 unused)
};

MCV_HD void epnp_qr_solve(double (&A)[6][4], double (&b)[6], double (&X)[4]) {
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    for (int k = 0; k < nc; ++k) {
        // epnp::qr_solve's pivot scan: |A[k][k]| twice, then rows k+1 .. nr-2 (never row nr-1)
        double eta = __builtin_fabs(A[k][k]);
        for (int i = k + 1; i < nr; ++i) {
            const double elt = __builtin_fabs(A[i - 1][k]);
            if (eta < elt) eta = elt;
        }
        if (eta == 0) return;   // A1[k] = A2[k] = 0 and X unchanged
        double sum2 = 0.0;
        const double inv_eta = 1. / eta;
        for (int i = k; i < nr; ++i) {
            A[i][k] *= inv_eta;
            sum2 += A[i][k] * A[i][k];
        }
        double sigma = __builtin_sqrt(sum2);
        if (A[k][k] < 0) sigma = -sigma;
        A[k][k] += sigma;
        A1[k] = sigma * A[k][k];
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; ++j) {
            double sum = 0;
            for (int i = k; i < nr; ++i) sum += A[i][k] * A[i][j];
            const double tau = sum / A1[k];
            for (int i = k; i < nr; ++i) A[i][j] -= tau * A[i][k];
        }
    }
    for (int j = 0; j < nc; ++j) {
        double tau = 0;
        for (int i = j; i < nr; ++i) tau += A[i][j] * b[i];
        tau /= A1[j];
        for (int i = j; i < nr; ++i) b[i] -= tau * A[i][j];
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; --i) {
        double sum = 0;
        for (int j = i + 1; j < nc; ++j) sum += A[i][j] * X[j];
        X[i] = (b[i] - sum) / A2[i];
    }
}

// Views of the 12 x 12 working matrix: ws(r, c). After the SVD and compute_L_6x10 its rows 0..5 hold
// L_6x10 (columns 0..9) and rho (column 10), rows 8..11 the null-space vectors. EpnpWsRef: a plain
// 12 x 12 array (host); EpnpWsSoA: element (r, c) of one hypothesis at p[(12 r + c) s] (structure of
// arrays over a launch's hypotheses: the split device generate's global scratch).
struct EpnpWsRef {
    double (&A)[12][12];
    MCV_HD double& operator()(int r, int c) const { return A[r][c]; }
};
struct EpnpWsSoA {
    double* p;
    int64_t s;
    MCV_HD double& operator()(int r, int c) const { return p[(int64_t)(12 * r + c) * s]; }
};
// L_6x10 and rho alone (rows 0..5, columns 0..10) at p[11 r + c]: the betas kernel's per-lane LDS copy,
// which Gauss-Newton re-reads every iteration.
struct EpnpLRef {
    double* p;
    MCV_HD double& operator()(int r, int c) const { return p[11 * r + c]; }
};

// jacobi_svd_core's tail for the 12 x 12 without V (EPnP's cvSVD of M^T M) on a view: the row norms,
// the descending selection sort (row swaps) and the cv::RNG completion of null rows, in the generic
// loop's order. W: the squared norms the sweeps left (in), nothing useful (out).
template <class WS>
MCV_HD void jacobi12_tail(const WS& A, double (&W)[12]) {
    const double eps = kDblEpsilon * 10, minval = kDblMin;
    for (int i = 0; i < 12; ++i) {
        double sd = 0;
        MCV_SMALL_UNROLL
        for (int k = 0; k < 12; ++k) sd += A(i, k) * A(i, k);
        W[i] = __builtin_sqrt(sd);
    }
    for (int i = 0; i < 11; ++i) {
        int j = i;
        double wj = W[i];
        for (int k = i + 1; k < 12; ++k)
            if (wj < W[k]) j = k, wj = W[k];
        if (j != i) {
            const double tw = W[i]; W[i] = W[j]; W[j] = tw;
            MCV_SMALL_UNROLL
            for (int k = 0; k < 12; ++k) { const double t = A(i, k); A(i, k) = A(j, k); A(j, k) = t; }
        }
    }
    // row i in registers while it is completed / normalised (the view may be memory the compiler cannot
    // prove distinct from row j's)
    CvRng rng{0x12345678u};
    for (int i = 0; i < 12; ++i) {
        double sd = W[i];
        double ri[12];
        MCV_SMALL_UNROLL
        for (int k = 0; k < 12; ++k) ri[k] = A(i, k);
        for (int ii = 0; ii < 100 && sd <= minval; ++ii) {
            const double val0 = 1. / 12;
            MCV_SMALL_UNROLL
            for (int k = 0; k < 12; ++k) ri[k] = (rng.next() & 256) != 0 ? val0 : -val0;
            for (int it = 0; it < 2; ++it)
                for (int j = 0; j < i; ++j) {
                    double rj[12];
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < 12; ++k) rj[k] = A(j, k);
                    sd = 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < 12; ++k) sd += ri[k] * rj[k];
                    double asum = 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < 12; ++k) {
                        const double t = ri[k] - sd * rj[k];
                        ri[k] = t;
                        asum += __builtin_fabs(t);
                    }
                    asum = asum > eps * 100 ? 1 / asum : 0;
                    MCV_SMALL_UNROLL
                    for (int k = 0; k < 12; ++k) ri[k] *= asum;
                }
            sd = 0;
            MCV_SMALL_UNROLL
            for (int k = 0; k < 12; ++k) sd += ri[k] * ri[k];
            sd = __builtin_sqrt(sd);
        }
        const double s = sd > minval ? 1 / sd : 0.;
        MCV_SMALL_UNROLL
        for (int k = 0; k < 12; ++k) A(i, k) = ri[k] * s;
    }
}

// jacobi_svd_core's sweeps for the 12 x 12 without V (the device's EPnP SVD kernel) with the working
// matrix split by columns: columns 0..5 of row r at lo[6 r ..] (the caller's per-lane LDS slice,
// 37 KB per wave: four waves per CU), columns 6..11 in registers (hi[r]). The pair loop keeps i
// rolled and expands j at compile time (j12_pairs<J>), so row j's register half and W[j] are fixed
// registers and its LDS half sits at a constant offset; row i's register half and W[i] are read and
// written once per i through a wave-uniform branch chain (j12_get / j12_set; each case is pinned as a
// branch, so a read costs the matched case's moves, not a select over all rows), and row j + 1's LDS
// half is loaded before row j's rotation. The operations and their order are the generic loop's: p,
// the rotation and the two sums run over k = 0..11 in order, and W[i] / W[j] / the rows change where
// it changes them.
// A value moved through an empty asm tagged with the case number: the copies of one case cannot be
// merged with another case's into a load or store through a phi of addresses (which would keep the
// register rows in scratch).
#if defined(__HIP_DEVICE_COMPILE__)
#define MCV_PIN_CASE(x, q) asm volatile("; j12 case %1" : "+v"(x) : "i"(q))
#else
#define MCV_PIN_CASE(x, q) ((void)0)
#endif
template <int Q>
MCV_HD void j12_get(const double (&hi)[12][6], const double (&W)[12], int r, double* o, double& w) {
    if (Q == r) {
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) {
            double x = hi[Q][k];
            MCV_PIN_CASE(x, Q);
            o[k] = x;
        }
        double x = W[Q];
        MCV_PIN_CASE(x, Q);
        w = x;
    }
    if constexpr (Q < 10) j12_get<Q + 1>(hi, W, r, o, w);
}
template <int Q>
MCV_HD void j12_set(double (&hi)[12][6], double (&W)[12], int r, const double* o, double w, bool rot) {
    if (Q == r) {
        double x = w;
        MCV_PIN_CASE(x, Q);
        W[Q] = x;
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) {
            double y = rot ? o[k] : hi[Q][k];
            MCV_PIN_CASE(y, Q);
            hi[Q][k] = y;
        }
    }
    if constexpr (Q < 10) j12_set<Q + 1>(hi, W, r, o, w, rot);
}
template <int J>
MCV_HD void j12_pairs(double* lo, double (&hi)[12][6], double (&W)[12], int i, double (&ri)[12], double& wi,
                      double (&nx)[6], bool& changed, bool& iRot) {
    if (J > i) {
        const double eps = kDblEpsilon * 10;
        double rj[12];
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) rj[k] = nx[k];
        MCV_SMALL_UNROLL
        for (int k = 0; k < 6; ++k) rj[6 + k] = hi[J][k];
        if constexpr (J < 11)
            MCV_SMALL_UNROLL
            for (int k = 0; k < 6; ++k) nx[k] = lo[6 * (J + 1) + k];
        double a = wi, b = W[J], p = 0;
        MCV_SMALL_UNROLL
        for (int k = 0; k < 12; ++k) p += ri[k] * rj[k];
        if (!(__builtin_fabs(p) <= eps * __builtin_sqrt(a * b))) {
            p *= 2;
            double c, s;
            svd_rotation(p, a, b, c, s);
            a = b = 0;
            MCV_SMALL_UNROLL
            for (int k = 0; k < 12; ++k) {
                const double t0 = c * ri[k] + s * rj[k];
                const double t1 = -s * ri[k] + c * rj[k];
                ri[k] = t0;
                rj[k] = t1;
                a += t0 * t0;
                b += t1 * t1;
            }
            wi = a;
            W[J] = b;
            changed = true;
            iRot = true;
            MCV_SMALL_UNROLL
            for (int k = 0; k < 6; ++k) lo[6 * J + k] = rj[k];
            MCV_SMALL_UNROLL
            for (int k = 0; k < 6; ++k) hi[J][k] = rj[6 + k];
        }
    }
    if constexpr (J < 11) j12_pairs<J + 1>(lo, hi, W, i, ri, wi, nx, changed, iRot);
}
MCV_HD void jacobi12_sweeps_split(double* lo, double (&hi)[12][6], double (&W)[12]) {
    for (int iter = 0; iter < 30; ++iter) {
        bool changed = false;
        for (int i = 0; i < 11; ++i) {
            double ri[12], wi = 0, nx[6];
            MCV_SMALL_UNROLL
            for (int k = 0; k < 6; ++k) ri[k] = lo[6 * i + k];
            j12_get<0>(hi, W, i, ri + 6, wi);
            MCV_SMALL_UNROLL
            for (int k = 0; k < 6; ++k) nx[k] = lo[6 * (i + 1) + k];
            bool iRot = false;
            j12_pairs<1>(lo, hi, W, i, ri, wi, nx, changed, iRot);
            j12_set<0>(hi, W, i, ri + 6, wi, iRot);
            if (iRot)
                MCV_SMALL_UNROLL
                for (int k = 0; k < 6; ++k) lo[6 * i + k] = ri[k];
        }
        if (!changed) break;
    }
}

// L_6x10 row r at ws(r, 0 .. 9), rho[r] at ws(r, 10).
template <class WS>
MCV_HD void epnp_gauss_newton(const WS& ws, double (&be)[4]) {
    double X[4] = {0, 0, 0, 0};   // kept across iterations, as epnp::gauss_newton's x
    for (int it = 0; it < 5; ++it) {
#if defined(__HIP_DEVICE_COMPILE__)
        // re-read L and rho from the workspace every iteration (hoisted, they would hold 132 registers)
        asm volatile("" ::: "memory");
#endif
        double A[6][4], b[6];
        MCV_SMALL_UNROLL
        for (int i = 0; i < 6; ++i) {
            double l[11];
            MCV_SMALL_UNROLL
            for (int k = 0; k < 11; ++k) l[k] = ws(i, k);
            A[i][0] = 2 * l[0] * be[0] + l[1] * be[1] + l[3] * be[2] + l[6] * be[3];
            A[i][1] = l[1] * be[0] + 2 * l[2] * be[1] + l[4] * be[2] + l[7] * be[3];
            A[i][2] = l[3] * be[0] + l[4] * be[1] + 2 * l[5] * be[2] + l[8] * be[3];
            A[i][3] = l[6] * be[0] + l[7] * be[1] + l[8] * be[2] + 2 * l[9] * be[3];
            b[i] = l[10] - (l[0] * be[0] * be[0] + l[1] * be[0] * be[1] + l[2] * be[1] * be[1] +
                            l[3] * be[0] * be[2] + l[4] * be[1] * be[2] + l[5] * be[2] * be[2] +
                            l[6] * be[0] * be[3] + l[7] * be[1] * be[3] + l[8] * be[2] * be[3] +
                            l[9] * be[3] * be[3]);
        }
        epnp_qr_solve(A, b, X);
        MCV_SMALL_UNROLL
        for (int i = 0; i < 4; ++i) be[i] += X[i];
    }
}

// A: the 12 x 12 working matrix of the SVD (caller storage: a register / scratch array on the host,
// a per-lane LDS slice in the GPU hypothesis kernel).
typedef double EpnpWs[12][12];

// compute_pose from M^T M to the betas of the three approximations, in place: on entry A holds the
// full symmetric M^T M; on return its rows 11, 10, 9, 8 are the four null-space vectors v_0..v_3
// (rows of U^T), rows 0..5 hold L_6x10 (columns 0..9) and rho (column 10) — the working matrix keeps
// what the GPU lane would otherwise hold in registers (v, L, rho: 114 doubles).
// compute_L_6x10 and rho from the null-space vectors (rows 11, 10, 9, 8) into rows 0..5.
template <class WS>
MCV_HD void epnp_l_rows(const double (&cws)[4][3], const WS& A) {
    {
        const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
        MCV_SMALL_UNROLL
        for (int r = 0; r < 6; ++r) {
            // edge r = (a, b) of compute_L_6x10's dv loop (a = 0, b = 1, 2, 3, then 1-2, 1-3, 2-3)
            double dv[4][3];
            MCV_SMALL_UNROLL
            for (int i = 0; i < 4; ++i)
                MCV_SMALL_UNROLL
                for (int k = 0; k < 3; ++k) dv[i][k] = A(11 - i, 3 * pa[r] + k) - A(11 - i, 3 * pb[r] + k);
            A(r, 0) = dot3(dv[0], dv[0]);
            A(r, 1) = 2.0 * dot3(dv[0], dv[1]);
            A(r, 2) = dot3(dv[1], dv[1]);
            A(r, 3) = 2.0 * dot3(dv[0], dv[2]);
            A(r, 4) = 2.0 * dot3(dv[1], dv[2]);
            A(r, 5) = dot3(dv[2], dv[2]);
            A(r, 6) = 2.0 * dot3(dv[0], dv[3]);
            A(r, 7) = 2.0 * dot3(dv[1], dv[3]);
            A(r, 8) = 2.0 * dot3(dv[2], dv[3]);
            A(r, 9) = dot3(dv[3], dv[3]);
            const double* p1 = cws[pa[r]];
            const double* p2 = cws[pb[r]];
            A(r, 10) = (p1[0] - p2[0]) * (p1[0] - p2[0]) + (p1[1] - p2[1]) * (p1[1] - p2[1]) +
                       (p1[2] - p2[2]) * (p1[2] - p2[2]);
        }
    }
}

// The SVD of M^T M (in A on entry) and L_6x10 / rho.
MCV_HD void epnp_null_and_l(const double (&cws)[4][3], EpnpWs& A) {
    {
        // cvSVD(MtM, D, Ut, 0, MODIFY_A | U_T): Jacobi on transpose(MtM) (= MtM after completeSymm)
        double w[12];
        jacobi_svd<12, 12>(A, w, nullptr);
    }
    epnp_l_rows(cws, EpnpWsRef{A});
}

// Second half: the betas of the three approximations from L_6x10 / rho (ws rows 0..5).
template <class WS>
MCV_HD void epnp_betas_from_l(double (&betas)[4][4], const WS& A) {
    double rho[6];
    MCV_SMALL_UNROLL
    for (int i = 0; i < 6; ++i) rho[i] = A(i, 10);
    for (int k = 0; k < 4; ++k) betas[0][k] = 0;
    {   // approximation 1: [B11 B12 B13 B14]
        double L4[6][4], b4[4];
        MCV_SMALL_UNROLL
        for (int i = 0; i < 6; ++i) { L4[i][0] = A(i, 0); L4[i][1] = A(i, 1); L4[i][2] = A(i, 3); L4[i][3] = A(i, 6); }
        svd_solve6<4>(L4, rho, b4);
        double* be = betas[1];
        if (b4[0] < 0) {
            be[0] = __builtin_sqrt(-b4[0]);
            be[1] = -b4[1] / be[0];
            be[2] = -b4[2] / be[0];
            be[3] = -b4[3] / be[0];
        } else {
            be[0] = __builtin_sqrt(b4[0]);
            be[1] = b4[1] / be[0];
            be[2] = b4[2] / be[0];
            be[3] = b4[3] / be[0];
        }
        epnp_gauss_newton(A, betas[1]);
    }
    {   // approximation 2: [B11 B12 B22]
        double L3[6][3], b3[3];
        MCV_SMALL_UNROLL
        for (int i = 0; i < 6; ++i) { L3[i][0] = A(i, 0); L3[i][1] = A(i, 1); L3[i][2] = A(i, 2); }
        svd_solve6<3>(L3, rho, b3);
        double* be = betas[2];
        if (b3[0] < 0) {
            be[0] = __builtin_sqrt(-b3[0]);
            be[1] = (b3[2] < 0) ? __builtin_sqrt(-b3[2]) : 0.0;
        } else {
            be[0] = __builtin_sqrt(b3[0]);
            be[1] = (b3[2] > 0) ? __builtin_sqrt(b3[2]) : 0.0;
        }
        if (b3[1] < 0) be[0] = -be[0];
        be[2] = 0.0;
        be[3] = 0.0;
        epnp_gauss_newton(A, betas[2]);
    }
    {   // approximation 3: [B11 B12 B22 B13 B23]
        double L5[6][5], b5[5];
        MCV_SMALL_UNROLL
        for (int i = 0; i < 6; ++i)
            MCV_SMALL_UNROLL
            for (int k = 0; k < 5; ++k) L5[i][k] = A(i, k);
        svd_solve6<5>(L5, rho, b5);
        double* be = betas[3];
        if (b5[0] < 0) {
            be[0] = __builtin_sqrt(-b5[0]);
            be[1] = (b5[2] < 0) ? __builtin_sqrt(-b5[2]) : 0.0;
        } else {
            be[0] = __builtin_sqrt(b5[0]);
            be[1] = (b5[2] > 0) ? __builtin_sqrt(b5[2]) : 0.0;
        }
        if (b5[1] < 0) be[0] = -be[0];
        be[2] = b5[3] / be[0];
        be[3] = 0.0;
        epnp_gauss_newton(A, betas[3]);
    }
}

MCV_HD void epnp_betas_ws(const EpnpCtrl& C, double (&betas)[4][4], EpnpWs& A) {
    epnp_null_and_l(C.cws, A);
    epnp_betas_from_l(betas, EpnpWsRef{A});
}

// The same from the packed upper triangle of M^T M (the host inlier solve), with the null-space
// vectors copied out.
MCV_HD void epnp_betas(const double (&mtm)[kMtmSums], const EpnpCtrl& C, EpnpBetas& B, EpnpWs& A) {
    for (int a = 0; a < 12; ++a)
        for (int b = a; b < 12; ++b) A[a][b] = A[b][a] = mtm[mtm_index(a, b)];
    epnp_betas_ws(C, B.betas, A);
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 12; ++k) B.v[i][k] = A[11 - i][k];
}

MCV_HD void epnp_betas(const double (&mtm)[kMtmSums], const EpnpCtrl& C, EpnpBetas& B) {
    EpnpWs A;
    epnp_betas(mtm, C, B, A);
}

// Control points in the camera frame for one beta vector (compute_ccs).
MCV_HD void epnp_ccs(const EpnpBetas& B, const double (&be)[4], double (&ccs)[4][3]) {
    for (int j = 0; j < 4; ++j)
        for (int k = 0; k < 3; ++k) ccs[j][k] = 0.0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) ccs[j][k] += be[i] * B.v[i][3 * j + k];
}

// The same with the null-space vectors in the workspace (v_i = ws(11 - i, .), epnp_betas_ws).
template <class WS>
MCV_HD void epnp_ccs_ws(const WS& A, const double (&be)[4], double (&ccs)[4][3]) {
    MCV_SMALL_UNROLL
    for (int j = 0; j < 4; ++j)
        MCV_SMALL_UNROLL
        for (int k = 0; k < 3; ++k) ccs[j][k] = 0.0;
    MCV_SMALL_UNROLL
    for (int i = 0; i < 4; ++i)
        MCV_SMALL_UNROLL
        for (int j = 0; j < 4; ++j)
            MCV_SMALL_UNROLL
            for (int k = 0; k < 3; ++k) ccs[j][k] += be[i] * A(11 - i, 3 * j + k);
}

MCV_HD void epnp_pc(const double (&a)[4], const double (&ccs)[4][3], double (&pc)[3]) {
    for (int j = 0; j < 3; ++j) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
}

// estimate_R_and_t's tail: R = U V^T of ABt (cvSVD, no transposes), det fix, t = pc0 - R pw0.
MCV_HD void epnp_rt(const double (&abt)[3][3], const double (&pc0)[3], const double (&pw0)[3], double (&R)[3][3],
                    double (&t)[3]) {
    double A[3][3], w[3], Vt[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) A[i][j] = abt[j][i];
    jacobi_svd<3, 3>(A, w, Vt);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = A[0][i] * Vt[0][j] + A[1][i] * Vt[1][j] + A[2][i] * Vt[2][j];
    const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                       R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
    if (det < 0) {
        R[2][0] = -R[2][0];
        R[2][1] = -R[2][1];
        R[2][2] = -R[2][2];
    }
    for (int i = 0; i < 3; ++i) t[i] = pc0[i] - dot3(R[i], pw0);
}

// One term of reprojection_error.
MCV_HD double epnp_reproj_term(const double (&R)[3][3], const double (&t)[3], const EpnpCam& c, const double* pw,
                               double u, double v) {
    const double Xc = dot3(R[0], pw) + t[0];
    const double Yc = dot3(R[1], pw) + t[1];
    const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
    const double ue = c.uc + c.fu * Xc * inv_Zc;
    const double ve = c.vc + c.fv * Yc * inv_Zc;
    return __builtin_sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
}

// compute_pose's final choice: N = 1, then 2 / 3 if strictly smaller.
MCV_HD int epnp_pick(const double (&rep)[4]) {
    int N = 1;
    if (rep[2] < rep[1]) N = 2;
    if (rep[3] < rep[N]) N = 3;
    return N;
}

// Whole EPnP for a small point set held by the caller (RANSAC minimal sets, n = NP):
// pw[i] world points, us[i] pixel coordinates (undistorted normalised * f + c). Three parts, which the
// split device generate runs as three kernels: epnp_small_mtm (control points, alphas, M^T M into ws),
// epnp_null_and_l (the 12 x 12 SVD and L_6x10 in ws) and epnp_small_pose (betas, Gauss-Newton, the
// three poses and the pick).
template <int NP>
MCV_HD void epnp_small_mtm(const double (&pw)[NP][3], const double (&us)[NP][2], const EpnpCam& cam, EpnpCtrl& C,
                           double (&al)[NP][4], double (&mtm)[kMtmSums]) {
    {
        double sum[3] = {0, 0, 0};
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < 3; ++j) sum[j] += pw[i][j];
        double c0[3];
        for (int j = 0; j < 3; ++j) c0[j] = sum[j] / NP;
        double P[3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = a; b < 3; ++b) {
                double s = 0;
                for (int i = 0; i < NP; ++i) s += (pw[i][a] - c0[a]) * (pw[i][b] - c0[b]);
                P[a][b] = P[b][a] = s;
            }
        epnp_control(sum, P, NP, C);
    }
    for (int i = 0; i < NP; ++i) epnp_alphas(C, pw[i], al[i]);
    {
        for (int k = 0; k < kMtmSums; ++k) mtm[k] = 0;
        for (int i = 0; i < NP; ++i) {
            double r1[12], r2[12];
            epnp_m_rows(al[i], us[i][0], us[i][1], cam, r1, r2);
            int o = 0;
            for (int a = 0; a < 12; ++a)
                for (int b = a; b < 12; ++b, ++o) {
                    mtm[o] += r1[a] * r1[b];
                    mtm[o] += r2[a] * r2[b];
                }
        }
    }
}

template <int NP, class WS>
MCV_HD void epnp_small_pick(const double (&pw)[NP][3], const double (&us)[NP][2], const EpnpCam& cam,
                            const double (&al)[NP][4], const WS& ws, const double (&betas)[4][4],
                            double (&Rout)[3][3], double (&tout)[3]) {
    double pw0[3] = {0, 0, 0};
    for (int i = 0; i < NP; ++i)
        for (int j = 0; j < 3; ++j) pw0[j] += pw[i][j];
    for (int j = 0; j < 3; ++j) pw0[j] /= NP;
    // compute_pose's choice (epnp_pick: N = 1, then 2 / 3 if strictly smaller) as a running best
    double bestRep = 0;
    for (int N = 1; N <= 3; ++N) {
        double ccs[4][3], pc[NP][3];
        epnp_ccs_ws(ws, betas[N], ccs);
        for (int i = 0; i < NP; ++i) epnp_pc(al[i], ccs, pc[i]);
        if (pc[0][2] < 0.0)   // solve_for_sign
            for (int i = 0; i < NP; ++i)
                for (int j = 0; j < 3; ++j) pc[i][j] = -pc[i][j];
        double pc0[3] = {0, 0, 0};
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < 3; ++j) pc0[j] += pc[i][j];
        for (int j = 0; j < 3; ++j) pc0[j] /= NP;
        double abt[3][3];
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) abt[j][k] = 0;
        for (int i = 0; i < NP; ++i)
            for (int j = 0; j < 3; ++j)
                for (int k = 0; k < 3; ++k) abt[j][k] += (pc[i][j] - pc0[j]) * (pw[i][k] - pw0[k]);
        double R[3][3], t[3];
        epnp_rt(abt, pc0, pw0, R, t);
        double s = 0.0;
        for (int i = 0; i < NP; ++i) s += epnp_reproj_term(R, t, cam, pw[i], us[i][0], us[i][1]);
        const double rep = s / NP;
        if (N == 1 || rep < bestRep) {
            bestRep = rep;
            for (int i = 0; i < 3; ++i) {
                for (int j = 0; j < 3; ++j) Rout[i][j] = R[i][j];
                tout[i] = t[i];
            }
        }
    }
}

// The betas of the three approximations (v, L and rho in ws), then the three poses and the pick.
template <int NP, class WS>
MCV_HD void epnp_small_pose(const double (&pw)[NP][3], const double (&us)[NP][2], const EpnpCam& cam,
                            const double (&al)[NP][4], const WS& ws, double (&Rout)[3][3], double (&tout)[3]) {
    double betas[4][4];
    epnp_betas_from_l(betas, ws);
    epnp_small_pick<NP>(pw, us, cam, al, ws, betas, Rout, tout);
}

template <int NP>
MCV_HD void epnp_solve_small(const double (&pw)[NP][3], const double (&us)[NP][2], const EpnpCam& cam,
                             double (&Rout)[3][3], double (&tout)[3], EpnpWs& ws) {
    EpnpCtrl C;
    double al[NP][4];
    {
        double mtm[kMtmSums];
        epnp_small_mtm<NP>(pw, us, cam, C, al, mtm);
        for (int a = 0; a < 12; ++a)
            for (int b = a; b < 12; ++b) ws[a][b] = ws[b][a] = mtm[mtm_index(a, b)];
    }
    epnp_null_and_l(C.cws, ws);
    epnp_small_pose<NP>(pw, us, cam, al, EpnpWsRef{ws}, Rout, tout);
}

template <int NP>
MCV_HD void epnp_solve_small(const double (&pw)[NP][3], const double (&us)[NP][2], const EpnpCam& cam,
                             double (&Rout)[3][3], double (&tout)[3]) {
    EpnpWs ws;
    epnp_solve_small<NP>(pw, us, cam, Rout, tout, ws);
}

}  // namespace mcv
