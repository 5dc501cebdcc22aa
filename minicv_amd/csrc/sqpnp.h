// sqpnp.h — SQPnP (Terzakis & Lourakis, ECCV 2020) as OpenCV 4.x's calib3d sqpnp.cpp computes it
// [ext: OpenCV, not vendored in /root/reference]: cv::sqpnp::PoseSolver in the build without Eigen
// (Omega's null space from cv::SVD = JacobiSVDImpl_, epnp.h), nearest rotations by FOAM with the SVD
// fallback for |det| < 1e-4. It answers cvSolvePnP solverKind 6 (reference MiniCVNative.cpp:72-74,
// :82: solvePnP(SOLVEPNP_SQPNP) on undistortPoints' normalised coordinates).
//
// Split as the other solvePnP paths are: the O(n) loop of computeOmega (39 sums) and the cheirality
// count of positiveMajorityDepths run on the GPU as blocked fixed-order passes (mcv_epnp_pass modes
// kEpnpPassSqp / kEpnpPassSqpDepth, ransac_pnp.hip); the O(1) algebra below (Omega / P assembly,
// the 9 x 9 SVD, the SQP iterations, the solution list) runs on the host between them. Built with
// -ffp-contract=off; oracle/oracle_sqpnp.c restates the same algorithm in C and the two agree bit for
// bit (tests/test_gpu_pnp.py). Operation order follows the OpenCV file as written: Matx products
// summed from 0 in index order, cv::norm through normL2Sqr's four-way unrolled loop (parity with
// OpenCV's own bits is unpinned: no OpenCV here).
#pragma once
#include <cfloat>
#include <cmath>
#include <cstring>

#include "epnp.h"

namespace mcv {

static const int kSqpSums = 39;

// Accumulator a of computeOmega's per-point terms: omega's upper-triangle blocks (X2 .. Z2; -x X2 ..;
// -y X2 ..; |x|^2 X2 ..), qa_sum's row 0 (X, Y, Z; also sum_obj) and its right block (-x X ..; -y X ..;
// |x|^2 X ..), sum_img (x, y) and the sum of |x|^2.
MCV_HD double sqpnp_term(double x, double y, double X, double Y, double Z, int a) {
    const double sq = x * x + y * y;
    double q;
    int g;
    if (a < 24) {
        g = a / 6;
        const int k = a - 6 * g;
        q = k == 0 ? X * X : k == 1 ? X * Y : k == 2 ? X * Z : k == 3 ? Y * Y : k == 4 ? Y * Z : Z * Z;
    } else if (a < 36) {
        g = (a - 24) / 3;
        const int k = a - 24 - 3 * g;
        q = k == 0 ? X : k == 1 ? Y : Z;
    } else {
        return a == 36 ? x : a == 37 ? y : sq;
    }
    return g == 0 ? q : g == 1 ? -x * q : g == 2 ? -y * q : sq * q;
}

namespace sqp {

// normL2Sqr<double, double> (core base.hpp, CV_ENABLE_UNROLLED): what cv::norm of a Matx sums.
inline double norm_sqr(const double* a, int n) {
    double s = 0;
    int i = 0;
    for (; i <= n - 4; i += 4) s += a[i] * a[i] + a[i + 1] * a[i + 1] + a[i + 2] * a[i + 2] + a[i + 3] * a[i + 3];
    for (; i < n; i++) s += a[i] * a[i];
    return s;
}

inline double det9(const double* e) {
    return e[0] * e[4] * e[8] + e[1] * e[5] * e[6] + e[2] * e[3] * e[7] - e[6] * e[4] * e[2] - e[7] * e[5] * e[0] -
           e[8] * e[3] * e[1];
}

// analyticalInverse3x3Symm (lower triangle read; "det" is minus the determinant, as written there);
// below the 1e-8 threshold Qi keeps what it holds.
inline bool inv3_symm(const double* Q, double* Qi) {
    const double a = Q[0], b = Q[3], d = Q[4], c = Q[6], e = Q[7], f = Q[8];
    const double t2 = e * e, t4 = a * d, t7 = b * b, t9 = b * c, t12 = c * c;
    const double det = -t4 * f + a * t2 + t7 * f - 2.0 * t9 * e + t12 * d;
    if (std::fabs(det) < 1e-8) return false;
    const double t15 = 1.0 / det;
    const double t20 = (-b * f + c * e) * t15, t24 = (b * e - c * d) * t15, t30 = (a * e - t9) * t15;
    Qi[0] = (-d * f + t2) * t15;
    Qi[1] = Qi[3] = -t20;
    Qi[2] = Qi[6] = -t24;
    Qi[4] = -(a * f - t12) * t15;
    Qi[5] = Qi[7] = t30;
    Qi[8] = -(t4 - t7) * t15;
    return true;
}

// cv::determinant of a 3 x 3 (core lapack.cpp's explicit expansion)
inline double cv_det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

// nearestRotationMatrixSVD: U diag(1, 1, det U det Vt) Vt of cv::SVD(e33, FULL_UV).
inline void nearest_rot_svd(const double* e, double* r) {
    double At[3][3], w[3], Vt[3][3], U[9], D[9], T[9];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) At[i][k] = e[3 * k + i];
    jacobi_svd<3, 3>(At, w, Vt);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) U[3 * i + j] = At[j][i];
    const double detuv = cv_det3(U) * cv_det3(&Vt[0][0]);
    std::memset(D, 0, sizeof(D));
    D[0] = 1;
    D[4] = 1;
    D[8] = detuv;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += U[3 * i + k] * D[3 * k + j];
            T[3 * i + j] = s;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += T[3 * i + k] * Vt[k][j];
            r[3 * i + j] = s;
        }
}

// nearestRotationMatrixFOAM (Lourakis, ICPR 2016): lambda_max by Newton on FOAM's characteristic
// polynomial, then R = ((l^2 + |e|^2) e + 2 l adj(e)^T - 2 e e^T e) / (l (l^2 - |e|^2) - 2 det e).
inline void nearest_rot(const double* e, double* r) {
    const double det_e = e[0] * e[4] * e[8] - e[0] * e[5] * e[7] - e[1] * e[3] * e[8] + e[2] * e[3] * e[7] +
                         e[1] * e[6] * e[5] - e[2] * e[6] * e[4];
    if (std::fabs(det_e) < 1e-4) {
        nearest_rot_svd(e, r);
        return;
    }
    const double adj[9] = {e[4] * e[8] - e[5] * e[7], e[2] * e[7] - e[1] * e[8], e[1] * e[5] - e[2] * e[4],
                           e[5] * e[6] - e[3] * e[8], e[0] * e[8] - e[2] * e[6], e[2] * e[3] - e[0] * e[5],
                           e[3] * e[7] - e[4] * e[6], e[1] * e[6] - e[0] * e[7], e[0] * e[4] - e[1] * e[3]};
    double e_sq = e[0] * e[0], adj_sq = adj[0] * adj[0];
    for (int k = 1; k < 9; k++) {
        e_sq = e_sq + e[k] * e[k];
        adj_sq = adj_sq + adj[k] * adj[k];
    }
    double l = 2.0, lprev = 0.0;
    for (int i = 200; std::fabs(l - lprev) > 1e-12 * std::fabs(lprev) && i > 0; --i) {
        const double tmp = l * l - e_sq;
        const double p = tmp * tmp - 8.0 * l * det_e - 4.0 * adj_sq;
        const double pp = 8.0 * (0.5 * tmp * l - det_e);
        lprev = l;
        l -= p / pp;
    }
    const double a = l * l + e_sq;
    double eet[9], tmp[9];
    eet[0] = e[0] * e[0] + e[1] * e[1] + e[2] * e[2];
    eet[1] = e[0] * e[3] + e[1] * e[4] + e[2] * e[5];
    eet[2] = e[0] * e[6] + e[1] * e[7] + e[2] * e[8];
    eet[3] = eet[1];
    eet[4] = e[3] * e[3] + e[4] * e[4] + e[5] * e[5];
    eet[5] = e[3] * e[6] + e[4] * e[7] + e[5] * e[8];
    eet[6] = eet[2];
    eet[7] = eet[5];
    eet[8] = e[6] * e[6] + e[7] * e[7] + e[8] * e[8];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            tmp[3 * i + j] = eet[3 * i] * e[j] + eet[3 * i + 1] * e[3 + j] + eet[3 * i + 2] * e[6 + j];
    const double denom = 1.0 / (l * (l * l - e_sq) - 2.0 * det_e);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            r[3 * i + j] = (a * e[3 * i + j] + 2.0 * (l * adj[3 * j + i] - tmp[3 * i + j])) * denom;
}

// computeRowAndNullspace: H (9 x 6) = Gram-Schmidt of the constraint gradients in the order |r1|^2,
// |r2|^2, |r3|^2, r1.r2, r2.r3, r1.r3; K = J H (lower triangular); N (9 x 3) = three well-spread
// columns of the projector I - H H^T (column norm >= 0.1), orthonormalised.
inline void row_and_nullspace(const double* r, double (&H)[9][6], double (&N)[9][3], double (&K)[6][6]) {
    std::memset(H, 0, sizeof(H));
    std::memset(K, 0, sizeof(K));
    auto unit = [&](int c, int row0, int r0) {
        const double nr = std::sqrt(r[r0] * r[r0] + r[r0 + 1] * r[r0 + 1] + r[r0 + 2] * r[r0 + 2]);
        const double inr = nr > 1e-5 ? 1.0 / nr : 0.0;
        for (int k = 0; k < 3; k++) H[row0 + k][c] = r[r0 + k] * inr;
        K[c][c] = 2 * nr;
    };
    unit(0, 0, 0);
    unit(1, 3, 3);
    unit(2, 6, 6);
    auto normalise = [&](int c, int rows) {
        double s = 0;
        for (int i = 0; i < rows; i++) s += H[i][c] * H[i][c];
        const double in = 1.0 / std::sqrt(s);
        for (int i = 0; i < rows; i++) H[i][c] *= in;
    };
    // q4: j4 = (r2, r1, 0)
    const double d41 = r[3] * H[0][0] + r[4] * H[1][0] + r[5] * H[2][0];
    const double d42 = r[0] * H[3][1] + r[1] * H[4][1] + r[2] * H[5][1];
    for (int k = 0; k < 3; k++) {
        H[k][3] = r[3 + k] - d41 * H[k][0];
        H[3 + k][3] = r[k] - d42 * H[3 + k][1];
    }
    normalise(3, 6);
    K[3][0] = r[3] * H[0][0] + r[4] * H[1][0] + r[5] * H[2][0];
    K[3][1] = r[0] * H[3][1] + r[1] * H[4][1] + r[2] * H[5][1];
    K[3][3] = r[3] * H[0][3] + r[4] * H[1][3] + r[5] * H[2][3] + r[0] * H[3][3] + r[1] * H[4][3] + r[2] * H[5][3];
    // q5: j5 = (0, r3, r2)
    const double d52 = r[6] * H[3][1] + r[7] * H[4][1] + r[8] * H[5][1];
    const double d53 = r[3] * H[6][2] + r[4] * H[7][2] + r[5] * H[8][2];
    const double d54 = r[6] * H[3][3] + r[7] * H[4][3] + r[8] * H[5][3];
    for (int k = 0; k < 3; k++) {
        H[k][4] = -d54 * H[k][3];
        H[3 + k][4] = r[6 + k] - d52 * H[3 + k][1] - d54 * H[3 + k][3];
        H[6 + k][4] = r[3 + k] - d53 * H[6 + k][2];
    }
    normalise(4, 9);
    K[4][1] = r[6] * H[3][1] + r[7] * H[4][1] + r[8] * H[5][1];
    K[4][2] = r[3] * H[6][2] + r[4] * H[7][2] + r[5] * H[8][2];
    K[4][3] = r[6] * H[3][3] + r[7] * H[4][3] + r[8] * H[5][3];
    K[4][4] = r[6] * H[3][4] + r[7] * H[4][4] + r[8] * H[5][4] + r[3] * H[6][4] + r[4] * H[7][4] + r[5] * H[8][4];
    // q6: j6 = (r3, 0, r1)
    const double d61 = r[6] * H[0][0] + r[7] * H[1][0] + r[8] * H[2][0];
    const double d63 = r[0] * H[6][2] + r[1] * H[7][2] + r[2] * H[8][2];
    const double d64 = r[6] * H[0][3] + r[7] * H[1][3] + r[8] * H[2][3];
    const double d65 =
        r[6] * H[0][4] + r[7] * H[1][4] + r[8] * H[2][4] + r[0] * H[6][4] + r[1] * H[7][4] + r[2] * H[8][4];
    for (int k = 0; k < 3; k++) {
        H[k][5] = r[6 + k] - d61 * H[k][0] - d64 * H[k][3] - d65 * H[k][4];
        H[3 + k][5] = -d64 * H[3 + k][3] - d65 * H[3 + k][4];
        H[6 + k][5] = r[k] - d63 * H[6 + k][2] - d65 * H[6 + k][4];
    }
    normalise(5, 9);
    K[5][0] = r[6] * H[0][0] + r[7] * H[1][0] + r[8] * H[2][0];
    K[5][2] = r[0] * H[6][2] + r[1] * H[7][2] + r[2] * H[8][2];
    K[5][3] = r[6] * H[0][3] + r[7] * H[1][3] + r[8] * H[2][3];
    K[5][4] = r[6] * H[0][4] + r[7] * H[1][4] + r[8] * H[2][4] + r[0] * H[6][4] + r[1] * H[7][4] + r[2] * H[8][4];
    K[5][5] = r[6] * H[0][5] + r[7] * H[1][5] + r[8] * H[2][5] + r[0] * H[6][5] + r[1] * H[7][5] + r[2] * H[8][5];

    double Pc[9][9];   // columns of Pn = I - H H^T, one per row
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 6; k++) s += H[i][k] * H[j][k];
            Pc[j][i] = (i == j ? 1.0 : 0.0) - s;
        }
    auto dot9 = [](const double* a, const double* b) {
        double s = 0;
        for (int k = 0; k < 9; k++) s += a[k] * b[k];
        return s;
    };
    const double thr = 0.1;
    int i1 = 0, i2 = 0, i3 = 0;
    double max1 = DBL_MIN, min12 = DBL_MAX, min123 = DBL_MAX, cn[9];
    for (int i = 0; i < 9; i++) {
        cn[i] = std::sqrt(norm_sqr(Pc[i], 9));
        if (cn[i] >= thr && max1 < cn[i]) {
            max1 = cn[i];
            i1 = i;
        }
    }
    const double* v1 = Pc[i1];
    double n0[9], n1[9], n2[9];
    const double s1 = 1.0 / max1;
    for (int k = 0; k < 9; k++) n0[k] = v1[k] * s1;
    cn[i1] = -1.0;
    for (int i = 0; i < 9; i++)
        if (cn[i] >= thr) {
            const double c1 = std::fabs(dot9(Pc[i], v1) / cn[i]);
            if (c1 <= min12) {
                i2 = i;
                min12 = c1;
            }
        }
    const double* v2 = Pc[i2];
    {
        const double dd = dot9(v2, n0);
        for (int k = 0; k < 9; k++) n1[k] = v2[k] - dd * n0[k];
        const double s = 1.0 / std::sqrt(norm_sqr(n1, 9));
        for (int k = 0; k < 9; k++) n1[k] *= s;
    }
    cn[i2] = -1.0;
    for (int i = 0; i < 9; i++)
        if (cn[i] >= thr) {
            const double inv = 1.0 / cn[i];
            const double c1 = std::fabs(dot9(Pc[i], v1) * inv), c2 = std::fabs(dot9(Pc[i], v2) * inv);
            if (c1 + c2 <= min123) {
                i3 = i;
                min123 = c1 + c2;
            }
        }
    const double* v3 = Pc[i3];
    {
        const double a1 = dot9(v3, n1), a0 = dot9(v3, n0);
        for (int k = 0; k < 9; k++) n2[k] = v3[k] - a1 * n1[k] - a0 * n0[k];
        const double s = 1.0 / std::sqrt(norm_sqr(n2, 9));
        for (int k = 0; k < 9; k++) n2[k] *= s;
    }
    for (int k = 0; k < 9; k++) {
        N[k][0] = n0[k];
        N[k][1] = n1[k];
        N[k][2] = n2[k];
    }
}

struct Solver {
    double omega[81], p[27], s[9], u[81];   // u: rows = columns of OpenCV's u_ (rows of cv::SVD's vt)
    double mean[3];
    int nnull = -1;
    double rh[18][9], t[18][3], err[18];
    int nsol = 0;
};

// solveSQPSystem: delta = H x (K x = g by forward substitution) + N y, y minimising the linearised
// objective over the constraint null space.
inline void sqp_step(const Solver& S, const double* r, double* delta) {
    double H[9][6], N[9][3], K[6][6];
    row_and_nullspace(r, H, N, K);
    const double sn1 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2], sn2 = r[3] * r[3] + r[4] * r[4] + r[5] * r[5],
                 sn3 = r[6] * r[6] + r[7] * r[7] + r[8] * r[8];
    const double d12 = r[0] * r[3] + r[1] * r[4] + r[2] * r[5], d13 = r[0] * r[6] + r[1] * r[7] + r[2] * r[8],
                 d23 = r[3] * r[6] + r[4] * r[7] + r[5] * r[8];
    const double g[6] = {1 - sn1, 1 - sn2, 1 - sn3, -d12, -d23, -d13};
    double x[6];
    x[0] = g[0] / K[0][0];
    x[1] = g[1] / K[1][1];
    x[2] = g[2] / K[2][2];
    x[3] = (g[3] - K[3][0] * x[0] - K[3][1] * x[1]) / K[3][3];
    x[4] = (g[4] - K[4][1] * x[1] - K[4][2] * x[2] - K[4][3] * x[3]) / K[4][4];
    x[5] = (g[5] - K[5][0] * x[0] - K[5][2] * x[2] - K[5][3] * x[3] - K[5][4] * x[4]) / K[5][5];
    for (int i = 0; i < 9; i++) {
        double s = 0;
        for (int k = 0; k < 6; k++) s += H[i][k] * x[k];
        delta[i] = s;
    }
    double nto[3][9], W[9], Wi[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, A[3][9], v[9], y[3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 9; k++) s += N[k][i] * S.omega[9 * k + j];
            nto[i][j] = s;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 9; k++) s += nto[i][k] * N[k][j];
            W[3 * i + j] = s;
        }
    inv3_symm(W, Wi);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += -Wi[3 * i + k] * nto[k][j];
            A[i][j] = s;
        }
    for (int k = 0; k < 9; k++) v[k] = delta[k] + r[k];
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int k = 0; k < 9; k++) s += A[i][k] * v[k];
        y[i] = s;
    }
    for (int i = 0; i < 9; i++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s += N[i][k] * y[k];
        delta[i] = delta[i] + s;
    }
}

inline void run_sqp(const Solver& S, const double* r0, double* rh) {
    double r[9], delta[9];
    std::memcpy(r, r0, sizeof(r));
    double dsq = DBL_MAX;
    int step = 0;
    while (dsq > 1e-10 && step++ < 15) {
        sqp_step(S, r, delta);
        for (int k = 0; k < 9; k++) r[k] = r[k] + delta[k];
        dsq = norm_sqr(delta, 9);
    }
    double det_r = det9(r);
    if (det_r < 0) {
        for (int k = 0; k < 9; k++) r[k] = -r[k];
        det_r = -det_r;
    }
    if (det_r > 1.001) nearest_rot(r, rh);
    else std::memcpy(rh, r, sizeof(r));
}

}  // namespace sqp

// PoseSolver::solve's O(1) part from the 39 point sums. npos(rh, t) counts the points with positive
// depth (positiveMajorityDepths, only asked when the centroid's depth is not positive). Returns the
// number of solutions (0: none passed cheirality) or -1 / -2 / -3 for computeOmega's assertions
// (coordinate variance < 1e-5, s_0 < 1e-7, null space above 6); rh / t: the first solution.
template <class NPos>
int sqpnp_from_sums(const double (&S39)[kSqpSums], int n, NPos&& npos, double (&rh_out)[9], double (&t_out)[3]) {
    using namespace sqp;
    Solver S;
    double* om = S.omega;
    double qa[27];
    std::memset(om, 0, sizeof(S.omega));
    std::memset(qa, 0, sizeof(qa));
    auto OM = [&](int i, int j) -> double& { return om[9 * i + j]; };
    auto QA = [&](int i, int j) -> double& { return qa[9 * i + j]; };
    static const int up[24][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}, {0, 6}, {0, 7},
                                  {0, 8}, {1, 7}, {1, 8}, {2, 8}, {3, 6}, {3, 7}, {3, 8}, {4, 7},
                                  {4, 8}, {5, 8}, {6, 6}, {6, 7}, {6, 8}, {7, 7}, {7, 8}, {8, 8}};
    for (int a = 0; a < 24; a++) OM(up[a][0], up[a][1]) = S39[a];
    for (int k = 0; k < 3; k++) {
        QA(0, k) = S39[24 + k];
        QA(0, 6 + k) = S39[27 + k];
        QA(1, 6 + k) = S39[30 + k];
        QA(2, 6 + k) = S39[33 + k];
    }
    const double sx = S39[36], sy = S39[37], sqs = S39[38];
    for (int k = 0; k < 3; k++) {
        QA(1, 3 + k) = QA(0, k);
        QA(2, k) = QA(0, 6 + k);
        QA(2, 3 + k) = QA(1, 6 + k);
    }
    OM(1, 6) = OM(0, 7); OM(2, 6) = OM(0, 8); OM(2, 7) = OM(1, 8);
    OM(4, 6) = OM(3, 7); OM(5, 6) = OM(3, 8); OM(5, 7) = OM(4, 8);
    OM(3, 3) = OM(0, 0); OM(3, 4) = OM(0, 1); OM(3, 5) = OM(0, 2);
    OM(4, 4) = OM(1, 1); OM(4, 5) = OM(1, 2);
    OM(5, 5) = OM(2, 2);
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < i; j++) OM(i, j) = OM(j, i);
    const double dn = (double)n;
    const double Q[9] = {dn, 0, -sx, 0, dn, -sy, -sx, -sy, sqs};
    const double inv_n = 1.0 / dn;
    const double detQ = dn * (dn * sqs - sy * sy - sx * sx);
    if (!(detQ * inv_n * inv_n * inv_n >= 1e-5)) return -1;
    double Qi[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    inv3_symm(Q, Qi);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += -Qi[3 * i + k] * QA(k, j);
            S.p[9 * i + j] = s;
        }
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += QA(k, i) * S.p[9 * k + j];
            OM(i, j) = OM(i, j) + s;
        }
    {
        double At[9][9], Vt[9][9];
        for (int i = 0; i < 9; i++)
            for (int k = 0; k < 9; k++) At[i][k] = OM(k, i);
        jacobi_svd<9, 9>(At, S.s, Vt);
        std::memcpy(S.u, Vt, sizeof(Vt));
    }
    if (!(S.s[0] >= 1e-7)) return -2;
    while (S.s[7 - S.nnull] < 1e-7) S.nnull++;
    if (++S.nnull > 6) return -3;
    for (int k = 0; k < 3; k++) S.mean[k] = S39[24 + k] / dn;

    auto translation = [&](const double* rh, double* t) {
        for (int i = 0; i < 3; i++) {
            double s = 0;
            for (int k = 0; k < 9; k++) s += S.p[9 * i + k] * rh[k];
            t[i] = s;
        }
    };
    double min_err = DBL_MAX;
    auto check = [&](const double* rh, const double* t) {   // checkSolution
        bool ok = rh[6] * S.mean[0] + rh[7] * S.mean[1] + rh[8] * S.mean[2] + t[2] > 0;
        if (!ok) {
            const int pos = npos(rh, t);
            ok = pos >= n - pos;
        }
        if (!ok) return;
        double omr[9], err = 0;
        for (int i = 0; i < 9; i++) {
            double s = 0;
            for (int k = 0; k < 9; k++) s += om[9 * i + k] * rh[k];
            omr[i] = s;
        }
        for (int i = 0; i < 9; i++) err += omr[i] * rh[i];
        auto store = [&](int i) {
            std::memcpy(S.rh[i], rh, sizeof(double) * 9);
            std::memcpy(S.t[i], t, sizeof(double) * 3);
            S.err[i] = err;
        };
        if (std::fabs(min_err - err) > 1e-6) {
            if (min_err > err) {
                min_err = err;
                store(0);
                S.nsol = 1;
            }
            return;
        }
        bool found = false;
        for (int i = 0; i < S.nsol; i++) {
            double d[9];
            for (int k = 0; k < 9; k++) d[k] = S.rh[i][k] - rh[k];
            if (norm_sqr(d, 9) < 1e-10) {
                if (S.err[i] > err) store(i);
                found = true;
                break;
            }
        }
        if (!found && S.nsol < 18) store(S.nsol++);
        if (min_err > err) min_err = err;
    };
    auto try_vector = [&](const double* e) {   // both signs: nearest rotation, SQP, check
        double r[9], rh[9], t[3], ne[9];
        nearest_rot(e, r);
        run_sqp(S, r, rh);
        translation(rh, t);
        check(rh, t);
        for (int k = 0; k < 9; k++) ne[k] = -e[k];
        nearest_rot(ne, r);
        run_sqp(S, r, rh);
        translation(rh, t);
        check(rh, t);
    };
    const int nep = S.nnull > 0 ? S.nnull : 1;
    const double sqrt3 = std::sqrt(3.0);
    for (int i = 9 - nep; i < 9; i++) {
        double e[9];
        for (int k = 0; k < 9; k++) e[k] = sqrt3 * S.u[9 * i + k];
        const double s1 = e[0] * e[0] + e[1] * e[1] + e[2] * e[2], s2 = e[3] * e[3] + e[4] * e[4] + e[5] * e[5],
                     s3 = e[6] * e[6] + e[7] * e[7] + e[8] * e[8];
        const double d12 = e[0] * e[3] + e[1] * e[4] + e[2] * e[5], d13 = e[0] * e[6] + e[1] * e[7] + e[2] * e[8],
                     d23 = e[3] * e[6] + e[4] * e[7] + e[5] * e[8];
        const double oerr =
            (s1 - 1) * (s1 - 1) + (s2 - 1) * (s2 - 1) + (s3 - 1) * (s3 - 1) + 2 * (d12 * d12 + d13 * d13 + d23 * d23);
        if (oerr < 1e-8) {   // already a rotation up to sign: SQP skipped
            double rh[9], t[3];
            const double de = det9(e);
            for (int k = 0; k < 9; k++) rh[k] = de * e[k];
            translation(rh, t);
            check(rh, t);
        } else {
            try_vector(e);
        }
    }
    for (int c = 1; min_err > 3 * S.s[9 - nep - c] && 9 - nep - c > 0; c++) try_vector(S.u + 9 * (9 - nep - c));
    if (S.nsol > 0) {
        std::memcpy(rh_out, S.rh[0], sizeof(rh_out));
        std::memcpy(t_out, S.t[0], sizeof(t_out));
    }
    return S.nsol;
}

}  // namespace mcv
