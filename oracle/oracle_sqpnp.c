/*
 * oracle_sqpnp.c — CPU restatement of SQPnP (Terzakis & Lourakis, "A Consistently Fast and Globally
 * Optimal Solution to the Perspective-n-Point Problem", ECCV 2020) as OpenCV 4.x's calib3d
 * sqpnp.cpp computes it (cv::sqpnp::PoseSolver: the build without Eigen, so Omega's null space comes
 * from cv::SVD = JacobiSVDImpl_; nearest rotations by FOAM with the SVD fallback for |det| < 1e-4),
 * behind solvePnP(SOLVEPNP_SQPNP) on undistortPoints' normalised coordinates: the solverKind 6 path of
 * the reference's cvSolvePnP (/root/reference/src/MiniCVNative/MiniCVNative.cpp:72-74, :82).
 * TEST INFRASTRUCTURE ONLY (rules: oracle.c header).
 *
 * OpenCV is not vendored in /root/reference and not installed here [ext]: this restates the published
 * algorithm and the operation order of that file as written (Matx products summed from 0 in index
 * order, cv::norm through normL2Sqr's four-way unrolled loop); parity with OpenCV's own bits is
 * unpinned. The solution is pinned by exact geometry instead (noise-free correspondences of a known
 * pose give that pose back; the global minimum of the object-space error is checked against
 * perturbed poses: tests/test_oracle_pnp.py). The GPU path (minicv_amd/csrc/sqpnp.h over the device
 * sums of ransac_pnp.hip) must equal this file bit for bit.
 *
 * The 39 sums over the points run in blocks of SQP_BLOCK consecutive points (each block from 0 in
 * point order, then the block sums in order): the sequential order of computeOmega when n <= 1024.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <float.h>
#include "oracle_int.h"

#define SQP_BLOCK 1024
#define SQP_NSUM 39

/* The per-point terms of computeOmega, in accumulator order: omega's upper-triangle blocks (X2 .. Z2;
 * -x X2 ..; -y X2 ..; |x|^2 X2 ..), qa_sum's row 0 (X, Y, Z = sum_obj too), rows 0 / 1 / 2 of its
 * right block (-x X ..; -y X ..; |x|^2 X ..), sum_img and the sum of |x|^2. */
void orc_sqpnp_terms(double x, double y, double X, double Y, double Z, double* t) {
    const double sq = x * x + y * y;
    const double X2 = X * X, XY = X * Y, XZ = X * Z, Y2 = Y * Y, YZ = Y * Z, Z2 = Z * Z;
    const double q6[6] = {X2, XY, XZ, Y2, YZ, Z2};
    for (int k = 0; k < 6; k++) {
        t[k] = q6[k];
        t[6 + k] = -x * q6[k];
        t[12 + k] = -y * q6[k];
        t[18 + k] = sq * q6[k];
    }
    const double p3[3] = {X, Y, Z};
    for (int k = 0; k < 3; k++) {
        t[24 + k] = p3[k];
        t[27 + k] = -x * p3[k];
        t[30 + k] = -y * p3[k];
        t[33 + k] = sq * p3[k];
    }
    t[36] = x;
    t[37] = y;
    t[38] = sq;
}

/* normL2Sqr<double, double> (core base.hpp, CV_ENABLE_UNROLLED): what cv::norm of a Matx sums. */
static double cv_norm_sqr(const double* a, int n) {
    double s = 0;
    int i = 0;
    for (; i <= n - 4; i += 4) s += a[i] * a[i] + a[i + 1] * a[i + 1] + a[i + 2] * a[i + 2] + a[i + 3] * a[i + 3];
    for (; i < n; i++) s += a[i] * a[i];
    return s;
}

static double det9(const double* e) {
    return e[0] * e[4] * e[8] + e[1] * e[5] * e[6] + e[2] * e[3] * e[7] - e[6] * e[4] * e[2] - e[7] * e[5] * e[0] -
           e[8] * e[3] * e[1];
}

/* analyticalInverse3x3Symm: reads the lower triangle; below the threshold Qinv is left as it is. */
static int inv3_symm(const double* Q, double* Qi) {
    const double a = Q[0], b = Q[3], d = Q[4], c = Q[6], e = Q[7], f = Q[8];
    const double t2 = e * e, t4 = a * d, t7 = b * b, t9 = b * c, t12 = c * c;
    const double det = -t4 * f + a * t2 + t7 * f - 2.0 * t9 * e + t12 * d;
    if (fabs(det) < 1e-8) return 0;
    const double t15 = 1.0 / det;
    const double t20 = (-b * f + c * e) * t15, t24 = (b * e - c * d) * t15, t30 = (a * e - t9) * t15;
    Qi[0] = (-d * f + t2) * t15;
    Qi[1] = Qi[3] = -t20;
    Qi[2] = Qi[6] = -t24;
    Qi[4] = -(a * f - t12) * t15;
    Qi[5] = Qi[7] = t30;
    Qi[8] = -(t4 - t7) * t15;
    return 1;
}

/* cv::determinant of a 3 x 3 (lapack.cpp) */
static double cv_det3(const double* M) {
    return M[0] * (M[4] * M[8] - M[5] * M[7]) - M[1] * (M[3] * M[8] - M[5] * M[6]) +
           M[2] * (M[3] * M[7] - M[4] * M[6]);
}

/* nearestRotationMatrixSVD: U diag(1, 1, det U det Vt) Vt of cv::SVD(e33, FULL_UV). */
static void nearest_rot_svd(const double* e, double* r) {
    double At[9], w[3], Vt[9], U[9], D[9], T[9];
    for (int i = 0; i < 3; i++)
        for (int k = 0; k < 3; k++) At[3 * i + k] = e[3 * k + i];
    orc_jsvd(At, w, Vt, 3, 3, 3);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) U[3 * i + j] = At[3 * j + i];
    const double detuv = cv_det3(U) * cv_det3(Vt);
    memset(D, 0, sizeof(D));
    D[0] = 1; D[4] = 1; D[8] = detuv;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += U[3 * i + k] * D[3 * k + j];
            T[3 * i + j] = s;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += T[3 * i + k] * Vt[3 * k + j];
            r[3 * i + j] = s;
        }
}

/* nearestRotationMatrixFOAM (Lourakis, ICPR 2016): lambda_max by Newton on FOAM's characteristic
 * polynomial, then R = ((l^2 + |e|^2) e + 2 l adj(e)^T - 2 e e^T e) / (l (l^2 - |e|^2) - 2 det e). */
static void nearest_rot(const double* e, double* r) {
    const double det_e = e[0] * e[4] * e[8] - e[0] * e[5] * e[7] - e[1] * e[3] * e[8] + e[2] * e[3] * e[7] +
                         e[1] * e[6] * e[5] - e[2] * e[6] * e[4];
    if (fabs(det_e) < 1e-4) {
        nearest_rot_svd(e, r);
        return;
    }
    double adj[9];
    adj[0] = e[4] * e[8] - e[5] * e[7]; adj[1] = e[2] * e[7] - e[1] * e[8]; adj[2] = e[1] * e[5] - e[2] * e[4];
    adj[3] = e[5] * e[6] - e[3] * e[8]; adj[4] = e[0] * e[8] - e[2] * e[6]; adj[5] = e[2] * e[3] - e[0] * e[5];
    adj[6] = e[3] * e[7] - e[4] * e[6]; adj[7] = e[1] * e[6] - e[0] * e[7]; adj[8] = e[0] * e[4] - e[1] * e[3];
    double e_sq = e[0] * e[0], adj_sq = adj[0] * adj[0];
    for (int k = 1; k < 9; k++) {
        e_sq = e_sq + e[k] * e[k];
        adj_sq = adj_sq + adj[k] * adj[k];
    }
    double l = 2.0, lprev = 0.0;
    for (int i = 200; fabs(l - lprev) > 1e-12 * fabs(lprev) && i > 0; --i) {
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

/* computeRowAndNullspace: the Jacobian row space H (9 x 6, Gram-Schmidt of the six constraint
 * gradients in the order |r1|^2, |r2|^2, |r3|^2, r1.r2, r2.r3, r1.r3), K = J H (lower triangular) and
 * a null-space basis N (9 x 3) from three well-spread columns of I - H H^T (norm threshold 0.1). */
static void row_and_nullspace(const double* r, double H[9][6], double N[9][3], double K[6][6]) {
    memset(H, 0, sizeof(double) * 54);
    memset(K, 0, sizeof(double) * 36);
    const double n1 = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    const double in1 = n1 > 1e-5 ? 1.0 / n1 : 0.0;
    H[0][0] = r[0] * in1; H[1][0] = r[1] * in1; H[2][0] = r[2] * in1;
    K[0][0] = 2 * n1;
    const double n2 = sqrt(r[3] * r[3] + r[4] * r[4] + r[5] * r[5]);
    const double in2 = n2 > 1e-5 ? 1.0 / n2 : 0.0;
    H[3][1] = r[3] * in2; H[4][1] = r[4] * in2; H[5][1] = r[5] * in2;
    K[1][1] = 2 * n2;
    const double n3 = sqrt(r[6] * r[6] + r[7] * r[7] + r[8] * r[8]);
    const double in3 = n3 > 1e-5 ? 1.0 / n3 : 0.0;
    H[6][2] = r[6] * in3; H[7][2] = r[7] * in3; H[8][2] = r[8] * in3;
    K[2][2] = 2 * n3;
    /* q4: j4 = (r2, r1, 0) */
    const double d41 = r[3] * H[0][0] + r[4] * H[1][0] + r[5] * H[2][0];
    const double d42 = r[0] * H[3][1] + r[1] * H[4][1] + r[2] * H[5][1];
    H[0][3] = r[3] - d41 * H[0][0]; H[1][3] = r[4] - d41 * H[1][0]; H[2][3] = r[5] - d41 * H[2][0];
    H[3][3] = r[0] - d42 * H[3][1]; H[4][3] = r[1] - d42 * H[4][1]; H[5][3] = r[2] - d42 * H[5][1];
    {
        double s = 0;
        for (int i = 0; i < 6; i++) s += H[i][3] * H[i][3];
        const double in4 = 1.0 / sqrt(s);
        for (int i = 0; i < 6; i++) H[i][3] *= in4;
    }
    K[3][0] = r[3] * H[0][0] + r[4] * H[1][0] + r[5] * H[2][0];
    K[3][1] = r[0] * H[3][1] + r[1] * H[4][1] + r[2] * H[5][1];
    K[3][3] = r[3] * H[0][3] + r[4] * H[1][3] + r[5] * H[2][3] + r[0] * H[3][3] + r[1] * H[4][3] + r[2] * H[5][3];
    /* q5: j5 = (0, r3, r2) */
    const double d52 = r[6] * H[3][1] + r[7] * H[4][1] + r[8] * H[5][1];
    const double d53 = r[3] * H[6][2] + r[4] * H[7][2] + r[5] * H[8][2];
    const double d54 = r[6] * H[3][3] + r[7] * H[4][3] + r[8] * H[5][3];
    H[0][4] = -d54 * H[0][3]; H[1][4] = -d54 * H[1][3]; H[2][4] = -d54 * H[2][3];
    H[3][4] = r[6] - d52 * H[3][1] - d54 * H[3][3];
    H[4][4] = r[7] - d52 * H[4][1] - d54 * H[4][3];
    H[5][4] = r[8] - d52 * H[5][1] - d54 * H[5][3];
    H[6][4] = r[3] - d53 * H[6][2]; H[7][4] = r[4] - d53 * H[7][2]; H[8][4] = r[5] - d53 * H[8][2];
    {
        double s = 0;
        for (int i = 0; i < 9; i++) s += H[i][4] * H[i][4];
        const double in5 = 1.0 / sqrt(s);
        for (int i = 0; i < 9; i++) H[i][4] *= in5;
    }
    K[4][1] = r[6] * H[3][1] + r[7] * H[4][1] + r[8] * H[5][1];
    K[4][2] = r[3] * H[6][2] + r[4] * H[7][2] + r[5] * H[8][2];
    K[4][3] = r[6] * H[3][3] + r[7] * H[4][3] + r[8] * H[5][3];
    K[4][4] = r[6] * H[3][4] + r[7] * H[4][4] + r[8] * H[5][4] + r[3] * H[6][4] + r[4] * H[7][4] + r[5] * H[8][4];
    /* q6: j6 = (r3, 0, r1) */
    const double d61 = r[6] * H[0][0] + r[7] * H[1][0] + r[8] * H[2][0];
    const double d63 = r[0] * H[6][2] + r[1] * H[7][2] + r[2] * H[8][2];
    const double d64 = r[6] * H[0][3] + r[7] * H[1][3] + r[8] * H[2][3];
    const double d65 = r[6] * H[0][4] + r[7] * H[1][4] + r[8] * H[2][4] + r[0] * H[6][4] + r[1] * H[7][4] + r[2] * H[8][4];
    H[0][5] = r[6] - d61 * H[0][0] - d64 * H[0][3] - d65 * H[0][4];
    H[1][5] = r[7] - d61 * H[1][0] - d64 * H[1][3] - d65 * H[1][4];
    H[2][5] = r[8] - d61 * H[2][0] - d64 * H[2][3] - d65 * H[2][4];
    H[3][5] = -d64 * H[3][3] - d65 * H[3][4];
    H[4][5] = -d64 * H[4][3] - d65 * H[4][4];
    H[5][5] = -d64 * H[5][3] - d65 * H[5][4];
    H[6][5] = r[0] - d63 * H[6][2] - d65 * H[6][4];
    H[7][5] = r[1] - d63 * H[7][2] - d65 * H[7][4];
    H[8][5] = r[2] - d63 * H[8][2] - d65 * H[8][4];
    {
        double s = 0;
        for (int i = 0; i < 9; i++) s += H[i][5] * H[i][5];
        const double in6 = 1.0 / sqrt(s);
        for (int i = 0; i < 9; i++) H[i][5] *= in6;
    }
    K[5][0] = r[6] * H[0][0] + r[7] * H[1][0] + r[8] * H[2][0];
    K[5][2] = r[0] * H[6][2] + r[1] * H[7][2] + r[2] * H[8][2];
    K[5][3] = r[6] * H[0][3] + r[7] * H[1][3] + r[8] * H[2][3];
    K[5][4] = r[6] * H[0][4] + r[7] * H[1][4] + r[8] * H[2][4] + r[0] * H[6][4] + r[1] * H[7][4] + r[2] * H[8][4];
    K[5][5] = r[6] * H[0][5] + r[7] * H[1][5] + r[8] * H[2][5] + r[0] * H[6][5] + r[1] * H[7][5] + r[2] * H[8][5];

    /* null-space projector Pn = I - H H^T, columns as rows of Pc (Pn is the column source) */
    double Pc[9][9];
    for (int i = 0; i < 9; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 6; k++) s += H[i][k] * H[j][k];
            Pc[j][i] = (i == j ? 1.0 : 0.0) - s;
        }
    const double thr = 0.1;
    int i1 = 0, i2 = 0, i3 = 0;
    double max1 = DBL_MIN, min12 = DBL_MAX, min123 = DBL_MAX, cn[9];
    for (int i = 0; i < 9; i++) {
        cn[i] = sqrt(cv_norm_sqr(Pc[i], 9));
        if (cn[i] >= thr && max1 < cn[i]) {
            max1 = cn[i];
            i1 = i;
        }
    }
    const double* v1 = Pc[i1];
    const double s1 = 1.0 / max1;
    double n0[9], nn1[9], nn2[9];
    for (int k = 0; k < 9; k++) n0[k] = v1[k] * s1;
    cn[i1] = -1.0;
    for (int i = 0; i < 9; i++)
        if (cn[i] >= thr) {
            double dd = 0;
            for (int k = 0; k < 9; k++) dd += Pc[i][k] * v1[k];
            const double c1 = fabs(dd / cn[i]);
            if (c1 <= min12) {
                i2 = i;
                min12 = c1;
            }
        }
    const double* v2 = Pc[i2];
    {
        double dd = 0;
        for (int k = 0; k < 9; k++) dd += v2[k] * n0[k];
        for (int k = 0; k < 9; k++) nn1[k] = v2[k] - dd * n0[k];
        const double s = 1.0 / sqrt(cv_norm_sqr(nn1, 9));
        for (int k = 0; k < 9; k++) nn1[k] *= s;
    }
    cn[i2] = -1.0;
    for (int i = 0; i < 9; i++)
        if (cn[i] >= thr) {
            const double inv = 1.0 / cn[i];
            double d1 = 0, d2 = 0;
            for (int k = 0; k < 9; k++) d1 += Pc[i][k] * v1[k];
            for (int k = 0; k < 9; k++) d2 += Pc[i][k] * v2[k];
            const double c1 = fabs(d1 * inv), c2 = fabs(d2 * inv);
            if (c1 + c2 <= min123) {
                i3 = i;
                min123 = c1 + c2;
            }
        }
    const double* v3 = Pc[i3];
    {
        double a1 = 0, a0 = 0;
        for (int k = 0; k < 9; k++) a1 += v3[k] * nn1[k];
        for (int k = 0; k < 9; k++) a0 += v3[k] * n0[k];
        for (int k = 0; k < 9; k++) nn2[k] = v3[k] - a1 * nn1[k] - a0 * n0[k];
        const double s = 1.0 / sqrt(cv_norm_sqr(nn2, 9));
        for (int k = 0; k < 9; k++) nn2[k] *= s;
    }
    for (int k = 0; k < 9; k++) {
        N[k][0] = n0[k];
        N[k][1] = nn1[k];
        N[k][2] = nn2[k];
    }
}

typedef struct {
    double omega[81], p[27], s[9], u[81];   /* u: column c of u_ at u[9 c ..] (rows of cv::SVD's vt) */
    double mean[3];
    int nnull;
    double rh[18][9], t[18][3], err[18];
    int nsol;
    const double* world;
    int n;
} Sqp;

/* solveSQPSystem: delta = H x (K x = g, forward substitution) + N y, y minimising the linearised
 * objective over the null space. */
static void sqp_step(const Sqp* S, const double* r, double* delta) {
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
    double nto[3][9], W[9], Wi[9], A[3][9], v[9], y[3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 9; j++) {
            double s = 0;
            for (int k = 0; k < 9; k++) s += N[k][i] * S->omega[9 * k + j];
            nto[i][j] = s;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 9; k++) s += nto[i][k] * N[k][j];
            W[3 * i + j] = s;
        }
    memset(Wi, 0, sizeof(Wi));
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

static void run_sqp(const Sqp* S, const double* r0, double* rh) {
    double r[9], delta[9];
    memcpy(r, r0, sizeof(r));
    double dsq = DBL_MAX;
    int step = 0;
    while (dsq > 1e-10 && step++ < 15) {
        sqp_step(S, r, delta);
        for (int k = 0; k < 9; k++) r[k] = r[k] + delta[k];
        dsq = cv_norm_sqr(delta, 9);
    }
    double det_r = det9(r);
    if (det_r < 0) {
        for (int k = 0; k < 9; k++) r[k] = -r[k];
        det_r = -det_r;
    }
    if (det_r > 1.001) nearest_rot(r, rh);
    else memcpy(rh, r, sizeof(r));
}

static void translation(const Sqp* S, const double* rh, double* t) {
    for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int k = 0; k < 9; k++) s += S->p[9 * i + k] * rh[k];
        t[i] = s;
    }
}

/* checkSolution: cheirality (centroid depth, else the majority of the points), then the solution
 * list keyed by the squared error r^T Omega r. */
static void check_solution(Sqp* S, const double* rh, const double* t, double* min_err) {
    int ok = rh[6] * S->mean[0] + rh[7] * S->mean[1] + rh[8] * S->mean[2] + t[2] > 0;
    if (!ok) {
        int npos = 0, nneg = 0;
        for (int i = 0; i < S->n; i++) {
            const double* P = S->world + 3 * (size_t)i;
            if (rh[6] * P[0] + rh[7] * P[1] + rh[8] * P[2] + t[2] > 0) ++npos;
            else ++nneg;
        }
        ok = npos >= nneg;
    }
    if (!ok) return;
    double om[9], err = 0;
    for (int i = 0; i < 9; i++) {
        double s = 0;
        for (int k = 0; k < 9; k++) s += S->omega[9 * i + k] * rh[k];
        om[i] = s;
    }
    for (int i = 0; i < 9; i++) err += om[i] * rh[i];
    if (fabs(*min_err - err) > 1e-6) {
        if (*min_err > err) {
            *min_err = err;
            memcpy(S->rh[0], rh, sizeof(double) * 9);
            memcpy(S->t[0], t, sizeof(double) * 3);
            S->err[0] = err;
            S->nsol = 1;
        }
        return;
    }
    int found = 0;
    for (int i = 0; i < S->nsol; i++) {
        double d[9];
        for (int k = 0; k < 9; k++) d[k] = S->rh[i][k] - rh[k];
        if (cv_norm_sqr(d, 9) < 1e-10) {
            if (S->err[i] > err) {
                memcpy(S->rh[i], rh, sizeof(double) * 9);
                memcpy(S->t[i], t, sizeof(double) * 3);
                S->err[i] = err;
            }
            found = 1;
            break;
        }
    }
    if (!found && S->nsol < 18) {
        memcpy(S->rh[S->nsol], rh, sizeof(double) * 9);
        memcpy(S->t[S->nsol], t, sizeof(double) * 3);
        S->err[S->nsol] = err;
        S->nsol++;
    }
    if (*min_err > err) *min_err = err;
}

static void try_vector(Sqp* S, const double* e, double* min_err) {
    double r[9], rh[9], t[3], ne[9];
    nearest_rot(e, r);
    run_sqp(S, r, rh);
    translation(S, rh, t);
    check_solution(S, rh, t, min_err);
    for (int k = 0; k < 9; k++) ne[k] = -e[k];
    nearest_rot(ne, r);
    run_sqp(S, r, rh);
    translation(S, rh, t);
    check_solution(S, rh, t, min_err);
}

/* The O(1) part of PoseSolver::solve from the 39 point sums: Omega / P assembly, the SVD and the
 * solution search. Returns the number of solutions (0: none with positive depth), or -1 / -2 / -3
 * for computeOmega's assertions (coordinate variance, s_0, null-space dimension). rh / t: the first
 * solution. */
int orc_sqpnp_from_sums(const double* S39, int n, const double* world, double* rh_out, double* t_out) {
    Sqp* S = (Sqp*)calloc(1, sizeof(Sqp));
    S->world = world;
    S->n = n;
    double* om = S->omega;
    double qa[27];
    memset(qa, 0, sizeof(qa));
#define OM(i, j) om[9 * (i) + (j)]
#define QA(i, j) qa[9 * (i) + (j)]
    static const int up[24][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}, {0, 6}, {0, 7}, {0, 8}, {1, 7}, {1, 8},
                                  {2, 8}, {3, 6}, {3, 7}, {3, 8}, {4, 7}, {4, 8}, {5, 8}, {6, 6}, {6, 7}, {6, 8}, {7, 7},
                                  {7, 8}, {8, 8}};
    for (int a = 0; a < 24; a++) OM(up[a][0], up[a][1]) = S39[a];
    for (int k = 0; k < 3; k++) {
        QA(0, k) = S39[24 + k];
        QA(0, 6 + k) = S39[27 + k];
        QA(1, 6 + k) = S39[30 + k];
        QA(2, 6 + k) = S39[33 + k];
    }
    const double sx = S39[36], sy = S39[37], sqs = S39[38];
    QA(1, 3) = QA(0, 0); QA(1, 4) = QA(0, 1); QA(1, 5) = QA(0, 2);
    QA(2, 0) = QA(0, 6); QA(2, 1) = QA(0, 7); QA(2, 2) = QA(0, 8);
    QA(2, 3) = QA(1, 6); QA(2, 4) = QA(1, 7); QA(2, 5) = QA(1, 8);
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
    const double var = detQ * inv_n * inv_n * inv_n;
    int ret = 0;
    if (!(var >= 1e-5)) {
        ret = -1;
        goto done;
    }
    {
        double Qi[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        inv3_symm(Q, Qi);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 9; j++) {
                double s = 0;
                for (int k = 0; k < 3; k++) s += -Qi[3 * i + k] * QA(k, j);
                S->p[9 * i + j] = s;
            }
        for (int i = 0; i < 9; i++)
            for (int j = 0; j < 9; j++) {
                double s = 0;
                for (int k = 0; k < 3; k++) s += QA(k, i) * S->p[9 * k + j];
                OM(i, j) = OM(i, j) + s;
            }
        double At[81], Vt[81];
        for (int i = 0; i < 9; i++)
            for (int k = 0; k < 9; k++) At[9 * i + k] = OM(k, i);
        orc_jsvd(At, S->s, Vt, 9, 9, 9);
        memcpy(S->u, Vt, sizeof(Vt));
    }
    if (!(S->s[0] >= 1e-7)) {
        ret = -2;
        goto done;
    }
    S->nnull = -1;
    while (S->s[7 - S->nnull] < 1e-7) S->nnull++;
    if (++S->nnull > 6) {
        ret = -3;
        goto done;
    }
    for (int k = 0; k < 3; k++) S->mean[k] = S39[24 + k] / dn;
    {
        double min_err = DBL_MAX;
        const int nep = S->nnull > 0 ? S->nnull : 1;
        const double sqrt3 = sqrt(3.0);
        for (int i = 9 - nep; i < 9; i++) {
            double e[9];
            for (int k = 0; k < 9; k++) e[k] = sqrt3 * S->u[9 * i + k];
            const double s1 = e[0] * e[0] + e[1] * e[1] + e[2] * e[2], s2 = e[3] * e[3] + e[4] * e[4] + e[5] * e[5],
                         s3 = e[6] * e[6] + e[7] * e[7] + e[8] * e[8];
            const double d12 = e[0] * e[3] + e[1] * e[4] + e[2] * e[5], d13 = e[0] * e[6] + e[1] * e[7] + e[2] * e[8],
                         d23 = e[3] * e[6] + e[4] * e[7] + e[5] * e[8];
            const double oerr = (s1 - 1) * (s1 - 1) + (s2 - 1) * (s2 - 1) + (s3 - 1) * (s3 - 1) +
                                2 * (d12 * d12 + d13 * d13 + d23 * d23);
            if (oerr < 1e-8) {
                double rh[9], t[3];
                const double de = det9(e);
                for (int k = 0; k < 9; k++) rh[k] = de * e[k];
                translation(S, rh, t);
                check_solution(S, rh, t, &min_err);
            } else {
                try_vector(S, e, &min_err);
            }
        }
        int c = 1;
        while (min_err > 3 * S->s[9 - nep - c] && 9 - nep - c > 0) {
            try_vector(S, S->u + 9 * (9 - nep - c), &min_err);
            c++;
        }
    }
    ret = S->nsol;
    if (ret > 0) {
        memcpy(rh_out, S->rh[0], sizeof(double) * 9);
        memcpy(t_out, S->t[0], sizeof(double) * 3);
    }
done:
#undef OM
#undef QA
    free(S);
    return ret;
}

/* solvePnP(SOLVEPNP_SQPNP) on double inputs: undistortPoints (normalised, double), the blocked point
 * sums and the solve. Returns the solver's code (> 0: the first solution's R in rh9, t in t3). */
int orc_sqpnp_pose(const double* img, const double* world, int n, const double* cam8, double* rh9, double* t3) {
    double S39[SQP_NSUM], part[SQP_NSUM], t[SQP_NSUM];
    memset(S39, 0, sizeof(S39));
    for (int b0 = 0; b0 < n; b0 += SQP_BLOCK) {
        const int b1 = b0 + SQP_BLOCK < n ? b0 + SQP_BLOCK : n;
        memset(part, 0, sizeof(part));
        for (int i = b0; i < b1; i++) {
            double x, y;
            orc_undistort(cam8, img[2 * i], img[2 * i + 1], &x, &y);
            orc_sqpnp_terms(x, y, world[3 * i], world[3 * i + 1], world[3 * i + 2], t);
            for (int a = 0; a < SQP_NSUM; a++) part[a] += t[a];
        }
        for (int a = 0; a < SQP_NSUM; a++) S39[a] += part[a];
    }
    return orc_sqpnp_from_sums(S39, n, world, rh9, t3);
}

/* ... and Rodrigues: the cvSolvePnP kind 6 answer (rvec, tvec). */
int orc_sqpnp(const double* img, const double* world, int n, const double* cam8, double* rvec, double* tvec) {
    double rh[9], tt[3];
    const int r = orc_sqpnp_pose(img, world, n, cam8, rh, tt);
    if (r > 0) {
        orc_rodrigues_inv(rh, rvec);
        memcpy(tvec, tt, sizeof(tt));
    }
    return r;
}
