// linalg.h — small dense fp64 linear algebra for the host side of the shim (n <= 9):
// cyclic Jacobi eigen-decomposition (what cv::eigen does for symmetric double matrices) and the
// eigen-based solve / invert used by the Levenberg-Marquardt refine (cv::solve / cv::invert with
// DECOMP_EIG). These run once per call on 8x8 / 9x9 matrices; the O(N) work that feeds them runs
// on the GPU (reduce.h).
#pragma once

#include <cmath>
#include <cfloat>
#include <algorithm>

namespace mcv {

// Symmetric A (n x n, row-major, destroyed). Eigenvalues descending in w[n]; eigenvectors as the
// ROWS of V (V[i*n + j] = component j of eigenvector i), matching cv::eigen's layout.
inline void jacobi_eigen(double* A, int n, double* w, double* V) {
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0, diag = 0;
        for (int i = 0; i < n; ++i) {
            diag += A[i * n + i] * A[i * n + i];
            for (int j = i + 1; j < n; ++j) off += A[i * n + j] * A[i * n + j];
        }
        if (off <= DBL_MIN || off <= diag * 1e-32) break;
        for (int p = 0; p < n; ++p) {
            for (int q = p + 1; q < n; ++q) {
                const double apq = A[p * n + q];
                if (apq == 0) continue;
                const double app = A[p * n + p], aqq = A[q * n + q];
                const double theta = (aqq - app) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {   // A <- J^T A J
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {   // rows of V are eigenvectors
                    const double vpk = V[p * n + k], vqk = V[q * n + k];
                    V[p * n + k] = c * vpk - s * vqk;
                    V[q * n + k] = s * vpk + c * vqk;
                }
            }
        }
    }
    for (int i = 0; i < n; ++i) w[i] = A[i * n + i];
    // selection sort, descending (stable for equal values)
    for (int i = 0; i < n - 1; ++i) {
        int m = i;
        for (int j = i + 1; j < n; ++j)
            if (w[j] > w[m]) m = j;
        if (m != i) {
            std::swap(w[i], w[m]);
            for (int k = 0; k < n; ++k) std::swap(V[i * n + k], V[m * n + k]);
        }
    }
}

// x = pinv(A) b for symmetric A via its eigen-decomposition (cv::solve(..., DECOMP_EIG)).
inline void eig_solve(const double* A, int n, const double* b, double* x) {
    double M[81], w[9], V[81];
    for (int i = 0; i < n * n; ++i) M[i] = A[i];
    jacobi_eigen(M, n, w, V);
    double wmax = 0;
    for (int i = 0; i < n; ++i) wmax = std::max(wmax, std::fabs(w[i]));
    const double thr = wmax * n * DBL_EPSILON;
    for (int j = 0; j < n; ++j) x[j] = 0;
    for (int i = 0; i < n; ++i) {
        if (std::fabs(w[i]) <= thr) continue;
        double d = 0;
        for (int k = 0; k < n; ++k) d += V[i * n + k] * b[k];
        d /= w[i];
        for (int j = 0; j < n; ++j) x[j] += d * V[i * n + j];
    }
}

// Ainv = pinv(A) for symmetric A (cv::invert(..., DECOMP_EIG)).
inline void eig_invert(const double* A, int n, double* Ainv) {
    double M[81], w[9], V[81];
    for (int i = 0; i < n * n; ++i) M[i] = A[i];
    jacobi_eigen(M, n, w, V);
    double wmax = 0;
    for (int i = 0; i < n; ++i) wmax = std::max(wmax, std::fabs(w[i]));
    const double thr = wmax * n * DBL_EPSILON;
    for (int i = 0; i < n * n; ++i) Ainv[i] = 0;
    for (int e = 0; e < n; ++e) {
        if (std::fabs(w[e]) <= thr) continue;
        const double iw = 1.0 / w[e];
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) Ainv[i * n + j] += V[e * n + i] * iw * V[e * n + j];
    }
}

}  // namespace mcv
