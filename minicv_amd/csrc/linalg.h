// linalg.h — small dense fp64 linear algebra for the host side of the shim (n <= 9):
// cv::eigen's JacobiImpl_ restated (OpenCV 4.x core lapack.cpp [ext]) and the eigen-based solve /
// invert used by the Levenberg-Marquardt refine (cv::solve / cv::invert with DECOMP_EIG, SVBkSb). These run once per call on 8x8 / 9x9 matrices; the O(N) work that feeds them runs
// on the GPU (reduce.h).
#pragma once

#include <cmath>
#include <cfloat>
#include <algorithm>

namespace mcv {

// lapack.cpp's hypot template (the one JacobiImpl_ calls): the larger magnitude times
// sqrt(1 + ratio^2).
inline double cv_hypot_d(double a, double b) {
    a = std::fabs(a);
    b = std::fabs(b);
    if (a > b) {
        b /= a;
        return a * std::sqrt(1 + b * b);
    }
    if (b > 0) {
        a /= b;
        return b * std::sqrt(1 + a * a);
    }
    return 0;
}

// cv::eigen for a symmetric double matrix = hal::Jacobi = JacobiImpl_<double> (OpenCV 4.x core
// lapack.cpp) [ext, restated]: classical Jacobi with the pivot found through per-row (indR) and
// per-column (indC) maxima of the strict upper triangle (first maximum on ties), stop when the
// pivot |p| <= DBL_EPSILON or after n*n*30 rotations, W = the running diagonal, V rows = the
// eigenvectors, then a selection sort to descending eigenvalues. A (n x n, row-major) is destroyed.
inline void jacobi_eigen(double* A, int n, double* W, double* V) {
    const double eps = DBL_EPSILON;
    int indR[9], indC[9];
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) V[i * n + j] = 0.0;
        V[i * n + i] = 1.0;
    }
    double mv = 0;
    int i, k, m;
    for (k = 0; k < n; ++k) {
        W[k] = A[(n + 1) * k];
        if (k < n - 1) {
            for (m = k + 1, mv = std::fabs(A[n * k + m]), i = k + 2; i < n; ++i) {
                const double val = std::fabs(A[n * k + i]);
                if (mv < val) mv = val, m = i;
            }
            indR[k] = m;
        }
        if (k > 0) {
            for (m = 0, mv = std::fabs(A[k]), i = 1; i < k; ++i) {
                const double val = std::fabs(A[n * i + k]);
                if (mv < val) mv = val, m = i;
            }
            indC[k] = m;
        }
    }
    const int maxIters = n * n * 30;
    if (n > 1)
        for (int iters = 0; iters < maxIters; ++iters) {
            // pivot (k, l)
            for (k = 0, mv = std::fabs(A[indR[0]]), i = 1; i < n - 1; ++i) {
                const double val = std::fabs(A[n * i + indR[i]]);
                if (mv < val) mv = val, k = i;
            }
            int l = indR[k];
            for (i = 1; i < n; ++i) {
                const double val = std::fabs(A[n * indC[i] + i]);
                if (mv < val) mv = val, k = indC[i], l = i;
            }
            const double p = A[n * k + l];
            if (std::fabs(p) <= eps) break;
            const double y = (W[l] - W[k]) * 0.5;
            double t = std::fabs(y) + cv_hypot_d(p, y);
            double sn = cv_hypot_d(p, t);
            const double c = t / sn;
            sn = p / sn;
            t = (p / t) * p;
            if (y < 0) sn = -sn, t = -t;
            A[n * k + l] = 0;
            W[k] -= t;
            W[l] += t;
            auto rot = [&](double& v0, double& v1) {
                const double a0 = v0, b0 = v1;
                v0 = a0 * c - b0 * sn;
                v1 = a0 * sn + b0 * c;
            };
            for (i = 0; i < k; ++i) rot(A[n * i + k], A[n * i + l]);
            for (i = k + 1; i < l; ++i) rot(A[n * k + i], A[n * i + l]);
            for (i = l + 1; i < n; ++i) rot(A[n * k + i], A[n * l + i]);
            for (i = 0; i < n; ++i) rot(V[n * k + i], V[n * l + i]);
            for (int j = 0; j < 2; ++j) {
                const int idx = j == 0 ? k : l;
                if (idx < n - 1) {
                    for (m = idx + 1, mv = std::fabs(A[n * idx + m]), i = idx + 2; i < n; ++i) {
                        const double val = std::fabs(A[n * idx + i]);
                        if (mv < val) mv = val, m = i;
                    }
                    indR[idx] = m;
                }
                if (idx > 0) {
                    for (m = 0, mv = std::fabs(A[idx]), i = 1; i < idx; ++i) {
                        const double val = std::fabs(A[n * i + idx]);
                        if (mv < val) mv = val, m = i;
                    }
                    indC[idx] = m;
                }
            }
        }
    for (k = 0; k < n - 1; ++k) {   // descending
        m = k;
        for (i = k + 1; i < n; ++i)
            if (W[m] < W[i]) m = i;
        if (k != m) {
            std::swap(W[m], W[k]);
            for (i = 0; i < n; ++i) std::swap(V[n * m + i], V[n * k + i]);
        }
    }
}

// cv::solve(A, b, x, DECOMP_EIG) for symmetric A: eigen (JacobiImpl_) then SVBkSb with u = v = the
// eigenvector rows: threshold = 2 DBL_EPSILON x sum of w (signed), x = sum over w_i beyond it of
// (u_i . b) / w_i v_i, in index order [ext, restated].
inline void eig_solve(const double* A, int n, const double* b, double* x) {
    double M[81], w[9], V[81];
    for (int i = 0; i < n * n; ++i) M[i] = A[i];
    jacobi_eigen(M, n, w, V);
    double thr = 0;
    for (int i = 0; i < n; ++i) thr += w[i];
    thr *= DBL_EPSILON * 2;
    for (int j = 0; j < n; ++j) x[j] = 0;
    for (int i = 0; i < n; ++i) {
        double wi = w[i];
        if (std::fabs(wi) <= thr) continue;
        wi = 1 / wi;
        double s = 0;
        for (int j = 0; j < n; ++j) s += V[i * n + j] * b[j];
        s *= wi;
        for (int j = 0; j < n; ++j) x[j] = x[j] + s * V[i * n + j];
    }
}

// cv::invert(A, Ainv, DECOMP_EIG) for symmetric A: SVBkSb with b = I (row k of the inverse
// accumulates v_i[k] (u_i[j] / w_i)).
inline void eig_invert(const double* A, int n, double* Ainv) {
    double M[81], w[9], V[81];
    for (int i = 0; i < n * n; ++i) M[i] = A[i];
    jacobi_eigen(M, n, w, V);
    double thr = 0;
    for (int i = 0; i < n; ++i) thr += w[i];
    thr *= DBL_EPSILON * 2;
    for (int i = 0; i < n * n; ++i) Ainv[i] = 0;
    for (int e = 0; e < n; ++e) {
        double wi = w[e];
        if (std::fabs(wi) <= thr) continue;
        wi = 1 / wi;
        double buf[9];
        for (int j = 0; j < n; ++j) buf[j] = V[e * n + j] * wi;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) Ainv[i * n + j] = Ainv[i * n + j] + V[e * n + i] * buf[j];
    }
}

}  // namespace mcv
