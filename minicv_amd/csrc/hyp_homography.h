// hyp_homography.h — one RANSAC homography hypothesis: sample 4 correspondences, check the
// subset, solve the minimal DLT, emit the fp32 model the inlier sweep uses. Compiled for gfx950
// (kernel `mcv_h_generate`) and for the host (mcvHostHypothesis test hook). Built with
// -ffp-contract=off: every expression rounds as written, so host and device agree bit for bit.
//
// Semantics restated from OpenCV 4.x calib3d (not present in this container, version unpinned,
// SURVEY.md §8c) — the reference's own call sites are MiniCVNative.cpp:177,204 (findEssentialMat,
// the same RANSACPointSetRegistrator loop):
//   * subset check   = HomographyEstimatorCallback::checkSubset: haveCollinearPoints on both point
//                      sets (last point vs lines through earlier pairs, FLT_EPSILON test), then the
//                      4-triangle orientation-consistency test (Marquez-Neila et al. 2013);
//   * minimal solver = runKernel itself: centroid + mean-|dev| scaling, the 9x9 LtL, cv::eigen
//                      (JacobiImpl_, jacobi_eig.h), de-normalisation, 1/H22 (MCV_FLAG_FAST_MINIMAL:
//                      8x8 elimination with h22 = 1, opt-in);
//   * error          = HomographyEstimatorCallback::computeError: fp32, model cast to float,
//                      ww = 1/(h6 x + h7 y + 1), err = dx^2 + dy^2; inlier iff err <= (float)thr^2.
#pragma once

#include "mcv_common.h"
#include "jacobi_eig.h"

namespace mcv {

struct HModelF { float h[8]; };   // rows 0..1 and h20, h21 of H / H22 (h22 == 1 implied)

// OpenCV Matx_DetOp<double,3> expansion order.
MCV_HD double det3(double a00, double a01, double a02, double a10, double a11, double a12,
                   double a20, double a21, double a22) {
    return a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
}

// haveCollinearPoints(ms, 4): point 3 against lines through pairs of points 0..2.
// Differences are float - float (rounded to float), then promoted, as in OpenCV.
MCV_HD bool have_collinear4(const float* px, const float* py) {
    const int i = 3;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int j = 0; j < i; ++j) {
        const double dx1 = (double)(px[j] - px[i]);
        const double dy1 = (double)(py[j] - py[i]);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int k = 0; k < j; ++k) {
            const double dx2 = (double)(px[k] - px[i]);
            const double dy2 = (double)(py[k] - py[i]);
            if (fabs(dx2 * dy1 - dy2 * dx1) <= (double)kFltEpsilon * (fabs(dx1) + fabs(dy1) + fabs(dx2) + fabs(dy2)))
                return true;
        }
    }
    return false;
}

MCV_HD bool h_check_subset(const float* sx, const float* sy, const float* dx, const float* dy) {
    if (have_collinear4(sx, sy) || have_collinear4(dx, dy)) return false;
    const int tt[4][3] = {{0, 1, 2}, {1, 2, 3}, {0, 2, 3}, {0, 1, 3}};
    int negative = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        const int a = tt[i][0], b = tt[i][1], c = tt[i][2];
        const double dA = det3(sx[a], sy[a], 1.0, sx[b], sy[b], 1.0, sx[c], sy[c], 1.0);
        const double dB = det3(dx[a], dy[a], 1.0, dx[b], dy[b], 1.0, dx[c], dy[c], 1.0);
        negative += (dA * dB < 0) ? 1 : 0;
    }
    return negative == 0 || negative == 4;
}

// C = A * B for 3x3 row-major, sum order ((a0 b0 + a1 b1) + a2 b2).
MCV_HD void mat3_mul(const double* A, const double* B, double* C) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 3; ++i)
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int j = 0; j < 3; ++j)
            C[3 * i + j] = A[3 * i + 0] * B[0 * 3 + j] + A[3 * i + 1] * B[1 * 3 + j] + A[3 * i + 2] * B[2 * 3 + j];
}

// MCV_FLAG_FAST_MINIMAL (opt-in): runKernel's normalisation, then the 8x8 system (h22 = 1) by
// Gaussian elimination with partial pivoting instead of the eigen-solve — the same null vector up to
// the eigen-solve's convergence error (~1e-11 relative), 50x cheaper on the GPU.
// Returns false when degenerate (zero scale, zero pivot, non-finite result).
MCV_HD bool h_solve4_elim(const float* sx, const float* sy, const float* dx, const float* dy, double* H) {
    // Normalisation (runKernel): centroids and mean absolute deviations, in double.
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        cmx += (double)dx[i]; cmy += (double)dy[i];
        cMx += (double)sx[i]; cMy += (double)sy[i];
    }
    cmx /= 4; cmy /= 4; cMx /= 4; cMy /= 4;
    double smx = 0, smy = 0, sMx = 0, sMy = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        smx += fabs((double)dx[i] - cmx); smy += fabs((double)dy[i] - cmy);
        sMx += fabs((double)sx[i] - cMx); sMy += fabs((double)sy[i] - cMy);
    }
    if (fabs(smx) < kDblEpsilon || fabs(smy) < kDblEpsilon || fabs(sMx) < kDblEpsilon || fabs(sMy) < kDblEpsilon)
        return false;
    smx = 4 / smx; smy = 4 / smy; sMx = 4 / sMx; sMy = 4 / sMy;

    // Augmented 8x9 system for Hn (h22 = 1) in normalised coordinates.
    double a[8][9];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        const double x = ((double)dx[i] - cmx) * smx, y = ((double)dy[i] - cmy) * smy;
        const double X = ((double)sx[i] - cMx) * sMx, Y = ((double)sy[i] - cMy) * sMy;
        double* r0 = a[2 * i];
        double* r1 = a[2 * i + 1];
        r0[0] = X; r0[1] = Y; r0[2] = 1; r0[3] = 0; r0[4] = 0; r0[5] = 0; r0[6] = -(x * X); r0[7] = -(x * Y); r0[8] = x;
        r1[0] = 0; r1[1] = 0; r1[2] = 0; r1[3] = X; r1[4] = Y; r1[5] = 1; r1[6] = -(y * X); r1[7] = -(y * Y); r1[8] = y;
    }
    // Forward elimination with partial pivoting (first maximum wins). Row swaps are done with
    // selects over all rows so the matrix stays in registers on the device.
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int c = 0; c < 8; ++c) {
        int p = c;
        double best = fabs(a[c][c]);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int r = c + 1; r < 8; ++r) {
            const double v = fabs(a[r][c]);
            if (v > best) { best = v; p = r; }
        }
        if (!(best > 0)) return false;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int r = c + 1; r < 8; ++r) {
            const bool sw = (r == p);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int k = c; k < 9; ++k) {
                const double t = a[c][k];
                a[c][k] = sw ? a[r][k] : t;
                a[r][k] = sw ? t : a[r][k];
            }
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int r = c + 1; r < 8; ++r) {
            const double f = a[r][c] / a[c][c];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int k = c + 1; k < 9; ++k) a[r][k] = a[r][k] - f * a[c][k];
        }
    }
    double h[8];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 7; i >= 0; --i) {
        double s = a[i][8];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int k = i + 1; k < 8; ++k) s = s - a[i][k] * h[k];
        h[i] = s / a[i][i];
    }
    const double Hn[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9];
    mat3_mul(invHnorm, Hn, T);
    mat3_mul(T, Hnorm2, H);
    const double s = 1. / H[8];
    bool ok = true;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 9; ++i) {
        H[i] = H[i] * s;
        ok = ok && isfinite(H[i]);
    }
    return ok;
}

// runKernel's normalisation: centroids and mean absolute deviations in double -> nm = {cmx, cmy, smx,
// smy, cMx, cMy, sMx, sMy} (the scales already inverted, 4 / sum). False when a scale vanishes
// (runKernel returns 0).
MCV_HD bool h_norm4(const float* sx, const float* sy, const float* dx, const float* dy, double (&nm)[8]) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        cmx += (double)dx[i]; cmy += (double)dy[i];
        cMx += (double)sx[i]; cMy += (double)sy[i];
    }
    cmx /= 4; cmy /= 4; cMx /= 4; cMy /= 4;
    double smx = 0, smy = 0, sMx = 0, sMy = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        smx += fabs((double)dx[i] - cmx); smy += fabs((double)dy[i] - cmy);
        sMx += fabs((double)sx[i] - cMx); sMy += fabs((double)sy[i] - cMy);
    }
    if (fabs(smx) < kDblEpsilon || fabs(smy) < kDblEpsilon || fabs(sMx) < kDblEpsilon || fabs(sMy) < kDblEpsilon)
        return false;
    nm[0] = cmx; nm[1] = cmy; nm[2] = 4 / smx; nm[3] = 4 / smy;
    nm[4] = cMx; nm[5] = cMy; nm[6] = 4 / sMx; nm[7] = 4 / sMy;
    return true;
}

// runKernel's LtL[j][k] += Lx[j] Lx[k] + Ly[j] Ly[k] (k >= j, points in order, from +0): diagonal ->
// ws[kEigW..], strict upper triangle -> ws[kEigA..] (the eigen workspace's layout, both slice kinds).
// False when an entry is not finite.
template <class WS>
MCV_HD bool h_ltl4(const float* sx, const float* sy, const float* dx, const float* dy, const double (&nm)[8], WS& ws) {
    const double cmx = nm[0], cmy = nm[1], smx = nm[2], smy = nm[3], cMx = nm[4], cMy = nm[5], sMx = nm[6],
                 sMy = nm[7];
    double dg[9], up[36];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int e = 0; e < 36; ++e) up[e] = 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int e = 0; e < 9; ++e) dg[e] = 0.0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 4; ++i) {
        const double x = ((double)dx[i] - cmx) * smx, y = ((double)dy[i] - cmy) * smy;
        const double X = ((double)sx[i] - cMx) * sMx, Y = ((double)sy[i] - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int j = 0; j < 9; ++j) {
            dg[j] += Lx[j] * Lx[j] + Ly[j] * Ly[j];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int k = j + 1; k < 9; ++k) up[eig_tri(j, k)] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
        }
    }
    bool fin = true;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int e = 0; e < 36; ++e) {
        fin = fin && isfinite(up[e]);
        ws[kEigA + e] = up[e];
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int e = 0; e < 9; ++e) {
        fin = fin && isfinite(dg[e]);
        ws[kEigW + e] = dg[e];
    }
    return fin;
}

// H0 (the eigenvector) -> H = invHnorm H0 Hnorm2 (3x3 gemm order), scaled by 1/H22 (convertTo). False
// when the result is not finite (a non-finite model counts no inlier in OpenCV: the same RANSAC outcome
// as no model).
MCV_HD bool h_from_eig(const double (&H0)[9], const double (&nm)[8], double* H) {
    const double cmx = nm[0], cmy = nm[1], smx = nm[2], smy = nm[3], cMx = nm[4], cMy = nm[5], sMx = nm[6],
                 sMy = nm[7];
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double T[9];
    mat3_mul(invHnorm, H0, T);
    mat3_mul(T, Hnorm2, H);
    const double s = 1. / H[8];
    bool ok = true;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < 9; ++i) {
        H[i] = H[i] * s;
        ok = ok && isfinite(H[i]);
    }
    return ok;
}

// Minimal 4-point homography src -> dst = HomographyEstimatorCallback::runKernel on the sample:
// centroid + mean-|dev| normalisation (h_norm4), the LtL (h_ltl4), cv::eigen (eig9_jacobi,
// jacobi_eig.h) -> H0 = the eigenvector of the smallest eigenvalue, H = invHnorm H0 Hnorm2 / H22
// (h_from_eig). Returns false when the scales vanish, the LtL or the result is not finite.
template <class WS>
MCV_HD bool h_solve4(const float* sx, const float* sy, const float* dx, const float* dy, double* H, WS& ws,
                     bool fast = false) {
    if (fast) return h_solve4_elim(sx, sy, dx, dy, H);
    double nm[8];
    if (!h_norm4(sx, sy, dx, dy, nm)) return false;
    if (!h_ltl4(sx, sy, dx, dy, nm, ws)) return false;
    double w[9];
    const int r = eig9_jacobi(ws, w, 8);
    double H0[9];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int j = 0; j < 9; ++j) H0[j] = ws[kEigV + 9 * r + j];
    return h_from_eig(H0, nm, H);
}

// The sample search: OpenCV's getSubset attempts with the subset check (none for a tabled sampler),
// the accepted sample's points and indices. False = the sampler is exhausted (OpenCV's `break`).
MCV_HD bool h_sample(const float* pts4, int N, const Sampler& smp, uint64_t hyp, float* sx, float* sy, float* dx,
                     float* dy, int* idx) {
    SubsetSrc<4> src(smp, hyp);
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, *reinterpret_cast<int(*)[4]>(idx));
        if (got < 0) break;
        if (got == 0) continue;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = 0; i < 4; ++i) {
            const float* p = pts4 + 4 * (int64_t)idx[i];
            sx[i] = p[0]; sy[i] = p[1]; dx[i] = p[2]; dy[i] = p[3];
        }
        if (!src.tabled() && !h_check_subset(sx, sy, dx, dy)) continue;
        return true;
    }
    return false;
}

// The fp32 sweep model of H (rows 0..1 and h20, h21 as float); false when one is not finite.
MCV_HD bool h_model_f(const double* H, HModelF* mf) {
    bool ok = true;
    for (int i = 0; i < 8; ++i) {
        mf->h[i] = (float)H[i];
        ok = ok && isfinite(mf->h[i]);
    }
    return ok;
}

// One hypothesis: returns 1 (model written), kStatusNoModel, or kStatusNoSample.
// pts4: N packed {x, y, x', y'}. idx_out (optional) receives the accepted sample.
template <class WS>
MCV_HD int h_hypothesis(const float* pts4, int N, const Sampler& smp, uint64_t hyp, double* H, HModelF* mf,
                        int* idx_out, WS& ws, bool fast = false) {
    float sx[4], sy[4], dx[4], dy[4];
    int idx[4];
    // The sample search and the solve are kept apart: with the solve inside the attempt loop, lanes of
    // one wave that accept their sample at different attempts would each run the eigen-solve in a
    // separate pass of the loop (one pass per distinct attempt count).
    if (!h_sample(pts4, N, smp, hyp, sx, sy, dx, dy, idx)) return kStatusNoSample;
    if (idx_out) for (int i = 0; i < 4; ++i) idx_out[i] = idx[i];
    if (!h_solve4(sx, sy, dx, dy, H, ws, fast)) return kStatusNoModel;
    return h_model_f(H, mf) ? 1 : kStatusNoModel;
}

// HomographyEstimatorCallback::computeError for one correspondence, two bit-level definitions
// (the reference's own arithmetic is build-dependent: OpenCV's x86-64 SSE baseline — the
// reference's Linux/AMD64 target — evaluates the expression unfused, clang's default
// -ffp-contract=on on arm64 contracts it into FMAs):
//   op by op (default): every operation rounded as written, IEEE division (h_error); the sweep
//                    decides it without dividing (mcv_h_verify_cert, ransac_h.hip);
//   fused (MCV_FLAG_FUSED_ERROR): w = fma(h6,x,fma(h7,y,1)); ww = RN(1/w);
//                    ex = fma(fma(h0,x,fma(h1,y,h2)), ww, -mx); ey likewise; e = fma(ex,ex,ey*ey).
// Inlier iff e <= (float)thr^2 in both.
MCV_HD float h_error(const float* h, float x, float y, float mx, float my) {
    const float ww = 1.f / (h[6] * x + h[7] * y + 1.f);
    const float ex = (h[0] * x + h[1] * y + h[2]) * ww - mx;
    const float ey = (h[3] * x + h[4] * y + h[5]) * ww - my;
    return ex * ex + ey * ey;
}

MCV_HD float h_denominator_fused(const float* h, float x, float y) { return fmaf(h[6], x, fmaf(h[7], y, 1.f)); }

MCV_HD float h_error_fused_ww(const float* h, float x, float y, float mx, float my, float ww) {
    const float ex = fmaf(fmaf(h[0], x, fmaf(h[1], y, h[2])), ww, -mx);
    const float ey = fmaf(fmaf(h[3], x, fmaf(h[4], y, h[5])), ww, -my);
    return fmaf(ex, ex, ey * ey);
}

// Reference form of the fused error (IEEE division): host twin and rare-path fallback.
MCV_HD float h_error_fused(const float* h, float x, float y, float mx, float my) {
    return h_error_fused_ww(h, x, y, mx, my, 1.f / h_denominator_fused(h, x, y));
}

// |w| inside the range where rcp_newton(w) == 1.f / w (exhaustively verified).
MCV_HD bool rcp_newton_ok(float w) { return fabsf(w) >= 0x1p-126f && fabsf(w) < 0x1p126f; }

}  // namespace mcv
