// pnp_host.cpp — host side of the PnP path behind the reference's exports
// cvSolvePnPRansac, cvSolvePnP, cvRefinePnPLM, cvRefinePnPVVS, solveAp3p
// (MiniCVNative.cpp:48-163, ap3p.cpp:282-317) plus cvSolvePnPRansacCfg.
//
// solvePnPRansac (OpenCV 4.x, restated [ext]): points -> fp32; N == 4 -> one minimal solve, all
// inliers; else RANSACPointSetRegistrator(PnPRansacCallback, 4, reprojectionError, confidence,
// iterationsCount) -> the best model's mask -> solvePnP on the inliers. Here the hypotheses run
// on the GPU (ransac_pnp.hip) with the sequential replay of ransac_host.cpp, and the final solve
// on the inliers is Levenberg-Marquardt from the best hypothesis' pose (the ITERATIVE refinement
// OpenCV uses with an extrinsic guess) with its O(N) sums on the GPU.
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include "linalg.h"
#include "plan.h"
#include "hyp_pnp.h"
#include "pnp_pk.h"
#include "sqpnp.h"

#include <cmath>
#include <cfloat>
#include <cstring>
#include <algorithm>
#include <vector>
#include <algorithm>

namespace mcv {

// ---- rotation algebra (host) --------------------------------------------------------------------
static void skew(const double* v, double* S) {
    S[0] = 0; S[1] = -v[2]; S[2] = v[1];
    S[3] = v[2]; S[4] = 0; S[5] = -v[0];
    S[6] = -v[1]; S[7] = v[0]; S[8] = 0;
}
static void mul33(const double* A, const double* B, double* C) {
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// Rodrigues r -> R (row-major) and dR/dr_j (dR + 9 j), Gallego & Yezzi (2015):
//   dR/dr_j = (r_j [r]x + [r x ((I - R) e_j)]x) R / |r|^2;  [e_j]x for |r| -> 0.
void rodrigues(const double* r, double* R, double* dR) {
    const double th2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
    const double th = std::sqrt(th2);
    double S[9];
    skew(r, S);
    if (th < 1e-12) {
        for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0 ? 1.0 : 0.0) + S[k];
        if (dR)
            for (int j = 0; j < 3; ++j) {
                double e[3] = {0, 0, 0};
                e[j] = 1;
                skew(e, dR + 9 * j);
            }
        return;
    }
    const double s = std::sin(th), c = std::cos(th);
    double S2[9];
    mul33(S, S, S2);
    for (int k = 0; k < 9; ++k) R[k] = (k % 4 == 0 ? 1.0 : 0.0) + (s / th) * S[k] + ((1 - c) / th2) * S2[k];
    if (!dR) return;
    for (int j = 0; j < 3; ++j) {
        double w[3];   // (I - R) e_j
        for (int i = 0; i < 3; ++i) w[i] = (i == j ? 1.0 : 0.0) - R[3 * i + j];
        double rx[3] = {r[1] * w[2] - r[2] * w[1], r[2] * w[0] - r[0] * w[2], r[0] * w[1] - r[1] * w[0]};
        double A[9], B[9];
        skew(rx, A);
        for (int k = 0; k < 9; ++k) A[k] = (r[j] * S[k] + A[k]) / th2;
        mul33(A, R, B);
        for (int k = 0; k < 9; ++k) dR[9 * j + k] = B[k];
    }
}

// R -> r (axis * angle); robust near 0 and pi.
void rodrigues_inv(const double* R, double* r) {
    const double w[3] = {(R[7] - R[5]) * 0.5, (R[2] - R[6]) * 0.5, (R[3] - R[1]) * 0.5};
    const double s = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = std::max(-1.0, std::min(1.0, c));
    if (s > 1e-7) {
        const double th = std::atan2(s, c);
        for (int k = 0; k < 3; ++k) r[k] = w[k] * (th / s);
        return;
    }
    if (c > 0) {
        for (int k = 0; k < 3; ++k) r[k] = w[k];
        return;
    }
    // theta ~ pi: axis from the largest diagonal of (R + I) / 2
    int m = 0;
    for (int k = 1; k < 3; ++k)
        if (R[4 * k] > R[4 * m]) m = k;
    double ax[3];
    for (int k = 0; k < 3; ++k) ax[k] = (R[3 * m + k] + R[3 * k + m]) * 0.25 + (k == m ? 0.5 : 0.0);
    double n = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
    for (int k = 0; k < 3; ++k) ax[k] /= n;
    if (ax[0] * w[0] + ax[1] * w[1] + ax[2] * w[2] < 0)
        for (int k = 0; k < 3; ++k) ax[k] = -ax[k];
    const double th = std::atan2(s, c);
    for (int k = 0; k < 3; ++k) r[k] = ax[k] * th;
}

// ---- plan helpers -----------------------------------------------------------------------------
static void set_camera(Plan& P, const double* K9, const double* dist4) {
    P.pnpCam[0] = K9[0]; P.pnpCam[1] = K9[4]; P.pnpCam[2] = K9[2]; P.pnpCam[3] = K9[5];
    for (int k = 0; k < 4; ++k) P.pnpCam[4 + k] = dist4 ? dist4[k] : 0.0;
    if (!(K9[0] != 0) || !(K9[4] != 0) || !std::isfinite(K9[0]) || !std::isfinite(K9[4]))
        fail("camera matrix needs finite non-zero fx, fy");
}

static void pnp_pack(Plan& P, const mcvV2d* img, const mcvV3d* world, int N, void* d_out, hipStream_t s) {
    P.raw.ensure((size_t)N * 5);
    MCV_HIP(hipMemcpyAsync(P.raw.p, img, (size_t)N * sizeof(mcvV2d), hipMemcpyHostToDevice, s));
    MCV_HIP(hipMemcpyAsync(P.raw.p + 2 * (size_t)N, world, (size_t)N * sizeof(mcvV3d), hipMemcpyHostToDevice, s));
    launch_pnp_pack(P.raw.p, P.raw.p + 2 * (size_t)N, N, d_out, s);
    MCV_HIP(hipGetLastError());
}

static bool fused_pnp(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_FUSED_ERROR) != 0; }
// MCV_FLAG_FAST_MINIMAL: AP3P hypotheses from the real-root finder instead of the reference's Ferrari quartic
static bool fast_ap3p(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_FAST_MINIMAL) != 0; }
bool pnp_cfg_epnp(const RansacConfig& cfg) { return pnp_kind_epnp(pnp_kind(cfg.pnpKind)); }

// AP3P / EPnP generate: every hypothesis on the device, the reference's arithmetic included (AP3P's
// complex-pow branch runs glibc's clog / exp / cos / atan2 as restated in glibc_math.h).
static void pnp_generate_exact(Plan& P, const void* d_pts, int N, const Sampler& smp, int64_t hypBegin, int hypCount,
                               bool epnp, bool fast, void* d_models, int* d_counts, hipStream_t s) {
    if (epnp) P.escratch.ensure((size_t)std::min(hypCount, kEpnpPiece) * kEpnpSplitDoubles);
    launch_pnp_generate(d_pts, N, P.pnpCam, smp, hypBegin, hypCount, epnp, d_models, d_counts,
                        epnp ? P.escratch.p : nullptr, s, fast);
    MCV_HIP(hipGetLastError());
}

void p_evaluate_chunk(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t hypBegin, int hypCount,
                      int* d_counts, hipStream_t s) {
    const float thr2 = (float)(cfg.threshold * cfg.threshold);
    const bool epnp = pnp_cfg_epnp(cfg);
    const Sampler smp = P.sampler(cfg);
    {
        ProfScope pg("pnp_generate", s);
        pnp_generate_exact(P, d_pts, N, smp, hypBegin, hypCount, epnp, fast_ap3p(cfg), P.models.p, d_counts, s);
    }
    mark_chunk(P, hypBegin, hypCount, smp, d_pts, N, epnp ? 1 : (fast_ap3p(cfg) ? 2 : 0), s);
    P.bb4.ensure(4);
    P.pairs.ensure((size_t)(N + 1) * kPnpPairFloatsPerPoint);
    launch_pnp_extent(d_pts, N, P.bb4.p, P.pairs.p, s);
    ProfScope ps("pnp_verify", s);
    launch_pnp_verify(d_pts, N, P.pnpCam, P.models.p, d_counts, hypCount, thr2, fused_pnp(cfg), P.bb4.p, P.pairs.p, s);
}

static PnpOneOut pnp_fetch_one(Plan& P, hipStream_t s) {
    PnpOneOut one;
    MCV_HIP(hipMemcpyAsync(P.h_one.p, P.one.p, sizeof(PnpOneOut), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    std::memcpy(&one, P.h_one.p, sizeof(PnpOneOut));
    return one;
}

static int pnp_mask_count(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, const double* R, const double* t,
                          uint8_t* d_mask, hipStream_t s) {
    const float thr2 = (float)(cfg.threshold * cfg.threshold);
    MCV_HIP(hipMemsetAsync(P.count.p, 0, sizeof(int), s));
    launch_pnp_mask(d_pts, N, P.pnpCam, R, t, thr2, fused_pnp(cfg), d_mask, P.count.p, s);
    MCV_HIP(hipGetLastError());
    MCV_HIP(hipMemcpyAsync(P.h_i.p, P.count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    return P.h_i.p[0];
}

// Levenberg-Marquardt on (rvec, t) over the (masked) correspondences: damping A + lambda diag(A),
// lambda from 1e-3 (x10 on rejection, /10 on acceptance), at most maxIters accepted-or-rejected
// steps, stop when the step is below FLT_EPSILON relative to the parameters or the cost stalls.
void pnp_lm(Plan& P, const void* d_pts, int N, const uint8_t* d_mask, double* rvec, double* t, int maxIters,
            hipStream_t s) {
    double p[6] = {rvec[0], rvec[1], rvec[2], t[0], t[1], t[2]};
    auto eval = [&](const double* q, bool wantJ, double* A, double* g) -> double {
        double R[9], dR[27], buf[28];
        rodrigues(q, R, wantJ ? dR : nullptr);
        reduce_to_host(P, s, 28, buf, [&](double* part, double* red) {
            pnp_reduce_lm(d_pts, N, d_mask, P.pnpCam, R, q + 3, wantJ ? dR : nullptr, wantJ, part, red, s);
        });
        if (wantJ) {
            int o = 0;
            for (int j = 0; j < 6; ++j)
                for (int k = j; k < 6; ++k) { A[6 * j + k] = buf[o]; A[6 * k + j] = buf[o]; ++o; }
            for (int j = 0; j < 6; ++j) g[j] = buf[21 + j];
        }
        return buf[27];
    };
    double A[36], g[6];
    double S = eval(p, true, A, g);
    double lambda = 1e-3;
    for (int it = 0; it < maxIters; ++it) {
        double M[36], rhs[6], d[6];
        for (int k = 0; k < 36; ++k) M[k] = A[k];
        for (int k = 0; k < 6; ++k) {
            M[7 * k] = A[7 * k] + lambda * std::max(A[7 * k], DBL_EPSILON);
            rhs[k] = -g[k];
        }
        eig_solve(M, 6, rhs, d);
        double q[6], dn = 0, pn = 0;
        for (int k = 0; k < 6; ++k) {
            q[k] = p[k] + d[k];
            dn = std::max(dn, std::fabs(d[k]));
            pn = std::max(pn, std::fabs(p[k]));
        }
        // the normal equations at q ride along with its cost (one synchronisation per step); on
        // acceptance they equal the re-evaluation at the new p (same sums, same order)
        double Aq[36], gq[6];
        const double Sq = eval(q, true, Aq, gq);
        if (Sq < S) {
            const bool stall = (S - Sq) <= FLT_EPSILON * S;
            for (int k = 0; k < 6; ++k) p[k] = q[k];
            lambda = std::max(lambda * 0.1, 1e-12);
            S = Sq;
            std::memcpy(A, Aq, sizeof(Aq));
            std::memcpy(g, gq, sizeof(gq));
            if (stall || dn <= FLT_EPSILON * (pn + FLT_EPSILON)) break;
        } else {
            lambda *= 10;
            if (dn <= FLT_EPSILON * (pn + FLT_EPSILON) || lambda > 1e16) break;
        }
    }
    for (int k = 0; k < 3; ++k) { rvec[k] = p[k]; t[k] = p[3 + k]; }
}

// Virtual visual servoing (solvePnPRefineVVS restated): v = -lambda (L^T L)^+ L^T e on the
// normalised image plane, cMo <- exp(v)^-1 cMo, 20 iterations or |v| < FLT_EPSILON.
void pnp_vvs(Plan& P, const void* d_pts, int N, double* rvec, double* t, int maxIters, double lambda, hipStream_t s) {
    double R[9];
    rodrigues(rvec, R, nullptr);
    for (int it = 0; it < maxIters; ++it) {
        double buf[28];
        reduce_to_host(P, s, 28, buf, [&](double* part, double* red) {
            pnp_reduce_vvs(d_pts, N, nullptr, P.pnpCam, R, t, part, red, s);
        });
        double A[36], g[6], v[6];
        int o = 0;
        for (int j = 0; j < 6; ++j)
            for (int k = j; k < 6; ++k) { A[6 * j + k] = buf[o]; A[6 * k + j] = buf[o]; ++o; }
        for (int j = 0; j < 6; ++j) g[j] = buf[21 + j];
        eig_solve(A, 6, g, v);
        double vn = 0;
        for (int k = 0; k < 6; ++k) { v[k] = -lambda * v[k]; vn += v[k] * v[k]; }
        // T = exp(v): rotation Rodrigues(w), translation V u
        const double* u = v;
        const double* w = v + 3;
        double Rw[9], S[9], S2[9], V[9];
        rodrigues(w, Rw, nullptr);
        skew(w, S);
        mul33(S, S, S2);
        const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2], th = std::sqrt(th2);
        const double a = th < 1e-8 ? 0.5 : (1 - std::cos(th)) / th2;
        const double b = th < 1e-8 ? 1.0 / 6.0 : (th - std::sin(th)) / (th2 * th);
        for (int k = 0; k < 9; ++k) V[k] = (k % 4 == 0 ? 1.0 : 0.0) + a * S[k] + b * S2[k];
        double tt[3];
        for (int i = 0; i < 3; ++i) tt[i] = V[3 * i] * u[0] + V[3 * i + 1] * u[1] + V[3 * i + 2] * u[2];
        // cMo <- T^-1 cMo: R' = Rw^T R, t' = Rw^T (t - tt)
        double Rn[9], tn[3];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) Rn[3 * i + j] = Rw[i] * R[j] + Rw[3 + i] * R[3 + j] + Rw[6 + i] * R[6 + j];
        for (int i = 0; i < 3; ++i)
            tn[i] = Rw[i] * (t[0] - tt[0]) + Rw[3 + i] * (t[1] - tt[1]) + Rw[6 + i] * (t[2] - tt[2]);
        std::memcpy(R, Rn, sizeof(R));
        std::memcpy(t, tn, sizeof(tn));
        if (std::sqrt(vn) < FLT_EPSILON) break;
    }
    rodrigues_inv(R, rvec);
}

// EPnP (epnp.h, OpenCV compute_pose) over n points already on the device as double world points
// d_pw[3n] and pixel observations d_us[2n]: the O(n) loops run as blocked fixed-order passes
// (mcv_epnp_pass), the 3x3 / 12x12 / 6xK algebra between them here on the host. The passes whose inputs
// are only means of the previous pass's sums (Pw0 after SumPw, Abt after Pc) take them on the device
// (round 6), so the solve costs four host round trips: {SumPw, Pw0}, MtM, {Pc, Abt}, Reproj.
// first (optional): {SumPw, Pw0} already ran and came back with the caller's synchronisation.
struct EpnpFirst {
    double sum[3], p6[6], p0[3];
};

// Host sums of a pass's block partials, in block order from 0 (as the device's derived means).
static void epnp_sums(const std::vector<double>& part, size_t off, int nacc, int nblk, double* out) {
    for (int a = 0; a < nacc; ++a) {
        double t = 0;
        for (int b = 0; b < nblk; ++b) t += part[off + (size_t)a * nblk + b];
        out[a] = t;
    }
}

static void epnp_device(Plan& P, const double* d_pw, const double* d_us, int n, double* R9, double* t3,
                        hipStream_t s, const EpnpFirst* first = nullptr) {
    if (n < 4) fail("EPnP needs at least 4 points (n=%d)", n);
    EpnpPassArgs A;
    std::memset(&A, 0, sizeof(A));
    A.cam = EpnpCam{P.pnpCam[0], P.pnpCam[1], P.pnpCam[2], P.pnpCam[3]};
    const int nblk = (n + kEpnpBlock - 1) / kEpnpBlock;
    P.part.ensure((size_t)kMtmSums * nblk);   // two passes at once: [0, 9 nblk) and [9 nblk, 36 nblk)
    std::vector<double> part((size_t)kMtmSums * nblk);
    auto launch = [&](int mode, int nacc, size_t off, const double* prev) {
        launch_epnp_pass(mode, d_pw, d_us, n, A, nacc, P.part.p + off, s, nullptr, prev);
        MCV_HIP(hipGetLastError());
    };
    auto fetch = [&](size_t count, double* extra = nullptr, const double* d_extra = nullptr, size_t nextra = 0) {
        MCV_HIP(hipMemcpyAsync(part.data(), P.part.p, count * sizeof(double), hipMemcpyDeviceToHost, s));
        if (extra) MCV_HIP(hipMemcpyAsync(extra, d_extra, nextra * sizeof(double), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
    };
    const size_t off1 = (size_t)9 * nblk;
    double sum[3], p6[6], p0[3], mtm[kMtmSums], pcs[9], abt[27], rep3[3];
    if (first) {
        std::memcpy(sum, first->sum, sizeof(sum));
        std::memcpy(p6, first->p6, sizeof(p6));
        std::memcpy(p0, first->p0, sizeof(p0));
    } else {
        launch(kEpnpPassSumPw, 3, 0, nullptr);
        launch(kEpnpPassPw0, 6, off1, P.part.p);   // centroid from SumPw's partials on the device
        fetch(off1 + (size_t)6 * nblk, p0, d_pw, 3);
        epnp_sums(part, 0, 3, nblk, sum);
        epnp_sums(part, off1, 6, nblk, p6);
    }
    for (int j = 0; j < 3; ++j) A.c0[j] = sum[j] / n;
    const double P3[3][3] = {{p6[0], p6[1], p6[2]}, {p6[1], p6[3], p6[4]}, {p6[2], p6[4], p6[5]}};
    epnp_control(sum, P3, n, A.C);
    launch(kEpnpPassMtm, kMtmSums, 0, nullptr);
    fetch((size_t)kMtmSums * nblk);
    epnp_sums(part, 0, kMtmSums, nblk, mtm);
    EpnpBetas B;
    epnp_betas(mtm, A.C, B);
    double al0[4];
    epnp_alphas(A.C, p0, al0);
    for (int N = 0; N < 3; ++N) {
        epnp_ccs(B, B.betas[N + 1], A.ccs[N]);
        double pc[3];
        epnp_pc(al0, A.ccs[N], pc);
        if (pc[2] < 0.0)   // solve_for_sign on the first point; -ccs gives exactly the negated pcs
            for (int j = 0; j < 4; ++j)
                for (int k = 0; k < 3; ++k) A.ccs[N][j][k] = -A.ccs[N][j][k];
    }
    for (int j = 0; j < 3; ++j) A.pw0[j] = sum[j] / n;
    launch(kEpnpPassPc, 9, 0, nullptr);
    launch(kEpnpPassAbt, 27, off1, P.part.p);   // pc0 from Pc's partials on the device
    fetch(off1 + (size_t)27 * nblk);
    epnp_sums(part, 0, 9, nblk, pcs);
    epnp_sums(part, off1, 27, nblk, abt);
    for (int N = 0; N < 3; ++N)
        for (int j = 0; j < 3; ++j) A.pc0[N][j] = pcs[3 * N + j] / n;
    for (int N = 0; N < 3; ++N) {
        double ab[3][3];
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) ab[j][k] = abt[9 * N + 3 * j + k];
        epnp_rt(ab, A.pc0[N], A.pw0, A.R[N], A.t[N]);
    }
    launch(kEpnpPassReproj, 3, 0, nullptr);
    fetch((size_t)3 * nblk);
    epnp_sums(part, 0, 3, nblk, rep3);
    const double rep[4] = {0, rep3[0] / n, rep3[1] / n, rep3[2] / n};
    const int N = epnp_pick(rep) - 1;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) R9[3 * i + j] = A.R[N][i][j];
        t3[i] = A.t[N][i];
    }
}

// solvePnP(SOLVEPNP_SQPNP) (reference MiniCVNative.cpp:72-74, :82): undistortPoints' normalised
// coordinates and the computeOmega sums as one device pass, the SQPnP algebra on the host (sqpnp.h),
// the positive-depth count of positiveMajorityDepths as a device pass when the centroid check fails.
// Returns sqpnp_from_sums' code; R9 / t3: the first solution.
static int sqpnp_device(Plan& P, const double* d_pw, const double* d_us, int n, double* R9, double* t3,
                        hipStream_t s) {
    EpnpPassArgs A;
    std::memset(&A, 0, sizeof(A));
    const int nblk = (n + kEpnpBlock - 1) / kEpnpBlock;
    std::vector<double> part;
    auto pass = [&](int mode, int nacc, double* out) {
        P.part.ensure((size_t)nacc * nblk);
        launch_epnp_pass(mode, d_pw, d_us, n, A, nacc, P.part.p, s);
        MCV_HIP(hipGetLastError());
        part.resize((size_t)nacc * nblk);
        MCV_HIP(hipMemcpyAsync(part.data(), P.part.p, part.size() * sizeof(double), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        for (int a = 0; a < nacc; ++a) {
            double t = 0;
            for (int b = 0; b < nblk; ++b) t += part[(size_t)a * nblk + b];
            out[a] = t;
        }
    };
    double sums[kSqpSums];
    pass(kEpnpPassSqp, kSqpSums, sums);
    auto npos = [&](const double* rh, const double* t) {
        for (int k = 0; k < 3; ++k) A.R[0][2][k] = rh[6 + k];
        A.t[0][2] = t[2];
        double c;
        pass(kEpnpPassSqpDepth, 1, &c);
        return (int)c;
    };
    double rh[9], t[3];
    const int r = sqpnp_from_sums(sums, n, npos, rh, t);
    if (r > 0) {
        std::memcpy(R9, rh, sizeof(rh));
        std::memcpy(t3, t, sizeof(t));
    }
    return r;
}

// solvePnPRansac's final EPnP: the inliers (compressElems order) of the float points as doubles,
// image points through undistortPoints with a double result.
// Round 6: the compaction, the prep and the first two passes run on the device count, and the count,
// their sums and the first point return with one synchronisation (four before).
static void epnp_inliers(Plan& P, const void* d_pts, int N, const uint8_t* d_mask, double* R9, double* t3,
                         hipStream_t s) {
    P.eidx.ensure((size_t)std::max(N, 1));
    launch_mask_compact(d_mask, N, P.eidx.p, P.count.p, s);
    MCV_HIP(hipGetLastError());
    P.epw.ensure((size_t)3 * std::max(N, 1));
    P.eus.ensure((size_t)2 * std::max(N, 1));
    launch_epnp_prep(d_pts, P.eidx.p, nullptr, nullptr, N, P.pnpCam, P.epw.p, P.eus.p, s, false, P.count.p);
    EpnpPassArgs A;
    std::memset(&A, 0, sizeof(A));
    const int nblkMax = (N + kEpnpBlock - 1) / kEpnpBlock;
    P.part.ensure((size_t)9 * nblkMax);
    double* d_sum = P.part.p;
    double* d_p6 = P.part.p + (size_t)3 * nblkMax;
    launch_epnp_pass(kEpnpPassSumPw, P.epw.p, P.eus.p, N, A, 3, d_sum, s, P.count.p);
    launch_epnp_pass(kEpnpPassPw0, P.epw.p, P.eus.p, N, A, 6, d_p6, s, P.count.p, d_sum);
    MCV_HIP(hipGetLastError());
    std::vector<double> part((size_t)9 * nblkMax);
    EpnpFirst F;
    MCV_HIP(hipMemcpyAsync(P.h_i.p, P.count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipMemcpyAsync(part.data(), P.part.p, part.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipMemcpyAsync(F.p0, P.epw.p, sizeof(F.p0), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    const int n = P.h_i.p[0];
    if (n < 4) fail("EPnP needs at least 4 points (n=%d)", n);
    // the device count's block stride; Pw0's region starts at 3 nblkMax
    const int nblk = (n + kEpnpBlock - 1) / kEpnpBlock;
    epnp_sums(part, 0, 3, nblk, F.sum);
    epnp_sums(part, (size_t)3 * nblkMax, 6, nblk, F.p6);
    epnp_device(P, P.epw.p, P.eus.p, n, R9, t3, s, &F);
}

// Device API finalize: winner -> mask -> the inlier solve of the kind (solvePnPRansac's tail):
// ITERATIVE refines the RANSAC pose with LM (useExtrinsicGuess = true), every other kind runs EPnP
// on the inliers (P3P / AP3P switch to EPnP there). model9 = {rvec, tvec, 0, 0, 0}.
int p_finalize(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t hyp, double* model9,
               uint8_t* d_mask, hipStream_t s) {
    PnpOneOut one;
    const bool epnp = pnp_cfg_epnp(cfg);
    const Sampler smp = P.sampler(cfg);
    int count = 0;
    if (P.last.covers(hyp, smp, d_pts, N, epnp ? 1 : (fast_ap3p(cfg) ? 2 : 0))) {
        // the winner's pose straight from the last chunk's model buffer (the same code produced it)
        // instead of a single-lane re-solve; its mask and count from that slot too, so the pose, the
        // count and the freshness check return with one synchronisation
        const PnpPose* d_m = (const PnpPose*)P.models.p + (hyp - P.last.begin);
        MCV_HIP(hipMemcpyAsync(P.h_one.p, d_m, sizeof(PnpPose), hipMemcpyDeviceToHost, s));
        queue_chunk_check(P, d_pts, N, s);
        MCV_HIP(hipMemsetAsync(P.count.p, 0, sizeof(int), s));
        launch_pnp_mask_dev(d_pts, N, P.pnpCam, d_m, (float)(cfg.threshold * cfg.threshold), fused_pnp(cfg), d_mask,
                            P.count.p, s);
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipMemcpyAsync(P.h_i.p, P.count.p, sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        if (!chunk_fresh(P)) {   // the points changed since the chunk was evaluated: re-solve
            P.last.clear();
            return p_finalize(P, d_pts, N, cfg, hyp, model9, d_mask, s);
        }
        PnpPose pose;
        std::memcpy(&pose, P.h_one.p, sizeof(PnpPose));
        std::memcpy(one.R, pose.R, sizeof(one.R));
        std::memcpy(one.t, pose.t, sizeof(one.t));
        one.status = 1;
        count = P.h_i.p[0];
    } else {
        launch_pnp_one(d_pts, N, P.pnpCam, smp, hyp, epnp, (PnpOneOut*)P.one.p, s, fast_ap3p(cfg));
        MCV_HIP(hipGetLastError());
        one = pnp_fetch_one(P, s);
        if (one.status != 1) fail("winning hypothesis %lld has no model (status %d)", (long long)hyp, one.status);
        count = pnp_mask_count(P, d_pts, N, cfg, one.R, one.t, d_mask, s);
    }
    double r[3], t[3] = {one.t[0], one.t[1], one.t[2]};
    rodrigues_inv(one.R, r);
    if (!(cfg.flags & MCV_FLAG_NO_REFINE) && count > 0) {
        if (pnp_kind(cfg.pnpKind) == 0) {
            pnp_lm(P, d_pts, N, d_mask, r, t, 20, s);
        } else {
            double R2[9];
            epnp_inliers(P, d_pts, N, d_mask, R2, t, s);
            rodrigues_inv(R2, r);
        }
    }
    for (int k = 0; k < 3; ++k) { model9[k] = r[k]; model9[3 + k] = t[k]; model9[6 + k] = 0; }
    return count;
}

struct PnpResult {
    bool ok = false;
    int count = 0;
    double r[3] = {0, 0, 0}, t[3] = {0, 0, 0};
};

// The RANSAC export body. Mask of the best hypothesis stays in P.mask (d_mask).
static PnpResult pnp_ransac(Plan& P, const mcvV2d* img, const mcvV3d* world, int N, const double* K9,
                            const double* dist, const RansacConfig& cfg, hipStream_t s) {
    PnpResult res;
    set_camera(P, K9, dist);
    P.reserve(N, 1);
    pnp_pack(P, img, world, N, P.ptsd.p, s);
    const bool epnp = pnp_cfg_epnp(cfg);
    if (N == 4 || (epnp && N == 5)) {
        // npoints == model_points: one solvePnP on all points (P3P for 4, here AP3P; EPnP for 5)
        if (N == 4) launch_pnp_solve4(P.ptsd.p, P.pnpCam, (PnpOneOut*)P.one.p, s, fast_ap3p(cfg));
        else launch_pnp_solve5(P.ptsd.p, P.pnpCam, (PnpOneOut*)P.one.p, s);
        MCV_HIP(hipGetLastError());
        PnpOneOut one = pnp_fetch_one(P, s);
        if (one.status != 1) return res;
        rodrigues_inv(one.R, res.r);
        for (int k = 0; k < 3; ++k) res.t[k] = one.t[k];
        launch_fill_u8(P.mask.p, N, 1, s);
        res.count = N;
        res.ok = true;
        return res;
    }
    const int64_t best = ransac_search(P, P.ptsd.p, N, cfg, s);
    if (best < 0) return res;
    double model9[9];
    res.count = p_finalize(P, P.ptsd.p, N, cfg, best, model9, P.mask.p, s);
    for (int k = 0; k < 3; ++k) { res.r[k] = model9[k]; res.t[k] = model9[3 + k]; }
    res.ok = true;
    return res;
}

static RansacConfig pnp_config(int iters, float thr, double conf, int kind) {
    RansacConfig c;
    std::memset(&c, 0, sizeof(c));
    c.threshold = (double)thr;
    c.confidence = conf;
    c.maxIters = iters;
    c.method = MCV_METHOD_RANSAC;
    c.pnpKind = kind;
    c.flags = MCV_FLAG_CV_SAMPLER;   // solvePnPRansac's own sample stream (the reference's API has no seed)
    return c;
}

static bool pnp_ransac_export(const mcvV2d* img, const mcvV3d* world, int N, const mcvM33d& K, const double* dist,
                              const RansacConfig& cfg, mcvV3d* tVec, mcvV3d* rVec, int* inlierCount,
                              int* outInliers) {
    if (inlierCount) *inlierCount = 0;
    if (!img || !world || !tVec || !rVec || !inlierCount) fail("cvSolvePnPRansac: null argument");
    if (N < 4) fail("cvSolvePnPRansac: need at least 4 correspondences (N=%d)", N);
    if (!(cfg.confidence > 0 && cfg.confidence < 1)) fail("cvSolvePnPRansac: confidence must be in (0,1)");
    check_flags(cfg, "cvSolvePnPRansac");
    require_device();
    Plan& P = thread_plan(MCV_MODEL_PNP);
    hipStream_t s = P.own_stream();
    const PnpResult r = pnp_ransac(P, img, world, N, K.M, dist, cfg, s);
    if (!r.ok) {
        set_last_error("cvSolvePnPRansac: RANSAC found no pose with >= 4 inliers");
        return false;
    }
    rVec->X = r.r[0]; rVec->Y = r.r[1]; rVec->Z = r.r[2];
    tVec->X = r.t[0]; tVec->Y = r.t[1]; tVec->Z = r.t[2];
    std::vector<uint8_t> m(N);
    MCV_HIP(hipMemcpyAsync(m.data(), P.mask.p, (size_t)N, hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    int c = 0;
    for (int i = 0; i < N; ++i)
        if (m[i]) {
            if (outInliers) outInliers[c] = i;
            ++c;
        }
    *inlierCount = c;
    return true;
}

}  // namespace mcv

using namespace mcv;

extern "C" MCV_API mcvBool cvSolvePnPRansac(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N,
                                         const mcvM33d K, const double* distortionCoeffs, const int solverKind,
                                         const int iterationsCount, const float reprojectionError,
                                         const double confidence, mcvV3d* tVec, mcvV3d* rVec, int* inlierCount,
                                         int* outInliers) {
    MCV_GUARD(false, {
        const RansacConfig cfg = pnp_config(iterationsCount, reprojectionError, confidence, pnp_kind(solverKind));
        return pnp_ransac_export(imgPoints, worldPoints, N, K, distortionCoeffs, cfg, tVec, rVec, inlierCount,
                                 outInliers);
    })
}

extern "C" MCV_API mcvBool cvSolvePnPRansacCfg(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N,
                                            const mcvM33d K, const double* distortionCoeffs, const RansacConfig* cfgp,
                                            mcvV3d* tVec, mcvV3d* rVec, int* inlierCount, int* outInliers) {
    MCV_GUARD(false, {
        RansacConfig cfg = cfgp ? *cfgp : pnp_config(100, 8.0f, 0.99, 0);
        if (cfg.method != MCV_METHOD_RANSAC) fail("cvSolvePnPRansacCfg: only RANSAC (method 8)");
        return pnp_ransac_export(imgPoints, worldPoints, N, K, distortionCoeffs, cfg, tVec, rVec, inlierCount,
                                 outInliers);
    })
}

extern "C" MCV_API mcvBool cvSolvePnP(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                                   const double* distortionCoeffs, const int solverKind, mcvV3d* tVec, mcvV3d* rVec) {
    MCV_GUARD(false, {
        if (!imgPoints || !worldPoints || !tVec || !rVec) fail("cvSolvePnP: null argument");
        // solverKind as MiniCVNative.cpp:54-75 maps it (6 = SQPNP, unknown = ITERATIVE)
        const int kind = solverKind >= 0 && solverKind <= 6 ? solverKind : 0;
        // solvePnPGeneric's point-count assertion: SQPnP from 3 points, the others from 4
        if (N < (kind == 6 ? 3 : 4)) fail("cvSolvePnP: need at least %d correspondences (N=%d)", kind == 6 ? 3 : 4, N);
        const bool p3p = kind == 2 || kind == 5;
        if (p3p && N != 4) fail("cvSolvePnP: P3P / AP3P need exactly 4 points (N=%d)", N);
        require_device();
        Plan& P = thread_plan(MCV_MODEL_PNP);
        hipStream_t s = P.own_stream();
        PnpResult r;
        if (p3p) {
            r = pnp_ransac(P, imgPoints, worldPoints, N, K.M, distortionCoeffs, pnp_config(1, 1.f, 0.99, kind), s);
        } else if (kind == 6) {
            set_camera(P, K.M, distortionCoeffs);
            P.raw.ensure((size_t)N * 5);
            MCV_HIP(hipMemcpyAsync(P.raw.p, imgPoints, (size_t)N * sizeof(mcvV2d), hipMemcpyHostToDevice, s));
            MCV_HIP(hipMemcpyAsync(P.raw.p + 2 * (size_t)N, worldPoints, (size_t)N * sizeof(mcvV3d),
                                   hipMemcpyHostToDevice, s));
            P.epw.ensure((size_t)3 * N);
            P.eus.ensure((size_t)2 * N);
            launch_epnp_prep(nullptr, nullptr, P.raw.p, P.raw.p + 2 * (size_t)N, N, P.pnpCam, P.epw.p, P.eus.p, s,
                             true);
            MCV_HIP(hipGetLastError());
            double R9[9];
            const int code = sqpnp_device(P, P.epw.p, P.eus.p, N, R9, r.t, s);
            // computeOmega's CV_Asserts (an exception in OpenCV): a failure with the reason
            if (code == -1) fail("cvSolvePnP(SQPNP): point coordinate variance below 1e-5 (degenerate image points)");
            if (code == -2) fail("cvSolvePnP(SQPNP): Omega's largest singular value below 1e-7");
            if (code == -3) fail("cvSolvePnP(SQPNP): Omega's null space has more than 6 dimensions");
            if (code > 0) {
                rodrigues_inv(R9, r.r);
                r.ok = true;
            }
        } else {
            // EPnP on all points in double (solvePnPGeneric keeps the caller's CV_64F points);
            // ITERATIVE: then LM over all points from that pose (the reference's DLT or homography
            // initialisation is not restated: DESIGN.md §3)
            set_camera(P, K.M, distortionCoeffs);
            P.reserve(N, 1);
            pnp_pack(P, imgPoints, worldPoints, N, P.ptsd.p, s);
            P.epw.ensure((size_t)3 * N);
            P.eus.ensure((size_t)2 * N);
            launch_epnp_prep(nullptr, nullptr, P.raw.p, P.raw.p + 2 * (size_t)N, N, P.pnpCam, P.epw.p, P.eus.p, s);
            MCV_HIP(hipGetLastError());
            double R9[9];
            epnp_device(P, P.epw.p, P.eus.p, N, R9, r.t, s);
            rodrigues_inv(R9, r.r);
            r.ok = std::isfinite(r.r[0]) && std::isfinite(r.r[1]) && std::isfinite(r.r[2]) && std::isfinite(r.t[0]) &&
                   std::isfinite(r.t[1]) && std::isfinite(r.t[2]);
            if (r.ok && kind == 0) pnp_lm(P, P.ptsd.p, N, nullptr, r.r, r.t, 20, s);
        }
        if (!r.ok) {
            set_last_error("cvSolvePnP: no pose");
            return false;
        }
        rVec->X = r.r[0]; rVec->Y = r.r[1]; rVec->Z = r.r[2];
        tVec->X = r.t[0]; tVec->Y = r.t[1]; tVec->Z = r.t[2];
        return true;
    })
}

static void refine_common(const mcvV2d* img, const mcvV3d* world, int N, const mcvM33d& K, const double* dist,
                          mcvV3d* tVec, mcvV3d* rVec, bool vvs) {
    if (!img || !world || !tVec || !rVec) fail("cvRefinePnP: null argument");
    if (N < 3) fail("cvRefinePnP: need at least 3 correspondences (N=%d)", N);
    require_device();
    Plan& P = thread_plan(MCV_MODEL_PNP);
    hipStream_t s = P.own_stream();
    set_camera(P, K.M, dist);
    P.reserve(N, 1);
    pnp_pack(P, img, world, N, P.ptsd.p, s);
    double r[3] = {rVec->X, rVec->Y, rVec->Z}, t[3] = {tVec->X, tVec->Y, tVec->Z};
    if (vvs) pnp_vvs(P, P.ptsd.p, N, r, t, 20, 1.0, s);
    else pnp_lm(P, P.ptsd.p, N, nullptr, r, t, 20, s);
    rVec->X = r[0]; rVec->Y = r[1]; rVec->Z = r[2];
    tVec->X = t[0]; tVec->Y = t[1]; tVec->Z = t[2];
}

extern "C" MCV_API int mcvHostSqpnp(const double* img, const double* world, int N, const double* cam8, double* R9,
                                    double* t3) {
    MCV_GUARD(-4, {
        if (!img || !world || !cam8 || !R9 || !t3 || N < 3) fail("mcvHostSqpnp: bad argument");
        PnpCamera c;
        c.fx = cam8[0]; c.fy = cam8[1]; c.cx = cam8[2]; c.cy = cam8[3];
        c.k1 = cam8[4]; c.k2 = cam8[5]; c.p1 = cam8[6]; c.p2 = cam8[7];
        double sums[kSqpSums];
        for (int a = 0; a < kSqpSums; ++a) sums[a] = 0;
        for (int b0 = 0; b0 < N; b0 += kEpnpBlock) {   // mcv_epnp_pass's order: blocks, each from 0
            const int b1 = std::min(N, b0 + kEpnpBlock);
            double part[kSqpSums];
            for (int a = 0; a < kSqpSums; ++a) part[a] = 0;
            for (int i = b0; i < b1; ++i) {
                double x, y;
                pnp_undistort(c, img[2 * (size_t)i], img[2 * (size_t)i + 1], x, y);
                const double* P = world + 3 * (size_t)i;
                for (int a = 0; a < kSqpSums; ++a) part[a] += sqpnp_term(x, y, P[0], P[1], P[2], a);
            }
            for (int a = 0; a < kSqpSums; ++a) sums[a] += part[a];
        }
        auto npos = [&](const double* rh, const double* t) {
            int k = 0;
            for (int i = 0; i < N; ++i) {
                const double* P = world + 3 * (size_t)i;
                k += rh[6] * P[0] + rh[7] * P[1] + rh[8] * P[2] + t[2] > 0;
            }
            return k;
        };
        double rh[9], t[3];
        const int r = sqpnp_from_sums(sums, N, npos, rh, t);
        if (r > 0) {
            std::memcpy(R9, rh, sizeof(rh));
            std::memcpy(t3, t, sizeof(t));
        }
        return r;
    })
}

extern "C" MCV_API void cvRefinePnPLM(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                                      const double* distortionCoeffs, mcvV3d* tVec, mcvV3d* rVec) {
    try {
        clear_last_error();
        refine_common(imgPoints, worldPoints, N, K, distortionCoeffs, tVec, rVec, false);
    } catch (const std::exception& e) {
        set_last_error(e.what());
    }
}

extern "C" MCV_API void cvRefinePnPVVS(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N,
                                       const mcvM33d K, const double* distortionCoeffs, mcvV3d* tVec, mcvV3d* rVec) {
    try {
        clear_last_error();
        refine_common(imgPoints, worldPoints, N, K, distortionCoeffs, tVec, rVec, true);
    } catch (const std::exception& e) {
        set_last_error(e.what());
    }
}

extern "C" MCV_API int solveAp3p(mcvM33d* Rs, mcvV3d* ts, double mu0, double mv0, double X0, double Y0, double Z0,
                                 double mu1, double mv1, double X1, double Y1, double Z1, double mu2, double mv2,
                                 double X2, double Y2, double Z2, double inv_fx, double inv_fy, double cx_fx,
                                 double cy_fy) {
    MCV_GUARD(0, {
        if (!Rs || !ts) fail("solveAp3p: null argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_PNP);
        hipStream_t s = P.own_stream();
        P.reserve(4, 1);
        Ap3pIn in;
        const double mu[3] = {mu0, mu1, mu2}, mv[3] = {mv0, mv1, mv2};
        const double W[3][3] = {{X0, Y0, Z0}, {X1, Y1, Z1}, {X2, Y2, Z2}};
        for (int i = 0; i < 3; ++i) {
            in.mu[i] = mu[i];
            in.mv[i] = mv[i];
            for (int k = 0; k < 3; ++k) in.W[i][k] = W[i][k];
        }
        in.inv_fx = inv_fx; in.inv_fy = inv_fy; in.cx_fx = cx_fx; in.cy_fy = cy_fy;
        P.one.ensure(sizeof(Ap3pOut));
        P.h_one.ensure(sizeof(Ap3pOut));
        launch_pnp_ap3p(in, (Ap3pOut*)P.one.p, s);
        MCV_HIP(hipGetLastError());
        Ap3pOut out;
        MCV_HIP(hipMemcpyAsync(P.h_one.p, P.one.p, sizeof(Ap3pOut), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        std::memcpy(&out, P.h_one.p, sizeof(Ap3pOut));
        for (int k = 0; k < out.count; ++k) {
            for (int j = 0; j < 9; ++j) Rs[k].M[j] = out.R[k][j];
            ts[k].X = out.t[k][0]; ts[k].Y = out.t[k][1]; ts[k].Z = out.t[k][2];
        }
        return out.count;
    })
}

// Host build of the solveAp3p export's computation (bearings + ap3p_compute_poses_ref).
extern "C" MCV_API int mcvHostSolveAp3p(const double* mu3, const double* mv3, const double* W9, double inv_fx,
                                        double inv_fy, double cx_fx, double cy_fy, double* R36, double* t12) {
    double b[3][3], w[3][3];
    for (int i = 0; i < 3; ++i) {
        double mu = inv_fx * mu3[i] - cx_fx;
        double mv = inv_fy * mv3[i] - cy_fy;
        const double nrm = std::sqrt(mu * mu + mv * mv + 1);
        const double mk = 1. / nrm;
        mu = mu * mk;
        mv = mv * mk;
        b[i][0] = mu; b[i][1] = mv; b[i][2] = mk;
        for (int k = 0; k < 3; ++k) w[i][k] = W9[3 * i + k];
    }
    double Rr[kPnpMaxSolutions][9], tr[kPnpMaxSolutions][3];
    const int n = ap3p_compute_poses_ref(b, w, Rr, tr);
    for (int s = 0; s < n; ++s) {
        for (int k = 0; k < 9; ++k) R36[9 * s + k] = Rr[s][k];
        for (int k = 0; k < 3; ++k) t12[3 * s + k] = tr[s][k];
    }
    return n;
}

extern "C" MCV_API int mcvPackPnP(const mcvV2d* img, const mcvV3d* world, int N, void* d_pts, void* stream) {
    MCV_GUARD(0, {
        if (!img || !world || !d_pts || N < 0) fail("mcvPackPnP: bad argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_PNP);
        pnp_pack(P, img, world, N, d_pts, (hipStream_t)stream);
        MCV_HIP(hipStreamSynchronize((hipStream_t)stream));
        return 1;
    })
}

extern "C" MCV_API int mcvRansacPlanSetCamera(mcvRansacPlan* plan, const double* K9, const double* dist4) {
    MCV_GUARD(0, {
        Plan* P = reinterpret_cast<Plan*>(plan);
        if (!P || !K9) fail("mcvRansacPlanSetCamera: null argument");
        set_camera(*P, K9, dist4);
        return 1;
    })
}

// ---- host twins (test hooks) ------------------------------------------------------------------
extern "C" MCV_API void mcvHostRodrigues(const double* r, double* R, double* dR27) { rodrigues(r, R, dR27); }
extern "C" MCV_API void mcvHostRodriguesInv(const double* R, double* r) { rodrigues_inv(R, r); }

static int host_pnp(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R9, double* t3,
                    int* idx4, bool fast) {
    if (!pts || !cam8 || !R9 || !t3 || N < 4) fail("mcvHostPnP: bad argument");
    PnpCamera c{cam8[0], cam8[1], cam8[2], cam8[3], cam8[4], cam8[5], cam8[6], cam8[7]};
    PnpPose p;
    for (int k = 0; k < 9; ++k) p.R[k] = 0;
    for (int k = 0; k < 3; ++k) p.t[k] = 0;
    const int st = pnp_hypothesis((const PnpPoint*)pts, N, c, Sampler{seed, nullptr}, (uint64_t)hyp, p, idx4, fast);
    for (int k = 0; k < 9; ++k) R9[k] = p.R[k];
    for (int k = 0; k < 3; ++k) t3[k] = p.t[k];
    return st;
}

extern "C" MCV_API int mcvHostPnP(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R9,
                                  double* t3, int* idx4) {
    MCV_GUARD(kStatusNoSample - 1, { return host_pnp(pts, N, cam8, seed, hyp, R9, t3, idx4, false); })
}

extern "C" MCV_API int mcvHostPnPFast(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp,
                                      double* R9, double* t3, int* idx4) {
    MCV_GUARD(kStatusNoSample - 1, { return host_pnp(pts, N, cam8, seed, hyp, R9, t3, idx4, true); })
}

extern "C" MCV_API int mcvHostPnPEpnp(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp,
                                      double* R9, double* t3, int* idx5) {
    MCV_GUARD(kStatusNoSample - 1, {
        if (!pts || !cam8 || !R9 || !t3 || N < 5) fail("mcvHostPnPEpnp: bad argument");
        PnpCamera c{cam8[0], cam8[1], cam8[2], cam8[3], cam8[4], cam8[5], cam8[6], cam8[7]};
        PnpPose p;
        for (int k = 0; k < 9; ++k) p.R[k] = 0;
        for (int k = 0; k < 3; ++k) p.t[k] = 0;
        const int st = pnp_hypothesis_epnp((const PnpPoint*)pts, N, c, Sampler{seed, nullptr}, (uint64_t)hyp, p, idx5);
        for (int k = 0; k < 9; ++k) R9[k] = p.R[k];
        for (int k = 0; k < 3; ++k) t3[k] = p.t[k];
        return st;
    })
}

// Host build of epnp_solve_small<5> (pw: 5 x 3 world points, us: 5 x 2 pixels, cam4 = fu, fv, uc, vc).
extern "C" MCV_API void mcvHostEpnp5(const double* pw15, const double* us10, const double* cam4, double* R9,
                                     double* t3) {
    double pw[5][3], us[5][2], R[3][3], t[3];
    for (int i = 0; i < 5; ++i) {
        for (int k = 0; k < 3; ++k) pw[i][k] = pw15[3 * i + k];
        for (int k = 0; k < 2; ++k) us[i][k] = us10[2 * i + k];
    }
    epnp_solve_small<5>(pw, us, EpnpCam{cam4[0], cam4[1], cam4[2], cam4[3]}, R, t);
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) R9[3 * i + j] = R[i][j];
        t3[i] = t[i];
    }
}

// Test hook: the device's per-hypothesis poses. pts: host PnpPoint[N] (8 floats each); kind: the
// solverKind (EPnP kernel unless 2 / 5). Writes poses12[h] = {R (9), t (3)} and status[h] (1 or a
// kStatus* code). Returns hypCount, -1 on failure.
extern "C" MCV_API int mcvTestPnpHypotheses(const float* pts, int N, const double* cam8, uint64_t seed,
                                            int64_t hypBegin, int hypCount, int kind, double* poses12,
                                            int* status) {
    MCV_GUARD(-1, {
        if (!pts || !cam8 || !poses12 || !status || N < 5 || hypCount <= 0) fail("mcvTestPnpHypotheses: bad argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_PNP);
        hipStream_t s = P.own_stream();
        P.reserve(N, hypCount);
        for (int k = 0; k < 8; ++k) P.pnpCam[k] = cam8[k];
        MCV_HIP(hipMemcpyAsync(P.ptsd.p, pts, (size_t)N * sizeof(PnpPoint), hipMemcpyHostToDevice, s));
        const bool fast = (kind & MCV_HOST_FAST_MINIMAL) != 0;
        kind &= ~MCV_HOST_FAST_MINIMAL;
        pnp_generate_exact(P, P.ptsd.p, N, Sampler{seed, nullptr}, hypBegin, hypCount, pnp_kind_epnp(pnp_kind(kind)),
                           fast, P.models.p, P.counts.p, s);
        std::vector<PnpPose> m((size_t)hypCount);
        MCV_HIP(hipMemcpyAsync(m.data(), P.models.p, m.size() * sizeof(PnpPose), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipMemcpyAsync(status, P.counts.p, (size_t)hypCount * sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        P.last.clear();
        for (int h = 0; h < hypCount; ++h) {
            if (status[h] == 0) status[h] = 1;
            for (int k = 0; k < 9; ++k) poses12[12 * (size_t)h + k] = status[h] == 1 ? m[h].R[k] : 0.0;
            for (int k = 0; k < 3; ++k) poses12[12 * (size_t)h + 9 + k] = status[h] == 1 ? m[h].t[k] : 0.0;
        }
        return hypCount;
    })
}

extern "C" MCV_API int mcvTestPnpSweep(const float* pts, int N, const double* cam8, const double* poses12, int nPoses,
                                       float thr2, int fused, int mode, int* counts) {
    MCV_GUARD(-1, {
        if (!pts || !cam8 || !poses12 || !counts || N <= 0 || nPoses <= 0) fail("mcvTestPnpSweep: bad argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_PNP);
        hipStream_t s = P.own_stream();
        P.reserve(N, nPoses);
        for (int k = 0; k < 8; ++k) P.pnpCam[k] = cam8[k];
        MCV_HIP(hipMemcpyAsync(P.ptsd.p, pts, (size_t)N * sizeof(PnpPoint), hipMemcpyHostToDevice, s));
        std::vector<PnpPose> m((size_t)nPoses);
        for (int h = 0; h < nPoses; ++h) {
            for (int k = 0; k < 9; ++k) m[h].R[k] = poses12[12 * (size_t)h + k];
            for (int k = 0; k < 3; ++k) m[h].t[k] = poses12[12 * (size_t)h + 9 + k];
        }
        MCV_HIP(hipMemcpyAsync(P.models.p, m.data(), m.size() * sizeof(PnpPose), hipMemcpyHostToDevice, s));
        MCV_HIP(hipMemsetAsync(P.counts.p, 0, (size_t)nPoses * sizeof(int), s));
        P.bb4.ensure(4);
        P.pairs.ensure((size_t)(N + 1) * kPnpPairFloatsPerPoint);
        launch_pnp_extent(P.ptsd.p, N, P.bb4.p, P.pairs.p, s);
        launch_pnp_verify(P.ptsd.p, N, P.pnpCam, P.models.p, P.counts.p, nPoses, thr2, fused != 0,
                          mode == 0 ? P.bb4.p : nullptr, P.pairs.p, s);
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipMemcpyAsync(counts, P.counts.p, (size_t)nPoses * sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        P.last.clear();
        return nPoses;
    });
}

// fused bit 1 (value 2): the cheap tier alone (its decided lanes must equal the exact test too).
extern "C" MCV_API int mcvHostPnpCert(const float* pts, int N, const double* cam8, const double* R9, const double* t3,
                                      float thr2, int fused, int* decision, int* exact) {
    const int tiers = (fused & 2) ? 1 : 3;
    fused &= 1;
    const PnpPoint* q = (const PnpPoint*)pts;
    double ext[3] = {0, 0, 0};
    for (int i = 0; i < N; ++i) {
        const double v[3] = {q[i].X, q[i].Y, q[i].Z};
        for (int k = 0; k < 3; ++k) ext[k] = std::isfinite(v[k]) ? std::fmax(ext[k], std::fabs(v[k])) : INFINITY;
    }
    const PnpPkCam pc = pnp_pk_cam_host(cam8, thr2);
    PnpPkPose pp;
    pnp_pk_pose(R9, t3, ext, pc, pp);
    PnpCamera cam{cam8[0], cam8[1], cam8[2], cam8[3], cam8[4], cam8[5], cam8[6], cam8[7]};
    int bad = 0;
    for (int i = 0; i < N; ++i) {
        const int d = pc.ok ? pnp_pk_decide_host(pc, pp, q[i].X, q[i].Y, q[i].Z, q[i].u, q[i].v, tiers) : -1;
        const int e = pnp_error(cam, R9, t3, q[i].X, q[i].Y, q[i].Z, q[i].u, q[i].v, fused != 0) <= thr2 ? 1 : 0;
        decision[i] = d;
        exact[i] = e;
        if (d >= 0 && d != e) ++bad;
    }
    return bad;
}


// Test hook: the glibc restatements of glibc_math.h over arrays (fn 0 cbrt(a), 1 hypot(a, b),
// 2 clog's real part of a + i b, 3 x^2 + y^2 - 1, 4 exp(a), 5 log(a), 6 log1p(a), 7 cos(a),
// 8 atan2(a, b)). Returns n, -1 on a bad fn.
extern "C" MCV_API int mcvHostGlibcMath(int fn, const double* a, const double* b, int n, double* out) {
    if (fn < 0 || fn > 8 || n < 0 || !a || !out || ((fn == 1 || fn == 2 || fn == 3 || fn == 8) && !b)) return -1;
    for (int i = 0; i < n; ++i) {
        switch (fn) {
            case 0: out[i] = glibc_cbrt(a[i]); break;
            case 1: out[i] = glibc_hypot(a[i], b[i]); break;
            case 2: out[i] = glibc_clog_re(a[i], b[i]); break;
            case 3: out[i] = glibc_x2y2m1(a[i], b[i]); break;
            case 4: out[i] = glibc_exp(a[i]); break;
            case 5: out[i] = glibc_log(a[i]); break;
            case 6: out[i] = glibc_log1p(a[i]); break;
            case 7: out[i] = glibc_cos(a[i]); break;
            default: out[i] = glibc_atan2(a[i], b[i]); break;
        }
    }
    return n;
}
