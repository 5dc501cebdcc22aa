// ransac_f_host.cpp — host side of cvFindFundamentalMat (new export; OpenCV 4.x
// cv::findFundamentalMat(points1, points2, FM_RANSAC / FM_8POINT, thr, conf, maxIters, mask)
// semantics, restated [ext]): the RANSAC result is the best hypothesis' model (OpenCV does not
// refit F on the inliers); FM_8POINT (method 0 here) fits all points.
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include "linalg.h"
#include "hyp_fundamental.h"
#include "hyp_f7.h"
#include "sampson_pk.h"
#include "plan.h"

#include <cmath>
#include <cfloat>
#include <cstring>

namespace mcv {

int f_error_kind(const RansacConfig& cfg) {
    const int e = cfg.errorKind == MCV_FERR_EPIPOLAR ? 1 : 0;
    return e * 2 + ((cfg.flags & MCV_FLAG_FUSED_ERROR) ? 0 : 1);
}

int f_finalize(Plan& P, const float* d_pts, int N, const RansacConfig& cfg, int64_t hyp, double* F, uint8_t* d_mask,
               hipStream_t s) {
    const double t = effective_threshold(cfg);
    const float thr2 = (float)(t * t);
    FOneOut* d_one = (FOneOut*)P.one.p;
    const bool fast = (cfg.flags & MCV_FLAG_FAST_MINIMAL) != 0;
    FOneOut one;
    const Sampler smp = P.sampler(cfg);
    if (!(cfg.flags & MCV_FLAG_SEVEN_POINT) && P.last.covers(hyp, smp, d_pts, N, fast ? 11 : 10)) {
        // the winner's model straight from the last chunk's buffer (the same code produced it) instead
        // of a single-lane re-solve (the eigen-solve's ~0.5 ms latency)
        const FModelD* d_m = (const FModelD*)P.models.p + (hyp - P.last.begin);
        MCV_HIP(hipMemcpyAsync(P.h_one.p, d_m, sizeof(FModelD), hipMemcpyDeviceToHost, s));
        queue_chunk_check(P, d_pts, N, s);
        MCV_HIP(hipStreamSynchronize(s));
        if (!chunk_fresh(P)) {   // the points changed since the chunk was evaluated: re-solve
            P.last.clear();
            return f_finalize(P, d_pts, N, cfg, hyp, F, d_mask, s);
        }
        std::memcpy(one.F, P.h_one.p, sizeof(FModelD));
        one.status = 1;
    } else {
        if (cfg.flags & MCV_FLAG_SEVEN_POINT) launch_f7_one(d_pts, N, smp, hyp, d_one, s);   // hyp = model slot
        else launch_f_one(d_pts, N, smp, hyp, d_one, s, fast);
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipMemcpyAsync(P.h_one.p, d_one, sizeof(FOneOut), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        std::memcpy(&one, P.h_one.p, sizeof(FOneOut));
    }
    if (one.status != 1) fail("winning hypothesis %lld has no model (status %d)", (long long)hyp, one.status);
    MCV_HIP(hipMemsetAsync(P.count.p, 0, sizeof(int), s));
    launch_f_mask(d_pts, N, one.F, thr2, f_error_kind(cfg), d_mask, P.count.p, s);
    MCV_HIP(hipGetLastError());
    MCV_HIP(hipMemcpyAsync(P.h_i.p, P.count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < 9; ++k) F[k] = one.F[k];
    return P.h_i.p[0];
}

// run8Point over all correspondences: GPU fp64 sums (centroids, Euclidean distances, A^T A), then the
// 9x9 eigen-solve (JacobiImpl_), rank 2 (JacobiSVD) and de-normalisation here. Returns N, or 0 if
// degenerate (a mean distance below FLT_EPSILON, or one of the 8 largest eigenvalues below
// DBL_EPSILON).
int f_fit_all(Plan& P, const float* d_pts, int N, hipStream_t s, double* F) {
    double sums[5];
    reduce_to_host(P, s, 5, sums, [&](double* part, double* red) { h_reduce_sums(d_pts, N, nullptr, part, red, s); });
    const double n = sums[4];
    const double t = 1. / n;
    double c4[4] = {sums[0] * t, sums[1] * t, sums[2] * t, sums[3] * t};   // c2x, c2y, c1x, c1y
    double dev[2];
    reduce_to_host(P, s, 2, dev, [&](double* part, double* red) { f_reduce_eucdev(d_pts, N, nullptr, c4, part, red, s); });
    double scale2 = dev[0] * t, scale1 = dev[1] * t;
    if (scale1 < FLT_EPSILON || scale2 < FLT_EPSILON) return 0;
    scale1 = std::sqrt(2.) / scale1;
    scale2 = std::sqrt(2.) / scale2;
    double s4[4] = {scale2, scale2, scale1, scale1};
    double ata[45];
    reduce_to_host(P, s, 45, ata, [&](double* part, double* red) { f_reduce_ata(d_pts, N, nullptr, c4, s4, part, red, s); });
    double A[81], w[9], V[81];
    int o = 0;
    for (int j = 0; j < 9; ++j)
        for (int k = j; k < 9; ++k) { A[j * 9 + k] = ata[o]; A[k * 9 + j] = ata[o]; ++o; }
    jacobi_eigen(A, 9, w, V);
    int i = 0;
    for (; i < 9; ++i)
        if (std::fabs(w[i]) < DBL_EPSILON) break;
    if (i < 8) return 0;
    double F0[9];
    for (int k = 0; k < 9; ++k) F0[k] = V[8 * 9 + k];
    f_rank2(F0);
    if (!f_denormalize(F0, c4[2], c4[3], s4[2], s4[3], c4[0], c4[1], s4[0], s4[1], F)) return 0;
    return N;
}

int f_host_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F9, float* Ff9, int* sampleIdx,
                      bool fast) {
    if (N < 8) fail("N < 8");
    for (int k = 0; k < 9; ++k) F9[k] = 0;
    EigWsLocal ws;
    const int st = f_hypothesis(pts4, N, Sampler{seed, nullptr}, (uint64_t)hyp, F9, sampleIdx, ws, fast);
    for (int k = 0; k < 9; ++k) Ff9[k] = (float)F9[k];
    return st;
}

}  // namespace mcv

using namespace mcv;

// Host build of one 7-point hypothesis (f7_hypothesis): F27 = up to 3 models, idx7 = the sample.
extern "C" MCV_API int mcvHostF7(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F27, int* idx7) {
    MCV_GUARD(kStatusNoSample - 1, {
        if (!pts4 || !F27 || N < 7) fail("mcvHostF7: bad argument");
        double F[kF7Slots][9];
        for (int s = 0; s < kF7Slots; ++s)
            for (int k = 0; k < 9; ++k) F[s][k] = 0.0;
        const int n = f7_hypothesis(pts4, N, Sampler{seed, nullptr}, (uint64_t)hyp, F, idx7);
        for (int s = 0; s < kF7Slots; ++s)
            for (int k = 0; k < 9; ++k) F27[9 * s + k] = F[s][k];
        return n;
    })
}

// Host twin of the certified Sampson prefilter (sampson_pk.h) for one fp64 model over host float4 points
// {x1, y1, x2, y2}: decision[i] = 1 certified inlier, 0 certified outlier, -1 undecided; exact[i] = the
// fp64 test f_error(kind, ...) <= thr2 (kind 0 fused / 1 op-by-op Sampson). The point-set bound is the
// sweep's (max |coordinate| per column). Returns the number of decided points that differ from the
// exact test (must be 0).
extern "C" MCV_API int mcvHostSampsonCert(const float* pts4, int N, const double* F9, float thr2, int kind,
                                          int* decision, int* exact) {
    double bb[4] = {0, 0, 0, 0};
    for (int i = 0; i < N; ++i)
        for (int c = 0; c < 4; ++c) {
            const double v = pts4[4 * i + c];
            bb[c] = std::isfinite(v) ? std::fmax(bb[c], std::fabs(v)) : INFINITY;
        }
    const SampsonPkCut cut = sampson_pk_cut_host(sampson_cut(thr2));
    double Dm;
    const SampsonPkBound b = sampson_pk_bound(F9, bb[0], bb[1], bb[2], bb[3], &Dm);
    const SpkCut1 k = spk_cut1(b, Dm, cut.L32, cut.H32);
    float f[9];
    for (int j = 0; j < 9; ++j) f[j] = (float)F9[j];
    int bad = 0;
    for (int i = 0; i < N; ++i) {
        const float* q = pts4 + 4 * (size_t)i;
        const int d = spk_decide_host(f, k, q[0], q[1], q[2], q[3]);
        const int e = f_error(kind, F9, q[0], q[1], q[2], q[3]) <= thr2 ? 1 : 0;
        decision[i] = d;
        exact[i] = e;
        if (d >= 0 && d != e) ++bad;
    }
    return bad;
}
