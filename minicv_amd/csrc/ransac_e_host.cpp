// ransac_e_host.cpp — host side of the essential-matrix path behind the
// reference's own exports cvRecoverPose / cvRecoverPoses / cvFivePoint (MiniCVNative.cpp:165-215,
// 368-382) and the new cvFindEssentialMat.
//
// Semantics restated from OpenCV 4.x [ext, absent here; SURVEY.md §8c]:
//   findEssentialMat(p1, p2, focal, pp, RANSAC, prob, threshold, mask), maxIters 1000:
//     points -> (x - pp) / focal in fp64, threshold / focal, RANSACPointSetRegistrator with
//     EMEstimatorCallback (5-point minimal sets, up to 10 models per sample, Sampson error).
//     count == 5 -> one solve on all points, mask all 1.
//   decomposeEssentialMat(E) -> R1, R2, t.
//   recoverPose(E, p1, p2, R, t, focal, pp, mask): the 4 (R, +-t) candidates, DLT triangulation,
//     cheirality with distance 50 over the masked points, first maximum of the 4 counts.
// The sampling / replay / verify split is the same as for homographies (ransac_host.cpp).
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include "hyp_essential.h"
#include "plan.h"

#include <cmath>
#include <cstring>
#include <algorithm>

namespace mcv {

static const double kCheiralityDist = 50.0;   // recoverPose's distanceThresh for the focal/pp overload

static int e_kind(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_FUSED_ERROR) ? 0 : 1; }
// MCV_FLAG_FAST_MINIMAL: the replacement five-point solver (Gauss-Jordan null space, polynomial-product
// constraints, Illinois real roots) instead of the reference's (fivepoint.cpp / five_point_ref.h).
static bool e_fast(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_FAST_MINIMAL) != 0; }

void e_evaluate_chunk(Plan& P, const double* d_pts, int N, const RansacConfig& cfg, int64_t hypBegin, int hypCount,
                      int* d_counts, hipStream_t s) {
    const float thr2 = (float)(cfg.threshold * cfg.threshold);
    const Sampler smp = P.sampler(cfg);
    const bool fast = e_fast(cfg);
    {
        ProfScope pg("e_generate", s);
        if (fast) {   // opt-in: the Illinois replacement solver (hyp_essential.h / five_point_wave.h)
            if (hypCount >= kEStageMinHyps) P.estage.ensure((size_t)hypCount * sizeof(EStage));
            launch_e_generate(d_pts, N, smp, hypBegin, hypCount, P.models.p, P.dslot.p, P.ndense.p, d_counts,
                              hypCount >= kEStageMinHyps ? P.estage.p : nullptr, s);
        } else {      // default: the reference's own five-point solver (five_point_ref.h)
            P.estage.ensure(e5_stage_bytes(hypCount));
            launch_e5_generate(d_pts, N, smp, hypBegin, hypCount, P.models.p, P.dslot.p, P.ndense.p, d_counts,
                               P.estage.p, s);
        }
    }
    mark_chunk(P, hypBegin, hypCount, smp, d_pts, N, fast ? 31 : 30, s);
    P.bb4.ensure(4);
    P.pts.ensure((size_t)N * 4);
    launch_abs_bound4(d_pts, true, N, P.bb4.p, P.pts.p, s);   // fp32 copy + bounds for the prefilter
    ProfScope ps("e_verify", s);
    launch_e_verify(d_pts, N, P.models.p, P.dslot.p, P.ndense.p, hypCount * kEModelSlots, d_counts, thr2, e_kind(cfg),
                    s, P.pts.p, P.bb4.p);
}

static EOneOut e_one(Plan& P, const double* d_pts, int N, const Sampler& smp, int64_t hyp, bool fast,
                     hipStream_t s) {
    EOneOut* d_one = (EOneOut*)P.one.p;
    if (fast) launch_e_one(d_pts, N, smp, hyp, d_one, s);
    else launch_e5_one(d_pts, N, smp, hyp, d_one, s);
    MCV_HIP(hipGetLastError());
    EOneOut one;
    MCV_HIP(hipMemcpyAsync(P.h_one.p, d_one, sizeof(EOneOut), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    std::memcpy(&one, P.h_one.p, sizeof(EOneOut));
    return one;
}

static int e_mask_count(Plan& P, const double* d_pts, int N, const RansacConfig& cfg, const double* E,
                        uint8_t* d_mask, hipStream_t s) {
    const float thr2 = (float)(cfg.threshold * cfg.threshold);
    MCV_HIP(hipMemsetAsync(P.count.p, 0, sizeof(int), s));
    launch_e_mask(d_pts, N, E, thr2, e_kind(cfg), d_mask, P.count.p, s);
    MCV_HIP(hipGetLastError());
    MCV_HIP(hipMemcpyAsync(P.h_i.p, P.count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    return P.h_i.p[0];
}

// Winner (model slot) -> E and its mask. OpenCV keeps the best hypothesis' model as is.
int e_finalize(Plan& P, const double* d_pts, int N, const RansacConfig& cfg, int64_t slot, double* E,
               uint8_t* d_mask, hipStream_t s) {
    const int64_t hyp = slot / kEModelSlots;
    const int k = (int)(slot % kEModelSlots);
    bool have = false;
    const Sampler smp = P.sampler(cfg);
    if (P.last.covers(hyp, smp, d_pts, N, e_fast(cfg) ? 31 : 30)) {
        const int local = (int)((hyp - P.last.begin) * kEModelSlots + k);
        int* d_found = P.ndense.p + 7;
        uint8_t* d_out = P.one.p;
        launch_e_fetch(P.models.p, P.dslot.p, P.ndense.p, (int)(P.last.count * kEModelSlots), local, d_out, d_found, s);
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipMemcpyAsync(P.h_one.p, d_out, 9 * sizeof(double), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipMemcpyAsync(P.h_i.p, d_found, sizeof(int), hipMemcpyDeviceToHost, s));
        queue_chunk_check(P, d_pts, N, s);
        MCV_HIP(hipStreamSynchronize(s));
        if (!chunk_fresh(P)) P.last.clear();   // the points changed since the chunk was evaluated: re-solve
        else if (P.h_i.p[0] == 1) {
            std::memcpy(E, P.h_one.p, 9 * sizeof(double));
            have = true;
        }
    }
    if (!have) {
        const EOneOut one = e_one(P, d_pts, N, smp, hyp, e_fast(cfg), s);
        if (one.status <= k) fail("winning slot %lld has no model (status %d)", (long long)slot, one.status);
        for (int j = 0; j < 9; ++j) E[j] = one.E[k][j];
    }
    return e_mask_count(P, d_pts, N, cfg, E, d_mask, s);
}

// Upload the pixel pairs and normalise them on the device.
static void e_pack(Plan& P, const mcvV2d* a, const mcvV2d* b, int N, double focal, mcvV2d pp, double* d_out,
                   hipStream_t s) {
    if (!(focal != 0) || !std::isfinite(focal)) fail("focal length must be finite and non-zero (got %g)", focal);
    P.raw.ensure((size_t)N * 4);
    MCV_HIP(hipMemcpyAsync(P.raw.p, a, (size_t)N * sizeof(mcvV2d), hipMemcpyHostToDevice, s));
    MCV_HIP(hipMemcpyAsync(P.raw.p + 2 * (size_t)N, b, (size_t)N * sizeof(mcvV2d), hipMemcpyHostToDevice, s));
    launch_e_pack(P.raw.p, N, focal, pp.X, pp.Y, d_out, s);
    MCV_HIP(hipGetLastError());
}

// Five-point solve on the first 5 device-resident correspondences (count == modelPoints case).
static EOneOut e_solve_first5(Plan& P, const double* d_pts, hipStream_t s) {
    double h[20];
    MCV_HIP(hipMemcpyAsync(P.h_one.p, d_pts, 5 * 4 * sizeof(double), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    std::memcpy(h, P.h_one.p, sizeof(h));
    EFiveIn in;
    for (int i = 0; i < 5; ++i) {
        in.x1[i] = h[4 * i]; in.y1[i] = h[4 * i + 1]; in.x2[i] = h[4 * i + 2]; in.y2[i] = h[4 * i + 3];
    }
    EOneOut* d_one = (EOneOut*)P.one.p;
    launch_e_fivepoint(in, d_one, s);
    MCV_HIP(hipGetLastError());
    EOneOut one;
    MCV_HIP(hipMemcpyAsync(P.h_one.p, d_one, sizeof(EOneOut), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    std::memcpy(&one, P.h_one.p, sizeof(EOneOut));
    return one;
}

struct EResult {
    int count = 0;       // inliers (0: failed)
    int nmodels = 0;     // N == 5 path: number of solutions
    double E[9];
};

// findEssentialMat on host pixel pairs. cfg.threshold in pixels. Mask stays on the device (P.mask).
static EResult e_find(Plan& P, const mcvV2d* a, const mcvV2d* b, int N, double focal, mcvV2d pp,
                      const RansacConfig& cfgPix, hipStream_t s) {
    RansacConfig cfg = cfgPix;
    cfg.threshold = cfgPix.threshold / ((focal + focal) / 2);   // OpenCV: threshold /= (fx + fy) / 2
    P.reserve(N, 1);
    e_pack(P, a, b, N, focal, pp, P.ptsd.p, s);
    EResult r;
    if (N == 5) {
        const EOneOut one = e_solve_first5(P, P.ptsd.p, s);
        r.nmodels = std::max(one.status, 0);
        if (r.nmodels == 1) {
            for (int j = 0; j < 9; ++j) r.E[j] = one.E[0][j];
            r.count = 5;
        }
        launch_fill_u8(P.mask.p, N, 1, s);
        MCV_HIP(hipGetLastError());
        return r;
    }
    const int64_t best = ransac_search(P, P.ptsd.p, N, cfg, s);
    if (best < 0) return r;
    r.nmodels = 1;
    r.count = e_finalize(P, P.ptsd.p, N, cfg, best, r.E, P.mask.p, s);
    return r;
}

static RansacConfig e_config(const RansacConfig* cfgp) {
    if (cfgp) return *cfgp;
    RansacConfig c;
    std::memset(&c, 0, sizeof(c));
    c.threshold = 1.0;
    c.confidence = 0.999;
    c.maxIters = 1000;
    c.method = MCV_METHOD_RANSAC;
    c.flags = MCV_FLAG_CV_SAMPLER;   // OpenCV's own sample stream (no seed in the reference's API)
    return c;
}

static RansacConfig e_config(const RecoverPoseConfig* rc) {
    RansacConfig c = e_config((const RansacConfig*)nullptr);
    c.threshold = rc->InlierThreshold;
    c.confidence = rc->Probability;
    return c;
}

static void e_check(const RansacConfig& cfg, const char* who) {
    check_flags(cfg, who);
    if (cfg.method != MCV_METHOD_RANSAC) fail("%s: only RANSAC (method 8) is supported for E", who);
    if (!(cfg.confidence > 0 && cfg.confidence < 1)) fail("%s: confidence must be in (0,1)", who);
}

// recoverPose: decompose E, count the masked correspondences passing each candidate's cheirality
// test on the GPU, keep the first maximum (good1 >= others, then good2, good3, else 4).
static int e_recover(Plan& P, int N, const double* E, const uint8_t* d_mask, double* R, double* t, hipStream_t s) {
    double R1[9], R2[9], t0[3];
    e_decompose(E, R1, R2, t0);
    double P4[4][12];
    const double* Rs[4] = {R1, R2, R1, R2};
    const double sg[4] = {1, 1, -1, -1};
    for (int k = 0; k < 4; ++k) {
        for (int j = 0; j < 9; ++j) P4[k][j] = Rs[k][j];
        for (int j = 0; j < 3; ++j) P4[k][9 + j] = sg[k] > 0 ? t0[j] : -t0[j];
    }
    launch_e_cheirality(P.ptsd.p, N, d_mask, &P4[0][0], kCheiralityDist, P.ndense.p + 4, s);
    MCV_HIP(hipGetLastError());
    P.h_i.ensure(8);
    MCV_HIP(hipMemcpyAsync(P.h_i.p, P.ndense.p + 4, 4 * sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    const int g[4] = {P.h_i.p[0], P.h_i.p[1], P.h_i.p[2], P.h_i.p[3]};
    int pick = 3;
    if (g[0] >= g[1] && g[0] >= g[2] && g[0] >= g[3]) pick = 0;
    else if (g[1] >= g[0] && g[1] >= g[2] && g[1] >= g[3]) pick = 1;
    else if (g[2] >= g[0] && g[2] >= g[1] && g[2] >= g[3]) pick = 2;
    for (int j = 0; j < 9; ++j) R[j] = P4[pick][j];
    for (int j = 0; j < 3; ++j) t[j] = P4[pick][9 + j];
    return g[pick];
}

}  // namespace mcv

using namespace mcv;

extern "C" MCV_API int cvFindEssentialMat(const mcvV2d* a, const mcvV2d* b, const int N, double focal, mcvV2d pp,
                                          const RansacConfig* cfgp, mcvM33d* E, uint8_t* mask) {
    MCV_GUARD(0, {
        if (!a || !b || !E || N < 0) fail("cvFindEssentialMat: null argument or negative N");
        if (mask) std::memset(mask, 0, (size_t)N);
        if (N < 5) fail("cvFindEssentialMat: need at least 5 correspondences (N=%d)", N);
        const RansacConfig cfg = e_config(cfgp);
        e_check(cfg, "cvFindEssentialMat");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_ESSENTIAL);
        hipStream_t s = P.own_stream();
        const EResult r = e_find(P, a, b, N, focal, pp, cfg, s);
        if (r.count <= 0) {
            if (N == 5) fail("cvFindEssentialMat: N == 5 gave %d solutions (OpenCV returns them stacked)", r.nmodels);
            fail("cvFindEssentialMat: RANSAC found no model with >= 5 inliers");
        }
        if (mask) {
            MCV_HIP(hipMemcpyAsync(mask, P.mask.p, (size_t)N, hipMemcpyDeviceToHost, s));
            MCV_HIP(hipStreamSynchronize(s));
        }
        for (int k = 0; k < 9; ++k) E->M[k] = r.E[k];
        return r.count;
    })
}

extern "C" MCV_API mcvBool cvRecoverPoses(const RecoverPoseConfig* config, const int N, const mcvV2d* pa,
                                       const mcvV2d* pb, mcvM33d* rMat1, mcvM33d* rMat2, mcvV3d* tVec, uint8_t* ms) {
    MCV_GUARD(false, {
        if (N < 5) return false;   // MiniCVNative.cpp:167
        if (!config || !pa || !pb || !rMat1 || !rMat2 || !tVec || !ms) fail("cvRecoverPoses: null argument");
        const RansacConfig cfg = e_config(config);
        e_check(cfg, "cvRecoverPoses");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_ESSENTIAL);
        hipStream_t s = P.own_stream();
        const EResult r = e_find(P, pa, pb, N, config->FocalLength, config->PrincipalPoint, cfg, s);
        if (r.nmodels == 0) { set_last_error("cvRecoverPoses: no essential matrix"); return false; }
        MCV_HIP(hipMemcpyAsync(ms, P.mask.p, (size_t)N, hipMemcpyDeviceToHost, s));   // :179-183
        MCV_HIP(hipStreamSynchronize(s));
        if (r.count <= 0) { set_last_error("cvRecoverPoses: E is not 3x3 (several N == 5 solutions)"); return false; }
        double t[3];
        e_decompose(r.E, rMat1->M, rMat2->M, t);   // :186
        tVec->X = t[0]; tVec->Y = t[1]; tVec->Z = t[2];
        return true;
    })
}

extern "C" MCV_API int cvRecoverPose(const RecoverPoseConfig* config, const int N, const mcvV2d* pa, const mcvV2d* pb,
                                     mcvM33d* rMat, mcvV3d* tVec, uint8_t* ms) {
    MCV_GUARD(0, {
        if (!config || !pa || !pb || !rMat || !tVec || !ms || N < 0) fail("cvRecoverPose: null argument");
        if (N < 5) fail("cvRecoverPose: need at least 5 correspondences (N=%d)", N);
        const RansacConfig cfg = e_config(config);
        e_check(cfg, "cvRecoverPose");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_ESSENTIAL);
        hipStream_t s = P.own_stream();
        const EResult r = e_find(P, pa, pb, N, config->FocalLength, config->PrincipalPoint, cfg, s);
        if (r.nmodels == 0) fail("cvRecoverPose: no essential matrix");
        MCV_HIP(hipMemcpyAsync(ms, P.mask.p, (size_t)N, hipMemcpyDeviceToHost, s));   // :206-210
        MCV_HIP(hipStreamSynchronize(s));
        if (r.count <= 0) fail("cvRecoverPose: E is not 3x3 (several N == 5 solutions)");
        double t[3];
        const int good = e_recover(P, N, r.E, P.mask.p, rMat->M, t, s);   // :212
        tVec->X = t[0]; tVec->Y = t[1]; tVec->Z = t[2];
        return good;
    })
}

extern "C" MCV_API int cvFivePoint(const mcvV2d* pa, const mcvV2d* pb, mcvM33d* Es) {
    MCV_GUARD(0, {
        if (!pa || !pb || !Es) fail("cvFivePoint: null argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_ESSENTIAL);
        hipStream_t s = P.own_stream();
        P.reserve(5, 1);
        EFiveIn in;
        for (int i = 0; i < 5; ++i) { in.x1[i] = pa[i].X; in.y1[i] = pa[i].Y; in.x2[i] = pb[i].X; in.y2[i] = pb[i].Y; }
        EOneOut* d_one = (EOneOut*)P.one.p;
        launch_e_fivepoint(in, d_one, s);
        MCV_HIP(hipGetLastError());
        EOneOut one;
        MCV_HIP(hipMemcpyAsync(P.h_one.p, d_one, sizeof(EOneOut), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        std::memcpy(&one, P.h_one.p, sizeof(EOneOut));
        const int n = std::max(one.status, 0);
        for (int k = 0; k < n; ++k)
            for (int j = 0; j < 9; ++j) Es[k].M[j] = one.E[k][j];
        return n;
    })
}

extern "C" MCV_API int mcvPackEssential(const mcvV2d* a, const mcvV2d* b, int N, double focal, mcvV2d pp,
                                        double* d_pts4, void* stream) {
    MCV_GUARD(0, {
        if (!a || !b || !d_pts4 || N < 0) fail("mcvPackEssential: bad argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_ESSENTIAL);
        e_pack(P, a, b, N, focal, pp, d_pts4, (hipStream_t)stream);
        MCV_HIP(hipStreamSynchronize((hipStream_t)stream));
        return 1;
    })
}

// ---- host twins (test hooks) -------------------------------------------------------------------
// Host twin with the opt-in replacement solver (MCV_FLAG_FAST_MINIMAL).
extern "C" MCV_API int mcvHostEssentialFast(const double* pts4, int N, uint64_t seed, int64_t hyp, double* E90,
                                            int* sampleIdx) {
    MCV_GUARD(kStatusNoSample - 1, {
        if (!pts4 || !E90 || N < 5) fail("mcvHostEssentialFast: bad argument");
        double E[kEMaxModels][9];
        const int n = e_hypothesis(pts4, N, Sampler{seed, nullptr}, (uint64_t)hyp, E, sampleIdx);
        for (int s = 0; s < kEMaxModels; ++s)
            for (int k = 0; k < 9; ++k) E90[9 * s + k] = s < n ? E[s][k] : 0.0;
        return n;
    })
}

extern "C" MCV_API int mcvHostFivePoint(const double* p20, double* E90) {
    MCV_GUARD(-1, {
        if (!p20 || !E90) fail("mcvHostFivePoint: null argument");
        double E[kEMaxModels][9];
        const int n = e_solve5(p20, p20 + 5, p20 + 10, p20 + 15, E);
        for (int s = 0; s < kEMaxModels; ++s)
            for (int k = 0; k < 9; ++k) E90[9 * s + k] = s < n ? E[s][k] : 0.0;
        return n;
    })
}

extern "C" MCV_API int mcvHostRealRoots(const double* c, int deg, int fixed, double* roots) {
    MCV_GUARD(-1, {
        if (!c || !roots || deg < 0 || deg > 10 || (fixed && deg != 4)) fail("mcvHostRealRoots: bad arguments");
        if (fixed) {
            const double c5[5] = {c[0], c[1], c[2], c[3], c[4]};
            double r4[4];
            const int n = e_poly_real_roots_fixed<4>(c5, r4);
            for (int k = 0; k < n; ++k) roots[k] = r4[k];
            return n;
        }
        return e_poly_real_roots(c, deg, roots);
    })
}

extern "C" MCV_API void mcvHostDecomposeEssential(const double* E9, double* R1, double* R2, double* t3) {
    e_decompose(E9, R1, R2, t3);
}
