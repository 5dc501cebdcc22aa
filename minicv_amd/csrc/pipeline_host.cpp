// pipeline_host.cpp — cvMatchFeatures / cvMatchAndFindModel: descriptors of
// two DetectorResults go to the GPU once; knn-2 matching, filtering, compaction, the gather of
// matched keypoints into float4 correspondences and the RANSAC search all run on device-resident
// buffers; only the pair list, the mask and the model come back.
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include "plan.h"

#include <climits>
#include <cstring>

namespace mcv {

namespace {
struct PipeWork {
    DevBuf<uint8_t> da, db, kpa, kpb, keep;
    DevBuf<int> idx, di1, di2, idxBack, diBack, cnt, off, pairs;
    DevBuf<float> df1, df2, dfBack, dist;
    PinnedBuf<int> h_total;
};
PipeWork& pipe_work() {
    thread_local PipeWork w;
    return w;
}

const int kElemU8 = 0, kElemF32 = 5;

void check_result(const DetectorResult* r, const char* who, const char* which) {
    if (!r) fail("%s: %s is NULL", who, which);
    if (r->PointCount < 0 || r->DescriptorEntries < 0) fail("%s: %s has negative sizes", who, which);
    if (r->PointCount > 0 && (!r->Points || !r->Descriptors)) fail("%s: %s has NULL arrays", who, which);
    if (r->PointCount > 0 && r->DescriptorEntries % r->PointCount != 0)
        fail("%s: %s DescriptorEntries %d not a multiple of PointCount %d", who, which, r->DescriptorEntries,
             r->PointCount);
}
}  // namespace

// Match a -> b on the GPU and compact the surviving pairs in query order. Device outputs:
// w.pairs (2 per match), w.dist, pts4 (float4 per match, written to d_pts4). Returns the count.
static int match_compact(const DetectorResult* a, const DetectorResult* b, const MatchConfig& cfg, PipeWork& w,
                         float* d_pts4_or_null, Plan* P, hipStream_t s, const char* who) {
    check_result(a, who, "a");
    check_result(b, who, "b");
    const int na = a->PointCount, nb = b->PointCount;
    if (na == 0 || nb == 0) return 0;
    if (a->DescriptorElementType != b->DescriptorElementType)
        fail("%s: descriptor element types differ (%d vs %d)", who, a->DescriptorElementType, b->DescriptorElementType);
    const int dim = a->DescriptorEntries / na;
    if (b->DescriptorEntries / nb != dim) fail("%s: descriptor widths differ", who);
    const bool ham = a->DescriptorElementType == kElemU8;
    if (!ham && a->DescriptorElementType != kElemF32)
        fail("%s: descriptor element type %d unsupported (0 = uint8 Hamming, 5 = float32 L2)", who,
             a->DescriptorElementType);
    const size_t esz = ham ? 1 : 4;
    w.da.ensure((size_t)a->DescriptorEntries * esz);
    w.db.ensure((size_t)b->DescriptorEntries * esz);
    w.kpa.ensure((size_t)na * sizeof(KeyPoint2d));
    w.kpb.ensure((size_t)nb * sizeof(KeyPoint2d));
    MCV_HIP(hipMemcpyAsync(w.da.p, a->Descriptors, (size_t)a->DescriptorEntries * esz, hipMemcpyHostToDevice, s));
    MCV_HIP(hipMemcpyAsync(w.db.p, b->Descriptors, (size_t)b->DescriptorEntries * esz, hipMemcpyHostToDevice, s));
    MCV_HIP(hipMemcpyAsync(w.kpa.p, a->Points, (size_t)na * sizeof(KeyPoint2d), hipMemcpyHostToDevice, s));
    MCV_HIP(hipMemcpyAsync(w.kpb.p, b->Points, (size_t)nb * sizeof(KeyPoint2d), hipMemcpyHostToDevice, s));
    w.idx.ensure(na);
    w.keep.ensure(na);
    const int nblk = (na + 255) / 256;
    w.cnt.ensure(nblk);
    w.off.ensure(nblk + 1);
    w.pairs.ensure((size_t)2 * na);
    w.dist.ensure(na);
    int* idxBack = nullptr;
    if (ham) {
        w.di1.ensure(na); w.di2.ensure(na);
        launch_match_hamming(w.da.p, na, w.db.p, nb, dim, w.idx.p, w.di1.p, nullptr, w.di2.p, s);
        if (cfg.crossCheck) {
            w.idxBack.ensure(nb); w.diBack.ensure(nb);
            launch_match_hamming(w.db.p, nb, w.da.p, na, dim, w.idxBack.p, w.diBack.p, nullptr, nullptr, s);
            idxBack = w.idxBack.p;
        }
    } else {
        w.df1.ensure(na); w.df2.ensure(na);
        launch_match_l2((const float*)w.da.p, na, (const float*)w.db.p, nb, dim, w.idx.p, w.df1.p, nullptr, w.df2.p,
                        s);
        if (cfg.crossCheck) {
            w.idxBack.ensure(nb); w.dfBack.ensure(nb);
            launch_match_l2((const float*)w.db.p, nb, (const float*)w.da.p, na, dim, w.idxBack.p, w.dfBack.p, nullptr,
                            nullptr, s);
            idxBack = w.idxBack.p;
        }
    }
    float* d_pts4 = d_pts4_or_null;
    if (!d_pts4) {
        P->reserve(na, 1);
        d_pts4 = P->pts.p;
    }
    launch_match_compact(w.idx.p, ham ? w.di1.p : nullptr, ham ? w.di2.p : nullptr, ham ? nullptr : w.df1.p,
                         ham ? nullptr : w.df2.p, idxBack, na, cfg.ratio, cfg.maxDistance, w.kpa.p, w.kpb.p,
                         (int)sizeof(KeyPoint2d), w.keep.p, w.cnt.p, w.off.p, w.pairs.p, w.dist.p, d_pts4, s);
    MCV_HIP(hipGetLastError());
    w.h_total.ensure(1);
    MCV_HIP(hipMemcpyAsync(w.h_total.p, w.off.p + nblk, sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    return w.h_total.p[0];
}

}  // namespace mcv

using namespace mcv;

extern "C" MCV_API int cvMatchFeatures(const DetectorResult* a, const DetectorResult* b, const MatchConfig* cfgp,
                                       int* pairs, float* dist, int maxPairs) {
    MCV_GUARD(-1, {
        if (!pairs) fail("cvMatchFeatures: pairs is NULL");
        MatchConfig cfg = cfgp ? *cfgp : MatchConfig{0.8f, 0, 0.f, MCV_MODEL_HOMOGRAPHY};
        require_device();
        Plan& P = thread_plan(MCV_MODEL_HOMOGRAPHY);
        hipStream_t s = P.own_stream();
        PipeWork& w = pipe_work();
        const int n = match_compact(a, b, cfg, w, nullptr, &P, s, "cvMatchFeatures");
        if (n > maxPairs) fail("cvMatchFeatures: %d matches exceed maxPairs %d", n, maxPairs);
        if (n > 0) {
            MCV_HIP(hipMemcpyAsync(pairs, w.pairs.p, (size_t)2 * n * sizeof(int), hipMemcpyDeviceToHost, s));
            if (dist) MCV_HIP(hipMemcpyAsync(dist, w.dist.p, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s));
            MCV_HIP(hipStreamSynchronize(s));
        }
        return n;
    })
}

extern "C" MCV_API int cvMatchAndFindModel(const DetectorResult* a, const DetectorResult* b, const MatchConfig* mcfgp,
                                           const RansacConfig* rcfgp, mcvM33d* M, int* pairs, uint8_t* mask,
                                           int maxPairs, int* matchCount) {
    MCV_GUARD(0, {
        if (matchCount) *matchCount = 0;
        if (!M || !pairs || !mask) fail("cvMatchAndFindModel: null argument");
        const MatchConfig mcfg = mcfgp ? *mcfgp : MatchConfig{0.8f, 0, 0.f, MCV_MODEL_HOMOGRAPHY};
        if (mcfg.model != MCV_MODEL_HOMOGRAPHY && mcfg.model != MCV_MODEL_FUNDAMENTAL)
            fail("cvMatchAndFindModel: model %d unsupported (homography or fundamental)", mcfg.model);
        RansacConfig rcfg = config_or_default(rcfgp);
        if (!rcfgp && mcfg.model == MCV_MODEL_FUNDAMENTAL) rcfg.confidence = 0.99;
        if (rcfg.method != MCV_METHOD_RANSAC) fail("cvMatchAndFindModel: only RANSAC (method 8)");
        check_flags(rcfg, "cvMatchAndFindModel");
        if (!(rcfg.confidence > 0 && rcfg.confidence < 1)) fail("cvMatchAndFindModel: confidence must be in (0,1)");
        require_device();
        Plan& P = thread_plan(mcfg.model);
        hipStream_t s = P.own_stream();
        PipeWork& w = pipe_work();
        const int n = match_compact(a, b, mcfg, w, nullptr, &P, s, "cvMatchAndFindModel");
        if (n > maxPairs) fail("cvMatchAndFindModel: %d matches exceed maxPairs %d", n, maxPairs);
        if (matchCount) *matchCount = n;
        if (n > 0) MCV_HIP(hipMemcpyAsync(pairs, w.pairs.p, (size_t)2 * n * sizeof(int), hipMemcpyDeviceToHost, s));
        std::memset(mask, 0, (size_t)(n > 0 ? n : 0));
        const int m = model_points(mcfg.model);
        if (n < m) {
            MCV_HIP(hipStreamSynchronize(s));
            fail("cvMatchAndFindModel: %d matches, need at least %d", n, m);
        }
        P.reserve(n, 1);
        const int64_t best = ransac_search(P, P.pts.p, n, rcfg, s);
        if (best < 0) fail("cvMatchAndFindModel: RANSAC found no model with >= %d inliers", m);
        double model9[9];
        const int count = finalize(P, P.pts.p, n, rcfg, best, model9, P.mask.p, s);
        MCV_HIP(hipMemcpyAsync(mask, P.mask.p, (size_t)n, hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        for (int k = 0; k < 9; ++k) M->M[k] = model9[k];
        return count;
    })
}
