// cv_sampler.cpp — OpenCV's own RANSAC sample stream (MCV_FLAG_CV_SAMPLER; the default of the
// reference-signature exports cvRecoverPose(s) and cvSolvePnPRansac, which take no seed).
//
// The reference's RANSAC runs inside cv::findEssentialMat (MiniCVNative.cpp:177,204) and
// cv::solvePnPRansac (MiniCVNative.cpp:125), i.e. RANSACPointSetRegistrator::run [ext: OpenCV 4.x
// calib3d/src/ptsetreg.cpp]: one `RNG rng((uint64)-1)` per call, and per iteration
// getSubset(m1, m2, ms1, ms2, rng, 10000): up to 10000 attempts, each drawing modelPoints indices
// with rng.uniform(0, count), an index equal to an earlier one of the same attempt drawn again, then
// the callback's checkSubset on the gathered subset (homography: collinearity of either point set
// + the orientation consistency of the 4 triangles; fundamental: collinearity; essential / PnP:
// none). No draw depends on a model or an inlier count, so the whole stream is a function of the
// point set alone: it is generated here, sequentially, before the GPU evaluates the hypotheses
// (microseconds for the reference's maxIters <= a few thousand), and the generate kernels read
// row h instead of the Philox stream (mcv_common.h SubsetSrc). The checks are the same host-compiled
// functions the kernels run (hyp_homography.h, hyp_fundamental.h), on the same float4 points.
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "mcv_common.h"
#include "hyp_homography.h"
#include "hyp_fundamental.h"
#include "plan.h"
#include "kernels.h"

#include <vector>
#include <cstring>

namespace mcv {

bool cv_sampler(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_CV_SAMPLER) != 0; }

void check_flags(const RansacConfig& cfg, const char* who) {
    if (cfg.flags & MCV_FLAG_RETIRED_4)
        fail("%s: flag bit 4 is retired (it meant 'unfused error' in the round-1 header; the op-by-op error is "
             "now the default and the FMA-contracted one is MCV_FLAG_FUSED_ERROR = 64)", who);
}

// Subset check of the model family: 1 homography, 2 fundamental (7- or 8-point), 0 none.
static int check_kind(int model) {
    return model == MCV_MODEL_HOMOGRAPHY ? 1 : (model == MCV_MODEL_FUNDAMENTAL ? 2 : 0);
}

template <int M>
static bool subset_ok(int check, const float* pts4, const int* idx) {
    if (check == 0) return true;
    float x1[M], y1[M], x2[M], y2[M];
    for (int i = 0; i < M; ++i) {
        const float* p = pts4 + 4 * (int64_t)idx[i];
        x1[i] = p[0]; y1[i] = p[1]; x2[i] = p[2]; y2[i] = p[3];
    }
    if (check == 1) {
        if constexpr (M == 4) return h_check_subset(x1, y1, x2, y2);
        return false;
    }
    return !(have_collinear_last<M>(x1, y1) || have_collinear_last<M>(x2, y2));
}

// Rows [0, rows) of the stream; rows from the first failed getSubset on are -1. Returns the number
// of accepted rows.
template <int M>
static int64_t cv_subsets(int check, const float* pts4, int N, int64_t rows, int* out) {
    CvRng rng{~(uint64_t)0};
    int64_t h = 0;
    for (; h < rows; ++h) {
        int* idx = out + (int64_t)M * h;
        bool ok = false;
        for (int attempt = 0; attempt < kMaxAttempts && !ok; ++attempt) {
            for (int i = 0; i < M; ++i) {
                bool dup;
                do {
                    idx[i] = rng.uniform(0, N);
                    dup = false;
                    for (int j = 0; j < i; ++j) dup = dup || idx[j] == idx[i];
                } while (dup);
            }
            ok = subset_ok<M>(check, pts4, idx);
        }
        if (!ok) break;
    }
    for (int64_t r = h; r < rows; ++r)
        for (int i = 0; i < M; ++i) out[(int64_t)M * r + i] = -1;
    return h;
}

static int64_t cv_subsets_m(int m, int check, const float* pts4, int N, int64_t rows, int* out) {
    switch (m) {
        case 4: return cv_subsets<4>(check, pts4, N, rows, out);
        case 5: return cv_subsets<5>(check, pts4, N, rows, out);
        case 7: return cv_subsets<7>(check, pts4, N, rows, out);
        case 8: return cv_subsets<8>(check, pts4, N, rows, out);
        default: fail("cv sampler: unsupported sample size %d", m);
    }
    return 0;
}

// Hypothesis budget of the table mode (getSubset's stream is sequential by definition).
static const int64_t kCvTableMaxRows = 1 << 24;

void cv_table_build(int model, const RansacConfig& cfg, const float* h_pts4, int N, int64_t rows,
                    std::vector<int>& out) {
    const int m = model_points_cfg(model, cfg);
    if (N < m) fail("cv sampler: N=%d below the minimal sample %d", N, m);
    if (rows > kCvTableMaxRows)
        fail("cv sampler: %lld hypotheses exceed the sequential stream's budget (%lld); use the Philox sampler",
             (long long)rows, (long long)kCvTableMaxRows);
    const int check = check_kind(model);
    if (check && !h_pts4) fail("cv sampler: the subset check needs the host points");
    out.resize((size_t)m * (size_t)std::max<int64_t>(rows, 1));
    cv_subsets_m(m, check, h_pts4, N, rows, out.data());
}

bool cv_table_reads_points(int model) { return check_kind(model) != 0; }

uint64_t cv_table_points_fp(int model, const float* h_pts4, int N) {
    return cv_table_reads_points(model) && h_pts4 ? host_fingerprint(h_pts4, (size_t)N * 16) : 0;
}

void cv_table_upload(Plan& P, const std::vector<int>& t, int m, int64_t rows, int N, uint64_t pointsFp,
                     hipStream_t s) {
    P.subsets.ensure((size_t)m * (size_t)std::max<int64_t>(rows, 1));
    MCV_HIP(hipMemcpyAsync(P.subsets.p, t.data(), (size_t)m * rows * sizeof(int), hipMemcpyHostToDevice, s));
    MCV_HIP(hipStreamSynchronize(s));
    P.subsetRows = rows;
    P.subsetM = m;
    P.subsetN = N;
    P.subsetFp = pointsFp;
    P.last.clear();
}

void cv_table_prepare(Plan& P, const void* d_pts, const float* h_pts4, int N, const RansacConfig& cfg, int64_t rows,
                      hipStream_t s) {
    std::vector<float> host;
    if (check_kind(P.model) && !h_pts4) {   // the checks read the float4 points the GPU sees
        host.resize((size_t)N * 4);
        MCV_HIP(hipMemcpyAsync(host.data(), d_pts, (size_t)N * 16, hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        h_pts4 = host.data();
    }
    std::vector<int> t;
    cv_table_build(P.model, cfg, h_pts4, N, rows, t);
    cv_table_upload(P, t, model_points_cfg(P.model, cfg), rows, N, cv_table_points_fp(P.model, h_pts4, N), s);
}

Sampler Plan::sampler(const RansacConfig& cfg) const {
    Sampler smp;
    smp.seed = cfg.seed;
    smp.table = cv_sampler(cfg) ? subsets.p : nullptr;
    return smp;
}

}  // namespace mcv

using namespace mcv;

extern "C" MCV_API int64_t mcvCvSubsets(int model, int m, const float* pts4, int N, int64_t rows, int* out) {
    MCV_GUARD(-1, {
        if (!out || rows < 0 || N < m || m < 1) fail("mcvCvSubsets: bad argument");
        const int check = model == MCV_MODEL_HOMOGRAPHY ? 1 : (model == MCV_MODEL_FUNDAMENTAL ? 2 : 0);
        if (check && !pts4) fail("mcvCvSubsets: the homography / fundamental checks need pts4");
        if (check == 1 && m != 4) fail("mcvCvSubsets: homography samples have 4 points");
        return cv_subsets_m(m, check, pts4, N, rows, out);
    })
}
