// ransac_host.cpp — host orchestration of the RANSAC hot path behind the C-ABI.
//
// cvFindHomography (new export, conventions of cvRecoverPose, MiniCVNative.cpp:197-215):
//   pack V2d -> float4 on device  ->  [chunks of hypotheses: generate + verify on the GPU,
//   counts back, OpenCV-order sequential replay on the host (adaptive niters)]  ->  finalize:
//   mask of the winner, refit on its inliers (runKernel: GPU reductions + 9x9 Jacobi here),
//   10 Levenberg-Marquardt iterations (GPU reductions + 8x8 solve here)  ->  H, mask.
// Mirrors cv::findHomography(..., RANSAC, thr, mask, maxIters, conf) of OpenCV 4.x
// [ext: calib3d/src/fundam.cpp, ptsetreg.cpp, levmarq.cpp — absent here, SURVEY.md §8c].
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include "linalg.h"
#include "mcv_common.h"
#include "hyp_homography.h"
#include "plan.h"

#include <cmath>
#include <cfloat>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <memory>

namespace mcv {

// ------------------------------------------------------------------------------------------
// Sequential replay (RANSACPointSetRegistrator::run loop order + RANSACUpdateNumIters).
// ------------------------------------------------------------------------------------------
int ransac_update_num_iters(double p, double ep, int modelPoints, int64_t maxIters) {
    p = std::max(p, 0.);
    p = std::min(p, 1.);
    ep = std::max(ep, 0.);
    ep = std::min(ep, 1.);
    double num = std::max(1. - p, DBL_MIN);
    double denom = 1. - std::pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return (denom >= 0 || -num >= (double)maxIters * (-denom)) ? (int)maxIters : (int)std::lrint(num / denom);
}

}  // namespace mcv

using namespace mcv;

extern "C" MCV_API void mcvReplayInit(mcvReplayState* st, int maxIters) {
    st->niters = std::max(maxIters, 1);
    st->bestIndex = -1;
    st->bestCount = 0;
    st->stopped = 0;
}

namespace mcv {
// One chunk of the RANSACPointSetRegistrator::run loop: hypothesis `it` = one getSubset +
// runKernel; its models (slots) are tried in order, each improvement updates niters; the loop
// condition is checked per hypothesis.
static int replay_chunk(mcvReplayState* st, const int* counts, int64_t hypBegin, int64_t hypCount, int slots, int N,
                        int modelPoints, double confidence, int fixedIters) {
    if (st->stopped) return 1;
    for (int64_t i = 0; i < hypCount; ++i) {
        const int64_t it = hypBegin + i;
        if (it >= st->niters) { st->stopped = 1; return 1; }
        const int* c = counts + i * slots;
        if (c[0] == kStatusNoSample) { st->stopped = 1; return 1; }
        for (int k = 0; k < slots; ++k) {
            if (c[k] < 0) continue;
            if (c[k] > std::max(st->bestCount, modelPoints - 1)) {
                st->bestCount = c[k];
                st->bestIndex = it * slots + k;
                if (!fixedIters)
                    st->niters = ransac_update_num_iters(confidence, (double)(N - c[k]) / N, modelPoints, st->niters);
            }
        }
    }
    if (hypBegin + hypCount >= st->niters) { st->stopped = 1; return 1; }
    return 0;
}
}  // namespace mcv

extern "C" MCV_API int mcvReplayChunk(mcvReplayState* st, const int* counts, int64_t hypBegin, int64_t hypCount,
                                      int N, int modelPoints, double confidence, int fixedIters) {
    return replay_chunk(st, counts, hypBegin, hypCount, 1, N, modelPoints, confidence, fixedIters);
}

extern "C" MCV_API int mcvReplayChunkModels(mcvReplayState* st, const int* counts, int64_t hypBegin,
                                            int64_t hypCount, int slotsPerHyp, int N, int modelPoints,
                                            double confidence, int fixedIters) {
    if (slotsPerHyp < 1) slotsPerHyp = 1;
    return replay_chunk(st, counts, hypBegin, hypCount, slotsPerHyp, N, modelPoints, confidence, fixedIters);
}

namespace mcv {

// ------------------------------------------------------------------------------------------
// Plan
// ------------------------------------------------------------------------------------------
void Plan::reserve(int n, int64_t hyps) {
    if (n > maxN) maxN = n;
    if (hyps > maxHyps) maxHyps = hyps;
    const size_t slots = (size_t)model_slots(model);
    if (model == MCV_MODEL_ESSENTIAL || model == MCV_MODEL_PNP) {
        ptsd.ensure((size_t)maxN * 4);
        raw.ensure((size_t)maxN * 4);
        dslot.ensure((size_t)maxHyps * slots);
        ndense.ensure(8);
        if (model == MCV_MODEL_ESSENTIAL && maxHyps >= kEStageMinHyps) estage.ensure((size_t)maxHyps * sizeof(EStage));
    } else {
        pts.ensure((size_t)maxN * 4);
    }
    models.ensure((size_t)maxHyps * model_bytes(model));
    if (model == MCV_MODEL_HOMOGRAPHY) h64.ensure((size_t)maxHyps * 9);
    counts.ensure((size_t)maxHyps * slots);
    pkey.ensure(512);
    pfail.ensure(512);
    key.ensure(2);
    part.ensure((size_t)kReduceMaxBlocksHost * 64);
    red.ensure(64);
    mask.ensure((size_t)maxN);
    count.ensure(1);
    bbox.ensure(4);
    one.ensure(512);
    h_counts.ensure((size_t)maxHyps * slots);
    h_red.ensure(64);
    if (model != MCV_MODEL_ESSENTIAL && model != MCV_MODEL_PNP) h_pack.ensure((size_t)maxN * 4);
    one.ensure(sizeof(EOneOut));
    h_one.ensure(sizeof(EOneOut));
    h_i.ensure(4);
}

size_t model_bytes(int model) {
    if (model == MCV_MODEL_PNP) return 96;
    return model == MCV_MODEL_ESSENTIAL ? 72 * kEModelSlots : (model == MCV_MODEL_FUNDAMENTAL ? 80 : 32);
}
int model_slots(int model) { return model == MCV_MODEL_ESSENTIAL ? kEModelSlots : 1; }
static bool f_seven(int model, const RansacConfig& cfg) {
    return model == MCV_MODEL_FUNDAMENTAL && (cfg.flags & MCV_FLAG_SEVEN_POINT) != 0;
}
int model_slots_cfg(int model, const RansacConfig& cfg) { return f_seven(model, cfg) ? kF7Slots : model_slots(model); }

hipStream_t Plan::own_stream() {
    if (!stream) MCV_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    return stream;
}

Plan::~Plan() {
    if (stream) (void)hipStreamDestroy(stream);
}

// Per-thread cached plans for the host-pointer exports (one per device and model).
Plan& thread_plan(int model, int shard) {
    int dev = 0;
    MCV_HIP(hipGetDevice(&dev));
    thread_local std::vector<std::unique_ptr<Plan>> plans;
    for (auto& p : plans)
        if (p->device == dev && p->model == model && p->shard == shard) return *p;
    plans.emplace_back(new Plan());
    plans.back()->device = dev;
    plans.back()->model = model;
    plans.back()->shard = shard;
    return *plans.back();
}

size_t point_bytes(int model, int N) {
    return (size_t)N * (model == MCV_MODEL_ESSENTIAL || model == MCV_MODEL_PNP ? 32 : 16);
}

// Device-resident point buffer of a plan (layout per model) and its size in bytes.
static void* plan_points(Plan& P, int N, size_t* bytes) {
    *bytes = point_bytes(P.model, N);
    return P.model == MCV_MODEL_ESSENTIAL || P.model == MCV_MODEL_PNP ? (void*)P.ptsd.p : (void*)P.pts.p;
}

void mark_chunk(Plan& P, int64_t begin, int64_t count, const Sampler& smp, const void* d_pts, int N, int kind,
                hipStream_t s) {
    P.fp.ensure(2);
    P.h_fp.ensure(2);
    P.last.set(begin, count, smp, d_pts, N, kind);
    launch_fingerprint(d_pts, point_bytes(P.model, N), P.fp.p, s);
}

void queue_chunk_check(Plan& P, const void* d_pts, int N, hipStream_t s) {
    launch_fingerprint(d_pts, point_bytes(P.model, N), P.fp.p + 1, s);
    MCV_HIP(hipMemcpyAsync(P.h_fp.p, P.fp.p, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, s));
}

uint64_t device_fingerprint(Plan& P, const void* d_pts, int N, hipStream_t s) {
    P.fp.ensure(2);
    P.h_fp.ensure(2);
    launch_fingerprint(d_pts, point_bytes(P.model, N), P.fp.p + 1, s);
    MCV_HIP(hipMemcpyAsync(P.h_fp.p + 1, P.fp.p + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    return P.h_fp.p[1];
}

void pack_points(Plan& P, const mcvV2d* a, const mcvV2d* b, int N, float* d_dst, hipStream_t s) {
    P.h_pack.ensure((size_t)N * 4);
    float* h = P.h_pack.p;
    for (int i = 0; i < N; ++i) {   // OpenCV: points.convertTo(CV_32F)
        h[4 * i + 0] = (float)a[i].X;
        h[4 * i + 1] = (float)a[i].Y;
        h[4 * i + 2] = (float)b[i].X;
        h[4 * i + 3] = (float)b[i].Y;
    }
    MCV_HIP(hipMemcpyAsync(d_dst, h, (size_t)N * 16, hipMemcpyHostToDevice, s));
    MCV_HIP(hipStreamSynchronize(s));
}

double effective_threshold(const RansacConfig& cfg) { return cfg.threshold > 0 ? cfg.threshold : 3.0; }
bool fused_error(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_FUSED_ERROR) != 0; }
bool fast_minimal(const RansacConfig& cfg) { return (cfg.flags & MCV_FLAG_FAST_MINIMAL) != 0; }

// HomographyEstimatorCallback::runKernel over the masked correspondences (mask == NULL: all).
bool h_refit(Plan& P, const float* d_pts, int N, const uint8_t* d_mask, hipStream_t s, double* H) {
    // the three passes (sums -> centroids -> |deviations| -> scales -> LtL) chained on the device,
    // one read-back; the host re-derives c4 / s4 with the same divisions and checks them
    double r[62];
    reduce_to_host(P, s, 62, r, [&](double* part, double* red) { h_refit_chain(d_pts, N, d_mask, part, red, s); });
    const double* sums = r;
    const double count = sums[4];
    if (count <= 0) return false;
    double c4[4] = {sums[0] / count, sums[1] / count, sums[2] / count, sums[3] / count};   // cm.x, cm.y, cM.x, cM.y
    const double* dev = r + 9;
    for (int k = 0; k < 4; ++k)
        if (std::fabs(dev[k]) < DBL_EPSILON) return false;
    double s4[4] = {count / dev[0], count / dev[1], count / dev[2], count / dev[3]};   // sm.x, sm.y, sM.x, sM.y
    const double* ltl = r + 17;
    double A[81], w[9], V[81];
    int o = 0;
    for (int j = 0; j < 9; ++j)
        for (int k = j; k < 9; ++k) { A[j * 9 + k] = ltl[o]; A[k * 9 + j] = ltl[o]; ++o; }
    jacobi_eigen(A, 9, w, V);
    const double* H0 = V + 8 * 9;   // eigenvector of the smallest eigenvalue
    const double invHnorm[9] = {1. / s4[0], 0, c4[0], 0, 1. / s4[1], c4[1], 0, 0, 1};
    const double Hnorm2[9] = {s4[2], 0, -c4[2] * s4[2], 0, s4[3], -c4[3] * s4[3], 0, 0, 1};
    double T[9], R[9];
    mat3_mul(invHnorm, H0, T);
    mat3_mul(T, Hnorm2, R);
    const double sc = 1. / R[8];
    for (int k = 0; k < 9; ++k) {
        H[k] = R[k] * sc;
        if (!std::isfinite(H[k])) return false;
    }
    return true;
}

// LMSolver::create(HomographyRefineCallback(src, dst), 10)->run(H8) — the classic LMSolverImpl
// (Marquardt-Nielsen lambda control, eigen-based solve). The O(N) JtJ / Jtr / |r|^2 sums run on
// the GPU; the 8x8 algebra runs here.
void h_lm_refine(Plan& P, const float* d_pts, int N, const uint8_t* d_mask, hipStream_t s, double* H, int maxIters) {
    const int lx = 8;
    const double epsx = FLT_EPSILON, epsf = FLT_EPSILON;
    double x[8], xd[8], d[8], v[8], A[64], Ap[64], D[8], temp_d[8];
    for (int i = 0; i < 8; ++i) x[i] = H[i];
    auto compute = [&](const double* h, bool wantJ, double* Aout, double* vout) -> double {
        double buf[45];
        if (wantJ) {
            reduce_to_host(P, s, 45, buf, [&](double* part, double* red) { h_reduce_lm(d_pts, N, d_mask, h, true, part, red, s); });
            int o = 0;
            for (int j = 0; j < 8; ++j)
                for (int k = j; k < 8; ++k) { Aout[j * 8 + k] = buf[o]; Aout[k * 8 + j] = buf[o]; ++o; }
            for (int j = 0; j < 8; ++j) vout[j] = buf[36 + j];
            return buf[44];
        }
        reduce_to_host(P, s, 1, buf, [&](double* part, double* red) { h_reduce_lm(d_pts, N, d_mask, h, false, part, red, s); });
        return buf[0];
    };
    double S = compute(x, true, A, v);
    for (int i = 0; i < lx; ++i) D[i] = A[i * lx + i];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        for (int i = 0; i < lx * lx; ++i) Ap[i] = A[i];
        for (int i = 0; i < lx; ++i) Ap[i * lx + i] += lambda * D[i];
        eig_solve(Ap, lx, v, d);
        for (int i = 0; i < lx; ++i) xd[i] = x[i] - d[i];
        // JtJ / Jtr at xd ride along with its cost (one synchronisation per step): on acceptance they
        // are exactly what LMSolverImpl's re-evaluation at the new x returns (same sums, same order;
        // the cost is summed identically by OpLM and OpLMErr)
        double Ad[64], vd[8];
        const double Sd = compute(xd, true, Ad, vd);
        for (int i = 0; i < lx; ++i) {   // temp_d = -A d + 2 v
            double acc = 0;
            for (int k = 0; k < lx; ++k) acc += A[i * lx + k] * d[k];
            temp_d[i] = -acc + 2 * v[i];
        }
        double dS = 0;
        for (int i = 0; i < lx; ++i) dS += d[i] * temp_d[i];
        const double R = (S - Sd) / (std::fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int i = 0; i < lx; ++i) t += d[i] * v[i];
            double nu = (Sd - S) / (std::fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = std::min(std::max(nu, 2.), 10.);
            if (lambda == 0) {
                eig_invert(A, lx, Ap);
                double maxval = DBL_EPSILON;
                for (int i = 0; i < lx; ++i) maxval = std::max(maxval, std::fabs(Ap[i * lx + i]));
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            for (int i = 0; i < lx; ++i) x[i] = xd[i];
            std::memcpy(A, Ad, sizeof(Ad));
            std::memcpy(v, vd, sizeof(vd));
        }
        ++iter;
        double dn = 0;
        for (int i = 0; i < lx; ++i) dn = std::max(dn, std::fabs(d[i]));
        const bool proceed = iter < maxIters && dn >= epsx && S >= epsf * epsf;
        if (!proceed) break;
    }
    for (int i = 0; i < 8; ++i) H[i] = x[i];
}

// Evaluate one chunk of hypotheses on the device (generate + verify [+ best key]).
void evaluate_chunk(Plan& P, const void* d_ptsv, int N, const RansacConfig& cfg, int64_t hypBegin, int hypCount,
                    int* d_counts, uint64_t* d_key, hipStream_t s) {
    if (P.model == MCV_MODEL_ESSENTIAL) {
        e_evaluate_chunk(P, (const double*)d_ptsv, N, cfg, hypBegin, hypCount, d_counts, s);
        if (d_key)
            launch_best(d_counts, hypCount * kEModelSlots, hypBegin * kEModelSlots, model_points(P.model), P.pkey.p,
                        P.pfail.p, d_key, s);
        MCV_HIP(hipGetLastError());
        return;
    }
    if (P.model == MCV_MODEL_PNP) {
        p_evaluate_chunk(P, d_ptsv, N, cfg, hypBegin, hypCount, d_counts, s);
        if (d_key)
            launch_best(d_counts, hypCount, hypBegin, model_points_cfg(P.model, cfg), P.pkey.p, P.pfail.p, d_key, s);
        MCV_HIP(hipGetLastError());
        return;
    }
    const float* d_pts = (const float*)d_ptsv;
    const double t = effective_threshold(cfg);
    const float thr2 = (float)(t * t);
    if (P.model == MCV_MODEL_HOMOGRAPHY) {
        const bool fused = fused_error(cfg);
        P.pairs.ensure((size_t)(N + 1) / 2 * 8);
        launch_h_pair(d_pts, N, P.pairs.p, s);
        if (fused) {
            launch_bbox(d_pts, N, P.bbox.p, s);
        } else {
            P.bb4.ensure(4);
            launch_abs_bound4(d_pts, false, N, P.bb4.p, nullptr, s);
        }
        const Sampler smp = P.sampler(cfg);
        {
            ProfScope pg("h_generate", s);
            if (!fast_minimal(cfg)) P.hgen.ensure(h_gen_scratch_bytes(hypCount));
            launch_h_generate(d_pts, N, smp, hypBegin, hypCount, P.models.p, P.h64.p, d_counts, s,
                              fast_minimal(cfg), fast_minimal(cfg) ? nullptr : P.hgen.p);
        }
        // the winner's models can come straight from this chunk's buffers (h_finalize)
        mark_chunk(P, hypBegin, hypCount, smp, d_pts, N, fast_minimal(cfg) ? 21 : 20, s);
        ProfScope ps("h_verify", s);
        if (!fused) {
            // default: OpenCV's op-by-op error, certified division-free packed sweep
            launch_h_verify_certified(d_pts, P.pairs.p, N, P.models.p, d_counts, hypCount, thr2, P.bb4.p, s);
        } else {
            launch_h_verify_packed(d_pts, P.pairs.p, N, P.models.p, d_counts, hypCount, thr2, P.bbox.p, s);
        }
    } else if (f_seven(P.model, cfg)) {
        // OpenCV FM_RANSAC: 7-point samples, 3 model slots per hypothesis (slot keys like essential)
        P.last.clear();
        launch_f7_generate(d_pts, N, P.sampler(cfg), hypBegin, hypCount, P.models.p, d_counts, s);
        P.bb4.ensure(4);
        launch_abs_bound4(d_pts, false, N, P.bb4.p, nullptr, s);
        {
            ProfScope ps("f_verify", s);
            launch_f_verify(d_pts, N, P.models.p, d_counts, hypCount * kF7Slots, thr2, f_error_kind(cfg), s, P.bb4.p);
        }
        if (d_key)
            launch_best(d_counts, hypCount * kF7Slots, hypBegin * kF7Slots, 7, P.pkey.p, P.pfail.p, d_key, s);
        MCV_HIP(hipGetLastError());
        return;
    } else {
        const Sampler smp = P.sampler(cfg);
        {
            ProfScope pg("f_generate", s);
            launch_f_generate(d_pts, N, smp, hypBegin, hypCount, P.models.p, d_counts, s, fast_minimal(cfg));
        }
        // the winner's fp64 model can come straight from this chunk's buffer (f_finalize)
        mark_chunk(P, hypBegin, hypCount, smp, d_pts, N, fast_minimal(cfg) ? 11 : 10, s);
        P.bb4.ensure(4);
        launch_abs_bound4(d_pts, false, N, P.bb4.p, nullptr, s);
        ProfScope ps("f_verify", s);
        launch_f_verify(d_pts, N, P.models.p, d_counts, hypCount, thr2, f_error_kind(cfg), s, P.bb4.p);
    }
    if (d_key) launch_best(d_counts, hypCount, hypBegin, model_points(P.model), P.pkey.p, P.pfail.p, d_key, s);
    MCV_HIP(hipGetLastError());
}

int model_points(int model) { return model == MCV_MODEL_FUNDAMENTAL ? 8 : (model == MCV_MODEL_ESSENTIAL ? 5 : 4); }
// (homography and PnP with the AP3P kernel: 4)
int model_points_cfg(int model, const RansacConfig& cfg) {
    if (f_seven(model, cfg)) return 7;
    return model == MCV_MODEL_PNP && pnp_cfg_epnp(cfg) ? 5 : model_points(model);
}

// Winner -> mask (+ refit + LM). Returns inlier count, 0 on failure. Synchronises s.
int h_finalize(Plan& P, const float* d_pts, int N, const RansacConfig& cfg, int64_t hyp, double* H, uint8_t* d_mask,
               hipStream_t s) {
    const double t = effective_threshold(cfg);
    const float thr2 = (float)(t * t);
    // winner re-solve -> mask from the device-side record -> one read-back of both
    HOneOut* d_one = (HOneOut*)P.one.p;
    const Sampler smp = P.sampler(cfg);
    const bool cached = P.last.covers(hyp, smp, d_pts, N, fast_minimal(cfg) ? 21 : 20);
    if (cached) {
        // the winner's fp64 and fp32 models straight from the last chunk's buffers (the same code
        // produced them) instead of a single-lane eigen re-solve (~0.4 ms); a winner has status 1
        const int64_t local = hyp - P.last.begin;
        MCV_HIP(hipMemcpyAsync(d_one->H, P.h64.p + 9 * local, 9 * sizeof(double), hipMemcpyDeviceToDevice, s));
        MCV_HIP(hipMemcpyAsync(d_one->hf, P.models.p + local * sizeof(HModelF), sizeof(HModelF),
                               hipMemcpyDeviceToDevice, s));
        P.h_i.p[1] = 1;
        MCV_HIP(hipMemcpyAsync(&d_one->status, P.h_i.p + 1, sizeof(int), hipMemcpyHostToDevice, s));
        queue_chunk_check(P, d_pts, N, s);
    } else {
        launch_h_one(d_pts, N, smp, hyp, d_one, s, fast_minimal(cfg));
    }
    MCV_HIP(hipMemsetAsync(P.count.p, 0, sizeof(int), s));
    launch_h_mask_one(d_pts, N, d_one, thr2, fused_error(cfg), d_mask, P.count.p, s);
    MCV_HIP(hipGetLastError());
    HOneOut one;
    MCV_HIP(hipMemcpyAsync(P.h_one.p, d_one, sizeof(HOneOut), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipMemcpyAsync(P.h_i.p, P.count.p, sizeof(int), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    if (cached && !chunk_fresh(P)) {   // the points changed since the chunk was evaluated: re-solve
        P.last.clear();
        return h_finalize(P, d_pts, N, cfg, hyp, H, d_mask, s);
    }
    std::memcpy(&one, P.h_one.p, sizeof(HOneOut));
    if (one.status != 1) fail("winning hypothesis %lld has no model (status %d)", (long long)hyp, one.status);
    const int count = P.h_i.p[0];
    for (int k = 0; k < 9; ++k) H[k] = one.H[k];
    if (cfg.flags & MCV_FLAG_NO_REFINE) return count;
    if (N > 4 && count > 0) {
        double Hr[9];
        if (h_refit(P, d_pts, N, d_mask, s, Hr))
            for (int k = 0; k < 9; ++k) H[k] = Hr[k];
        h_lm_refine(P, d_pts, N, d_mask, s, H, 10);
    }
    return count;
}

int finalize(Plan& P, const void* d_ptsv, int N, const RansacConfig& cfg, int64_t hyp, double* model9,
             uint8_t* d_mask, hipStream_t s) {
    if (P.model == MCV_MODEL_ESSENTIAL) return e_finalize(P, (const double*)d_ptsv, N, cfg, hyp, model9, d_mask, s);
    if (P.model == MCV_MODEL_PNP) return p_finalize(P, d_ptsv, N, cfg, hyp, model9, d_mask, s);
    const float* d_pts = (const float*)d_ptsv;
    if (P.model == MCV_MODEL_HOMOGRAPHY) return h_finalize(P, d_pts, N, cfg, hyp, model9, d_mask, s);
    return f_finalize(P, d_pts, N, cfg, hyp, model9, d_mask, s);
}

// Full RANSAC on device-resident points with the OpenCV sequential-replay semantics.
// cfg.deviceCount > 1: every chunk is split into that many contiguous hypothesis ranges evaluated
// concurrently by per-shard workspaces on devices 0, 1, ... (round-robin over the visible GPUs;
// points replicated once by peer copy), counts concatenated in order, then the same replay — the
// answer is identical to one device. Returns the best hypothesis (slot) index or -1.
int64_t ransac_search(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, hipStream_t s,
                      const float* h_pts4) {
    const int m = model_points_cfg(P.model, cfg);
    const int slots = model_slots_cfg(P.model, cfg);
    // plans size their slot buffers by model_slots(model): a mode with more slots per hypothesis
    // (7-point F) reserves that many times the hypotheses
    const int64_t slotScale = slots / model_slots(P.model);
    mcvReplayState st;
    mcvReplayInit(&st, cfg.maxIters);
    const bool fixed = (cfg.flags & MCV_FLAG_FIXED_ITERS) != 0;
    int ndev = 1;
    MCV_HIP(hipGetDeviceCount(&ndev));
    const int shards = std::max(1, std::min(cfg.deviceCount, kMaxShards));
    int home = 0;
    MCV_HIP(hipGetDevice(&home));
    // the calling thread's device is restored on every exit, exceptions included (later calls on
    // this thread resolve their plans and allocations by the current device)
    struct DeviceRestore {
        int dev;
        ~DeviceRestore() { (void)hipSetDevice(dev); }
    } restore{home};
    struct Shard { Plan* P; const void* pts; hipStream_t s; int dev; };
    std::vector<Shard> sh;
    sh.push_back({&P, d_pts, s, home});
    // OpenCV's sample stream: the whole budget's subsets up front (niters only shrinks), uploaded to
    // every shard's workspace
    std::vector<int> table;
    uint64_t tableFp = 0;
    const int64_t tableRows = std::max(cfg.maxIters, 1);
    if (cv_sampler(cfg)) {
        std::vector<float> host;
        if (!h_pts4 && P.model != MCV_MODEL_ESSENTIAL && P.model != MCV_MODEL_PNP) {
            host.resize((size_t)N * 4);
            MCV_HIP(hipMemcpyAsync(host.data(), d_pts, (size_t)N * 16, hipMemcpyDeviceToHost, s));
            MCV_HIP(hipStreamSynchronize(s));
            h_pts4 = host.data();
        }
        cv_table_build(P.model, cfg, h_pts4, N, tableRows, table);
        tableFp = cv_table_points_fp(P.model, h_pts4, N);
        cv_table_upload(P, table, m, tableRows, N, tableFp, s);
    }
    if (shards > 1) {
        size_t bytes = 0;
        MCV_HIP(hipStreamSynchronize(s));
        for (int k = 1; k < shards; ++k) {
            const int dev = (home + k) % ndev;
            MCV_HIP(hipSetDevice(dev));
            Plan& Pk = thread_plan(P.model, k);
            Pk.reserve(N, slotScale);
            std::memcpy(Pk.pnpCam, P.pnpCam, sizeof(P.pnpCam));
            void* dst = plan_points(Pk, N, &bytes);
            hipStream_t sk = Pk.own_stream();
            MCV_HIP(hipMemcpyPeerAsync(dst, dev, d_pts, home, bytes, sk));
            if (cv_sampler(cfg)) cv_table_upload(Pk, table, m, tableRows, N, tableFp, sk);
            sh.push_back({&Pk, dst, sk, dev});
        }
        MCV_HIP(hipSetDevice(home));
    }
    int64_t begin = 0;
    // adaptive calls start small (niters shrinks with the first good model); a fixed budget is
    // evaluated in chunks of kChunkMax from the start
    int64_t chunk = std::min<int64_t>(std::max<int64_t>(st.niters, 1), fixed ? kChunkMax : kChunkFirst);
    P.h_keys.ensure(2 * kMaxShards);
    while (!st.stopped) {
        const int64_t remaining = st.niters - begin;
        if (remaining <= 0) break;
        const int cnt = (int)std::min<int64_t>(remaining, chunk);
        P.reserve(N, cnt * slotScale);
        const int nsh = std::min<int>((int)sh.size(), cnt);
        // fixed iterations: the sequential replay's answer is the first maximum over the counts >= m
        // before the first sampler failure, so each shard reduces its range on its own device to the
        // packed key (count << 32 | ~slot) + its first failure and sends 16 B; only a chunk with a
        // sampler failure (degenerate data) falls back to gathering the counts. Adaptive calls gather
        // the counts (4 B per model slot) and replay them in order.
        int64_t off = 0;
        for (int k = 0; k < nsh; ++k) {
            const int ck = (int)(cnt / nsh + (k < cnt % nsh ? 1 : 0));
            Shard& x = sh[k];
            if (k > 0) {
                MCV_HIP(hipSetDevice(x.dev));
                x.P->reserve(N, ck * slotScale);
            }
            evaluate_chunk(*x.P, x.pts, N, cfg, begin + off, ck, x.P->counts.p, fixed ? x.P->key.p : nullptr, x.s);
            if (fixed)
                MCV_HIP(hipMemcpyAsync(P.h_keys.p + 2 * k, x.P->key.p, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                       x.s));
            else
                MCV_HIP(hipMemcpyAsync(P.h_counts.p + off * slots, x.P->counts.p, (size_t)ck * slots * sizeof(int),
                                       hipMemcpyDeviceToHost, x.s));
            off += ck;
        }
        for (int k = 0; k < nsh; ++k) {
            if (k > 0) MCV_HIP(hipSetDevice(sh[k].dev));
            MCV_HIP(hipStreamSynchronize(sh[k].s));
        }
        bool replayed = false;
        if (fixed) {
            uint64_t best = 0;
            bool failed = false;
            for (int k = 0; k < nsh; ++k) {
                best = std::max(best, P.h_keys.p[2 * k]);
                failed = failed || (int64_t)P.h_keys.p[2 * k + 1] != INT64_MAX;
            }
            if (!failed) {
                const int c = (int)(best >> 32);
                if (best != 0 && c > std::max(st.bestCount, m - 1)) {
                    st.bestCount = c;
                    st.bestIndex = (int64_t)(0xFFFFFFFFull - (best & 0xFFFFFFFFull));
                }
                replayed = true;
            } else {   // a sampler failure inside the chunk: the counts, in order
                off = 0;
                for (int k = 0; k < nsh; ++k) {
                    const int ck = (int)(cnt / nsh + (k < cnt % nsh ? 1 : 0));
                    if (k > 0) MCV_HIP(hipSetDevice(sh[k].dev));
                    MCV_HIP(hipMemcpy(P.h_counts.p + off * slots, sh[k].P->counts.p, (size_t)ck * slots * sizeof(int),
                                      hipMemcpyDeviceToHost));
                    off += ck;
                }
            }
        }
        if (nsh > 1) MCV_HIP(hipSetDevice(home));
        if (!replayed) replay_chunk(&st, P.h_counts.p, begin, cnt, slots, N, m, cfg.confidence, fixed ? 1 : 0);
        begin += cnt;
        if (begin >= st.niters) st.stopped = 1;
        chunk = std::min<int64_t>(chunk * 2, kChunkMax);
    }
    return st.bestIndex;
}

void require_device() {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        fail("no HIP device available (hipGetDeviceCount: %s, n=%d); the MI355X path has no CPU fallback",
             hipGetErrorString(e), n);
}

RansacConfig config_or_default(const RansacConfig* cfg) {
    if (cfg) return *cfg;
    RansacConfig c;
    std::memset(&c, 0, sizeof(c));
    c.threshold = 3.0;
    c.confidence = 0.995;
    c.maxIters = 2000;
    c.method = MCV_METHOD_RANSAC;
    c.flags = MCV_FLAG_CV_SAMPLER;   // no seed given: OpenCV's own sample stream
    return c;
}

}  // namespace mcv

// ------------------------------------------------------------------------------------------
// Exports
// ------------------------------------------------------------------------------------------
extern "C" MCV_API int cvFindHomography(const mcvV2d* src, const mcvV2d* dst, const int N, const RansacConfig* cfgp,
                                        mcvM33d* H, uint8_t* mask) {
    MCV_GUARD(0, {
        if (!src || !dst || !H || N < 0) fail("cvFindHomography: null argument or negative N");
        if (mask) std::memset(mask, 0, (size_t)N);
        if (N < 4) fail("cvFindHomography: need at least 4 correspondences (N=%d)", N);
        const RansacConfig cfg = config_or_default(cfgp);
        check_flags(cfg, "cvFindHomography");
        if (cfg.method != MCV_METHOD_RANSAC && cfg.method != MCV_METHOD_LSQ)
            fail("cvFindHomography: unsupported method %d", cfg.method);
        if (cfg.method == MCV_METHOD_RANSAC && !(cfg.confidence > 0 && cfg.confidence < 1))
            fail("cvFindHomography: confidence must be in (0,1)");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_HOMOGRAPHY);
        hipStream_t s = P.own_stream();
        P.reserve(N, 1);
        pack_points(P, src, dst, N, P.pts.p, s);
        double Hm[9];
        int count = 0;
        if (cfg.method == MCV_METHOD_LSQ || N == 4) {
            if (!h_refit(P, P.pts.p, N, nullptr, s, Hm)) fail("cvFindHomography: degenerate point set");
            if (N > 4) h_lm_refine(P, P.pts.p, N, nullptr, s, Hm, 10);
            if (mask) std::memset(mask, 1, (size_t)N);
            count = N;
        } else {
            const int64_t best = ransac_search(P, P.pts.p, N, cfg, s, P.h_pack.p);
            if (best < 0) fail("cvFindHomography: RANSAC found no model with >= 4 inliers");
            count = h_finalize(P, P.pts.p, N, cfg, best, Hm, P.mask.p, s);
            if (mask) {
                MCV_HIP(hipMemcpyAsync(mask, P.mask.p, (size_t)N, hipMemcpyDeviceToHost, s));
                MCV_HIP(hipStreamSynchronize(s));
            }
        }
        for (int k = 0; k < 9; ++k) H->M[k] = Hm[k];
        return count;
    })
}

extern "C" MCV_API mcvRansacPlan* mcvRansacPlanCreate(int model, int maxN, int64_t maxHyps) {
    MCV_GUARD(nullptr, {
        if (model < MCV_MODEL_HOMOGRAPHY || model > MCV_MODEL_PNP)
            fail("unknown model %d", model);
        require_device();
        std::unique_ptr<Plan> p(new Plan());
        MCV_HIP(hipGetDevice(&p->device));
        p->model = model;
        p->reserve(std::max(maxN, 1), std::max<int64_t>(maxHyps, 1));
        return reinterpret_cast<mcvRansacPlan*>(p.release());
    })
}

extern "C" MCV_API void mcvRansacPlanDestroy(mcvRansacPlan* plan) {
    try {
        delete reinterpret_cast<Plan*>(plan);
    } catch (...) {
    }
}

extern "C" MCV_API int mcvPackCorrespondences(const mcvV2d* a, const mcvV2d* b, int N, float* d_pts4, void* stream) {
    MCV_GUARD(0, {
        if (!a || !b || !d_pts4 || N < 0) fail("mcvPackCorrespondences: bad argument");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_HOMOGRAPHY);
        pack_points(P, a, b, N, d_pts4, (hipStream_t)stream);
        return 1;
    })
}

namespace mcv {
// The CV-sampler table of P cannot serve hypotheses [.., rowsNeeded) of a search over these points:
// a search that starts at 0 (begin == 0), too few rows, another sample size, another N, or (H / F,
// whose checkSubset reads the points) other point content. The content check synchronises s.
static bool cv_table_stale(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t begin,
                           int64_t rowsNeeded, hipStream_t s) {
    if (begin == 0 || P.subsetRows < rowsNeeded || P.subsetM != model_points_cfg(P.model, cfg) || P.subsetN != N)
        return true;
    return cv_table_reads_points(P.model) && device_fingerprint(P, d_pts, N, s) != P.subsetFp;
}
}  // namespace mcv

extern "C" MCV_API int mcvRansacEvaluate(mcvRansacPlan* plan, const void* d_pts4, int N, const RansacConfig* cfg,
                                         int64_t hypBegin, int64_t hypCount, uint64_t* d_key, int* d_counts,
                                         void* stream) {
    MCV_GUARD(0, {
        Plan* P = reinterpret_cast<Plan*>(plan);
        if (!P || !d_pts4 || !cfg || !d_key) fail("mcvRansacEvaluate: null argument");
        if (N < model_points_cfg(P->model, *cfg)) fail("mcvRansacEvaluate: N=%d below the minimal sample", N);
        const int64_t scale = model_slots_cfg(P->model, *cfg) / model_slots(P->model);
        if (hypCount <= 0 || hypCount * scale > P->maxHyps)
            fail("mcvRansacEvaluate: hypCount %lld (x%lld slots) outside plan capacity %lld", (long long)hypCount,
                 (long long)scale, (long long)P->maxHyps);
        if (hypBegin < 0 || (hypBegin + hypCount) * model_slots_cfg(P->model, *cfg) > 0xFFFFFFFFll)
            fail("mcvRansacEvaluate: hypothesis (slot) index beyond 2^32");
        check_flags(*cfg, "mcvRansacEvaluate");
        if (cv_sampler(*cfg) && cv_table_stale(*P, d_pts4, N, *cfg, hypBegin, hypBegin + hypCount, (hipStream_t)stream))
            // a search starts at hypothesis 0, and a table drawn for other points is never reused: the
            // stream is rebuilt from the current points
            cv_table_prepare(*P, d_pts4, nullptr, N, *cfg, std::max<int64_t>(hypBegin + hypCount, cfg->maxIters),
                             (hipStream_t)stream);
        evaluate_chunk(*P, d_pts4, N, *cfg, hypBegin, (int)hypCount, d_counts ? d_counts : P->counts.p, d_key,
                       (hipStream_t)stream);
        return 1;
    })
}

extern "C" MCV_API int mcvRansacFinalize(mcvRansacPlan* plan, const void* d_pts4, int N, const RansacConfig* cfg,
                                         int64_t hypIndex, double* model9, uint8_t* d_mask, void* stream) {
    MCV_GUARD(0, {
        Plan* P = reinterpret_cast<Plan*>(plan);
        if (!P || !d_pts4 || !cfg || !model9 || !d_mask) fail("mcvRansacFinalize: null argument");
        if (hypIndex < 0) fail("mcvRansacFinalize: no winning hypothesis");
        check_flags(*cfg, "mcvRansacFinalize");
        P->reserve(N, 1);
        const int64_t hyp = hypIndex / model_slots_cfg(P->model, *cfg);
        if (cv_sampler(*cfg) && cv_table_stale(*P, d_pts4, N, *cfg, 1, hyp + 1, (hipStream_t)stream))
            cv_table_prepare(*P, d_pts4, nullptr, N, *cfg, std::max<int64_t>(hyp + 1, cfg->maxIters),
                             (hipStream_t)stream);
        return finalize(*P, d_pts4, N, *cfg, hypIndex, model9, d_mask, (hipStream_t)stream);
    })
}

extern "C" MCV_API int mcvHostHypothesis(int model, const float* pts4, int N, uint64_t seed, int64_t hyp,
                                         double* model9, float* modelf9, int* sampleIdx) {
    MCV_GUARD(kStatusNoSample - 1, {
        if (!pts4 || !model9 || !modelf9) fail("mcvHostHypothesis: null argument");
        const bool fast = (model & MCV_HOST_FAST_MINIMAL) != 0;
        model &= ~MCV_HOST_FAST_MINIMAL;
        if (model == MCV_MODEL_HOMOGRAPHY) {
            if (N < 4) fail("N < 4");
            HModelF mf;
            for (int k = 0; k < 9; ++k) model9[k] = 0;
            for (int k = 0; k < 8; ++k) mf.h[k] = 0;
            EigWsLocal ws;
            const int st = h_hypothesis(pts4, N, Sampler{seed, nullptr}, (uint64_t)hyp, model9, &mf, sampleIdx, ws,
                                        fast);
            for (int k = 0; k < 8; ++k) modelf9[k] = mf.h[k];
            modelf9[8] = 1.f;
            return st;
        }
        return f_host_hypothesis(pts4, N, seed, hyp, model9, modelf9, sampleIdx, fast);
    })
}

extern "C" MCV_API void mcvHostPhilox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                      uint32_t* out4) {
    U4 c;
    c.x = c0; c.y = c1; c.z = c2; c.w = c3;
    const U4 r = philox4x32_10(c, k0, k1);
    out4[0] = r.x; out4[1] = r.y; out4[2] = r.z; out4[3] = r.w;
}

extern "C" MCV_API int cvFindFundamentalMat(const mcvV2d* a, const mcvV2d* b, const int N, const RansacConfig* cfgp,
                                            mcvM33d* F, uint8_t* mask) {
    MCV_GUARD(0, {
        if (!a || !b || !F || N < 0) fail("cvFindFundamentalMat: null argument or negative N");
        if (mask) std::memset(mask, 0, (size_t)N);
        RansacConfig cfg = config_or_default(cfgp);
        if (!cfgp) cfg.confidence = 0.99;
        check_flags(cfg, "cvFindFundamentalMat");
        const bool seven = (cfg.flags & MCV_FLAG_SEVEN_POINT) != 0;
        if (seven && cfg.method == MCV_METHOD_RANSAC && N != 7 && N < 15)
            fail("cvFindFundamentalMat: 7-point FM_RANSAC needs N >= 15 (OpenCV uses LMeDS below that; N=%d)", N);
        if (!seven && N < 8) fail("cvFindFundamentalMat: need at least 8 correspondences (N=%d)", N);
        if (seven && N < 7) fail("cvFindFundamentalMat: need at least 7 correspondences (N=%d)", N);
        if (cfg.method != MCV_METHOD_RANSAC && cfg.method != MCV_METHOD_LSQ)
            fail("cvFindFundamentalMat: unsupported method %d", cfg.method);
        if (cfg.method == MCV_METHOD_RANSAC && !(cfg.confidence > 0 && cfg.confidence < 1))
            fail("cvFindFundamentalMat: confidence must be in (0,1)");
        require_device();
        Plan& P = thread_plan(MCV_MODEL_FUNDAMENTAL);
        hipStream_t s = P.own_stream();
        P.reserve(N, 1);
        pack_points(P, a, b, N, P.pts.p, s);
        double Fm[9];
        int count = 0;
        if (seven && N == 7) {
            // findFundamentalMat with npoints == 7: run7Point once (the first of its models), mask all 1
            launch_f7_direct(P.pts.p, (FOneOut*)P.one.p, s);
            MCV_HIP(hipGetLastError());
            FOneOut one;
            MCV_HIP(hipMemcpyAsync(P.h_one.p, P.one.p, sizeof(FOneOut), hipMemcpyDeviceToHost, s));
            MCV_HIP(hipStreamSynchronize(s));
            std::memcpy(&one, P.h_one.p, sizeof(FOneOut));
            if (one.status <= 0) fail("cvFindFundamentalMat: degenerate 7-point set");
            for (int k = 0; k < 9; ++k) Fm[k] = one.F[k];
            if (mask) std::memset(mask, 1, (size_t)N);
            count = N;
        } else if (cfg.method == MCV_METHOD_LSQ || N == 8) {
            count = f_fit_all(P, P.pts.p, N, s, Fm);
            if (count <= 0) fail("cvFindFundamentalMat: degenerate point set");
            if (mask) std::memset(mask, 1, (size_t)N);
        } else {
            const int64_t best = ransac_search(P, P.pts.p, N, cfg, s, P.h_pack.p);
            if (best < 0) fail("cvFindFundamentalMat: RANSAC found no model with >= %d inliers", seven ? 7 : 8);
            count = f_finalize(P, P.pts.p, N, cfg, best, Fm, P.mask.p, s);
            if (mask) {
                MCV_HIP(hipMemcpyAsync(mask, P.mask.p, (size_t)N, hipMemcpyDeviceToHost, s));
                MCV_HIP(hipStreamSynchronize(s));
            }
        }
        for (int k = 0; k < 9; ++k) F->M[k] = Fm[k];
        return count;
    })
}
