// plan.h — device workspace of one RANSAC problem family (homography or fundamental) on one GPU.
#pragma once

#include "minicv_native.h"
#include "mcv_runtime.h"
#include "mcv_common.h"
#include <stdint.h>
#include <vector>

namespace mcv {

// Host-API chunking of the hypothesis stream for the adaptive (sequential-replay) search.
static const int64_t kChunkFirst = 4096;
static const int64_t kChunkMax = 1 << 20;

size_t model_bytes(int model);   // device model bytes per hypothesis
int model_points(int model);
int model_points_cfg(int model, const RansacConfig& cfg);   // PnP: 5 with the EPnP kernel; F 7-point: 7
int model_slots_cfg(int model, const RansacConfig& cfg);    // F 7-point: 3 model slots per hypothesis
int model_slots(int model);      // model slots per hypothesis (essential: 10)

// Key of the last evaluated chunk. A winner inside it takes its model from the chunk's buffers
// instead of a re-solve; the key names everything that produced those buffers (the hypothesis
// range, the sample source, the point buffer and N, the minimal solver), and every evaluate replaces
// it, so any other evaluate in between, or a different solver / sampler, invalidates it. The points'
// content is keyed too: the evaluate fingerprints the buffer (Plan::fp[0], mark_chunk), finalize
// fingerprints it again and re-solves the winner when the two differ (a caller that rewrote the
// buffer in place, same pointer and N, between evaluate and finalize).
struct LastChunk {
    int64_t begin = -1, count = 0;
    uint64_t seed = 0;
    const int* table = nullptr;
    const void* pts = nullptr;
    int N = 0;
    int kind = -1;            // H: 20 eigen, 21 elimination; F: 10 / 11; E: 30 / 31; PnP: 1 EPnP, 0 AP3P
    void set(int64_t b, int64_t c, const Sampler& smp, const void* p, int n, int k) {
        begin = b; count = c; seed = smp.seed; table = smp.table; pts = p; N = n; kind = k;
    }
    void clear() { *this = LastChunk(); }
    bool covers(int64_t hyp, const Sampler& smp, const void* p, int n, int k) const {
        return begin >= 0 && hyp >= begin && hyp < begin + count && seed == smp.seed && table == smp.table &&
               pts == p && N == n && kind == k;
    }
};

struct Plan {
    int model = MCV_MODEL_HOMOGRAPHY;
    int device = 0;
    int shard = 0;
    int maxN = 0;
    int64_t maxHyps = 0;
    hipStream_t stream = nullptr;   // only for the host-pointer exports

    DevBuf<float> pts;        // packed float4 correspondences (host-API path)
    DevBuf<uint8_t> models;   // per-hypothesis fp32 models
    DevBuf<int> counts;       // per-hypothesis status / inlier count
    DevBuf<uint64_t> pkey;    // best-key partials
    DevBuf<int64_t> pfail;
    DevBuf<uint64_t> key;
    DevBuf<double> part;      // reduction partials
    DevBuf<double> red;       // reduction result
    DevBuf<uint8_t> mask;
    DevBuf<int> count;
    DevBuf<float> bbox;       // max |x|, max |y| of the source points (fused fast-path bound)
    DevBuf<double> bb4;       // F / E: max |x1|, |y1|, |x2|, |y2| (packed-fp32 Sampson prefilter bound)
    DevBuf<double> h64;       // homography: each hypothesis' fp64 model (finalize takes the winner's)
    DevBuf<uint8_t> hgen;     // homography: the split eigen generate's scratch (rotation log of one piece)
    DevBuf<float> pairs;      // paired point layout of the packed sweeps (homography 8, PnP 12 floats per 2)
    DevBuf<uint8_t> one;      // single-hypothesis output record
    DevBuf<double> ptsd;      // essential: double4 normalised correspondences
    DevBuf<double> raw;       // essential: uploaded V2d pairs (a then b)
    DevBuf<int> dslot;        // essential: slot of each dense model
    DevBuf<uint8_t> estage;   // essential: per-hypothesis EStage of the split five-point solve
    DevBuf<int> ndense;       // essential: dense model count, 4 cheirality counters, fetch flag
    double pnpCam[8] = {1, 1, 0, 0, 0, 0, 0, 0};   // PnP: fx, fy, cx, cy, k1, k2, p1, p2
    DevBuf<double> epw;       // PnP: EPnP solve points (world, double)
    DevBuf<double> eus;       // PnP: EPnP solve points (pixels of the undistorted observations)
    DevBuf<int> eidx;         // PnP: inlier indices of the EPnP solve
    DevBuf<double> escratch;  // PnP: the split EPnP generate's per-hypothesis state (kEpnpSplitDoubles each)
    LastChunk last;           // the last evaluated chunk (finalize takes the winner's model from its buffers)
    DevBuf<int> subsets;      // MCV_FLAG_CV_SAMPLER: OpenCV's getSubset stream, subsetM ints per hypothesis
    int64_t subsetRows = 0;   // hypotheses [0, subsetRows) covered by `subsets`
    int subsetM = 0;
    int subsetN = 0;          // the N the table was drawn for (its rows index [0, subsetN))
    uint64_t subsetFp = 0;    // H / F: fingerprint of the points whose checkSubset accepted the rows
    DevBuf<uint64_t> fp;      // [0] the last chunk's points (mark_chunk), [1] the points at finalize / check
    PinnedBuf<uint64_t> h_fp;
    Sampler sampler(const RansacConfig& cfg) const;
    PinnedBuf<int> h_counts;
    PinnedBuf<double> h_red;
    PinnedBuf<float> h_pack;
    PinnedBuf<uint8_t> h_one;
    PinnedBuf<int> h_i;
    PinnedBuf<uint64_t> h_keys;   // per-shard best key + first failure (fixed-iteration searches)

    void reserve(int n, int64_t hyps);
    hipStream_t own_stream();
    ~Plan();
};

Plan& thread_plan(int model, int shard = 0);   // current device; shard > 0: extra per-device workspaces
static const int kMaxShards = 16;

// Sum V doubles over (masked) correspondences: GPU two-stage reduction, result to host.
template <class F>
inline void reduce_to_host(Plan& P, hipStream_t s, int V, double* out, F launch) {
    launch(P.part.p, P.red.p);
    MCV_HIP(hipGetLastError());
    MCV_HIP(hipMemcpyAsync(P.h_red.p, P.red.p, V * sizeof(double), hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < V; ++i) out[i] = P.h_red.p[i];
}

// Opt-in kernel timing with HIP events recorded on the launch stream (bench.py's live roofline).
// mcvProfileEnable(n): every n-th launch of each named scope is timed (n = 1: all of them). An event
// pair costs the stream ~3 us each way, 17 % of the 36 us cfg2 Hamming step when every launch is
// timed (scripts/exp/ham_gap.py); a sample keeps the average launch duration and not that cost.
bool prof_enabled();
bool prof_sample(const char* name);   // prof_enabled() and this launch is one of the sampled ones
void prof_record(const char* name, hipEvent_t a, hipEvent_t b);
hipEvent_t prof_event();   // a timing event (reused across mcvProfileReset)
struct ProfScope {
    const char* name;
    hipStream_t s;
    hipEvent_t a = nullptr, b = nullptr;
    ProfScope(const char* n, hipStream_t st) : name(n), s(st) {
        if (prof_sample(n) && (a = prof_event()) && (b = prof_event())) (void)hipEventRecord(a, s);
    }
    ~ProfScope() {
        if (a && b) {
            (void)hipEventRecord(b, s);
            prof_record(name, a, b);
        }
    }
};
void pack_points(Plan& P, const mcvV2d* a, const mcvV2d* b, int N, float* d_dst, hipStream_t s);
size_t point_bytes(int model, int N);   // device point buffer: 16 N (H / F float4), 32 N (E double4, PnP)
// Evaluate side: P.last = this chunk, and the fingerprint of its points -> P.fp[0] (async).
void mark_chunk(Plan& P, int64_t begin, int64_t count, const Sampler& smp, const void* d_pts, int N, int kind,
                hipStream_t s);
// Finalize side, on the cached-model path: the current points' fingerprint -> P.fp[1], both to
// P.h_fp (async; chunk_fresh reads them after the caller's next stream synchronisation).
void queue_chunk_check(Plan& P, const void* d_pts, int N, hipStream_t s);
inline bool chunk_fresh(const Plan& P) { return P.h_fp.p[0] == P.h_fp.p[1]; }
// The device points' fingerprint, synchronously (CV-sampler table checks).
uint64_t device_fingerprint(Plan& P, const void* d_pts, int N, hipStream_t s);
double effective_threshold(const RansacConfig& cfg);
bool cv_sampler(const RansacConfig& cfg);   // MCV_FLAG_CV_SAMPLER
void check_flags(const RansacConfig& cfg, const char* who);   // rejects the retired bit 4
// OpenCV's subset stream (cv_sampler.cpp): rows [0, rows) for P's model / cfg, uploaded to P.subsets.
// h_pts4: host float4 points for the models with a checkSubset (H, F); nullptr = read from d_pts.
void cv_table_build(int model, const RansacConfig& cfg, const float* h_pts4, int N, int64_t rows, std::vector<int>& out);
void cv_table_upload(Plan& P, const std::vector<int>& t, int m, int64_t rows, int N, uint64_t pointsFp,
                     hipStream_t s);
bool cv_table_reads_points(int model);   // the table depends on the points (H / F checkSubset), not only N
// host float4 points -> the fingerprint a table records (0 for the models whose table ignores them)
uint64_t cv_table_points_fp(int model, const float* h_pts4, int N);
void cv_table_prepare(Plan& P, const void* d_pts, const float* h_pts4, int N, const RansacConfig& cfg, int64_t rows,
                      hipStream_t s);
bool fused_error(const RansacConfig& cfg);
RansacConfig config_or_default(const RansacConfig* cfg);
int64_t ransac_search(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, hipStream_t s,
                      const float* h_pts4 = nullptr);
int finalize(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t hyp, double* model9,
             uint8_t* d_mask, hipStream_t s);
void evaluate_chunk(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t hypBegin, int hypCount,
                    int* d_counts, uint64_t* d_key, hipStream_t s);

// fundamental-matrix family (ransac_f.hip / ransac_f_host.cpp)
int f_error_kind(const RansacConfig& cfg);
int f_finalize(Plan& P, const float* d_pts, int N, const RansacConfig& cfg, int64_t hyp, double* F, uint8_t* d_mask,
               hipStream_t s);
int f_fit_all(Plan& P, const float* d_pts, int N, hipStream_t s, double* F);
int f_host_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F9, float* Ff9, int* sampleIdx,
                      bool fast);

// PnP family (ransac_pnp.hip / pnp_host.cpp)
void p_evaluate_chunk(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t hypBegin, int hypCount,
                      int* d_counts, hipStream_t s);
int p_finalize(Plan& P, const void* d_pts, int N, const RansacConfig& cfg, int64_t hyp, double* model9,
               uint8_t* d_mask, hipStream_t s);
bool pnp_cfg_epnp(const RansacConfig& cfg);   // minimal sets of 5 for EPnP (solverKind 0/1/3/4)

// essential-matrix family (ransac_e.hip / ransac_e_host.cpp)
void e_evaluate_chunk(Plan& P, const double* d_pts, int N, const RansacConfig& cfg, int64_t hypBegin, int hypCount,
                      int* d_counts, hipStream_t s);
int e_finalize(Plan& P, const double* d_pts, int N, const RansacConfig& cfg, int64_t slot, double* E,
               uint8_t* d_mask, hipStream_t s);

}  // namespace mcv
