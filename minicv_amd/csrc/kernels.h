// kernels.h — host-side launchers of the gfx950 kernels (definitions in *.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "epnp.h"

namespace mcv {

// Hypotheses per wave in the inlier sweep (models live in SGPRs: 8 per hypothesis).
static const int kVerifyHypPerWave = 6;
// Correspondences per lane per trip of the sweep (independent loads in flight).
static const int kVerifyPtsPerLane = 2;
// Upper bound of reduction partial blocks (reduce.h).
static const int kReduceMaxBlocksHost = 1024;

// ---- homography (ransac_h.hip)
struct HOneOut {
    double H[9];
    float hf[8];
    int status;
    int idx[4];
};
void launch_h_one(const float* d_pts4, int N, Sampler smp, int64_t hyp, HOneOut* d_out, hipStream_t s, bool fast);
void launch_h_mask_one(const float* d_pts4, int N, const HOneOut* d_one, float thr2, bool fused, uint8_t* d_mask,
                       int* d_count, hipStream_t s);
// d_scratch (h_gen_scratch_bytes(hypCount) bytes): the split eigen generate's rotation log, samples
// and overflow list (ransac_h.hip); nullptr runs the one-pass solve.
void launch_h_generate(const float* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_models,
                       double* d_h64, int* d_counts, hipStream_t s, bool fast, void* d_scratch = nullptr);
size_t h_gen_scratch_bytes(int hypCount);
void launch_h_verify(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount, float thr2,
                     bool fused, const float* d_bbox, hipStream_t s);
void launch_bbox(const float* d_pts4, int N, float* d_bbox, hipStream_t s);
// Packed-f32 sweep of the fused error over the paired layout (ransac_h.hip, HPair: 32 B per 2).
void launch_h_pair(const float* d_pts4, int N, void* d_pairs, hipStream_t s);
void launch_h_verify_packed(const float* d_pts4, const void* d_pairs, int N, const void* d_models, int* d_counts,
                            int hypCount, float thr2, const float* d_bbox, hipStream_t s);
// Certified division-free sweep of the op-by-op error (the default) + exact recount of its redo slots;
// d_bb = launch_abs_bound4 of the float4 points.
void launch_h_verify_certified(const float* d_pts4, const void* d_pairs, int N, const void* d_models, int* d_counts,
                               int hypCount, float thr2, const double* d_bb, hipStream_t s);
void launch_h_mask(const float* d_pts4, int N, const float* hf8, float thr2, bool fused, uint8_t* d_mask,
                   int* d_count, hipStream_t s);
void h_reduce_sums(const float* d_pts4, int N, const uint8_t* d_mask, double* d_part, double* d_out, hipStream_t s);
void h_refit_chain(const float* d_pts4, int N, const uint8_t* d_mask, double* d_part, double* d_red, hipStream_t s);
void h_reduce_absdev(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, double* d_part,
                     double* d_out, hipStream_t s);
void h_reduce_ltl(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, const double* s4,
                  double* d_part, double* d_out, hipStream_t s);
void h_reduce_lm(const float* d_pts4, int N, const uint8_t* d_mask, const double* h8, bool wantJ, double* d_part,
                 double* d_out, hipStream_t s);

// ---- fundamental (ransac_f.hip)
static const int kVerifyFHypPerWave = 4;
static const int kVerifyFPtsPerLane = 2;
struct FOneOut {
    double F[9];
    int status;
    int idx[8];
};
void launch_f_generate(const float* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_models,
                       int* d_counts, hipStream_t s, bool fast);
void launch_f_one(const float* d_pts4, int N, Sampler smp, int64_t hyp, FOneOut* d_out, hipStream_t s, bool fast);
// 7-point (MCV_FLAG_SEVEN_POINT): 3 model slots per hypothesis (models[3h + s], counts[3h + s]).
void launch_f7_generate(const float* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_models,
                        int* d_counts, hipStream_t s);
void launch_f7_one(const float* d_pts4, int N, Sampler smp, int64_t slot, FOneOut* d_out, hipStream_t s);
void launch_f7_direct(const float* d_pts4, FOneOut* d_out, hipStream_t s);   // N == 7: run7Point, first model
void launch_f_verify(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount, float thr2,
                     int kind, hipStream_t s, const double* d_bb = nullptr);
// max |x1|, |y1|, |x2|, |y2| of float4 (fp64 = false) or double4 points -> d_bb[4] (fp64); with
// d_out32 (double4 input) also the float4-rounded copy of the points.
void launch_abs_bound4(const void* d_pts4, bool fp64, int N, double* d_bb, float* d_out32, hipStream_t s);
void launch_f_mask(const float* d_pts4, int N, const double* F9, float thr2, int kind, uint8_t* d_mask, int* d_count,
                   hipStream_t s);
// c4 = {c2x, c2y, c1x, c1y}; d_out = {sum |p2 - c2|, sum |p1 - c1|} (Euclidean).
void f_reduce_eucdev(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, double* d_part,
                     double* d_out, hipStream_t s);
void f_reduce_ata(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, const double* s4,
                  double* d_part, double* d_out, hipStream_t s);

// ---- essential (ransac_e.hip)
static const int kVerifyEModelsPerWave = 4;
static const int kEGenLanes = 16;   // lanes per hypothesis of mcv_e_generate_wave (five_point_wave.h)
static const int kVerifyEPtsPerLane = 2;   // correspondences per lane per trip (variant screen)
static const int kEModelSlots = 10;
struct EOneOut {
    double E[10][9];
    int status;    // model count (0 = no model) or -2 (no sample)
    int idx[5];
};
struct EFiveIn { double x1[5], y1[5], x2[5], y2[5]; };
// Five-point solve split at the root finder (mcv_e_stage -> mcv_e_roots): the null basis, B(z) and
// det B(z) of one hypothesis; status 1 = solved up to the roots, 0 = degenerate, -2 = no sample.
struct EStage {
    double nb[4][9];
    double bx[3][4], by[3][4], bc[3][5];
    double det[11];
    int status, pad;
};
static const int kEStageMinHyps = 32768;   // hypCount from which generate takes the split path
static const int kEStageLanes = 16;        // lanes per hypothesis of its matrix phases
static const int kERootLanes = 4;          // lanes per hypothesis of its root finder (1: one lane)
void launch_e_pack(const double* d_ab, int N, double f, double cx, double cy, double* d_pts4, hipStream_t s);
void launch_e_generate(const double* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_dense,
                       int* d_denseSlot, int* d_nDense, int* d_counts, void* d_stage, hipStream_t s);
void launch_e_verify(const double* d_pts4, int N, const void* d_dense, const int* d_denseSlot, const int* d_nDense,
                     int maxModels, int* d_counts, float thr2, int kind, hipStream_t s, const float* d_pts32 = nullptr,
                     const double* d_bb = nullptr);
// The reference's five-point solver (five_point_ref.h) over a chunk: the default RANSAC generate.
size_t e5_stage_bytes(int hypCount);
void launch_e5_generate(const double* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_dense,
                        int* d_denseSlot, int* d_nDense, int* d_counts, void* d_stage, hipStream_t s);
void launch_e5_one(const double* d_pts4, int N, Sampler smp, int64_t hyp, EOneOut* d_out, hipStream_t s);
void launch_e_fetch(const void* d_dense, const int* d_denseSlot, const int* d_nDense, int maxModels, int slot,
                    void* d_out, int* d_found, hipStream_t s);
void launch_e_one(const double* d_pts4, int N, Sampler smp, int64_t hyp, EOneOut* d_out, hipStream_t s);
void launch_e_mask(const double* d_pts4, int N, const double* E9, float thr2, int kind, uint8_t* d_mask, int* d_count,
                   hipStream_t s);
void launch_e_cheirality(const double* d_pts4, int N, const uint8_t* d_mask, const double* P4x12, double dist,
                         int* d_good4, hipStream_t s);
void launch_e_fivepoint(const EFiveIn& in, EOneOut* d_out, hipStream_t s);

// ---- PnP (ransac_pnp.hip); cam8 = {fx, fy, cx, cy, k1, k2, p1, p2}
static const int kVerifyPnpPosesPerWave = 3;
struct PnpOneOut {
    double R[9];
    double t[3];
    int status;
    int idx[5];
};
struct Ap3pIn { double mu[3], mv[3], W[3][3], inv_fx, inv_fy, cx_fx, cy_fy; };
struct Ap3pOut {
    double R[4][9];
    double t[4][3];
    int count;
    int cplx;   // the quartic took the complex-pow branch (glibc's clog / exp / cos / atan2, restated)
};
void launch_pnp_pack(const double* d_img, const double* d_world, int N, void* d_pts, hipStream_t s);
// fast (MCV_FLAG_FAST_MINIMAL): the AP3P kernel's real-root-finder quartic instead of the reference's Ferrari
// d_epnpScratch: kEpnpSplitDoubles x min(hypCount, kEpnpPiece) doubles (EPnP's split generate runs over
// sub-ranges of kEpnpPiece hypotheses; unused by AP3P). Round 6: 2^20 (2.4 GB at 2^20 hypotheses): one
// piece per chunk, 27.3-27.5 ms a PnP step against 27.9-28.2 ms with 2^18 pieces (610 MB; each of the
// five kernels per piece drains its slowest waves) and 27.7-27.9 with 2^19, same box alternating.
static const int kEpnpPiece = 1 << 20;
void launch_pnp_generate(const void* d_pts, int N, const double* cam8, Sampler smp, int64_t hypBegin, int hypCount,
                         bool epnp, void* d_models, int* d_counts, double* d_epnpScratch, hipStream_t s,
                         bool fast = false);
// d_ext: 3 doubles of device scratch filled by launch_pnp_extent (the certified sweep's bound);
// d_pairs: kPnpPairFloatsPerPoint x N floats it fills with the sweep's pair layout.
static const int kPnpPairFloatsPerPoint = 6;
void launch_pnp_extent(const void* d_pts, int N, double* d_ext, float* d_pairs, hipStream_t s);
void launch_pnp_verify(const void* d_pts, int N, const double* cam8, const void* d_models, int* d_counts, int hypCount,
                       float thr2, bool fused, const double* d_ext, const float* d_pairs, hipStream_t s);
void launch_pnp_one(const void* d_pts, int N, const double* cam8, Sampler smp, int64_t hyp, bool epnp,
                    PnpOneOut* d_out, hipStream_t s, bool fast = false);
void launch_pnp_solve5(const void* d_pts, const double* cam8, PnpOneOut* d_out, hipStream_t s);
void launch_mask_compact(const uint8_t* d_mask, int N, int* d_idx, int* d_count, hipStream_t s);
// EPnP over n points: d_pts (+ optional index list d_idx) fp32 PnpPoints, or d_img / d_world fp64.
// normalized: d_us = undistortPoints' normalised coordinates (SQPnP) instead of x f + c (EPnP).
// d_n (optional, fp32 points only): the point count on the device (a compaction's output); n is then
// an upper bound that sizes the grid.
void launch_epnp_prep(const void* d_pts, const int* d_idx, const double* d_img, const double* d_world, int n,
                      const double* cam8, double* d_pw, double* d_us, hipStream_t s, bool normalized = false,
                      const int* d_n = nullptr);
// SQPnP passes (sqpnp.h): the 39 computeOmega sums; the positive-depth count of the pose R[0] / t[0].
enum { kEpnpPassSumPw = 0, kEpnpPassPw0 = 1, kEpnpPassMtm = 2, kEpnpPassPc = 3, kEpnpPassAbt = 4, kEpnpPassReproj = 5,
       kEpnpPassSqp = 6, kEpnpPassSqpDepth = 7 };
struct EpnpPassArgs {
    EpnpCtrl C;
    EpnpCam cam;
    double c0[3];            // Pw0: centroid
    double ccs[3][4][3];     // Pc / Abt: sign-fixed control points of N = 1, 2, 3
    double pc0[3][3];        // Abt
    double pw0[3];           // Abt
    double R[3][3][3];       // Reproj
    double t[3][3];
};
// d_n (optional): the point count on the device, n an upper bound; the partials keep the stride of the
// device count's blocks (part[acc * nblk + blk], nblk = ceil(*d_n / kEpnpBlock)). d_prev (optional, Pw0 /
// Abt): the previous pass's partials, from which the pass takes its centroid / pc0 on the device.
void launch_epnp_pass(int mode, const double* d_pw, const double* d_us, int n, const EpnpPassArgs& a, int nacc,
                      double* d_part, hipStream_t s, const int* d_n = nullptr, const double* d_prev = nullptr);
void launch_pnp_solve4(const void* d_pts, const double* cam8, PnpOneOut* d_out, hipStream_t s, bool fast = false);
void launch_pnp_mask(const void* d_pts, int N, const double* cam8, const double* R9, const double* t3, float thr2,
                     bool fused, uint8_t* d_mask, int* d_count, hipStream_t s);
// The same mask for a pose already on the device (a chunk's model slot): no host round trip first.
void launch_pnp_mask_dev(const void* d_pts, int N, const double* cam8, const void* d_pose, float thr2, bool fused,
                         uint8_t* d_mask, int* d_count, hipStream_t s);
void launch_pnp_ap3p(const Ap3pIn& in, Ap3pOut* d_out, hipStream_t s);
void pnp_reduce_lm(const void* d_pts, int N, const uint8_t* d_mask, const double* cam8, const double* R9,
                   const double* t3, const double* dR27, bool wantJ, double* d_part, double* d_out, hipStream_t s);
void pnp_reduce_vvs(const void* d_pts, int N, const uint8_t* d_mask, const double* cam8, const double* R9,
                    const double* t3, double* d_part, double* d_out, hipStream_t s);

// ---- shared (ransac_h.hip)
void launch_best(const int* d_counts, int n, int64_t hypBegin, int minCount, uint64_t* d_pkey, int64_t* d_pfail,
                 uint64_t* d_out, hipStream_t s);
void launch_fill_u8(uint8_t* d, int n, uint8_t v, hipStream_t s);

// ---- point-buffer fingerprints (plan_guard.hip; mcv_common.h fp_term): d_out = the sum, async
void launch_fingerprint(const void* d_buf, size_t bytes, uint64_t* d_out, hipStream_t s);
uint64_t host_fingerprint(const void* h_buf, size_t bytes);

// ---- match -> RANSAC hand-off (match_pipeline.hip)
void launch_match_compact(const int* d_idx, const int* d_di1, const int* d_di2, const float* d_df1,
                          const float* d_df2, const int* d_idxBack, int nq, float ratio, float maxDist,
                          const uint8_t* d_kpA, const uint8_t* d_kpB, int kpStride, uint8_t* d_keep, int* d_cnt,
                          int* d_off, int* d_pairs, float* d_dist, float* d_pts4, hipStream_t s);

// ---- matchers (match_hamming.hip, match_l2.hip)
static constexpr int kHammingFormGemm = 0, kHammingFormPopcount = 1;
int launch_match_hamming(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int bytesPerDesc, int* d_idx,
                         int* d_dist, int* d_idx2, int* d_dist2, hipStream_t s, int form = kHammingFormGemm);
int launch_match_l2(const float* d_q, int nq, const float* d_t, int nt, int dim, int* d_idx, float* d_dist,
                    int* d_idx2, float* d_dist2, hipStream_t s);
int l2_last_exact_scans();
int l2_last_gemm_form();

// ---- CameraPose.findScaled (scaled_pose.hip)
struct ScaledSetup;
void launch_scaled(const ScaledSetup& S, const double* d_w3, const double* d_o2, int N, double* d_soa,
                   double* d_scales, uint8_t* d_used, double* d_costs, long long* d_out, hipStream_t s);

}  // namespace mcv
