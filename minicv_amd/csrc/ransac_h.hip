// ransac_h.hip — gfx950 kernels of the homography RANSAC hot path.
//
//   mcv_h_generate  one lane per hypothesis: Philox sample -> subset check -> 4-pt DLT (fp64)
//                   -> fp32 model (32 B) + status.                       [SURVEY §2 K1, first half]
//   mcv_h_verify<K> the inlier sweep: each wave owns K hypotheses held in SGPRs and streams all N
//                   packed correspondences (float4, 16 B, coalesced, L2-resident) through its 64
//                   lanes; per hypothesis one v_cmp + wave ballot + s_bcnt1 -> scalar count.
//                                                                        [SURVEY §2 K1, the hot loop]
//   mcv_best_*      packed-key argmax (count << 32 | ~idx) with OpenCV's "first strictly greater
//                   wins" order and the sampler-failure `break`.         [SURVEY §2 K3]
//   mcv_h_mask      inlier mask of the winning model (same fp32 error).  [SURVEY §2 K4, mask]
//   refit / LM      fixed-order fp64 reductions over the inliers (reduce.h): centroid, mean |dev|,
//                   the 9x9 LtL of runKernel, and the 8x8 JtJ / Jtr / |r|^2 of the LM refine.
//
// Built with -ffp-contract=off (see hyp_homography.h): the fp32 error rounds exactly like the
// host oracle, which is what makes the inlier masks bit-exact.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include "mcv_common.h"
#include "hyp_homography.h"
#include "reduce.h"
#include "kernels.h"
#include "minicv_native.h"

namespace mcv {

// ------------------------------------------------------------------------------------------
// Hypothesis generation
// ------------------------------------------------------------------------------------------
// One lane per hypothesis; the runKernel eigen-solve's working set (127 doubles) in LDS, one slice
// per lane (jacobi_eig.h): 40.6 KB per 40-lane block, 4 blocks per CU. FAST = MCV_FLAG_FAST_MINIMAL
// (no workspace).
template <bool FAST, int L = kEigLanes>
__global__ __launch_bounds__(FAST ? 256 : L) void mcv_h_generate(const float* __restrict__ pts4, int N, Sampler smp,
                                                     int64_t hypBegin, int hypCount, HModelF* __restrict__ models,
                                                     double* __restrict__ h64, int* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hypCount) return;
    double H[9];
    HModelF mf;
    int st;
    if constexpr (FAST) {
        EigWsLocal unused;   // the elimination never touches it (folded away)
        st = h_hypothesis(pts4, N, smp, (uint64_t)(hypBegin + i), H, &mf, nullptr, unused, true);
    } else {
        __shared__ double lds[kEigWs * L];
        EigWsLane ws{lds + threadIdx.x * kEigWs};
        st = h_hypothesis(pts4, N, smp, (uint64_t)(hypBegin + i), H, &mf, nullptr, ws);
    }
    if (st == 1) {
        models[i] = mf;
        for (int j = 0; j < 9; ++j) h64[9 * (int64_t)i + j] = H[j];
        counts[i] = 0;
    } else {
        // the zero model (w = 1 everywhere) keeps the packed sweep's slot well-defined
        for (int j = 0; j < 8; ++j) mf.h[j] = 0.f;
        models[i] = mf;
        counts[i] = st;
    }
}

// The default generate as two passes over the split eigen-solve (round 6; jacobi_eig.h):
//   mcv_h_gen_aw  lane per hypothesis: sample, subset check, runKernel's normalisation and LtL, then
//                 JacobiImpl_ on the upper triangle and W only (a 45-double LDS slice per lane, 360 B
//                 against the one-pass solve's 1016 B: 2.8x the lanes per CU) with every rotation's
//                 (c, s, k, l) logged to HBM (16 B; SoA by hypothesis, so a wave's log writes and reads
//                 are contiguous); the sort of W names the eigenvector's row r;
//   mcv_h_gen_v   lane per hypothesis: V rebuilt from the log (an 81-double slice), row r -> H0, the
//                 de-normalisation and the fp32 model (the normalisation recomputed from the stored
//                 sample's four points);
//   mcv_h_gen_ovf the one-pass solve for the lanes whose rotation count exceeded the log's capacity
//                 (kEigLogCap; a cfg3 LtL takes 110-157 rotations) — normally none.
// Every value is computed by the same operations in the same order as the one-pass solve, so the
// models are the same bits (tests: the whole-range cfg3 counts, the eigen stress test).
static constexpr int kEigLogCap = 192;
// the log rows pass 1 may use (mcvTestEigLogCap lowers it so the tests drive the overflow path)
static int g_eig_log_cap = kEigLogCap;
// 56 x 360 B = 19.7 KB: 8 blocks (two waves per SIMD) per CU. Screen (with 376-byte slices): 40 / 64 /
// 32-lane blocks (10 / 6 / 13 per CU) 6.6 / 5.7 / 6.7 ms against 5.2 ms of generate per 2^20 at 54.
static constexpr int kHGenAwLanes = 56;
// pass 2: one column of V per lane (9 lanes per hypothesis, 7 hypotheses per 63-lane block), 4 log
// loads in flight. Round-6 screen at cfg3 (generate ms per 2^20 hypotheses, pass 1 ~3.7 of it): one
// lane per hypothesis with one load ahead 5.78, with 8 ahead 5.78; 3 lanes x 3 columns 5.16-5.17 (V
// transposed 5.06); 9 lanes 4.76-4.81 (8 loads ahead, V transposed, 14 hypotheses per block: the same).
// Every 9-lane form moves the same 288 LDS bytes per rotation and hypothesis: LDS-bandwidth-bound.
static constexpr int kHGenVG = 9, kHGenVQ = 7, kHGenVD = 4;
static constexpr int kHGenOvfBlocks = 64;
// meta: >= 0 -> rotation count | r << 16 (pass 2 builds the model); kMetaDone: pass 1 wrote the
// status; kMetaOverflow: mcv_h_gen_ovf solves it
static constexpr int kMetaDone = -1, kMetaOverflow = -2;

__device__ __forceinline__ void h_store_none(HModelF* models, int* counts, int i, int st) {
    HModelF mf;
    for (int j = 0; j < 8; ++j) mf.h[j] = 0.f;   // the zero model (w = 1) keeps the sweep's slot defined
    models[i] = mf;
    counts[i] = st;
}

template <int L>
__global__ __launch_bounds__(L) void mcv_h_gen_aw(const float* __restrict__ pts4, int N, Sampler smp,
                                                  int64_t hypBegin, int count, HModelF* __restrict__ models,
                                                  int* __restrict__ counts, int4* __restrict__ sidx,
                                                  int* __restrict__ meta, EigRot* __restrict__ log, int logStride,
                                                  int* __restrict__ ovf, int ovfBase, int logCap) {
    const int j = blockIdx.x * L + threadIdx.x;   // lane within the piece
    if (j >= count) return;
    const int i = ovfBase + j;                    // hypothesis within the chunk
    __shared__ double lds[kEigAwWs * L];
    EigWsLane ws{lds + threadIdx.x * kEigAwWs};
    float sx[4], sy[4], dx[4], dy[4];
    int idx[4];
    double nm[8];
    int st = 0;
    if (!h_sample(pts4, N, smp, (uint64_t)(hypBegin + i), sx, sy, dx, dy, idx)) st = kStatusNoSample;
    else if (!h_norm4(sx, sy, dx, dy, nm) || !h_ltl4(sx, sy, dx, dy, nm, ws)) st = kStatusNoModel;
    if (st != 0) {
        h_store_none(models, counts, i, st);
        meta[j] = kMetaDone;
        return;
    }
    double w[9];
    int nrot = 0;
    const int r = eig9_jacobi<EigWsLane, true>(ws, w, 8, &nrot, log + j, logStride, logCap);
    sidx[j] = make_int4(idx[0], idx[1], idx[2], idx[3]);
    if (nrot < 0) {
        meta[j] = kMetaOverflow;
        ovf[1 + atomicAdd(ovf, 1)] = i;
        return;
    }
    meta[j] = nrot | (r << 16);
}

// Pass 2: G lanes per hypothesis (9 / G columns of V each; G = 1 or 3), Q hypotheses per block.
template <int G, int Q, int D, bool TR = false>
__global__ __launch_bounds__(G * Q) void mcv_h_gen_v(const float* __restrict__ pts4, int count, int base,
                                                     const int4* __restrict__ sidx, const int* __restrict__ meta,
                                                     const EigRot* __restrict__ log, int logStride,
                                                     HModelF* __restrict__ models, double* __restrict__ h64,
                                                     int* __restrict__ counts) {
    constexpr int C = 9 / G;
    const int h = threadIdx.x / G, g = threadIdx.x - h * G;   // hypothesis of the block, column group
    const int j = blockIdx.x * Q + h;
    __shared__ double lds[kEigVWs * Q];
    EigWsLane v{lds + h * kEigVWs};
    const int m = j < count ? meta[j] : kMetaDone;
    if (m >= 0) {
#pragma unroll
        for (int i = 0; i < 9; ++i)
#pragma unroll
            for (int c = 0; c < C; ++c) v[TR ? 9 * (g * C + c) + i : 9 * i + g * C + c] = (i == g * C + c) ? 1.0 : 0.0;
        eig9_replay_cols<C, D, TR>(v, g * C, log + j, logStride, m & 0xffff);
    }
    if constexpr (G > 1) __syncthreads();   // the row's other columns come from the group's other lanes
    if (m < 0 || g != 0) return;
    const int i = base + j;
    const int r = m >> 16;
    double H0[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) H0[k] = v[TR ? 9 * k + r : 9 * r + k];
    const int4 id = sidx[j];
    const int ix[4] = {id.x, id.y, id.z, id.w};
    float sx[4], sy[4], dx[4], dy[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 q = reinterpret_cast<const float4*>(pts4)[ix[k]];
        sx[k] = q.x; sy[k] = q.y; dx[k] = q.z; dy[k] = q.w;
    }
    double nm[8], H[9];
    HModelF mf;
    (void)h_norm4(sx, sy, dx, dy, nm);   // pass 1 accepted this sample: the same values again
    if (h_from_eig(H0, nm, H) && h_model_f(H, &mf)) {
        models[i] = mf;
        for (int k = 0; k < 9; ++k) h64[9 * (int64_t)i + k] = H[k];
        counts[i] = 0;
    } else {
        h_store_none(models, counts, i, kStatusNoModel);
    }
}

template <int L>
__global__ __launch_bounds__(L) void mcv_h_gen_ovf(const float* __restrict__ pts4, int N, Sampler smp,
                                                   int64_t hypBegin, const int* __restrict__ ovf,
                                                   HModelF* __restrict__ models, double* __restrict__ h64,
                                                   int* __restrict__ counts) {
    __shared__ double lds[kEigWs * L];
    EigWsLane ws{lds + threadIdx.x * kEigWs};
    const int n = ovf[0];
    for (int j = blockIdx.x * L + threadIdx.x; j < n; j += gridDim.x * L) {
        const int i = ovf[1 + j];
        double H[9];
        HModelF mf;
        const int st = h_hypothesis(pts4, N, smp, (uint64_t)(hypBegin + i), H, &mf, nullptr, ws);
        if (st == 1) {
            models[i] = mf;
            for (int k = 0; k < 9; ++k) h64[9 * (int64_t)i + k] = H[k];
            counts[i] = 0;
        } else {
            h_store_none(models, counts, i, st);
        }
    }
}

// One hypothesis in full (finalize path): fp64 model, fp32 model, status, sample.
__global__ void mcv_h_one(const float* __restrict__ pts4, int N, Sampler smp, int64_t hyp, HOneOut* __restrict__ out,
                          bool fast) {
    __shared__ double lds[kEigWs];
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    EigWsLane ws{lds};
    HOneOut o;
    HModelF mf;
    for (int j = 0; j < 9; ++j) o.H[j] = 0;
    for (int j = 0; j < 8; ++j) mf.h[j] = 0;
    o.status = h_hypothesis(pts4, N, smp, (uint64_t)hyp, o.H, &mf, o.idx, ws, fast);
    for (int j = 0; j < 8; ++j) o.hf[j] = mf.h[j];
    *out = o;
}

// ------------------------------------------------------------------------------------------
// Inlier sweep. Wave w evaluates hypotheses [w*K, w*K+K). The hypothesis index is made provably
// wave-uniform (readfirstlane), so the models come in through scalar loads and every VALU op
// reads its model coefficient straight from an SGPR; the counts accumulate in SGPRs too.
// ------------------------------------------------------------------------------------------
// Class mask of v_cmp_class_f32 for "not a normal number" (sNaN, qNaN, +-inf, +-denormal, +-0).
static constexpr int kClassNotNormal = 0x001 | 0x002 | 0x004 | 0x010 | 0x020 | 0x040 | 0x080 | 0x200;

// Wave mask of lanes whose w falls in the classes `cls`: one v_cmp_class_f32 writing an SGPR pair
// (the builtin + ballot pair lowers to cmp + cndmask + cmp on ROCm 7.2).
__device__ __forceinline__ uint64_t class_mask(float w, int cls) {
    uint64_t m;
    asm("v_cmp_class_f32_e64 %0, %1, %2" : "=s"(m) : "v"(w), "s"(cls));
    return m;
}

// One trip of the sweep: P correspondences per lane against the wave's K hypotheses.
// PRED: lane predicates (ragged tail only). FUSED fast path: rcp_newton, with the trip redone by
// IEEE division when any denominator is zero / denormal / non-finite.
template <int K, int P, bool FUSED, bool PRED>
__device__ __forceinline__ void h_sweep_trip(const float (&hm)[K][8], const float4 (&q)[P], const bool (&v)[P],
                                             float thr2, bool fast, uint32_t (&cnt)[K]) {
    auto vote = [&](int j, bool pred) -> uint32_t {
        if constexpr (PRED)
            return (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(v[j] && pred));
        else
            return (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(pred));
    };
    if constexpr (FUSED) {
        if (fast) {
            uint64_t bad = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) {
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    const float w = h_denominator_fused(hm[k], q[j].x, q[j].y);
                    bad |= class_mask(w, kClassNotNormal);
                    const float e = h_error_fused_ww(hm[k], q[j].x, q[j].y, q[j].z, q[j].w, rcp_newton(w));
                    cnt[k] += vote(j, e <= thr2);
                }
            }
            if (__builtin_expect(bad == 0, 1)) return;
#pragma unroll
            for (int k = 0; k < K; ++k) {   // replace this trip's fast counts by the exact ones
#pragma unroll
                for (int j = 0; j < P; ++j) {
                    const float w = h_denominator_fused(hm[k], q[j].x, q[j].y);
                    const float f = h_error_fused_ww(hm[k], q[j].x, q[j].y, q[j].z, q[j].w, rcp_newton(w));
                    const float e = h_error_fused_ww(hm[k], q[j].x, q[j].y, q[j].z, q[j].w, 1.f / w);
                    cnt[k] = cnt[k] - vote(j, f <= thr2) + vote(j, e <= thr2);
                }
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)   // exact for the whole wave
#pragma unroll
            for (int j = 0; j < P; ++j)
                cnt[k] += vote(j, h_error_fused(hm[k], q[j].x, q[j].y, q[j].z, q[j].w) <= thr2);
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < P; ++j) cnt[k] += vote(j, h_error(hm[k], q[j].x, q[j].y, q[j].z, q[j].w) <= thr2);
    }
}

// redo: count only the slots the packed sweep marked kStatusRedo (a wave with none exits).
template <int K, int P, bool FUSED>
__global__ __launch_bounds__(256) void mcv_h_verify(const float4* __restrict__ pts, int N,
                                                    const HModelF* __restrict__ models, int* __restrict__ counts,
                                                    int hypCount, float thr2, const float* __restrict__ bbox,
                                                    int redo) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;

    float hm[K][8];
    bool valid[K];
    bool any = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = (hk < hypCount) && (redo ? counts[hk] == kStatusRedo : counts[hk] >= 0);
        any = any || valid[k];
        const HModelF m = models[valid[k] ? hk : h0];
#pragma unroll
        for (int j = 0; j < 8; ++j) hm[k][j] = valid[k] ? m.h[j] : __builtin_nanf("");
        // h2 and h5 meet another uniform operand in fma(h1, y, h2) / fma(h4, y, h5); a VALU op
        // reads at most one SGPR (gfx9 constant-bus limit), so keep those two in VGPRs and the
        // other six in SGPRs (no per-use v_mov, and SGPR pressure stays below the spill point).
        asm volatile("" : "+v"(hm[k][2]));
        asm volatile("" : "+v"(hm[k][5]));
    }

    if (!any) return;
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;

    // Fused fast path precondition, per hypothesis: max |w| over the points' bounding box stays
    // below 2^125, so every denominator is below 2^126 (the exhaustively verified range of
    // rcp_newton). The lower end (0, denormal, inf, NaN) is checked per point.
    bool fast = FUSED;
    if constexpr (FUSED) {
        const float X = bbox[0], Y = bbox[1];
        bool anyValidBig = false;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float wmax = fabsf(hm[k][6]) * X + fabsf(hm[k][7]) * Y + 1.f;
            anyValidBig = anyValidBig || (valid[k] && !(wmax < 0x1p125f));
        }
        fast = !anyValidBig;
    }

    // Wave-uniform trip count (the counts are per-wave SGPR sums of ballots: every lane must take
    // part in every ballot). P correspondences per lane per trip (P loads in flight); full trips
    // run unpredicated, the ragged tail once with lane predicates.
    constexpr int TRIP = 64 * P;
    const int nFull = N / TRIP * TRIP;
    bool vt[P];
#pragma unroll
    for (int j = 0; j < P; ++j) vt[j] = true;
    for (int base = 0; base < nFull; base += TRIP) {
        float4 q[P];
#pragma unroll
        for (int j = 0; j < P; ++j) q[j] = pts[base + 64 * j + lane];
        h_sweep_trip<K, P, FUSED, false>(hm, q, vt, thr2, fast, cnt);
    }
    if (nFull < N) {
        float4 q[P];
        bool v[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int p = nFull + 64 * j + lane;
            v[j] = p < N;
            q[j] = pts[v[j] ? p : 0];
        }
        h_sweep_trip<K, P, FUSED, true>(hm, q, v, thr2, fast, cnt);
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) counts[h0 + k] = (int)cnt[k];
    }
}

// ------------------------------------------------------------------------------------------
// Packed-f32 inlier sweep (fused error). Two correspondences share a 64-bit VGPR pair per
// coordinate, so every FMA of the error runs as one v_pk_fma_f32 over both (a VOP3 v_fma_f32
// issues at the same cost as a v_pk_fma_f32 on gfx950: the packed form halves the FMA issue).
// Layout: HPair p = correspondences (2p, 2p+1) as {x, y, x', y'} pairs, 32 B; an odd N is padded
// with {0, 0, NaN, NaN}, whose error is NaN (never an inlier) and whose w is 1 (never "bad").
// Model coefficients stay in SGPRs and are broadcast to both halves with op_sel / op_sel_hi.
// Every operation rounds exactly like h_denominator_fused / rcp_newton / h_error_fused_ww.
// ------------------------------------------------------------------------------------------
typedef float f2 __attribute__((ext_vector_type(2)));
struct HPair {
    f2 x, y, mx, my;
};

__global__ __launch_bounds__(256) void mcv_h_pair(const float4* __restrict__ pts, int N, HPair* __restrict__ out) {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= (N + 1) / 2) return;
    const float4 a = pts[2 * p];
    const float nan = __builtin_nanf("");
    const float4 b = 2 * p + 1 < N ? pts[2 * p + 1] : make_float4(0.f, 0.f, nan, nan);
    HPair o;
    o.x = f2{a.x, b.x};
    o.y = f2{a.y, b.y};
    o.mx = f2{a.z, b.z};
    o.my = f2{a.w, b.w};
    out[p] = o;
}

// Packed FMA through the compiler (llvm.fma.v2f32 -> v_pk_fma_f32): it folds a splat of an SGPR
// coefficient into op_sel / op_sel_hi and inserts the wait states between dependent packed ops
// (hand-written asm would not get them: the hazard recognizer does not see into inline asm).
__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// Broadcast one half of a coefficient pair: a shuffle the backend folds into op_sel / op_sel_hi.
__device__ __forceinline__ f2 lo(f2 v) { return __builtin_shufflevector(v, v, 0, 0); }
__device__ __forceinline__ f2 hi(f2 v) { return __builtin_shufflevector(v, v, 1, 1); }

// One trip: NP pairs per lane against the wave's K hypotheses.
template <int K, int NP, bool PRED>
__device__ __forceinline__ void h_pk_trip(const f2 (&hp)[K][4], const f2 (&hc)[K], const HPair (&q)[NP],
                                          const bool (&v)[NP], float thr2, f2 one, uint32_t (&cnt)[K],
                                          float (&wmin)[NP]) {
    auto vote = [&](int j, bool pred) -> uint32_t {
        if constexpr (PRED)
            return (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(v[j] && pred));
        else
            return (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(pred));
    };
#pragma unroll
    for (int k = 0; k < K; ++k) {
        // Re-define the pairs in the trip (no instruction): a broadcast is then built per use and
        // folds into op_sel / op_sel_hi, instead of being hoisted out of the loop as a splat pair
        // (which doubles the SGPRs the models take and spills them).
        f2 p0 = hp[k][0], p1 = hp[k][1], p2 = hp[k][2], p3 = hp[k][3];   // (h0,h1) .. (h6,h7)
        f2 c = hc[k];                                                       // (h2, h5)
        asm volatile("" : "+s"(p0), "+s"(p1), "+s"(p2), "+s"(p3), "+v"(c));
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            f2 W = pk_fma(lo(p3), q[j].x, pk_fma(hi(p3), q[j].y, one));
            const f2 U = pk_fma(lo(p0), q[j].x, pk_fma(hi(p0), q[j].y, lo(c)));
            const f2 V = pk_fma(hi(p1), q[j].x, pk_fma(lo(p2), q[j].y, hi(c)));
            // smallest |w| per lane and pair slot (one v_min3_f32 with |.| modifiers; an fma result
            // is canonical, so no quieting op): |w| < 2^-126 (0, denormal) is a "bad" denominator.
            // One accumulator per slot j keeps the min chains short (a single running min was
            // 4% slower than the two v_cmp_class per pair it replaces; two chains are 4% faster).
            // A NaN w (NaN point) is not tracked: the fast and the exact error are both NaN there
            // (outlier); the bounding-box precondition rules out an infinite w.
            wmin[j] = __builtin_fminf(__builtin_fminf(wmin[j], __builtin_fabsf(W.x)), __builtin_fabsf(W.y));
            f2 R = f2{__builtin_amdgcn_rcpf(W.x), __builtin_amdgcn_rcpf(W.y)};
            const f2 E = pk_fma(-W, R, one);              // fma(-w, r, 1)
            R = pk_fma(E, R, R);                          // fma(e, r, r)
            const f2 DX = pk_fma(U, R, -q[j].mx);         // fma(u, r, -x')
            const f2 DY = pk_fma(V, R, -q[j].my);         // fma(v, r, -y')
            const f2 ERR = pk_fma(DX, DX, DY * DY);       // fma(ex, ex, ey * ey)
            cnt[k] += vote(j, ERR.x <= thr2) + vote(j, ERR.y <= thr2);
        }
    }
}

// A wave whose hypotheses fail the bounding-box precondition, or which meets a "bad" denominator
// (0, denormal, inf, NaN) in any trip, marks its valid slots kStatusRedo instead of writing
// counts; mcv_h_verify<.., redo = true> then recounts exactly those slots with the scalar sweep
// (IEEE division fallback). Keeping the exact path out of this kernel keeps its registers free.
template <int K, int NP>
__global__ __launch_bounds__(256) void mcv_h_verify_pk(const HPair* __restrict__ pairs, int nPairs,
                                                       const HModelF* __restrict__ models, int* __restrict__ counts,
                                                       int hypCount, float thr2, const float* __restrict__ bbox) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;

    // Every slot below hypCount holds a model (mcv_h_generate writes the zero model, w = 1, for a
    // failed hypothesis); slots past hypCount re-read the last one. Reading the models unselected
    // keeps the (h0,h1) .. (h6,h7) SGPR pairs intact: coefficients broadcast by op_sel.
    f2 hp[K][4], hc[K];
    bool valid[K];
    const float X = bbox[0], Y = bbox[1];
    bool fast = true;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = (hk < hypCount) && (counts[hk] >= 0);
        const f2* mp = (const f2*)&models[hk < hypCount ? hk : hypCount - 1];
#pragma unroll
        for (int j = 0; j < 4; ++j) hp[k][j] = mp[j];
        // h2, h5 are the addends of fma(h1, y, h2) / fma(h4, y, h5), beside an SGPR multiplier:
        // one VGPR pair per hypothesis (constant-bus limit), broadcast by op_sel as well.
        hc[k] = f2{hp[k][1].x, hp[k][2].y};
        asm volatile("" : "+v"(hc[k]));
        // precondition (as mcv_h_verify): max |w| over the bounding box below 2^125
        const float wmax = fabsf(hp[k][3].x) * X + fabsf(hp[k][3].y) * Y + 1.f;
        fast = fast && !(valid[k] && !(wmax < 0x1p125f));
    }
    const f2 one = f2{1.f, 1.f};

    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    float wmin[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) wmin[j] = 1.0f;
    if (fast) {
        constexpr int TRIP = 64 * NP;
        const int nFull = nPairs / TRIP * TRIP;
        bool vt[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) vt[j] = true;
        for (int base = 0; base < nFull; base += TRIP) {
            HPair q[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j) q[j] = pairs[base + 64 * j + lane];
            h_pk_trip<K, NP, false>(hp, hc, q, vt, thr2, one, cnt, wmin);
        }
        if (nFull < nPairs) {
            HPair q[NP];
            bool v[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j) {
                const int p = nFull + 64 * j + lane;
                v[j] = p < nPairs;
                q[j] = pairs[v[j] ? p : 0];
            }
            h_pk_trip<K, NP, true>(hp, hc, q, v, thr2, one, cnt, wmin);
        }
    }
    float wm = wmin[0];
#pragma unroll
    for (int j = 1; j < NP; ++j) wm = __builtin_fminf(wm, wmin[j]);
    const bool redo = !fast || __builtin_amdgcn_ballot_w64(!(wm >= 0x1p-126f)) != 0;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) counts[h0 + k] = redo ? kStatusRedo : (int)cnt[k];
    }
}

// ------------------------------------------------------------------------------------------
// Certified division-free sweep of the op-by-op error (the default: OpenCV's computeError as an
// x86-64 SSE build evaluates it, h_error). Per pair of correspondences in packed f32:
//   W = fma(h6,x,fma(h7,y,1)), U = fma(h0,x,fma(h1,y,h2)), V likewise,
//   DX = fma(-x',W,U), DY = fma(-y',W,V), L = fma(DX,DX,fma(DY,DY,b_in)), W2 = W*W,
//   I = fma(W2, a_in, L), X = fma(W2, d, b_x);
//   I < 0                     -> certified inlier
//   bits(I) <= bits(X)        -> undecided (0 <= I <= X as floats); otherwise certified outlier.
// The reference error times w^2 lies within relative (t + O(u)) and absolute O(u^2 G^2 / t) of
// DX^2 + DY^2, and w^2 within the same of W2 (derivation in DESIGN.md §4); a_in, d (launch) and
// b_in, b_x (per model) put the two cuts outside those intervals, so a decided lane has the answer
// of the op-by-op fp32 error bit for bit. 13 packed ops + 4 VOPC e32 compares per pair, no
// reciprocal (the fused sweep: 12 packed + 2 v_rcp_f32 + v_min3 + 2 compares). Undecided lanes
// (where points crowd the threshold, ~1e-4 of evaluations on the cfg3 data) are recorded per trip
// and resolved after the sweep with the exact error and IEEE division.
// ------------------------------------------------------------------------------------------
// Band parameter: relative half-width ~ t + O(u) around thr2 w^2, absolute part ~ (7.5 u G)^2 / t.
// One t for every model keeps the slopes launch constants.
static constexpr double kCertT = 0x1p-11;   // band parameter (screened 2^-12 / 2^-11 / 2^-10: DESIGN.md §7)
static constexpr double kCertSlop = 0x1p-18;   // covers the O(u) factors (< 16 u = 2^-20 in total)

struct HCertSlopes {
    f2 a;       // {a_in (<= 0), d (>= 0)}
    double t;   // band parameter the per-model offsets use
};

HCertSlopes h_cert_slopes_host(float thr2) {
    const double T = (double)thr2, t = kCertT, u = 0x1p-24;
    // inlier cut: |a_in| <= T (1-t)/(1+t) (1 - slop), rounded towards zero
    const double ain = -T * (1.0 - t) / (1.0 + t) * (1.0 - kCertSlop);
    float fi = (float)ain;
    if ((double)fi < ain) fi = std::nextafter(fi, 0.0f);
    // outlier cut: |a_in| + d (1 - 2u) >= T (1+t)/(1-t) (1 + slop), d rounded up
    const double need = T * (1.0 + t) / (1.0 - t) * (1.0 + kCertSlop);
    const double d = (need + (double)fi) / (1.0 - 2 * u);
    float fd = (float)d;
    if ((double)fd < d) fd = std::nextafter(fd, __builtin_inff());
    HCertSlopes c;
    c.a = f2{fi, fd};
    c.t = t;
    return c;
}

// Per-model offsets b = {b_in, b_x} (both > 0); false when the model or the point set leaves the
// domain of the error bound (the wave then hands its slots to the exact scalar sweep).
// bb = {max|x|, max|y|, max|x'|, max|y'|} of the correspondences (inf when any is NaN / inf).
__device__ __forceinline__ bool h_cert_offsets(const float* h, const double* bb, float thr2, double t, f2& b) {
    const double X = bb[0], Y = bb[1], MX = bb[2], MY = bb[3];
    const double u = 0x1p-24;
    const double Bu = fabs((double)h[0]) * X + fabs((double)h[1]) * Y + fabs((double)h[2]);
    const double Bv = fabs((double)h[3]) * X + fabs((double)h[4]) * Y + fabs((double)h[5]);
    const double Bw = fabs((double)h[6]) * X + fabs((double)h[7]) * Y + 1.0;
    const double Gx = Bu + MX * Bw + 0x1p-40, Gy = Bv + MY * Bw + 0x1p-40;
    const double T = (double)thr2;
    const bool ok = X <= 0x1p40 && Y <= 0x1p40 && MX <= 0x1p40 && MY <= 0x1p40 && Bw <= 0x1p50 &&
                    Gx <= 0x1p50 && Gy <= 0x1p50 && T >= 0x1p-100 && T <= 0x1p20;   // false for NaN
    const double cx = 7.5 * u * Gx, cy = 7.5 * u * Gy, cw = 5.1 * u * Bw;
    const double C = cx * cx + cy * cy, Cw = cw * cw;
    const double tiny = 0x1p-120 + 0x1p-140 * Bw * Bw;
    const double K1 = (1.0 + 2 * kCertSlop) * ((1.0 + 1.0 / t) * C + T * Cw / t) + tiny;
    const double K2 = (1.0 + 2 * kCertSlop) / (1.0 - t) * (C / t + T * (1.0 + 1.0 / t) * Cw) + tiny;
    const float bin = __double2float_ru(K1);
    const double bx = (K2 + (double)bin) * (1.0 + kCertSlop);
    b = f2{bin, __double2float_ru(bx)};
    return ok;
}

// Unpacked model k (for the exact path): h[0..7] from the coefficient pairs.
template <int K>
__device__ __forceinline__ void h_cert_model(const f2 (&hp)[K][4], int k, float (&h)[8]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        h[2 * j] = hp[k][j].x;
        h[2 * j + 1] = hp[k][j].y;
    }
}

// The certified values of one pair of correspondences against one model: I and X (see above).
// a = {a_in, d} (shared), b = the model's {b_in, b_x}, c = {h2, h5}.
__device__ __forceinline__ void h_cert_values(f2 p0, f2 p1, f2 p2, f2 p3, f2 c, f2 a, f2 b, const HPair& q, f2 one,
                                              f2& I, f2& X) {
    const f2 W = pk_fma(lo(p3), q.x, pk_fma(hi(p3), q.y, one));      // fma(h6,x,fma(h7,y,1))
    const f2 U = pk_fma(lo(p0), q.x, pk_fma(hi(p0), q.y, lo(c)));    // fma(h0,x,fma(h1,y,h2))
    const f2 V = pk_fma(hi(p1), q.x, pk_fma(lo(p2), q.y, hi(c)));    // fma(h3,x,fma(h4,y,h5))
    const f2 DX = pk_fma(-q.mx, W, U);
    const f2 DY = pk_fma(-q.my, W, V);
    const f2 L = pk_fma(DX, DX, pk_fma(DY, DY, lo(b)));
    const f2 W2 = W * W;
    I = pk_fma(W2, lo(a), L);
    X = pk_fma(W2, hi(a), hi(b));
}

// Lane masks from the certified values: inliers and
// undecided lanes per half.
__device__ __forceinline__ void h_cert_masks(f2 I, f2 X, uint64_t& inx, uint64_t& iny, uint64_t& ux,
                                             uint64_t& uy) {
    inx = __builtin_amdgcn_ballot_w64(I.x < 0.0f);
    iny = __builtin_amdgcn_ballot_w64(I.y < 0.0f);
    ux = __builtin_amdgcn_ballot_w64(__float_as_uint(I.x) <= __float_as_uint(X.x));
    uy = __builtin_amdgcn_ballot_w64(__float_as_uint(I.y) <= __float_as_uint(X.y));
}

// h_error of both correspondences of a pair, packed, operation for operation (every product and sum
// rounded as written) with the reciprocal by rcp_exact_bounded, which equals the IEEE 1.f / w for
// every |w| < 2^126 (exhaustive GPU check, mcvTestRcpExhaustive mode 5): bit-identical to h_error in
// the certified sweep's domain (|w| <= Bw (1 + 2^-20), Bw <= 2^50).
__device__ __forceinline__ f2 h_error_pk(f2 p0, f2 p1, f2 p2, f2 p3, const HPair& q) {
    const f2 w = (lo(p3) * q.x + hi(p3) * q.y) + f2{1.f, 1.f};
    const f2 ww = f2{rcp_exact_bounded(w.x), rcp_exact_bounded(w.y)};   // |w| <= 2^51 in the certified domain
    const f2 ex = ((lo(p0) * q.x + hi(p0) * q.y) + lo(p1)) * ww - q.mx;
    const f2 ey = ((hi(p1) * q.x + lo(p2) * q.y) + hi(p2)) * ww - q.my;
    return ex * ex + ey * ey;
}

// One trip: NP pairs per lane against the wave's K models. vx / vy: lanes whose first / second
// correspondence of pair slot j exists (tail trip only). Returns the mask of models with an
// undecided lane in this trip (bit k); their certified counts are already in cnt.
template <int K, int NP, bool PRED>
__device__ __forceinline__ uint32_t h_cert_trip(f2 (&hp)[K][4], const f2 (&hc)[K], f2 a, const f2 (&cb)[K],
                                                const HPair (&q)[NP], const uint64_t (&vx)[NP],
                                                const uint64_t (&vy)[NP], f2 one, uint32_t (&cnt)[K]) {
    uint32_t undecided = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        // re-defined in place every trip (no copy): the loop cannot hoist the broadcasts, so each use
        // reads the SGPR pair through op_sel
        asm volatile("" : "+s"(hp[k][0]), "+s"(hp[k][1]), "+s"(hp[k][2]), "+s"(hp[k][3]));
        uint64_t und = 0;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            f2 I, X;
            h_cert_values(hp[k][0], hp[k][1], hp[k][2], hp[k][3], hc[k], a, cb[k], q[j], one, I, X);
            uint64_t inx, iny, ux, uy;
            if constexpr (PRED) {
                h_cert_masks(I, X, inx, iny, ux, uy);
                inx &= vx[j];
                iny &= vy[j];
                und |= (ux & vx[j]) | (uy & vy[j]);
            } else {
                h_cert_masks(I, X, inx, iny, ux, uy);
                und |= ux | uy;
            }
            cnt[k] += (uint32_t)__popcll(inx) + (uint32_t)__popcll(iny);
        }
        undecided |= (und != 0) ? (1u << k) : 0u;
    }
    return undecided;
}

// The exact op-by-op error for the undecided lanes of the models in `und`, with the models still in
// registers (compile-time model index; the branch per model is
// wave-uniform and rarely taken).
template <int K, int NP, bool PRED>
__device__ __forceinline__ void h_cert_fix_regs(uint32_t und, const f2 (&hp)[K][4], const f2 (&hc)[K], f2 a,
                                                const f2 (&cb)[K], const HPair (&q)[NP], const uint64_t (&vx)[NP],
                                                const uint64_t (&vy)[NP], float thr2, f2 one, uint32_t (&cnt)[K]) {
    const uint64_t me = 1ull << (__lane_id() & 63);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (!(und & (1u << k))) continue;
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            f2 I, X;
            h_cert_values(hp[k][0], hp[k][1], hp[k][2], hp[k][3], hc[k], a, cb[k], q[j], one, I, X);
            uint64_t inx, iny, ux, uy;
            h_cert_masks(I, X, inx, iny, ux, uy);
            if constexpr (PRED) {
                ux &= vx[j];
                uy &= vy[j];
            }
            if ((ux | uy) == 0) continue;
            const f2 e = h_error_pk(hp[k][0], hp[k][1], hp[k][2], hp[k][3], q[j]);
            cnt[k] += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64((ux & me) != 0 && e.x <= thr2)) +
                      (uint32_t)__popcll(__builtin_amdgcn_ballot_w64((uy & me) != 0 && e.y <= thr2));
        }
    }
}

// The exact op-by-op error (IEEE division) for the undecided lanes of model hk at the trip starting
// at pair `base` (re-read from memory; validity from the pair counts). Returns their inlier count.
template <int NP>
__device__ __noinline__ uint32_t h_cert_resolve(const HPair* __restrict__ pairs, int nPairs, int nComplete, int base,
                                                const HModelF* __restrict__ models, int hk, f2 a, f2 b, float thr2) {
    const int lane = threadIdx.x & 63;
    const uint64_t me = 1ull << lane;
    const f2* mp = (const f2*)&models[hk];
    const f2 m0 = mp[0], m1 = mp[1], m2 = mp[2], m3 = mp[3];
    const float h[8] = {m0.x, m0.y, m1.x, m1.y, m2.x, m2.y, m3.x, m3.y};
    const f2 one = f2{1.f, 1.f};
    uint32_t add = 0;
    for (int j = 0; j < NP; ++j) {
        const int p = base + 64 * j + lane;
        const uint64_t vx = __builtin_amdgcn_ballot_w64(p < nPairs), vy = __builtin_amdgcn_ballot_w64(p < nComplete);
        const HPair q = pairs[p < nPairs ? p : 0];
        f2 I, X;
        h_cert_values(m0, m1, m2, m3, f2{m1.x, m2.y}, a, b, q, one, I, X);
        uint64_t inx, iny, ux, uy;
        h_cert_masks(I, X, inx, iny, ux, uy);
        ux &= vx;
        uy &= vy;
        bool ex = false, ey = false;
        if (ux & me) ex = h_error(h, q.x.x, q.y.x, q.mx.x, q.my.x) <= thr2;
        if (uy & me) ey = h_error(h, q.x.y, q.y.y, q.mx.y, q.my.y) <= thr2;
        add += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(ex)) + (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(ey));
    }
    return add;
}

// A wave whose models or point set leave the bound's domain marks its valid slots kStatusRedo
// (recounted by the exact scalar sweep mcv_h_verify<.., false> with redo = 1), as does a wave
// whose undecided trips overflow its event list. Trips with undecided lanes are only recorded in
// the sweep (LDS event list: trip base << 8 | model mask) and resolved after it, so the exact
// division stays out of the sweep's registers.
// nComplete = N / 2 pairs hold two correspondences; pair nComplete (odd N) holds one.
static constexpr int kCertEvents = 256;   // per wave

template <int K, int NP>
__global__ __launch_bounds__(256) void mcv_h_verify_cert(const HPair* __restrict__ pairs, int nPairs, int nComplete,
                                                         const HModelF* __restrict__ models, int* __restrict__ counts,
                                                         int hypCount, float thr2, HCertSlopes slopes,
                                                         const double* __restrict__ bb) {
    static_assert(K <= 8, "model mask in 8 bits");
    __shared__ uint32_t events[4][kCertEvents];
    __shared__ f2 offsets[4][K];
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int wib = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;

    f2 hp[K][4], hc[K], cb[K];
    bool valid[K];
    bool fast = true;
    double b4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b4[j] = bb[j];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = (hk < hypCount) && (counts[hk] >= 0);
        const f2* mp = (const f2*)&models[hk < hypCount ? hk : hypCount - 1];
#pragma unroll
        for (int j = 0; j < 4; ++j) hp[k][j] = mp[j];
        hc[k] = f2{hp[k][1].x, hp[k][2].y};
        float h[8];
        h_cert_model<K>(hp, k, h);
        const bool ok = h_cert_offsets(h, b4, thr2, slopes.t, cb[k]);
        fast = fast && (ok || !valid[k]);
        if (lane == 0) offsets[wib][k] = cb[k];
        __builtin_amdgcn_wave_barrier();
        // VGPR-resident: hc and cb meet an SGPR coefficient or another model operand in the same
        // packed op (constant-bus limit)
        asm volatile("" : "+v"(hc[k]), "+v"(cb[k]));
    }
    const f2 one = f2{1.f, 1.f};
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    int nev = 0;
    // an event records the trip index (base / TRIP: < 2^24 for any N < 2^31, pairs = N / 2) and the
    // undecided-model mask in its low 8 bits
    constexpr int TRIP = 64 * NP;
    if (fast) {
        const int nFull = nComplete / TRIP * TRIP;
        uint64_t all[NP];
#pragma unroll
        for (int j = 0; j < NP; ++j) all[j] = ~0ull;
        for (int base = 0; base < nFull; base += TRIP) {
            HPair q[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j) q[j] = pairs[base + 64 * j + lane];
            const uint32_t und = h_cert_trip<K, NP, false>(hp, hc, slopes.a, cb, q, all, all, one, cnt);
            if (__builtin_expect(und != 0, 0))
                h_cert_fix_regs<K, NP, false>(und, hp, hc, slopes.a, cb, q, all, all, thr2, one, cnt);
        }
        for (int base = nFull; base < nPairs; base += TRIP) {
            HPair q[NP];
            uint64_t vx[NP], vy[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j) {
                const int p = base + 64 * j + lane;
                vx[j] = __builtin_amdgcn_ballot_w64(p < nPairs);
                vy[j] = __builtin_amdgcn_ballot_w64(p < nComplete);
                q[j] = pairs[p < nPairs ? p : 0];
            }
            const uint32_t und = h_cert_trip<K, NP, true>(hp, hc, slopes.a, cb, q, vx, vy, one, cnt);
            if (und != 0) {
                if (nev < kCertEvents && lane == 0) events[wib][nev] = ((uint32_t)(base / TRIP) << 8) | und;
                ++nev;
            }
        }
        if (nev > kCertEvents) fast = false;   // too many to resolve here: exact recount of the wave
        else if (nev > 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            for (int e = 0; e < nev; ++e) {
                const uint32_t ev = __builtin_amdgcn_readfirstlane(events[wib][e]);
                const int base = (int)(ev >> 8) * TRIP;
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (!(ev & (1u << k))) continue;
                    const int hk = h0 + k < hypCount ? h0 + k : hypCount - 1;
                    cnt[k] += h_cert_resolve<NP>(pairs, nPairs, nComplete, base, models, hk, slopes.a,
                                                 offsets[wib][k], thr2);
                }
            }
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) counts[h0 + k] = fast ? (int)cnt[k] : kStatusRedo;
    }
}

// Bounding box of the source points: bbox[0] = max |x|, bbox[1] = max |y| (one block; the
// ordering of float maxima is exact, so the result does not depend on the reduction order).
__global__ __launch_bounds__(1024) void mcv_bbox(const float4* __restrict__ pts, int N, float* __restrict__ bbox) {
    __shared__ float sx[16], sy[16];
    float mx = 0, my = 0;
    for (int i = threadIdx.x; i < N; i += 1024) {
        const float4 q = pts[i];
        mx = fmaxf(mx, fabsf(q.x));
        my = fmaxf(my, fabsf(q.y));
        if (q.x != q.x || q.y != q.y) mx = __builtin_inff();   // NaN coordinate: force exact path
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        mx = fmaxf(mx, __shfl_xor(mx, off, 64));
        my = fmaxf(my, __shfl_xor(my, off, 64));
    }
    if ((threadIdx.x & 63) == 0) { sx[threadIdx.x >> 6] = mx; sy[threadIdx.x >> 6] = my; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) { mx = fmaxf(mx, sx[w]); my = fmaxf(my, sy[w]); }
        bbox[0] = mx;
        bbox[1] = my;
    }
}

// ------------------------------------------------------------------------------------------
// Best packed key + first sampler failure.
// ------------------------------------------------------------------------------------------
static const int kBestThreads = 256;
static const int kBestMaxBlocks = 512;

__device__ __forceinline__ uint64_t pack_key(int count, int64_t hyp, int minCount) {
    return count >= minCount ? (((uint64_t)(uint32_t)count << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)hyp)) : 0ull;
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return v;
}
__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int64_t o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ void block_maxmin(uint64_t& key, int64_t& fail) {
    __shared__ uint64_t sk[kBestThreads / 64];
    __shared__ int64_t sf[kBestThreads / 64];
    key = wave_max_u64(key);
    fail = wave_min_i64(fail);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { sk[wave] = key; sf[wave] = fail; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBestThreads / 64; ++w) {
            key = sk[w] > key ? sk[w] : key;
            fail = sf[w] < fail ? sf[w] : fail;
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(kBestThreads) void mcv_best_partial(const int* __restrict__ counts, int n,
                                                                 int64_t hypBegin, int minCount,
                                                                 uint64_t* __restrict__ pkey,
                                                                 int64_t* __restrict__ pfail) {
    uint64_t key = 0;
    int64_t fail = INT64_MAX;
    for (int i = blockIdx.x * kBestThreads + threadIdx.x; i < n; i += gridDim.x * kBestThreads) {
        const int c = counts[i];
        const uint64_t k = pack_key(c, hypBegin + i, minCount);
        key = k > key ? k : key;
        if (c == kStatusNoSample && hypBegin + i < fail) fail = hypBegin + i;
    }
    block_maxmin(key, fail);
    if (threadIdx.x == 0) { pkey[blockIdx.x] = key; pfail[blockIdx.x] = fail; }
}

// out[0] = best key among hypotheses before the first sampler failure; out[1] = that failure.
__global__ __launch_bounds__(kBestThreads) void mcv_best_final(const uint64_t* __restrict__ pkey,
                                                               const int64_t* __restrict__ pfail, int nblocks,
                                                               const int* __restrict__ counts, int n,
                                                               int64_t hypBegin, int minCount,
                                                               uint64_t* __restrict__ out) {
    __shared__ int64_t s_fail;
    uint64_t key = 0;
    int64_t fail = INT64_MAX;
    for (int b = threadIdx.x; b < nblocks; b += kBestThreads) {
        key = pkey[b] > key ? pkey[b] : key;
        fail = pfail[b] < fail ? pfail[b] : fail;
    }
    block_maxmin(key, fail);
    if (threadIdx.x == 0) s_fail = fail;
    __syncthreads();
    fail = s_fail;
    if (fail != INT64_MAX) {
        // Rare (degenerate input): only hypotheses before the failure count.
        key = 0;
        const int lim = (int)(fail - hypBegin);
        for (int i = threadIdx.x; i < lim; i += kBestThreads) {
            const uint64_t k = pack_key(counts[i], hypBegin + i, minCount);
            key = k > key ? k : key;
        }
        int64_t dummy = INT64_MAX;
        block_maxmin(key, dummy);
    }
    if (threadIdx.x == 0) {
        out[0] = key;
        out[1] = (uint64_t)fail;
    }
}

// ------------------------------------------------------------------------------------------
// Inlier mask of one model (count via per-wave ballot + one atomic per wave).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mcv_h_mask(const float4* __restrict__ pts, int N, HModelF m, float thr2,
                                                  int fused, uint8_t* __restrict__ mask, int* __restrict__ count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < N) {
        const float4 q = pts[i];
        const float e = fused ? h_error_fused(m.h, q.x, q.y, q.z, q.w) : h_error(m.h, q.x, q.y, q.z, q.w);
        in = e <= thr2;
        mask[i] = in ? 1 : 0;
    }
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (int)__popcll(b));
}

// The same, with the model read from the winner record mcv_h_one wrote (no host round trip).
__global__ __launch_bounds__(256) void mcv_h_mask_one(const float4* __restrict__ pts, int N,
                                                      const HOneOut* __restrict__ one, float thr2, int fused,
                                                      uint8_t* __restrict__ mask, int* __restrict__ count) {
    HModelF m;
#pragma unroll
    for (int j = 0; j < 8; ++j) m.h[j] = one->hf[j];
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < N) {
        const float4 q = pts[i];
        const float e = fused ? h_error_fused(m.h, q.x, q.y, q.z, q.w) : h_error(m.h, q.x, q.y, q.z, q.w);
        in = e <= thr2;
        mask[i] = in ? 1 : 0;
    }
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (int)__popcll(b));
}

__global__ void mcv_fill_u8(uint8_t* __restrict__ p, int n, uint8_t v) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = v;
}

// ------------------------------------------------------------------------------------------
// Refit (HomographyEstimatorCallback::runKernel over the inliers) and LM
// (HomographyRefineCallback::compute) reductions.
// ------------------------------------------------------------------------------------------
struct OpSums {   // 5: sum dst.x, dst.y, src.x, src.y, count
    const float4* pts; const uint8_t* mask;
    __device__ void operator()(int i, double (&a)[5]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        a[0] += (double)q.z; a[1] += (double)q.w; a[2] += (double)q.x; a[3] += (double)q.y; a[4] += 1.0;
    }
};
struct OpAbsDev {  // 4: sum |dst - cm|, |src - cM|
    const float4* pts; const uint8_t* mask; double cmx, cmy, cMx, cMy;
    __device__ void operator()(int i, double (&a)[4]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        a[0] += fabs((double)q.z - cmx); a[1] += fabs((double)q.w - cmy);
        a[2] += fabs((double)q.x - cMx); a[3] += fabs((double)q.y - cMy);
    }
};
struct OpAbsDevD {  // OpAbsDev with the centroids read from device memory (chained refit)
    const float4* pts; const uint8_t* mask; const double* c4;
    __device__ void operator()(int i, double (&a)[4]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        a[0] += fabs((double)q.z - c4[0]); a[1] += fabs((double)q.w - c4[1]);
        a[2] += fabs((double)q.x - c4[2]); a[3] += fabs((double)q.y - c4[3]);
    }
};
struct OpLtL {     // 45: upper triangle of LtL, row-major
    const float4* pts; const uint8_t* mask; double cmx, cmy, cMx, cMy, smx, smy, sMx, sMy;
    __device__ void operator()(int i, double (&a)[45]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        const double x = ((double)q.z - cmx) * smx, y = ((double)q.w - cmy) * smy;
        const double X = ((double)q.x - cMx) * sMx, Y = ((double)q.y - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        int o = 0;
#pragma unroll
        for (int j = 0; j < 9; ++j)
#pragma unroll
            for (int k = j; k < 9; ++k) a[o++] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
};
struct OpLM {      // 45: JtJ upper triangle (36), Jtr (8), |r|^2 (1)
    const float4* pts; const uint8_t* mask; double h[8];
    __device__ void operator()(int i, double (&a)[45]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        const double Mx = q.x, My = q.y;
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > kDblEpsilon ? 1. / ww : 0;
        const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
        const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
        const double rx = xi - (double)q.z, ry = yi - (double)q.w;
        const double Jx[8] = {Mx * ww, My * ww, ww, 0, 0, 0, -Mx * ww * xi, -My * ww * xi};
        const double Jy[8] = {0, 0, 0, Mx * ww, My * ww, ww, -Mx * ww * yi, -My * ww * yi};
        int o = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int k = j; k < 8; ++k) a[o++] += Jx[j] * Jx[k] + Jy[j] * Jy[k];
#pragma unroll
        for (int j = 0; j < 8; ++j) a[36 + j] += Jx[j] * rx + Jy[j] * ry;
        a[44] += rx * rx + ry * ry;
    }
};
struct OpLMErr {   // 1: |r|^2 only
    const float4* pts; const uint8_t* mask; double h[8];
    __device__ void operator()(int i, double (&a)[1]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        const double Mx = q.x, My = q.y;
        double ww = h[6] * Mx + h[7] * My + 1.;
        ww = fabs(ww) > kDblEpsilon ? 1. / ww : 0;
        const double rx = (h[0] * Mx + h[1] * My + h[2]) * ww - (double)q.z;
        const double ry = (h[3] * Mx + h[4] * My + h[5]) * ww - (double)q.w;
        a[0] += rx * rx + ry * ry;
    }
};

// ------------------------------------------------------------------------------------------
// Launchers (host side, called from ransac_host.cpp)
// ------------------------------------------------------------------------------------------
// Rows of the split generate's scratch per piece: the whole call up to 2^20 hypotheses (3.2 GB of
// rotation log at 192 entries of 16 B). Round 6, same box: one piece 4.40 ms per 2^20 against 4.85 ms
// for pieces of two rounds of mcv_h_gen_aw's resident lanes (5 pieces: each launch drains its slowest
// waves, whose rotation counts vary per lane), 4.69 / 4.67 for pieces of four rounds / two halves.
static constexpr int kHGenMaxPiece = 1 << 20;
static int h_gen_piece(int hypCount) { return std::min(hypCount, kHGenMaxPiece); }

size_t h_gen_scratch_bytes(int hypCount) {
    const size_t piece = (size_t)h_gen_piece(hypCount);
    return piece * kEigLogCap * sizeof(EigRot) + piece * (sizeof(int4) + sizeof(int)) +
           ((size_t)hypCount + 1) * sizeof(int);
}

void launch_h_generate(const float* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_models,
                       double* d_h64, int* d_counts, hipStream_t s, bool fast, void* d_scratch) {
    if (fast) {
        hipLaunchKernelGGL(mcv_h_generate<true>, dim3((hypCount + 255) / 256), dim3(256), 0, s, d_pts4, N, smp, hypBegin,
                           hypCount, (HModelF*)d_models, d_h64, d_counts);
        return;
    }
    if (!d_scratch) {   // the one-pass solve: kEigLanes per block, one wave per SIMD (jacobi_eig.h)
        hipLaunchKernelGGL((mcv_h_generate<false, kEigLanes>), dim3((hypCount + kEigLanes - 1) / kEigLanes),
                           dim3(kEigLanes), 0, s, d_pts4, N, smp, hypBegin, hypCount, (HModelF*)d_models, d_h64,
                           d_counts);
        return;
    }
    const int piece = h_gen_piece(hypCount);
    char* b = (char*)d_scratch;
    EigRot* log = (EigRot*)b;
    b += (size_t)piece * kEigLogCap * sizeof(EigRot);
    int4* sidx = (int4*)b;
    b += (size_t)piece * sizeof(int4);
    int* meta = (int*)b;
    b += (size_t)piece * sizeof(int);
    int* ovf = (int*)b;
    (void)hipMemsetAsync(ovf, 0, sizeof(int), s);   // errors surface at the caller's hipGetLastError
    for (int base = 0; base < hypCount; base += piece) {
        const int cnt = std::min(piece, hypCount - base);
        hipLaunchKernelGGL(mcv_h_gen_aw<kHGenAwLanes>, dim3((cnt + kHGenAwLanes - 1) / kHGenAwLanes),
                           dim3(kHGenAwLanes), 0, s, d_pts4, N, smp, hypBegin, cnt, (HModelF*)d_models, d_counts, sidx,
                           meta, log, piece, ovf, base, g_eig_log_cap);
        hipLaunchKernelGGL((mcv_h_gen_v<kHGenVG, kHGenVQ, kHGenVD>), dim3((cnt + kHGenVQ - 1) / kHGenVQ),
                           dim3(kHGenVG * kHGenVQ), 0, s, d_pts4, cnt, base, sidx, meta, log, piece, (HModelF*)d_models,
                           d_h64, d_counts);
    }
    hipLaunchKernelGGL(mcv_h_gen_ovf<kEigLanes>, dim3(kHGenOvfBlocks), dim3(kEigLanes), 0, s, d_pts4, N, smp, hypBegin,
                       ovf, (HModelF*)d_models, d_h64, d_counts);
}

void launch_h_one(const float* d_pts4, int N, Sampler smp, int64_t hyp, HOneOut* d_out, hipStream_t s, bool fast) {
    hipLaunchKernelGGL(mcv_h_one, dim3(1), dim3(64), 0, s, d_pts4, N, smp, hyp, d_out, fast);
}

void launch_bbox(const float* d_pts4, int N, float* d_bbox, hipStream_t s) {
    hipLaunchKernelGGL(mcv_bbox, dim3(1), dim3(1024), 0, s, (const float4*)d_pts4, N, d_bbox);
}

template <int K, int P>
static void launch_h_verify_kp(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount,
                               float thr2, bool fused, const float* d_bbox, hipStream_t s, int redo = 0) {
    const int waves = (hypCount + K - 1) / K;
    const int blocks = (waves + 3) / 4;
    if (fused)
        hipLaunchKernelGGL((mcv_h_verify<K, P, true>), dim3(blocks), dim3(256), 0, s, (const float4*)d_pts4, N,
                           (const HModelF*)d_models, d_counts, hypCount, thr2, d_bbox, redo);
    else
        hipLaunchKernelGGL((mcv_h_verify<K, P, false>), dim3(blocks), dim3(256), 0, s, (const float4*)d_pts4, N,
                           (const HModelF*)d_models, d_counts, hypCount, thr2, d_bbox, redo);
}

void launch_h_verify(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount, float thr2,
                     bool fused, const float* d_bbox, hipStream_t s) {
    launch_h_verify_kp<kVerifyHypPerWave, kVerifyPtsPerLane>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused,
                                                             d_bbox, s);
}

template <int K, int NP>
static void launch_h_verify_pk_k(const void* d_pairs, int N, const void* d_models, int* d_counts, int hypCount,
                                 float thr2, const float* d_bbox, hipStream_t s) {
    const int waves = (hypCount + K - 1) / K;
    const int blocks = (waves + 3) / 4;
    hipLaunchKernelGGL((mcv_h_verify_pk<K, NP>), dim3(blocks), dim3(256), 0, s, (const HPair*)d_pairs, (N + 1) / 2,
                       (const HModelF*)d_models, d_counts, hypCount, thr2, d_bbox);
}

void launch_h_pair(const float* d_pts4, int N, void* d_pairs, hipStream_t s) {
    const int np = (N + 1) / 2;
    hipLaunchKernelGGL(mcv_h_pair, dim3((np + 255) / 256), dim3(256), 0, s, (const float4*)d_pts4, N,
                       (HPair*)d_pairs);
}

// Packed sweep (fused error, <8, 2>: DESIGN.md §7's screen) + the exact recount of the slots it
// marked kStatusRedo.
void launch_h_verify_packed(const float* d_pts4, const void* d_pairs, int N, const void* d_models, int* d_counts,
                            int hypCount, float thr2, const float* d_bbox, hipStream_t s) {
    launch_h_verify_pk_k<8, 2>(d_pairs, N, d_models, d_counts, hypCount, thr2, d_bbox, s);
    launch_h_verify_kp<kVerifyHypPerWave, kVerifyPtsPerLane>(d_pts4, N, d_models, d_counts, hypCount, thr2, true,
                                                             d_bbox, s, 1);
}

template <int K, int NP>
static void launch_h_verify_cert_k(const void* d_pairs, int N, const void* d_models, int* d_counts, int hypCount,
                                   float thr2, const double* d_bb, hipStream_t s) {
    const int waves = (hypCount + K - 1) / K;
    const int blocks = (waves + 3) / 4;
    hipLaunchKernelGGL((mcv_h_verify_cert<K, NP>), dim3(blocks), dim3(256), 0, s, (const HPair*)d_pairs, (N + 1) / 2,
                       N / 2, (const HModelF*)d_models, d_counts, hypCount, thr2, h_cert_slopes_host(thr2), d_bb);
}

// Certified sweep of the op-by-op error + the exact recount of the slots it marks kStatusRedo.
// <6, 1>: screened against <4, 2>, <4, 1>, <5, 1>, <3, 2>, <8, 2> and t = 2^-12 / 2^-11 / 2^-10
// (28.8 ms vs 29.6-33 ms at cfg3; scripts/gpu_r02_cert.sh); re-screened in round 5 (same box: 29.9-30.0 ms
// against 30.7-30.9 / 30.4-30.5 / 31.0-31.1 ms for <4, 1> / <5, 1> / <4, 2>; scripts/gpu_r05_am.sh).
void launch_h_verify_certified(const float* d_pts4, const void* d_pairs, int N, const void* d_models, int* d_counts,
                               int hypCount, float thr2, const double* d_bb, hipStream_t s) {
    launch_h_verify_cert_k<6, 1>(d_pairs, N, d_models, d_counts, hypCount, thr2, d_bb, s);
    launch_h_verify_kp<kVerifyHypPerWave, kVerifyPtsPerLane>(d_pts4, N, d_models, d_counts, hypCount, thr2, false,
                                                             nullptr, s, 1);
}

void launch_best(const int* d_counts, int n, int64_t hypBegin, int minCount, uint64_t* d_pkey, int64_t* d_pfail,
                 uint64_t* d_out, hipStream_t s) {
    int nb = (n + kBestThreads * 8 - 1) / (kBestThreads * 8);
    if (nb < 1) nb = 1;
    if (nb > kBestMaxBlocks) nb = kBestMaxBlocks;
    hipLaunchKernelGGL(mcv_best_partial, dim3(nb), dim3(kBestThreads), 0, s, d_counts, n, hypBegin, minCount, d_pkey,
                       d_pfail);
    hipLaunchKernelGGL(mcv_best_final, dim3(1), dim3(kBestThreads), 0, s, d_pkey, d_pfail, nb, d_counts, n, hypBegin,
                       minCount, d_out);
}

void launch_h_mask(const float* d_pts4, int N, const float* hf8, float thr2, bool fused, uint8_t* d_mask,
                   int* d_count, hipStream_t s) {
    HModelF m;
    for (int j = 0; j < 8; ++j) m.h[j] = hf8[j];
    hipLaunchKernelGGL(mcv_h_mask, dim3((N + 255) / 256), dim3(256), 0, s, (const float4*)d_pts4, N, m, thr2,
                       fused ? 1 : 0, d_mask, d_count);
}

void launch_h_mask_one(const float* d_pts4, int N, const HOneOut* d_one, float thr2, bool fused, uint8_t* d_mask,
                       int* d_count, hipStream_t s) {
    hipLaunchKernelGGL(mcv_h_mask_one, dim3((N + 255) / 256), dim3(256), 0, s, (const float4*)d_pts4, N, d_one, thr2,
                       fused ? 1 : 0, d_mask, d_count);
}

void launch_fill_u8(uint8_t* d, int n, uint8_t v, hipStream_t s) {
    hipLaunchKernelGGL(mcv_fill_u8, dim3((n + 255) / 256), dim3(256), 0, s, d, n, v);
}

void h_reduce_sums(const float* d_pts4, int N, const uint8_t* d_mask, double* d_part, double* d_out, hipStream_t s) {
    OpSums op{(const float4*)d_pts4, d_mask};
    run_reduce<5>(N, op, d_part, d_out, s);
}
void h_reduce_absdev(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, double* d_part,
                     double* d_out, hipStream_t s) {
    OpAbsDev op{(const float4*)d_pts4, d_mask, c4[0], c4[1], c4[2], c4[3]};
    run_reduce<4>(N, op, d_part, d_out, s);
}
void h_reduce_ltl(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, const double* s4,
                  double* d_part, double* d_out, hipStream_t s) {
    OpLtL op{(const float4*)d_pts4, d_mask, c4[0], c4[1], c4[2], c4[3], s4[0], s4[1], s4[2], s4[3]};
    run_reduce<45>(N, op, d_part, d_out, s);
}
struct OpLtLD {    // OpLtL with centroids / scales read from device memory (chained refit)
    const float4* pts; const uint8_t* mask; const double* c4; const double* s4;
    __device__ void operator()(int i, double (&a)[45]) const {
        OpLtL op{pts, mask, c4[0], c4[1], c4[2], c4[3], s4[0], s4[1], s4[2], s4[3]};
        op(i, a);
    }
};

// refit statistics between the chained passes: c4 = sums / count, s4 = count / absdev (the same
// IEEE divisions the host performs, so the passes see bit-identical constants)
__global__ void mcv_refit_stats(double* __restrict__ red, int stage) {
    if (threadIdx.x >= 4) return;
    const int k = threadIdx.x;
    if (stage == 0) red[5 + k] = red[k] / red[4];
    else red[13 + k] = red[4] / red[9 + k];
}

// HomographyEstimatorCallback::runKernel's three passes chained on the device (no host round trip):
// red[0..4] = sums, red[5..8] = centroids, red[9..12] = |dev| sums, red[13..16] = scales,
// red[17..61] = LtL.
void h_refit_chain(const float* d_pts4, int N, const uint8_t* d_mask, double* d_part, double* d_red, hipStream_t s) {
    const float4* p = (const float4*)d_pts4;
    run_reduce<5>(N, OpSums{p, d_mask}, d_part, d_red, s);
    hipLaunchKernelGGL(mcv_refit_stats, dim3(1), dim3(64), 0, s, d_red, 0);
    run_reduce<4>(N, OpAbsDevD{p, d_mask, d_red + 5}, d_part, d_red + 9, s);
    hipLaunchKernelGGL(mcv_refit_stats, dim3(1), dim3(64), 0, s, d_red, 1);
    run_reduce<45>(N, OpLtLD{p, d_mask, d_red + 5, d_red + 13}, d_part, d_red + 17, s);
}

void h_reduce_lm(const float* d_pts4, int N, const uint8_t* d_mask, const double* h8, bool wantJ, double* d_part,
                 double* d_out, hipStream_t s) {
    if (wantJ) {
        OpLM op{(const float4*)d_pts4, d_mask, {h8[0], h8[1], h8[2], h8[3], h8[4], h8[5], h8[6], h8[7]}};
        run_reduce<45>(N, op, d_part, d_out, s);
    } else {
        OpLMErr op{(const float4*)d_pts4, d_mask, {h8[0], h8[1], h8[2], h8[3], h8[4], h8[5], h8[6], h8[7]}};
        run_reduce<1>(N, op, d_part, d_out, s);
    }
}

}  // namespace mcv


// Test hook: the split generate's usable log rows in [0, 192] (lanes needing more go to the one-pass
// overflow kernel); returns the previous value. Not thread-safe: tests only.
extern "C" MCV_API int mcvTestEigLogCap(int cap) {
    const int prev = mcv::g_eig_log_cap;
    mcv::g_eig_log_cap = cap < 0 ? 0 : cap > mcv::kEigLogCap ? mcv::kEigLogCap : cap;
    return prev;
}
