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
#include <cstdlib>
#include "mcv_common.h"
#include "hyp_homography.h"
#include "reduce.h"
#include "kernels.h"

namespace mcv {

// ------------------------------------------------------------------------------------------
// Hypothesis generation
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mcv_h_generate(const float* __restrict__ pts4, int N, uint64_t seed,
                                                      int64_t hypBegin, int hypCount, HModelF* __restrict__ models,
                                                      int* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hypCount) return;
    double H[9];
    HModelF mf;
    const int st = h_hypothesis(pts4, N, seed, (uint64_t)(hypBegin + i), H, &mf, nullptr);
    if (st == 1) {
        models[i] = mf;
        counts[i] = 0;
    } else {
        counts[i] = st;
    }
}

// One hypothesis in full (finalize path): fp64 model, fp32 model, status, sample.
__global__ void mcv_h_one(const float* __restrict__ pts4, int N, uint64_t seed, int64_t hyp, HOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    HOneOut o;
    HModelF mf;
    for (int j = 0; j < 9; ++j) o.H[j] = 0;
    for (int j = 0; j < 8; ++j) mf.h[j] = 0;
    o.status = h_hypothesis(pts4, N, seed, (uint64_t)hyp, o.H, &mf, o.idx);
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

template <int K, int P, bool FUSED>
__global__ __launch_bounds__(256) void mcv_h_verify(const float4* __restrict__ pts, int N,
                                                    const HModelF* __restrict__ models, int* __restrict__ counts,
                                                    int hypCount, float thr2, const float* __restrict__ bbox) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;

    float hm[K][8];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = (hk < hypCount) && (counts[hk] >= 0);
        const HModelF m = models[valid[k] ? hk : h0];
#pragma unroll
        for (int j = 0; j < 8; ++j) hm[k][j] = valid[k] ? m.h[j] : __builtin_nanf("");
        // h2 and h5 meet another uniform operand in fma(h1, y, h2) / fma(h4, y, h5); a VALU op
        // reads at most one SGPR (gfx9 constant-bus limit), so keep those two in VGPRs and the
        // other six in SGPRs (no per-use v_mov, and SGPR pressure stays below the spill point).
        asm volatile("" : "+v"(hm[k][2]));
        asm volatile("" : "+v"(hm[k][5]));
    }

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
void launch_h_generate(const float* d_pts4, int N, uint64_t seed, int64_t hypBegin, int hypCount, void* d_models,
                       int* d_counts, hipStream_t s) {
    const int blocks = (hypCount + 255) / 256;
    hipLaunchKernelGGL(mcv_h_generate, dim3(blocks), dim3(256), 0, s, d_pts4, N, seed, hypBegin, hypCount,
                       (HModelF*)d_models, d_counts);
}

void launch_h_one(const float* d_pts4, int N, uint64_t seed, int64_t hyp, HOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_h_one, dim3(1), dim3(64), 0, s, d_pts4, N, seed, hyp, d_out);
}

void launch_bbox(const float* d_pts4, int N, float* d_bbox, hipStream_t s) {
    hipLaunchKernelGGL(mcv_bbox, dim3(1), dim3(1024), 0, s, (const float4*)d_pts4, N, d_bbox);
}

template <int K, int P>
static void launch_h_verify_kp(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount,
                               float thr2, bool fused, const float* d_bbox, hipStream_t s) {
    const int waves = (hypCount + K - 1) / K;
    const int blocks = (waves + 3) / 4;
    if (fused)
        hipLaunchKernelGGL((mcv_h_verify<K, P, true>), dim3(blocks), dim3(256), 0, s, (const float4*)d_pts4, N,
                           (const HModelF*)d_models, d_counts, hypCount, thr2, d_bbox);
    else
        hipLaunchKernelGGL((mcv_h_verify<K, P, false>), dim3(blocks), dim3(256), 0, s, (const float4*)d_pts4, N,
                           (const HModelF*)d_models, d_counts, hypCount, thr2, d_bbox);
}

// Sweep shape (hypotheses per wave K, correspondences per lane per trip P). MCV_SWEEP_VARIANT
// selects an alternative for tuning experiments (tests/bench only); the default is kVerify*.
static int sweep_variant() {
    static int v = [] {
        const char* e = getenv("MCV_SWEEP_VARIANT");
        return e ? atoi(e) : 0;
    }();
    return v;
}

void launch_h_verify(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount, float thr2,
                     bool fused, const float* d_bbox, hipStream_t s) {
    switch (sweep_variant()) {
        case 1: launch_h_verify_kp<8, 4>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 2: launch_h_verify_kp<4, 4>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 3: launch_h_verify_kp<8, 1>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 4: launch_h_verify_kp<6, 2>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 5: launch_h_verify_kp<4, 2>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 6: launch_h_verify_kp<6, 3>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 7: launch_h_verify_kp<5, 2>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 8: launch_h_verify_kp<6, 1>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 9: launch_h_verify_kp<4, 3>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 10: launch_h_verify_kp<3, 2>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        case 11: launch_h_verify_kp<7, 2>(d_pts4, N, d_models, d_counts, hypCount, thr2, fused, d_bbox, s); break;
        default:
            launch_h_verify_kp<kVerifyHypPerWave, kVerifyPtsPerLane>(d_pts4, N, d_models, d_counts, hypCount, thr2,
                                                                     fused, d_bbox, s);
    }
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
