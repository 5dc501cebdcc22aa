// ransac_f.hip — gfx950 kernels of the fundamental-matrix RANSAC path.
//
//   mcv_f_generate      one lane per hypothesis: Philox sample of 8 -> collinearity check ->
//                       8-point solve + rank 2 (fp64) -> FModelD (72 B) + status.
//   mcv_f7_generate     MCV_FLAG_SEVEN_POINT: lane per hypothesis, 7-point sample -> run7Point (JacobiSVD
//                       null space, cubic) -> up to 3 FModelD slots + per-slot status.
//   mcv_f_verify<K, E>  inlier sweep: wave = K hypotheses (fp64 models in VGPRs), 64 lanes stream
//                       the packed float4 correspondences; per (hypothesis, point) the fp64
//                       Sampson / epipolar error E, cast to float, ballot + s_bcnt1 count.
//   mcv_f_verify_pk<KP,P> the Sampson sweep with the certified packed-fp32 prefilter
//                       (sampson_pk.h): wave = KP model pairs, undecided lanes re-tested in fp64.
//   mcv_abs_bound4      max |x1|, |y1|, |x2|, |y2| over the point set (the prefilter's bound).
//   mcv_f_mask          inlier mask of the winner.
//   OpFAtA              fixed-order fp64 reduction of A^T A (run8Point over all points).
#include "mcv_common.h"
#include "hyp_fundamental.h"
#include "hyp_f7.h"
#include "sampson_pk.h"
#include "reduce.h"
#include "kernels.h"
#include "mcv_runtime.h"
#include <cstdlib>
#include <algorithm>
#include <cmath>

namespace mcv {

// One lane per hypothesis; run8Point's eigen-solve working set in LDS, one column per lane.
// FAST = MCV_FLAG_FAST_MINIMAL (no workspace).
template <bool FAST, int L = kEigLanes>
__global__ __launch_bounds__(FAST ? 256 : L) void mcv_f_generate(const float* __restrict__ pts4, int N, Sampler smp,
                                                     int64_t hypBegin, int hypCount, FModelD* __restrict__ models,
                                                     int* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hypCount) return;
    FModelD m;
    int st;
    if constexpr (FAST) {
        EigWsLocal unused;   // the elimination never touches it (folded away)
        st = f_hypothesis(pts4, N, smp, (uint64_t)(hypBegin + i), m.f, nullptr, unused, true);
    } else {
        __shared__ double lds[kEigWs * L];
        EigWsLane ws{lds + threadIdx.x * kEigWs};
        st = f_hypothesis(pts4, N, smp, (uint64_t)(hypBegin + i), m.f, nullptr, ws);
    }
    if (st == 1) {
        models[i] = m;
        counts[i] = 0;
    } else {
        counts[i] = st;
    }
}

__global__ void mcv_f_one(const float* __restrict__ pts4, int N, Sampler smp, int64_t hyp, FOneOut* __restrict__ out,
                          bool fast) {
    __shared__ double lds[kEigWs];
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    EigWsLane ws{lds};
    FOneOut o;
    for (int j = 0; j < 9; ++j) o.F[j] = 0;
    for (int j = 0; j < 8; ++j) o.idx[j] = -1;
    o.status = f_hypothesis(pts4, N, smp, (uint64_t)hyp, o.F, o.idx, ws, fast);
    *out = o;
}

template <int K, int P, int KIND>
__global__ __launch_bounds__(256) void mcv_f_verify(const float4* __restrict__ pts, int N,
                                                    const FModelD* __restrict__ models, int* __restrict__ counts,
                                                    int hypCount, float thr2, double lo, double hi) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;
    double fm[K][9];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = (hk < hypCount) && (counts[hk] >= 0);
        const FModelD m = models[valid[k] ? hk : h0];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            fm[k][j] = valid[k] ? m.f[j] : f_dummy_model(j);
            asm volatile("" : "+v"(fm[k][j]));   // VGPR operands: no constant-bus moves in the fp64 FMAs
        }
    }
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    const int step = 64 * P;
    const int nFull = N - N % step;
    for (int base = 0; base < nFull; base += step) {
        float4 q[P];
#pragma unroll
        for (int p = 0; p < P; ++p) q[p] = pts[base + 64 * p + lane];
#pragma unroll
        for (int p = 0; p < P; ++p) f_sweep_point<K, KIND>(fm, q[p].x, q[p].y, q[p].z, q[p].w, true, thr2, lo, hi, cnt);
    }
    for (int base = nFull; base < N; base += 64) {
        const int p = base + lane;
        const bool v = p < N;
        const float4 q = pts[v ? p : 0];
        f_sweep_point<K, KIND>(fm, q.x, q.y, q.z, q.w, v, thr2, lo, hi, cnt);
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) counts[h0 + k] = (int)cnt[k];
    }
}

// Point-set bounds for the packed prefilter: bb = max |x1|, |y1|, |x2|, |y2| as fp64 bit patterns
// (non-negative doubles order like their bits; NaN coordinates force +inf, i.e. no certification).
// With out32 (double4 input) the points are also written rounded to float4 for the fp32 sweep.
template <class T4>
__global__ __launch_bounds__(256) void mcv_abs_bound4(const T4* __restrict__ pts, int N,
                                                      unsigned long long* __restrict__ bb, float4* __restrict__ out32) {
    double m0 = 0, m1 = 0, m2 = 0, m3 = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const T4 q = pts[i];
        const double x = q.x, y = q.y, z = q.z, w = q.w;
        m0 = x == x ? fmax(m0, fabs(x)) : __builtin_inf();
        m1 = y == y ? fmax(m1, fabs(y)) : __builtin_inf();
        m2 = z == z ? fmax(m2, fabs(z)) : __builtin_inf();
        m3 = w == w ? fmax(m3, fabs(w)) : __builtin_inf();
        if (out32) out32[i] = float4{(float)q.x, (float)q.y, (float)q.z, (float)q.w};
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        m0 = fmax(m0, __shfl_xor(m0, off, 64));
        m1 = fmax(m1, __shfl_xor(m1, off, 64));
        m2 = fmax(m2, __shfl_xor(m2, off, 64));
        m3 = fmax(m3, __shfl_xor(m3, off, 64));
    }
    // block maximum first: one atomic per block and coordinate (per-wave atomics on 4 addresses
    // serialised to ~190 us at 500k points)
    __shared__ double sm[4][4];
    const int wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sm[wv][0] = m0; sm[wv][1] = m1; sm[wv][2] = m2; sm[wv][3] = m3;
    }
    __syncthreads();
    if (threadIdx.x < 4) {
        const int c = threadIdx.x;
        const double m = fmax(fmax(sm[0][c], sm[1][c]), fmax(sm[2][c], sm[3][c]));
        atomicMax(bb + c, (unsigned long long)__double_as_longlong(m));
    }
}

// Grid = (model waves) x (point chunks of `chunk` points, a multiple of 64 P): with one chunk a wave sweeps
// all N points and the last round of waves leaves SIMDs idle (8192 waves of 8 models at 65536
// hypotheses = 2.7 rounds of 3 waves per SIMD); chunks even the rounds out, their partial counts are
// added atomically (the generate kernel zeroed every valid slot).
template <int KP, int P>
__global__ __launch_bounds__(256) void mcv_f_verify_pk(const float4* __restrict__ pts, int N, int chunk, bool xcdMap,
                                                       const FModelD* __restrict__ models, int* __restrict__ counts,
                                                       int hypCount, float thr2, int kind, SampsonPkCut cut,
                                                       const double* __restrict__ bb) {
    constexpr int K = 2 * KP;
    // XCD-aware (block, chunk) order: blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
    // speed only), so with the chunk = linear block id mod C (C | 8) every XCD streams one chunk of the
    // points through its own L2 (500k correspondences = 8 MB, 1 MB per chunk at C = 8)
    const unsigned lin = blockIdx.x + blockIdx.y * gridDim.x;
    const unsigned bx = xcdMap ? lin / gridDim.y : blockIdx.x, by = xcdMap ? lin % gridDim.y : blockIdx.y;
    const int wave = __builtin_amdgcn_readfirstlane((int)((bx * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    // the block's 4 K counts leave through LDS in one contiguous store (a wave's own K counts were a
    // partial-sector write each: 8.2 MiB written per launch at K = 6, 4 MiB of counts): no early return
    // before that barrier, a wave past the end just sweeps nothing
    __shared__ int blockCounts[4 * K];
    const double B[4] = {bb[0], bb[1], bb[2], bb[3]};
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) valid[k] = (h0 + k < hypCount) && (counts[h0 + k] >= 0);
    SampsonPkPair pr[KP];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
        double Fa[9], Fb[9];
        const FModelD ma = models[valid[2 * kp] ? h0 + 2 * kp : 0];   // slot 0 exists (hypCount >= 1)
        const FModelD mb = models[valid[2 * kp + 1] ? h0 + 2 * kp + 1 : 0];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            Fa[j] = valid[2 * kp] ? ma.f[j] : f_dummy_model(j);
            Fb[j] = valid[2 * kp + 1] ? mb.f[j] : f_dummy_model(j);
        }
        spk_make_pair(pr[kp], Fa, Fb, B, cut);
        // VGPR operands (the pairs are wave-uniform): no constant-bus moves inside the packed ops
#pragma unroll
        for (int j = 0; j < 9; ++j) asm volatile("" : "+v"(pr[kp].f[j]));
        asm volatile("" : "+v"(pr[kp].ain));
        asm volatile("" : "+v"(pr[kp].bin));
        asm volatile("" : "+v"(pr[kp].aout));
        asm volatile("" : "+v"(pr[kp].bout));
    }
    auto f64 = [&](int k, double (&F)[9]) {
        const int hk = valid[k] ? h0 + k : -1;
#pragma unroll
        for (int j = 0; j < 9; ++j) F[j] = hk >= 0 ? models[hk].f[j] : f_dummy_model(j);
    };
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    const int step = 64 * P;
    const int p0 = (int)by * chunk;
    const int p1 = h0 < hypCount ? min(N, p0 + chunk) : p0;
    const int nFull = p0 + (p1 - p0) / step * step;
    for (int base = p0; base < nFull; base += step) {
        float4 q[P];
#pragma unroll
        for (int p = 0; p < P; ++p) q[p] = pts[base + 64 * p + lane];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const float4 qp = q[p];
            auto x64 = [&](double& x1, double& y1, double& x2, double& y2) { x1 = qp.x; y1 = qp.y; x2 = qp.z; y2 = qp.w; };
            spk_sweep_point<KP>(pr, qp, true, cut.L32, cut.H32, kind, thr2, f64, x64, cnt);
        }
    }
    for (int base = nFull; base < p1; base += 64) {
        const int p = base + lane;
        const bool v = p < p1;
        const float4 q = pts[v ? p : p0];
        auto x64 = [&](double& x1, double& y1, double& x2, double& y2) { x1 = q.x; y1 = q.y; x2 = q.z; y2 = q.w; };
        spk_sweep_point<KP>(pr, q, v, cut.L32, cut.H32, kind, thr2, f64, x64, cnt);
    }
    // lane k stages model k's count (-1: not a valid model, nothing written), then the block's 4 K
    // contiguous slots go out as one store (or one atomic each when the points are chunked)
    int mine = 0;
    bool mv = false;
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (lane == k) mine = (int)cnt[k], mv = valid[k];
    if (lane < K) blockCounts[(threadIdx.x >> 6) * K + lane] = mv ? mine : -1;
    __syncthreads();
    if (threadIdx.x < 4 * K) {
        const int v = blockCounts[threadIdx.x];
        const int slot = (wave - (int)(threadIdx.x >> 6)) * K + (int)threadIdx.x;   // the block's first model + t
        if (v >= 0) {
            if (gridDim.y == 1) counts[slot] = v;
            else if (v) atomicAdd(counts + slot, v);
        }
    }
}

// Grid-stride, one count atomic per block (per-wave atomics on the one counter serialised to
// ~90 us at 500k correspondences).
__global__ __launch_bounds__(256) void mcv_f_mask(const float4* __restrict__ pts, int N, FModelD m, float thr2,
                                                  int kind, uint8_t* __restrict__ mask, int* __restrict__ count) {
    int c = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const float4 q = pts[i];
        const bool in = f_error(kind, m.f, q.x, q.y, q.z, q.w) <= thr2;
        mask[i] = in ? 1 : 0;
        c += in ? 1 : 0;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
    __shared__ int sc[4];
    if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int t = sc[0] + sc[1] + sc[2] + sc[3];
        if (t) atomicAdd(count, t);
    }
}

struct OpFAtA {   // 45: upper triangle of A^T A, rows (X2X1, X2Y1, X2, Y2X1, Y2Y1, Y2, X1, Y1, 1)
    const float4* pts; const uint8_t* mask; double c1x, c1y, s1x, s1y, c2x, c2y, s2x, s2y;
    __device__ void operator()(int i, double (&a)[45]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        const double X1 = ((double)q.x - c1x) * s1x, Y1 = ((double)q.y - c1y) * s1y;
        const double X2 = ((double)q.z - c2x) * s2x, Y2 = ((double)q.w - c2y) * s2y;
        const double r[9] = {X2 * X1, X2 * Y1, X2, Y2 * X1, Y2 * Y1, Y2, X1, Y1, 1.0};
        int o = 0;
#pragma unroll
        for (int j = 0; j < 9; ++j)
#pragma unroll
            for (int k = j; k < 9; ++k) a[o++] += r[j] * r[k];
    }
};

__global__ __launch_bounds__(64) void mcv_f7_generate(const float* __restrict__ pts4, int N, Sampler smp,
                                                      int64_t hypBegin, int hypCount, FModelD* __restrict__ models,
                                                      int* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hypCount) return;
    double F[kF7Slots][9];
    const int st = f7_hypothesis(pts4, N, smp, (uint64_t)(hypBegin + i), F, nullptr);
    for (int s = 0; s < kF7Slots; ++s) {
        if (st > s) {
            FModelD m;
            for (int j = 0; j < 9; ++j) m.f[j] = F[s][j];
            models[kF7Slots * (size_t)i + s] = m;
            counts[kF7Slots * (size_t)i + s] = 0;
        } else {
            counts[kF7Slots * (size_t)i + s] = (s == 0 && st == kStatusNoSample) ? kStatusNoSample : kStatusNoModel;
        }
    }
}

__global__ void mcv_f7_one(const float* __restrict__ pts4, int N, Sampler smp, int64_t slot,
                           FOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double F[kF7Slots][9];
    int idx[7] = {-1, -1, -1, -1, -1, -1, -1};
    const int s = (int)(slot % kF7Slots);
    const int st = f7_hypothesis(pts4, N, smp, (uint64_t)(slot / kF7Slots), F, idx);
    FOneOut o;
    o.status = st > s ? 1 : (st < 0 ? st : kStatusNoModel);
    for (int j = 0; j < 9; ++j) o.F[j] = st > s ? F[s][j] : 0.0;
    for (int j = 0; j < 8; ++j) o.idx[j] = j < 7 ? idx[j] : -1;
    *out = o;
}

__global__ void mcv_f7_direct(const float* __restrict__ pts4, FOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    float x1[7], y1[7], x2[7], y2[7];
    for (int i = 0; i < 7; ++i) {
        x1[i] = pts4[4 * i]; y1[i] = pts4[4 * i + 1]; x2[i] = pts4[4 * i + 2]; y2[i] = pts4[4 * i + 3];
    }
    double F[kF7Slots][9];
    const int n = f_solve7(x1, y1, x2, y2, F);
    FOneOut o;
    o.status = n > 0 ? n : kStatusNoModel;
    for (int j = 0; j < 9; ++j) o.F[j] = n > 0 ? F[0][j] : 0.0;
    for (int j = 0; j < 8; ++j) o.idx[j] = j < 7 ? j : -1;
    *out = o;
}

void launch_f7_generate(const float* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_models,
                        int* d_counts, hipStream_t s) {
    hipLaunchKernelGGL(mcv_f7_generate, dim3((hypCount + 63) / 64), dim3(64), 0, s, d_pts4, N, smp, hypBegin,
                       hypCount, (FModelD*)d_models, d_counts);
}

void launch_f7_one(const float* d_pts4, int N, Sampler smp, int64_t slot, FOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_f7_one, dim3(1), dim3(64), 0, s, d_pts4, N, smp, slot, d_out);
}

void launch_f7_direct(const float* d_pts4, FOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_f7_direct, dim3(1), dim3(64), 0, s, d_pts4, d_out);
}

void launch_f_generate(const float* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_models,
                       int* d_counts, hipStream_t s, bool fast) {
    if (fast)
        hipLaunchKernelGGL(mcv_f_generate<true>, dim3((hypCount + 255) / 256), dim3(256), 0, s, d_pts4, N, smp, hypBegin,
                           hypCount, (FModelD*)d_models, d_counts);
    else   // kEigLanes per block: LDS-bound occupancy, one wave per SIMD (jacobi_eig.h)
        hipLaunchKernelGGL((mcv_f_generate<false, kEigLanes>), dim3((hypCount + kEigLanes - 1) / kEigLanes),
                           dim3(kEigLanes), 0, s, d_pts4, N, smp, hypBegin, hypCount, (FModelD*)d_models, d_counts);
}

void launch_f_one(const float* d_pts4, int N, Sampler smp, int64_t hyp, FOneOut* d_out, hipStream_t s, bool fast) {
    hipLaunchKernelGGL(mcv_f_one, dim3(1), dim3(64), 0, s, d_pts4, N, smp, hyp, d_out, fast);
}

template <int K, int P>
static void launch_f_verify_kp(const float4* p, int N, const FModelD* m, int* d_counts, int hypCount, float thr2,
                               int kind, double lo, double hi, hipStream_t s) {
    const int blocks = ((hypCount + K - 1) / K + 3) / 4;
    switch (kind) {
        case 0: hipLaunchKernelGGL((mcv_f_verify<K, P, 0>), dim3(blocks), dim3(256), 0, s, p, N, m, d_counts, hypCount, thr2, lo, hi); break;
        case 1: hipLaunchKernelGGL((mcv_f_verify<K, P, 1>), dim3(blocks), dim3(256), 0, s, p, N, m, d_counts, hypCount, thr2, lo, hi); break;
        case 2: hipLaunchKernelGGL((mcv_f_verify<K, P, 2>), dim3(blocks), dim3(256), 0, s, p, N, m, d_counts, hypCount, thr2, lo, hi); break;
        default: hipLaunchKernelGGL((mcv_f_verify<K, P, 3>), dim3(blocks), dim3(256), 0, s, p, N, m, d_counts, hypCount, thr2, lo, hi); break;
    }
}

void launch_abs_bound4(const void* d_pts4, bool fp64, int N, double* d_bb, float* d_out32, hipStream_t s) {
    (void)hipMemsetAsync(d_bb, 0, 4 * sizeof(double), s);
    if (N <= 0) return;
    const int blocks = std::min(256, (N + 255) / 256);
    if (fp64)
        hipLaunchKernelGGL(mcv_abs_bound4<double4>, dim3(blocks), dim3(256), 0, s, (const double4*)d_pts4, N,
                           (unsigned long long*)d_bb, (float4*)d_out32);
    else
        hipLaunchKernelGGL(mcv_abs_bound4<float4>, dim3(blocks), dim3(256), 0, s, (const float4*)d_pts4, N,
                           (unsigned long long*)d_bb, (float4*)nullptr);
}

template <int KP, int P>
static void launch_f_verify_pk_kp(const float4* p, int N, const FModelD* m, int* d_counts, int hypCount, float thr2,
                                  int kind, const SampsonPkCut& cut, const double* d_bb, hipStream_t s) {
    const int waves = (hypCount + 2 * KP - 1) / (2 * KP);
    const int blocks = (waves + 3) / 4;
    // point chunks of at least 8192 points (the per-wave model setup stays small against the sweep), as
    // many as even out the last round of resident waves (tail_chunks). Round 6, same box, alternating:
    // 2^17 / 2^18 / 2^19 hypotheses (the 8- / 4- / 2-rank shares) 28.5 / 56.0 / 110.8 ms a step against
    // 28.7-28.8 / 56.4-56.5 / 112.9 with the fixed ~64-waves-per-SIMD target (2^17: 3 chunks, 16.0005
    // rounds of 4 waves per SIMD); 2^20 keeps one chunk. PnP's verify measured slower with more chunks
    // (its per-wave pose setup): not used there.
    static const int64_t resident = resident_waves(mcv_f_verify_pk<KP, P>, 256);
    const int step = 64 * P;
    // No L2-sized chunking: 2^20 hypotheses x 500k points in 8 per-XCD chunks of 1 MB cut the fetches
    // 4.0 -> 0.61 GB per launch but took eight count atomics per model (32 MiB of writes against the
    // 4 MiB of one store each) for 222.2 vs 224.1 ms; a block-shared form (four chunks per block,
    // counts added in LDS behind a barrier: 8 MiB) measured 279 ms. The sweep is VALU-bound, so the
    // whole point set streams from the 256 MB MALL and each model's count is one store.
    const int maxChunks = std::max(1, N / 8192);
    int chunks = tail_chunks(waves, resident, maxChunks);
    int chunk = (N + chunks - 1) / chunks;
    chunk = (chunk + step - 1) / step * step;
    chunks = std::max(1, (N + chunk - 1) / chunk);
    hipLaunchKernelGGL((mcv_f_verify_pk<KP, P>), dim3(blocks, chunks), dim3(256), 0, s, p, N, chunk,
                       (8 % chunks) == 0, m, d_counts, hypCount, thr2, kind, cut, d_bb);
}

void launch_f_verify(const float* d_pts4, int N, const void* d_models, int* d_counts, int hypCount, float thr2,
                     int kind, hipStream_t s, const double* d_bb) {
    const float4* p = (const float4*)d_pts4;
    const FModelD* m = (const FModelD*)d_models;
    const SampsonCut c = sampson_cut(thr2);
    if (d_bb && kind <= 1) {   // Sampson: certified packed-fp32 prefilter, 3 model pairs per wave (four waves
        // per SIMD at 121 VGPRs; round 5, same box: 218.2 ms per launch against 225.5 for 4 pairs at three
        // waves per SIMD, 219.0-219.7 for 3 pairs x 2 points a trip, 233.5 for 2 pairs x 2 points)
        launch_f_verify_pk_kp<3, 1>(p, N, m, d_counts, hypCount, thr2, kind, sampson_pk_cut_host(c), d_bb, s);
        return;
    }
    launch_f_verify_kp<kVerifyFHypPerWave, kVerifyFPtsPerLane>(p, N, m, d_counts, hypCount, thr2, kind, c.lo, c.hi, s);
}

void launch_f_mask(const float* d_pts4, int N, const double* F9, float thr2, int kind, uint8_t* d_mask, int* d_count,
                   hipStream_t s) {
    FModelD m;
    for (int j = 0; j < 9; ++j) m.f[j] = F9[j];
    if (N <= 0) return;
    hipLaunchKernelGGL(mcv_f_mask, dim3(std::min(512, (N + 255) / 256)), dim3(256), 0, s, (const float4*)d_pts4, N, m,
                       thr2, kind, d_mask, d_count);
}

// run8Point's scale sums: sum of the Euclidean distances to the centroids, {image 2, image 1}.
struct OpFEucDev {
    const float4* pts; const uint8_t* mask; double c2x, c2y, c1x, c1y;
    __device__ void operator()(int i, double (&a)[2]) const {
        if (mask && !mask[i]) return;
        const float4 q = pts[i];
        const double dx2 = (double)q.z - c2x, dy2 = (double)q.w - c2y;
        const double dx1 = (double)q.x - c1x, dy1 = (double)q.y - c1y;
        a[0] += sqrt(dx2 * dx2 + dy2 * dy2);
        a[1] += sqrt(dx1 * dx1 + dy1 * dy1);
    }
};

void f_reduce_eucdev(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, double* d_part,
                     double* d_out, hipStream_t s) {
    OpFEucDev op{(const float4*)d_pts4, d_mask, c4[0], c4[1], c4[2], c4[3]};
    run_reduce<2>(N, op, d_part, d_out, s);
}

void f_reduce_ata(const float* d_pts4, int N, const uint8_t* d_mask, const double* c4, const double* s4,
                  double* d_part, double* d_out, hipStream_t s) {
    // c4 = {c2x, c2y, c1x, c1y} and s4 likewise (OpSums / OpAbsDev order: dst first)
    OpFAtA op{(const float4*)d_pts4, d_mask, c4[2], c4[3], s4[2], s4[3], c4[0], c4[1], s4[0], s4[1]};
    run_reduce<45>(N, op, d_part, d_out, s);
}

}  // namespace mcv
