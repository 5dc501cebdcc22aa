// ransac_e.hip — gfx950 kernels of the essential-matrix RANSAC path behind cvRecoverPose(s)
// (reference MiniCVNative.cpp:165-215, fivepoint.cpp:233-339).
//
//   mcv_e_pack          V2d pairs -> double4 normalised camera coordinates (x - cx) / f.
//   mcv_e_generate_wave<G> one G-lane group per hypothesis (4 per wave at G = 16): Philox sample of
//                       5 -> five-point solve (fp64, up to 10 models; five_point_wave.h spreads each
//                       step over the group's lanes with the working matrices in LDS) -> all 10
//                       slot statuses + models appended to a dense list (atomic slot allocation;
//                       results are keyed by slot, so the order of the dense list never reaches an
//                       output). mcv_e_stage + mcv_e_roots_g: the split form for large chunks.
//   mcv_e_verify<K,P,E> inlier sweep over the dense model list: wave = K models in VGPRs, 64
//                       lanes stream the double4 correspondences, fp64 Sampson error cast to
//                       float, ballot + popcount; the count lands in the model's slot.
//   mcv_e_verify_pk     the same sweep through the certified packed-fp32 prefilter (sampson_pk.h)
//                       over a float4 copy of the points; undecided lanes re-tested in fp64.
//   mcv_e_one           recompute one hypothesis (winner) -> all its models (one wave).
//   mcv_e_mask          inlier mask of the winner.
//   mcv_e_cheirality    recoverPose: one lane per (RANSAC inlier, (R, t) candidate) cheirality test.
// The reference's five-point solver (the default RANSAC generate, cvFivePoint): ransac_e5.hip.
#include "mcv_common.h"
#include "hyp_essential.h"
#include "five_point_wave.h"
#include "sampson_pk.h"
#include "kernels.h"
#include <algorithm>
#include <cstdlib>

namespace mcv {

__global__ __launch_bounds__(256) void mcv_e_pack(const double2* __restrict__ a, const double2* __restrict__ b, int N,
                                                  double f, double cx, double cy, double4* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const double2 p = a[i], q = b[i];
    double4 o;
    o.x = (p.x - cx) / f;
    o.y = (p.y - cy) / f;
    o.z = (q.x - cx) / f;
    o.w = (q.y - cy) / f;
    out[i] = o;
}

template <int G>
__global__ __launch_bounds__(64) void mcv_e_generate_wave(const double* __restrict__ pts4, int N, Sampler smp,
                                                          int64_t hypBegin, int hypCount, EModel* __restrict__ dense,
                                                          int* __restrict__ denseSlot, int* __restrict__ nDense,
                                                          int* __restrict__ counts) {
    __shared__ EWave S[64 / G];
    const EGroup<G> g(threadIdx.x);
    EWave& W = S[g.base / G];
    const int i = blockIdx.x * (64 / G) + g.base / G;
    if (i >= hypCount) return;
    double E[9];
    const int n = ew_hypothesis(W, g, pts4, N, smp, (uint64_t)(hypBegin + i), E, nullptr);
    const int m = n > 0 ? n : 0;
    if (g.sub < kEMaxModels)
        counts[(int64_t)i * kEMaxModels + g.sub] =
            g.sub < m ? 0 : (g.sub == 0 && n == kStatusNoSample ? kStatusNoSample : kStatusNoModel);
    int base = 0;
    if (g.sub == 0 && m > 0) base = atomicAdd(nDense, m);
    base = __shfl(base, g.base);
    if (g.sub < m) {
        EModel em;
        for (int k = 0; k < 9; ++k) em.e[k] = E[k];
        dense[base + g.sub] = em;
        denseSlot[base + g.sub] = i * kEMaxModels + g.sub;
    }
}

// Split path, part 1: matrix phases of G-lane groups -> EStage per hypothesis.
template <int G>
__global__ __launch_bounds__(64) void mcv_e_stage(const double* __restrict__ pts4, int N, Sampler smp,
                                                  int64_t hypBegin, int hypCount, EStage* __restrict__ st) {
    __shared__ EWave S[64 / G];
    const EGroup<G> g(threadIdx.x);
    const int i = blockIdx.x * (64 / G) + g.base / G;
    if (i >= hypCount) return;
    ew_stage_hypothesis(S[g.base / G], g, pts4, N, smp, (uint64_t)(hypBegin + i), st + i);
}

// Split path, part 2: GR lanes per hypothesis — the derivative levels' intervals dealt
// over the group (ew_group_roots), models by root over the group's lanes, statuses + dense append.
template <int GR>
__global__ __launch_bounds__(64) void mcv_e_roots_g(const EStage* __restrict__ st, int hypCount,
                                                    EModel* __restrict__ dense, int* __restrict__ denseSlot,
                                                    int* __restrict__ nDense, int* __restrict__ counts) {
    __shared__ ERootLds L[64 / GR];
    __shared__ int okAll[64 / GR][kEMaxModels];
    const int sub = threadIdx.x & (GR - 1), grp = threadIdx.x / GR;
    const int i = blockIdx.x * (64 / GR) + grp;
    if (i >= hypCount) return;
    ERootLds& S = L[grp];
    const EStage* h = st + i;
    const int status = h->status;
    const int nr = status == 1 ? ew_group_roots<GR>(S, h->det, sub) : 0;
    double E[kEMaxModels / GR + 1][9];
    bool ok[kEMaxModels / GR + 1];
#pragma unroll
    for (int u = 0; u <= kEMaxModels / GR; ++u) {
        const int r = sub + GR * u;
        ok[u] = r < nr && e_model_at(h->bx, h->by, h->bc, h->nb[0], h->nb[1], h->nb[2], h->nb[3], S.rp[r], E[u]);
        if (r < kEMaxModels) okAll[grp][r] = ok[u] ? 1 : 0;
    }
    ew_sync();
    int m = 0;
    for (int r = 0; r < nr; ++r) m += okAll[grp][r];
    for (int s = sub; s < kEMaxModels; s += GR)
        counts[(int64_t)i * kEMaxModels + s] =
            s < m ? 0 : (s == 0 && status == kStatusNoSample ? kStatusNoSample : kStatusNoModel);
    int base = 0;
    if (sub == 0 && m > 0) base = atomicAdd(nDense, m);
    base = __shfl(base, grp * GR);
#pragma unroll
    for (int u = 0; u <= kEMaxModels / GR; ++u) {
        const int r = sub + GR * u;
        if (!ok[u]) continue;
        int pos = 0;
        for (int t = 0; t < r; ++t) pos += okAll[grp][t];
        EModel em;
#pragma unroll
        for (int k = 0; k < 9; ++k) em.e[k] = E[u][k];
        dense[base + pos] = em;
        denseSlot[base + pos] = i * kEMaxModels + pos;
    }
}

template <int K, int P, int KIND>
__global__ __launch_bounds__(256) void mcv_e_verify(const double4* __restrict__ pts, int N,
                                                    const EModel* __restrict__ dense,
                                                    const int* __restrict__ denseSlot, const int* __restrict__ nDense,
                                                    int* __restrict__ counts, float thr2, double lo, double hi) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int total = __builtin_amdgcn_readfirstlane(*nDense);
    const int m0 = wave * K;
    if (m0 >= total) return;
    double em[K][9];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        valid[k] = m0 + k < total;
        const EModel m = dense[valid[k] ? m0 + k : m0];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            em[k][j] = valid[k] ? m.e[j] : f_dummy_model(j);
            asm volatile("" : "+v"(em[k][j]));
        }
    }
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    // P correspondences per lane per trip (loads in flight), then a 64-wide predicated tail
    const int step = 64 * P;
    const int nFull = N - N % step;
    for (int base = 0; base < nFull; base += step) {
        double4 q[P];
#pragma unroll
        for (int j = 0; j < P; ++j) q[j] = pts[base + 64 * j + lane];
#pragma unroll
        for (int j = 0; j < P; ++j) f_sweep_point<K, KIND>(em, q[j].x, q[j].y, q[j].z, q[j].w, true, thr2, lo, hi, cnt);
    }
    for (int base = nFull; base < N; base += 64) {
        const int p = base + lane;
        const bool v = p < N;
        const double4 q = pts[v ? p : 0];
        f_sweep_point<K, KIND>(em, q.x, q.y, q.z, q.w, v, thr2, lo, hi, cnt);
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k]) counts[denseSlot[m0 + k]] = (int)cnt[k];
    }
}

// Grid = (model waves over the dense list) x (point chunks of `chunk` points, a multiple of 64 P): the
// partial counts of a model's chunks are added atomically (mcv_e5_roots / the fast roots kernel zeroed
// every model slot), and the extra rounds of shorter waves shrink the idle tail of the last round.
template <int KP, int P>
__global__ __launch_bounds__(256) void mcv_e_verify_pk(const float4* __restrict__ pts32,
                                                       const double4* __restrict__ pts, int N, int chunk, bool xcdMap,
                                                       const EModel* __restrict__ dense,
                                                       const int* __restrict__ denseSlot,
                                                       const int* __restrict__ nDense, int* __restrict__ counts,
                                                       float thr2, int kind, SampsonPkCut cut,
                                                       const double* __restrict__ bb) {
    constexpr int K = 2 * KP;
    // XCD-aware (block, chunk) order as in mcv_f_verify_pk: chunk = linear block id mod C (C | 8)
    const unsigned lin = blockIdx.x + blockIdx.y * gridDim.x;
    const unsigned bx = xcdMap ? lin / gridDim.y : blockIdx.x, by = xcdMap ? lin % gridDim.y : blockIdx.y;
    const int wave = __builtin_amdgcn_readfirstlane((int)((bx * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int total = __builtin_amdgcn_readfirstlane(*nDense);
    const int m0 = wave * K;
    __shared__ int blockCounts[4 * K];
    // a block's waves leave together (the count staging's barrier): a wave past the list stages nothing
    if ((int)((bx * 256u) >> 6) * K >= total) return;   // the whole block is past the list
    const bool live = m0 < total;
    const double B[4] = {bb[0], bb[1], bb[2], bb[3]};
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) valid[k] = m0 + k < total;
    SampsonPkPair pr[KP];
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
        double Fa[9], Fb[9];
        const EModel ma = dense[valid[2 * kp] ? m0 + 2 * kp : m0];
        const EModel mb = dense[valid[2 * kp + 1] ? m0 + 2 * kp + 1 : m0];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            Fa[j] = valid[2 * kp] ? ma.e[j] : f_dummy_model(j);
            Fb[j] = valid[2 * kp + 1] ? mb.e[j] : f_dummy_model(j);
        }
        spk_make_pair(pr[kp], Fa, Fb, B, cut);
#pragma unroll
        for (int j = 0; j < 9; ++j) asm volatile("" : "+v"(pr[kp].f[j]));
        asm volatile("" : "+v"(pr[kp].ain));
        asm volatile("" : "+v"(pr[kp].bin));
        asm volatile("" : "+v"(pr[kp].aout));
        asm volatile("" : "+v"(pr[kp].bout));
    }
    auto f64 = [&](int k, double (&F)[9]) {
        const int mk = valid[k] ? m0 + k : -1;
#pragma unroll
        for (int j = 0; j < 9; ++j) F[j] = mk >= 0 ? dense[mk].e[j] : f_dummy_model(j);
    };
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    const int step = 64 * P;
    const int p0 = (int)by * chunk;
    const int p1 = live ? min(N, p0 + chunk) : p0;   // a wave past the list sweeps nothing
    const int nFull = p0 + (p1 - p0) / step * step;
    for (int base = p0; base < nFull; base += step) {
        float4 q[P];
#pragma unroll
        for (int p = 0; p < P; ++p) q[p] = pts32[base + 64 * p + lane];
#pragma unroll
        for (int p = 0; p < P; ++p) {
            const int idx = base + 64 * p + lane;
            auto x64 = [&](double& x1, double& y1, double& x2, double& y2) {
                const double4 d = pts[idx];
                x1 = d.x; y1 = d.y; x2 = d.z; y2 = d.w;
            };
            spk_sweep_point<KP>(pr, q[p], true, cut.L32, cut.H32, kind, thr2, f64, x64, cnt);
        }
    }
    for (int base = nFull; base < p1; base += 64) {
        const int p = base + lane;
        const bool v = p < p1;
        const int idx = v ? p : p0;
        const float4 q = pts32[idx];
        auto x64 = [&](double& x1, double& y1, double& x2, double& y2) {
            const double4 d = pts[idx];
            x1 = d.x; y1 = d.y; x2 = d.z; y2 = d.w;
        };
        spk_sweep_point<KP>(pr, q, v, cut.L32, cut.H32, kind, thr2, f64, x64, cnt);
    }
    // lane k stages model k's count (-1: no model), then the block's 4 K dense models go out from one
    // instruction (F's round-5 staging): their slots lie in one or two appending waves' hypothesis
    // ranges, so the block writes a few cache lines instead of one partial line per wave
    int mine = 0;
    bool mv = false;
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (lane == k) mine = (int)cnt[k], mv = valid[k];
    if (lane < K) blockCounts[(threadIdx.x >> 6) * K + lane] = mv ? mine : -1;
    __syncthreads();
    if (threadIdx.x < 4 * K) {
        const int v = blockCounts[threadIdx.x];
        if (v >= 0) {
            const int slot = denseSlot[(wave - (int)(threadIdx.x >> 6)) * K + (int)threadIdx.x];
            if (gridDim.y == 1) counts[slot] = v;
            else if (v) atomicAdd(counts + slot, v);
        }
    }
}

// Winner's model straight from the dense list of the last evaluated chunk (slot -> model), instead
// of a single-lane five-point re-solve (the same code produced it, so the model is identical).
__global__ __launch_bounds__(256) void mcv_e_fetch(const EModel* __restrict__ dense, const int* __restrict__ denseSlot,
                                                   const int* __restrict__ nDense, int slot,
                                                   EModel* __restrict__ out, int* __restrict__ found) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < *nDense && denseSlot[i] == slot) {
        *out = dense[i];
        *found = 1;
    }
}

__global__ __launch_bounds__(64) void mcv_e_one(const double* __restrict__ pts4, int N, Sampler smp, int64_t hyp,
                                                EOneOut* __restrict__ out) {
    __shared__ EWave S;
    const EGroup<64> g(threadIdx.x);
    const int lane = threadIdx.x;
    double E[9];
    int idx[5] = {-1, -1, -1, -1, -1};
    const int n = ew_hypothesis(S, g, pts4, N, smp, (uint64_t)hyp, E, idx);
    if (lane == 0) {
        out->status = n;
        for (int i = 0; i < 5; ++i) out->idx[i] = idx[i];
    }
    if (lane < kEMaxModels)
        for (int k = 0; k < 9; ++k) out->E[lane][k] = lane < n ? E[k] : 0.0;
}

__global__ __launch_bounds__(256) void mcv_e_mask(const double4* __restrict__ pts, int N, EModel m, float thr2,
                                                  int kind, uint8_t* __restrict__ mask, int* __restrict__ count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < N) {
        const double4 q = pts[i];
        in = f_error(kind, m.e, q.x, q.y, q.z, q.w) <= thr2;
        mask[i] = in ? 1 : 0;
    }
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (int)__popcll(b));
}

struct EPoseCands { double P[4][12]; };

__global__ __launch_bounds__(256) void mcv_e_cheirality(const double4* __restrict__ pts, int N,
                                                        const uint8_t* __restrict__ mask, EPoseCands c, double dist,
                                                        int* __restrict__ good4) {
    // one lane per (correspondence, candidate): the four 4x4 Jacobi solves of a correspondence run
    // side by side instead of one after another (this kernel is on cvRecoverPose's latency path)
    const int t = blockIdx.x * 256 + threadIdx.x;
    const int i = t >> 2, k = t & 3;
    const bool act = i < N && (!mask || mask[i]);
    double4 q = {0, 0, 0, 0};
    if (act) q = pts[i];
    double P[12];
#pragma unroll
    for (int j = 0; j < 12; ++j)
        P[j] = k == 0 ? c.P[0][j] : (k == 1 ? c.P[1][j] : (k == 2 ? c.P[2][j] : c.P[3][j]));
    const bool g = e_cheirality(P, q.x, q.y, q.z, q.w, dist) && act;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
        const uint64_t b = __ballot(g && k == kk);
        if ((threadIdx.x & 63) == 0 && b) atomicAdd(good4 + kk, (int)__popcll(b));
    }
}

// ---- launchers ---------------------------------------------------------------------------------
void launch_e_pack(const double* d_ab, int N, double f, double cx, double cy, double* d_pts4, hipStream_t s) {
    if (N <= 0) return;
    const double2* a = (const double2*)d_ab;
    hipLaunchKernelGGL(mcv_e_pack, dim3((N + 255) / 256), dim3(256), 0, s, a, a + N, N, f, cx, cy,
                       (double4*)d_pts4);
}

void launch_e_generate(const double* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_dense,
                       int* d_denseSlot, int* d_nDense, int* d_counts, void* d_stage, hipStream_t s) {
    (void)hipMemsetAsync(d_nDense, 0, sizeof(int), s);
    if (hypCount <= 0) return;
    static_assert(kEGenLanes == 16 && kEStageLanes == 16 && kERootLanes == 4, "launch shapes below");
    if (d_stage) {   // many hypotheses: matrix phases per 16-lane group, roots per 4-lane group
        EStage* st = (EStage*)d_stage;
        hipLaunchKernelGGL(mcv_e_stage<16>, dim3((hypCount + 3) / 4), dim3(64), 0, s, d_pts4, N, smp, hypBegin,
                           hypCount, st);
        hipLaunchKernelGGL(mcv_e_roots_g<4>, dim3((hypCount + 15) / 16), dim3(64), 0, s, st, hypCount,
                           (EModel*)d_dense, d_denseSlot, d_nDense, d_counts);
        return;
    }
    hipLaunchKernelGGL(mcv_e_generate_wave<16>, dim3((hypCount + 3) / 4), dim3(64), 0, s, d_pts4, N, smp, hypBegin,
                       hypCount, (EModel*)d_dense, d_denseSlot, d_nDense, d_counts);
}

template <int K, int P>
static void launch_e_verify_kp(const double4* p, int N, const EModel* m, const int* d_denseSlot, const int* d_nDense,
                               int maxModels, int* d_counts, float thr2, int kind, double lo, double hi,
                               hipStream_t s) {
    const int blocks = ((maxModels + K - 1) / K + 3) / 4;
    if (kind == 0)
        hipLaunchKernelGGL((mcv_e_verify<K, P, 0>), dim3(blocks), dim3(256), 0, s, p, N, m, d_denseSlot, d_nDense,
                           d_counts, thr2, lo, hi);
    else
        hipLaunchKernelGGL((mcv_e_verify<K, P, 1>), dim3(blocks), dim3(256), 0, s, p, N, m, d_denseSlot, d_nDense,
                           d_counts, thr2, lo, hi);
}

// Certified sweep shape: KP model pairs per wave, P correspondences per lane per trip.
template <int KP, int P>
static void launch_e_verify_pk_kp(const float4* p32, const double4* p, int N, const EModel* m, const int* d_denseSlot,
                                  const int* d_nDense, int maxModels, int* d_counts, float thr2, int kind,
                                  const SampsonPkCut& cut, const double* d_bb, hipStream_t s) {
    const int blocks = ((maxModels + 2 * KP - 1) / (2 * KP) + 3) / 4;
    // point chunks of at least 50000 correspondences (screen at N = 100k: one chunk
    // 12.16 ms, 16384-point chunks 12.25, 32768 12.04, 50000 11.92). At 2^20 hypotheses one chunk writes
    // 62 instead of 284 MB of partial counts per launch but streams the whole 4.8 MB point set through
    // each XCD's 4 MB L2 (24.8 GB of fetches per launch against 0.7 GB; the same 223 ms a step): kept at two.
    // Round 6: one chunk once the model waves alone fill >= 32 rounds of the chip (2^20 hypotheses:
    // ~470k waves) — the counts are then plain stores of the block-staged slots: WRITE_SIZE per launch
    // 97.6 -> 41.2 MiB (two chunks' atomics before), the same verify time (one box, alternating: 301.1 /
    // 301.7 ms against 300.3 / 300.5 with two chunks, scripts/exp/e_chunks.py's workload); smaller
    // calls keep the chunks for their last round's tail.
    constexpr int minChunk = 50000;
    const int step = 64 * P;
    int chunks = (int64_t)blocks * 4 >= 32 * 1024 ? 1 : std::max(1, N / minChunk);
    int chunk = (N + chunks - 1) / chunks;
    chunk = (chunk + step - 1) / step * step;
    chunks = std::max(1, (N + chunk - 1) / chunk);
    hipLaunchKernelGGL((mcv_e_verify_pk<KP, P>), dim3(blocks, chunks), dim3(256), 0, s, p32, p, N, chunk,
                       (8 % chunks) == 0, m, d_denseSlot, d_nDense, d_counts, thr2, kind, cut, d_bb);
}

void launch_e_verify(const double* d_pts4, int N, const void* d_dense, const int* d_denseSlot, const int* d_nDense,
                     int maxModels, int* d_counts, float thr2, int kind, hipStream_t s, const float* d_pts32,
                     const double* d_bb) {
    if (d_pts32 && d_bb) {   // certified packed-fp32 prefilter, 3 model pairs per wave
        launch_e_verify_pk_kp<3, 2>((const float4*)d_pts32, (const double4*)d_pts4, N, (const EModel*)d_dense,
                                    d_denseSlot, d_nDense, maxModels, d_counts, thr2, kind,
                                    sampson_pk_cut_host(sampson_cut(thr2)), d_bb, s);
        return;
    }
    const SampsonCut c = sampson_cut(thr2);
    launch_e_verify_kp<kVerifyEModelsPerWave, kVerifyEPtsPerLane>((const double4*)d_pts4, N, (const EModel*)d_dense,
                                                                  d_denseSlot, d_nDense, maxModels, d_counts, thr2,
                                                                  kind, c.lo, c.hi, s);
}

void launch_e_fetch(const void* d_dense, const int* d_denseSlot, const int* d_nDense, int maxModels, int slot,
                    void* d_out, int* d_found, hipStream_t s) {
    (void)hipMemsetAsync(d_found, 0, sizeof(int), s);
    hipLaunchKernelGGL(mcv_e_fetch, dim3((maxModels + 255) / 256), dim3(256), 0, s, (const EModel*)d_dense,
                       d_denseSlot, d_nDense, slot, (EModel*)d_out, d_found);
}

void launch_e_one(const double* d_pts4, int N, Sampler smp, int64_t hyp, EOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_e_one, dim3(1), dim3(64), 0, s, d_pts4, N, smp, hyp, d_out);
}

void launch_e_mask(const double* d_pts4, int N, const double* E9, float thr2, int kind, uint8_t* d_mask, int* d_count,
                   hipStream_t s) {
    EModel m;
    for (int j = 0; j < 9; ++j) m.e[j] = E9[j];
    hipLaunchKernelGGL(mcv_e_mask, dim3((N + 255) / 256), dim3(256), 0, s, (const double4*)d_pts4, N, m, thr2, kind,
                       d_mask, d_count);
}

void launch_e_cheirality(const double* d_pts4, int N, const uint8_t* d_mask, const double* P4x12, double dist,
                         int* d_good4, hipStream_t s) {
    EPoseCands c;
    for (int k = 0; k < 4; ++k)
        for (int j = 0; j < 12; ++j) c.P[k][j] = P4x12[12 * k + j];
    (void)hipMemsetAsync(d_good4, 0, 4 * sizeof(int), s);
    hipLaunchKernelGGL(mcv_e_cheirality, dim3((4 * (int64_t)N + 255) / 256), dim3(256), 0, s, (const double4*)d_pts4,
                       N, d_mask, c, dist, d_good4);
}


}  // namespace mcv

