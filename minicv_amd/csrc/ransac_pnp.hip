// ransac_pnp.hip — gfx950 kernels of the PnP-RANSAC path behind cvSolvePnPRansac
// (reference MiniCVNative.cpp:93-139, ap3p.cpp:123-317).
//
//   mcv_pnp_pack         V2d image + V3d world -> PnpPoint (fp32, 32 B) on the device.
//   mcv_pnp_generate     one lane per hypothesis: Philox sample of 4 -> undistort -> AP3P
//                        (3 points) + 4th-point selection (fp64) -> PnpPose (96 B) + status.
//   mcv_pnp_verify<K,F>  inlier sweep, 2-D grid: a wave holds K poses (fp64, VGPRs) and one chunk
//                        of the correspondences; projectPoints (k1, k2, p1, p2) in fp64, fp32
//                        squared pixel error, ballot + popcount; chunk partial counts are added
//                        with integer atomics (order-free, exact). The 2-D split keeps the chip
//                        busy at the reference's default 100 iterations.
//   mcv_pnp_generate<1>  EPnP kernels (solverKind 0/1/3/4): 5-point samples, epnp.h per lane.
//   mcv_pnp_one / _mask  winner recompute, inlier mask.
//   mcv_epnp_pass<MODE>  EPnP over the inliers / all points: blocked fixed-order fp64 sums of the
//                        O(n) loops; the O(1) algebra between the passes runs on the host (epnp.h).
//   OpPnpLM / OpPnpVVS   fixed-order fp64 reductions for the LM refit / VVS refinement.
//   mcv_pnp_ap3p         solveAp3p export: one AP3P solve (3 points).
#include "mcv_common.h"
#include "hyp_pnp.h"
#include "pnp_pk.h"
#include "sqpnp.h"
#include "reduce.h"
#include "kernels.h"
#include <cstdlib>

namespace mcv {

__global__ __launch_bounds__(256) void mcv_pnp_pack(const double* __restrict__ img, const double* __restrict__ world,
                                                    int N, PnpPoint* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    PnpPoint p;
    p.X = (float)world[3 * (size_t)i];
    p.Y = (float)world[3 * (size_t)i + 1];
    p.Z = (float)world[3 * (size_t)i + 2];
    p.u = (float)img[2 * (size_t)i];
    p.v = (float)img[2 * (size_t)i + 1];
    p.pad0 = p.pad1 = p.pad2 = 0.f;
    out[i] = p;
}

// AP3P: one hypothesis per lane, one kernel.
__global__ __launch_bounds__(64) void mcv_pnp_generate(const PnpPoint* __restrict__ pts, int N, PnpCamera cam,
                                                       Sampler smp, int64_t hypBegin, int hypCount,
                                                       PnpPose* __restrict__ models, int* __restrict__ counts,
                                                       bool fast) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hypCount) return;
    PnpPose p;
    const int st = pnp_hypothesis(pts, N, cam, smp, (uint64_t)(hypBegin + i), p, nullptr, fast);
    if (st == 1) {
        models[i] = p;
        counts[i] = 0;
    } else {
        counts[i] = st;
    }
}

// EPnP: pnp_hypothesis_epnp split in five kernels (hyp_pnp.h, EpnpSplit). The sweeps kernel keeps half
// of each lane's 12 x 12 in LDS (37 KB per wave, four waves per CU) and half in registers; the betas
// kernel keeps L_6x10 / rho in a per-lane LDS slice; the others hold no LDS.
__global__ __launch_bounds__(256) void mcv_epnp_split_mtm(const PnpPoint* __restrict__ pts, int N, PnpCamera cam,
                                                          Sampler smp, int64_t hypBegin, int hypCount, EpnpSplit X,
                                                          int* __restrict__ counts) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= hypCount) return;
    counts[i] = pnp_epnp_split_mtm(pts, N, cam, smp, (uint64_t)(hypBegin + i), X, i) == 1 ? 0 : kStatusNoSample;
}
__global__ __launch_bounds__(64) void mcv_epnp_split_sweeps(EpnpSplit X, const int* __restrict__ counts,
                                                             int hypCount) {
    __shared__ double lds[64 * kEpnpLoStride];
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= hypCount || counts[i] < 0) return;
    pnp_epnp_split_sweeps(X, i, lds + (size_t)threadIdx.x * kEpnpLoStride);
}
__global__ __launch_bounds__(256) void mcv_epnp_split_tail(EpnpSplit X, const int* __restrict__ counts, int hypCount) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= hypCount || counts[i] < 0) return;
    pnp_epnp_split_tail(X, i);
}
__global__ __launch_bounds__(64) void mcv_epnp_split_betas(EpnpSplit X, const int* __restrict__ counts, int hypCount) {
    __shared__ double lds[64 * 67];
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= hypCount || counts[i] < 0) return;
    pnp_epnp_split_betas(X, i, lds + threadIdx.x * 67);
}
__global__ __launch_bounds__(256) void mcv_epnp_split_pose(PnpCamera cam, EpnpSplit X, PnpPose* __restrict__ models,
                                                           const int* __restrict__ counts, int hypCount) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= hypCount || counts[i] < 0) return;
    PnpPose p;
    pnp_epnp_split_pose(cam, X, i, p);
    models[i] = p;
}

template <int K, bool FUSED>
__global__ __launch_bounds__(256) void mcv_pnp_verify(const PnpPoint* __restrict__ pts, int N, int chunk,
                                                      PnpCamera cam, const PnpPose* __restrict__ models,
                                                      int* __restrict__ counts, int hypCount, float thr2) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;
    double R[K][9], t[K][3];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = hk < hypCount && counts[hk] >= 0;
        const PnpPose m = models[valid[k] ? hk : h0];
#pragma unroll
        for (int j = 0; j < 9; ++j) R[k][j] = valid[k] ? m.R[j] : (j % 4 == 0 ? 1.0 : 0.0);
#pragma unroll
        for (int j = 0; j < 3; ++j) t[k][j] = valid[k] ? m.t[j] : 1e30;
        // poses in VGPRs: 4 x 12 doubles in SGPRs spill into VGPR lanes (v_readlane per use)
#pragma unroll
        for (int j = 0; j < 9; ++j) asm volatile("" : "+v"(R[k][j]));
#pragma unroll
        for (int j = 0; j < 3; ++j) asm volatile("" : "+v"(t[k][j]));
    }
    const int p0 = blockIdx.y * chunk;
    const int p1 = min(N, p0 + chunk);
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    for (int base = p0; base < p1; base += 64) {
        const int p = base + lane;
        const bool v = p < p1;
        const PnpPoint q = pts[v ? p : p0];
        // every lane evaluates (the padding lanes re-read point p0): `v && err <= thr2` would
        // short-circuit into a divergent branch around the whole projection
        const uint64_t vm = __builtin_amdgcn_ballot_w64(v);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float e = pnp_error(cam, R[k], t[k], q.X, q.Y, q.Z, q.u, q.v, FUSED);
            cnt[k] += (uint32_t)__popcll(vm & __builtin_amdgcn_ballot_w64(e <= thr2));
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k] && cnt[k]) atomicAdd(counts + h0 + k, (int)cnt[k]);
    }
}

// Point extents for the prefilter's bound: ext = {max |X|, max |Y|, max |Z|} as the ordered bit
// patterns of non-negative doubles (atomicMax; zeroed by the caller), inf for a non-finite coordinate.
// Also writes the sweep's pair layout: points 2j, 2j + 1 as kPnpPairFloats floats {X0 X1 Y0 Y1 | Z0 Z1
// U0 U1 | V0 V1 - -} at pairs + kPnpPairFloats j (three 16-byte loads give a lane its packed operands).
static constexpr int kPnpPairFloats = 2 * kPnpPairFloatsPerPoint;
__global__ __launch_bounds__(256) void mcv_pnp_extent(const PnpPoint* __restrict__ pts, int N,
                                                      unsigned long long* __restrict__ ext, float* __restrict__ pairs) {
    double m0 = 0, m1 = 0, m2 = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < N; i += gridDim.x * 256) {
        const PnpPoint q = pts[i];
        float* o = pairs + (size_t)(i >> 1) * kPnpPairFloats + (i & 1);
        o[0] = q.X; o[2] = q.Y; o[4] = q.Z; o[6] = q.u; o[8] = q.v;
        const double x = q.X, y = q.Y, z = q.Z;
        m0 = x - x == 0 ? fmax(m0, fabs(x)) : __builtin_inf();
        m1 = y - y == 0 ? fmax(m1, fabs(y)) : __builtin_inf();
        m2 = z - z == 0 ? fmax(m2, fabs(z)) : __builtin_inf();
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        m0 = fmax(m0, __shfl_xor(m0, off, 64));
        m1 = fmax(m1, __shfl_xor(m1, off, 64));
        m2 = fmax(m2, __shfl_xor(m2, off, 64));
    }
    __shared__ double sm[4][3];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sm[w][0] = m0; sm[w][1] = m1; sm[w][2] = m2; }
    __syncthreads();
    if (threadIdx.x < 3) {
        double m = sm[0][threadIdx.x];
        for (int k = 1; k < 4; ++k) m = fmax(m, sm[k][threadIdx.x]);
        atomicMax(ext + threadIdx.x, (unsigned long long)__double_as_longlong(m));
    }
}

// Exact inlier count of one pose over the 128 points [base, base + 128) n [p0, p1) (two per lane):
// the reference's fp64 projection + fp32 error (pnp_error). The prefilter's undecided trips.
__device__ __forceinline__ uint32_t pnp_exact_trip(const PnpPoint* __restrict__ pts, int base, int p0, int p1,
                                                PnpCamera cam, const PnpPose* __restrict__ models, int hk,
                                                float thr2, bool fused) {
    const int lane = threadIdx.x & 63;
    double R[9], t[3];
    const PnpPose m = models[hk];
    for (int j = 0; j < 9; ++j) R[j] = m.R[j];
    for (int j = 0; j < 3; ++j) t[j] = m.t[j];
    uint32_t c = 0;
    for (int h = 0; h < 2; ++h) {
        const int i = base + 2 * lane + h;
        const bool v = i < p1;
        const PnpPoint q = pts[v ? i : p0];
        const bool in = v && pnp_error(cam, R, t, q.X, q.Y, q.Z, q.u, q.v, fused) <= thr2;
        c += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(in));
    }
    return c;
}

// Certified packed-fp32 sweep (pnp_pk.h): a wave holds K poses (fp32 copies + bound constants, wave-
// uniform) and streams a chunk of the points two per lane (lane l of a trip reads points base + 2l,
// base + 2l + 1: 64 contiguous bytes). Per (pose, point pair): the packed projection, the bound, two
// cuts; a trip whose lanes are all decided adds its certified inliers, a trip with an undecided lane
// is recorded (LDS event list: trip << 8 | pose mask) and recounted exactly after the sweep. An
// event-list overflow recounts the wave's chunk exactly. Partial counts by integer atomics.
static constexpr int kPnpEvents = 192;   // per wave
// LANE form (round 4, the default): the log holds undecided (point, pose) lanes instead of (trip, pose
// mask) events, and the recount takes 64 of them per pass, one per lane: a trip with one undecided
// lane costs one lane of an fp64 pass instead of a whole fp64 trip. Entry = (point - p0) << 3 | pose.
static constexpr int kPnpLaneEvents = 512;   // per wave

// A wave-uniform pair into SGPRs (readfirstlane is an int builtin: bit copies).
__device__ __forceinline__ pkf2 pk_uniform(pkf2 v) {
    return pkf2{__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.x))),
                __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v.y)))};
}

template <int K, int WPE, bool LANE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void mcv_pnp_verify_pk(const PnpPoint* __restrict__ pts, int N, int chunk,
                                                         PnpCamera cam, PnpPkCam pc, const PnpPose* __restrict__ models,
                                                         int* __restrict__ counts, int hypCount, float thr2, bool fused,
                                                         const double* __restrict__ ext, const float* __restrict__ pairs) {
    static_assert(K <= 8, "pose mask in 8 bits");
    constexpr int kCap = LANE ? kPnpLaneEvents : kPnpEvents;
    __shared__ uint32_t events[4][kCap];
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int wib = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;
    const double e3[3] = {ext[0], ext[1], ext[2]};
    const pkf2 z2 = pkf2{0.0f, 0.0f};
    PnpPkCamV<pkf2> cv = pnp_pk_cam_v<pkf2>(pc, z2);
    asm volatile("" : "+v"(cv.k1), "+v"(cv.cx), "+v"(cv.cy), "+v"(cv.A2), "+v"(cv.Cg), "+v"(cv.thrLo), "+v"(cv.twoT));
    // the projection's coefficient pairs in SGPRs; the exact tier's (rarely run) in VGPR pairs
    cv.k2tp1 = pk_uniform(cv.k2tp1); cv.tp2p1 = pk_uniform(cv.tp2p1); cv.p2fx = pk_uniform(cv.p2fx);
    cv.fyA4 = pk_uniform(cv.fyA4);
    asm volatile("" : "+v"(cv.cpu13), "+v"(cv.Fgnt), "+v"(cv.gkHi));
    PnpPkPoseV<pkf2> pp[K];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = hk < hypCount && counts[hk] >= 0;
        const PnpPose m = models[valid[k] ? hk : h0];
        PnpPkPose p;
        pnp_pk_pose(m.R, m.t, e3, pc, p);
        pp[k] = pnp_pk_pose_v<pkf2>(p, z2);
        pp[k].zmin = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(pp[k].zmin)));
        asm volatile("" : "+v"(pp[k].t0), "+v"(pp[k].t1), "+v"(pp[k].t2), "+v"(pp[k].c1));
        asm volatile("" : "+v"(pp[k].qPl), "+v"(pp[k].qLh), "+v"(pp[k].qHW), "+v"(pp[k].qB0), "+v"(pp[k].qB1));
        // pose coefficient pairs in SGPRs, read through op_sel. (K = 4 poses' pairs plus the ballot masks
        // of their interleaved tests overflow the SGPR file by ~15 spilled dwords per trip; the VGPR-pair
        // placement that avoids it measured slower: 1.92 vs 1.79 ms at the PnP bench. K = 3, the
        // default since round 3, spills less: 1.62 vs 1.72 ms at K = 4, 1.78 ms at K = 5)
        pp[k].r01 = pk_uniform(pp[k].r01); pp[k].r23 = pk_uniform(pp[k].r23); pp[k].r45 = pk_uniform(pp[k].r45);
        pp[k].r67 = pk_uniform(pp[k].r67); pp[k].r8c2 = pk_uniform(pp[k].r8c2);
    }
    uint32_t validMask = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) validMask |= valid[k] ? 1u << k : 0u;
    const int p0 = blockIdx.y * chunk;
    const int p1 = min(N, p0 + chunk);
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    int nev = 0;
    // one trip: 128 points (two per lane) against the K poses; vm0 / vm1 = the lanes whose points exist
    auto trip = [&](int base, pkf2 X, pkf2 Y, pkf2 Z, pkf2 U, pkf2 V, uint64_t vm0, uint64_t vm1) {
        const int i0 = base + 2 * lane, i1 = i0 + 1;
        uint32_t und = 0;
        asm volatile("" : "+s"(cv.k2tp1), "+s"(cv.tp2p1), "+s"(cv.p2fx), "+s"(cv.fyA4));
        // every pose's projection, bound and masks first, in one basic block (the K dependent chains
        // interleave), then the counts and the log
        uint64_t in0[K], in1[K], out0[K], out1[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            asm volatile("" : "+s"(pp[k].r01), "+s"(pp[k].r23), "+s"(pp[k].r45), "+s"(pp[k].r67), "+s"(pp[k].r8c2));
            const PnpPkProj<pkf2> o = pnp_pk_project<pkf2>(cv, pp[k], X, Y, Z, U, V);
            pkf2 lo, hi;
            pnp_pk_bound<pkf2>(cv, pp[k], o, lo, hi);
            const uint64_t d0 = __builtin_amdgcn_ballot_w64(fabsf(o.Zc.x) >= pp[k].zmin);
            const uint64_t d1 = __builtin_amdgcn_ballot_w64(fabsf(o.Zc.y) >= pp[k].zmin);
            in0[k] = __builtin_amdgcn_ballot_w64(o.S.x < lo.x) & d0;
            in1[k] = __builtin_amdgcn_ballot_w64(o.S.y < lo.y) & d1;
            out0[k] = __builtin_amdgcn_ballot_w64(o.S.x > hi.x) & d0;
            out1[k] = __builtin_amdgcn_ballot_w64(o.S.y > hi.y) & d1;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t u = (vm0 & ~(in0[k] | out0[k])) | (vm1 & ~(in1[k] | out1[k]));
            const uint32_t c = (uint32_t)__popcll(in0[k] & vm0) + (uint32_t)__popcll(in1[k] & vm1);
            if constexpr (LANE) {
                // the decided lanes count now; the undecided ones go to the log, one entry per lane
                cnt[k] += c;
                if (u != 0 && ((validMask >> k) & 1u)) {   // wave-uniform, rare
                    const uint64_t ud0 = vm0 & ~(in0[k] | out0[k]), ud1 = vm1 & ~(in1[k] | out1[k]);
                    const int n0 = __popcll(ud0), n1 = __popcll(ud1);
                    if (nev + n0 + n1 <= kCap) {
                        const uint64_t lt = (1ull << lane) - 1ull;
                        if ((ud0 >> lane) & 1ull)
                            events[wib][nev + __popcll(ud0 & lt)] = ((uint32_t)(i0 - p0) << 3) | (uint32_t)k;
                        if ((ud1 >> lane) & 1ull)
                            events[wib][nev + n0 + __popcll(ud1 & lt)] = ((uint32_t)(i1 - p0) << 3) | (uint32_t)k;
                    }
                    nev += n0 + n1;
                }
            } else {
                // branch-free: a trip with an undecided lane adds nothing here (recounted exactly later)
                const uint32_t bit = u != 0 ? 1u << k : 0u;
                und |= bit;
                cnt[k] += bit ? 0u : c;
            }
        }
        if constexpr (!LANE) {
            und &= validMask;
            if (__builtin_expect(und != 0, 0)) {
                if (nev < kPnpEvents && lane == 0) events[wib][nev] = ((uint32_t)((base - p0) >> 7) << 8) | und;
                ++nev;
            }
        }
    };
    // full trips: every point exists (chunks are multiples of 128 points); operands straight from the pair
    // layout, no bounds or address selects
    const int nFull = p0 + (p1 - p0) / 128 * 128;
    const float4* pr4 = reinterpret_cast<const float4*>(pairs) + (size_t)(p0 / 2 + lane) * (kPnpPairFloats / 4);
    for (int base = p0; base < nFull; base += 128, pr4 += 64 * (kPnpPairFloats / 4)) {
        const float4 a = pr4[0], b = pr4[1], c = pr4[2];
        trip(base, pkf2{a.x, a.y}, pkf2{a.z, a.w}, pkf2{b.x, b.y}, pkf2{b.z, b.w}, pkf2{c.x, c.y}, ~0ull, ~0ull);
    }
    if (nFull < p1) {   // the chunk's partial trip
        const int base = nFull;
        const int i0 = base + 2 * lane, i1 = i0 + 1;
        const bool v0 = i0 < p1, v1 = i1 < p1;
        const PnpPoint a = pts[v0 ? i0 : p0];
        const PnpPoint b = pts[v1 ? i1 : p0];
        trip(base, pkf2{a.X, b.X}, pkf2{a.Y, b.Y}, pkf2{a.Z, b.Z}, pkf2{a.u, b.u}, pkf2{a.v, b.v},
             __builtin_amdgcn_ballot_w64(v0), __builtin_amdgcn_ballot_w64(v1));
    }
    if constexpr (LANE) {
        // exact recount, 64 logged lanes per pass; an overflowing log recounts every (point, pose) of
        // the chunk (same single inlined copy of the fp64 error)
        const bool overflow = nev > kCap;
        if (overflow) {
#pragma unroll
            for (int k = 0; k < K; ++k) cnt[k] = 0;
        }
        const int total = overflow ? (p1 - p0) * K : nev;
        if (total > 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        for (int j0 = 0; j0 < total; j0 += 64) {
            const int j = j0 + lane;
            bool act = j < total;
            int k, i;
            if (overflow) {
                k = j % K;
                i = p0 + j / K;
            } else {
                const uint32_t ev = events[wib][act ? j : 0];
                k = (int)(ev & 7u);
                i = p0 + (int)(ev >> 3);
            }
            act = act && ((validMask >> k) & 1u) != 0;
            const PnpPose m = models[act ? h0 + k : h0];
            const PnpPoint q = pts[act ? i : p0];
            double R[9], t[3];
            for (int r = 0; r < 9; ++r) R[r] = m.R[r];
            for (int r = 0; r < 3; ++r) t[r] = m.t[r];
            const bool in = act && pnp_error(cam, R, t, q.X, q.Y, q.Z, q.u, q.v, fused) <= thr2;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) cnt[kk] += (uint32_t)__popcll(__builtin_amdgcn_ballot_w64(in && k == kk));
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (valid[k] && cnt[k]) atomicAdd(counts + h0 + k, (int)cnt[k]);
        }
        return;
    }
    // exact recount of the logged (trip, pose) events; too many undecided trips (a pose outside the
    // bound's domain) recount every trip of the chunk for every pose. One inlined copy of the fp64 trip
    // serves both (a called function would put its frame and the caller's saved registers in scratch).
    const bool overflow = nev > kPnpEvents;
    if (overflow) {
#pragma unroll
        for (int k = 0; k < K; ++k) cnt[k] = 0;
    }
    const int nres = overflow ? (p1 - p0 + 127) / 128 : nev;
    if (nres > 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
    for (int e = 0; e < nres; ++e) {
        const uint32_t ev = overflow ? (((uint32_t)e << 8) | validMask)
                                     : (uint32_t)__builtin_amdgcn_readfirstlane(events[wib][e]);
        const int base = p0 + (int)(ev >> 8) * 128;
        uint32_t m = ev & 0xFFu;
        while (m != 0) {   // wave-uniform
            const int k = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t c = pnp_exact_trip(pts, base, p0, p1, cam, models, h0 + k, thr2, fused);
#pragma unroll
            for (int kk = 0; kk < K; ++kk) cnt[kk] += kk == k ? c : 0u;
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k] && cnt[k]) atomicAdd(counts + h0 + k, (int)cnt[k]);
    }
}

__global__ void mcv_pnp_one(const PnpPoint* __restrict__ pts, int N, PnpCamera cam, Sampler smp, int64_t hyp,
                            bool epnp, bool fast, PnpOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    PnpPose p;
    for (int k = 0; k < 9; ++k) p.R[k] = 0;
    for (int k = 0; k < 3; ++k) p.t[k] = 0;
    int idx[5] = {-1, -1, -1, -1, -1};
    out->status = epnp ? pnp_hypothesis_epnp(pts, N, cam, smp, (uint64_t)hyp, p, idx)
                       : pnp_hypothesis(pts, N, cam, smp, (uint64_t)hyp, p, idx, fast);
    for (int k = 0; k < 9; ++k) out->R[k] = p.R[k];
    for (int k = 0; k < 3; ++k) out->t[k] = p.t[k];
    for (int k = 0; k < 5; ++k) out->idx[k] = idx[k];
}

// solvePnP(EPNP) on exactly 5 float correspondences (solvePnPRansac's npoints == model_points case).
__global__ void mcv_pnp_solve5(const PnpPoint* __restrict__ pts, PnpCamera cam, PnpOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    PnpPoint p5[5];
    for (int i = 0; i < 5; ++i) p5[i] = pts[i];
    PnpPose p;
    pnp_epnp5(cam, p5, p);
    out->status = 1;
    for (int k = 0; k < 9; ++k) out->R[k] = p.R[k];
    for (int k = 0; k < 3; ++k) out->t[k] = p.t[k];
    for (int k = 0; k < 5; ++k) out->idx[k] = k;
}

// Direct four-point solve on given normalised points (N == 4 path of solvePnPRansac / solvePnP).
__global__ void mcv_pnp_solve4(const PnpPoint* __restrict__ pts, PnpCamera cam, bool fast, PnpOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double x[4], y[4], W[4][3];
    for (int i = 0; i < 4; ++i) {
        const PnpPoint p = pts[i];
        pnp_undistort(cam, (double)p.u, (double)p.v, x[i], y[i]);
        W[i][0] = p.X; W[i][1] = p.Y; W[i][2] = p.Z;
    }
    PnpPose p;
    for (int k = 0; k < 9; ++k) p.R[k] = 0;
    for (int k = 0; k < 3; ++k) p.t[k] = 0;
    out->status = (fast ? pnp_ap3p4(cam, x, y, W, p) : pnp_ap3p4_cv(cam, x, y, W, p)) ? 1 : kStatusNoModel;
    for (int k = 0; k < 9; ++k) out->R[k] = p.R[k];
    for (int k = 0; k < 3; ++k) out->t[k] = p.t[k];
    for (int k = 0; k < 4; ++k) out->idx[k] = k;
    out->idx[4] = -1;
}

// mp (optional): the pose read from the device instead of the by-value m.
__global__ __launch_bounds__(256) void mcv_pnp_mask(const PnpPoint* __restrict__ pts, int N, PnpCamera cam,
                                                    PnpPose m, const PnpPose* __restrict__ mp, float thr2, bool fused,
                                                    uint8_t* __restrict__ mask, int* __restrict__ count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (mp) m = *mp;
    if (i < N) {
        const PnpPoint q = pts[i];
        in = pnp_error(cam, m.R, m.t, q.X, q.Y, q.Z, q.u, q.v, fused) <= thr2;
        mask[i] = in ? 1 : 0;
    }
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (int)__popcll(b));
}

// The reference's solveAp3p (ap3p.cpp:282-317): bearings from (inv_fx u - cx_fx, ...), the solutions
// of its own Ferrari quartic path in its order (ap3p_compute_poses_ref).
__global__ void mcv_pnp_ap3p(Ap3pIn in, Ap3pOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double b[3][3], w[3][3];
    for (int i = 0; i < 3; ++i) {
        double mu = in.inv_fx * in.mu[i] - in.cx_fx;
        double mv = in.inv_fy * in.mv[i] - in.cy_fy;
        const double nrm = sqrt(mu * mu + mv * mv + 1);
        const double mk = 1. / nrm;
        mu = mu * mk;
        mv = mv * mk;
        b[i][0] = mu; b[i][1] = mv; b[i][2] = mk;
        for (int k = 0; k < 3; ++k) w[i][k] = in.W[i][k];
    }
    double Rr[kPnpMaxSolutions][9], tr[kPnpMaxSolutions][3];
    bool cplx = false;
    const int n = ap3p_compute_poses_ref(b, w, Rr, tr, &cplx);
    out->cplx = cplx ? 1 : 0;
    out->count = n;
    for (int s = 0; s < kPnpMaxSolutions; ++s) {
        for (int k = 0; k < 9; ++k) out->R[s][k] = s < n ? Rr[s][k] : 0.0;
        for (int k = 0; k < 3; ++k) out->t[s][k] = s < n ? tr[s][k] : 0.0;
    }
}

// ---- LM / VVS reductions ---------------------------------------------------------------------
// Per correspondence: residual r = projectPoints(X) - observed (pixels, fp64) and its Jacobian
// w.r.t. (rvec, t) through dR/drvec (host Rodrigues derivative). 28 sums: J^T J upper (21),
// J^T r (6), |r|^2 (1).
struct OpPnpLM {
    const PnpPoint* pts; const uint8_t* mask; PnpCamera c; double R[9]; double t[3]; double dR[27]; bool wantJ;
    __device__ void operator()(int i, double (&a)[28]) const {
        if (mask && !mask[i]) return;
        const PnpPoint q = pts[i];
        const double X = q.X, Y = q.Y, Z = q.Z;
        const double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
        const double Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        const double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        const double iz = Zc != 0 ? 1.0 / Zc : 1.0;
        const double x = Xc * iz, y = Yc * iz;
        const double r2 = x * x + y * y, r4 = r2 * r2;
        const double cdist = 1.0 + c.k1 * r2 + c.k2 * r4;
        const double xd = x * cdist + c.p1 * (2.0 * x * y) + c.p2 * (r2 + 2.0 * x * x);
        const double yd = y * cdist + c.p1 * (r2 + 2.0 * y * y) + c.p2 * (2.0 * x * y);
        const double ru = xd * c.fx + c.cx - (double)q.u;
        const double rv = yd * c.fy + c.cy - (double)q.v;
        a[27] += ru * ru + rv * rv;
        if (!wantJ) return;
        const double dcr = c.k1 + 2.0 * c.k2 * r2;              // d cdist / d r2
        const double dxdx = cdist + x * dcr * 2.0 * x + 2.0 * c.p1 * y + 6.0 * c.p2 * x;
        const double dxdy = x * dcr * 2.0 * y + 2.0 * c.p1 * x + 2.0 * c.p2 * y;
        const double dydx = y * dcr * 2.0 * x + 2.0 * c.p1 * x + 2.0 * c.p2 * y;
        const double dydy = cdist + y * dcr * 2.0 * y + 6.0 * c.p1 * y + 2.0 * c.p2 * x;
        // d(x, y) / d(Xc, Yc, Zc) = iz [[1, 0, -x], [0, 1, -y]]
        const double du[3] = {c.fx * dxdx * iz, c.fx * dxdy * iz, c.fx * (-dxdx * x - dxdy * y) * iz};
        const double dv[3] = {c.fy * dydx * iz, c.fy * dydy * iz, c.fy * (-dydx * x - dydy * y) * iz};
        double Ju[6], Jv[6];
#pragma unroll
        for (int j = 0; j < 3; ++j) {   // dXc/drvec_j = dR/dr_j * X
            const double* d = dR + 9 * j;
            const double gx = d[0] * X + d[1] * Y + d[2] * Z;
            const double gy = d[3] * X + d[4] * Y + d[5] * Z;
            const double gz = d[6] * X + d[7] * Y + d[8] * Z;
            Ju[j] = du[0] * gx + du[1] * gy + du[2] * gz;
            Jv[j] = dv[0] * gx + dv[1] * gy + dv[2] * gz;
            Ju[3 + j] = du[j];
            Jv[3 + j] = dv[j];
        }
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j)
#pragma unroll
            for (int k = j; k < 6; ++k) a[o++] += Ju[j] * Ju[k] + Jv[j] * Jv[k];
#pragma unroll
        for (int j = 0; j < 6; ++j) a[21 + j] += Ju[j] * ru + Jv[j] * rv;
    }
};

// VVS (solvePnPRefineVVS, [ext]): normalised-plane feature error e = (x, y) - undistorted observed
// point, interaction matrix L (2 x 6, camera-frame twist (v, w)); sums L^T L (21), L^T e (6), |e|^2.
struct OpPnpVVS {
    const PnpPoint* pts; const uint8_t* mask; PnpCamera c; double R[9]; double t[3];
    __device__ void operator()(int i, double (&a)[28]) const {
        if (mask && !mask[i]) return;
        const PnpPoint q = pts[i];
        const double X = q.X, Y = q.Y, Z = q.Z;
        const double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
        const double Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        const double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        const double iz = Zc != 0 ? 1.0 / Zc : 1.0;
        const double x = Xc * iz, y = Yc * iz;
        double xo, yo;
        pnp_undistort(c, (double)q.u, (double)q.v, xo, yo);
        const double ex = x - xo, ey = y - yo;
        const double Lx[6] = {-iz, 0.0, x * iz, x * y, -(1.0 + x * x), y};
        const double Ly[6] = {0.0, -iz, y * iz, 1.0 + y * y, -x * y, -x};
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j)
#pragma unroll
            for (int k = j; k < 6; ++k) a[o++] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
#pragma unroll
        for (int j = 0; j < 6; ++j) a[21 + j] += Lx[j] * ex + Ly[j] * ey;
        a[27] += ex * ex + ey * ey;
    }
};

// ---- EPnP on a large point set (the inlier solve of solvePnPRansac, solvePnP(EPNP)) ----------
// Mask -> ascending index list (one block, 1024 threads, chunked ballot scan): the inliers in the
// order compressElems keeps them.
__global__ __launch_bounds__(1024) void mcv_mask_compact(const uint8_t* __restrict__ mask, int N,
                                                         int* __restrict__ idx, int* __restrict__ count) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    int base = 0;
    for (int c0 = 0; c0 < N; c0 += 1024) {
        const int i = c0 + tid;
        const bool f = i < N && mask[i] != 0;
        const uint64_t b = __ballot(f);
        const int below = (int)__popcll(b & ((1ull << lane) - 1));
        if (lane == 0) wsum[wv] = (int)__popcll(b);
        __syncthreads();
        int off = 0, tot = 0;
        for (int w = 0; w < 16; ++w) {
            off += w < wv ? wsum[w] : 0;
            tot += wsum[w];
        }
        if (f) idx[base + off + below] = i;
        base += tot;
        __syncthreads();
    }
    if (tid == 0) *count = base;
}

// Points of the solve in double: pw = world, us = undistortPoints (double result) * f + c.
__global__ __launch_bounds__(256) void mcv_epnp_prep_f32(const PnpPoint* __restrict__ pts, const int* __restrict__ idx,
                                                         int n, PnpCamera c, double* __restrict__ pw,
                                                         double* __restrict__ us, const int* __restrict__ nDev) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (nDev) n = *nDev;
    if (i >= n) return;
    const PnpPoint p = pts[idx ? idx[i] : i];
    double x, y;
    pnp_undistort(c, (double)p.u, (double)p.v, x, y);
    us[2 * (size_t)i] = x * c.fx + c.cx;
    us[2 * (size_t)i + 1] = y * c.fy + c.cy;
    pw[3 * (size_t)i] = p.X;
    pw[3 * (size_t)i + 1] = p.Y;
    pw[3 * (size_t)i + 2] = p.Z;
}

__global__ __launch_bounds__(256) void mcv_epnp_prep_f64(const double* __restrict__ img, const double* __restrict__ world,
                                                         int n, PnpCamera c, double* __restrict__ pw,
                                                         double* __restrict__ us, bool normalized) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double x, y;
    pnp_undistort(c, img[2 * (size_t)i], img[2 * (size_t)i + 1], x, y);
    us[2 * (size_t)i] = normalized ? x : x * c.fx + c.cx;
    us[2 * (size_t)i + 1] = normalized ? y : y * c.fy + c.cy;
    for (int k = 0; k < 3; ++k) pw[3 * (size_t)i + k] = world[3 * (size_t)i + k];
}

// 128 points a tile (round 5; 32 before): a quarter of the barrier rounds per 1024-point block, the
// same per-accumulator point order (the sums are unchanged)
static constexpr int kEpnpTile = 128;
static constexpr int kEpnpTermCols = 39;   // the widest non-MtM pass (kSqpSums); MtM stages 24 doubles a point

// One (point, accumulator) term of a pass — the body of the corresponding epnp.cpp loop; the MtM
// pass adds two products per point (r1 and r2 rows), the others one (t[1] unused).
template <int MODE>
__device__ __forceinline__ void epnp_pass_term(const double* __restrict__ pw, const double* __restrict__ us,
                                               const EpnpPassArgs& A, int i, int acc, double (&t)[2]) {
    const double* p = pw + 3 * (size_t)i;
    if (MODE == kEpnpPassSumPw) {
        t[0] = p[acc];
    } else if (MODE == kEpnpPassPw0) {
        const int a = acc < 3 ? 0 : (acc < 5 ? 1 : 2);
        const int b = acc < 3 ? acc : (acc < 5 ? acc - 2 : 2);
        t[0] = (p[a] - A.c0[a]) * (p[b] - A.c0[b]);
    } else if (MODE == kEpnpPassMtm) {
        int a = 0, r = acc;
        while (a < 12 && r >= 12 - a) { r -= 12 - a; ++a; }
        const int b = a + r;
        double al[4], r1[12], r2[12];
        epnp_alphas(A.C, p, al);
        epnp_m_rows(al, us[2 * (size_t)i], us[2 * (size_t)i + 1], A.cam, r1, r2);
        t[0] = r1[a] * r1[b];
        t[1] = r2[a] * r2[b];
    } else if (MODE == kEpnpPassPc) {
        double al[4], pc[3];
        epnp_alphas(A.C, p, al);
        epnp_pc(al, A.ccs[acc / 3], pc);
        t[0] = pc[acc % 3];
    } else if (MODE == kEpnpPassAbt) {
        const int N = acc / 9, j = (acc % 9) / 3, k = acc % 3;
        double al[4], pc[3];
        epnp_alphas(A.C, p, al);
        epnp_pc(al, A.ccs[N], pc);
        t[0] = (pc[j] - A.pc0[N][j]) * (p[k] - A.pw0[k]);
    } else if (MODE == kEpnpPassSqp) {
        t[0] = sqpnp_term(us[2 * (size_t)i], us[2 * (size_t)i + 1], p[0], p[1], p[2], acc);
    } else if (MODE == kEpnpPassSqpDepth) {
        t[0] = A.R[0][2][0] * p[0] + A.R[0][2][1] * p[1] + A.R[0][2][2] * p[2] + A.t[0][2] > 0 ? 1.0 : 0.0;
    } else {
        t[0] = epnp_reproj_term(A.R[acc], A.t[acc], A.cam, p, us[2 * (size_t)i], us[2 * (size_t)i + 1]);
    }
}

// One workgroup per block of kEpnpBlock points, one lane per accumulator: each accumulator adds its
// block's terms in point order from 0 (the O(n) loops of epnp.cpp), exactly as a sequential loop
// would. The terms of a tile of kEpnpTile points are computed by all lanes in parallel into LDS
// first, so the ordered chains only add. Partials part[acc * nblk + blk], summed over blocks in
// order on the host.
template <int MODE>
__global__ __launch_bounds__(256) void mcv_epnp_pass(const double* __restrict__ pw, const double* __restrict__ us,
                                                     int n, EpnpPassArgs A, int nacc, int nblk,
                                                     double* __restrict__ part, const int* __restrict__ nDev,
                                                     const double* __restrict__ prev) {
    if (nDev) {   // the grid covers the upper bound: blocks past the device count's write nothing
        n = *nDev;
        nblk = (n + kEpnpBlock - 1) / kEpnpBlock;
        if ((int)blockIdx.x >= nblk) return;
    }
    // prev (optional): the previous pass's partials (same n), whose means this pass needs, summed over
    // the blocks in order from 0 and divided by n exactly as the host does: Pw0's centroid from SumPw,
    // Abt's pc0 from Pc. Saves the host round trip between the two passes.
    if (prev && MODE == kEpnpPassPw0)
        for (int j = 0; j < 3; ++j) {
            double t = 0;
            for (int b = 0; b < nblk; ++b) t += prev[(size_t)j * nblk + b];
            A.c0[j] = t / n;
        }
    if (prev && MODE == kEpnpPassAbt)
        for (int a = 0; a < 9; ++a) {
            double t = 0;
            for (int b = 0; b < nblk; ++b) t += prev[(size_t)a * nblk + b];
            A.pc0[a / 3][a % 3] = t / n;
        }
    static_assert(kSqpSums <= kEpnpTermCols && 24 <= kEpnpTermCols && 27 <= kEpnpTermCols, "term tile width");
    __shared__ double term[kEpnpTile * kEpnpTermCols];
    int ma = 0, mb = 0;   // MtM: the accumulator's (row, column) of the upper triangle
    if (MODE == kEpnpPassMtm) {
        int r = threadIdx.x;
        while (ma < 12 && r >= 12 - ma) { r -= 12 - ma; ++ma; }
        mb = ma + r;
    }
    const int blk = blockIdx.x;
    const int i0 = blk * kEpnpBlock;
    const int i1 = min(n, i0 + kEpnpBlock);
    const int acc = threadIdx.x;
    double s = 0;
    for (int t0 = i0; t0 < i1; t0 += kEpnpTile) {
        const int tn = min(kEpnpTile, i1 - t0);
        if (MODE == kEpnpPassMtm) {
            // 78 accumulators share a point's two M rows: one lane per point computes them, the
            // ordered lanes form their products from LDS
            double* rows = term;   // [kEpnpTile][24]
            for (int j = threadIdx.x; j < tn; j += 256) {
                const int i = t0 + j;
                double al[4], r1[12], r2[12];
                epnp_alphas(A.C, pw + 3 * (size_t)i, al);
                epnp_m_rows(al, us[2 * (size_t)i], us[2 * (size_t)i + 1], A.cam, r1, r2);
                for (int k = 0; k < 12; ++k) { rows[j * 24 + k] = r1[k]; rows[j * 24 + 12 + k] = r2[k]; }
            }
            __syncthreads();
            if (acc < nacc)
                for (int j = 0; j < tn; ++j) {
                    s += rows[j * 24 + ma] * rows[j * 24 + mb];
                    s += rows[j * 24 + 12 + ma] * rows[j * 24 + 12 + mb];
                }
        } else if (MODE == kEpnpPassPc || MODE == kEpnpPassAbt) {
            // a point's three camera-frame positions (and, for A B^T, its centred world point) once
            // per point instead of once per accumulator; the accumulators' terms are the same
            // operations on the same values (Pc: pc[j]; Abt: (pc[j] - pc0[N][j]) * (p[k] - pw0[k]))
            constexpr int W = MODE == kEpnpPassPc ? 9 : 12;
            double* rows = term;   // [kEpnpTile][W]
            for (int j = threadIdx.x; j < tn; j += 256) {
                const double* p = pw + 3 * (size_t)(t0 + j);
                double al[4];
                epnp_alphas(A.C, p, al);
#pragma unroll
                for (int N = 0; N < 3; ++N) {
                    double pc[3];
                    epnp_pc(al, A.ccs[N], pc);
#pragma unroll
                    for (int c = 0; c < 3; ++c) rows[j * W + 3 * N + c] = MODE == kEpnpPassPc ? pc[c] : pc[c] - A.pc0[N][c];
                }
                if (MODE == kEpnpPassAbt)
#pragma unroll
                    for (int k = 0; k < 3; ++k) rows[j * W + 9 + k] = p[k] - A.pw0[k];
            }
            __syncthreads();
            if (acc < nacc) {
                if (MODE == kEpnpPassPc) {
                    for (int j = 0; j < tn; ++j) s += rows[j * W + acc];
                } else {
                    const int a = 3 * (acc / 9) + (acc % 9) / 3, b = 9 + acc % 3;
                    for (int j = 0; j < tn; ++j) s += rows[j * W + a] * rows[j * W + b];
                }
            }
        } else {
            for (int w = threadIdx.x; w < tn * nacc; w += 256) {
                const int j = w / nacc, a = w - j * nacc;
                double t[2];
                epnp_pass_term<MODE>(pw, us, A, t0 + j, a, t);
                term[j * nacc + a] = t[0];
            }
            __syncthreads();
            if (acc < nacc)
                for (int j = 0; j < tn; ++j) s += term[j * nacc + acc];
        }
        __syncthreads();
    }
    if (acc < nacc) part[(size_t)acc * nblk + blk] = s;
}

// ---- launchers --------------------------------------------------------------------------------
static PnpCamera to_cam(const double* cam8) {
    PnpCamera c;
    c.fx = cam8[0]; c.fy = cam8[1]; c.cx = cam8[2]; c.cy = cam8[3];
    c.k1 = cam8[4]; c.k2 = cam8[5]; c.p1 = cam8[6]; c.p2 = cam8[7];
    return c;
}

void launch_pnp_pack(const double* d_img, const double* d_world, int N, void* d_pts, hipStream_t s) {
    if (N <= 0) return;
    hipLaunchKernelGGL(mcv_pnp_pack, dim3((N + 255) / 256), dim3(256), 0, s, d_img, d_world, N, (PnpPoint*)d_pts);
}

void launch_pnp_generate(const void* d_pts, int N, const double* cam8, Sampler smp, int64_t hypBegin, int hypCount,
                         bool epnp, void* d_models, int* d_counts, double* d_epnpScratch, hipStream_t s, bool fast) {
    if (!epnp) {
        hipLaunchKernelGGL(mcv_pnp_generate, dim3((hypCount + 63) / 64), dim3(64), 0, s, (const PnpPoint*)d_pts, N,
                           to_cam(cam8), smp, hypBegin, hypCount, (PnpPose*)d_models, d_counts, fast);
        return;
    }
    // sub-ranges of at most kEpnpPiece hypotheses reuse one scratch of kEpnpPiece x kEpnpSplitDoubles
    // doubles (2.4 GB at the 2^20 piece: one piece per chunk measured 2.3 % faster than 2^18 pieces of
    // 610 MB, kernels.h; the footprint is documented in INTEGRATION.md §5)
    const PnpCamera cam = to_cam(cam8);
    const int piece = std::min(hypCount, kEpnpPiece);
    const int64_t S = piece;
    const EpnpSplit X{d_epnpScratch, d_epnpScratch + kMtmSums * S, d_epnpScratch + (kMtmSums + kEpnpCtx) * S,
                      d_epnpScratch + (kMtmSums + kEpnpCtx + 144) * S, S};
    for (int off = 0; off < hypCount; off += piece) {
        const int n = std::min(piece, hypCount - off);
        int* cnt = d_counts + off;
        PnpPose* mdl = (PnpPose*)d_models + off;
        hipLaunchKernelGGL(mcv_epnp_split_mtm, dim3((n + 255) / 256), dim3(256), 0, s, (const PnpPoint*)d_pts, N, cam,
                           smp, hypBegin + off, n, X, cnt);
        hipLaunchKernelGGL(mcv_epnp_split_sweeps, dim3((n + 63) / 64), dim3(64), 0, s, X, (const int*)cnt, n);
        hipLaunchKernelGGL(mcv_epnp_split_tail, dim3((n + 255) / 256), dim3(256), 0, s, X, (const int*)cnt, n);
        hipLaunchKernelGGL(mcv_epnp_split_betas, dim3((n + 63) / 64), dim3(64), 0, s, X, (const int*)cnt, n);
        hipLaunchKernelGGL(mcv_epnp_split_pose, dim3((n + 255) / 256), dim3(256), 0, s, cam, X, mdl, (const int*)cnt, n);
    }
}

// Grid of a pose-wave x point-chunk sweep: waves x chunks >= ~8 waves per SIMD, chunks >= 2048
// points, chunk a multiple of `align`.
static void pnp_verify_grid(int N, int hypCount, int K, int align, dim3& grid, int& chunk) {
    const int waves = (hypCount + K - 1) / K;
    int chunks = (8192 + waves - 1) / waves;
    const int maxChunks = (N + 2047) / 2048;
    if (chunks > maxChunks) chunks = maxChunks;
    if (chunks < 1) chunks = 1;
    chunk = (N + chunks - 1) / chunks;
    chunk = (chunk + align - 1) / align * align;
    chunks = (N + chunk - 1) / chunk;
    if (chunks < 1) chunks = 1;
    grid = dim3((waves + 3) / 4, chunks);
}

template <int K>
static void launch_pnp_verify_k(const void* d_pts, int N, const double* cam8, const void* d_models, int* d_counts,
                                int hypCount, float thr2, bool fused, hipStream_t s) {
    dim3 grid;
    int chunk;
    pnp_verify_grid(N, hypCount, K, 64, grid, chunk);
    const PnpPoint* p = (const PnpPoint*)d_pts;
    const PnpPose* m = (const PnpPose*)d_models;
    if (fused)
        hipLaunchKernelGGL((mcv_pnp_verify<K, true>), grid, dim3(256), 0, s, p, N, chunk, to_cam(cam8), m, d_counts,
                           hypCount, thr2);
    else
        hipLaunchKernelGGL((mcv_pnp_verify<K, false>), grid, dim3(256), 0, s, p, N, chunk, to_cam(cam8), m, d_counts,
                           hypCount, thr2);
}

template <int K>
static void launch_pnp_verify_pk_k(const void* d_pts, int N, const double* cam8, const PnpPkCam& pc,
                                   const void* d_models, int* d_counts, int hypCount, float thr2, bool fused,
                                   const double* d_ext, const float* d_pairs, hipStream_t s) {
    dim3 grid;
    int chunk;
    pnp_verify_grid(N, hypCount, K, 128, grid, chunk);
    // the per-lane log of undecided (point, pose) lanes needs (point - p0) << 3 in 32 bits; a larger
    // chunk takes the trip log (a whole fp64 trip per undecided (trip, pose))
    if (chunk < (1 << 28))
        hipLaunchKernelGGL((mcv_pnp_verify_pk<K, 5, true>), grid, dim3(256), 0, s, (const PnpPoint*)d_pts, N,
                           chunk, to_cam(cam8), pc, (const PnpPose*)d_models, d_counts, hypCount, thr2, fused, d_ext,
                           d_pairs);
    else
        hipLaunchKernelGGL((mcv_pnp_verify_pk<K, 3, false>), grid, dim3(256), 0, s, (const PnpPoint*)d_pts, N, chunk,
                           to_cam(cam8), pc, (const PnpPose*)d_models, d_counts, hypCount, thr2, fused, d_ext,
                           d_pairs);
}

void launch_pnp_extent(const void* d_pts, int N, double* d_ext, float* d_pairs, hipStream_t s) {
    (void)hipMemsetAsync(d_ext, 0, 3 * sizeof(double), s);   // errors surface at the caller's hipGetLastError
    if (N <= 0) return;
    int blocks = (N + 255) / 256;
    if (blocks > 256) blocks = 256;
    hipLaunchKernelGGL(mcv_pnp_extent, dim3(blocks), dim3(256), 0, s, (const PnpPoint*)d_pts, N,
                       (unsigned long long*)d_ext, d_pairs);
}

// The certified packed-fp32 sweep (kVerifyPnpPosesPerWave poses per wave); the all-fp64 sweep when the
// camera / threshold leaves the bound's domain. d_ext = launch_pnp_extent's output.
void launch_pnp_verify(const void* d_pts, int N, const double* cam8, const void* d_models, int* d_counts, int hypCount,
                       float thr2, bool fused, const double* d_ext, const float* d_pairs, hipStream_t s) {
    const PnpPkCam pc = pnp_pk_cam_host(cam8, thr2);
    if (pc.ok && d_ext && d_pairs)
        launch_pnp_verify_pk_k<kVerifyPnpPosesPerWave>(d_pts, N, cam8, pc, d_models, d_counts, hypCount, thr2, fused,
                                                       d_ext, d_pairs, s);
    else
        launch_pnp_verify_k<kVerifyPnpPosesPerWave>(d_pts, N, cam8, d_models, d_counts, hypCount, thr2, fused, s);
}

void launch_pnp_one(const void* d_pts, int N, const double* cam8, Sampler smp, int64_t hyp, bool epnp,
                    PnpOneOut* d_out, hipStream_t s, bool fast) {
    hipLaunchKernelGGL(mcv_pnp_one, dim3(1), dim3(64), 0, s, (const PnpPoint*)d_pts, N, to_cam(cam8), smp, hyp, epnp,
                       fast, d_out);
}

void launch_pnp_solve5(const void* d_pts, const double* cam8, PnpOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_pnp_solve5, dim3(1), dim3(64), 0, s, (const PnpPoint*)d_pts, to_cam(cam8), d_out);
}

void launch_mask_compact(const uint8_t* d_mask, int N, int* d_idx, int* d_count, hipStream_t s) {
    hipLaunchKernelGGL(mcv_mask_compact, dim3(1), dim3(1024), 0, s, d_mask, N, d_idx, d_count);
}

// d_n applies to the fp32 points (the inlier solve); the fp64 form always takes n.
void launch_epnp_prep(const void* d_pts, const int* d_idx, const double* d_img, const double* d_world, int n,
                      const double* cam8, double* d_pw, double* d_us, hipStream_t s, bool normalized, const int* d_n) {
    if (n <= 0) return;
    if (d_pts)
        hipLaunchKernelGGL(mcv_epnp_prep_f32, dim3((n + 255) / 256), dim3(256), 0, s, (const PnpPoint*)d_pts, d_idx, n,
                           to_cam(cam8), d_pw, d_us, d_n);
    else
        hipLaunchKernelGGL(mcv_epnp_prep_f64, dim3((n + 255) / 256), dim3(256), 0, s, d_img, d_world, n, to_cam(cam8),
                           d_pw, d_us, normalized);
}

void launch_epnp_pass(int mode, const double* d_pw, const double* d_us, int n, const EpnpPassArgs& a, int nacc,
                      double* d_part, hipStream_t s, const int* d_n, const double* d_prev) {
    if (d_prev && mode != kEpnpPassPw0 && mode != kEpnpPassAbt) d_prev = nullptr;   // only these take means
    const int nblk = (n + kEpnpBlock - 1) / kEpnpBlock;
    if (nblk <= 0) return;
    const dim3 grid(nblk), block(256);   // nacc <= 78 accumulators, one lane each
    switch (mode) {
        case kEpnpPassSumPw: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassSumPw>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        case kEpnpPassPw0: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassPw0>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        case kEpnpPassMtm: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassMtm>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        case kEpnpPassPc: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassPc>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        case kEpnpPassAbt: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassAbt>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        case kEpnpPassSqp: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassSqp>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        case kEpnpPassSqpDepth: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassSqpDepth>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev); break;
        default: hipLaunchKernelGGL(mcv_epnp_pass<kEpnpPassReproj>, grid, block, 0, s, d_pw, d_us, n, a, nacc, nblk, d_part, d_n, d_prev);
    }
}

void launch_pnp_solve4(const void* d_pts, const double* cam8, PnpOneOut* d_out, hipStream_t s, bool fast) {
    hipLaunchKernelGGL(mcv_pnp_solve4, dim3(1), dim3(64), 0, s, (const PnpPoint*)d_pts, to_cam(cam8), fast, d_out);
}

void launch_pnp_mask(const void* d_pts, int N, const double* cam8, const double* R9, const double* t3, float thr2,
                     bool fused, uint8_t* d_mask, int* d_count, hipStream_t s) {
    PnpPose m;
    for (int k = 0; k < 9; ++k) m.R[k] = R9[k];
    for (int k = 0; k < 3; ++k) m.t[k] = t3[k];
    hipLaunchKernelGGL(mcv_pnp_mask, dim3((N + 255) / 256), dim3(256), 0, s, (const PnpPoint*)d_pts, N, to_cam(cam8),
                       m, (const PnpPose*)nullptr, thr2, fused, d_mask, d_count);
}

void launch_pnp_mask_dev(const void* d_pts, int N, const double* cam8, const void* d_pose, float thr2, bool fused,
                         uint8_t* d_mask, int* d_count, hipStream_t s) {
    PnpPose m{};
    hipLaunchKernelGGL(mcv_pnp_mask, dim3((N + 255) / 256), dim3(256), 0, s, (const PnpPoint*)d_pts, N, to_cam(cam8),
                       m, (const PnpPose*)d_pose, thr2, fused, d_mask, d_count);
}

void launch_pnp_ap3p(const Ap3pIn& in, Ap3pOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_pnp_ap3p, dim3(1), dim3(64), 0, s, in, d_out);
}

void pnp_reduce_lm(const void* d_pts, int N, const uint8_t* d_mask, const double* cam8, const double* R9,
                   const double* t3, const double* dR27, bool wantJ, double* d_part, double* d_out, hipStream_t s) {
    OpPnpLM op;
    op.pts = (const PnpPoint*)d_pts;
    op.mask = d_mask;
    op.c = to_cam(cam8);
    for (int k = 0; k < 9; ++k) op.R[k] = R9[k];
    for (int k = 0; k < 3; ++k) op.t[k] = t3[k];
    for (int k = 0; k < 27; ++k) op.dR[k] = dR27 ? dR27[k] : 0.0;
    op.wantJ = wantJ;
    run_reduce<28>(N, op, d_part, d_out, s);
}

void pnp_reduce_vvs(const void* d_pts, int N, const uint8_t* d_mask, const double* cam8, const double* R9,
                    const double* t3, double* d_part, double* d_out, hipStream_t s) {
    OpPnpVVS op;
    op.pts = (const PnpPoint*)d_pts;
    op.mask = d_mask;
    op.c = to_cam(cam8);
    for (int k = 0; k < 9; ++k) op.R[k] = R9[k];
    for (int k = 0; k < 3; ++k) op.t[k] = t3[k];
    run_reduce<28>(N, op, d_part, d_out, s);
}

}  // namespace mcv
