// scaled_pose.hip — gfx950 kernels of CameraPose.findScaled (CameraPose.fs:39-134).
//
//   mcv_scaled_pack        AoS V3d world points + V2d observations -> SoA fp64 (5 coalesced streams)
//   mcv_scaled_candidates  lane per observation: the two candidate scales (or "skipped")
//   mcv_scaled_costs       the O(N^2) verify: a workgroup owns 64 candidate scales; 4 waves project
//                          double-buffered LDS tiles of observations (Camera.project1) for all of
//                          them while a fifth wave adds the previous tile's terms to each candidate's
//                          running fp64 sum in list order, as the managed loop does:
//                          avgReprojectionError bit for bit (+inf when nothing is visible).
//   mcv_scaled_best        first strictly smaller cost in candidate order: min of (cost bits,
//                          index) over the finite costs (costs are >= 0, so their bit patterns
//                          order like the values), plus the evaluated-candidate count.
//
// Bound: fp64 VALU (2 IEEE divisions + 22 other fp64 ops per (candidate, observation)); the
// 40 N-byte SoA point set streams from L2 (K candidates per load).
#include "hyp_scaled.h"
#include "kernels.h"
#include "plan.h"

namespace mcv {

__global__ __launch_bounds__(256) void mcv_scaled_pack(const double* __restrict__ w3, const double* __restrict__ o2,
                                                       int N, double* __restrict__ soa) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    soa[i] = w3[3 * (size_t)i];
    soa[(size_t)N + i] = w3[3 * (size_t)i + 1];
    soa[2 * (size_t)N + i] = w3[3 * (size_t)i + 2];
    soa[3 * (size_t)N + i] = o2[2 * (size_t)i];
    soa[4 * (size_t)N + i] = o2[2 * (size_t)i + 1];
}

__global__ __launch_bounds__(256) void mcv_scaled_candidates(ScaledSetup S, const double* __restrict__ soa, int N,
                                                             double* __restrict__ scales,
                                                             uint8_t* __restrict__ used) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    double sx = __builtin_nan(""), sy = __builtin_nan("");
    const bool ok = scaled_candidate(S, soa[i], soa[(size_t)N + i], soa[2 * (size_t)N + i], soa[3 * (size_t)N + i],
                                     soa[4 * (size_t)N + i], sx, sy);
    scales[2 * (size_t)i] = ok ? sx : __builtin_nan("");
    scales[2 * (size_t)i + 1] = ok ? sy : __builtin_nan("");
    used[i] = ok ? 1 : 0;
}

// A workgroup owns kScaledCands candidate scales and streams the N observations in tiles of
// kScaledTile. Compute waves 0..7 (lane l = candidate l, its dstCam(s) location in VGPRs) each project
// a contiguous eighth of tile t (observations broadcast from LDS, staged by wave 8) for all the group's
// candidates and park the terms in LDS buffer t % 2 (an invisible observation parks -0.0: adding
// it leaves any running sum unchanged, and a visible term d = dx^2 + dy^2 is never -0.0). Wave 8
// meanwhile adds tile t - 1's terms to each candidate's running fp64 sum in list order —
// avgReprojectionError's `sum <- sum + d` loop (CameraPose.fs:83-91) bit for bit — and counts the
// visible ones; one barrier per tile hands the buffers over.
static const int kScaledCands = 64;
static const int kScaledTile = 32;
static const int kScaledComputeWaves = 8;
static const int kScaledThreads = (kScaledComputeWaves + 1) * 64;

__global__ __launch_bounds__(kScaledThreads) void mcv_scaled_costs(ScaledSetup S, const double* __restrict__ soa,
                                                                   int N, const double* __restrict__ scales,
                                                                   const uint8_t* __restrict__ used, int nCand,
                                                                   double* __restrict__ costs) {
    __shared__ double terms[2][kScaledTile][kScaledCands];
    __shared__ double obs[2][5][kScaledTile];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int c = blockIdx.x * kScaledCands + lane;
    const int cc = c < nCand ? c : nCand - 1;
    double loc[3];
    scaled_location(S, scales[cc], loc);
    const int per = kScaledTile / kScaledComputeWaves;   // observations per compute wave and tile
    const int sw = kScaledComputeWaves;                   // the staging / summing wave
    const int ntiles = (N + kScaledTile - 1) / kScaledTile;
    // the summing wave stages tile t's observations (5 SoA streams) into obs[t % 2]; past N: the last one
    auto stage = [&](int t) {
        if (lane < kScaledTile) {
            const int j0 = t * kScaledTile + lane;
            const int j = j0 < N ? j0 : N - 1;
#pragma unroll
            for (int q = 0; q < 5; ++q) obs[t & 1][q][lane] = soa[(size_t)q * N + j];
        }
    };
    if (wv == sw) stage(0);
    __syncthreads();
    double sum = 0.0;
    int cnt = 0;
    for (int t = 0; t <= ntiles; ++t) {
        if (wv < sw && t < ntiles) {
            double (*buf)[kScaledCands] = terms[t & 1];
            const double (*o)[kScaledTile] = obs[t & 1];
            const int r0 = wv * per;
            const int j0 = t * kScaledTile + r0;
#pragma unroll 4
            for (int k = 0; k < per; ++k) {
                double e;
                const bool vis = scaled_term(S, loc, o[0][r0 + k], o[1][r0 + k], o[2][r0 + k], o[3][r0 + k],
                                             o[4][r0 + k], e);
                buf[r0 + k][lane] = (vis && j0 + k < N) ? e : -0.0;
            }
        }
        if (wv == sw) {
            if (t + 1 < ntiles) stage(t + 1);
            if (t > 0) {
                const double (*buf)[kScaledCands] = terms[(t - 1) & 1];
#pragma unroll 8
                for (int k = 0; k < kScaledTile; ++k) {
                    const double d = buf[k][lane];
                    sum = sum + d;
                    cnt += __double_as_longlong(d) != (long long)0x8000000000000000ull ? 1 : 0;
                }
            }
        }
        __syncthreads();
    }
    if (wv == sw && c < nCand) costs[c] = (!used[c >> 1] || cnt == 0) ? __builtin_inf() : sum / (double)cnt;
}

// out[0] = best candidate index (-1: none), out[1] = number of evaluated candidates.
__global__ __launch_bounds__(1024) void mcv_scaled_best(const double* __restrict__ costs,
                                                        const uint8_t* __restrict__ used, int nCand,
                                                        long long* __restrict__ out) {
    __shared__ unsigned long long sb[16];
    __shared__ int si[16], sn[16];
    const unsigned long long kInfBits = 0x7FF0000000000000ull;
    unsigned long long best = ~0ull;
    int bi = -1, n = 0;
    for (int c = threadIdx.x; c < nCand; c += 1024) {
        if (used[c >> 1]) ++n;
        const unsigned long long b = (unsigned long long)__double_as_longlong(costs[c]);
        // finite, non-negative costs only (+inf never wins: strict <; NaN never compares smaller)
        if (used[c >> 1] && b < kInfBits && (b < best || (b == best && c < bi))) {
            best = b;
            bi = c;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long ob = __shfl_xor(best, off, 64);
        const int oi = __shfl_xor(bi, off, 64);
        n += __shfl_xor(n, off, 64);
        if (oi >= 0 && (ob < best || (ob == best && (bi < 0 || oi < bi)))) {
            best = ob;
            bi = oi;
        }
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        sb[w] = best;
        si[w] = bi;
        sn[w] = n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < 16; ++k) {
            n += sn[k];
            if (si[k] >= 0 && (sb[k] < best || (sb[k] == best && (bi < 0 || si[k] < bi)))) {
                best = sb[k];
                bi = si[k];
            }
        }
        out[0] = bi;
        out[1] = n;
    }
}

void launch_scaled(const ScaledSetup& S, const double* d_w3, const double* d_o2, int N, double* d_soa,
                   double* d_scales, uint8_t* d_used, double* d_costs, long long* d_out, hipStream_t s) {
    const int nCand = 2 * N;
    hipLaunchKernelGGL(mcv_scaled_pack, dim3((N + 255) / 256), dim3(256), 0, s, d_w3, d_o2, N, d_soa);
    hipLaunchKernelGGL(mcv_scaled_candidates, dim3((N + 255) / 256), dim3(256), 0, s, S, d_soa, N, d_scales,
                       d_used);
    {
        ProfScope ps("scaled_costs", s);
        hipLaunchKernelGGL(mcv_scaled_costs, dim3((nCand + kScaledCands - 1) / kScaledCands), dim3(kScaledThreads),
                           0, s, S, d_soa, N, d_scales, d_used, nCand, d_costs);
    }
    hipLaunchKernelGGL(mcv_scaled_best, dim3(1), dim3(1024), 0, s, d_costs, d_used, nCand, d_out);
}

}  // namespace mcv
