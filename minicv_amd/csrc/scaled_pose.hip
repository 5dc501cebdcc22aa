// scaled_pose.hip — gfx950 kernels of CameraPose.findScaled (CameraPose.fs:39-134).
//
//   mcv_scaled_pack        AoS V3d world points + V2d observations -> SoA fp64 (5 coalesced streams)
//   mcv_scaled_candidates  lane per observation: the two candidate scales (or "skipped")
//   mcv_scaled_costs<K>    the O(N^2) verify: a wave owns K candidate scales (their dstCam(s)
//                          locations are wave-uniform: SGPRs), its 64 lanes stream all N observations,
//                          project them (Camera.project1) and accumulate sum |c - obs|^2 and the
//                          visible count in fp64; a fixed-order wave tree gives each candidate's
//                          avgReprojectionError (+inf when nothing is visible).
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

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ int wave_sum_i32(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <int K>
__global__ __launch_bounds__(256) void mcv_scaled_costs(ScaledSetup S, const double* __restrict__ soa, int N,
                                                        const double* __restrict__ scales,
                                                        const uint8_t* __restrict__ used, int nCand,
                                                        double* __restrict__ costs) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int c0 = wave * K;
    if (c0 >= nCand) return;
    double loc[K][3];
    bool live = false;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int c = c0 + k < nCand ? c0 + k : c0;
        scaled_location(S, scales[c], loc[k]);
        live = live || (c0 + k < nCand && used[(c0 + k) >> 1]);
    }
    if (!live) {   // every candidate of this wave was skipped by the reference loop
        if (lane < K && c0 + lane < nCand) costs[c0 + lane] = __builtin_inf();
        return;
    }
    double sum[K];
    int cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        sum[k] = 0.0;
        cnt[k] = 0;
    }
    const double* wx = soa;
    const double* wy = soa + N;
    const double* wz = soa + 2 * (size_t)N;
    const double* ox = soa + 3 * (size_t)N;
    const double* oy = soa + 4 * (size_t)N;
    for (int i = lane; i < N; i += 64) {
        const double x = wx[i], y = wy[i], z = wz[i], u = ox[i], v = oy[i];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double e;
            const bool vis = scaled_term(S, loc[k], x, y, z, u, v, e);
            sum[k] += vis ? e : 0.0;   // select, not a branch (an invisible e may be NaN / inf)
            cnt[k] += vis ? 1 : 0;
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double s = wave_sum_f64(sum[k]);
        const int n = wave_sum_i32(cnt[k]);
        const int c = c0 + k;
        if (lane == 0 && c < nCand)
            costs[c] = (!used[c >> 1] || n == 0) ? __builtin_inf() : s / (double)n;
    }
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

static const int kScaledPerWave = 8;

void launch_scaled(const ScaledSetup& S, const double* d_w3, const double* d_o2, int N, double* d_soa,
                   double* d_scales, uint8_t* d_used, double* d_costs, long long* d_out, hipStream_t s) {
    const int nCand = 2 * N;
    hipLaunchKernelGGL(mcv_scaled_pack, dim3((N + 255) / 256), dim3(256), 0, s, d_w3, d_o2, N, d_soa);
    hipLaunchKernelGGL(mcv_scaled_candidates, dim3((N + 255) / 256), dim3(256), 0, s, S, d_soa, N, d_scales,
                       d_used);
    const int waves = (nCand + kScaledPerWave - 1) / kScaledPerWave;
    {
        ProfScope ps("scaled_costs", s);
        hipLaunchKernelGGL((mcv_scaled_costs<kScaledPerWave>), dim3((waves + 3) / 4), dim3(256), 0, s, S, d_soa, N,
                           d_scales, d_used, nCand, d_costs);
    }
    hipLaunchKernelGGL(mcv_scaled_best, dim3(1), dim3(1024), 0, s, d_costs, d_used, nCand, d_out);
}

}  // namespace mcv
