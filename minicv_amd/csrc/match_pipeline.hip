// match_pipeline.hip — device-resident hand-off from descriptor matching to RANSAC (SURVEY §8f
// row f3): the knn-2 matcher's outputs are filtered (Lowe ratio, mutual check, max distance) and
// compacted in query order on the GPU, and the surviving pairs' keypoint coordinates are gathered
// straight into the float4 correspondence layout the RANSAC sweep reads — no host round trip
// between the two kernels (the reference's caller copies DetectorResult arrays to managed memory
// and back, OpenCV.fs:481-524).
//
//   mcv_match_filter   keep[i] for query i
//   mcv_block_count    per-256 block counts of keep
//   mcv_scan_blocks    exclusive scan of the block counts (one block, fixed order)
//   mcv_match_scatter  order-preserving compaction: pairs, distances, float4 {xa, ya, xb, yb}
#include <hip/hip_runtime.h>
#include <climits>
#include <cmath>
#include "kernels.h"

namespace mcv {

__global__ __launch_bounds__(256) void mcv_match_filter(const int* __restrict__ idx, const int* __restrict__ di1,
                                                        const int* __restrict__ di2, const float* __restrict__ df1,
                                                        const float* __restrict__ df2,
                                                        const int* __restrict__ idxBack, int nq, float ratio,
                                                        float maxDist, uint8_t* __restrict__ keep) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= nq) return;
    const int j = idx[i];
    bool k = j >= 0;
    float d1, d2;
    if (di1) {
        d1 = (float)di1[i];
        d2 = di2[i] == INT_MAX ? INFINITY : (float)di2[i];
    } else {
        d1 = df1[i];
        d2 = df2[i];
    }
    if (ratio > 0) k = k && d1 < ratio * d2;
    if (maxDist > 0) k = k && d1 <= maxDist;
    if (idxBack && j >= 0) k = k && idxBack[j] == i;
    keep[i] = k ? 1 : 0;
}

__global__ __launch_bounds__(256) void mcv_block_count(const uint8_t* __restrict__ keep, int n, int* __restrict__ cnt) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool k = i < n && keep[i];
    const uint64_t b = __ballot(k);
    __shared__ int w[4];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = (int)__popcll(b);
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// Exclusive scan of nb block counts in one block (sequential chunks of 1024, fixed order);
// off[nb] = total.
__global__ __launch_bounds__(1024) void mcv_scan_blocks(const int* __restrict__ cnt, int nb, int* __restrict__ off) {
    __shared__ int sh[1024];
    __shared__ int carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < nb; base += 1024) {
        const int i = base + threadIdx.x;
        const int v = i < nb ? cnt[i] : 0;
        sh[threadIdx.x] = v;
        __syncthreads();
        for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan
            const int t = threadIdx.x >= o ? sh[threadIdx.x - o] : 0;
            __syncthreads();
            sh[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < nb) off[i] = carry + sh[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += sh[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) off[nb] = carry;
}

__global__ __launch_bounds__(256) void mcv_match_scatter(const uint8_t* __restrict__ keep, const int* __restrict__ idx,
                                                         const int* __restrict__ di1, const float* __restrict__ df1,
                                                         const int* __restrict__ off, int n,
                                                         const uint8_t* __restrict__ kpA,
                                                         const uint8_t* __restrict__ kpB, int kpStride,
                                                         int* __restrict__ pairs, float* __restrict__ dist,
                                                         float4* __restrict__ pts) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool k = i < n && keep[i];
    const uint64_t b = __ballot(k);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    __shared__ int w[4];
    if (lane == 0) w[wv] = (int)__popcll(b);
    __syncthreads();
    int base = off[blockIdx.x];
    for (int q = 0; q < wv; ++q) base += w[q];
    if (!k) return;
    const int pos = base + (int)__popcll(b & ((1ull << lane) - 1));
    const int j = idx[i];
    pairs[2 * pos] = i;
    pairs[2 * pos + 1] = j;
    if (dist) dist[pos] = di1 ? (float)di1[i] : df1[i];
    const float* pa = (const float*)(kpA + (size_t)i * kpStride);
    const float* pb = (const float*)(kpB + (size_t)j * kpStride);
    pts[pos] = make_float4(pa[0], pa[1], pb[0], pb[1]);
}

// Filter + compaction; returns nothing (the total lands in d_off[nblocks]).
void launch_match_compact(const int* d_idx, const int* d_di1, const int* d_di2, const float* d_df1,
                          const float* d_df2, const int* d_idxBack, int nq, float ratio, float maxDist,
                          const uint8_t* d_kpA, const uint8_t* d_kpB, int kpStride, uint8_t* d_keep, int* d_cnt,
                          int* d_off, int* d_pairs, float* d_dist, float* d_pts4, hipStream_t s) {
    const int nb = (nq + 255) / 256;
    hipLaunchKernelGGL(mcv_match_filter, dim3(nb), dim3(256), 0, s, d_idx, d_di1, d_di2, d_df1, d_df2, d_idxBack, nq,
                       ratio, maxDist, d_keep);
    hipLaunchKernelGGL(mcv_block_count, dim3(nb), dim3(256), 0, s, d_keep, nq, d_cnt);
    hipLaunchKernelGGL(mcv_scan_blocks, dim3(1), dim3(1024), 0, s, d_cnt, nb, d_off);
    hipLaunchKernelGGL(mcv_match_scatter, dim3(nb), dim3(256), 0, s, d_keep, d_idx, d_di1, d_df1, d_off, nq, d_kpA,
                       d_kpB, kpStride, d_pairs, d_dist, (float4*)d_pts4);
}

}  // namespace mcv
