// reduce.h — deterministic (fixed-order) fp64 block reductions used by the refit / LM passes.
// A pass maps every correspondence to V partial sums (functor Op), reduces them per workgroup
// (wave shuffles, then LDS across the 4 waves) into partials[block][V]; a second one-block
// pass sums the partials in block order. No atomics: results are bitwise reproducible run to run.
#pragma once

#include <hip/hip_runtime.h>
#include "kernels.h"

namespace mcv {

static const int kReduceThreads = 256;
static const int kReduceMaxBlocks = kReduceMaxBlocksHost;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Reduce acc[V] over the workgroup; thread 0 of the block gets the totals in out[V].
template <int V>
__device__ __forceinline__ void block_sum(double (&acc)[V], double* __restrict__ out) {
    __shared__ double sh[kReduceThreads / 64][V];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int v = 0; v < V; ++v) {
        const double s = wave_sum(acc[v]);
        if (lane == 0) sh[wave][v] = s;
    }
    __syncthreads();
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
        double s = 0;
#pragma unroll
        for (int w = 0; w < kReduceThreads / 64; ++w) s += sh[w][v];
        out[v] = s;
    }
}

template <int V, class Op>
__global__ __launch_bounds__(kReduceThreads) void reduce_pass(int n, Op op, double* __restrict__ partials) {
    double acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0;
    for (int i = blockIdx.x * kReduceThreads + threadIdx.x; i < n; i += gridDim.x * kReduceThreads) op(i, acc);
    block_sum<V>(acc, partials + (size_t)blockIdx.x * V);
}

template <int V>
__global__ __launch_bounds__(kReduceThreads) void reduce_final(int nblocks, const double* __restrict__ partials,
                                                              double* __restrict__ out) {
    double acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0;
    for (int b = threadIdx.x; b < nblocks; b += kReduceThreads) {
#pragma unroll
        for (int v = 0; v < V; ++v) acc[v] += partials[(size_t)b * V + v];
    }
    block_sum<V>(acc, out);
}

inline int reduce_blocks(int n) {
    int b = (n + kReduceThreads - 1) / kReduceThreads;
    if (b < 1) b = 1;
    if (b > kReduceMaxBlocks) b = kReduceMaxBlocks;
    return b;
}

// Run a two-stage reduction on `stream`; result lands in d_out[V] (device).
template <int V, class Op>
inline void run_reduce(int n, const Op& op, double* d_partials, double* d_out, hipStream_t stream) {
    const int nb = reduce_blocks(n);
    hipLaunchKernelGGL((reduce_pass<V, Op>), dim3(nb), dim3(kReduceThreads), 0, stream, n, op, d_partials);
    hipLaunchKernelGGL((reduce_final<V>), dim3(1), dim3(kReduceThreads), 0, stream, nb, d_partials, d_out);
}

}  // namespace mcv
