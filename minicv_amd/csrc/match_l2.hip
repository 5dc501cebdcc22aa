// match_l2.hip — brute-force L2 matcher posed as an fp32 GEMM on the matrix cores
// (cv::BFMatcher(NORM_L2).knnMatch(k = 2) semantics [ext: OpenCV features2d]; descriptor layout
// = DetectorResult / ImageFeatures row-major [n][dim] float, MiniCVNative.h:22-28, OpenCV.fs:263-281).
//
//   |q - t|^2 = |q|^2 + |t|^2 - 2 q.t ; argmin over t needs only s(t) = |t|^2 - 2 q.t.
//
// mcv_l2_mfma<DP>: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD = the fp32 peak).
//   A = 32 train rows of a tile (from LDS), B = 32 queries (resident in VGPRs for the whole
//   kernel), D[i][j] = t_i . q_j. The 32x32 accumulator puts one query on each lane (col = lane & 31)
//   and 16 train rows in its registers, so the top-2 epilogue is lane-local: no cross-lane
//   reduction per tile, one shuffle at the end to merge the two lane halves.
//   Operands use a parity-split row layout (even dims, then odd dims): lane half h takes dims
//   2s + h, so 4 consecutive k-steps are one 16-byte read (ds_read_b128 / global_load_dwordx4).
//   Train tiles are double-buffered in LDS (row stride DP + 4 floats: conflict-free b128 reads),
//   register-staged: the next tile's global loads are issued before this tile's MFMAs and written
//   to LDS after them; one barrier per tile.
//   Grid = (query blocks of 128) x (train chunks); a merge kernel folds the per-chunk top-2s.
// Ties: scores compared as (score, train index) pairs — lowest index wins, like BFMatcher's scan.
#include "kernels.h"
#include "mcv_runtime.h"
#include "plan.h"
#include <cmath>

namespace mcv {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct L2Part { float b1, b2; int i1, i2; };

__device__ __forceinline__ bool lex_less(float a, int ia, float b, int ib) {
    return (a < b) | ((a == b) & ((unsigned)ia < (unsigned)ib));   // idx -1 sorts last
}

// Branchless top-2 insertion (selects, no divergent control flow in the epilogue).
__device__ __forceinline__ void top2_push(float& b1, int& i1, float& b2, int& i2, float s, int i) {
    const bool c1 = lex_less(s, i, b1, i1);
    const bool c2 = lex_less(s, i, b2, i2);
    const float nb2 = c1 ? b1 : (c2 ? s : b2);
    const int ni2 = c1 ? i1 : (c2 ? i : i2);
    b1 = c1 ? s : b1;
    i1 = c1 ? i : i1;
    b2 = nb2;
    i2 = ni2;
}

// Parity-split, zero-padded copy [nPad][DP] + squared norms (fp32 FMA chain in dim order).
__global__ void mcv_l2_prep(const float* __restrict__ src, int n, int dim, int DP, int nPad, float* __restrict__ dst,
                            float* __restrict__ norms, float padNorm) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nPad) return;
    float acc = 0.f;
    for (int k = lane; k < DP; k += 64) {
        const float v = (r < n && k < dim) ? src[(size_t)r * dim + k] : 0.f;
        dst[(size_t)r * DP + (k & 1) * (DP / 2) + (k >> 1)] = v;
    }
    if (lane == 0) {
        if (r < n) {
            for (int k = 0; k < dim; ++k) {
                const float v = src[(size_t)r * dim + k];
                acc = fmaf(v, v, acc);
            }
        }
        norms[r] = r < n ? acc : padNorm;
    }
}

template <int DP>
__device__ __forceinline__ void l2_gload(const float* __restrict__ tp, const float* __restrict__ tnorm, int tile,
                                         float4 (&stg)[DP / 32], float& nstg) {
    constexpr int ROWS_PER_PASS = 256 / (DP / 4);
    const int srow = threadIdx.x / (DP / 4), sc4 = threadIdx.x % (DP / 4);
#pragma unroll
    for (int r = 0; r < DP / 32; ++r)
        stg[r] = reinterpret_cast<const float4*>(tp + (size_t)(tile * 32 + srow + r * ROWS_PER_PASS) * DP)[sc4];
    if (threadIdx.x < 32) nstg = tnorm[tile * 32 + threadIdx.x];
}

template <int DP>
__device__ __forceinline__ void l2_lstore(float* __restrict__ lds, float* __restrict__ lnorm,
                                          const float4 (&stg)[DP / 32], float nstg) {
    constexpr int ROWF = DP + 4;
    constexpr int ROWS_PER_PASS = 256 / (DP / 4);
    const int srow = threadIdx.x / (DP / 4), sc4 = threadIdx.x % (DP / 4);
#pragma unroll
    for (int r = 0; r < DP / 32; ++r)
        *reinterpret_cast<float4*>(&lds[(srow + r * ROWS_PER_PASS) * ROWF + sc4 * 4]) = stg[r];
    if (threadIdx.x < 32) lnorm[threadIdx.x] = nstg;
}

template <int DP>
__global__ __launch_bounds__(256, 2) void mcv_l2_mfma(const float* __restrict__ qp, const float* __restrict__ tp,
                                                     const float* __restrict__ tnorm, int ntTiles,
                                                     int tilesPerChunk, int nqPad, L2Part* __restrict__ part) {
    constexpr int KS = DP / 2;          // MFMA k-steps (2 dims each)
    constexpr int ROWF = DP + 4;        // padded LDS row, floats
    constexpr int PER = DP / 32;        // float4 staging loads per thread per tile (32 rows x DP)
    __shared__ __attribute__((aligned(16))) float lds[2][32 * ROWF];
    __shared__ float lnorm[2][32];

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int q0 = (blockIdx.x * 4 + wave) * 32;

    // B fragments: query q0 + col, dims 2s + h  (parity-split row: offset h * KS + s)
    float b[KS];
    {
        const float4* qrow = reinterpret_cast<const float4*>(qp + (size_t)(q0 + col) * DP + h * KS);
#pragma unroll
        for (int s4 = 0; s4 < KS / 4; ++s4) {
            const float4 v = qrow[s4];
            b[4 * s4 + 0] = v.x; b[4 * s4 + 1] = v.y; b[4 * s4 + 2] = v.z; b[4 * s4 + 3] = v.w;
        }
    }

    const int tBegin = blockIdx.y * tilesPerChunk;
    const int tEnd = min(tBegin + tilesPerChunk, ntTiles);
    float b1 = INFINITY, b2 = INFINITY;
    int i1 = -1, i2 = -1;

    // Register staging of the next train tile (32 rows x DP floats = PER float4 per thread).
    float4 stg[PER];
    float nstg = 0.f;

    if (tBegin < tEnd) {
        l2_gload<DP>(tp, tnorm, tBegin, stg, nstg);
        l2_lstore<DP>(lds[0], lnorm[0], stg, nstg);
    }
    __syncthreads();
    for (int t = tBegin; t < tEnd; ++t) {
        const int buf = (t - tBegin) & 1;
        const bool more = t + 1 < tEnd;
        // next tile's loads in flight under this tile's MFMAs (the last trip reloads its own tile
        // into the idle buffer: no branch around the staging registers)
        l2_gload<DP>(tp, tnorm, more ? t + 1 : t, stg, nstg);
        floatx16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        const float* arow = &lds[buf][col * ROWF + h * KS];
#pragma unroll
        for (int s4 = 0; s4 < KS / 4; ++s4) {
            const float4 a = *reinterpret_cast<const float4*>(arow + 4 * s4);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[4 * s4 + 0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[4 * s4 + 1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[4 * s4 + 2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[4 * s4 + 3], acc, 0, 0, 0);
        }
        // epilogue: lane = query col, register r = train row (r&3) + 8(r>>2) + 4h, rows ascending
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
            const float s = fmaf(-2.f, acc[r], lnorm[buf][row]);
            top2_push(b1, i1, b2, i2, s, t * 32 + row);
        }
        l2_lstore<DP>(lds[buf ^ 1], lnorm[buf ^ 1], stg, nstg);
        __syncthreads();
    }
    // merge the two lane halves that hold the same query
    const float ob1 = __shfl_xor(b1, 32, 64), ob2 = __shfl_xor(b2, 32, 64);
    const int oi1 = __shfl_xor(i1, 32, 64), oi2 = __shfl_xor(i2, 32, 64);
    if (h == 0) {
        top2_push(b1, i1, b2, i2, ob1, oi1);
        top2_push(b1, i1, b2, i2, ob2, oi2);
        L2Part p;
        p.b1 = b1; p.b2 = b2; p.i1 = i1; p.i2 = i2;
        part[(size_t)blockIdx.y * nqPad + q0 + col] = p;
    }
}

__global__ void mcv_l2_merge(const L2Part* __restrict__ part, int nq, int nqPad, int nchunks,
                             const float* __restrict__ qnorm, int* __restrict__ idx, float* __restrict__ dist,
                             int* __restrict__ idx2, float* __restrict__ dist2) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    float b1 = INFINITY, b2 = INFINITY;
    int i1 = -1, i2 = -1;
    for (int c = 0; c < nchunks; ++c) {
        const L2Part p = part[(size_t)c * nqPad + q];
        top2_push(b1, i1, b2, i2, p.b1, p.i1);
        top2_push(b1, i1, b2, i2, p.b2, p.i2);
    }
    const float qn = qnorm[q];
    idx[q] = i1;
    dist[q] = i1 >= 0 ? sqrtf(fmaxf(qn + b1, 0.f)) : INFINITY;
    if (idx2) idx2[q] = i2;
    if (dist2) dist2[q] = i2 >= 0 ? sqrtf(fmaxf(qn + b2, 0.f)) : INFINITY;
}

struct L2Work {
    DevBuf<float> qp, tp, qn, tn;
    DevBuf<L2Part> part;
};

int launch_match_l2(const float* d_q, int nq, const float* d_t, int nt, int dim, int* d_idx, float* d_dist,
                    int* d_idx2, float* d_dist2, hipStream_t s) {
    if (dim <= 0 || dim > 256) fail("cvMatchL2: dim %d outside [1, 256]", dim);
    if (nq <= 0) return 0;
    thread_local L2Work wk;
    const int DP = dim <= 32 ? 32 : dim <= 64 ? 64 : dim <= 128 ? 128 : 256;
    const int nqPad = (nq + 127) / 128 * 128;
    const int ntPad = nt > 0 ? (nt + 31) / 32 * 32 : 32;
    const int ntTiles = ntPad / 32;
    wk.qp.ensure((size_t)nqPad * DP);
    wk.tp.ensure((size_t)ntPad * DP);
    wk.qn.ensure(nqPad);
    wk.tn.ensure(ntPad);
    hipLaunchKernelGGL(mcv_l2_prep, dim3((nqPad + 3) / 4), dim3(256), 0, s, d_q, nq, dim, DP, nqPad, wk.qp.p, wk.qn.p,
                       0.f);
    // padding rows get a NaN norm: their scores are NaN and never enter a top-2
    hipLaunchKernelGGL(mcv_l2_prep, dim3((ntPad + 3) / 4), dim3(256), 0, s, d_t, nt, dim, DP, ntPad, wk.tp.p, wk.tn.p,
                       __builtin_nanf(""));
    const int qblocks = nqPad / 128;
    int nchunks = (2048 + qblocks - 1) / qblocks;
    if (nchunks > ntTiles) nchunks = ntTiles;
    if (nchunks < 1) nchunks = 1;
    const int tilesPerChunk = (ntTiles + nchunks - 1) / nchunks;
    nchunks = (ntTiles + tilesPerChunk - 1) / tilesPerChunk;
    wk.part.ensure((size_t)nchunks * nqPad);
    dim3 grid(qblocks, nchunks);
    {
        ProfScope ps("l2_mfma", s);
        switch (DP) {
            case 32: hipLaunchKernelGGL((mcv_l2_mfma<32>), grid, dim3(256), 0, s, wk.qp.p, wk.tp.p, wk.tn.p, ntTiles, tilesPerChunk, nqPad, wk.part.p); break;
            case 64: hipLaunchKernelGGL((mcv_l2_mfma<64>), grid, dim3(256), 0, s, wk.qp.p, wk.tp.p, wk.tn.p, ntTiles, tilesPerChunk, nqPad, wk.part.p); break;
            case 128: hipLaunchKernelGGL((mcv_l2_mfma<128>), grid, dim3(256), 0, s, wk.qp.p, wk.tp.p, wk.tn.p, ntTiles, tilesPerChunk, nqPad, wk.part.p); break;
            default: hipLaunchKernelGGL((mcv_l2_mfma<256>), grid, dim3(256), 0, s, wk.qp.p, wk.tp.p, wk.tn.p, ntTiles, tilesPerChunk, nqPad, wk.part.p); break;
        }
    }
    hipLaunchKernelGGL(mcv_l2_merge, dim3((nq + 255) / 256), dim3(256), 0, s, wk.part.p, nq, nqPad, nchunks, wk.qn.p,
                       d_idx, d_dist, d_idx2, d_dist2);
    MCV_HIP(hipGetLastError());
    return nq;
}

}  // namespace mcv
