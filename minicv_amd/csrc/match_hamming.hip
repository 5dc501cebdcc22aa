// match_hamming.hip — brute-force Hamming matcher (cv::BFMatcher(NORM_HAMMING).knnMatch(k = 2)
// semantics [ext: OpenCV features2d]; descriptor layout = DetectorResult / ImageFeatures
// row-major [n][bytes], MiniCVNative.h:22-28, OpenCV.fs:478-524).
//
// Integer VALU work, not a GEMM: per (query, train) pair W x (v_xor_b32 + v_bcnt_u32_b32) on
// 32-bit words, then a packed-key top-2 update. Layout on the chip:
//   * lane = query: each lane keeps its query's W words in VGPRs;
//   * wave-uniform train index: the train descriptor arrives by scalar loads (SGPRs), so each
//     XOR reads it as its scalar operand — no LDS traffic at all;
//   * the train set is split into S chunks over the grid (>= ~4k waves to fill 256 CUs), each
//     (query-wave, chunk) keeps a top-2 of packed keys key = dist << 22 | trainIdx, so
//     min(key) is "smallest distance, then lowest train index" (BFMatcher's first-minimum rule);
//   * a merge kernel folds the S partial top-2s per query.
#include "kernels.h"
#include "mcv_runtime.h"
#include "plan.h"
#include <climits>

namespace mcv {

static const int kIdxBits = 22;
static const uint32_t kIdxMask = (1u << kIdxBits) - 1;

template <int W>
__global__ __launch_bounds__(256) void mcv_hamming_partial(const uint32_t* __restrict__ q, int nq,
                                                           const uint32_t* __restrict__ t, int nt, int chunkLen,
                                                           uint2* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int qwave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    const int chunk = blockIdx.y;
    const int qi = qwave * 64 + lane;
    const int tBegin = chunk * chunkLen;
    const int tEnd = min(tBegin + chunkLen, nt);
    if (qwave * 64 >= nq) return;

    uint32_t qv[W];
    const int qsafe = qi < nq ? qi : nq - 1;
#pragma unroll
    for (int w = 0; w < W; ++w) qv[w] = q[(size_t)qsafe * W + w];

    uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;
    int j = tBegin;
    for (; j + 1 < tEnd; j += 2) {
        const uint32_t* ta = t + (size_t)j * W;
        const uint32_t* tb = ta + W;
        uint32_t da = 0, db = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            da = da + __popc(qv[w] ^ ta[w]);
            db = db + __popc(qv[w] ^ tb[w]);
        }
        const uint32_t ka = (da << kIdxBits) | (uint32_t)j;
        const uint32_t kb = (db << kIdxBits) | (uint32_t)(j + 1);
        m2 = min(m2, max(m1, ka));
        m1 = min(m1, ka);
        m2 = min(m2, max(m1, kb));
        m1 = min(m1, kb);
    }
    if (j < tEnd) {
        const uint32_t* ta = t + (size_t)j * W;
        uint32_t da = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) da += __popc(qv[w] ^ ta[w]);
        const uint32_t ka = (da << kIdxBits) | (uint32_t)j;
        m2 = min(m2, max(m1, ka));
        m1 = min(m1, ka);
    }
    if (qi < nq) part[(size_t)chunk * nq + qi] = make_uint2(m1, m2);
}

__global__ __launch_bounds__(256) void mcv_hamming_merge(const uint2* __restrict__ part, int nq, int nchunks,
                                                         int* __restrict__ idx, int* __restrict__ dist,
                                                         int* __restrict__ idx2, int* __restrict__ dist2) {
    const int qi = blockIdx.x * 256 + threadIdx.x;
    if (qi >= nq) return;
    uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;
    for (int c = 0; c < nchunks; ++c) {
        const uint2 p = part[(size_t)c * nq + qi];
        m2 = min(m2, max(m1, p.x));
        m1 = min(m1, p.x);
        m2 = min(m2, p.y);
    }
    idx[qi] = m1 == 0xFFFFFFFFu ? -1 : (int)(m1 & kIdxMask);
    dist[qi] = m1 == 0xFFFFFFFFu ? INT_MAX : (int)(m1 >> kIdxBits);
    if (idx2) idx2[qi] = m2 == 0xFFFFFFFFu ? -1 : (int)(m2 & kIdxMask);
    if (dist2) dist2[qi] = m2 == 0xFFFFFFFFu ? INT_MAX : (int)(m2 >> kIdxBits);
}

// Re-pack [n][bytes] rows into zero-padded [n][W] 32-bit words (XOR of the zero pads is 0).
__global__ void mcv_hamming_repack(const uint8_t* __restrict__ src, int n, int bytes, int W,
                                   uint32_t* __restrict__ dst) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n * W) return;
    const int r = i / W, w = i % W;
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int c = 4 * w + b;
        if (c < bytes) v |= (uint32_t)src[(size_t)r * bytes + c] << (8 * b);
    }
    dst[i] = v;
}

struct HammingWork {
    DevBuf<uint32_t> qpack, tpack;
    DevBuf<uint2> part;
};

int launch_match_hamming(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int bytesPerDesc, int* d_idx,
                         int* d_dist, int* d_idx2, int* d_dist2, hipStream_t s) {
    if (bytesPerDesc < 1 || bytesPerDesc > 64) fail("cvMatchHamming: bytesPerDesc %d outside [1, 64]", bytesPerDesc);
    if (nt < 0 || nt > (int)kIdxMask) fail("cvMatchHamming: nt %d outside [0, 2^22)", nt);
    if (nq <= 0) return 0;
    thread_local HammingWork wk;
    const int W = bytesPerDesc <= 32 ? 8 : 16;
    const uint32_t* q = (const uint32_t*)d_q;
    const uint32_t* t = (const uint32_t*)d_t;
    const bool aligned = (((uintptr_t)d_q | (uintptr_t)d_t) & 3) == 0;
    if (bytesPerDesc != 4 * W || !aligned) {
        wk.qpack.ensure((size_t)nq * W);
        wk.tpack.ensure((size_t)(nt > 0 ? nt : 1) * W);
        hipLaunchKernelGGL(mcv_hamming_repack, dim3((nq * W + 255) / 256), dim3(256), 0, s, d_q, nq, bytesPerDesc, W,
                           wk.qpack.p);
        if (nt > 0)
            hipLaunchKernelGGL(mcv_hamming_repack, dim3((nt * W + 255) / 256), dim3(256), 0, s, d_t, nt,
                               bytesPerDesc, W, wk.tpack.p);
        q = wk.qpack.p;
        t = wk.tpack.p;
    }
    const int qwaves = (nq + 63) / 64;
    int nchunks = (4096 + qwaves - 1) / qwaves;
    const int maxChunks = nt > 0 ? (nt + 63) / 64 : 1;
    if (nchunks > maxChunks) nchunks = maxChunks;
    if (nchunks < 1) nchunks = 1;
    const int chunkLen = nt > 0 ? (nt + nchunks - 1) / nchunks : 0;
    wk.part.ensure((size_t)nchunks * nq);
    dim3 grid((qwaves + 3) / 4, nchunks);
    ProfScope ps("hamming", s);
    if (W == 8)
        hipLaunchKernelGGL((mcv_hamming_partial<8>), grid, dim3(256), 0, s, q, nq, t, nt, chunkLen, wk.part.p);
    else
        hipLaunchKernelGGL((mcv_hamming_partial<16>), grid, dim3(256), 0, s, q, nq, t, nt, chunkLen, wk.part.p);
    hipLaunchKernelGGL(mcv_hamming_merge, dim3((nq + 255) / 256), dim3(256), 0, s, wk.part.p, nq, nchunks, d_idx,
                       d_dist, d_idx2, d_dist2);
    MCV_HIP(hipGetLastError());
    return nq;
}

}  // namespace mcv
