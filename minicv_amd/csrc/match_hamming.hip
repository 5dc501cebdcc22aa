// match_hamming.hip — brute-force Hamming matcher (cv::BFMatcher(NORM_HAMMING).knnMatch(k = 2)
// semantics [ext: OpenCV features2d]; descriptor layout = DetectorResult / ImageFeatures
// row-major [n][bytes], MiniCVNative.h:22-28, OpenCV.fs:478-524).
//
// Integer VALU work, not a GEMM: per (query, train) pair W x (v_xor_b32 + v_bcnt_u32_b32) on
// 32-bit words, then a packed-key top-2 update. Layout on the chip:
//   * lane = query: each lane keeps its query's W words in VGPRs;
//   * wave-uniform train index: the train descriptor arrives by scalar loads (SGPRs), so each
//     XOR reads it as its scalar operand — no LDS traffic at all;
//   * train descriptors are staged in two ping-pong SGPR groups of 16 dwords (NB = 1, default) or
//     32 (NB = 2) by hand-issued s_load_dwordx16 bursts, so the scalar-load latency hides behind a
//     group of VALU work;
//   * the train set is split into S chunks over the grid (~16k waves; NB, waves and queries per
//     lane screened in scripts/sweep_hamming.sh); a block = one query-wave x 4 consecutive chunks, each
//     (query-wave, chunk) keeps a top-2 of packed keys key = dist << 22 | trainIdx, so
//     min(key) is "smallest distance, then lowest train index" (BFMatcher's first-minimum rule);
//   * the block merges its 4 waves' top-2s in LDS; a merge kernel folds the S/4 partials per query.
// Issue cost per (query, train) pair on gfx950, measured (scripts/exp/valu_rate.hip): the VOP2
// v_xor_b32 / v_min_u32 take 2 cycles per wave64 instruction, the VOP3-only v_bcnt_u32_b32 /
// v_med3_u32 / v_lshl_or_b32 take 4 — 8 x (2 + 4) + 4 + 4 + 2 = 58 SIMD cycles per 64 pairs.
#include "kernels.h"
#include "mcv_runtime.h"
#include "plan.h"
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

namespace mcv {

static const int kIdxBits = 22;
static const uint32_t kIdxMask = (1u << kIdxBits) - 1;

// Top-2 of packed keys: with m1 <= m2 the new second best is med3(m1, k, m2) (one VALU op).
__device__ __forceinline__ void top2_push(uint32_t& m1, uint32_t& m2, uint32_t k) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(m1), "v"(k), "v"(m2));
    m2 = r;
    m1 = min(m1, k);
}

// popcount(a ^ b) + acc as one v_xor_b32 + one accumulating v_bcnt_u32_b32 (the compiler would
// otherwise re-associate the sum into v_bcnt(x, 0) + v_add3 trees: 1/3 more adds).
__device__ __forceinline__ uint32_t xor_bcnt(uint32_t a, uint32_t b, uint32_t acc) {
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(a ^ b), "v"(acc));
    return r;
}

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// 16 dwords (two 256-bit descriptors, or one 512-bit one) into SGPRs by one s_load_dwordx16,
// issued by hand. The waitcnt pass does not see it: every use goes through sgpr_wait() first.
// `live0/live1` (the other buffer) are tied to the load so the scheduler can neither consume the
// other buffer above it nor hand its registers to this one.
__device__ __forceinline__ u32x16 sload16(const uint32_t* p, u32x16& live0, u32x16& live1) {
    u32x16 r;
    asm volatile("s_load_dwordx16 %0, %3, 0x0" : "=&s"(r), "+s"(live0), "+s"(live1) : "s"(p));
    return r;
}
__device__ __forceinline__ u32x16 sload16(const uint32_t* p, u32x16& live0) {
    u32x16 r;
    asm volatile("s_load_dwordx16 %0, %2, 0x0" : "=&s"(r), "+s"(live0) : "s"(p));
    return r;
}
// Scalar loads return out of order: only lgkmcnt(0) is a valid wait. The buffers are tied to the
// wait (no use above it) and so is the running top-2 (the previous group's VALU work stays above).
template <int Q>
__device__ __forceinline__ void sgpr_wait(u32x16& a, u32x16& b, uint32_t (&m1)[Q], uint32_t (&m2)[Q]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(a), "+s"(b), "+v"(m1[0]), "+v"(m2[0]));
    if (Q > 1) asm volatile("; keep %0 %1" : "+v"(m1[Q - 1]), "+v"(m2[Q - 1]));
}
template <int Q>
__device__ __forceinline__ void sgpr_wait(u32x16& a, uint32_t (&m1)[Q], uint32_t (&m2)[Q]) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(a), "+v"(m1[0]), "+v"(m2[0]));
    if (Q > 1) asm volatile("; keep %0 %1" : "+v"(m1[Q - 1]), "+v"(m2[Q - 1]));
}

template <int W>
__device__ __forceinline__ uint32_t hamming_key_v(const uint32_t* qv, const u32x16& v, int off, int j) {
    uint32_t d = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) d = xor_bcnt(qv[w], v[off + w], d);
    return (d << kIdxBits) | (uint32_t)j;
}

// Lane = Q queries (their W words each in VGPRs); a wave covers 64 Q consecutive queries.
// A group = 16 NB dwords (NB = 2: 4 x 256-bit or 2 x 512-bit descriptors; NB = 1: half that) in NB
// SGPR vectors. Two groups ping-pong: wait(A) -> issue B -> consume A -> wait(B) -> issue A' ->
// consume B, so each burst's latency (K$ miss -> L2) hides behind a whole group of VALU work.
// NB = 1 halves the SGPRs the buffers take (occupancy: 8 waves per SIMD instead of 7).
template <int W, int Q, int NB>
__global__ __launch_bounds__(256) void mcv_hamming_partial(const uint32_t* __restrict__ q, int nq,
                                                           const uint32_t* __restrict__ t, int nt, int chunkLen,
                                                           uint2* __restrict__ part) {
    constexpr int G = 16 * NB / W;  // descriptors per group
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // block = one query-wave x 4 consecutive train chunks (one per wave), merged in LDS at the end:
    // a quarter of the partial top-2s for the merge kernel to read
    const int qwave = blockIdx.x;
    const int chunk = blockIdx.y * 4 + wv;
    const int tBegin = min(chunk * chunkLen, nt);
    const int tEnd = min(tBegin + chunkLen, nt);
    if (qwave * 64 * Q >= nq) return;   // block-uniform

    uint32_t qv[Q][W];
#pragma unroll
    for (int r = 0; r < Q; ++r) {
        const int qi = (qwave * Q + r) * 64 + lane;
        const int qsafe = qi < nq ? qi : nq - 1;
#pragma unroll
        for (int w = 0; w < W; ++w) qv[r][w] = q[(size_t)qsafe * W + w];
    }

    uint32_t m1[Q], m2[Q];
#pragma unroll
    for (int r = 0; r < Q; ++r) m1[r] = m2[r] = 0xFFFFFFFFu;
    const int nGroups = (tEnd - tBegin) / G;
    int j = tBegin;
    auto consume = [&](const u32x16& lo, const u32x16& hi, int jj) {
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int off = k * W;
#pragma unroll
            for (int r = 0; r < Q; ++r) {
                const uint32_t key = off < 16 ? hamming_key_v<W>(qv[r], lo, off, jj + k)
                                               : hamming_key_v<W>(qv[r], hi, off - 16, jj + k);
                top2_push(m1[r], m2[r], key);
            }
        }
    };
    if (nGroups > 0 && NB == 2) {
        const uint32_t* tp = t + (size_t)j * W;
        u32x16 a0 = {}, a1 = {}, b0 = {}, b1 = {};
        a0 = sload16(tp, b0, b1);
        a1 = sload16(tp + 16, b0, b1);
        int g = 0;
        for (; g + 1 < nGroups; g += 2, j += 2 * G) {
            sgpr_wait<Q>(a0, a1, m1, m2);
            const uint32_t* tb = t + (size_t)(j + G) * W;
            b0 = sload16(tb, a0, a1);
            b1 = sload16(tb + 16, a0, a1);
            consume(a0, a1, j);
            sgpr_wait<Q>(b0, b1, m1, m2);
            const uint32_t* ta = t + (size_t)(g + 2 < nGroups ? j + 2 * G : j) * W;
            a0 = sload16(ta, b0, b1);
            a1 = sload16(ta + 16, b0, b1);
            consume(b0, b1, j + G);
        }
        sgpr_wait<Q>(a0, a1, m1, m2);
        if (g < nGroups) {
            consume(a0, a1, j);
            j += G;
        }
    } else if (nGroups > 0) {   // NB == 1: one 16-dword vector per group
        const uint32_t* tp = t + (size_t)j * W;
        u32x16 a0 = {}, b0 = {};
        a0 = sload16(tp, b0);
        int g = 0;
        for (; g + 1 < nGroups; g += 2, j += 2 * G) {
            sgpr_wait<Q>(a0, m1, m2);
            b0 = sload16(t + (size_t)(j + G) * W, a0);
            consume(a0, a0, j);
            sgpr_wait<Q>(b0, m1, m2);
            a0 = sload16(t + (size_t)(g + 2 < nGroups ? j + 2 * G : j) * W, b0);
            consume(b0, b0, j + G);
        }
        sgpr_wait<Q>(a0, m1, m2);
        if (g < nGroups) {
            consume(a0, a0, j);
            j += G;
        }
    }
    for (; j < tEnd; ++j) {
        const uint32_t* td = t + (size_t)j * W;
#pragma unroll
        for (int r = 0; r < Q; ++r) {
            uint32_t d = 0;
#pragma unroll
            for (int w = 0; w < W; ++w) d = xor_bcnt(qv[r][w], td[w], d);
            top2_push(m1[r], m2[r], (d << kIdxBits) | (uint32_t)j);
        }
    }
    __shared__ uint2 sm[4][64 * Q];
#pragma unroll
    for (int r = 0; r < Q; ++r) sm[wv][r * 64 + lane] = make_uint2(m1[r], m2[r]);
    __syncthreads();
    if (wv != 0) return;
#pragma unroll
    for (int r = 0; r < Q; ++r) {
#pragma unroll
        for (int o = 1; o < 4; ++o) {
            const uint2 p = sm[o][r * 64 + lane];
            top2_push(m1[r], m2[r], p.x);
            top2_push(m1[r], m2[r], p.y);
        }
        const int qi = (qwave * Q + r) * 64 + lane;
        if (qi < nq) part[(size_t)blockIdx.y * nq + qi] = make_uint2(m1[r], m2[r]);
    }
}

// Eight lanes per query (chunks c = j mod 8 on lane j, then a 3-step butterfly): the fold is
// load-latency-bound, so a query's chunks are read in parallel and 8x more CUs take part.
__global__ __launch_bounds__(256) void mcv_hamming_merge(const uint2* __restrict__ part, int nq, int nchunks,
                                                         int* __restrict__ idx, int* __restrict__ dist,
                                                         int* __restrict__ idx2, int* __restrict__ dist2) {
    const int qi = blockIdx.x * 32 + (threadIdx.x >> 3);
    const int j = threadIdx.x & 7;
    uint32_t m1 = 0xFFFFFFFFu, m2 = 0xFFFFFFFFu;
    if (qi < nq) {
#pragma unroll 4
        for (int c = j; c < nchunks; c += 8) {
            const uint2 p = part[(size_t)c * nq + qi];
            m2 = min(m2, max(m1, p.x));
            m1 = min(m1, p.x);
            m2 = min(m2, p.y);
        }
    }
#pragma unroll
    for (int off = 1; off < 8; off <<= 1) {   // keys are distinct (index field): min / max merge exactly
        const uint32_t o1 = __shfl_xor(m1, off, 64), o2 = __shfl_xor(m2, off, 64);
        m2 = min(max(m1, o1), min(m2, o2));
        m1 = min(m1, o1);
    }
    if (qi >= nq || j != 0) return;
    idx[qi] = m1 == 0xFFFFFFFFu ? -1 : (int)(m1 & kIdxMask);
    dist[qi] = m1 == 0xFFFFFFFFu ? INT_MAX : (int)(m1 >> kIdxBits);
    if (idx2) idx2[qi] = m2 == 0xFFFFFFFFu ? -1 : (int)(m2 & kIdxMask);
    if (dist2) dist2[qi] = m2 == 0xFFFFFFFFu ? INT_MAX : (int)(m2 >> kIdxBits);
}

// ---- The GEMM form (default since round 4; fp4 operands since round 6): Hamming distance as a dot
// product on the matrix cores, v_mfma_f32_32x32x64_f8f6f4 with both operands in fp4 (e2m1) — K = 64
// per instruction at the cycles of the i8 form's K = 32, so half the matrix time of round 4-5's
// v_mfma_i32_32x32x32_i8, and a cheaper operand expansion.
// Encoding. Dword d (0..3) of a 32-bit descriptor word w holds bit 4k + d of w in its nibble k, so one
// word is one lane's 32 K elements (4 dwords) and the lane halves h = 0 / 1 (K [0, 32) / [32, 64)) take
// words s of their half rows at k step s — the same map for both operands, so element k of a train
// row meets element k of a query row. A train bit t becomes the nibble 0.5 t / 1.0 t / 2.0 t / 2.0 t for
// d = 0 / 1 / 2 / 3 (w & 0x1.., w & 0x2.., w & 0x4.., (w >> 1) & 0x4..: no shift for d < 3), a query
// bit q the nibble +-2 / +-1 / +-0.5 / +-0.5 with the sign bit = q, so every product is exactly
// t (1 - 2 q) and the sum over a row pair is pt - 2 dot = ham - pq (pq = the query's popcount; the
// zero pad bits have t = 0 and add nothing).
// Key. The accumulator starts at C = Kp + (4064 + r) / 4096 (r = the row inside the 32-row tile; Kp =
// 32 W bits), so a row's f32 result is H + f with H = Kp + ham - pq in [0, 2 Kp] and f = (4064 + r) /
// 4096 in [0, 1): every value is a multiple of 2^-12 below 2^11, exact in f32 at every step of the
// chain, and positive, so the float and its bit pattern order alike: the tile's scores fold into the
// kept top-2 by min3 / med3 (top2_tile16) and the fold across segments stays on the bit patterns. Rows of earlier tiles must rank below a later tile's at
// equal distance (the lowest index wins): instead of raising C by 32 rows per tile, the kept top-2 keys
// move down by 32 / 4096 at the top of each tile (2 v_add_f32 per query tile instead of 16 integer adds
// to C, and C stays loop-invariant). A key kept from tile k of an n-tile segment has moved n - 1 - k
// times (<= 127, so f >= 0), and the epilogue recovers j' = 32 k + r = 4096 f - 4064 + 32 (n - 1), then
// the popcount form's key (ham << 22 | trainIdx) with ham = H - Kp + pq (bit for bit the same rule).
// Rows past nt get 2^20 after the chain (a branch once per launch), kept keys start at 2^30 (moving
// them down leaves them there); both are >= 2^19 and fold to "no match".
// Queries are expanded once per segment into VGPR-resident B fragments; each train tile is loaded packed
// (16 B of a 256-bit row per lane) one tile ahead and expanded in registers right before its MFMAs
// (round 6: no LDS tile, no per-tile barrier; the round-5 LDS staging shared the expansion between a
// block's four waves and measured the same).
__device__ __forceinline__ int32_t ham_train_f4(uint32_t w, int d) {
    return (int32_t)(d == 0 ? w & 0x11111111u : d == 1 ? w & 0x22222222u : d == 2 ? w & 0x44444444u
                                                                                   : (w >> 1) & 0x44444444u);
}
__device__ __forceinline__ int32_t ham_query_f4(uint32_t w, int d) {
    return (int32_t)(d == 0 ? 0x44444444u | ((w << 3) & 0x88888888u)
                     : d == 1 ? 0x22222222u | ((w << 2) & 0x88888888u)
                     : d == 2 ? 0x11111111u | ((w << 1) & 0x88888888u)
                              : 0x11111111u | (w & 0x88888888u));
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
static constexpr int kHamChunkRows = 4096;   // j' < 4096: the key's 12 fraction bits
static constexpr int kHamJ0 = kHamChunkRows - 32;   // a new row's fraction field (4064 + r)
static constexpr uint32_t kHamKeptStart = 0x4E800000u;   // 2^30 as f32
static constexpr uint32_t kHamMaskedRow = 0x49800000u;   // 2^20 as f32

// Block = WPB waves x QT query tiles of 32 (VGPR-resident B fragments); the waves of a block walk the
// same train tiles (their 1 KB loads hit L1 after the first) and each expanded A fragment feeds QT
// MFMAs.
// Partition (round 5, stream-K style): the (query block, train tile) steps in query-block-major order
// are cut into gridDim.x equal contiguous ranges (at most 128 tiles, the key's 4096-row index field),
// one per block, so every block does the same work to a tile (the (query block, chunk) grid it
// replaces left its second round of resident blocks three quarters full at cfg2). A range's part of
// one query block is a segment; segment k of a query block (k = the block - the block holding the
// query block's first tile) writes its top-2 per query to part[k][query], and the block that
// completes a query block's last segment (an arrival counter per query block against its segment
// count) folds them into the outputs as mcv_hamming_merge does, without a second launch. The XCDs'
// L2s are not coherent, and an agent-scope fence writes back or invalidates a whole L2 (per block:
// 30 -> 93 us), so every cross-block value is a device-scope atomic instead: the partials are stored
// and read with agent-scope atomic stores / loads (sc1: performed at the device-coherent level, never
// stale in an L2), each block waits for its stores to complete (s_waitcnt vmcnt(0), a compiler barrier
// too) before its agent-scope arrival add, and the last block's loads are issued after that add returns.
// The tile's top-2 tree runs on the keys as floats (positive, finite, no denormals: their order is the
// bit patterns' order, and min / med3 return one of their operands bit for bit), through operations the
// compiler emits itself: these read MFMA results directly, and the hazard recognizer pads an MFMA ->
// VALU read only for instructions it generated (a v_min3_u32 / v_med3_u32 inline-asm form of this tree
// gave wrong keys for 512-bit descriptors, whose 8-long MFMA chains end right before it).
__device__ __forceinline__ float fmin3k(float a, float b, float c) { return fminf(fminf(a, b), c); }
__device__ __forceinline__ float fmed3k(float a, float b, float c) { return __builtin_amdgcn_fmed3f(a, b, c); }
// Two top-2 pairs (x1 <= x2), (y1 <= y2) merged into x: the minimum, and the second smallest of the four,
// min(max(x1, y1), min(x2, y2)) = med3(x1, y1, min(x2, y2)) (min(x2, y2) >= min(x1, y1)).
__device__ __forceinline__ void top2_merge(float& x1, float& x2, float y1, float y2) {
    const float s2 = fmed3k(x1, y1, fminf(x2, y2));
    x1 = fminf(x1, y1);
    x2 = s2;
}
// The top-2 of a lane's 16 scores of a tile as a tree (round 6): five triples (min3 / med3: the smallest
// two of three in two instructions), the sixteenth pushed into the fifth, four pairwise merges, then one
// merge into the kept pair — ~86 issue cycles against 96 for 16 sequential med3 / min pushes, and a
// dependency depth of 5 merges instead of 8 pushes per chain. Keys are distinct (the row fraction)
// except masked rows, which fold to "no match" whatever their order.
__device__ __forceinline__ void top2_tile16(uint32_t& m1, uint32_t& m2, const f32x16& k) {
    float a1[5], a2[5];
#pragma unroll
    for (int g = 0; g < 5; ++g) {
        a1[g] = fmin3k(k[3 * g], k[3 * g + 1], k[3 * g + 2]);
        a2[g] = fmed3k(k[3 * g], k[3 * g + 1], k[3 * g + 2]);
    }
    top2_merge(a1[0], a2[0], a1[1], a2[1]);
    top2_merge(a1[2], a2[2], a1[3], a2[3]);
    a2[4] = fmed3k(a1[4], k[15], a2[4]);
    a1[4] = fminf(a1[4], k[15]);
    top2_merge(a1[0], a2[0], a1[2], a2[2]);
    top2_merge(a1[0], a2[0], a1[4], a2[4]);
    float x1 = __uint_as_float(m1), x2 = __uint_as_float(m2);
    top2_merge(x1, x2, a1[0], a2[0]);
    m1 = __float_as_uint(x1);
    m2 = __float_as_uint(x2);
}
template <int W, int QT, int WPB>
__global__ __launch_bounds__(64 * WPB, 2) void mcv_hamming_mfma(const uint32_t* __restrict__ q, int nq,
                                                             const uint32_t* __restrict__ t, int nt, int ntTiles,
                                                             int qblocks, uint2* __restrict__ part,
                                                             unsigned* __restrict__ arrivals, int* __restrict__ oIdx,
                                                             int* __restrict__ oDist, int* __restrict__ oIdx2,
                                                             int* __restrict__ oDist2) {
    static_assert(QT % 2 == 0 || QT == 1, "the fold takes QT / 2 queries per thread");
    constexpr int KS = W / 2;              // k steps: one word per lane half each (K = 64 bits)
    constexpr int Kp = 32 * W;             // bits per row
    constexpr int NV = W / 8;              // uint4 per lane per half row
    __shared__ int lastBlock;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int B = (int)gridDim.x, blk = (int)blockIdx.x;
    const int64_t Wt = (int64_t)qblocks * ntTiles;
    const int64_t end = (int64_t)(blk + 1) * Wt / B;
    for (int64_t pos = (int64_t)blk * Wt / B; pos < end;) {
        const int bx = (int)(pos / ntTiles);
        const int64_t itemStart = (int64_t)bx * ntTiles, itemEnd = itemStart + ntTiles;
        const int64_t segEnd = end < itemEnd ? end : itemEnd;
        const int tBegin = (int)(pos - itemStart), tEnd = tBegin + (int)(segEnd - pos);
        // the blocks holding the query block's first and last tiles (the largest j with j Wt / B <= tile)
        const int j0 = (int)(((itemStart + 1) * B - 1) / Wt), j1 = (int)((itemEnd * B - 1) / Wt);
        const int slot = blk - j0, nseg = j1 - j0 + 1;
        const int q0 = (bx * WPB + wave) * QT * 32;
        i32x4 bq[QT][KS];
        int pq[QT];   // the query's popcount (both halves)
        {
            uint4 qw[QT][NV];   // the lane's half query row: 16-byte loads, all issued before the expansion
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const int qi = min(q0 + 32 * qt + col, nq - 1);
                const uint4* qr = reinterpret_cast<const uint4*>(q + (size_t)qi * W + (W / 2) * h);
#pragma unroll
                for (int v = 0; v < NV; ++v) qw[qt][v] = qr[v];
            }
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                int c = 0;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const uint4 u4 = qw[qt][s >> 2];
                    const int wi = s & 3;
                    const uint32_t wd = wi == 0 ? u4.x : wi == 1 ? u4.y : wi == 2 ? u4.z : u4.w;
                    bq[qt][s] = i32x4{ham_query_f4(wd, 0), ham_query_f4(wd, 1), ham_query_f4(wd, 2),
                                      ham_query_f4(wd, 3)};
                    c += __popc(wd);
                }
                pq[qt] = c + __shfl_xor(c, 32, 64);
            }
        }
        uint32_t m1[QT], m2[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) m1[qt] = m2[qt] = kHamKeptStart;
        // the lane's half of its train row (words [W h / 2, W h / 2 + W / 2): 16 B at W = 8) straight
        // from global memory, the next tile's in flight under this tile's MFMAs (the block's four waves
        // read the same 1 KB tile: L1 hits after the first)
        auto tload = [&](int tl, uint4 (&dst)[NV]) {
            const int row = min(tl * 32 + col, nt - 1);
            const uint4* src = reinterpret_cast<const uint4*>(t + (size_t)row * W + (W / 2) * h);
#pragma unroll
            for (int v = 0; v < NV; ++v) dst[v] = src[v];
        };
        // accumulator start values Kp + (4064 + r) / 4096, rebuilt per segment from one opaque VGPR (the
        // compiler otherwise keeps all 16 across the segment loop and spills them)
        f32x16 c0;
        int rbase = kHamJ0 + 4 * h;
        asm volatile("" : "+v"(rbase));
#pragma unroll
        for (int i = 0; i < 16; ++i) c0[i] = (float)Kp + (float)(rbase + (i & 3) + 8 * (i >> 2)) * (1.0f / 4096.0f);
        uint4 tw[NV], nx[NV];
        tload(tBegin, tw);
        for (int tl = tBegin; tl < tEnd; ++tl) {
            tload(min(tl + 1, tEnd - 1), nx);
            // the kept keys move 32 rows down (the first tile: start values only, which stay at 2^30)
            auto down = [](uint32_t& k) { k = __float_as_uint(__uint_as_float(k) - 32.0f / 4096.0f); };
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) { down(m1[qt]); down(m2[qt]); }
            // priority 0 for the MFMAs, 1 for the expansion and top-2 updates (as mcv_l2_gemm's epilogue)
            __builtin_amdgcn_s_setprio(0);
            f32x16 acc[QT];
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                const uint4 u4 = tw[s >> 2];
                const int wi = s & 3;
                const uint32_t w = wi == 0 ? u4.x : wi == 1 ? u4.y : wi == 2 ? u4.z : u4.w;
                const i32x8 a = i32x8{ham_train_f4(w, 0), ham_train_f4(w, 1), ham_train_f4(w, 2), ham_train_f4(w, 3),
                                      0, 0, 0, 0};
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    const i32x8 b = i32x8{bq[qt][s][0], bq[qt][s][1], bq[qt][s][2], bq[qt][s][3], 0, 0, 0, 0};
                    // cbsz = blgp = 4: both operands fp4 (4 VGPRs each); zero scales select the unscaled form
                    acc[qt] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, s == 0 ? c0 : acc[qt], 4, 4, 0, 0,
                                                                              0, 0);
                }
            }
            if (__builtin_expect(tl * 32 + 32 > nt, 0)) {   // rows past nt (wave-uniform; once per launch)
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        if (tl * 32 + (i & 3) + 8 * (i >> 2) + 4 * h >= nt) acc[qt][i] = __uint_as_float(kHamMaskedRow);
                    asm volatile("" : "+v"(acc[qt]));
                }
            }
            __builtin_amdgcn_s_setprio(1);
            // the tile's 16 scores per lane and query tile merged as a tree (round 6: two sequential
            // chains of 8 pushes before — cfg2 18.0 -> 17.5 us, 10k x 40k 47.2 -> 44.1 us, same box)
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) top2_tile16(m1[qt], m2[qt], acc[qt]);
#pragma unroll
            for (int v = 0; v < NV; ++v) tw[v] = nx[v];
        }
        // lanes l and l + 32 hold the same query (other rows): merge, then the popcount form's keys
        const uint32_t base = (uint32_t)tBegin * 32;
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            const uint32_t o1 = __shfl_xor(m1[qt], 32, 64), o2 = __shfl_xor(m2[qt], 32, 64);
            top2_push(m1[qt], m2[qt], o1);
            top2_push(m1[qt], m2[qt], o2);
            auto glob = [&](uint32_t k) {
                // masked rows and start values are >= 2^19; a real key H + f is below 2 Kp + 1 <= 1025
                const float kf = __uint_as_float(k);
                if (kf >= 524288.0f) return 0xFFFFFFFFu;
                const int H = (int)kf;
                const int jp = (int)((kf - (float)H) * 4096.0f) - (kHamJ0 - 32 * (tEnd - tBegin - 1));
                return ((uint32_t)(H - Kp + pq[qt]) << kIdxBits) | (base + (uint32_t)jp);
            };
            const int qi = q0 + 32 * qt + col;
            // Memory ordering of the fold (why no release / acquire fence is needed). The hand-off is the
            // write-through form MI355X_MICROARCH.md's correctness table lists in place of the agent-scope
            // release / acquire pair: (1) EVERY store of the handed-off partials is an agent-scope atomic
            // store, which gfx950 issues with sc1 — performed at the device-coherent level, past this CU's
            // L1 and any XCD's L2, never left dirty in a non-coherent cache; (2) each storing wave drains
            // them (s_waitcnt vmcnt(0) below) and the block's barrier follows before thread 0's arrival
            // add, so the add is issued only after every partial of the block has been performed; (3) the
            // arrival counter is itself an agent-scope atomic, and the last arriver reads the partials only
            // after its add has returned (the __syncthreads after it), with agent-scope atomic loads (sc1:
            // served from the coherent level, never from a stale L1 / L2 line). A counter value of nseg - 1
            // therefore implies every segment's partials are visible to those loads. The agent-scope fence
            // this replaces writes back / invalidates a whole XCD L2 per block (30 -> 93 us per launch).
            if (h == 0 && qi < nq) {
                const uint64_t v = (uint64_t)glob(m1[qt]) | ((uint64_t)glob(m2[qt]) << 32);
                __hip_atomic_store(reinterpret_cast<uint64_t*>(part) + (size_t)slot * nq + qi, v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            lastBlock = __hip_atomic_fetch_add(arrivals + bx, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                        (unsigned)(nseg - 1);
        __syncthreads();
        if (lastBlock) {
          for (int qx = 0; qx < (QT + 1) / 2; ++qx) {
            const int qm = bx * (QT * 32 * WPB) + threadIdx.x + 64 * WPB * qx;
            if (qm < nq && (QT > 1 || threadIdx.x < 32 * WPB)) {
                uint32_t a1 = 0xFFFFFFFFu, a2 = 0xFFFFFFFFu;
                // every partial of a batch of FB in flight before the first fold: the sc1 loads come from
                // the coherent level (~1-2 us each), and a query block spans ~19 segments at cfg2 (~77
                // for a 2500-query shard); eight per batch made the fold a chain of 3-10 round trips
                constexpr int FB = 24;
                for (int c0 = 0; c0 < nseg; c0 += FB) {
                    uint64_t pv[FB];
#pragma unroll
                    for (int u = 0; u < FB; ++u)
                        pv[u] = c0 + u < nseg ? __hip_atomic_load(reinterpret_cast<const uint64_t*>(part) +
                                                                      (size_t)(c0 + u) * nq + qm,
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                              : ~0ull;
#pragma unroll
                    for (int u = 0; u < FB; ++u) {
                        const uint2 pc = make_uint2((uint32_t)pv[u], (uint32_t)(pv[u] >> 32));
                        a2 = min(a2, max(a1, pc.x));
                        a1 = min(a1, pc.x);
                        a2 = min(a2, pc.y);
                    }
                }
                oIdx[qm] = a1 == 0xFFFFFFFFu ? -1 : (int)(a1 & kIdxMask);
                oDist[qm] = a1 == 0xFFFFFFFFu ? INT_MAX : (int)(a1 >> kIdxBits);
                if (oIdx2) oIdx2[qm] = a2 == 0xFFFFFFFFu ? -1 : (int)(a2 & kIdxMask);
                if (oDist2) oDist2[qm] = a2 == 0xFFFFFFFFu ? INT_MAX : (int)(a2 >> kIdxBits);
            }
          }
            if (threadIdx.x == 0) arrivals[bx] = 0u;   // re-armed for the next launch (ordered by the kernel boundary)
        }
        pos = segEnd;
    }
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
    DevBuf<unsigned> arrivals;   // per query block of the GEMM form (zero between launches)
    size_t arrivalsZeroed = 0;
    StreamFence fence;   // calls on different streams take turns on these buffers
};

// The GEMM form's launch: WPB waves per block, QT query tiles per wave; stream-K ranges over the resident
// blocks (occupancy of this instantiation).
template <int WPB, int QT>
static void launch_ham_gemm(HammingWork& wk, int W, const uint32_t* q, int nq, const uint32_t* t, int nt, int* d_idx,
                            int* d_dist, int* d_idx2, int* d_dist2, hipStream_t s) {
    const int qblocks = (nq + 32 * QT * WPB - 1) / (32 * QT * WPB);
    const int ntTiles = (nt + 31) / 32;
    static const int cus = [] {
        int d = 0, n = 0;
        (void)hipGetDevice(&d);
        return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0 ? n : 256;
    }();
    auto kern = W == 8 ? mcv_hamming_mfma<8, QT, WPB> : mcv_hamming_mfma<16, QT, WPB>;
    int perCu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, kern, 64 * WPB, 0) != hipSuccess || perCu <= 0) perCu = 1;
    const int64_t Wt = (int64_t)qblocks * ntTiles;
    // equal ranges of the (query block, tile) steps: ~24 tiles each between one and two blocks per CU
    // (round 6 grid sweep, fp4 form, B = 128..768: 1250 / 2500 / 5000 / 10000 queries x 10k best at
    // 128-256 / 192-256 / 256 / 512 blocks — fewer, longer ranges amortise the per-range query expansion
    // and keep a query block's segments within one batch of the fold's loads), within the resident
    // blocks, and at most 128 tiles per range (the key's index field)
    int64_t B = std::min<int64_t>(std::max<int64_t>((Wt + 23) / 24, cus), 2 * (int64_t)cus);
    B = std::min<int64_t>(B, (int64_t)perCu * cus);
    B = std::max<int64_t>(B, (Wt + kHamChunkRows / 32 - 1) / (kHamChunkRows / 32));
    B = std::max<int64_t>(1, std::min(B, Wt));
    if (B > INT_MAX) fail("cvMatchHamming: %lld ranges", (long long)B);
    int maxSeg = 1;
    for (int64_t x = 0; x < qblocks; ++x) {
        const int64_t j0 = ((x * ntTiles + 1) * B - 1) / Wt, j1 = ((x + 1) * ntTiles * B - 1) / Wt;
        maxSeg = std::max(maxSeg, (int)(j1 - j0 + 1));
    }
    wk.part.ensure((size_t)maxSeg * nq);
    if (wk.arrivalsZeroed < (size_t)qblocks) {
        wk.arrivals.ensure((size_t)qblocks);
        MCV_HIP(hipMemsetAsync(wk.arrivals.p, 0, wk.arrivals.n * sizeof(unsigned), s));
        wk.arrivalsZeroed = wk.arrivals.n;
    }
    ProfScope ps("hamming", s);
    hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(64 * WPB), 0, s, q, nq, t, nt, ntTiles, qblocks, wk.part.p,
                       wk.arrivals.p, d_idx, d_dist, d_idx2, d_dist2);
}

int launch_match_hamming(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int bytesPerDesc, int* d_idx,
                         int* d_dist, int* d_idx2, int* d_dist2, hipStream_t s, int form) {
    if (bytesPerDesc < 1 || bytesPerDesc > 64) fail("cvMatchHamming: bytesPerDesc %d outside [1, 64]", bytesPerDesc);
    if (nt < 0 || nt > (int)kIdxMask) fail("cvMatchHamming: nt %d outside [0, 2^22)", nt);
    if (nq <= 0) return 0;
    int dev = 0;   // per host thread and device (DevBuf does not follow a device switch)
    MCV_HIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= 16) fail("cvMatchHamming: device %d outside the 16 per-thread workspaces", dev);
    thread_local HammingWork works[16];
    HammingWork& wk = works[dev];
    wk.fence.enter(s);
    const int W = bytesPerDesc <= 32 ? 8 : 16;
    const uint32_t* q = (const uint32_t*)d_q;
    const uint32_t* t = (const uint32_t*)d_t;
    // the GEMM form reads each lane's half train row as 16-byte vectors
    const bool aligned = (((uintptr_t)d_q | (uintptr_t)d_t) & 15) == 0;
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
    // form 1: the XOR / popcount sweep (mcvMatchHammingDeviceForm); 0: the fp4 GEMM (default)
    if (form == kHammingFormGemm && nt > 0) {
        // 4 waves per block, 2 query tiles per wave (cfg2 screens: round 4, 1 query tile 33.6 vs 32.1 us;
        // round 6 without the LDS staging, 10k x 10k / 1250 x 10k / 10k x 40k: 2 waves per block 29.7 /
        // 18.7 / 87.6 us, 8 waves 28.3 / 15.7 / 91.7, against 28.1-31.4 / 14.9-15.3 / 87.3-99.4 for 4;
        // 4 query tiles per wave spill at 256 VGPRs), one block per resident slot (3 per CU at 256-bit
        // descriptors, 2 at 512-bit).
        // small problems (the multi-GPU shares): one query tile per wave, twice the query blocks, so the
        // ranges stay ~24 tiles over more blocks (round 6, same box alternating: 1250 / 5000 x 10k
        // 11.2-11.4 -> 10.0-10.1 / 14.4-14.6 -> 13.4 us; cfg2 17.7 -> 18.2-18.5 and 10k x 40k 46.0 -> 64.1
        // us the other way)
        const int64_t steps2 = (int64_t)((nq + 255) / 256) * ((nt + 31) / 32);
        if (steps2 <= 8192)
            launch_ham_gemm<4, 1>(wk, W, q, nq, t, nt, d_idx, d_dist, d_idx2, d_dist2, s);
        else
            launch_ham_gemm<4, 2>(wk, W, q, nq, t, nt, d_idx, d_dist, d_idx2, d_dist2, s);
        MCV_HIP(hipGetLastError());
        wk.fence.leave(s);
        return nq;
    }
    // popcount form: one query per lane, one SGPR vector per staged group, ~16384 waves
    // (scripts/sweep_hamming.sh: 2 queries per lane and 2-vector groups screened slower)
    constexpr int targetWaves = 16384, Q = 1, NB = 1;
    const int qwaves = (nq + 64 * Q - 1) / (64 * Q);
    int nchunks = (targetWaves + qwaves - 1) / qwaves;
    const int maxChunks = nt > 0 ? (nt + 63) / 64 : 1;
    if (nchunks > maxChunks) nchunks = maxChunks;
    if (nchunks < 1) nchunks = 1;
    const int chunkLen = nt > 0 ? (nt + nchunks - 1) / nchunks : 0;
    const int nparts = (nchunks + 3) / 4;
    wk.part.ensure((size_t)nparts * nq);
    dim3 grid(qwaves, nparts);
    {
        ProfScope ps("hamming", s);
        hipLaunchKernelGGL((W == 8 ? mcv_hamming_partial<8, Q, NB> : mcv_hamming_partial<16, Q, NB>), grid, dim3(256),
                           0, s, q, nq, t, nt, chunkLen, wk.part.p);
    }
    hipLaunchKernelGGL(mcv_hamming_merge, dim3((nq + 31) / 32), dim3(256), 0, s, wk.part.p, nq, nparts, d_idx,
                       d_dist, d_idx2, d_dist2);
    MCV_HIP(hipGetLastError());
    wk.fence.leave(s);
    return nq;
}

}  // namespace mcv

