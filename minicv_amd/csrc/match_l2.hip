// match_l2.hip — brute-force L2 matcher posed as an fp32 GEMM on the matrix cores
// (cv::BFMatcher(NORM_L2).knnMatch(k = 2) semantics [ext: OpenCV features2d]; descriptor layout
// = DetectorResult / ImageFeatures row-major [n][dim] float, MiniCVNative.h:22-28, OpenCV.fs:263-281).
//
//   |q - t|^2 = |q|^2 + |t|^2 - 2 q.t ; argmin over t needs only s(t) = |t|^2 - 2 q.t.
//
// mcv_l2_mfma<DP, TR>: v_mfma_f32_32x32x2_f32 (exact f32 FMA chain, 64 FLOP/clk/SIMD = the fp32
//   peak). A = TR train rows of a tile (from LDS), B = 32 queries (resident in VGPRs for the whole
//   kernel), D[i][j] = t_i . q_j. The 32x32 accumulator puts one query on each lane (col = lane & 31)
//   and 16 train rows in its registers, so the top-2 epilogue is lane-local: no cross-lane
//   reduction per tile, one shuffle at the end to merge the two lane halves.
//   Operands use a parity-split row layout (even dims, then odd dims): lane half h takes dims
//   2s + h, so 4 consecutive k-steps are one 16-byte read (ds_read_b128 / global_load_dwordx4).
//   Train tiles are double-buffered in LDS (row stride DP + 4 floats: conflict-free b128 reads),
//   register-staged: the next tile's global loads are issued before this tile's MFMAs and written
//   to LDS after them; one barrier per tile. The epilogue takes the tile's norms as 4 b128 reads
//   and inserts each score with 2 v_cmp + 6 v_cndmask (no divergent branch per score: the branchy
//   form the compiler chose cost 7 % of the kernel, 5.80 -> 5.38 ms at cfg5).
//   Grid = (query blocks of 128) x (train chunks); each lane keeps its top-3 GEMM-form scores.
// mcv_l2_gemm<DP> (f16 domain): the same GEMM form on the f16 matrix pipe (16x the f32 MFMA rate) with every
//   fp32 operand split into f16 hi + lo (x = hi + lo + r, |r| <= 2^-22 |x| + 2^-13): q.t ~ qh.th +
//   qh.tl + ql.th in two 32x32x16 accumulator chains (hi.hi; hi.lo then lo.hi) — 24 MFMAs of 32
//   cycles per 32 x 32 x 128 tile against 64 of 64 cycles in f32. f16 x f16 products are exact in f32; the dropped ql.tl and the
//   split residuals add 2^-21 |q| |t| + 2^-12.9 sqrt(dim) (|q| + |t|) to the nomination's error
//   bound (mcv_l2_refine's tol16), so the exact answer is unchanged. Used when every coordinate of
//   both sets is finite with |x| < 2^15 (fp16 range); mcv_l2_prep16 records max |x| per block and each
//   launch picks its form from those maxima on the device (no host round trip, no empty launch).
// mcv_l2_refine folds the per-chunk top-3s and makes the result exact: the three candidates' exact
//   squared distances (fp64 direct sum in dim order, the oracle's definition) give the top-2 unless a
//   bound on the GEMM form's rounding leaves room for another train (near-ties), in which case the
//   query is queued for mcv_l2_exact_scan (exact distance to every train). idx / dist are then
//   exactly the direct-sum answer: dist = (float)sqrt(exact d^2), ties -> lowest train index.
#include "kernels.h"
#include "mcv_runtime.h"
#include "plan.h"
#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace mcv {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
static constexpr unsigned kL2F16MaxBits = 0x47000000u;   // 32768.0f: |x| below it fits fp16 (max 65504)

// Maxima as float bits (non-negative floats; their writers clamp NaN to +inf): n words at p, folded
// by the calling wave (collective: every lane of the wave calls it and gets the wave-uniform result).
// mcv_l2_prep16 leaves kL2MaxSlots atomic maxima of max |x| (both sets) and of the train norms, so no
// launch of its own folds them; the DP > 128 path's mcv_l2_umax leaves one word.
struct L2Max {
    const unsigned* p;
    int n;
    int stride;   // words between consecutive maxima
};
__device__ __forceinline__ unsigned l2_max_bits(L2Max m) {
    unsigned v = 0;
    for (int i = (int)(threadIdx.x & 63); i < m.n; i += 64) {
        const unsigned x = m.p[i * m.stride];
        v = x > v ? x : v;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned o = __shfl_xor(v, off, 64);
        v = o > v ? o : v;
    }
    return (unsigned)__builtin_amdgcn_readfirstlane((int)v);
}
// The f16-split path's domain: max |x| over both sets below 2^15 (p null: the f32 path only).
__device__ __forceinline__ bool l2_f16_domain(L2Max dom) { return dom.p && l2_max_bits(dom) < kL2F16MaxBits; }

struct L2Part { float b1, b2, b3; int i1, i2, i3; };

// A GEMM segment's partial top-3 for query q into its slot, and empty partials (+inf, index -1: they
// change no merge) into the nEmpty slots after it that no segment of this (query block, chunk) item
// writes (mcv_l2_gemm's partition). Memory ordering: unlike the Hamming GEMM's in-kernel fold, the L2
// partials are folded by mcv_l2_refine, the next launch on the same stream; the kernel boundary writes
// back the producing kernel's L2 lines and the consumer starts with invalidated caches, so plain stores
// and loads suffice here (a stream-K fold inside mcv_l2_gemm measured slower: DESIGN.md §7).
__device__ __forceinline__ void l2_part_store(L2Part* __restrict__ part, int nqPad, int slot, int nEmpty, int q,
                                              const L2Part& p) {
    part[(size_t)slot * nqPad + q] = p;
    for (int e = 1; e <= nEmpty; ++e) {
        L2Part z;
        z.b1 = z.b2 = z.b3 = INFINITY;
        z.i1 = z.i2 = z.i3 = -1;
        part[(size_t)(slot + e) * nqPad + q] = z;
    }
}

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

// Epilogue insertion for one lane's scores in ascending train-index order (a later index never wins
// a tie, so strict < decides): top-2 (score, index) with 2 v_cmp + 6 v_cndmask on VCC (no divergent
// branch per score), plus b3 = the third-smallest score seen, index-free, by one v_med3_f32
// (b3 <- med3(s, b2, b3) = min(b3, max(s, b2)) while b2 <= b3: a score that misses the top-2, or
// the b2 it displaces, is a third-place candidate). Padding rows score +inf and change nothing.
__device__ __forceinline__ void top2b3_push_asc(float& b1, int& i1, float& b2, int& i2, float& b3, float s, int i) {
    float tb;
    int ti;
    asm volatile(
        "v_med3_f32 %[b3], %[s], %[b2], %[b3]\n\t"
        "v_cmp_lt_f32_e32 vcc, %[s], %[b2]\n\t"
        "v_cndmask_b32_e32 %[tb], %[b2], %[s], vcc\n\t"
        "v_cndmask_b32_e32 %[ti], %[i2], %[i], vcc\n\t"
        "v_cmp_lt_f32_e32 vcc, %[s], %[b1]\n\t"
        "v_cndmask_b32_e32 %[b2], %[tb], %[b1], vcc\n\t"
        "v_cndmask_b32_e32 %[i2], %[ti], %[i1], vcc\n\t"
        "v_cndmask_b32_e32 %[b1], %[b1], %[s], vcc\n\t"
        "v_cndmask_b32_e32 %[i1], %[i1], %[i], vcc"
        : [b1] "+v"(b1), [i1] "+v"(i1), [b2] "+v"(b2), [i2] "+v"(i2), [b3] "+v"(b3), [tb] "=&v"(tb),
          [ti] "=&v"(ti)
        : [s] "v"(s), [i] "v"(i)
        : "vcc");
}

// Third-smallest value of a merged set, index-free: fold value v into (b1 <= b2 <= b3) by value.
__device__ __forceinline__ void third_fold(float& c1, float& c2, float& c3, float v) {
    const float lo1 = fminf(c1, v), hi1 = fmaxf(c1, v);
    const float lo2 = fminf(c2, hi1), hi2 = fmaxf(c2, hi1);
    c1 = lo1;
    c2 = lo2;
    c3 = fminf(c3, hi2);
}

// Parity-split, zero-padded copy [nPad][DP] + squared norms (fp32, wave tree sum: the order only
// affects the GEMM form, whose rounding the exact re-rank bounds whatever the order). One launch
// covers the query and the train set (rows of q, then rows of t). dim > 128 only (DP = 256: the f32
// GEMM form reads these copies); for dim <= 128 mcv_l2_prep16 writes the norms and the f32 form
// (outside the f16 domain) reads the caller's rows.
struct L2PrepF32 {
    const float* src;
    int n, nPad;
    float* dst;
    float* norms;
    float padNorm;
};
__global__ void mcv_l2_prep(L2PrepF32 q, L2PrepF32 t, int dim, int DP) {
    const int lane = threadIdx.x & 63;
    for (int rr = blockIdx.x * 4 + (threadIdx.x >> 6); rr < q.nPad + t.nPad; rr += gridDim.x * 4) {
        const bool isq = rr < q.nPad;
        const int r = isq ? rr : rr - q.nPad, n = isq ? q.n : t.n;
        const float* src = isq ? q.src : t.src;
        float* dst = isq ? q.dst : t.dst;
        float acc = 0.f;
        for (int k = lane; k < DP; k += 64) {
            const float v = (r < n && k < dim) ? src[(size_t)r * dim + k] : 0.f;
            dst[(size_t)r * DP + (k & 1) * (DP / 2) + (k >> 1)] = v;
            acc = fmaf(v, v, acc);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (lane == 0) (isq ? q.norms : t.norms)[r] = r < n ? acc : (isq ? q.padNorm : t.padNorm);
    }
}

// Row-per-wave preps run grid-stride over at most this many 4-wave blocks.
static constexpr int kL2PrepBlocks = 16384;
static int l2_prep_blocks(int nPad) { return std::min((nPad + 3) / 4, kL2PrepBlocks); }

// Max of non-negative float bit patterns over a[0, na) and b[0, nb) -> *out, and over c[0, nc) ->
// *out2 when c is given (bit order = float order; NaN -> +inf): per-block maxima, the last block to
// finish folds them, writes the results and re-arms its counter (grid-wide, one launch, no host round
// trip). The DP > 128 path's train-norm maximum (the f16-capable path folds mcv_l2_prep16's per-block
// maxima where they are read).
static constexpr int kL2MaxBlocks = 64;
__global__ __launch_bounds__(256) void mcv_l2_umax(const unsigned* __restrict__ a, int na,
                                                   const unsigned* __restrict__ b, int nb,
                                                   const unsigned* __restrict__ c, int nc,
                                                   unsigned* __restrict__ part, unsigned* __restrict__ count,
                                                   unsigned* __restrict__ out, unsigned* __restrict__ out2) {
    __shared__ unsigned sm[2][4];
    __shared__ bool last;
    auto fold = [&](unsigned m, int j) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const unsigned o = __shfl_xor(m, off, 64);
            m = o > m ? o : m;
        }
        if ((threadIdx.x & 63) == 0) sm[j][threadIdx.x >> 6] = m;
        __syncthreads();
        m = sm[j][0];
        for (int w = 1; w < 4; ++w) m = sm[j][w] > m ? sm[j][w] : m;
        return m;
    };
    auto clampv = [](unsigned v) { return v > 0x7f800000u ? 0x7f800000u : v; };   // NaN (any sign bit) -> +inf
    unsigned m = 0, m2 = 0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < na + nb; i += gridDim.x * 256) {
        const unsigned v = clampv(i < na ? a[i] : b[i - na]);
        m = v > m ? v : m;
    }
    if (c)
        for (int i = blockIdx.x * 256 + threadIdx.x; i < nc; i += gridDim.x * 256) {
            const unsigned v = clampv(c[i]);
            m2 = v > m2 ? v : m2;
        }
    m = fold(m, 0);
    m2 = fold(m2, 1);
    if (threadIdx.x == 0) {
        part[blockIdx.x] = m;
        part[gridDim.x + blockIdx.x] = m2;
        __threadfence();
        last = atomicAdd(count, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    unsigned r = 0, r2 = 0;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += 256) {
        const unsigned v = __atomic_load_n(&part[i], __ATOMIC_RELAXED);
        const unsigned v2 = __atomic_load_n(&part[gridDim.x + i], __ATOMIC_RELAXED);
        r = v > r ? v : r;
        r2 = v2 > r2 ? v2 : r2;
    }
    __syncthreads();
    r = fold(r, 0);
    r2 = fold(r2, 1);
    if (threadIdx.x == 0) {
        *out = r;
        if (c) *out2 = r2;
        *count = 0u;
    }
}

// Stage TR train rows x DP floats (TR * DP / 1024 float4 per thread) + their norms.
template <int DP, int TR>
__device__ __forceinline__ void l2_gload(const float* __restrict__ tp, const float* __restrict__ tnorm, int tile,
                                         float4 (&stg)[TR * DP / 1024], float& nstg) {
    constexpr int ROWS_PER_PASS = 256 / (DP / 4);
    const int srow = threadIdx.x / (DP / 4), sc4 = threadIdx.x % (DP / 4);
#pragma unroll
    for (int r = 0; r < TR * DP / 1024; ++r)
        stg[r] = reinterpret_cast<const float4*>(tp + (size_t)(tile * TR + srow + r * ROWS_PER_PASS) * DP)[sc4];
    if (threadIdx.x < TR) nstg = tnorm[tile * TR + threadIdx.x];
}

template <int DP, int TR>
__device__ __forceinline__ void l2_lstore(float* __restrict__ lds, float* __restrict__ lnorm,
                                          const float4 (&stg)[TR * DP / 1024], float nstg) {
    constexpr int ROWF = DP + 4;
    constexpr int ROWS_PER_PASS = 256 / (DP / 4);
    const int srow = threadIdx.x / (DP / 4), sc4 = threadIdx.x % (DP / 4);
#pragma unroll
    for (int r = 0; r < TR * DP / 1024; ++r)
        *reinterpret_cast<float4*>(&lds[(srow + r * ROWS_PER_PASS) * ROWF + sc4 * 4]) = stg[r];
    if (threadIdx.x < TR) lnorm[threadIdx.x] = nstg;
}

// Stage a tile from the caller's row-major train set instead (the f32 form inside the f16-capable
// launch, DP <= 128): element e = thread + 256 j of the tile (row e / DP, dim e % DP; zero outside
// [0, nt) x [0, dim)), stored at its parity-split LDS position.
template <int DP, int TR>
__device__ __forceinline__ void l2_gload_raw(const float* __restrict__ traw, int nt, int dim,
                                             const float* __restrict__ tnorm, int tile, float (&stg)[TR * DP / 256],
                                             float& nstg) {
#pragma unroll
    for (int j = 0; j < TR * DP / 256; ++j) {
        const int e = threadIdx.x + 256 * j, r = tile * TR + e / DP, k = e % DP;
        stg[j] = r < nt && k < dim ? traw[(size_t)r * dim + k] : 0.f;
    }
    if (threadIdx.x < TR) nstg = tnorm[tile * TR + threadIdx.x];
}

template <int DP, int TR>
__device__ __forceinline__ void l2_lstore_raw(float* __restrict__ lds, float* __restrict__ lnorm,
                                              const float (&stg)[TR * DP / 256], float nstg) {
    constexpr int ROWF = DP + 4;
#pragma unroll
    for (int j = 0; j < TR * DP / 256; ++j) {
        const int e = threadIdx.x + 256 * j, r = e / DP, k = e % DP;
        lds[r * ROWF + (k & 1) * (DP / 2) + (k >> 1)] = stg[j];
    }
    if (threadIdx.x < TR) lnorm[threadIdx.x] = nstg;
}

// The f32 GEMM form (one block = 4 waves x 32 queries, a tile = TR train rows = TR / 32 independent
// 32x32 accumulator chains per wave, interleaved k-step by k-step: they share the query operands b[],
// so the matrix pipe never waits on one chain's dependent-accumulator latency). RAW: queries and train
// rows straight from the caller's arrays (raw, nq / nt / dim); otherwise the padded parity-split
// copies of mcv_l2_prep. lds: 2 TR (DP + 4) floats, lnorm: 2 TR floats.
template <int DP, int TR, bool RAW>
__device__ __forceinline__ void l2_gemm32_body(const float* __restrict__ qsrc, const float* __restrict__ tsrc, int nq,
                                               int nt, int dim, const float* __restrict__ tnorm, int tBegin,
                                               int tEnd, int nqPad, L2Part* __restrict__ part, int bx, int slot,
                                               int nEmpty, float* __restrict__ lds, float* __restrict__ lnorm) {
    constexpr int KS = DP / 2;          // MFMA k-steps (2 dims each)
    constexpr int ROWF = DP + 4;        // padded LDS row, floats
    constexpr int PER = RAW ? TR * DP / 256 : TR * DP / 1024;   // staging registers per thread per tile
    constexpr int NC = TR / 32;         // accumulator chains
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int q0 = (bx * 4 + wave) * 32;

    // B fragments: query q0 + col, dims 2s + h  (parity-split row: offset h * KS + s)
    float b[KS];
    if constexpr (RAW) {
        const int qq = q0 + col;
#pragma unroll
        for (int s = 0; s < KS; ++s) b[s] = qq < nq && 2 * s + h < dim ? qsrc[(size_t)qq * dim + 2 * s + h] : 0.f;
    } else {
        const float4* qrow = reinterpret_cast<const float4*>(qsrc + (size_t)(q0 + col) * DP + h * KS);
#pragma unroll
        for (int s4 = 0; s4 < KS / 4; ++s4) {
            const float4 v = qrow[s4];
            b[4 * s4 + 0] = v.x; b[4 * s4 + 1] = v.y; b[4 * s4 + 2] = v.z; b[4 * s4 + 3] = v.w;
        }
    }

    float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
    int i1 = -1, i2 = -1;

    // Register staging of the next train tile.
    using Stg = std::conditional_t<RAW, float, float4>;
    Stg stg[PER];
    float nstg = 0.f;
    auto gload = [&](int tile) {
        if constexpr (RAW) l2_gload_raw<DP, TR>(tsrc, nt, dim, tnorm, tile, stg, nstg);
        else l2_gload<DP, TR>(tsrc, tnorm, tile, stg, nstg);
    };
    auto lstore = [&](int buf) {
        if constexpr (RAW) l2_lstore_raw<DP, TR>(lds + buf * TR * ROWF, lnorm + buf * TR, stg, nstg);
        else l2_lstore<DP, TR>(lds + buf * TR * ROWF, lnorm + buf * TR, stg, nstg);
    };

    if (tBegin < tEnd) {
        gload(tBegin);
        lstore(0);
    }
    __syncthreads();
    for (int t = tBegin; t < tEnd; ++t) {
        const int buf = (t - tBegin) & 1;
        const bool more = t + 1 < tEnd;
        // next tile's loads in flight under this tile's MFMAs (the last trip reloads its own tile
        // into the idle buffer: no branch around the staging registers)
        gload(more ? t + 1 : t);
        // the tile's norms for this lane's rows (8j + 4h .. 8j + 4h + 3 of each chain: 4 b128 reads),
        // fetched ahead of the MFMA chain so the epilogue never waits on LDS
        float4 nv[NC][4];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                nv[c][j] = *reinterpret_cast<const float4*>(&lnorm[buf * TR + 32 * c + 8 * j + 4 * h]);
        floatx16 acc[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
#pragma unroll
        for (int s4 = 0; s4 < KS / 4; ++s4) {
            float4 a[NC];
#pragma unroll
            for (int c = 0; c < NC; ++c)
                a[c] = *reinterpret_cast<const float4*>(&lds[buf * TR * ROWF + (32 * c + col) * ROWF + h * KS + 4 * s4]);
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c].x, b[4 * s4 + 0], acc[c], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c].y, b[4 * s4 + 1], acc[c], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c].z, b[4 * s4 + 2], acc[c], 0, 0, 0);
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c].w, b[4 * s4 + 3], acc[c], 0, 0, 0);
        }
        // epilogue: lane = query col, register r of chain c = train row 32c + (r&3) + 8(r>>2) + 4h;
        // chains in order, rows ascending within a chain: ascending train index per lane
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 32 * c + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float4 n4 = nv[c][r >> 2];
                const float nrm = (r & 3) == 0 ? n4.x : (r & 3) == 1 ? n4.y : (r & 3) == 2 ? n4.z : n4.w;
                const float s = fmaf(-2.f, acc[c][r], nrm);
                // a score >= b3 (or NaN, which the exact definition never ranks) changes nothing
                if (s < b3) top2b3_push_asc(b1, i1, b2, i2, b3, s, t * TR + row);
            }
        lstore(buf ^ 1);
        __syncthreads();
    }
    // merge the two lane halves that hold the same query
    const float ob1 = __shfl_xor(b1, 32, 64), ob2 = __shfl_xor(b2, 32, 64), ob3 = __shfl_xor(b3, 32, 64);
    const int oi1 = __shfl_xor(i1, 32, 64), oi2 = __shfl_xor(i2, 32, 64);
    if (h == 0) {
        float c1 = b1, c2 = b2, c3 = b3;   // third smallest over both halves' values
        third_fold(c1, c2, c3, ob1);
        third_fold(c1, c2, c3, ob2);
        third_fold(c1, c2, c3, ob3);
        top2_push(b1, i1, b2, i2, ob1, oi1);
        top2_push(b1, i1, b2, i2, ob2, oi2);
        L2Part p;
        p.b1 = b1; p.b2 = b2; p.b3 = c3; p.i1 = i1; p.i2 = i2; p.i3 = -1;
        l2_part_store(part, nqPad, slot, nEmpty, q0 + col, p);
    }
}

// The f32 GEMM form over mcv_l2_prep's padded copies (dim > 128).
template <int DP, int TR>
__global__ __launch_bounds__(256, 2) void mcv_l2_mfma(const float* __restrict__ qp, const float* __restrict__ tp,
                                                     const float* __restrict__ tnorm, int ntTiles,
                                                     int tilesPerChunk, int nqPad, L2Part* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float lds[2 * TR * (DP + 4)];
    __shared__ __attribute__((aligned(16))) float lnorm[2 * TR];
    const int tBegin = blockIdx.y * tilesPerChunk;
    l2_gemm32_body<DP, TR, false>(qp, tp, 0, 0, 0, tnorm, tBegin, min(tBegin + tilesPerChunk, ntTiles), nqPad, part,
                                  blockIdx.x, blockIdx.y, 0, lds, lnorm);
}

// ---- f16-split GEMM form ---------------------------------------------------------------------

// Row-major split copies [nPad][DP] (hi = RN f16 of x, lo = RN f16 of the exact fp32 residual x - hi),
// zero padding, the fp32 squared norms, and the maxima the later launches fold: slot[blockIdx % S] =
// max |x| over the block's rows of both sets (float bits; a non-finite coordinate records +inf, out of
// the f16 domain) and slot[S + blockIdx % S] = max train norm (NaN -> +inf), S = kL2MaxSlots, by one
// atomicMax per block and quantity. The slots sit kL2SlotStride words apart: device atomics on one
// 256-byte span serialise (~12 ns each: 3500 blocks' atomics on 16 adjacent words took the cfg5 share's
// prep from 9.3 to 45 us, scripts/exp/prep_bench.hip; 256-byte spacing 9.9 us). The slots
// come in two sets used by alternate calls: this launch accumulates into `slot` (zeroed by the
// previous call) and zeroes `next` for the call after (stream order separates both from every
// reader). One launch covers both sets (rows of q, then rows of t; grid-stride) and zeroes the
// call's exact-scan queue.
// VEC (dim % 4 == 0, 16-B aligned rows): a lane converts one float4, G = DP / 4 lanes a row, 256 / DP
// rows per wave-trip, two trips' loads in flight; the norm adds the lane's four squares (fmaf chain)
// and then the G lanes' partial sums by an xor tree. Otherwise a wave per row, lane-strided dims.
// Both norm orders are sums of dim fmaf-rounded terms, which the GEMM form's error bound
// (l2_gemm_tol: gamma_dim) covers in any order.
static constexpr int kL2MaxSlots = 16, kL2SlotStride = 64;
static constexpr int kL2PrepBlocksMax = 4096;
struct L2PrepF16 {
    const float* src;
    int n, nPad;
    _Float16* hi;
    _Float16* lo;
    float* norms;
    float padNorm;
};
__device__ __forceinline__ unsigned l2_abs_bits(float v) {
    const float a = fabsf(v);
    return a == a && a < __builtin_inff() ? __float_as_uint(a) : 0x7f800000u;
}
__device__ __forceinline__ unsigned l2_norm_bits(float v) {
    return __float_as_uint(v) > 0x7f800000u ? 0x7f800000u : __float_as_uint(v);   // NaN (any sign) -> +inf
}
template <bool VEC>
__global__ __launch_bounds__(256) void mcv_l2_prep16(L2PrepF16 q, L2PrepF16 t, int dim, int DP, int* __restrict__ ambCount,
                                                     unsigned* __restrict__ slot, unsigned* __restrict__ next) {
    __shared__ unsigned red[2][4];
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) *ambCount = 0;   // the exact-scan queue of this call
        if (threadIdx.x < 2 * kL2MaxSlots) next[threadIdx.x * kL2SlotStride] = 0u;
    }
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    const int nrows = q.nPad + t.nPad;
    unsigned m = 0, mt = 0;
    if constexpr (VEC) {
        const int G = DP / 4, RW = 64 / G;   // lanes per row, rows per wave-trip (q.nPad % RW == 0)
        const int sub = lane / G, c = lane % G;
        typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
        auto row_of = [&](int rr, bool& isq, int& r) {
            isq = rr < q.nPad;
            r = isq ? rr : rr - q.nPad;
        };
        for (int r0 = wave * RW; r0 < nrows; r0 += 2 * nw * RW) {
            // two wave-trips: rows r0 + sub and r0 + nw RW + sub, both loads issued first
            float4 v[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int rr = r0 + u * nw * RW + sub;
                bool isq;
                int r;
                row_of(rr, isq, r);
                const int n = isq ? q.n : t.n;
                const float* src = isq ? q.src : t.src;
                v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (rr < nrows && r < n && 4 * c < dim) v[u] = *reinterpret_cast<const float4*>(src + (size_t)r * dim + 4 * c);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int rr = r0 + u * nw * RW + sub;
                if (r0 + u * nw * RW >= nrows) break;   // wave-uniform
                bool isq;
                int r;
                row_of(rr, isq, r);
                const float x[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
                _Float16 hx[4], lx[4];
                float acc = 0.f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    hx[e] = (_Float16)x[e];
                    lx[e] = (_Float16)(x[e] - (float)hx[e]);
                    acc = fmaf(x[e], x[e], acc);
                    const unsigned b = l2_abs_bits(x[e]);
                    m = b > m ? b : m;
                }
                for (int off = G / 2; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
                if (rr < nrows) {
                    _Float16* hi = isq ? q.hi : t.hi;
                    _Float16* lo = isq ? q.lo : t.lo;
                    *reinterpret_cast<f16x4*>(hi + (size_t)r * DP + 4 * c) = f16x4{hx[0], hx[1], hx[2], hx[3]};
                    *reinterpret_cast<f16x4*>(lo + (size_t)r * DP + 4 * c) = f16x4{lx[0], lx[1], lx[2], lx[3]};
                    if (c == 0) {
                        const int n = isq ? q.n : t.n;
                        (isq ? q.norms : t.norms)[r] = r < n ? acc : (isq ? q.padNorm : t.padNorm);
                        if (!isq && r < n) {
                            const unsigned b = l2_norm_bits(acc);
                            mt = b > mt ? b : mt;
                        }
                    }
                }
            }
        }
    } else {
        for (int rr = wave; rr < nrows; rr += nw) {
            const bool isq = rr < q.nPad;
            const int r = isq ? rr : rr - q.nPad, n = isq ? q.n : t.n;
            const float* src = isq ? q.src : t.src;
            _Float16* hi = isq ? q.hi : t.hi;
            _Float16* lo = isq ? q.lo : t.lo;
            float acc = 0.f;
            for (int k = lane; k < DP; k += 64) {
                const float v = (r < n && k < dim) ? src[(size_t)r * dim + k] : 0.f;
                const _Float16 hv = (_Float16)v;
                hi[(size_t)r * DP + k] = hv;
                lo[(size_t)r * DP + k] = (_Float16)(v - (float)hv);
                acc = fmaf(v, v, acc);
                const unsigned b = l2_abs_bits(v);
                m = b > m ? b : m;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
            if (lane == 0) {
                (isq ? q.norms : t.norms)[r] = r < n ? acc : (isq ? q.padNorm : t.padNorm);
                if (!isq && r < n) {
                    const unsigned b = l2_norm_bits(acc);
                    mt = b > mt ? b : mt;
                }
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const unsigned o = __shfl_xor(m, off, 64), ot = __shfl_xor(mt, off, 64);
        m = o > m ? o : m;
        mt = ot > mt ? ot : mt;
    }
    if (lane == 0) red[0][threadIdx.x >> 6] = m, red[1][threadIdx.x >> 6] = mt;
    __syncthreads();
    if (threadIdx.x < 2) {
        unsigned r = 0;
        for (int w = 0; w < 4; ++w) r = red[threadIdx.x][w] > r ? red[threadIdx.x][w] : r;
        if (r) atomicMax(slot + (threadIdx.x * kL2MaxSlots + blockIdx.x % kL2MaxSlots) * kL2SlotStride, r);
    }
}

// A tile's scores (s = |t|^2 - 2 q.t from the two accumulator chains) -> the lane's running top-2 /
// third place (train rows in ascending index order across calls with increasing ranges). One
// wave-level test first: the tile's 16 scores per lane reduced by a min (v_min3), and the insertions
// (each behind its own s < b3: a score >= b3 changes neither the top-2 nor the third place) only when
// some lane's minimum beats its third place — past the first tiles one compare and one skipped branch
// per tile (round 4: against a compare-and-branch per score, 1.876-1.879 vs 1.886-1.891 ms at cfg5).
// The index carried is the tile-row index without the lane half's 4 h (wave-uniform, an SGPR operand
// of the selects); the caller adds 4 h to i1 / i2 at the end.
template <int NC>
__device__ __forceinline__ void l2_epilogue16(const floatx16 (&am)[NC], const floatx16 (&as)[NC], const float4 (&nv)[NC][4],
                                               int base, float& b1, int& i1, float& b2, int& i2, float& b3) {
    float sv[NC][16];
    float mn = __builtin_inff();
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float4 n4 = nv[c][r >> 2];
            const float nrm = (r & 3) == 0 ? n4.x : (r & 3) == 1 ? n4.y : (r & 3) == 2 ? n4.z : n4.w;
            sv[c][r] = fmaf(-2.f, am[c][r] + as[c][r], nrm);
            mn = fminf(mn, sv[c][r]);
        }
    if (mn < b3) {
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = 32 * c + (r & 3) + 8 * (r >> 2);
                if (sv[c][r] < b3) top2b3_push_asc(b1, i1, b2, i2, b3, sv[c][r], __builtin_amdgcn_readfirstlane(base + row));
            }
    }
}

// The f16-split GEMM form (body of mcv_l2_gemm). Block = WPB waves x 32 QT queries; per train tile of 32 rows and each
// 16-dim k block: A = the tile's hi / lo rows from LDS (one ds_read_b128 each: lane l holds row l & 31,
// dims 16 kb + 8 (l >> 5) + j), B = the wave's queries hi / lo (VGPR-resident, the same dims), three
// accumulator chains (hi.hi, then hi.lo and lo.hi into one) on v_mfma_f32_32x32x16_f16. One
// accumulator set per query set. WPB = 4, QT = 1: blocks of 128 queries, 3 blocks per CU (three waves
// per SIMD, amdgpu_waves_per_eu, overlap one wave's epilogue with the others' MFMAs). Screened in round
// 4 (cfg5): the round-3 form with two accumulator sets in turn 2.07 ms; QT = 2 at two waves per SIMD
// (252 VGPRs) 2.17 ms, at one wave per SIMD 2.98 ms; s_setprio 1 around the MFMA cluster 1.95 ms;
// 8-wave blocks 2.36 ms; four waves per SIMD (23 spilled VGPRs) 2.55 ms; the round-4 form 1.88 ms.
// Staging (round 5): the next tile arrives by LDS-DMA (global_load_lds_dwordx4: no staging registers,
// no ds_write pass), issued at the top of the current tile and retired by the tile's closing barrier.
// The DMA writes each wave-instruction's 64 x 16 B contiguously, so the tile image is unpadded
// [32 rows][DP halves] with its 16-byte chunks XOR-swizzled per row (chunk c of row r at c ^ key(r),
// key(r) = (r / (256 B / row bytes)) mod chunks per row; the swizzle goes on the DMA's per-lane source
// address): the fragment reads of 16 consecutive rows then hit 16 distinct 4-bank groups, as the
// padded rows of the register-staged form did.
template <int DP>
__device__ __forceinline__ int l2_swz_key(int r) {
    constexpr int RB = DP * 2, CPR = DP / 8;   // row bytes, 16-byte chunks per row
    return (r / (256 / RB)) & (CPR - 1);
}

template <int DP, int TR, int WPB>
__device__ __forceinline__ void l2_glds16(const _Float16* __restrict__ th, const _Float16* __restrict__ tl,
                                          const float* __restrict__ tnorm, int tile, _Float16* lh, _Float16* ll,
                                          float* ln) {
    typedef __attribute__((address_space(3))) void* lptr;
    typedef __attribute__((address_space(1))) void* gptr;
    constexpr int RB = DP * 2, PIECES = TR * RB / 1024;   // 1 KiB wave-instructions per image
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int arr = 0; arr < 2; ++arr) {
#pragma unroll
        for (int i = 0; i < (PIECES + WPB - 1) / WPB; ++i) {
            const int piece = wave + WPB * i;
            if (PIECES % WPB == 0 || piece < PIECES) {
                const int o = piece * 1024 + 16 * lane;   // byte offset in the image
                const int r = o / RB, c = ((o % RB) >> 4) ^ l2_swz_key<DP>(r);
                const _Float16* src = (arr ? tl : th) + ((size_t)tile * TR + r) * DP + 8 * c;
                __builtin_amdgcn_global_load_lds((gptr)src, (lptr)((arr ? ll : lh) + piece * 512), 16, 0, 0);
            }
        }
    }
    if (wave == WPB - 1 && lane < TR)
        __builtin_amdgcn_global_load_lds((gptr)(tnorm + (size_t)tile * TR + lane), (lptr)ln, 4, 0, 0);
}

template <int DP, int WPB, int QT>
__device__ __forceinline__ void l2_gemm16_body(const _Float16* __restrict__ qh, const _Float16* __restrict__ ql,
                                               const _Float16* __restrict__ th, const _Float16* __restrict__ tl,
                                               const float* __restrict__ tnorm, int tBegin, int tEnd,
                                               int nqPad, L2Part* __restrict__ part, int bx, int slot, int nEmpty,
                                               _Float16* __restrict__ img, float* __restrict__ lnb) {
    constexpr int TR = 32;
    constexpr int KB = DP / 16;
    constexpr int RB = DP * 2;
    // LDS: two buffers of [hi image | lo image] (TR x DP halves each), norms [2][TR]
    auto lh = [&](int buf) { return img + buf * 2 * TR * DP; };
    auto ll = [&](int buf) { return img + buf * 2 * TR * DP + TR * DP; };
    auto lnorm = [&](int buf) { return lnb + buf * TR; };
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int h = lane >> 5, col = lane & 31;
    const int key = l2_swz_key<DP>(col);
    const int q0 = (bx * WPB + wave) * 32 * QT;
    f16x8 bh[QT][KB], bl[QT][KB];
#pragma unroll
    for (int q = 0; q < QT; ++q) {
        const f16x8* rh = reinterpret_cast<const f16x8*>(qh + (size_t)(q0 + 32 * q + col) * DP + 8 * h);
        const f16x8* rl = reinterpret_cast<const f16x8*>(ql + (size_t)(q0 + 32 * q + col) * DP + 8 * h);
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            bh[q][kb] = rh[2 * kb];
            bl[q][kb] = rl[2 * kb];
        }
    }
    float b1[QT], b2[QT], b3[QT];
    int i1[QT], i2[QT];
#pragma unroll
    for (int q = 0; q < QT; ++q) b1[q] = b2[q] = b3[q] = INFINITY, i1[q] = i2[q] = -1;
    if (tBegin < tEnd) l2_glds16<DP, TR, WPB>(th, tl, tnorm, tBegin, lh(0), ll(0), lnorm(0));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the first tile and the query fragments
    __syncthreads();
    for (int t = tBegin; t < tEnd; ++t) {
        const int buf = (t - tBegin) & 1;
        // the next tile into the idle buffer (its last readers passed the previous tile's barrier)
        if (t + 1 < tEnd) l2_glds16<DP, TR, WPB>(th, tl, tnorm, t + 1, lh(buf ^ 1), ll(buf ^ 1), lnorm(buf ^ 1));
        floatx16 m[QT], sm[QT];
#pragma unroll
        for (int q = 0; q < QT; ++q)
#pragma unroll
            for (int r = 0; r < 16; ++r) m[q][r] = sm[q][r] = 0.f;
        const char* rowh = reinterpret_cast<const char*>(lh(buf)) + col * RB;
        const char* rowl = reinterpret_cast<const char*>(ll(buf)) + col * RB;
        // wave priority 0 for the MFMA block, 1 for the epilogue below: a wave that has its scores
        // gets through its VALU work ahead of the waves issuing MFMAs, and back to the matrix pipe
        // sooner (round 5, same box: GEMM 1.716 vs 1.739-1.747 ms, on another 1.736-1.744 vs 1.769-1.781 ms;
        // priority 1 around the MFMAs instead 1.754-1.762)
        __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            const int p = ((2 * kb + h) ^ key) << 4;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(rowh + p);
            const f16x8 al = *reinterpret_cast<const f16x8*>(rowl + p);
#pragma unroll
            for (int q = 0; q < QT; ++q) m[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[q][kb], m[q], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < QT; ++q) sm[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[q][kb], sm[q], 0, 0, 0);
#pragma unroll
            for (int q = 0; q < QT; ++q) sm[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[q][kb], sm[q], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(1);
        float4 nv[1][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) nv[0][j] = *reinterpret_cast<const float4*>(lnorm(buf) + 8 * j + 4 * h);
#pragma unroll
        for (int q = 0; q < QT; ++q) {
            const floatx16 am[1] = {m[q]}, as[1] = {sm[q]};
            l2_epilogue16<1>(am, as, nv, t * TR, b1[q], i1[q], b2[q], i2[q], b3[q]);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMA of the next tile landed
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < QT; ++q) {
        if (i1[q] >= 0) i1[q] += 4 * h;
        if (i2[q] >= 0) i2[q] += 4 * h;
        const float ob1 = __shfl_xor(b1[q], 32, 64), ob2 = __shfl_xor(b2[q], 32, 64), ob3 = __shfl_xor(b3[q], 32, 64);
        const int oi1 = __shfl_xor(i1[q], 32, 64), oi2 = __shfl_xor(i2[q], 32, 64);
        if (h == 0) {
            float c1 = b1[q], c2 = b2[q], c3 = b3[q];
            third_fold(c1, c2, c3, ob1);
            third_fold(c1, c2, c3, ob2);
            third_fold(c1, c2, c3, ob3);
            float x1 = b1[q], x2 = b2[q];
            int j1 = i1[q], j2 = i2[q];
            top2_push(x1, j1, x2, j2, ob1, oi1);
            top2_push(x1, j1, x2, j2, ob2, oi2);
            L2Part p;
            p.b1 = x1; p.b2 = x2; p.b3 = c3; p.i1 = j1; p.i2 = j2; p.i3 = -1;
            l2_part_store(part, nqPad, slot, nEmpty, q0 + 32 * q + col, p);
        }
    }
}

// One GEMM launch for dim <= 128 whatever the data: the f16-split form inside its domain, else the f32
// form on the caller's rows (l2_gemm32_body<.., RAW>), chosen per wave from mcv_l2_prep16's maxima —
// no host round trip and no second (empty) launch. The two bodies share the LDS (the larger: the f16
// form's 2 x 2 x 32 x (DP + 8) halves) and the f32 body fits the f16 form's register budget (three
// waves per SIMD). XCD-aware (query block, train chunk) order when the chunk count divides 8: blocks
// are dealt round-robin over the 8 XCDs, so chunk = linear block id mod C puts one chunk's train rows
// on each XCD's L2.
// Partition (round 5, stream-K style): the train set is split into C chunks (one per XCD group of
// blocks) and the grid is C x BX resident blocks; block b serves chunk x = b % C (blocks are dealt
// round-robin over the 8 XCDs, so with C = 8 each XCD's L2 holds one chunk) and, within it, the
// contiguous range [j W / BX, (j + 1) W / BX), j = b / C, of the chunk's W = qblocks x tiles
// (query block, tile) steps, query block by query block. Every block gets the same amount of work
// (to a tile), so no round of resident blocks is left partly empty — the (query block, chunk) grid
// this replaces ran 6 rounds for 5.6 rounds of work at cfg5. A (query block, chunk) item split over
// k blocks writes k partials: slot = x G + (j - the block holding the item's first tile), G = the most
// blocks an item spans, and the item's last segment writes empty partials into the slots up to G.
struct L2GemmArgs {
    const _Float16 *qh, *ql, *th, *tl;
    const float *qraw, *traw, *tnorm;
    int nq, nt, dim, ntTiles, nqPad;
    L2Part* part;
    L2Max dom;
    int qblocks, chunks, tilesPerChunk, bx, segs;   // C, the chunk length, BX, G
};
template <int DP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void mcv_l2_gemm(L2GemmArgs a) {
    constexpr int TR = 32, ROWH = DP + 8, ROWF = DP + 4;
    constexpr int HALVES = 2 * 2 * TR * ROWH, FLOATS = 2 * TR * ROWF;
    constexpr int BYTES = (HALVES * 2 > FLOATS * 4 ? HALVES * 2 : FLOATS * 4) + 2 * TR * 4;
    __shared__ __attribute__((aligned(16))) char smem[BYTES];
    float* lnorm = reinterpret_cast<float*>(smem + BYTES - 2 * TR * 4);
    const bool f16 = l2_f16_domain(a.dom);
    const int x = (int)blockIdx.x % a.chunks, j = (int)blockIdx.x / a.chunks;
    const int c0 = x * a.tilesPerChunk;
    const int len = min(a.tilesPerChunk, a.ntTiles - c0);   // this chunk's tiles
    if (len <= 0) return;
    const int64_t W = (int64_t)a.qblocks * len;
    const int64_t end = (int64_t)(j + 1) * W / a.bx;
    // the segments of this block's range, each handed to body(q, tBegin, tEnd, slot, nEmpty)
    auto segments = [&](auto&& body) {
        for (int64_t pos = (int64_t)j * W / a.bx; pos < end;) {
            const int q = (int)(pos / len);
            const int64_t itemStart = (int64_t)q * len, itemEnd = itemStart + len;
            const int64_t segEnd = end < itemEnd ? end : itemEnd;
            const int tBegin = c0 + (int)(pos - itemStart), tEnd = tBegin + (int)(segEnd - pos);
            // the block of this chunk group holding the item's first tile: the largest j0 with j0 W / BX <= itemStart
            const int j0 = (int)(((itemStart + 1) * a.bx - 1) / W);
            const int k = j - j0;
            body(q, tBegin, tEnd, x * a.segs + k, segEnd == itemEnd ? a.segs - 1 - k : 0);
            pos = segEnd;
            __syncthreads();   // the next segment's staging reuses the LDS buffers
        }
    };
    if (f16) {
        _Float16* lh = reinterpret_cast<_Float16*>(smem);
        segments([&](int q, int tBegin, int tEnd, int slot, int nEmpty) {
            l2_gemm16_body<DP, 4, 1>(a.qh, a.ql, a.th, a.tl, a.tnorm, tBegin, tEnd, a.nqPad, a.part, q, slot, nEmpty,
                                     lh, lnorm);
        });
    } else {
        segments([&](int q, int tBegin, int tEnd, int slot, int nEmpty) {
            l2_gemm32_body<DP, TR, true>(a.qraw, a.traw, a.nq, a.nt, a.dim, a.tnorm, tBegin, tEnd, a.nqPad, a.part, q,
                                         slot, nEmpty, reinterpret_cast<float*>(smem), lnorm);
        });
    }
}

__device__ __forceinline__ double l2_exact(const float* __restrict__ q, const float* __restrict__ t, int dim) {
    double d = 0;
    for (int k = 0; k < dim; ++k) {
        const double e = (double)q[k] - (double)t[k];
        d = d + e * e;
    }
    return d;
}

// Both candidates' exact squared distances in one pass (two independent sequential chains; float4
// loads when the rows are 16-byte aligned, issued P float4s ahead of their use: the sums are
// dependent chains, the loads are not). Each sum is l2_exact's, operation for operation.
__device__ __forceinline__ void l2_exact2(const float* __restrict__ q, const float* __restrict__ ta,
                                          const float* __restrict__ tb, int dim, double& da, double& db) {
    double a = 0, b = 0;
    const bool v4 = (dim & 3) == 0 && (((uintptr_t)q | (uintptr_t)ta | (uintptr_t)tb) & 15) == 0;
    if (v4) {
        const float4 *q4 = reinterpret_cast<const float4*>(q), *a4 = reinterpret_cast<const float4*>(ta),
                     *b4 = reinterpret_cast<const float4*>(tb);
        constexpr int P = 8;
        const int n4 = dim / 4;
        float4 x[P], y[P], z[P];
#pragma unroll
        for (int j = 0; j < P; ++j)
            if (j < n4) x[j] = q4[j], y[j] = a4[j], z[j] = b4[j];
        for (int k = 0; k < n4; k += P) {
#pragma unroll
            for (int j = 0; j < P; ++j) {
                if (k + j >= n4) break;
                const double xs[4] = {(double)x[j].x, (double)x[j].y, (double)x[j].z, (double)x[j].w};
                const double ys[4] = {(double)y[j].x, (double)y[j].y, (double)y[j].z, (double)y[j].w};
                const double zs[4] = {(double)z[j].x, (double)z[j].y, (double)z[j].z, (double)z[j].w};
                if (k + P + j < n4) x[j] = q4[k + P + j], y[j] = a4[k + P + j], z[j] = b4[k + P + j];
#pragma unroll
                for (int e4 = 0; e4 < 4; ++e4) {
                    const double e = xs[e4] - ys[e4], f = xs[e4] - zs[e4];
                    a = a + e * e;
                    b = b + f * f;
                }
            }
        }
    } else {
        for (int k = 0; k < dim; ++k) {
            const double x = (double)q[k], e = x - (double)ta[k], f = x - (double)tb[k];
            a = a + e * e;
            b = b + f * f;
        }
    }
    da = a;
    db = b;
}

__device__ __forceinline__ bool lex_less_d(double a, int ia, double b, int ib) {
    return (a < b) | ((a == b) & ((unsigned)ia < (unsigned)ib));
}

// The GEMM form's error bound on a (query, train) score: every train t's exact d^2 >= qn + score(t)
// - tol (qn = the query's fp32 norm, T2 = the largest fp32 train norm).
__device__ __forceinline__ double l2_gemm_tol(double qn, double T2, int dim, bool f16) {
    const double u = 0x1p-24;
    const double qa = sqrt(qn * (1.0 + 1e-6)), T = sqrt(T2);
    if (f16) {
        // f16 split, x = hi + lo + r with |lo| <= 2^-11 |x| + 2^-14, |r| <= 2^-22 |x| + 2^-13 (RN;
        // f16 subnormals flushed or not): q_i t_i - (qh th + qh tl + ql th) <= 3.01 2^-22 |q_i t_i|
        // + 1.0012 2^-13 (|q_i| + |t_i|) + 2^-25 per dim, so with Cauchy-Schwarz the dot's error is
        // E <= |q| T (2.2 dim u (1 + 2^-9) + 2^-20 + 3.02 u) (the f32-accumulated hi.hi chain and the
        // 2 dim-term hi.lo / lo.hi chain, whose terms are below 2^-10 of hi.hi's, at <= 2 u per step;
        // the split; the final add and the score's fma) + 1.25e-4 sqrt(dim) (|q| + T)
        // + dim 2^-25
        const double E = qa * T * (2.2 * dim * u * (1.0 + 0x1p-9) + 0x1p-20 + 3.02 * u) +
                         1.25e-4 * sqrt((double)dim) * (qa + T) + dim * 0x1p-25;
        return 1.01 * ((dim + 4) * u * (T2 + qn) + 2.0 * E) + 1e-30;
    }
    return 1.01 * (dim + 4) * u * (T2 + 2.0 * qa * T + qn) + 1e-30;
}

// Merge the per-chunk top-3s, then make the answer exact: the exact distances of the three GEMM-form
// candidates give the exact top-2 among them; every other train t has GEMM score >= the third's, so
// its exact d^2 >= approx3 - tol (tol bounds the GEMM form's rounding, below); when approx3 - tol
// exceeds the exact second best, no other train can enter the top-2 and the query is done. Otherwise
// (near-ties) it is queued for mcv_l2_exact_scan.
//   tol = 1.01 (dim + 4) u (T2max + 2 |q| sqrt(T2max) + |q|^2)
// covers the fp32 FMA chains of q.t and |t|^2 (gamma_dim each), the fma(-2, q.t, |t|^2), the fp32
// |q|^2 and the sum |q|^2 + s.
__global__ __launch_bounds__(64) void mcv_l2_refine(const L2Part* __restrict__ part, int nq, int nqPad, int nchunks, int nt, int dim,
                              const float* __restrict__ qnorm, L2Max tmax,
                              const float* __restrict__ qraw, const float* __restrict__ traw, int* __restrict__ idx,
                              float* __restrict__ dist, int* __restrict__ idx2, float* __restrict__ dist2,
                              int* __restrict__ ambCount, int* __restrict__ ambList, double* __restrict__ ambE2,
                              L2Max dom) {
    const bool f16 = l2_f16_domain(dom);
    const unsigned T2bits = l2_max_bits(tmax);
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    float b1 = INFINITY, b2 = INFINITY, c1 = INFINITY, c2 = INFINITY, c3 = INFINITY;
    int i1 = -1, i2 = -1;
    // eight partials in flight before the first fold (one load per iteration waited for its own
    // round trip: 16 dependent loads a query at cfg5); the loads past the end re-read the last slot
    // and fold as the empty entry (+inf, -1): an empty entry never displaces anything (lex_less sorts
    // index -1 last), so the fold order and the result are those of the plain loop. The index must be
    // -1 too: (+inf, a real index) would win against an empty second place and duplicate i1.
    for (int c0 = 0; c0 < nchunks; c0 += 8) {
        L2Part pp[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) pp[u] = part[(size_t)min(c0 + u, nchunks - 1) * nqPad + q];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const bool in = c0 + u < nchunks;
            const float s1 = in ? pp[u].b1 : INFINITY, s2 = in ? pp[u].b2 : INFINITY, s3 = in ? pp[u].b3 : INFINITY;
            top2_push(b1, i1, b2, i2, s1, in ? pp[u].i1 : -1);
            top2_push(b1, i1, b2, i2, s2, in ? pp[u].i2 : -1);
            third_fold(c1, c2, c3, s1);
            third_fold(c1, c2, c3, s2);
            third_fold(c1, c2, c3, s3);
        }
    }
    const float* qr = qraw + (size_t)q * dim;
    double e1 = INFINITY, e2 = INFINITY;
    int j1 = -1, j2 = -1;
    const int cand[2] = {i1, i2};
    double ec[2] = {INFINITY, INFINITY};
    // both candidates' sums together (a missing second candidate re-reads the first's row and is
    // skipped below; no candidate at all only when the train set is empty)
    if (i1 >= 0)
        l2_exact2(qr, traw + (size_t)i1 * dim, traw + (size_t)(i2 < 0 ? i1 : i2) * dim, dim, ec[0], ec[1]);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int j = cand[c];
        if (j < 0) continue;
        const double e = ec[c];
        if (lex_less_d(e, j, e1, j1)) { e2 = e1; j2 = j1; e1 = e; j1 = j; }
        else if (lex_less_d(e, j, e2, j2)) { e2 = e; j2 = j; }
    }
    // c3 = the third-smallest GEMM score: every train other than i1, i2 scores >= c3. With nt <= 2 the
    // candidates are every train row, unless a score was inf / NaN (fp32 norms overflow for |x| ~ 1e19
    // while the fp64 sums stay finite): a missing candidate sends the query to the exact scan.
    bool certain = nt == 0 || (nt <= 2 && i1 >= 0 && (nt < 2 || i2 >= 0));
    if (!certain && nt > 2 && i2 >= 0) {
        const double qn = (double)qnorm[q], T2 = (double)__uint_as_float(T2bits);
        const double tol = l2_gemm_tol(qn, T2, dim, f16);
        const double approx3 = (double)qnorm[q] + (double)c3;
        certain = approx3 - tol > e2 * (1.0 + 1e-12);   // every other train is strictly farther
    }
    if (!certain) {
        const int pos = atomicAdd(ambCount, 1);
        ambList[pos] = q;
        ambE2[pos] = j2 >= 0 ? e2 : INFINITY;   // the exact scan's filter bound (>= the true second best)
        return;
    }
    idx[q] = j1;
    dist[q] = j1 >= 0 ? (float)sqrt(e1) : INFINITY;
    if (idx2) idx2[q] = j2;
    if (dist2) dist2[q] = j2 >= 0 ? (float)sqrt(e2) : INFINITY;
}

// Exact scan of the queued queries. Work items = (batch of kL2ScanQ queued queries) x (train chunk),
// sized from the queue length on the device so that the fixed grid of kL2ScanBlocks workgroups is
// filled however few queries are queued (no host round trip): T = kL2ScanBlocks / batches chunks
// per batch (1 when batches >= kL2ScanBlocks). A workgroup stages its batch (fp32, from the raw
// queries through the queue) and then tiles of its chunk's train rows (row-major, straight from the
// caller's train set: the tile is contiguous memory) in LDS; the next tile's loads are in flight in
// registers while the current one is filtered. Per query it keeps the lexicographic (d^2, index) top-2
// of exact sums; an LDS tree merges the block, and mcv_l2_exact_merge folds the chunks in order.
// A certified fp32 filter decides which rows need the exact sum: refine's exact second best of the
// two GEMM candidates, e2c, bounds the true second best, and a row whose fp32 sum s (packed fp32,
// sub + fma per dimension) satisfies s > e2c (1 + (dim + 3) u 1.01) + 1e-30 has exact d^2 > e2c
// (|s - d^2| <= ((1 + gamma_dim)(1 + u)^2 - 1) d^2), so it can enter no top-2; every other row
// (a handful per query, NaN sums included) gets the exact fp64 sum in dim order — the oracle's
// summation, bit for bit (the query's fp64 values are its fp32 ones widened, as the oracle's).
// The tile replaced a lane-per-row walk over a transposed train copy whose dependent loads left the
// scan latency-bound (64 us at the 8-rank share, whatever the queue length; 42 us with no exact row).
static constexpr int kL2ScanQ = 32;
static constexpr int kL2ScanThreads = 1024;   // dim > 128: one 16-wave workgroup per CU
static constexpr int kL2ScanThreadsU = 512;   // dim <= 128 (mcv_l2_scan): 8 waves, 256 VGPRs each
static constexpr int kL2ScanBlocks = 256;
static constexpr int kL2TileFloats = 128 * 132;   // train tile: 128 rows of dimPad <= 128 (+4 pad)

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct L2Top2d { double d1, d2; int j1, j2; };

__device__ __forceinline__ void top2d_push(double& a1, int& k1, double& a2, int& k2, double e, int j) {
    if (lex_less_d(e, j, a1, k1)) { a2 = a1; k2 = k1; a1 = e; k1 = j; }
    else if (lex_less_d(e, j, a2, k2)) { a2 = e; k2 = j; }
}

__device__ __forceinline__ int l2_scan_chunks(int nbatch, int blocks) {
    return nbatch >= blocks ? 1 : blocks / nbatch;
}

__device__ __forceinline__ void l2_write_final(int q, const L2Top2d& r, int* idx, float* dist, int* idx2,
                                               float* dist2) {
    idx[q] = r.j1;
    dist[q] = r.j1 >= 0 ? (float)sqrt(r.d1) : INFINITY;
    if (idx2) idx2[q] = r.j2;
    if (dist2) dist2[q] = r.j2 >= 0 ? (float)sqrt(r.d2) : INFINITY;
}

// The exact fp64 distance of one row to one query by a whole wave (every lane active): lane k forms
// the k-th squared difference (each product rounded on its own, as in the sequential loop), then the
// products are added in dimension order off the lanes (v_readlane into an SGPR operand): the oracle's
// sum bit for bit. qcol = the query's fp32 column in LDS (stride kL2ScanQ), row = the tile row.
template <int QS = kL2ScanQ>
__device__ __forceinline__ double l2_exact_row_wave(const float* qcol, const float* row, int dim, int lane) {
    double p[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int k = c * 64 + lane;
        const double df = k < dim ? (double)qcol[k * QS] - (double)row[k] : 0.0;
        p[c] = df * df;
    }
    double d = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const int n = min(64, dim - c * 64);
        if (n <= 0) break;
        const unsigned long long bits = __double_as_longlong(p[c]);
        const int lo = (int)(unsigned)bits, hi = (int)(unsigned)(bits >> 32);
        for (int l = 0; l < n; ++l) {
            const unsigned long long v = (unsigned long long)(unsigned)__builtin_amdgcn_readlane(lo, l) |
                                         ((unsigned long long)(unsigned)__builtin_amdgcn_readlane(hi, l) << 32);
            d = d + __longlong_as_double((long long)v);
        }
    }
    return d;
}

// DPMAX = 128: tiles of 128 rows, 4 (NT = 1024) or 8 (NT = 512) queries per thread; DPMAX = 256: 64
// rows, 2 queries per thread (NT = 1024).
// Thread t filters tile row t % RT against queries (t / RT) * QG .. + QG - 1 (wave-uniform: the
// query values are LDS broadcasts). Work units = the grid's blocks.
template <int DPMAX, int NT>
__device__ __forceinline__ void l2_exact_scan_body(
    const float* __restrict__ qraw, const float* __restrict__ traw, int nt, int dim, int dimPad,
    const int* __restrict__ ambCount, const int* __restrict__ ambList, const double* __restrict__ ambE2,
    L2Top2d* __restrict__ part, int* __restrict__ idx, float* __restrict__ dist, int* __restrict__ idx2,
    float* __restrict__ dist2) {
    constexpr int NW = NT / 64;
    constexpr int RS = DPMAX + 4;                    // tile row stride (floats; 16-B aligned rows)
    constexpr int RT = kL2TileFloats / (128 + 4) * 128 / DPMAX;   // 128 or 64 rows
    constexpr int QG = kL2ScanQ * RT / NT;           // queries per thread: 4 or 2
    constexpr int RSTEP = NT / DPMAX;                // tile rows one pass of the workgroup loads
    constexpr int PER = RT / RSTEP;                  // tile elements per thread
    static_assert(QG == 2 || QG == 4 || QG == 8, "tile shape");
    __shared__ L2Top2d wtop[NW][kL2ScanQ];
    __shared__ double sthr[kL2ScanQ];
    __shared__ __attribute__((aligned(16))) float sq[DPMAX * kL2ScanQ];   // [dimPad][kL2ScanQ]
    __shared__ __attribute__((aligned(16))) float tile[RT * RS];
    const int n = *ambCount;
    const int nbatch = (n + kL2ScanQ - 1) / kL2ScanQ;
    if (nbatch == 0) return;
    const int T = l2_scan_chunks(nbatch, gridDim.x);
    const double F = 1.0 + 1.01 * (dim + 3) * 0x1p-24;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int trow = threadIdx.x % RT, qg = threadIdx.x / RT;
    // tile loads: thread t loads dimension t % DPMAX of rows t / DPMAX + i RSTEP (coalesced along each
    // row; dimensions >= dim load as zeros, an exact +0 in every sum; no division per element)
    const int ek = threadIdx.x & (DPMAX - 1), erb = threadIdx.x / DPMAX;
    const bool kin = ek < dim;
    auto tload = [&](float (&v)[PER], int r0, int re) {
        const float* src = traw + (size_t)(r0 + erb) * dim + ek;
        const int lim = re - r0 - erb;   // rows i RSTEP < lim are inside the chunk
#pragma unroll
        for (int i = 0; i < PER; ++i) v[i] = kin && i * RSTEP < lim ? src[(size_t)i * RSTEP * dim] : 0.f;
    };
    auto tstore = [&](const float (&v)[PER]) {
        float* dst = tile + erb * RS + ek;
#pragma unroll
        for (int i = 0; i < PER; ++i) dst[i * RSTEP * RS] = v[i];
    };
    for (int item = blockIdx.x; item < nbatch * T; item += gridDim.x) {
        const int batch = item / T, chunk = item % T;
        const int a0 = batch * kL2ScanQ;
        const int nb = min(kL2ScanQ, n - a0);
        const int jb = (int)((int64_t)chunk * nt / T), je = (int)((int64_t)(chunk + 1) * nt / T);
        float nxt[PER];
        tload(nxt, jb, je);   // the first tile's loads overlap the batch staging
        {
            // thread t stages query t % kL2ScanQ, dimensions t / kL2ScanQ + i NT / kL2ScanQ: one queue
            // read, then independent loads (the last batch's padding members are zeros, never reported)
            const int b = threadIdx.x % kL2ScanQ;
            const float* qr = b < nb ? qraw + (size_t)ambList[a0 + b] * dim : nullptr;
            for (int k = threadIdx.x / kL2ScanQ; k < dimPad; k += NT / kL2ScanQ)
                sq[k * kL2ScanQ + b] = qr && k < dim ? qr[k] : 0.f;
        }
        if (threadIdx.x < kL2ScanQ) {
            const int b = threadIdx.x;
            const double t = ambE2[a0 + min(b, nb - 1)] * F + 1e-30;
            // near fp32 overflow the filter decides nothing; the padding members skip every row
            sthr[b] = b >= nb ? -INFINITY : t < 1e38 ? t : INFINITY;
        }
        if (lane < kL2ScanQ) wtop[wv][lane] = L2Top2d{INFINITY, INFINITY, -1, -1};
        for (int r0 = jb; r0 < je; r0 += RT) {
            __syncthreads();   // the previous tile's readers are done (and the batch is staged)
            tstore(nxt);
            __syncthreads();
            if (r0 + RT < je) tload(nxt, r0 + RT, je);   // in flight while this tile is filtered
            const float* tr = tile + trow * RS;
            const float* qv = sq + qg * QG;
            f32x2 acc[QG / 2];
#pragma unroll
            for (int p = 0; p < QG / 2; ++p) acc[p] = (f32x2)(0.f);
            // 8 dimensions a trip, every LDS read of the trip issued before the first use; a wave whose
            // queries are all padding members of the last batch skips the trip loop (wave-uniform)
            const int kEnd = qg * QG < nb ? dimPad : 0;
            for (int k = 0; k < kEnd; k += 8) {
                const float4 t4a = *reinterpret_cast<const float4*>(tr + k);
                const float4 t4b = *reinterpret_cast<const float4*>(tr + k + 4);
                f32x2 qk[8][QG / 2];
#pragma unroll
                for (int kk = 0; kk < 8; ++kk)
#pragma unroll
                    for (int p = 0; p < QG / 2; ++p)
                        qk[kk][p] = *reinterpret_cast<const f32x2*>(qv + (k + kk) * kL2ScanQ + 2 * p);
                const float tk[8] = {t4a.x, t4a.y, t4a.z, t4a.w, t4b.x, t4b.y, t4b.z, t4b.w};
#pragma unroll
                for (int kk = 0; kk < 8; ++kk) {
                    const f32x2 tv = (f32x2)(tk[kk]);
#pragma unroll
                    for (int p = 0; p < QG / 2; ++p) {
                        const f32x2 df = qk[kk][p] - tv;
                        acc[p] = __builtin_elementwise_fma(df, df, acc[p]);
                    }
                }
            }
            uint32_t pend = 0;
            if (r0 + trow < je) {
#pragma unroll
                for (int p = 0; p < QG / 2; ++p) {
                    pend |= (uint32_t)!((double)acc[p].x > sthr[qg * QG + 2 * p]) << (2 * p);
                    pend |= (uint32_t)!((double)acc[p].y > sthr[qg * QG + 2 * p + 1]) << (2 * p + 1);
                }
            }
            // the rows the filter kept: exact sums by the whole wave, one (row, query) at a time
            uint64_t m = __ballot(pend != 0);
            while (m) {
                const int l = __ffsll((unsigned long long)m) - 1;
                m &= m - 1;
                const int rl = __builtin_amdgcn_readlane(trow, l);
                uint32_t pb = (uint32_t)__builtin_amdgcn_readlane((int)pend, l);
                while (pb) {
                    const int b = qg * QG + __builtin_ctz(pb);
                    pb &= pb - 1;
                    const double d = l2_exact_row_wave(sq + b, tile + rl * RS, dim, lane);
                    L2Top2d w = wtop[wv][b];
                    top2d_push(w.d1, w.j1, w.d2, w.j2, d, r0 + rl);
                    if (lane == 0) wtop[wv][b] = w;
                }
            }
        }
        __syncthreads();
        // fold the waves' top-2s (lexicographic: the order of candidates does not matter)
        if (threadIdx.x < nb) {
            const int b = threadIdx.x;
            L2Top2d r{INFINITY, INFINITY, -1, -1};
            for (int w = 0; w < NW; ++w) {
                const L2Top2d x = wtop[w][b];
                top2d_push(r.d1, r.j1, r.d2, r.j2, x.d1, x.j1);
                top2d_push(r.d1, r.j1, r.d2, r.j2, x.d2, x.j2);
            }
            if (T == 1) l2_write_final(ambList[a0 + b], r, idx, dist, idx2, dist2);
            else part[(size_t)(a0 + b) * T + chunk] = r;
        }
        __syncthreads();
    }
}

// Exact scan of the queued queries, f16 domain (round 4): the filter is the GEMM form itself. A
// (batch of 32 queued queries, train chunk) item runs the f16-split MFMA chains of mcv_l2_gemm
// over the chunk's 32-row tiles (A fragments straight from the split train copy, B = the batch's
// queries gathered through the queue), 4 waves taking tiles in turn; a (query, row) whose GEMM score
// is at most thr = e2 (1 + 1e-12) + tol - qn (refine's bound: every row's exact d^2 >= qn + score -
// tol, so a row above it cannot enter the top-2) gets the exact fp64 sum (the whole wave, lane-
// parallel, the oracle's order). About as many rows survive as with the fp32 filter (the ambiguous
// queries' near-ties), for 3 MFMAs per 16 dims instead of 2 packed VALU ops per dimension.
template <int DP>
__device__ __forceinline__ void l2_scan16_body(
    const _Float16* __restrict__ qh, const _Float16* __restrict__ ql, const _Float16* __restrict__ th,
    const _Float16* __restrict__ tl, const float* __restrict__ tnorm, const float* __restrict__ qnorm,
    unsigned tmaxBits, const float* __restrict__ qraw, const float* __restrict__ traw, int nt,
    int ntTiles, int dim, const int* __restrict__ ambCount, const int* __restrict__ ambList,
    const double* __restrict__ ambE2, L2Top2d* __restrict__ part, int* __restrict__ idx, float* __restrict__ dist,
    int* __restrict__ idx2, float* __restrict__ dist2) {
    // the block runs SB = NT / 256 independent 256-thread units (work units = SB x blocks); every
    // unit takes the same number of item rounds, so the block-wide barriers stay matched
    constexpr int KB = DP / 16, NW = 4, SB = kL2ScanThreadsU / 256;
    __shared__ L2Top2d wtop[SB][NW][kL2ScanQ];
    __shared__ float sthr[SB][kL2ScanQ];
    const int n = *ambCount;
    const int nbatch = (n + kL2ScanQ - 1) / kL2ScanQ;
    if (nbatch == 0) return;
    const int units = gridDim.x * SB;
    const int T = l2_scan_chunks(nbatch, units);
    const double T2 = (double)__uint_as_float(tmaxBits);
    const int sb = threadIdx.x >> 8, tid = threadIdx.x & 255;
    const int wv = tid >> 6, lane = tid & 63, h = lane >> 5, col = lane & 31;
    for (int base = blockIdx.x * SB; base < nbatch * T; base += units) {
        const int item = base + sb;
        const bool act = item < nbatch * T;
        const int batch = act ? item / T : 0, chunk = act ? item % T : 0;
        const int a0 = batch * kL2ScanQ;
        const int nb = act ? min(kL2ScanQ, n - a0) : 0;
        const int tb = (int)((int64_t)chunk * ntTiles / T), te = act ? (int)((int64_t)(chunk + 1) * ntTiles / T) : tb;
        if (tid < kL2ScanQ) {
            const int b = tid;
            float thr = -INFINITY;   // padding members keep nothing
            if (b < nb) {
                const int q = ambList[a0 + b];
                const double qn = (double)qnorm[q];
                const double x = ambE2[a0 + b] * (1.0 + 1e-12) + l2_gemm_tol(qn, T2, dim, true) - qn;
                // rounded up (and a little more) to fp32: the fp32 compare keeps a superset
                thr = x < 0x1p120 ? __double2float_ru(x + fabs(x) * 0x1p-40) : INFINITY;
            }
            sthr[sb][b] = thr;
        }
        if (lane < kL2ScanQ) wtop[sb][wv][lane] = L2Top2d{INFINITY, INFINITY, -1, -1};
        __syncthreads();
        const int qc = col < nb ? ambList[a0 + col] : -1;
        const float myThr = sthr[sb][col];
        f16x8 bh[KB], bl[KB];
        {
            const f16x8 z = (f16x8)((_Float16)0);
            const f16x8* rh = reinterpret_cast<const f16x8*>(qh + (size_t)(qc < 0 ? 0 : qc) * DP + 8 * h);
            const f16x8* rl = reinterpret_cast<const f16x8*>(ql + (size_t)(qc < 0 ? 0 : qc) * DP + 8 * h);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                bh[kb] = qc < 0 ? z : rh[2 * kb];
                bl[kb] = qc < 0 ? z : rl[2 * kb];
            }
        }
        for (int t = tb + wv; t < te; t += NW) {
            floatx16 m, sm;
#pragma unroll
            for (int r = 0; r < 16; ++r) m[r] = sm[r] = 0.f;
            const f16x8* ah8 = reinterpret_cast<const f16x8*>(th + ((size_t)t * 32 + col) * DP + 8 * h);
            const f16x8* al8 = reinterpret_cast<const f16x8*>(tl + ((size_t)t * 32 + col) * DP + 8 * h);
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const f16x8 ah = ah8[2 * kb], al = al8[2 * kb];
                m = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bh[kb], m, 0, 0, 0);
                sm = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, bl[kb], sm, 0, 0, 0);
                sm = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, bh[kb], sm, 0, 0, 0);
            }
            // lane (query col, half h) holds rows (r & 3) + 8 (r >> 2) + 4 h of the tile
            uint32_t keep = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 n4 = *reinterpret_cast<const float4*>(tnorm + (size_t)t * 32 + 8 * j + 4 * h);
                const float nn[4] = {n4.x, n4.y, n4.z, n4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * j + i;
                    const float sc = fmaf(-2.f, m[r] + sm[r], nn[i]);
                    keep |= (uint32_t)(sc <= myThr) << r;
                }
            }
            uint64_t mk = __ballot(keep != 0);
            while (mk) {
                const int l = __ffsll((unsigned long long)mk) - 1;
                mk &= mk - 1;
                uint32_t pb = (uint32_t)__builtin_amdgcn_readlane((int)keep, l);
                const int q = __builtin_amdgcn_readlane(qc, l);
                const int bq = l & 31, hh = l >> 5;
                while (pb) {
                    const int r = __builtin_ctz(pb);
                    pb &= pb - 1;
                    const int row = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
                    if (row >= nt) continue;   // padding rows (never below a finite threshold anyway)
                    const double d = l2_exact_row_wave<1>(qraw + (size_t)q * dim, traw + (size_t)row * dim, dim, lane);
                    L2Top2d w = wtop[sb][wv][bq];
                    top2d_push(w.d1, w.j1, w.d2, w.j2, d, row);
                    if (lane == 0) wtop[sb][wv][bq] = w;
                }
            }
        }
        __syncthreads();
        if (tid < nb) {
            const int b = tid;
            L2Top2d r{INFINITY, INFINITY, -1, -1};
            for (int w = 0; w < NW; ++w) {
                const L2Top2d x = wtop[sb][w][b];
                top2d_push(r.d1, r.j1, r.d2, r.j2, x.d1, x.j1);
                top2d_push(r.d1, r.j1, r.d2, r.j2, x.d2, x.j2);
            }
            if (T == 1) l2_write_final(ambList[a0 + b], r, idx, dist, idx2, dist2);
            else part[(size_t)(a0 + b) * T + chunk] = r;
        }
        __syncthreads();
    }
}

// The exact scan of the queued queries, one launch for dim <= 128: the MFMA-filtered form in the f16
// domain (2 x kL2ScanBlocks units of 256 threads), else the fp32-filter form (kL2ScanBlocks units; at
// 512 threads the rare out-of-domain scan runs half the waves of the dim > 128 one).
struct L2ScanArgs {
    const _Float16 *qh, *ql, *th, *tl;
    const float *tnorm, *qnorm, *qraw, *traw;
    int nt, ntTiles, dim, dimPad;
    const int *ambCount, *ambList;
    const double* ambE2;
    L2Top2d* part;
    int* idx;
    float* dist;
    int* idx2;
    float* dist2;
    L2Max dom, tmax;
};
template <int DP>
__global__ __launch_bounds__(kL2ScanThreadsU) void mcv_l2_scan(L2ScanArgs a) {
    if (l2_f16_domain(a.dom))
        l2_scan16_body<DP>(a.qh, a.ql, a.th, a.tl, a.tnorm, a.qnorm, l2_max_bits(a.tmax), a.qraw, a.traw, a.nt,
                           a.ntTiles, a.dim, a.ambCount, a.ambList, a.ambE2, a.part, a.idx, a.dist, a.idx2, a.dist2);
    else
        l2_exact_scan_body<128, kL2ScanThreadsU>(a.qraw, a.traw, a.nt, a.dim, a.dimPad, a.ambCount, a.ambList, a.ambE2,
                                                 a.part, a.idx, a.dist, a.idx2, a.dist2);
}

// dim > 128: the fp32-filter form alone.
template <int DPMAX>
__global__ __launch_bounds__(kL2ScanThreads) void mcv_l2_exact_scan(L2ScanArgs a) {
    l2_exact_scan_body<DPMAX, kL2ScanThreads>(a.qraw, a.traw, a.nt, a.dim, a.dimPad, a.ambCount, a.ambList, a.ambE2,
                                              a.part, a.idx, a.dist, a.idx2, a.dist2);
}

// Fold the per-chunk top-2s of each queued query (T > 1 only): one wave per query, lanes over the
// chunks, then a lexicographic butterfly (the top-2 of a set does not depend on the fold order).
__global__ __launch_bounds__(256) void mcv_l2_exact_merge(const int* __restrict__ ambCount,
                                                          const int* __restrict__ ambList,
                                                          const L2Top2d* __restrict__ part, int* __restrict__ idx,
                                                          float* __restrict__ dist, int* __restrict__ idx2,
                                                          float* __restrict__ dist2, int blocks, L2Max dom) {
    // the scan's work units: NT / 256 per block in the f16 domain (l2_scan16_body), one otherwise
    const int units = l2_f16_domain(dom) ? blocks * (kL2ScanThreadsU / 256) : blocks;
    const int n = *ambCount;
    const int nbatch = (n + kL2ScanQ - 1) / kL2ScanQ;
    if (nbatch == 0) return;
    const int T = l2_scan_chunks(nbatch, units);
    if (T == 1) return;
    const int lane = threadIdx.x & 63;
    for (int a = blockIdx.x * 4 + (threadIdx.x >> 6); a < n; a += gridDim.x * 4) {
        L2Top2d r{INFINITY, INFINITY, -1, -1};
        for (int c = lane; c < T; c += 64) {
            const L2Top2d p = part[(size_t)a * T + c];
            top2d_push(r.d1, r.j1, r.d2, r.j2, p.d1, p.j1);
            top2d_push(r.d1, r.j1, r.d2, r.j2, p.d2, p.j2);
        }
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const double o1 = __shfl_xor(r.d1, off, 64), o2 = __shfl_xor(r.d2, off, 64);
            const int k1 = __shfl_xor(r.j1, off, 64), k2 = __shfl_xor(r.j2, off, 64);
            top2d_push(r.d1, r.j1, r.d2, r.j2, o1, k1);
            top2d_push(r.d1, r.j1, r.d2, r.j2, o2, k2);
        }
        if (lane == 0) l2_write_final(ambList[a], r, idx, dist, idx2, dist2);
    }
}

struct L2Work {
    DevBuf<float> qp, tp, qn, tn;      // f32 padded copies (dim > 128), squared norms
    DevBuf<L2Part> part;
    DevBuf<unsigned> tmax;             // dim > 128: the train norms' maximum (mcv_l2_umax)
    DevBuf<int> amb;   // [0] = count, [1..] = queued queries
    DevBuf<L2Top2d> scanPart;   // exact-scan partials: < 4 kL2ScanBlocks x kL2ScanQ records
    DevBuf<_Float16> qh, ql, th, tl;   // f16-split copies (dim <= 128)
    DevBuf<unsigned> maxPart;          // dim > 128: mcv_l2_umax's per-block maxima (2 x kL2MaxBlocks)
    DevBuf<unsigned> slots;            // mcv_l2_prep16's maxima: two sets of 2 x kL2MaxSlots (strided; zeroed once)
    int slotSet = 0;                   // the set the next call accumulates into
    DevBuf<unsigned> maxCount;         // mcv_l2_umax's finish counter (zeroed once, re-armed by each launch)
    DevBuf<double> ambE2;              // per queued query: the filter bound (refine's exact second best)
    hipStream_t last = nullptr; // stream of the last match (the diagnostics read the queue length there)
    bool lastF16 = false;       // the last match launched the f16-capable path (its form decided on device)
    const unsigned* lastDom = nullptr;   // ... and its domain slots
    bool ran = false;           // a match ran on this thread (its stream may be the null stream)
    StreamFence fence;          // calls on different streams take turns on these buffers
};

// Per host thread and device (DevBuf does not follow a device switch of the calling thread).
static L2Work& l2_work() {
    int d = 0;
    MCV_HIP(hipGetDevice(&d));
    if (d < 0 || d >= 16) fail("cvMatchL2: device %d outside the 16 per-thread workspaces", d);
    thread_local L2Work wk[16];
    return wk[d];
}

// dim <= 128 (the f16-capable path) is five launches, with no host round trip and no empty launch:
//   mcv_l2_prep16 (split copies, norms, per-block maxima) -> mcv_l2_gemm (f16 form or f32 form, decided
//   per wave from the maxima) -> mcv_l2_refine -> mcv_l2_scan (MFMA-filtered or fp32-filter exact scan)
//   -> mcv_l2_exact_merge.
// dim > 128: mcv_l2_prep (padded f32 copies) -> mcv_l2_umax (train-norm maximum) -> mcv_l2_mfma ->
//   mcv_l2_refine -> mcv_l2_exact_scan -> mcv_l2_exact_merge.
int launch_match_l2(const float* d_q, int nq, const float* d_t, int nt, int dim, int* d_idx, float* d_dist,
                    int* d_idx2, float* d_dist2, hipStream_t s) {
    if (dim <= 0 || dim > 256) fail("cvMatchL2: dim %d outside [1, 256]", dim);
    if (nq <= 0) return 0;
    L2Work& wk = l2_work();
    wk.fence.enter(s);
    const int DP = dim <= 32 ? 32 : dim <= 64 ? 64 : dim <= 128 ? 128 : 256;
    const int nqPad = (nq + 255) / 256 * 256;   // whole 128-query blocks
    const bool f16 = DP <= 128;   // the f16-capable path (inside its domain: decided on the device)
    constexpr int TR = 32;        // train rows per tile (f32 form: 32 / 64 screened equal, scripts/sweep_l2.sh)
    const int ntPad = nt > 0 ? (nt + TR - 1) / TR * TR : TR;
    const int ntTiles = ntPad / TR;
    wk.qn.ensure(nqPad);
    wk.tn.ensure(ntPad);
    wk.amb.ensure((size_t)nq + 1);
    wk.ambE2.ensure((size_t)nq);
    L2Max dom{nullptr, 0, 1}, tmax{nullptr, 0, 1};
    if (f16) {
        wk.qh.ensure((size_t)nqPad * DP);
        wk.ql.ensure((size_t)nqPad * DP);
        wk.th.ensure((size_t)ntPad * DP);
        wk.tl.ensure((size_t)ntPad * DP);
        constexpr int setWords = 2 * kL2MaxSlots * kL2SlotStride;
        if (!wk.slots.p) {
            wk.slots.ensure(2 * setWords);
            MCV_HIP(hipMemsetAsync(wk.slots.p, 0, 2 * setWords * sizeof(unsigned), s));
        }
        unsigned* slot = wk.slots.p + setWords * wk.slotSet;
        unsigned* next = wk.slots.p + setWords * (wk.slotSet ^ 1);
        wk.slotSet ^= 1;
        const L2PrepF16 pq{d_q, nq, nqPad, wk.qh.p, wk.ql.p, wk.qn.p, 0.f};
        // padding rows get a +inf norm: their scores are +inf and never enter a top-2 or the third place
        const L2PrepF16 pt{d_t, nt, ntPad, wk.th.p, wk.tl.p, wk.tn.p, __builtin_inff()};
        const bool vec = dim % 4 == 0 && (((uintptr_t)d_q | (uintptr_t)d_t) & 15) == 0;
        // about two rows per lane group in flight per wave: 4096 blocks cover cfg5's 100k rows in ~3 trips
        const int rowsPerBlock = vec ? 4 * (256 / DP) * 2 : 4;
        const int blocks = std::max(1, std::min(kL2PrepBlocksMax, (nqPad + ntPad + rowsPerBlock - 1) / rowsPerBlock));
        if (vec)
            hipLaunchKernelGGL(mcv_l2_prep16<true>, dim3(blocks), dim3(256), 0, s, pq, pt, dim, DP, wk.amb.p, slot, next);
        else
            hipLaunchKernelGGL(mcv_l2_prep16<false>, dim3(blocks), dim3(256), 0, s, pq, pt, dim, DP, wk.amb.p, slot, next);
        dom = L2Max{slot, kL2MaxSlots, kL2SlotStride};
        tmax = L2Max{slot + kL2MaxSlots * kL2SlotStride, kL2MaxSlots, kL2SlotStride};
        wk.lastDom = slot;
    } else {
        wk.qp.ensure((size_t)nqPad * DP);
        wk.tp.ensure((size_t)ntPad * DP);
        wk.tmax.ensure(1);
        if (!wk.maxCount.p) {
            wk.maxCount.ensure(1);
            MCV_HIP(hipMemsetAsync(wk.maxCount.p, 0, sizeof(unsigned), s));
        }
        wk.maxPart.ensure(2 * kL2MaxBlocks);
        MCV_HIP(hipMemsetAsync(wk.amb.p, 0, sizeof(int), s));
        const L2PrepF32 pq{d_q, nq, nqPad, wk.qp.p, wk.qn.p, 0.f};
        const L2PrepF32 pt{d_t, nt, ntPad, wk.tp.p, wk.tn.p, __builtin_inff()};
        hipLaunchKernelGGL(mcv_l2_prep, dim3(l2_prep_blocks(nqPad + ntPad)), dim3(256), 0, s, pq, pt, dim, DP);
        hipLaunchKernelGGL(mcv_l2_umax, dim3(kL2MaxBlocks), dim3(256), 0, s,
                           reinterpret_cast<const unsigned*>(wk.tn.p), nt, nullptr, 0, nullptr, 0, wk.maxPart.p,
                           wk.maxCount.p, wk.tmax.p, nullptr);
        tmax = L2Max{wk.tmax.p, 1, 1};
    }
    const int qblocks = nqPad / 128;
    int nchunks = (2048 + qblocks - 1) / qblocks;
    if (f16) {
        // mcv_l2_gemm's partition: one train chunk per XCD, 3 resident blocks per CU (the f16 form's
        // register budget) split evenly over the chunks, each block an equal range of its chunk's
        // (query block, tile) steps (at least 16 tiles, so small calls keep few partials per query)
        static const int cus = [] {
            int d = 0, n = 0;
            (void)hipGetDevice(&d);
            return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && n > 0 ? n : 256;
        }();
        // (round 5, the same box alternating at cfg5: 1.905-1.909 ms per step against 1.996 ms for the
        // (query block, chunk) grid of 11 chunks chosen by round 4's round-count model)
        int C = std::min(8, ntTiles);
        const int tpc = (ntTiles + C - 1) / C;
        C = (ntTiles + tpc - 1) / tpc;
        int bx = std::max(1, 3 * cus / C);
        bx = (int)std::max<int64_t>(1, std::min<int64_t>(bx, (int64_t)qblocks * tpc / 16));
        int segs = 1;   // the most blocks one (query block, chunk) item spans
        for (int x = 0; x < C; ++x) {
            const int len = std::min(tpc, ntTiles - x * tpc);
            const int64_t W = (int64_t)qblocks * len;
            for (int q = 0; q < qblocks; ++q) {
                const int64_t s0 = (int64_t)q * len, s1 = s0 + len - 1;
                const int64_t j0 = ((s0 + 1) * bx - 1) / W, j1 = ((s1 + 1) * bx - 1) / W;
                segs = std::max<int>(segs, (int)(j1 - j0 + 1));
            }
        }
        nchunks = C * segs;
        wk.part.ensure((size_t)nchunks * nqPad);
        ProfScope ps("l2_mfma", s);
        const L2GemmArgs ga{wk.qh.p, wk.ql.p, wk.th.p, wk.tl.p, d_q, d_t, wk.tn.p, nq, nt, dim, ntTiles, nqPad,
                            wk.part.p, dom, qblocks, C, tpc, bx, segs};
        hipLaunchKernelGGL((DP == 32 ? mcv_l2_gemm<32> : DP == 64 ? mcv_l2_gemm<64> : mcv_l2_gemm<128>),
                           dim3(C * bx), dim3(256), 0, s, ga);
    } else {
        if (nchunks > ntTiles) nchunks = ntTiles;
        if (nchunks < 1) nchunks = 1;
        const int tilesPerChunk = (ntTiles + nchunks - 1) / nchunks;
        nchunks = (ntTiles + tilesPerChunk - 1) / tilesPerChunk;
        wk.part.ensure((size_t)nchunks * nqPad);
        ProfScope ps("l2_mfma", s);
        {
            hipLaunchKernelGGL((mcv_l2_mfma<256, TR>), dim3(qblocks, nchunks), dim3(256), 0, s, wk.qp.p, wk.tp.p,
                               wk.tn.p, ntTiles, tilesPerChunk, nqPad, wk.part.p);
        }
    }
    // one wave per block: the latency-bound exact sums of a rank's few thousand queries spread over
    // every CU (6250 queries: 40 -> 14 us)
    hipLaunchKernelGGL(mcv_l2_refine, dim3((nq + 63) / 64), dim3(64), 0, s, wk.part.p, nq, nqPad, nchunks, nt, dim,
                       wk.qn.p, tmax, d_q, d_t, d_idx, d_dist, d_idx2, d_dist2, wk.amb.p, wk.amb.p + 1,
                       wk.ambE2.p, dom);
    {
        ProfScope ps("l2_exact", s);
        constexpr int scanBlocks = kL2ScanBlocks;
        wk.scanPart.ensure((size_t)scanBlocks * (kL2ScanThreadsU / 256) * kL2ScanQ);
        const int dimPad = (dim + 7) / 8 * 8;   // the fp32 filter's 8-dimension trips over float4 rows
        const L2ScanArgs sa{wk.qh.p, wk.ql.p, wk.th.p, wk.tl.p, wk.tn.p, wk.qn.p, d_q, d_t, nt, ntTiles, dim, dimPad,
                            wk.amb.p, wk.amb.p + 1, wk.ambE2.p, wk.scanPart.p, d_idx, d_dist, d_idx2, d_dist2, dom,
                            tmax};
        if (f16) {
            switch (DP) {
                case 32: hipLaunchKernelGGL(mcv_l2_scan<32>, dim3(scanBlocks), dim3(kL2ScanThreadsU), 0, s, sa); break;
                case 64: hipLaunchKernelGGL(mcv_l2_scan<64>, dim3(scanBlocks), dim3(kL2ScanThreadsU), 0, s, sa); break;
                default: hipLaunchKernelGGL(mcv_l2_scan<128>, dim3(scanBlocks), dim3(kL2ScanThreadsU), 0, s, sa); break;
            }
        } else {
            hipLaunchKernelGGL(mcv_l2_exact_scan<256>, dim3(scanBlocks), dim3(kL2ScanThreads), 0, s, sa);
        }
        // the chunks' top-2s folded by a launch of their own: in the scan's last workgroup the fold is one
        // block's serial chain (+23 us at the 8-rank share, +170 us at 241 queued queries x 32 chunks)
        hipLaunchKernelGGL(mcv_l2_exact_merge, dim3(64), dim3(256), 0, s, wk.amb.p, wk.amb.p + 1, wk.scanPart.p, d_idx,
                           d_dist, d_idx2, d_dist2, scanBlocks, dom);
    }
    MCV_HIP(hipGetLastError());
    wk.fence.leave(s);
    wk.last = s;
    wk.lastF16 = f16;
    wk.ran = true;
    return nq;
}

// Queries the last launch_match_l2 of this thread sent to the exact scan (diagnostics; synchronises
// that launch's stream only).
int l2_last_exact_scans() {
    L2Work& wk = l2_work();
    if (!wk.amb.p) return 0;
    int n = 0;
    MCV_HIP(hipMemcpyAsync(&n, wk.amb.p, sizeof(int), hipMemcpyDeviceToHost, wk.last));
    MCV_HIP(hipStreamSynchronize(wk.last));
    return n;
}

int l2_last_gemm_form() {
    L2Work& wk = l2_work();
    if (!wk.ran) return 0;
    if (!wk.lastF16) return 32;
    unsigned m[kL2MaxSlots * kL2SlotStride];
    MCV_HIP(hipMemcpyAsync(m, wk.lastDom, sizeof(m), hipMemcpyDeviceToHost, wk.last));
    MCV_HIP(hipStreamSynchronize(wk.last));
    unsigned d = 0;
    for (int i = 0; i < kL2MaxSlots; ++i) d = m[i * kL2SlotStride] > d ? m[i * kL2SlotStride] : d;
    return d < kL2F16MaxBits ? 16 : 32;
}

}  // namespace mcv
