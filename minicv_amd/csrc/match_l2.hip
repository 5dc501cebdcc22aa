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
// mcv_l2_refine folds the per-chunk top-3s and makes the result exact: the three candidates' exact
//   squared distances (fp64 direct sum in dim order, the oracle's definition) give the top-2 unless a
//   bound on the GEMM form's rounding leaves room for another train (near-ties), in which case the
//   query is queued for mcv_l2_exact_scan (exact distance to every train). idx / dist are then
//   exactly the direct-sum answer: dist = (float)sqrt(exact d^2), ties -> lowest train index.
#include "kernels.h"
#include "mcv_runtime.h"
#include "plan.h"
#include <cmath>
#include <cstdlib>

namespace mcv {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct L2Part { float b1, b2, b3; int i1, i2, i3; };

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
// affects the GEMM form, whose rounding the exact re-rank bounds whatever the order).
__global__ void mcv_l2_prep(const float* __restrict__ src, int n, int dim, int DP, int nPad, float* __restrict__ dst,
                            float* __restrict__ norms, float padNorm, unsigned* __restrict__ unused) {
    const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (r >= nPad) return;
    float acc = 0.f;
    for (int k = lane; k < DP; k += 64) {
        const float v = (r < n && k < dim) ? src[(size_t)r * dim + k] : 0.f;
        dst[(size_t)r * DP + (k & 1) * (DP / 2) + (k >> 1)] = v;
        acc = fmaf(v, v, acc);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) norms[r] = r < n ? acc : padNorm;
}

// max over the real rows' norms (non-negative: float order = bit order); NaN -> +inf.
__global__ __launch_bounds__(1024) void mcv_l2_maxnorm(const float* __restrict__ norms, int n,
                                                      unsigned* __restrict__ out) {
    __shared__ float sm[16];
    float m = 0.f;
    for (int i = threadIdx.x; i < n; i += 1024) {
        const float v = norms[i];
        m = v == v ? fmaxf(m, v) : __builtin_inff();
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 16; ++w) m = fmaxf(m, sm[w]);
        *out = __float_as_uint(m);
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

// TR train rows per tile = TR / 32 independent 32x32 accumulator chains per wave, interleaved
// k-step by k-step (they share the query operands b[]): the matrix pipe never waits on one
// chain's dependent-accumulator latency.
template <int DP, int TR>
__global__ __launch_bounds__(256, 2) void mcv_l2_mfma(const float* __restrict__ qp, const float* __restrict__ tp,
                                                     const float* __restrict__ tnorm, int ntTiles,
                                                     int tilesPerChunk, int nqPad, L2Part* __restrict__ part) {
    constexpr int KS = DP / 2;          // MFMA k-steps (2 dims each)
    constexpr int ROWF = DP + 4;        // padded LDS row, floats
    constexpr int PER = TR * DP / 1024; // float4 staging loads per thread per tile (TR rows x DP)
    constexpr int NC = TR / 32;         // accumulator chains
    __shared__ __attribute__((aligned(16))) float lds[2][TR * ROWF];
    __shared__ __attribute__((aligned(16))) float lnorm[2][TR];

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
    float b1 = INFINITY, b2 = INFINITY, b3 = INFINITY;
    int i1 = -1, i2 = -1;

    // Register staging of the next train tile.
    float4 stg[PER];
    float nstg = 0.f;

    if (tBegin < tEnd) {
        l2_gload<DP, TR>(tp, tnorm, tBegin, stg, nstg);
        l2_lstore<DP, TR>(lds[0], lnorm[0], stg, nstg);
    }
    __syncthreads();
    for (int t = tBegin; t < tEnd; ++t) {
        const int buf = (t - tBegin) & 1;
        const bool more = t + 1 < tEnd;
        // next tile's loads in flight under this tile's MFMAs (the last trip reloads its own tile
        // into the idle buffer: no branch around the staging registers)
        l2_gload<DP, TR>(tp, tnorm, more ? t + 1 : t, stg, nstg);
        // the tile's norms for this lane's rows (8j + 4h .. 8j + 4h + 3 of each chain: 4 b128 reads),
        // fetched ahead of the MFMA chain so the epilogue never waits on LDS
        float4 nv[NC][4];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j) nv[c][j] = *reinterpret_cast<const float4*>(&lnorm[buf][32 * c + 8 * j + 4 * h]);
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
                a[c] = *reinterpret_cast<const float4*>(&lds[buf][(32 * c + col) * ROWF + h * KS + 4 * s4]);
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
                top2b3_push_asc(b1, i1, b2, i2, b3, s, t * TR + row);
            }
        l2_lstore<DP, TR>(lds[buf ^ 1], lnorm[buf ^ 1], stg, nstg);
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
        part[(size_t)blockIdx.y * nqPad + q0 + col] = p;
    }
}

// Exact squared distance (the oracle's definition: fp64 differences, sequential sum in dim order,
// every operation rounded as written).
__device__ __forceinline__ double l2_exact(const float* __restrict__ q, const float* __restrict__ t, int dim) {
    double d = 0;
    for (int k = 0; k < dim; ++k) {
        const double e = (double)q[k] - (double)t[k];
        d = d + e * e;
    }
    return d;
}

__device__ __forceinline__ bool lex_less_d(double a, int ia, double b, int ib) {
    return (a < b) | ((a == b) & ((unsigned)ia < (unsigned)ib));
}

// Merge the per-chunk top-3s, then make the answer exact: the exact distances of the three GEMM-form
// candidates give the exact top-2 among them; every other train t has GEMM score >= the third's, so
// its exact d^2 >= approx3 - tol (tol bounds the GEMM form's rounding, below); when approx3 - tol
// exceeds the exact second best, no other train can enter the top-2 and the query is done. Otherwise
// (near-ties) it is queued for mcv_l2_exact_scan.
//   tol = 1.01 (dim + 4) u (T2max + 2 |q| sqrt(T2max) + |q|^2)
// covers the fp32 FMA chains of q.t and |t|^2 (gamma_dim each), the fma(-2, q.t, |t|^2), the fp32
// |q|^2 and the sum |q|^2 + s.
__global__ void mcv_l2_refine(const L2Part* __restrict__ part, int nq, int nqPad, int nchunks, int nt, int dim,
                              const float* __restrict__ qnorm, const unsigned* __restrict__ tmaxBits,
                              const float* __restrict__ qraw, const float* __restrict__ traw, int* __restrict__ idx,
                              float* __restrict__ dist, int* __restrict__ idx2, float* __restrict__ dist2,
                              int* __restrict__ ambCount, int* __restrict__ ambList) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= nq) return;
    float b1 = INFINITY, b2 = INFINITY, c1 = INFINITY, c2 = INFINITY, c3 = INFINITY;
    int i1 = -1, i2 = -1;
    for (int c = 0; c < nchunks; ++c) {
        const L2Part p = part[(size_t)c * nqPad + q];
        top2_push(b1, i1, b2, i2, p.b1, p.i1);
        top2_push(b1, i1, b2, i2, p.b2, p.i2);
        third_fold(c1, c2, c3, p.b1);
        third_fold(c1, c2, c3, p.b2);
        third_fold(c1, c2, c3, p.b3);
    }
    const float* qr = qraw + (size_t)q * dim;
    double e1 = INFINITY, e2 = INFINITY;
    int j1 = -1, j2 = -1;
    const int cand[2] = {i1, i2};
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int j = cand[c];
        if (j < 0) continue;
        const double e = l2_exact(qr, traw + (size_t)j * dim, dim);
        if (lex_less_d(e, j, e1, j1)) { e2 = e1; j2 = j1; e1 = e; j1 = j; }
        else if (lex_less_d(e, j, e2, j2)) { e2 = e; j2 = j; }
    }
    // c3 = the third-smallest GEMM score: every train other than i1, i2 scores >= c3
    bool certain = nt <= 2;
    if (!certain && i2 >= 0) {
        const double qn = (double)qnorm[q], T2 = (double)__uint_as_float(*tmaxBits);
        const double u = 0x1p-24;
        const double tol = 1.01 * (dim + 4) * u * (T2 + 2.0 * sqrt(qn * (1.0 + 1e-6)) * sqrt(T2) + qn) + 1e-30;
        const double approx3 = (double)qnorm[q] + (double)c3;
        certain = approx3 - tol > e2 * (1.0 + 1e-12);   // every other train is strictly farther
    }
    if (!certain) {
        ambList[atomicAdd(ambCount, 1)] = q;
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
// per batch (1 when batches >= kL2ScanBlocks). The queries sit in LDS as fp64 (broadcast reads);
// each thread streams train rows of its chunk and keeps, per query, the lexicographic (d^2, index)
// top-2 of the exact sums; an LDS tree merges the block, and mcv_l2_exact_merge folds the chunks in
// order. Every sum runs in dim order in one lane: the oracle's summation, bit for bit.
static constexpr int kL2ScanQ = 8;
static constexpr int kL2ScanBlocks = 1024;

struct L2Top2d { double d1, d2; int j1, j2; };

__device__ __forceinline__ void top2d_push(double& a1, int& k1, double& a2, int& k2, double e, int j) {
    if (lex_less_d(e, j, a1, k1)) { a2 = a1; k2 = k1; a1 = e; k1 = j; }
    else if (lex_less_d(e, j, a2, k2)) { a2 = e; k2 = j; }
}

__device__ __forceinline__ int l2_scan_chunks(int nbatch) {
    return nbatch >= kL2ScanBlocks ? 1 : kL2ScanBlocks / nbatch;
}

__device__ __forceinline__ void l2_write_final(int q, const L2Top2d& r, int* idx, float* dist, int* idx2,
                                               float* dist2) {
    idx[q] = r.j1;
    dist[q] = r.j1 >= 0 ? (float)sqrt(r.d1) : INFINITY;
    if (idx2) idx2[q] = r.j2;
    if (dist2) dist2[q] = r.j2 >= 0 ? (float)sqrt(r.d2) : INFINITY;
}

__global__ __launch_bounds__(256) void mcv_l2_exact_scan(const float* __restrict__ qraw, const float* __restrict__ traw,
                                                         int nt, int dim, const int* __restrict__ ambCount,
                                                         const int* __restrict__ ambList, L2Top2d* __restrict__ part,
                                                         int* __restrict__ idx, float* __restrict__ dist,
                                                         int* __restrict__ idx2, float* __restrict__ dist2) {
    __shared__ double qs[kL2ScanQ][256];
    __shared__ double sd1[256], sd2[256];
    __shared__ int sj1[256], sj2[256];
    const int n = *ambCount;
    const int nbatch = (n + kL2ScanQ - 1) / kL2ScanQ;
    if (nbatch == 0) return;
    const int T = l2_scan_chunks(nbatch);
    for (int item = blockIdx.x; item < nbatch * T; item += gridDim.x) {
        const int batch = item / T, chunk = item % T;
        const int a0 = batch * kL2ScanQ;
        const int nb = min(kL2ScanQ, n - a0);
        const int jb = (int)((int64_t)chunk * nt / T), je = (int)((int64_t)(chunk + 1) * nt / T);
        for (int e = threadIdx.x; e < kL2ScanQ * dim; e += 256) {
            const int b = e / dim, k = e % dim;
            qs[b][k] = b < nb ? (double)qraw[(size_t)ambList[a0 + b] * dim + k] : 0.0;
        }
        __syncthreads();
        double e1[kL2ScanQ], e2[kL2ScanQ];
        int j1[kL2ScanQ], j2[kL2ScanQ];
#pragma unroll
        for (int b = 0; b < kL2ScanQ; ++b) { e1[b] = e2[b] = INFINITY; j1[b] = j2[b] = -1; }
        const bool vec4 = (dim & 3) == 0 && ((uintptr_t)traw & 15) == 0;   // 16-byte aligned rows: float4 loads
        for (int j = jb + threadIdx.x; j < je; j += 256) {
            const float* tr = traw + (size_t)j * dim;
            double d[kL2ScanQ];
#pragma unroll
            for (int b = 0; b < kL2ScanQ; ++b) d[b] = 0.0;
            if (vec4) {
                for (int k = 0; k < dim; k += 4) {
                    const float4 t4 = *reinterpret_cast<const float4*>(tr + k);
                    const double tv[4] = {(double)t4.x, (double)t4.y, (double)t4.z, (double)t4.w};
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
                        for (int b = 0; b < kL2ScanQ; ++b) {
                            const double df = qs[b][k + kk] - tv[kk];
                            d[b] = d[b] + df * df;
                        }
                }
            } else {
                for (int k = 0; k < dim; ++k) {
                    const double tv = (double)tr[k];
#pragma unroll
                    for (int b = 0; b < kL2ScanQ; ++b) {
                        const double df = qs[b][k] - tv;
                        d[b] = d[b] + df * df;
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < kL2ScanQ; ++b) top2d_push(e1[b], j1[b], e2[b], j2[b], d[b], j);
        }
#pragma unroll
        for (int b = 0; b < kL2ScanQ; ++b) {
            if (b >= nb) break;   // block-uniform
            sd1[threadIdx.x] = e1[b]; sd2[threadIdx.x] = e2[b]; sj1[threadIdx.x] = j1[b]; sj2[threadIdx.x] = j2[b];
            __syncthreads();
            for (int off = 128; off >= 1; off >>= 1) {
                if (threadIdx.x < off) {
                    double a1 = sd1[threadIdx.x], a2 = sd2[threadIdx.x];
                    int k1 = sj1[threadIdx.x], k2 = sj2[threadIdx.x];
                    top2d_push(a1, k1, a2, k2, sd1[threadIdx.x + off], sj1[threadIdx.x + off]);
                    top2d_push(a1, k1, a2, k2, sd2[threadIdx.x + off], sj2[threadIdx.x + off]);
                    sd1[threadIdx.x] = a1; sd2[threadIdx.x] = a2; sj1[threadIdx.x] = k1; sj2[threadIdx.x] = k2;
                }
                __syncthreads();
            }
            if (threadIdx.x == 0) {
                const L2Top2d r{sd1[0], sd2[0], sj1[0], sj2[0]};
                if (T == 1) l2_write_final(ambList[a0 + b], r, idx, dist, idx2, dist2);
                else part[(size_t)(a0 + b) * T + chunk] = r;
            }
            __syncthreads();
        }
    }
}

// Fold the per-chunk top-2s of each queued query in chunk order (T > 1 only).
__global__ void mcv_l2_exact_merge(const int* __restrict__ ambCount, const int* __restrict__ ambList,
                                   const L2Top2d* __restrict__ part, int* __restrict__ idx, float* __restrict__ dist,
                                   int* __restrict__ idx2, float* __restrict__ dist2) {
    const int n = *ambCount;
    const int nbatch = (n + kL2ScanQ - 1) / kL2ScanQ;
    if (nbatch == 0) return;
    const int T = l2_scan_chunks(nbatch);
    if (T == 1) return;
    for (int a = blockIdx.x * blockDim.x + threadIdx.x; a < n; a += gridDim.x * blockDim.x) {
        L2Top2d r{INFINITY, INFINITY, -1, -1};
        for (int c = 0; c < T; ++c) {
            const L2Top2d p = part[(size_t)a * T + c];
            top2d_push(r.d1, r.j1, r.d2, r.j2, p.d1, p.j1);
            top2d_push(r.d1, r.j1, r.d2, r.j2, p.d2, p.j2);
        }
        l2_write_final(ambList[a], r, idx, dist, idx2, dist2);
    }
}

struct L2Work {
    DevBuf<float> qp, tp, qn, tn;
    DevBuf<L2Part> part;
    DevBuf<unsigned> tmax;
    DevBuf<int> amb;   // [0] = count, [1..] = queued queries
    DevBuf<L2Top2d> scanPart;   // exact-scan partials: < kL2ScanBlocks x kL2ScanQ records
    hipStream_t last = nullptr; // stream of the last match (the diagnostics read the queue length there)
};

static L2Work& l2_work() {
    thread_local L2Work wk;
    return wk;
}

int launch_match_l2(const float* d_q, int nq, const float* d_t, int nt, int dim, int* d_idx, float* d_dist,
                    int* d_idx2, float* d_dist2, hipStream_t s) {
    if (dim <= 0 || dim > 256) fail("cvMatchL2: dim %d outside [1, 256]", dim);
    if (nq <= 0) return 0;
    L2Work& wk = l2_work();
    const int DP = dim <= 32 ? 32 : dim <= 64 ? 64 : dim <= 128 ? 128 : 256;
    const int nqPad = (nq + 127) / 128 * 128;
    static const int TRsel = [] {   // train rows per tile (variant screen: 32 or 64)
        const char* e = getenv("MCV_L2_TR");
        return e && atoi(e) == 64 ? 64 : 32;   // screened equal (scripts/sweep_l2.sh): keep one chain
    }();
    const int TR = DP <= 128 ? TRsel : 32;
    const int ntPad = nt > 0 ? (nt + TR - 1) / TR * TR : TR;
    const int ntTiles = ntPad / TR;
    wk.qp.ensure((size_t)nqPad * DP);
    wk.tp.ensure((size_t)ntPad * DP);
    wk.qn.ensure(nqPad);
    wk.tn.ensure(ntPad);
    wk.tmax.ensure(1);
    wk.amb.ensure((size_t)nq + 1);
    MCV_HIP(hipMemsetAsync(wk.amb.p, 0, sizeof(int), s));
    hipLaunchKernelGGL(mcv_l2_prep, dim3((nqPad + 3) / 4), dim3(256), 0, s, d_q, nq, dim, DP, nqPad, wk.qp.p, wk.qn.p,
                       0.f, (unsigned*)nullptr);
    // padding rows get a +inf norm: their scores are +inf and never enter a top-2 or the third place
    hipLaunchKernelGGL(mcv_l2_prep, dim3((ntPad + 3) / 4), dim3(256), 0, s, d_t, nt, dim, DP, ntPad, wk.tp.p, wk.tn.p,
                       __builtin_inff(), (unsigned*)nullptr);
    hipLaunchKernelGGL(mcv_l2_maxnorm, dim3(1), dim3(1024), 0, s, wk.tn.p, nt, wk.tmax.p);
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
#define MCV_L2_LAUNCH(D, T) hipLaunchKernelGGL((mcv_l2_mfma<D, T>), grid, dim3(256), 0, s, wk.qp.p, wk.tp.p, wk.tn.p, \
                                               ntTiles, tilesPerChunk, nqPad, wk.part.p)
        switch (DP) {
            case 32: if (TR == 64) MCV_L2_LAUNCH(32, 64); else MCV_L2_LAUNCH(32, 32); break;
            case 64: if (TR == 64) MCV_L2_LAUNCH(64, 64); else MCV_L2_LAUNCH(64, 32); break;
            case 128: if (TR == 64) MCV_L2_LAUNCH(128, 64); else MCV_L2_LAUNCH(128, 32); break;
            default: MCV_L2_LAUNCH(256, 32); break;
        }
#undef MCV_L2_LAUNCH
    }
    hipLaunchKernelGGL(mcv_l2_refine, dim3((nq + 255) / 256), dim3(256), 0, s, wk.part.p, nq, nqPad, nchunks, nt, dim,
                       wk.qn.p, wk.tmax.p, d_q, d_t, d_idx, d_dist, d_idx2, d_dist2, wk.amb.p, wk.amb.p + 1);
    {
        ProfScope ps("l2_exact", s);
        wk.scanPart.ensure((size_t)kL2ScanBlocks * kL2ScanQ);
        hipLaunchKernelGGL(mcv_l2_exact_scan, dim3(kL2ScanBlocks), dim3(256), 0, s, d_q, d_t, nt, dim, wk.amb.p,
                           wk.amb.p + 1, wk.scanPart.p, d_idx, d_dist, d_idx2, d_dist2);
        hipLaunchKernelGGL(mcv_l2_exact_merge, dim3(8), dim3(256), 0, s, wk.amb.p, wk.amb.p + 1, wk.scanPart.p, d_idx,
                           d_dist, d_idx2, d_dist2);
    }
    MCV_HIP(hipGetLastError());
    wk.last = s;
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

}  // namespace mcv
