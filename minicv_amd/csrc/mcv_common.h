// mcv_common.h — shared definitions for the MI355X MiniCVNative kernels and their host twins.
//
// Everything here is compiled twice: for gfx950 (kernels) and for x86-64 (shim host code and
// the mcvHost* test hooks). Files that include it are built with -ffp-contract=off so that every
// floating-point expression rounds exactly as written on both sides (bit-exact inlier masks).
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MCV_HD __host__ __device__ __forceinline__
#else
#define MCV_HD inline
#endif

namespace mcv {

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11). Counter-based: hypothesis i's random stream is a pure
// function of (seed, i), so hypotheses can be generated in any order, on any GPU, and replayed
// on the host. Replaces OpenCV's sequential cv::RNG(-1) in RANSACPointSetRegistrator::getSubset
// (documented divergence).
// ---------------------------------------------------------------------------------------------
struct U4 { uint32_t x, y, z, w; };

MCV_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)a * (uint64_t)b) >> 32);
}

MCV_HD U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = mulhi32(M0, c.x), lo0 = M0 * c.x;
        const uint32_t hi1 = mulhi32(M1, c.z), lo1 = M1 * c.z;
        U4 n;
        n.x = hi1 ^ c.y ^ k0;
        n.y = lo1;
        n.z = hi0 ^ c.w ^ k1;
        n.w = lo0;
        c = n;
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// Stream of 32-bit words for one hypothesis. Word s lives in block s/4 (one Philox call per
// block), lane s%4. Counter = {block, hyp_lo, hyp_hi, tag}, key = {seed_lo, seed_hi}.
static const uint32_t kStreamTag = 0x4D435631u;  // "MCV1"

struct HypStream {
    uint32_t k0, k1, hlo, hhi;
    uint32_t block;   // next block to generate
    U4 buf;
    int avail;        // words left in buf (taken from x..w in order)

    MCV_HD void init(uint64_t seed, uint64_t hyp) {
        k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32);
        hlo = (uint32_t)hyp; hhi = (uint32_t)(hyp >> 32);
        block = 0; avail = 0;
        buf.x = buf.y = buf.z = buf.w = 0;
    }
    MCV_HD uint32_t next() {
        if (avail == 0) {
            U4 c; c.x = block; c.y = hlo; c.z = hhi; c.w = kStreamTag;
            buf = philox4x32_10(c, k0, k1);
            ++block;
            avail = 4;
        }
        uint32_t v;
        switch (4 - avail) {
            case 0: v = buf.x; break;
            case 1: v = buf.y; break;
            case 2: v = buf.z; break;
            default: v = buf.w; break;
        }
        --avail;
        return v;
    }
    // Uniform index in [0, n): Lemire multiply-shift (deterministic, integer only).
    MCV_HD int uniform(int n) { return (int)mulhi32(next(), (uint32_t)n); }
};

// Sampler bounds. kMaxAttempts follows RANSACPointSetRegistrator::run's getSubset(..., 10000)
// [ext: OpenCV 4.x ptsetreg.cpp]; kMaxRedraw bounds the duplicate-rejection loop (OpenCV's is
// unbounded; with N >= m it terminates after a few draws in practice).
static const int kMaxAttempts = 10000;
static const int kMaxRedraw = 1000;

// cv::RNG (OpenCV core, [ext]): multiply-with-carry on a 64-bit state,
//   next() : state = (uint64)(unsigned)state * 4164903690 + (unsigned)(state >> 32), returns (unsigned)state
//   uniform(a, b) = a == b ? a : (int)(next() % (b - a) + a)
// RANSACPointSetRegistrator::run seeds one per call with (uint64)-1 and getSubset draws every index
// of every attempt from it, in order (cv_sampler.cpp generates that stream on the host).
struct CvRng {
    uint64_t s;
    MCV_HD uint32_t next() {
        s = (uint64_t)(uint32_t)s * 4164903690u + (uint32_t)(s >> 32);
        return (uint32_t)s;
    }
    MCV_HD int uniform(int a, int b) { return a == b ? a : (int)(next() % (uint32_t)(b - a) + (uint32_t)a); }
};

// Where a hypothesis' minimal sample comes from:
//   table == nullptr: the counter-based Philox stream of (seed, hypothesis) — any order, any GPU;
//   table != nullptr: OpenCV's own sequential stream, precomputed on the host (cv_sampler.cpp,
//     MCV_FLAG_CV_SAMPLER): row `hyp` holds the m indices getSubset accepted for that hypothesis
//     (its duplicate rejection and checkSubset already applied), or -1 in column 0 when getSubset
//     gave up after its 10000 attempts (the loop's `break`).
struct Sampler {
    uint64_t seed;
    const int* table;
};

// Subset source of one hypothesis. next(): 1 = a subset in idx (Philox: the caller still runs
// checkSubset and asks again on failure), 0 = draw again (Philox redraw bound), -1 = no subset.
template <int M>
struct SubsetSrc {
    HypStream rs;
    const int* row;
    MCV_HD SubsetSrc(const Sampler& smp, uint64_t hyp) : row(smp.table ? smp.table + (int64_t)M * (int64_t)hyp : nullptr) {
        rs.init(smp.seed, hyp);
    }
    MCV_HD bool tabled() const { return row != nullptr; }
    MCV_HD int next(int N, int (&idx)[M]);
};

// Per-hypothesis status codes stored in the counts array.
static const int kStatusNoModel = -1;   // minimal solver degenerate -> OpenCV `continue`
static const int kStatusNoSample = -2;  // sampler exhausted attempts -> OpenCV `break`
static const int kStatusRedo = -3;      // packed H sweep: count this slot again with the exact sweep
static const int kF7Slots = 3;          // 7-point fundamental (run7Point): model slots per hypothesis

static const double kDblEpsilon = 2.2204460492503131e-16;
static const float kFltEpsilon = 1.19209290e-07f;

// Draw m distinct indices from [0, N) with duplicate rejection (getSubset's inner loop).
// Returns false if the redraw bound is hit.
template <int M>
MCV_HD bool draw_distinct(HypStream& rs, int N, int (&idx)[M]) {
#pragma unroll
    for (int i = 0; i < M; ++i) {
        int tries = 0;
        int v = rs.uniform(N);
        for (;;) {
            bool dup = false;
#pragma unroll
            for (int j = 0; j < i; ++j) dup |= (idx[j] == v);
            if (!dup) break;
            if (++tries >= kMaxRedraw) return false;
            v = rs.uniform(N);
        }
        idx[i] = v;
    }
    return true;
}

template <int M>
MCV_HD int SubsetSrc<M>::next(int N, int (&idx)[M]) {
    if (row) {
#pragma unroll
        for (int i = 0; i < M; ++i) idx[i] = row[i];
        // a row is a subset of [0, N) by construction (the table is rebuilt whenever N or the points
        // change, ransac_host.cpp); an index outside it ends the stream instead of reading past pts
        bool in = true;
#pragma unroll
        for (int i = 0; i < M; ++i) in = in && (unsigned)idx[i] < (unsigned)N;
        return idx[0] >= 0 && in ? 1 : -1;
    }
    return draw_distinct<M>(rs, N, idx) ? 1 : 0;
}

// Fingerprint of a point buffer (the plan's stale-buffer guards): the sum mod 2^64 over its 32-bit
// words w_i of fp_term(i, w_i). Position-keyed, so a rewrite, a permutation or a resize changes it
// (up to 64-bit collisions); a sum, so the device computes it in any order (plan_guard.hip).
MCV_HD uint64_t fp_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
MCV_HD uint64_t fp_term(uint64_t i, uint32_t w) { return fp_mix(fp_mix(i) ^ (uint64_t)w); }

// v_rcp_f32 + one FMA Newton step: equals the IEEE 1.f / w for every |w| in [2^-126, 2^126)
// (exhaustive GPU check, mcvTestRcpExhaustive mode 3); callers guarantee that range.
MCV_HD float rcp_newton(float w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float r = __builtin_amdgcn_rcpf(w);
    const float e = __builtin_fmaf(-w, r, 1.0f);
    return __builtin_fmaf(e, r, r);
#else
    return 1.0f / w;
#endif
}

// Correctly rounded fp32 reciprocal for every w, without the division expansion: rcp_newton (equal
// to 1.f / w on |w| in [2^-126, 2^126), exhaustively) on w scaled by 2^24 when |w| is denormal (an
// exact power-of-two scaling into that domain; the product by 2^24 afterwards rounds the same way,
// overflow to inf included), +-inf for +-0, NaN for NaN. |w| >= 2^126 takes the IEEE division.
// rcp_newton with v_div_fixup alone misrounds denormal inputs (mcvTestRcpExhaustive mode 2); this
// form is checked over all 2^32 inputs (mode 0). Host: the IEEE division itself.
// rcp_exact for |w| < 2^126 (or NaN) only — callers that bound |w| (the certified sweep's exact
// path: |w| <= Bw (1 + 2^-20) <= 2^50) skip the division branch.
MCV_HD float rcp_exact_bounded(float w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float sc = __builtin_fabsf(w) < 0x1p-126f ? 0x1p24f : 1.0f;
    const float r = rcp_newton(w * sc) * sc;
    return w == 0.0f ? __builtin_copysignf(__builtin_inff(), w) : r;
#else
    return 1.0f / w;
#endif
}

MCV_HD float rcp_exact(float w) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float aw = __builtin_fabsf(w);
    if (__builtin_expect(aw >= 0x1p126f, 0)) return 1.0f / w;
    const float sc = aw < 0x1p-126f ? 0x1p24f : 1.0f;
    const float r = rcp_newton(w * sc) * sc;
    return w == 0.0f ? __builtin_copysignf(__builtin_inff(), w) : r;
#else
    return 1.0f / w;
#endif
}

// fp64 division without the v_div_scale / v_div_fixup wrapper. The IEEE expansion gfx950 runs
// for n / d is div_scale(d), div_scale(n), rcp, two Newton steps, q = n r, rem = fma(-d, q, n),
// div_fmas(rem, r, q), div_fixup: 11 VALU ops. When no operand needs scaling the div_scale ops
// return their inputs (VCC = 0, div_fmas = fma) and div_fixup passes a normal result through, so
//   rcp_f64_refined(d) = the refined reciprocal (5 ops, shared by every quotient over d)
//   div_f64_refined(n, d, r) = n / d bit for bit (3 ops)
// whenever d in +-[2^-64, 2^64] and 2^-900 <= |n| < 2^700 (or n = 0, up to the sign of the zero).
// Callers guard d and argue the n range (mcvTestDivF64 samples both: tests/test_gpu_selftest.py).
// Host: the IEEE division itself.
MCV_HD double rcp_f64_refined(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
#else
    return 1.0 / d;
#endif
}
MCV_HD double div_f64_refined(double n, double d, double r) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double q = n * r;
    const double rem = __builtin_fma(-d, q, n);
    return __builtin_fma(rem, r, q);
#else
    (void)r;
    return n / d;
#endif
}
// The denominator domain of the two helpers above.
MCV_HD bool div_f64_refined_domain(double d) { return __builtin_fabs(d) >= 0x1p-64 && __builtin_fabs(d) <= 0x1p64; }

// sqrt(x) for x in [1, 2] (the 1 + r^2, r <= 1, of a hypot): gfx950's correctly rounded fp64 sqrt
// expansion (v_rsq_f64, then g = x y, h = y / 2 and three fma refinement rounds) without its
// denormal scaling (ldexp by 0 here) and zero / infinity class select (never taken here) — the same
// bits as sqrt(x) on that range, 4 ops shorter on the rotation's dependent chain
// (mcvTestDivF64 mode 4 samples it: tests/test_gpu_selftest.py). Host: sqrt.
MCV_HD double sqrt_f64_1to2(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
#else
    return __builtin_sqrt(x);
#endif
}

}  // namespace mcv
