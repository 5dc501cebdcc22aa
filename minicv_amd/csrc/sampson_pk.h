// sampson_pk.h — certified packed-fp32 prefilter of the fp64 Sampson inlier test (F and E sweeps).
//
// The reference decides inlier <=> (float)(c * c / den) <= thr2 with c, den evaluated in fp64
// (f_err_sampson[_fused]). The sweep evaluates c and den in fp32 instead — two models per
// v_pk_fma_f32: 15 packed FMAs + 1 packed multiply for c and den, then c^2 and two linear cuts in den
// (1 packed multiply + 2 packed FMAs, spk_cut1) and 4 compares per model pair, i.e. 11.75 VALU issue
// slots per (model, correspondence) against 22 for the fp64 test — and decides every lane whose fp32
// values are far enough from the threshold to make the fp64 answer certain; the rest (a fraction
// ~1e-4 of evaluations) take the exact fp64 test.
//
// Error bound (u = 2^-24; inputs |x1| <= X1, |y1| <= Y1, |x2| <= X2, |y2| <= Y2 over the point set):
//   Ax = |F0| X1 + |F1| Y1 + |F2|, Ay, Az likewise, Bx = |F0| X2 + |F3| Y2 + |F6|, By = |F1| X2 + ...,
//   Mc = X2 Ax + Y2 Ay + Az, Dm = Ax^2 + Ay^2 + Bx^2 + By^2.
// Rounding the model (and, for E, the points) to fp32 and the fma chain give |ax32 - ax| <= 6u Ax
// and so on, |c32 - c| <= 10u Mc, |den32 - den| <= 16u Dm against the exact values, and the fp64
// evaluation sits within 1e-15 of them. We use Ec = 16u Mc, Ed = 24u Dm. Then, with
// L <= lo (1 - 2^-20) and H >= hi (1 + 2^-20) in fp32 (lo, hi: SampsonCut), and every remaining
// fp32 rounding (< 2^-21 relative in total) inside that 2^-20 margin:
//   (|c32| + Ec)^2 < den32 L - Ed L                 => c64^2 < den64 lo (1 - 2^-21)  => inlier
//   max(|c32| - Ec, 0)^2 > den32 H + Ed H           => c64^2 > den64 hi (1 + 2^-21)  => outlier
// (SampsonCut's argument: a quotient below mid (1 - 2^-50) rounds to <= thr2, above mid (1 + 2^-50)
// to > thr2). The bound holds while every magnitude is a normal fp32 far from overflow: a model with
// Mc or Dm outside [2^-90, 2^60] (or a non-finite bound) gets Ec = inf — every lane undecided.
// NaN / inf values fail both compares and so also fall back to fp64.
#pragma once

#include "mcv_common.h"
#include "hyp_fundamental.h"
#include <cmath>

namespace mcv {

struct SampsonPkBound { double Ec, Ed; };

MCV_HD SampsonPkBound sampson_pk_bound(const double* F, double X1, double Y1, double X2, double Y2,
                                       double* DmOut = nullptr) {
    const double a0 = fabs(F[0]), a1 = fabs(F[1]), a2 = fabs(F[2]), a3 = fabs(F[3]), a4 = fabs(F[4]);
    const double a5 = fabs(F[5]), a6 = fabs(F[6]), a7 = fabs(F[7]), a8 = fabs(F[8]);
    const double Ax = a0 * X1 + a1 * Y1 + a2, Ay = a3 * X1 + a4 * Y1 + a5, Az = a6 * X1 + a7 * Y1 + a8;
    const double Bx = a0 * X2 + a3 * Y2 + a6, By = a1 * X2 + a4 * Y2 + a7;
    const double Mc = X2 * Ax + Y2 * Ay + Az;
    const double Dm = Ax * Ax + Ay * Ay + Bx * Bx + By * By;
    SampsonPkBound b;
    const double u = 0x1p-24;
    b.Ec = 16.0 * u * Mc * (1.0 + 0x1p-30);
    b.Ed = 24.0 * u * Dm * (1.0 + 0x1p-30);
    const bool ok = Mc >= 0x1p-90 && Mc <= 0x1p60 && Dm >= 0x1p-90 && Dm <= 0x1p60 && Ax <= 0x1p60 &&
                    Ay <= 0x1p60 && Bx <= 0x1p60 && By <= 0x1p60;   // false for NaN too
    if (!ok) b.Ec = b.Ed = __builtin_inf();
    if (DmOut) *DmOut = Dm;
    return b;
}

#if defined(__HIPCC__)
typedef float sf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ sf2 spk_fma(sf2 a, sf2 b, sf2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ sf2 spk_lo(sf2 v) { return __builtin_shufflevector(v, v, 0, 0); }
__device__ __forceinline__ sf2 spk_hi(sf2 v) { return __builtin_shufflevector(v, v, 1, 1); }

// fp32 constants of the certified cut: L32 <= lo (1 - 2^-20), H32 >= hi (1 + 2^-20); the bound
// products are taken against those fp32 values and rounded outward, so that
// den32 L32 - Ed L32 <= den64 L32 and den32 H32 + Ed H32 >= den64 H32 hold exactly.
struct SampsonPkCut { float L32, H32; };
inline SampsonPkCut sampson_pk_cut_host(const SampsonCut& c) {
    SampsonPkCut k;
    k.L32 = -1.0f;   // lo <= 0: nothing certified inside
    if (c.lo > 0) {
        const double L = c.lo * (1.0 - 0x1p-20);
        float f = (float)L;
        if ((double)f > L) f = std::nextafter(f, 0.0f);
        k.L32 = f;
    }
    const double H = c.hi * (1.0 + 0x1p-20);
    float h = (float)H;
    if ((double)h < H) h = std::nextafter(h, __builtin_inff());
    k.H32 = h;
    return k;
}

MCV_HD float spk_f32_up(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __double2float_ru(v);
#else
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, __builtin_inff());
    return f;
#endif
}
MCV_HD float spk_f32_dn(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __double2float_rd(v);
#else
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -__builtin_inff());
    return f;
#endif
}

// Two models (one pair) in packed fp32, plus the linear cuts of the decision (below): c^2 against
// den ain + bin (inlier) and den aout + bout (outlier).
struct SampsonPkPair {
    sf2 f[9];
    sf2 ain, bin, aout, bout;
};

// The cuts in the form the sweep evaluates: one square and two FMAs per (model, correspondence).
// The certificate above needs, in exact arithmetic on the fp32 values c, den,
//   inlier:  (|c| + Ec)^2 < L (den - Ed),   outlier: max(|c| - Ec, 0)^2 > H (den + Ed).
// With 2 |c| Ec <= Ec (c^2 / K + K) for any K > 0 (AM-GM; equality at |c| = K) both follow from
//   c^2 (1 + Ec/K) + Ec K + Ec^2 < L (den - Ed)   <=>  c^2 < den ain + bin,
//     ain = L / (1 + e), bin = -(L Ed + Ec K + Ec^2) / (1 + e), e = Ec / K,
//   c^2 (1 - Ec/K) - Ec K + Ec^2 > H (den + Ed)   <=>  c^2 > den aout + bout   (K > Ec),
//     aout = H / (1 - e), bout = (H Ed + Ec K - Ec^2) / (1 - e)
// (for |c| < Ec the outlier left side is <= -Ec (K - Ec)^2 / K <= 0, so no such lane is certified).
// The cross term's slack Ec (|c| - K)^2 / K is smallest where the decision is close: K is the |c| of
// a point on the threshold with den = Dm / 4 (the typical den of the bench models lies in
// [0.01, 0.7] Dm). fp32 evaluation: c2 = c^2 (1 + d1) and the FMA's sum (den a + b)(1 + d2), |d| <= u
// = 2^-24, so a computed decision holds for the exact c^2 against (den a + b)(1 +- 2.0001 u). Inlier:
// den ain + bin > 0 whenever a lane passes (c2 >= 0); (den ain + bin)(1 + 2.0001 u) <= den ain' + bin'
// because ain carries a 2^-21 margin and bin < 0 only grows more negative under (1 + 2.0001 u).
// Outlier: (den aout + bout)(1 - 2.0001 u) >= den aout' + bout' needs the margin on both terms: aout
// carries 2^-21 and bout > 0 (H Ed + Ec (K - Ec) with K > 2 Ec) carries 2^-20 (with only
// 2^-40 on bout a lane whose den aout is small next to bout was not covered).
struct SpkCut1 { float ain, bin, aout, bout; };
MCV_HD SpkCut1 spk_cut1(const SampsonPkBound& b, double Dm, float L32, float H32) {
    SpkCut1 r;
    if (!(b.Ec < __builtin_inf()) || !(b.Ed < __builtin_inf())) {   // outside the bound's domain: undecided
        r.ain = 0.0f; r.bin = -1.0f; r.aout = __builtin_inff(); r.bout = __builtin_inff();
        return r;
    }
    const double H = (double)H32;
    double K = sqrt(H * Dm * 0.25);
    if (!(K > 2 * b.Ec)) K = 2 * b.Ec + 0x1p-120;
    const double e = b.Ec / K;
    const double ec2 = b.Ec * b.Ec, eck = b.Ec * K;
    if (L32 > 0) {
        const double L = (double)L32;
        r.ain = spk_f32_dn(L / (1.0 + e) * (1.0 - 0x1p-21));
        r.bin = -spk_f32_up((L * b.Ed + eck + ec2) / (1.0 + e) * (1.0 + 0x1p-40));
    } else {   // lo <= 0: nothing certified inside
        r.ain = 0.0f; r.bin = -1.0f;
    }
    r.aout = spk_f32_up(H / (1.0 - e) * (1.0 + 0x1p-21));
    r.bout = spk_f32_up((H * b.Ed + eck - ec2) / (1.0 - e) * (1.0 + 0x1p-20));
    return r;
}



// Build one pair from two fp64 models (F row-major) and the point-set bounds bb = {X1, Y1, X2, Y2}.
__device__ __forceinline__ void spk_make_pair(SampsonPkPair& P, const double* Fa, const double* Fb, const double* bb,
                                              const SampsonPkCut& k) {
#pragma unroll
    for (int j = 0; j < 9; ++j) P.f[j] = sf2{(float)Fa[j], (float)Fb[j]};
    double Dma, Dmb;
    const SampsonPkBound ba = sampson_pk_bound(Fa, bb[0], bb[1], bb[2], bb[3], &Dma);
    const SampsonPkBound bbn = sampson_pk_bound(Fb, bb[0], bb[1], bb[2], bb[3], &Dmb);
    const SpkCut1 ca = spk_cut1(ba, Dma, k.L32, k.H32), cb = spk_cut1(bbn, Dmb, k.L32, k.H32);
    P.ain = sf2{ca.ain, cb.ain};
    P.bin = sf2{ca.bin, cb.bin};
    P.aout = sf2{ca.aout, cb.aout};
    P.bout = sf2{ca.bout, cb.bout};
}

// One correspondence (p01 = {x1, y1}, p23 = {x2, y2}) against one model pair: lane masks of the
// certified inliers and of the undecided lanes, for model 2k (lo) and 2k + 1 (hi).
__device__ __forceinline__ void spk_test(const SampsonPkPair& P, sf2 p01, sf2 p23, float L32, float H32,
                                         uint64_t& in0, uint64_t& in1, uint64_t& amb0, uint64_t& amb1) {
    const sf2 x1 = spk_lo(p01), y1 = spk_hi(p01), x2 = spk_lo(p23), y2 = spk_hi(p23);
    const sf2 ax = spk_fma(P.f[0], x1, spk_fma(P.f[1], y1, P.f[2]));
    const sf2 ay = spk_fma(P.f[3], x1, spk_fma(P.f[4], y1, P.f[5]));
    const sf2 az = spk_fma(P.f[6], x1, spk_fma(P.f[7], y1, P.f[8]));
    const sf2 bx = spk_fma(P.f[0], x2, spk_fma(P.f[3], y2, P.f[6]));
    const sf2 by = spk_fma(P.f[1], x2, spk_fma(P.f[4], y2, P.f[7]));
    const sf2 c = spk_fma(x2, ax, spk_fma(y2, ay, az));
    const sf2 den = spk_fma(ax, ax, spk_fma(ay, ay, spk_fma(bx, bx, by * by)));
    const sf2 c2 = c * c;
    const sf2 r = spk_fma(den, P.ain, P.bin);
    const sf2 q = spk_fma(den, P.aout, P.bout);
    const uint64_t i0 = __builtin_amdgcn_ballot_w64(c2.x < r.x);
    const uint64_t i1 = __builtin_amdgcn_ballot_w64(c2.y < r.y);
    const uint64_t o0 = __builtin_amdgcn_ballot_w64(c2.x > q.x);
    const uint64_t o1 = __builtin_amdgcn_ballot_w64(c2.y > q.y);
    in0 = i0;
    in1 = i1;
    amb0 = ~(i0 | o0);
    amb1 = ~(i1 | o1);
}


// Host twin of one model's decision at one correspondence (the same fp32 operations as spk_test on one
// half of the packed pair): 1 certified inlier, 0 certified outlier, -1 undecided.
inline int spk_decide_host(const float (&f)[9], const SpkCut1& k, float x1, float y1, float x2, float y2) {
    const float ax = std::fmaf(f[0], x1, std::fmaf(f[1], y1, f[2]));
    const float ay = std::fmaf(f[3], x1, std::fmaf(f[4], y1, f[5]));
    const float az = std::fmaf(f[6], x1, std::fmaf(f[7], y1, f[8]));
    const float bx = std::fmaf(f[0], x2, std::fmaf(f[3], y2, f[6]));
    const float by = std::fmaf(f[1], x2, std::fmaf(f[4], y2, f[7]));
    const float c = std::fmaf(x2, ax, std::fmaf(y2, ay, az));
    const float by2 = by * by;
    const float den = std::fmaf(ax, ax, std::fmaf(ay, ay, std::fmaf(bx, bx, by2)));
    const float c2 = c * c;
    const float r = std::fmaf(den, k.ain, k.bin);
    const float q = std::fmaf(den, k.aout, k.bout);
    if (c2 < r) return 1;
    if (c2 > q) return 0;
    return -1;
}

// One sweep step of KP model pairs at one correspondence per lane (v: lane holds a point):
// certified inliers counted, undecided lanes re-tested in fp64 (f_error, kind 0/1) in one
// wave-uniform branch. F64 fetches model k's fp64 coefficients (global memory; the fallback is
// rare, so they are not kept in registers); X64 the lane's fp64 point.
template <int KP, class F64, class X64>
__device__ __forceinline__ void spk_sweep_point(const SampsonPkPair (&pr)[KP], float4 q, bool v, float L32, float H32,
                                                int kind, float thr2, const F64& f64, const X64& x64,
                                                uint32_t (&cnt)[2 * KP]) {
    const uint64_t vm = __builtin_amdgcn_ballot_w64(v);
    const sf2 p01 = sf2{q.x, q.y}, p23 = sf2{q.z, q.w};
    // certified inliers are counted at once and only the union of the undecided lanes stays live (few
    // scalar registers in the hot loop); the rare fallback recomputes a model's masks
    uint64_t anyAmb = 0;
#pragma unroll
    for (int kp = 0; kp < KP; ++kp) {
        uint64_t i0, i1, a0, a1;
        spk_test(pr[kp], p01, p23, L32, H32, i0, i1, a0, a1);
        cnt[2 * kp] += (uint32_t)__popcll(vm & i0);
        cnt[2 * kp + 1] += (uint32_t)__popcll(vm & i1);
        anyAmb |= vm & (a0 | a1);
    }
    if (__builtin_expect(anyAmb != 0, 0)) {
        const uint64_t me = 1ull << (__lane_id() & 63);
        double x1, y1, x2, y2;
        x64(x1, y1, x2, y2);
#pragma unroll
        for (int kp = 0; kp < KP; ++kp) {
            uint64_t i0, i1, a0, a1;
            spk_test(pr[kp], p01, p23, L32, H32, i0, i1, a0, a1);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint64_t amb = vm & (h ? a1 : a0);
                if (amb == 0) continue;
                const int k = 2 * kp + h;
                double F[9];
                f64(k, F);
                cnt[k] += (uint32_t)__popcll(
                    __builtin_amdgcn_ballot_w64((amb & me) != 0 && f_error(kind, F, x1, y1, x2, y2) <= thr2));
            }
        }
    }
}
#endif

}  // namespace mcv
