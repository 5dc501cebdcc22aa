// pnp_pk.h — certified packed-fp32 prefilter of the PnP inlier test (the
// sweep behind cvSolvePnPRansac, MiniCVNative.cpp:125).
//
// The exact decision (hyp_pnp.h pnp_error, the reference's PnPRansacCallback::computeError):
// (u, v) = projectPoints(X) in fp64 (pnp_project), U = (float)u, dx = uo - U, dy likewise in fp32,
// e = dx * dx + dy * dy (or fmaf), inlier iff e <= thr2. That costs ~60 fp64 instructions per
// (pose, point). This prefilter evaluates the same projection in fp32 — two points per
// v_pk_fma_f32, the pose in wave-uniform registers — together with a per-lane bound g on the
// distance between its pixel and the exact one, and decides every lane whose distance is certainly
// inside or outside the threshold circle; the rest take the exact fp64 test.
//
// Bound (u = 2^-24; extents Xm, Ym, Zm = max |X|, |Y|, |Z| over the points; M_r = sum_j |R_rj| Xm_j
// + |t_r| per row r of the pose):
//   Xc, Yc, Zc: three FMAs on fp32-rounded R, t:  |Xc32 - Xc| <= eX = 5u M_0 (eY, eZ likewise).
//   x = Xc / Zc by v_rcp_f32 (<= 1 ulp) and a multiply: with |Zc32| >= zmin = 2^10 eZ,
//     |x32 - x| <= delta = |1/Zc32| (c1 + m c2), c1 = max(eX, eY)(1 + 2^-10)(1 + 2^-7),
//     c2 = 1.6 eZ (1 + 2^-7) (the 1.6 also covers the reciprocal's and the product's rounding,
//     since eZ / |Zc32| >= 5u); m = max(|x32|, |y32|) (two VOP3 v_max_f32 with |.| modifiers per
//     point pair: packed arithmetic has no abs, and the AM-GM form (1 + r2) / 2 overstates m by
//     r2 / (2 m) where points project far off-image, which the rho^5 of L then multiplies).
//   distortion (xd, yd) = x (1 + k1 r2 + k2 r2^2 + 2 p1 y + 2 p2 x) + (p2, p1) r2 (the factored form
//     evaluated here): on the box |x|, |y| <= rho = m + delta its gradient's row sums are bounded by
//     L = 1 + rho (8 (|p1| + |p2|) + rho^2 (6 |k1| + 20 |k2| rho^2)), and its fp32 evaluation (depth 8
//     with the coefficient rounding) by 10 u rho L; so |xd32 - xd| <= L (delta + 10 u rho).
//   pixels: |u32 - u| + |(float)u - u| <= F L (delta + 13 u rho) + 3 u C, F = max |f|, C = max |c|
//     (fx / cx rounding, the FMA, the cast of the exact u to float); the fp64 path's own error is
//     ~2^-29 of that, inside the (1 + 2^-16) slack on F and C.
//   g = sqrt(2) (F L (delta + 13 u rho) + 4 u C) (1 + 2^-16) >= the Euclidean pixel distance.
// Decision (S = fl(D^2 + E^2), D = uo - u32, E = vo - v32; the exact e is within (1 +- 11u) of the
// squared distance of uo to the exact pixel, which is within g of sqrt(S)):
//   S < thr2 (1 - 2^-17) - 2T' g                     -> certified inlier (sqrt(S) + g < T)
//   S > thr2 (1 + 2^-17) + g (g (1 + 2^-17) + 2T')   -> certified outlier (sqrt(S) - g > T)
// with T' = sqrt(thr2) (1 + 2^-17): the 2^-17 margins cover every fp32 rounding of S, lo and hi and
// the (1 +- 11u) factors. NaN or inf anywhere fails both compares (undecided), as does a lane with
// |Zc32| < zmin (the domain of the 1/Zc bound) and every lane of a pose whose bound is not finite.
#pragma once

#include "mcv_common.h"
#include "hyp_pnp.h"
#include <cmath>

namespace mcv {

// Launch constants (host-built, pnp_pk_cam_host): the camera in fp32 and the bound's slopes.
struct PnpPkCam {
    float fx, fy, cx, cy, k1, k2, tp1, tp2, p1, p2;   // tp1 = 2 p1, tp2 = 2 p2 (exact)
    float A2, A4, cp;      // 6 |k1|, 20 |k2|, 8 (|p1| + |p2|), rounded up
    float half;            // 0.5 (1 + 2^-20), rounded up: m = fma(r2, half, half)
    float u13;             // 13 u (1 + 2^-16)
    float Fg, Cg;          // sqrt(2) F (1 + 2^-16), sqrt(2) 4u C (1 + 2^-16) + 2^-100, rounded up
    float twoT, thrLo, thrHi, gk;   // 2T', thr2 (1 - 2^-17) down, thr2 (1 + 2^-17) up, 1 + 2^-17
    int ok;                // 0: outside the bound's domain (the launch takes the exact fp64 sweep)
};

// Per-pose constants (computed per wave from the fp64 pose and the point extents).
// Cheap tier (round 4): on the domain r2 <= mc^2, |Zc32| >= zmin the per-lane bound g is at most
// alpha |iz| + beta, and with |iz| <= (iz^2 / kappa + kappa) / 2 (AM-GM) both cuts become one FMA in
// iz^2 = fl(iz * iz): S < LI0 - LI1 iz^2 (inlier), S > HO0 + HO1 iz^2 (outlier), decided only where
// w = fma(iz^2, P, r2) <= W (which implies both domain conditions). pnp_pk_pose derives them; a trip
// with a lane the cheap tier leaves undecided runs the exact per-lane bound (pnp_pk_bound).
struct PnpPkPose {
    float R[9], t[3];
    float c1, c2, zmin;
    float LI0, nLI1, HO0, HO1, W, P;   // the cheap tier's cuts (nLI1 = -LI1) and domain
    float HO0B, HO1B, WB, PB;          // its wide-domain outlier cut (r2 <= kPnpPkMc2B)
};
static constexpr double kPnpPkMc2 = 2.0;     // the cheap tier's domain: max(|x|, |y|)^2 <= r2 <= 2
static constexpr double kPnpPkMc2B = 64.0;   // ... and its outlier-only wide domain

MCV_HD float pk_f32_ru(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __double2float_ru(v);
#else
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, __builtin_inff());
    return f;
#endif
}
MCV_HD float pk_f32_rd(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __double2float_rd(v);
#else
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -__builtin_inff());
    return f;
#endif
}

inline PnpPkCam pnp_pk_cam_host(const double* cam8, float thr2) {
    const double fx = cam8[0], fy = cam8[1], cx = cam8[2], cy = cam8[3];
    const double k1 = cam8[4], k2 = cam8[5], p1 = cam8[6], p2 = cam8[7];
    PnpPkCam c;
    c.fx = (float)fx; c.fy = (float)fy; c.cx = (float)cx; c.cy = (float)cy;
    c.k1 = (float)k1; c.k2 = (float)k2; c.p1 = (float)p1; c.p2 = (float)p2;
    c.tp1 = 2.0f * c.p1; c.tp2 = 2.0f * c.p2;
    c.A2 = pk_f32_ru(6.0 * std::fabs(k1) * (1 + 0x1p-30));
    c.A4 = pk_f32_ru(20.0 * std::fabs(k2) * (1 + 0x1p-30));
    c.cp = pk_f32_ru(8.0 * (std::fabs(p1) + std::fabs(p2)) * (1 + 0x1p-30));
    c.half = pk_f32_ru(0.5 * (1 + 0x1p-20));
    const double u = 0x1p-24, s = 1.0 + 0x1p-16;
    c.u13 = pk_f32_ru(13.0 * u * s);
    const double F = std::fmax(std::fabs(fx), std::fabs(fy)), C = std::fmax(std::fabs(cx), std::fabs(cy));
    c.Fg = pk_f32_ru(std::sqrt(2.0) * F * s * (1 + 0x1p-30));
    c.Cg = pk_f32_ru(std::sqrt(2.0) * 4.0 * u * C * s * (1 + 0x1p-30) + 0x1p-100);
    const double T2 = (double)thr2, T = std::sqrt(T2);
    c.twoT = pk_f32_ru(2.0 * T * (1 + 0x1p-17) * (1 + 0x1p-30));
    c.thrLo = pk_f32_rd(T2 * (1 - 0x1p-17));
    c.thrHi = pk_f32_ru(T2 * (1 + 0x1p-17));
    c.gk = 1.0f + 0x1p-17f;
    // domain: finite camera (fp32-representable well away from overflow), finite non-negative thr2
    const double lim = 0x1p40;
    c.ok = std::fabs(fx) < lim && std::fabs(fy) < lim && std::fabs(cx) < lim && std::fabs(cy) < lim &&
           std::fabs(k1) < lim && std::fabs(k2) < lim && std::fabs(p1) < lim && std::fabs(p2) < lim &&
           T2 >= 0 && T2 < 0x1p60 && std::isfinite(c.Fg) && std::isfinite(c.twoT);
    return c;
}

// The cheap tier's constants for the domain r2 <= mc2 (derivation in pnp_pk_pose).
MCV_HD void pnp_pk_cheap(const PnpPkPose& p, const PnpPkCam& c, double tz, bool ok, double mc2, float& LI0, float& nLI1,
                         float& HO0, float& HO1, float& Wo, float& Po) {
    const double thrLo = c.thrLo, thrHi = c.thrHi, twoT = c.twoT, gk = c.gk;
    const double mc = sqrt(mc2), izc = (1.0 / (double)p.zmin) * (1 + 0x1p-22);
    const double a = ((double)p.c1 + mc * (double)p.c2) * (1 + 0x1p-40);
    const double rc = (mc + izc * a) * (1 + 0x1p-40), rc2 = rc * rc;
    const double Lc = (1.0 + rc * ((double)c.cp + rc2 * ((double)c.A2 + (double)c.A4 * rc2))) * (1 + 0x1p-38);
    const double alpha = (double)c.Fg * Lc * a * (1 + 0x1p-38);
    const double beta = ((double)c.Fg * Lc * (double)c.u13 * rc + (double)c.Cg) * (1 + 0x1p-38);
    const double kappa = 1.0 / fmax(fabs(tz), (double)p.zmin);
    const double uu = 2.0 * 0x1p-24;
    const double li0 = thrLo - twoT * (beta + alpha * kappa * 0.5) * (1 + 0x1p-38) - uu * thrLo;
    const double li1 = twoT * alpha * (1 + uu) / (2.0 * kappa) * (1 + 0x1p-20);
    const double ho0 = (thrHi + 2.0 * gk * beta * beta + twoT * (beta + alpha * kappa * 0.5)) * (1 + 0x1p-20);
    const double ho1 = (2.0 * gk * alpha * alpha + twoT * alpha / (2.0 * kappa)) * (1 + uu) * (1 + 0x1p-20);
    const double W = mc2 * (1 - 0x1p-20), P = W * (double)p.zmin * (double)p.zmin * (1 + 0x1p-18);
    const bool cok = ok && c.ok && li0 == li0 && li1 < 0x1p100 && ho0 < 0x1p100 && ho1 < 0x1p100 && P < 0x1p100 &&
                     P > 0x1p-100;
    LI0 = cok ? pk_f32_rd(li0) : -__builtin_inff();
    nLI1 = cok ? -pk_f32_ru(li1) : 0.0f;
    HO0 = cok ? pk_f32_ru(ho0) : __builtin_inff();
    HO1 = cok ? pk_f32_ru(ho1) : 0.0f;
    Wo = cok ? pk_f32_rd(W) : -1.0f;
    Po = cok ? pk_f32_ru(P) : 1.0f;
}

// ext = {Xm, Ym, Zm} (inf when any coordinate is not finite).
MCV_HD void pnp_pk_pose(const double* R, const double* t, const double* ext, const PnpPkCam& c, PnpPkPose& p) {
    for (int j = 0; j < 9; ++j) p.R[j] = (float)R[j];
    for (int j = 0; j < 3; ++j) p.t[j] = (float)t[j];
    double M[3];
    for (int r = 0; r < 3; ++r)
        M[r] = (fabs(R[3 * r]) * ext[0] + fabs(R[3 * r + 1]) * ext[1] + fabs(R[3 * r + 2]) * ext[2] + fabs(t[r])) *
               (1 + 0x1p-40);
    const double u = 0x1p-24;
    const double eXY = 5.0 * u * fmax(M[0], M[1]), eZ = 5.0 * u * M[2];
    const bool ok = M[0] <= 0x1p60 && M[1] <= 0x1p60 && M[2] <= 0x1p60;   // false for NaN
    p.c1 = ok ? pk_f32_ru(eXY * (1 + 0x1p-10) * (1 + 0x1p-7)) : __builtin_inff();
    p.c2 = ok ? pk_f32_ru(1.6 * eZ * (1 + 0x1p-7)) : __builtin_inff();
    p.zmin = ok ? pk_f32_ru(fmax(eZ * 0x1p10, 0x1p-100)) : __builtin_inff();
    // Cheap tier. On the domain the exact tier's quantities are bounded by (fp64, every step rounded
    // outward by the 2^-40 factors): |iz32| <= izc (1 + 2^-22) with izc = 1 / zmin; delta <= |iz| a,
    // a = c1 + mc c2; rho <= rc = mc + izc (1 + 2^-22) a; L <= Lc = L(rc); q = u13 rho + delta <=
    // u13 rc + |iz| a; g = Fg L q + Cg <= alpha |iz| + beta, alpha = Fg Lc a, beta = Fg Lc u13 rc + Cg.
    // iz2 = fl(iz32^2) >= iz32^2 (1 - u): |iz32| <= (iz2 (1 + 2u) / kappa + kappa) / 2 and
    // iz32^2 <= iz2 (1 + 2u). Inlier: thrLo - twoT g >= LI0 - LI1 iz2 with
    //   LI0 = thrLo - twoT (beta + alpha kappa / 2),  LI1 = twoT alpha (1 + 2u) / (2 kappa);
    // outlier (g^2 <= 2 alpha^2 iz32^2 + 2 beta^2): thrHi + gk g^2 + twoT g <= HO0 + HO1 iz2 with
    //   HO0 = thrHi + 2 gk beta^2 + twoT (beta + alpha kappa / 2),
    //   HO1 = (2 gk alpha^2 + twoT alpha / (2 kappa)) (1 + 2u).
    // The FMAs' rounding: LI0 lowered by 2u thrLo, LI1 / HO0 / HO1 raised by 2^-20 (an fp32 result
    // within u of the FMA's exact value then stays on the safe side). Domain: w = fl(fma(iz2, P, r2))
    // <= W, W = mc^2 (1 - 2^-20), P = W zmin^2 (1 + 2^-18), gives r2 <= W / (1 - u) (so m^2 <=
    // r2 / (1 - 2u) < mc^2) and iz2 <= 1 / (zmin^2 (1 + 2^-18) (1 - u)) (so 1 / |Zc32| <=
    // |iz32| (1 + 2^-22) < 1 / zmin); a NaN lane fails it. kappa = 1 / max(|t_z|, zmin): the cut is
    // tightest for points near the depth of the world origin.
    pnp_pk_cheap(p, c, t[2], ok, kPnpPkMc2, p.LI0, p.nLI1, p.HO0, p.HO1, p.W, p.P);
    float li0, nli1;
    pnp_pk_cheap(p, c, t[2], ok, kPnpPkMc2B, li0, nli1, p.HO0B, p.HO1B, p.WB, p.PB);
}

// Elementwise helpers: V = float (host twin, one point) or f2 (device, two points).
MCV_HD float pkv_fma(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fmaf(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}
MCV_HD float pkv_splat(float c, float) { return c; }
MCV_HD float pkv_rcp(float a) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(a);
#else
    return 1.0f / a;
#endif
}
MCV_HD float pkv_absmul(float a, float b) { return fabsf(a) * b; }
MCV_HD float pkv_absmax(float a, float b) { return fmaxf(fabsf(a), fabsf(b)); }

#if defined(__HIPCC__)
typedef float pkf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pkf2 pkv_fma(pkf2 a, pkf2 b, pkf2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ pkf2 pkv_splat(float c, pkf2) { return pkf2{c, c}; }
__device__ __forceinline__ pkf2 pkv_rcp(pkf2 a) { return pkf2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)}; }
__device__ __forceinline__ pkf2 pkv_absmul(pkf2 a, pkf2 b) { return pkf2{fabsf(a.x) * b.x, fabsf(a.y) * b.y}; }
__device__ __forceinline__ pkf2 pkv_absmax(pkf2 a, pkf2 b) {
    return pkf2{fmaxf(fabsf(a.x), fabsf(b.x)), fmaxf(fabsf(a.y), fabsf(b.y))};
}
#endif

// Coefficient pairs: two different wave-uniform constants in one 64-bit register pair, either half
// broadcast to both lanes of a packed op by op_sel (no per-use copy). Host twin: a plain struct.
struct PkPairH { float x, y; };
MCV_HD PkPairH pkp_make(float a, float b, float) { return PkPairH{a, b}; }
MCV_HD float pkp_lo(PkPairH p, float) { return p.x; }
MCV_HD float pkp_hi(PkPairH p, float) { return p.y; }
template <class V> struct PkPairOf { typedef PkPairH type; };
#if defined(__HIPCC__)
__device__ __forceinline__ pkf2 pkp_make(float a, float b, pkf2) { return pkf2{a, b}; }
__device__ __forceinline__ pkf2 pkp_lo(pkf2 p, pkf2) { return __builtin_shufflevector(p, p, 0, 0); }
__device__ __forceinline__ pkf2 pkp_hi(pkf2 p, pkf2) { return __builtin_shufflevector(p, p, 1, 1); }
template <> struct PkPairOf<pkf2> { typedef pkf2 type; };
#endif

// Launch constants, built once outside the sweep. Constant-bus rule (one scalar operand per VALU
// op): of two constants that meet in one FMA, one is a splatted vector (VGPR pair on the device),
// the other comes from a coefficient pair (SGPR pair).
template <class V>
struct PnpPkCamV {
    typedef typename PkPairOf<V>::type P;
    P k2tp1, tp2p1, p2fx, fyA4, cpu13, Fgnt, gkHi;   // {k2, tp1}, {tp2, p1}, {p2, fx}, {fy, A4}, {cp, u13}, {Fg, -twoT}, {gk, thrHi}
    V k1, cx, cy, A2, Cg, thrLo, twoT, one;
};
template <class V>
MCV_HD PnpPkCamV<V> pnp_pk_cam_v(const PnpPkCam& c, V z) {
    PnpPkCamV<V> v;
    v.k2tp1 = pkp_make(c.k2, c.tp1, z); v.tp2p1 = pkp_make(c.tp2, c.p1, z); v.p2fx = pkp_make(c.p2, c.fx, z);
    v.fyA4 = pkp_make(c.fy, c.A4, z); v.cpu13 = pkp_make(c.cp, c.u13, z); v.Fgnt = pkp_make(c.Fg, -c.twoT, z);
    v.gkHi = pkp_make(c.gk, c.thrHi, z);
    v.k1 = pkv_splat(c.k1, z); v.cx = pkv_splat(c.cx, z); v.cy = pkv_splat(c.cy, z); v.A2 = pkv_splat(c.A2, z);
    v.Cg = pkv_splat(c.Cg, z); v.thrLo = pkv_splat(c.thrLo, z); v.twoT = pkv_splat(c.twoT, z);
    v.one = pkv_splat(1.0f, z);
    return v;
}
// Pose: R and c2 as coefficient pairs, t and c1 splatted (each meets a pose coefficient in an FMA);
// the cheap tier's constants as VGPR pairs read through op_sel ({P, -LI1}, {LI0, HO1}, {HO0, W}).
template <class V>
struct PnpPkPoseV {
    typedef typename PkPairOf<V>::type P;
    P r01, r23, r45, r67, r8c2;
    V t0, t1, t2, c1;
    P qPl, qLh, qHW, qB0, qB1;   // ..., {PB, HO1B}, {HO0B, WB}
    float zmin;
};
template <class V>
MCV_HD PnpPkPoseV<V> pnp_pk_pose_v(const PnpPkPose& p, V z) {
    PnpPkPoseV<V> v;
    v.r01 = pkp_make(p.R[0], p.R[1], z); v.r23 = pkp_make(p.R[2], p.R[3], z); v.r45 = pkp_make(p.R[4], p.R[5], z);
    v.r67 = pkp_make(p.R[6], p.R[7], z); v.r8c2 = pkp_make(p.R[8], p.c2, z);
    v.t0 = pkv_splat(p.t[0], z); v.t1 = pkv_splat(p.t[1], z); v.t2 = pkv_splat(p.t[2], z);
    v.c1 = pkv_splat(p.c1, z);
    v.qPl = pkp_make(p.P, p.nLI1, z); v.qLh = pkp_make(p.LI0, p.HO1, z); v.qHW = pkp_make(p.HO0, p.W, z);
    v.qB0 = pkp_make(p.PB, p.HO1B, z); v.qB1 = pkp_make(p.HO0B, p.WB, z);
    v.zmin = p.zmin;
    return v;
}

// The projection of one point (V = float) or two points (V = f2) against one pose: S (squared fp32
// pixel distance), the cheap tier's cuts loC / hiC and domain value w (decided where w <= W), and the
// per-point values the exact tier needs (x, y, iz, Zc). Per point pair (packed): 33 packed ops and
// 2 v_rcp_f32.
template <class V>
struct PnpPkProj {
    V S, loC, hiC, w, x, y, iz, Zc, r2;
};
template <class V>
MCV_HD PnpPkProj<V> pnp_pk_project(const PnpPkCamV<V>& c, const PnpPkPoseV<V>& p, V X, V Y, V Z, V uo, V vo) {
    const V z = X;   // type tag only
    PnpPkProj<V> o;
    const V Xc = pkv_fma(pkp_lo(p.r01, z), X, pkv_fma(pkp_hi(p.r01, z), Y, pkv_fma(pkp_lo(p.r23, z), Z, p.t0)));
    const V Yc = pkv_fma(pkp_hi(p.r23, z), X, pkv_fma(pkp_lo(p.r45, z), Y, pkv_fma(pkp_hi(p.r45, z), Z, p.t1)));
    const V Zc = pkv_fma(pkp_lo(p.r67, z), X, pkv_fma(pkp_hi(p.r67, z), Y, pkv_fma(pkp_lo(p.r8c2, z), Z, p.t2)));
    const V iz = pkv_rcp(Zc);
    const V x = Xc * iz, y = Yc * iz;
    const V r2 = pkv_fma(x, x, y * y);
    const V cd = pkv_fma(r2, pkv_fma(pkp_lo(c.k2tp1, z), r2, c.k1), c.one);
    const V w = pkv_fma(pkp_hi(c.k2tp1, z), y, pkv_fma(pkp_lo(c.tp2p1, z), x, cd));
    const V xd = pkv_fma(x, w, pkp_lo(c.p2fx, z) * r2);
    const V yd = pkv_fma(y, w, pkp_hi(c.tp2p1, z) * r2);
    const V u = pkv_fma(pkp_hi(c.p2fx, z), xd, c.cx);
    const V v = pkv_fma(pkp_lo(c.fyA4, z), yd, c.cy);
    const V D = uo - u, E = vo - v;
    o.S = pkv_fma(D, D, E * E);
    // cheap tier
    const V iz2 = iz * iz;
    o.w = pkv_fma(iz2, pkp_lo(p.qPl, z), r2);
    o.loC = pkv_fma(iz2, pkp_hi(p.qPl, z), pkp_lo(p.qLh, z));
    o.hiC = pkv_fma(iz2, pkp_hi(p.qLh, z), pkp_lo(p.qHW, z));
    o.x = x; o.y = y; o.iz = iz; o.Zc = Zc; o.r2 = r2;
    return o;
}

// The exact tier's cuts for the lanes the cheap tier leaves undecided: the per-lane bound g from m =
// max(|x|, |y|) and |iz| (decided where |Zc| >= zmin). 12 packed ops, 2 v_max_f32 and 2 v_mul_f32 with |.|.
template <class V>
MCV_HD void pnp_pk_bound(const PnpPkCamV<V>& c, const PnpPkPoseV<V>& p, const PnpPkProj<V>& o, V& lo, V& hi) {
    const V z = o.x;
    const V m = pkv_absmax(o.x, o.y);
    const V delta = pkv_absmul(o.iz, pkv_fma(m, pkp_hi(p.r8c2, z), p.c1));
    const V rho = m + delta;
    const V rho2 = rho * rho;
    const V L = pkv_fma(rho, pkv_fma(rho2, pkv_fma(rho2, pkp_hi(c.fyA4, z), c.A2), pkp_lo(c.cpu13, z)), c.one);
    const V q = pkv_fma(rho, pkp_hi(c.cpu13, z), delta);
    const V g = pkv_fma(L * q, pkp_lo(c.Fgnt, z), c.Cg);
    lo = pkv_fma(g, pkp_hi(c.Fgnt, z), c.thrLo);
    hi = pkv_fma(g, pkv_fma(g, pkp_lo(c.gkHi, z), c.twoT), pkp_hi(c.gkHi, z));
}

// Host twin of the decision for one point: 1 certified inlier, 0 certified outlier, -1 undecided.
// tiers: 1 = the cheap tier only, 3 = the sweep's order (cheap, then the exact tier if undecided).
inline int pnp_pk_decide_host(const PnpPkCam& c, const PnpPkPose& p, float X, float Y, float Z, float uo, float vo,
                              int tiers = 3) {
    const PnpPkCamV<float> cv = pnp_pk_cam_v<float>(c, 0.0f);
    const PnpPkPoseV<float> pv = pnp_pk_pose_v<float>(p, 0.0f);
    const PnpPkProj<float> o = pnp_pk_project<float>(cv, pv, X, Y, Z, uo, vo);
    if (o.w <= p.W) {
        if (o.S < o.loC) return 1;
        if (o.S > o.hiC) return 0;
    }
    const float iz2 = o.iz * o.iz;   // the wide domain's outlier cut (the sweep's second step)
    if (fmaf(iz2, p.PB, o.r2) <= p.WB && o.S > fmaf(iz2, p.HO1B, p.HO0B)) return 0;
    if (!(tiers & 2)) return -1;
    float lo, hi;
    pnp_pk_bound<float>(cv, pv, o, lo, hi);
    if (!(std::fabs(o.Zc) >= p.zmin)) return -1;
    if (o.S < lo) return 1;
    if (o.S > hi) return 0;
    return -1;
}

}  // namespace mcv
