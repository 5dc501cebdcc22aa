// glibc_math.h — glibc 2.35's cbrt, hypot, exp, log, log1p, cos and atan2 restated operation for
// operation, and its clog's real part (host and device).
//
// The reference's AP3P solver (ap3p.cpp:10-59, solveQuartic) runs std::cbrt, std::sqrt of
// std::complex<double> and std::pow(std::complex<double>, double) through libstdc++, i.e. glibc's cbrt,
// csqrt (whose general branch calls glibc's hypot) and, for a complex resolvent, clog (log / log1p /
// hypot, atan2), exp and cos [ext: glibc 2.35, the container's and the GPU box's libm;
// sysdeps/ieee754/dbl-64]. None is correctly rounded, so a device that calls its own (ocml) functions
// returns other last bits, which the quartic's two Newton polish passes then carry into the pose. These
// restatements compute glibc's bits: every product, sum and quotient rounded as written, in glibc's
// order, with the fused multiply-adds of the FMA variants the x86_64 build selects for exp / log /
// cos / atan2 (below) and glibc's tables (glibc_tables.h). tests/test_glibc_math.py checks each
// against the host's libm bit for bit on millions of inputs.
#pragma once

#include "mcv_common.h"
#include "glibc_tables.h"

namespace mcv {

// frexp / ldexp by exponent arithmetic (exact, subnormals included) so the host twin and the device
// run one code path.
MCV_HD double glibc_frexp(double x, int* e) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_frexp(x, e);
#else
    return ::frexp(x, e);
#endif
}
MCV_HD double glibc_ldexp(double x, int e) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_ldexp(x, e);
#else
    return ::ldexp(x, e);
#endif
}

// s_cbrt.c (dbl-64): x = xm 2^xe with xm in [0.5, 1); a degree-6 polynomial estimate u of cbrt(xm),
// one Halley step ym = u (u^3 + 2 xm) / (2 u^3 + xm), the exponent's remainder by a table factor.
MCV_HD double glibc_cbrt(double x) {
    const double CBRT2 = 1.2599210498948731648, SQR_CBRT2 = 1.5874010519681994748;
    const double factor[5] = {1.0 / SQR_CBRT2, 1.0 / CBRT2, 1.0, CBRT2, SQR_CBRT2};
    int xe = 0;
    const double xm = glibc_frexp(fabs(x), &xe);
    // frexp's exponent is 0 for zero (and for inf / NaN on glibc): those return x + x
    if (xe == 0 && !(fabs(x) > 0 && fabs(x) < __builtin_inf())) return x + x;
    const double u = (0.354895765043919860 +
                      ((1.50819193781584896 +
                        ((-2.11499494167371287 +
                          ((2.44693122563534430 +
                            ((-1.83469277483613086 + (0.784932344976639262 - 0.145263899385486377 * xm) * xm) * xm)) *
                           xm)) *
                         xm)) *
                       xm));
    const double t2 = u * u * u;
    int r = xe % 3;   // C remainder: -2 .. 2
    double f = factor[2];
    f = r == -2 ? factor[0] : r == -1 ? factor[1] : r == 1 ? factor[3] : r == 2 ? factor[4] : f;
    const double ym = u * (t2 + 2.0 * xm) / (2.0 * t2 + xm) * f;
    return glibc_ldexp(x > 0.0 ? ym : -ym, xe / 3);
}

// e_hypot.c (glibc 2.35, the non-FMA kernel): h = sqrt(ax^2 + ay^2) corrected by one step from the
// exact residual, with the scalings that keep the squares in range.
MCV_HD double glibc_hypot_kernel(double ax, double ay) {
    double t1, t2;
    double h = sqrt(ax * ax + ay * ay);
    if (h <= 2.0 * ay) {
        const double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    } else {
        const double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

MCV_HD double glibc_hypot(double x, double y) {
    const double SCALE = 0x1p-600, LARGE_VAL = 0x1p+511, TINY_VAL = 0x1p-459, EPS = 0x1p-54;
    if (!(fabs(x) < __builtin_inf()) || !(fabs(y) < __builtin_inf())) {
        if (fabs(x) == __builtin_inf() || fabs(y) == __builtin_inf()) return __builtin_inf();
        return x + y;
    }
    x = fabs(x);
    y = fabs(y);
    double ax = x < y ? y : x;
    const double ay = x < y ? x : y;
    if (ax > LARGE_VAL) {
        if (ay <= ax * EPS) return ax + ay;
        return glibc_hypot_kernel(ax * SCALE, ay * SCALE) / SCALE;
    }
    if (ay < TINY_VAL) {
        if (ax >= ay / EPS) return ax + ay;
        ax = glibc_hypot_kernel(ax / SCALE, ay / SCALE) * SCALE;
        return ax;
    }
    if (ay <= ax * EPS) return ax + ay;
    return glibc_hypot_kernel(ax, ay);
}

}  // namespace mcv

namespace mcv {

// ---- exp / log / log1p / cos / atan2 of glibc 2.35 (the x86_64 build this image and the GPU box load) --
// exp, log, sin / cos and atan2 are multiarch in that build: a CPU with FMA (both hosts) runs the
// variants compiled with -mfma, whose C sources GCC contracts (-ffp-contract=fast) — every product whose
// only use is an addition or subtraction becomes one fused multiply-add. These restatements write those
// FMAs out explicitly (__builtin_fma: the device's v_fma_f64, the host's fma) and keep every other
// operation as written; the tables are glibc's data (glibc_tables.h, generated from the image's libm).
// log1p and hypot are not multiarch (baseline build, no FMA). Domains: the AP3P resolvent's arguments
// (finite, nonzero); tests/test_glibc_math.py pins each function against the host libm bit for bit.
MCV_HD uint64_t glibc_bits(double x) { return __builtin_bit_cast(uint64_t, x); }
MCV_HD double glibc_from_bits(uint64_t u) { return __builtin_bit_cast(double, u); }

// e_exp.c (ARM optimized-routines exp, N = 128): x = k ln2 / N + r, 2^(k / N) from the table, a
// degree-5 polynomial for e^r. Domain |x| < 512 (the specialcase scaling of over- / underflowing
// results is not restated; |x| < 2^-54 returns 1 + x).
MCV_HD double glibc_exp(double x) {
    const double InvLn2N = kGlibcExpC[0], Shift = kGlibcExpC[1], NegLn2hiN = kGlibcExpC[2],
                 NegLn2loN = kGlibcExpC[3], C2 = kGlibcExpC[4], C3 = kGlibcExpC[5], C4 = kGlibcExpC[6],
                 C5 = kGlibcExpC[7];
    const uint32_t abstop = (uint32_t)(glibc_bits(x) >> 52) & 0x7ff;
    if (abstop < 0x3c9) return 1.0 + x;   // |x| < 2^-54
    const double kd0 = __builtin_fma(InvLn2N, x, Shift);
    const uint64_t ki = glibc_bits(kd0);
    const double kd = kd0 - Shift;
    const double r = __builtin_fma(kd, NegLn2loN, __builtin_fma(kd, NegLn2hiN, x));
    const int idx = 2 * (int)(ki % 128);
    const uint64_t top = ki << 45;
    const double tail = glibc_from_bits(kGlibcExpTab[idx]);
    const uint64_t sbits = kGlibcExpTab[idx + 1] + top;
    const double r2 = r * r;
    const double tmp = __builtin_fma(r2 * r2, __builtin_fma(r, C5, C4), __builtin_fma(r2, __builtin_fma(r, C3, C2), tail + r));
    const double scale = glibc_from_bits(sbits);
    return __builtin_fma(scale, tmp, scale);
}

// e_log.c (ARM optimized-routines log, N = 128): x = 2^k z, z near c = 1 / invc (table), r = z invc - 1
// by one FMA, log x = k ln2 + log c + log1p(r) with a degree-6 polynomial. Domain: positive normal x
// outside [1 - 2^-4, 1 + 0x1.09p-4) (the close-to-1 polynomial is not restated) — clog calls log only
// for |z| outside that band.
MCV_HD double glibc_log(double x) {
    const double Ln2hi = kGlibcLogC[0], Ln2lo = kGlibcLogC[1], A0 = kGlibcLogC[2], A1 = kGlibcLogC[3],
                 A2 = kGlibcLogC[4], A3 = kGlibcLogC[5], A4 = kGlibcLogC[6];
    uint64_t ix = glibc_bits(x);
    if (ix >= 0x7ff0000000000000ull) return x;   // +inf, NaN
    if ((ix >> 52) == 0) {   // subnormal: normalise
        ix = glibc_bits(x * 0x1p52);
        ix -= 52ull << 52;
    }
    const uint64_t tmp = ix - 0x3fe6000000000000ull;
    const int i = (int)((tmp >> 45) % 128);
    const int64_t k = (int64_t)tmp >> 52;
    const uint64_t iz = ix - (tmp & (0xfffull << 52));
    const double invc = kGlibcLogTab[2 * i], logc = kGlibcLogTab[2 * i + 1];
    const double z = glibc_from_bits(iz);
    const double r = __builtin_fma(z, invc, -1.0);
    const double kd = (double)k;
    const double w = __builtin_fma(kd, Ln2hi, logc);
    const double hi = w + r;
    const double lo = __builtin_fma(kd, Ln2lo, (w - hi) + r);
    const double r2 = r * r;
    const double q = __builtin_fma(r2, __builtin_fma(r, A4, A3), __builtin_fma(r, A2, A1));
    const double y = __builtin_fma(r * r2, q, __builtin_fma(r2, A0, lo));
    return y + hi;
}

// s_log1p.c (fdlibm): log1p(x) = k ln2 + log(1 + f) with s = f / (2 + f), the Lp polynomial in s^2
// evaluated in glibc's split (Estrin) form, and the rounding correction c of 1 + x. Domain x > -1.
MCV_HD double glibc_log1p(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01, Lp3 = 2.857142874366239149e-01,
                 Lp4 = 2.222219843214978396e-01, Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                 Lp7 = 1.479819860511658591e-01;
    const int32_t hx = (int32_t)(glibc_bits(x) >> 32), ax = hx & 0x7fffffff;
    int32_t k = 1, hu = 0;
    double f = 0, c = 0;
    if (hx < 0x3FDA827A) {   // x < 0.41422
        if (ax < 0x3e200000) {   // |x| < 2^-29
            if (ax < 0x3c900000) return x;
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec3) {   // -0.2929 < x < 0.41422
            k = 0;
            f = x;
            hu = 1;
        }
    }
    if (k != 0) {
        double u;
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = (int32_t)(glibc_bits(u) >> 32);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
            c /= u;
        } else {
            u = x;
            hu = (int32_t)(glibc_bits(u) >> 32);
            k = (hu >> 20) - 1023;
            c = 0;
        }
        hu &= 0x000fffff;
        const uint64_t lo = glibc_bits(u) & 0xffffffffull;
        if (hu < 0x6a09e) {
            u = glibc_from_bits(((uint64_t)(uint32_t)(hu | 0x3ff00000) << 32) | lo);
        } else {
            k += 1;
            u = glibc_from_bits(((uint64_t)(uint32_t)(hu | 0x3fe00000) << 32) | lo);
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    const double hfsq = 0.5 * f * f;
    if (hu == 0) {   // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += k * ln2_lo;
            return k * ln2_hi + c;
        }
        const double R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
    }
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double R1 = z * Lp1, z2 = z * z;
    const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    const double R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// s_sin.c's do_sin / do_cos (IBM Accurate Mathematical Library): x = x_i + t with x_i = i / 128 (the
// table's sin / cos x_i as double-doubles), sin / cos of t by short polynomials.
MCV_HD double glibc_do_sin(double x, double dx) {
    const double sn3 = -1.66666666666664880952546298448555E-01, sn5 = 8.33333214285722277379541354343671E-03,
                 cs2 = 4.99999999999999999999950396842453E-01, cs4 = -4.16666666666664434524222570944589E-02,
                 cs6 = 1.38888874007937613028114285595617E-03, big = 0x1.8p45;
    const double xold = x;   // |x| >= 0.126 here (the Taylor branch is not restated)
    if (x <= 0) dx = -dx;
    const double ux = big + fabs(x);
    x = fabs(x) - (ux - big);
    const int k = (int)(uint32_t)glibc_bits(ux) << 2;
    const double sn = kGlibcSinCosTab[k], ssn = kGlibcSinCosTab[k + 1], cs = kGlibcSinCosTab[k + 2],
                 ccs = kGlibcSinCosTab[k + 3];
    const double xx = x * x;
    const double s = x + __builtin_fma(x * xx, __builtin_fma(xx, sn5, sn3), dx);
    const double c = __builtin_fma(x, dx, xx * __builtin_fma(xx, __builtin_fma(xx, cs6, cs4), cs2));
    const double cor = __builtin_fma(cs, s, __builtin_fma(-sn, c, __builtin_fma(s, ccs, ssn)));
    return __builtin_copysign(sn + cor, xold);
}
MCV_HD double glibc_do_cos(double x, double dx) {
    const double sn3 = -1.66666666666664880952546298448555E-01, sn5 = 8.33333214285722277379541354343671E-03,
                 cs2 = 4.99999999999999999999950396842453E-01, cs4 = -4.16666666666664434524222570944589E-02,
                 cs6 = 1.38888874007937613028114285595617E-03, big = 0x1.8p45;
    if (x < 0) dx = -dx;
    const double ux = big + fabs(x);
    x = fabs(x) - (ux - big) + dx;
    const int k = (int)(uint32_t)glibc_bits(ux) << 2;
    const double sn = kGlibcSinCosTab[k], ssn = kGlibcSinCosTab[k + 1], cs = kGlibcSinCosTab[k + 2],
                 ccs = kGlibcSinCosTab[k + 3];
    const double xx = x * x;
    const double s = __builtin_fma(x * xx, __builtin_fma(xx, sn5, sn3), x);
    const double c = xx * __builtin_fma(xx, __builtin_fma(xx, cs6, cs4), cs2);
    const double cor = __builtin_fma(-sn, s, __builtin_fma(-cs, c, __builtin_fma(-s, ssn, ccs)));
    return cs + cor;
}
// __cos for |x| < 2.426265 (2^-27 <= |x| < 0.855469: do_cos; above: sin(pi / 2 - |x|) with the 106-bit
// pi / 2). Domain |x| <= pi / 2 - 0.126 (do_sin's Taylor branch for |a| < 0.126 is not restated); the
// AP3P angle arg(w) / 3 is at most pi / 3.
MCV_HD double glibc_cos(double x) {
    const double hp0 = 0x1.921FB54442D18p0, hp1 = 0x1.1A62633145C07p-54;
    const uint32_t k = (uint32_t)(glibc_bits(x) >> 32) & 0x7fffffffu;
    if (k < 0x3e400000u) return 1.0;
    if (k < 0x3feb6000u) return glibc_do_cos(x, 0);
    const double y = hp0 - fabs(x);
    const double a = y + hp1;
    const double da = (y - a) + hp1;
    return glibc_do_sin(a, da);
}

// e_atan2.c (IBM Accurate Mathematical Library, glibc 2.35 without the multi-precision stage): u =
// min / max of |x|, |y| as a double-double (u, du: EMULV by FMA), atan u by a polynomial below 1/16
// or from the cij table's Taylor row at x_i, then the quadrant (pi / 2, pi with their low parts).
// Domain: finite x, y, not both zero, |x|, |y| in [2^-500, 2^500] up to the de-checks below.
MCV_HD double glibc_atan2(double y, double x) {
    const double hpi = 0x1.921fb54442d18p0, hpi1 = 0x1.1a62633145c07p-54, opi = 0x1.921fb54442d18p1,
                 opi1 = kGlibcOpi1, inv16 = 0x1p-4, TWO52 = 0x1p52, TWO8 = 256.0;
    const double d3 = kGlibcAtanD[0], d5 = kGlibcAtanD[1], d7 = kGlibcAtanD[2], d9 = kGlibcAtanD[3],
                 d11 = kGlibcAtanD[4], d13 = kGlibcAtanD[5];
    const int32_t ux = (int32_t)(glibc_bits(x) >> 32), uy = (int32_t)(glibc_bits(y) >> 32);
    if (y == 0) return (ux & 0x80000000) == 0 ? __builtin_copysign(0.0, y) : __builtin_copysign(opi, y);
    if (x == 0) return y > 0 ? hpi : -hpi;
    double ax = fabs(x), ay = fabs(y);
    const int32_t de = (uy & 0x7ff00000) - (ux & 0x7ff00000);
    if (de >= 59768832) return y > 0 ? hpi : -hpi;
    if (de <= -59768832) {
        if (x > 0) return __builtin_copysign(ay / ax, y);
        return y > 0 ? opi : -opi;
    }
    if (ax < 0x1p-500 || ay < 0x1p-500) {
        ax *= 0x1p500;
        ay *= 0x1p500;
    }
    if (ax > 0x1p500 || ay > 0x1p500) {
        ax *= 0x1p-500;
        ay *= 0x1p-500;
    }
    double u, du;
    if (ay < ax) {
        u = ay / ax;
        const double v = ax * u, vv = __builtin_fma(ax, u, -v);
        du = ((ay - v) - vv) / ax;
    } else {
        u = ax / ay;
        const double v = ay * u, vv = __builtin_fma(ay, u, -v);
        du = ((ax - v) - vv) / ay;
    }
    auto poly = [&](double v) {
        return __builtin_fma(v, __builtin_fma(v, __builtin_fma(v, __builtin_fma(v, __builtin_fma(v, d13, d11), d9), d7), d5), d3);
    };
    auto tab = [&](double v, const double* c) {   // c3 + v (c4 + v (c5 + v c6))
        return __builtin_fma(v, __builtin_fma(v, __builtin_fma(v, c[6], c[5]), c[4]), c[3]);
    };
    auto index = [&](double uu) { return (int)((TWO52 + TWO8 * uu) - TWO52) - 16; };
    double z;
    if (x > 0) {
        if (ay < ax) {   // (i) atan(ay / ax)
            if (u < inv16) {
                const double v = u * u;
                z = u + __builtin_fma(u * v, poly(v), du);
            } else {
                const double* c = kGlibcAtanCij + 7 * index(u);
                const double t3 = u - c[0];
                const double v = t3 + du;
                const double dv = fabs(t3) > fabs(du) ? ((t3 - v) + du) : ((du - v) + t3);
                const double t1 = c[1], t2 = c[2];
                const double zz = __builtin_fma(v, t2, __builtin_fma(dv, t2, v * v * tab(v, c)));
                z = t1 + zz;
            }
        } else if (u < inv16) {   // (ii) pi / 2 - atan(ax / ay)
            const double v = u * u;   // zz = u v P stays a product (the build does not fuse it)
            const double t2 = hpi - u;
            const double cor = (hpi > u) ? ((hpi - t2) - u) : (hpi - (u + t2));
            const double t3 = ((hpi1 + cor) - du) - u * v * poly(v);
            z = t2 + t3;
        } else {
            const double* c = kGlibcAtanCij + 7 * index(u);
            const double v = (u - c[0]) + du;
            const double zz = __builtin_fma(-v, __builtin_fma(v, tab(v, c), c[2]), hpi1);
            z = (hpi - c[1]) + zz;
        }
    } else if (ax < ay) {   // (iii) pi / 2 + atan(ax / ay)
        if (u < inv16) {
            const double v = u * u;
            const double t2 = hpi + u;
            const double cor = (hpi > u) ? ((hpi - t2) + u) : ((u - t2) + hpi);
            const double t3 = ((hpi1 + cor) + du) + u * v * poly(v);
            z = t2 + t3;
        } else {
            const double* c = kGlibcAtanCij + 7 * index(u);
            const double v = (u - c[0]) + du;
            const double zz = __builtin_fma(v, __builtin_fma(v, tab(v, c), c[2]), hpi1);
            z = (hpi + c[1]) + zz;
        }
    } else if (u < inv16) {   // (iv) pi - atan(ay / ax)
        const double v = u * u;
        const double t2 = opi - u;
        const double cor = (opi > u) ? ((opi - t2) - u) : (opi - (u + t2));
        const double t3 = ((opi1 + cor) - du) - u * v * poly(v);
        z = t2 + t3;
    } else {
        const double* c = kGlibcAtanCij + 7 * index(u);
        const double v = (u - c[0]) + du;
        const double zz = __builtin_fma(-v, __builtin_fma(v, tab(v, c), c[2]), opi1);
        z = (opi - c[1]) + zz;
    }
    return __builtin_copysign(z, y);
}

// x2y2m1.c (dbl-64): x^2 + y^2 - 1 from the exact product splits and -1, sorted by magnitude (glibc's
// qsort is a stable merge sort for five elements: an insertion sort here), each neighbour pair turned
// into a non-overlapping (hi, lo) by the fast two-sum and re-sorted, then summed from the top down.
MCV_HD void glibc_sort_abs(double* v, int n) {
    for (int i = 1; i < n; ++i) {
        const double x = v[i];
        int j = i - 1;
        while (j >= 0 && fabs(v[j]) > fabs(x)) {
            v[j + 1] = v[j];
            --j;
        }
        v[j + 1] = x;
    }
}
MCV_HD double glibc_x2y2m1(double x, double y) {
    double v[5];
    v[1] = x * x;
    v[0] = __builtin_fma(x, x, -v[1]);
    v[3] = y * y;
    v[2] = __builtin_fma(y, y, -v[3]);
    v[4] = -1.0;
    glibc_sort_abs(v, 5);
    for (int i = 0; i <= 3; ++i) {
        const double hi = v[i + 1] + v[i];
        const double lo = (v[i + 1] - hi) + v[i];
        v[i + 1] = hi;
        v[i] = lo;
        glibc_sort_abs(v + i + 1, 4 - i);
    }
    return v[4] + v[3] + v[2] + v[1] + v[0];
}

// The real part of s_clog_template.c's clog (glibc 2.35): log |z| through log1p of x^2 + y^2 - 1 for
// |z| near 1 (the branches that keep its relative accuracy there), log(hypot) elsewhere, with the
// scalings of huge and tiny arguments; log / log1p / hypot are the restatements above, so the result
// is glibc's on the device and on the host alike.
MCV_HD double glibc_clog_re(double re, double im) {
    const double DBL_MAX_ = 1.7976931348623157e308, DBL_MIN_ = 2.2250738585072014e-308;
    const double EPS = 2.2204460492503131e-16, LN2 = 0.693147180559945309417;
    double absx = fabs(re), absy = fabs(im);
    if (absx == 0 && absy == 0) return -1 / absx;
    if (absx < absy) {
        const double t = absx;
        absx = absy;
        absy = t;
    }
    int scale = 0;
    if (absx > DBL_MAX_ / 2) {
        scale = -1;
        absx = glibc_ldexp(absx, scale);
        absy = absy >= DBL_MIN_ * 2 ? glibc_ldexp(absy, scale) : 0;
    } else if (absx < DBL_MIN_ && absy < DBL_MIN_) {
        scale = 53;
        absx = glibc_ldexp(absx, scale);
        absy = glibc_ldexp(absy, scale);
    }
    if (absx == 1 && scale == 0) return glibc_log1p(absy * absy) / 2;
    if (absx > 1 && absx < 2 && absy < 1 && scale == 0) {
        double d2m1 = (absx - 1) * (absx + 1);
        if (absy >= EPS) d2m1 += absy * absy;
        return glibc_log1p(d2m1) / 2;
    }
    if (absx < 1 && absx >= 0.5 && absy < EPS / 2 && scale == 0) return glibc_log1p((absx - 1) * (absx + 1)) / 2;
    if (absx < 1 && absx >= 0.5 && scale == 0 && absx * absx + absy * absy >= 0.5)
        return glibc_log1p(glibc_x2y2m1(absx, absy)) / 2;
    return glibc_log(glibc_hypot(absx, absy)) - scale * LN2;
}

}  // namespace mcv
