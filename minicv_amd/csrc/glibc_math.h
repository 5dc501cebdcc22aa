// glibc_math.h — glibc 2.35's cbrt and hypot restated operation for operation, and the branch
// structure of its clog's real part (host and device).
//
// The reference's AP3P solver (ap3p.cpp:10-59, solveQuartic) runs std::cbrt and std::sqrt of
// std::complex<double> through libstdc++, i.e. glibc's cbrt and csqrt (whose general branch calls
// glibc's hypot) [ext: glibc 2.35, the container's and the GPU box's libm; sysdeps/ieee754/dbl-64
// s_cbrt.c and e_hypot.c]. Neither is correctly rounded, so a device that calls its own (ocml) cbrt /
// hypot returns other last bits, which the quartic's two Newton polish passes then carry into the
// pose. These restatements compute glibc's bits: every product, sum and quotient rounded as written,
// in glibc's order (the x86_64 build has no FMA in either function). tests/test_glibc_math.py checks
// both against the host's libm bit for bit on millions of inputs, and glibc_clog_re (with the host's
// log / log1p) against glibc's clog.
#pragma once

#include "mcv_common.h"

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
// scalings of huge and tiny arguments. The branch structure and every argument are glibc's; the
// log / log1p themselves are the device's (ocml) on the GPU and libm's in the host twin, so this part
// agrees with glibc to the last bit only where those two do (tests/test_gpu_pnp.py measures the share).
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
    if (absx == 1 && scale == 0) return log1p(absy * absy) / 2;
    if (absx > 1 && absx < 2 && absy < 1 && scale == 0) {
        double d2m1 = (absx - 1) * (absx + 1);
        if (absy >= EPS) d2m1 += absy * absy;
        return log1p(d2m1) / 2;
    }
    if (absx < 1 && absx >= 0.5 && absy < EPS / 2 && scale == 0) return log1p((absx - 1) * (absx + 1)) / 2;
    if (absx < 1 && absx >= 0.5 && scale == 0 && absx * absx + absy * absy >= 0.5)
        return log1p(glibc_x2y2m1(absx, absy)) / 2;
    return log(glibc_hypot(absx, absy)) - scale * LN2;
}

}  // namespace mcv
