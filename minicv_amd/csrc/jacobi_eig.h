// jacobi_eig.h — cv::eigen of a 9x9 symmetric matrix exactly as OpenCV 4.x computes it
// (hal::Jacobi -> JacobiImpl_<double>, core lapack.cpp [ext, restated]) for the minimal solvers
// of the RANSAC hypothesis kernels: HomographyEstimatorCallback::runKernel (LtL, 4 points) and
// run8Point (A = sum r r^T, 8 points) take the eigenvector of the smallest eigenvalue.
//
// JacobiImpl_ (the same algorithm as linalg.h's host jacobi_eigen, restated here in the form a
// GPU lane runs): classical Jacobi. The pivot (k, l) is the first maximum |A(i, indR[i])| over
// rows 0..n-2, then |A(indC[i], i)| over columns 1..n-1 — indR / indC hold per-row / per-column
// argmaxes of the strict upper triangle and are refreshed only for rows / columns k and l after a
// rotation (the others go stale, as in OpenCV). Stop when |p| <= DBL_EPSILON or after n*n*30
// rotations; y = (W[l] - W[k]) / 2, t = |y| + hypot(p, y), s = hypot(p, t), c = t / s, s = p / s,
// t = (p / t) p, signs flipped for y < 0; lapack.cpp's own hypot (cv_hypot, epnp.h). Only the strict
// upper triangle is read or written. Then a descending selection sort of W, rows of V swapped along.
//
// Layout: the working set is 127 doubles — [0, 36) the strict upper triangle packed by rows
// (eig_tri), [36, 45) W (the running diagonal), [45, 126) V row-major, a junk slot. On the GPU it lives in LDS,
// one 127-double slice per lane (EigWsLane; the odd stride keeps a half-wave's accesses to one
// element bank-conflict-free, a compile-time element index is an immediate offset); the data-
// dependent (k, l) indexing would otherwise put the matrices in scratch. On the host (twins, the
// single-lane winner kernels) it is a private array (EigWsLocal). Both run the same code and round
// identically (-ffp-contract=off; division and sqrt are IEEE on both sides).
// indR / indC are kept in registers as 4-bit fields of one 32-bit word each. The rotation's five
// quotients run gfx950's refined-reciprocal division inside its exact domain (eig_rotation).
#pragma once

#include <cstdlib>
#include <type_traits>
#include "mcv_common.h"
#include "epnp.h"   // cv_hypot (lapack.cpp's hypot)

namespace mcv {

// [0, 36) strict upper triangle, [36, 45) W, [45, 126) V, 126 = a junk slot (the rotation's
// branch-free form sends the two skipped indices there).
static constexpr int kEigA = 0, kEigW = 36, kEigV = 45, kEigJunk = 126, kEigWs = 127;
// The split solve (eig9_jacobi<WS, true> + eig9_replay): pass 1 keeps only the upper triangle and W
// (45 doubles, an odd lane stride: 360 B per lane instead of 1016; it runs the 7-pair lane-slice form,
// which needs no junk slot) and logs each
// rotation; pass 2 replays the log on V alone (81 doubles, odd stride). Same operations on the same
// values in the same order as the one-pass solve, so the same bits.
static constexpr int kEigAwWs = 45, kEigVWs = 81;
// One logged rotation: c (JacobiImpl_'s c = t / hypot(p, t) lies in [1/sqrt(2), 1], so its bits 62..53
// are always 0b0111111111 and bit 63 is 0: bits 63..53 carry (k << 4) | l instead) and s.
struct alignas(16) EigRot {
    double c, s;
};
MCV_HD bool eig_rot_c_ok(double c) { return c >= 0.5 && c <= 1.0; }
MCV_HD double eig_rot_pack(double c, int k, int l) {
    const uint64_t b = (__builtin_bit_cast(uint64_t, c) & ((1ull << 53) - 1)) | ((uint64_t)((k << 4) | l) << 53);
    return __builtin_bit_cast(double, b);
}
MCV_HD double eig_rot_c(double e, int& k, int& l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, e);
    const int kl = (int)(b >> 53);
    k = kl >> 4;
    l = kl & 15;
    return __builtin_bit_cast(double, (b & ((1ull << 53) - 1)) | (0x1FFull << 53));
}
// Lanes per hypothesis-kernel block: the 1016-byte working set per lane makes LDS the occupancy
// limit (160 KB per CU). 40 lanes = 4 blocks of 40.6 KB per CU, one wave on every SIMD (cfg3 screen,
// 2^20 hypotheses: 64 -> 39 lanes took the H generate 13.9 -> 11.4 ms; 39 vs 40 lanes 9.63 vs 9.34 ms
// in scripts/eig_lanes_screen.sh).
static constexpr int kEigLanes = 40;
// Packed index of A(r, c), r < c < 9: row r starts at 7r - r(r-1)/2 - 1 + (r + 1); the base is
// r(15 - r)/2 - 1 (r(15 - r) is even), one 24-bit multiply for a dynamic r.
MCV_HD int eig_row_base(int r) {
#if defined(__HIP_DEVICE_COMPILE__)
    return (int)(__umul24((unsigned)r, (unsigned)(15 - r)) >> 1) - 1;
#else
    return ((r * (15 - r)) >> 1) - 1;
#endif
}
MCV_HD int eig_tri(int r, int c) { return eig_row_base(r) + c; }

struct EigWsLocal {
    double d[kEigWs];
    MCV_HD double& operator[](int e) { return d[e]; }
};

// Lane-private slices of a __shared__ double[kEigWs * lanes] block: p = block + lane * kEigWs. The
// odd stride (127 doubles) puts a half-wave's 64-bit accesses to one element on distinct bank pairs,
// and every address is lane base + 8 e (a compile-time element is an immediate offset, a dynamic one
// a shift-add: no multiply by a non-power-of-two lane count).
struct EigWsLane {
    double* p;
    MCV_HD double& operator[](int e) { return p[e]; }
};

// Byte offsets of the rotated pairs per pivot: row tri(k, l) holds in word j (j < 7) the elements
// (A(i|k), A(i|l)) of the packed upper triangle as 8 e in the low / high 16 bits, for i = i_j, the j-th
// index outside {k, l} in increasing order (i_j = j + (j >= k) + (j >= l - 1)). The GPU lane-slice
// solver reads one 32-byte row per rotation (constant memory, L1-resident) instead of selecting the
// elements with ~100 integer ops, and rotates and rescans these 7 pairs only (round 6; before, 9 pairs
// with the two at i = k, l sent to a junk slot, whose (0, 0) rotated to (+0, +0) and never won a
// rescan: the same result with 12 more fp64 operations, 4 more LDS accesses and two more rescan steps
// per rotation). The host / generic path keeps the 9-pair branch-free form.
struct EigPairLut {
    uint32_t w[36][8];
};
constexpr EigPairLut eig_make_pair_lut7() {
    EigPairLut t{};
    for (int k = 0; k < 9; ++k)
        for (int l = k + 1; l < 9; ++l) {
            const int row = ((k * (15 - k)) >> 1) - 1 + l;
            int j = 0;
            for (int i = 0; i < 9; ++i) {
                if (i == k || i == l) continue;
                const int e0 = i < k ? ((i * (15 - i)) >> 1) - 1 + k : ((k * (15 - k)) >> 1) - 1 + i;
                const int e1 = i < l ? ((i * (15 - i)) >> 1) - 1 + l : ((l * (15 - l)) >> 1) - 1 + i;
                t.w[row][j++] = (uint32_t)(8 * e0) | ((uint32_t)(8 * e1) << 16);
            }
        }
    return t;
}
#if defined(__HIP__)
static __constant__ EigPairLut kEigPairLut7 = eig_make_pair_lut7();
#endif

// 4-bit fields: indR[i] at field i (i = 0..7), indC[i] at field i - 1 (i = 1..8).
MCV_HD int eig_nib(uint32_t x, int i) { return (int)((x >> (4 * i)) & 15u); }
MCV_HD uint32_t eig_set_nib(uint32_t x, int i, int v) {
    const uint32_t m = 15u << (4 * i);
    return (x & ~m) | (((uint32_t)v << (4 * i)) & m);
}

// JacobiImpl_'s rotation from the pivot p (|p| > DBL_EPSILON) and y = (W[l] - W[k]) / 2:
//   t = |y| + hypot(p, y); s = hypot(p, t); c = t / s; s = p / s; t = (p / t) p; signs for y < 0.
// Here t >= |p| and s >= t, so the second hypot's quotient is |p| / t and every divisor is at least
// |p| > 2^-64. Device: when the first hypot's larger operand stays below 2^60 and its quotient's
// numerator is 0 or at least 2^-900 (always, for the normalised systems of the minimal solvers),
// all five quotients take gfx950's refined-reciprocal form (bit-identical to IEEE there); a lane
// outside that domain takes the IEEE divisions (a branch no lane takes on these systems, so the
// wave skips it). Host: the IEEE divisions.
MCV_HD void eig_rotation(double p, double y, double& c, double& s, double& t) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double ap = __builtin_fabs(p), ay = __builtin_fabs(y);
    const bool ag = ap > ay;
    const double hi = ag ? ap : ay, lo = ag ? ay : ap;
    if (__builtin_expect(hi <= 0x1p60 && (lo == 0.0 || lo >= 0x1p-900), 1)) {
        const double r1 = div_f64_refined(lo, hi, rcp_f64_refined(hi));
        const double h1 = hi * sqrt_f64_1to2(1 + r1 * r1);   // r1 <= 1
        double tt = ay + h1;          // hypot(p, y): hi > 0 here, so the `else 0` case cannot occur
        const double rt = rcp_f64_refined(tt);
        const double r2 = div_f64_refined(ap, tt, rt);
        const double ss = tt * sqrt_f64_1to2(1 + r2 * r2);   // hypot(p, t) with t >= |p|
        const double rs = rcp_f64_refined(ss);
        c = div_f64_refined(tt, ss, rs);
        s = div_f64_refined(p, ss, rs);
        t = div_f64_refined(p, tt, rt) * p;
    } else {
        t = ay + cv_hypot(p, y);
        s = cv_hypot(p, t);
        c = t / s;
        s = p / s;
        t = (p / t) * p;
    }
#else
    t = __builtin_fabs(y) + cv_hypot(p, y);
    s = cv_hypot(p, t);
    c = t / s;
    s = p / s;
    t = (p / t) * p;
#endif
    if (y < 0) s = -s, t = -t;
}

// First maximum (by magnitude) of a candidate pair in scan order: the later one wins only when
// strictly greater. Values stay signed; the compare takes the magnitudes (operand modifiers).
MCV_HD void eig_pick(double& v, int& kl, double v2, int kl2) {
    const bool t = __builtin_fabs(v) < __builtin_fabs(v2);
    v = t ? v2 : v;
    kl = t ? kl2 : kl;
}

// cv::eigen on the 9x9 symmetric matrix whose strict upper triangle (packed) and diagonal the caller
// stored at ws[kEigA..] and ws[kEigW..]. On return w[] holds the eigenvalues in descending order and
// the function returns the workspace row of V (the original row index) that the sort moved to
// position `pos` — V row `pos` of OpenCV's result is ws[kEigV + 9 * ret + j]. Returns the rotation
// count through *iters when non-null (diagnostics).
//
// LOG = true (pass 1 of the split solve): the workspace is the 45-double AW slice, V is neither
// initialised nor rotated, and rotation t goes to log[t * logStride] (EigRot, c packed with k, l).
// *iters = the rotation count, or -1 when it would exceed logCap or a c falls outside [0.5, 1] (not
// for finite input; the caller then runs the one-pass solve). The return value is as above; the
// eigenvector is row `ret` of the V that eig9_replay rebuilds from the log.
template <class WS, bool LOG = false>
MCV_HD int eig9_jacobi(WS& ws, double (&w)[9], int pos, int* iters = nullptr, EigRot* log = nullptr,
                       int logStride = 0, int logCap = 0) {
    constexpr int n = 9;
    constexpr int junk = kEigJunk;   // the generic 9-pair form's skipped pairs (not with LOG: lane slices only)
    static_assert(!LOG || std::is_same<WS, EigWsLane>::value, "the logged solve runs on lane slices");
    if constexpr (!LOG) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = 0; i < n * n; ++i) ws[kEigV + i] = (i / n == i % n) ? 1.0 : 0.0;
    }
    if constexpr (!LOG) ws[junk] = 0.0;   // stays +0: the skipped pair rotates (0, 0) into (+0, +0)
    bool logOk = true;
    uint32_t indR = 0, indC = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int k = 0; k < n; ++k) {
        if (k < n - 1) {
            int m = k + 1;
            double mv = __builtin_fabs(ws[eig_tri(k, k + 1)]);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int i = k + 2; i < n; ++i) {
                const double val = __builtin_fabs(ws[eig_tri(k, i)]);
                if (mv < val) mv = val, m = i;
            }
            indR = eig_set_nib(indR, k, m);
        }
        if (k > 0) {
            int m = 0;
            double mv = __builtin_fabs(ws[eig_tri(0, k)]);
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int i = 1; i < k; ++i) {
                const double val = __builtin_fabs(ws[eig_tri(i, k)]);
                if (mv < val) mv = val, m = i;
            }
            indC = eig_set_nib(indC, k - 1, m);
        }
    }
    int it = 0;
    for (; it < n * n * 30; ++it) {
        // pivot (k, l): the first maximum over the 16 candidates in OpenCV's scan order (rows 0..7
        // through indR, then columns 1..8 through indC), as a pairwise tree (first wins on ties)
        double cv[16];
        int ck[16];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = 0; i < n - 1; ++i) {
            const int c = eig_nib(indR, i);
            cv[i] = ws[eig_row_base(i) + c];
            ck[i] = i * 16 + c;
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = 1; i < n; ++i) {
            const int r = eig_nib(indC, i - 1);
            cv[7 + i] = ws[eig_row_base(r) + i];
            ck[7 + i] = r * 16 + i;
        }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int h = 1; h < 16; h *= 2)
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int i = 0; i < 16; i += 2 * h) eig_pick(cv[i], ck[i], cv[i + h], ck[i + h]);
        const int k = ck[0] >> 4, l = ck[0] & 15;
        const int ekl = eig_tri(k, l);
        const double p = cv[0];   // = A(k, l)
        if (__builtin_fabs(p) <= kDblEpsilon) break;
        // every operand of the rotation is read before anything is written back (the reads do not
        // depend on the scalar chain, so their LDS latency hides behind it): W[k], W[l], for every
        // other i the pair (A(k|i), A(l|i)) of the upper triangle (i = k, l read and write the junk
        // slot), and V rows k and l
        const double wk = ws[kEigW + k], wl = ws[kEigW + l];
#if defined(__HIP_DEVICE_COMPILE__)
        if constexpr (std::is_same<WS, EigWsLane>::value) {
            // the 7 pairs of the indices outside {k, l} (kEigPairLut7: 2 vector loads from L1)
            constexpr int P7 = n - 2;
            const uint4* lr = reinterpret_cast<const uint4*>(kEigPairLut7.w[ekl]);
            const uint4 q0 = lr[0], q1 = lr[1];
            const uint32_t qw[P7] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z};
            char* const b = reinterpret_cast<char*>(ws.p);
            int o0[P7], o1[P7];
            double x0[P7], x1[P7], wa[n], wb[n];
#pragma unroll
            for (int j = 0; j < P7; ++j) {
                o0[j] = (int)(qw[j] & 0xffffu);
                o1[j] = (int)(qw[j] >> 16);
                x0[j] = *reinterpret_cast<const double*>(b + o0[j]);
                x1[j] = *reinterpret_cast<const double*>(b + o1[j]);
            }
            const int vk = kEigV + (k << 3) + k, vl = kEigV + (l << 3) + l;   // + 9 k, + 9 l
            if constexpr (!LOG) {
#pragma unroll
                for (int i = 0; i < n; ++i) {
                    wa[i] = ws[vk + i];
                    wb[i] = ws[vl + i];
                }
            }
            const double y = (wl - wk) * 0.5;
            double c, s, t;
            eig_rotation(p, y, c, s, t);
            if constexpr (LOG) {
                if (it >= logCap || !eig_rot_c_ok(c)) {
                    logOk = false;
                    break;
                }
                EigRot e;
                e.c = eig_rot_pack(c, k, l);
                e.s = s;
                log[(int64_t)it * logStride] = e;
            }
            ws[ekl] = 0;
            ws[kEigW + k] = wk - t;
            ws[kEigW + l] = wl + t;
            double nk[P7], nl[P7];
#pragma unroll
            for (int j = 0; j < P7; ++j) {
                nk[j] = x0[j] * c - x1[j] * s;
                nl[j] = x0[j] * s + x1[j] * c;
                *reinterpret_cast<double*>(b + o0[j]) = nk[j];
                *reinterpret_cast<double*>(b + o1[j]) = nl[j];
            }
            if constexpr (!LOG) {
#pragma unroll
                for (int i = 0; i < n; ++i) {
                    ws[vk + i] = wa[i] * c - wb[i] * s;
                    ws[vl + i] = wa[i] * s + wb[i] * c;
                }
            }
            // the rescans over the 7 pairs in index order: i_j > k <=> j >= k, i_j > l <=> j >= l - 1;
            // a tracker keeps the pair position j of its first maximum (-1: none beat the running 0, the
            // start index: k + 1 for a row, 0 for a column), mapped back to i_j at the end
            int jRk = -1, jCk = -1, jRl = -1, jCl = -1;
            double vRk = 0, vCk = 0, vRl = 0, vCl = 0;
#pragma unroll
            for (int j = 0; j < P7; ++j) {
                const double ak = __builtin_fabs(nk[j]), al = __builtin_fabs(nl[j]);
                const bool tRk = j >= k && __builtin_fabs(vRk) < ak, tCk = j < k && __builtin_fabs(vCk) < ak;
                const bool tRl = j >= l - 1 && __builtin_fabs(vRl) < al, tCl = j < l - 1 && __builtin_fabs(vCl) < al;
                vRk = tRk ? nk[j] : vRk; jRk = tRk ? j : jRk;
                vCk = tCk ? nk[j] : vCk; jCk = tCk ? j : jCk;
                vRl = tRl ? nl[j] : vRl; jRl = tRl ? j : jRl;
                vCl = tCl ? nl[j] : vCl; jCl = tCl ? j : jCl;
            }
            auto orig = [&](int j) { return j + (j >= k ? 1 : 0) + (j >= l - 1 ? 1 : 0); };
            const int mRk = jRk < 0 ? k + 1 : orig(jRk), mCk = jCk < 0 ? 0 : orig(jCk);
            const int mRl = jRl < 0 ? l + 1 : orig(jRl), mCl = jCl < 0 ? 0 : orig(jCl);
            if (k < n - 1) indR = eig_set_nib(indR, k, mRk);
            if (k > 0) indC = eig_set_nib(indC, k - 1, mCk);
            if (l < n - 1) indR = eig_set_nib(indR, l, mRl);
            indC = eig_set_nib(indC, l - 1, mCl);   // l >= 1
            continue;
        }
#endif
        const int rk = eig_row_base(k), rl = eig_row_base(l);
        int e0[n], e1[n];
        double a0[n], b0[n], va[n], vb[n];
        {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int i = 0; i < n; ++i) {
                // branch-free index selection (a select of LDS addresses feeding a load is otherwise
                // turned into control flow around each load)
                const int mk = -(int)(i < k), ml = -(int)(i < l), ms = -(int)(i == k || i == l);
                const int x0 = ((eig_row_base(i) + k) & mk) | ((rk + i) & ~mk);
                const int x1 = ((eig_row_base(i) + l) & ml) | ((rl + i) & ~ml);
                e0[i] = (junk & ms) | (x0 & ~ms);
                e1[i] = (junk & ms) | (x1 & ~ms);
                a0[i] = ws[e0[i]];
                b0[i] = ws[e1[i]];
            }
        }
        const int vk = kEigV + (k << 3) + k, vl = kEigV + (l << 3) + l;   // + 9 k, + 9 l
        if constexpr (!LOG) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int i = 0; i < n; ++i) {
                va[i] = ws[vk + i];
                vb[i] = ws[vl + i];
            }
        }
        const double y = (wl - wk) * 0.5;
        double c, s, t;
        eig_rotation(p, y, c, s, t);
        if constexpr (LOG) {
            if (it >= logCap || !eig_rot_c_ok(c)) {
                logOk = false;
                break;
            }
            EigRot e;
            e.c = eig_rot_pack(c, k, l);
            e.s = s;
            log[(int64_t)it * logStride] = e;
        }
        ws[ekl] = 0;
        ws[kEigW + k] = wk - t;
        ws[kEigW + l] = wl + t;
        // rotate rows and columns k and l; nk / nl keep the new values for the rescans (at i = k, l the
        // junk pair (0, 0) rotates to (+0, +0): A(k, l) = 0 without a select)
        double nk[n], nl[n];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = 0; i < n; ++i) {
            nk[i] = a0[i] * c - b0[i] * s;
            nl[i] = a0[i] * s + b0[i] * c;
            ws[e0[i]] = nk[i];
            ws[e1[i]] = nl[i];
        }
        // rotate eigenvectors
        if constexpr (!LOG) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
            for (int i = 0; i < n; ++i) {
                ws[vk + i] = va[i] * c - vb[i] * s;
                ws[vl + i] = va[i] * s + vb[i] * c;
            }
        }
        // refresh indR / indC of rows and columns k and l (first maximum by magnitude). OpenCV takes
        // the first in-range element unconditionally; here the index starts there (k + 1 for a row,
        // 0 for a column) with a running value of 0, which only a strictly larger |value| replaces —
        // the same index for finite values. Values stay signed (magnitudes through the compare).
        int mRk = k + 1, mCk = 0, mRl = l + 1, mCl = 0;
        double vRk = 0, vCk = 0, vRl = 0, vCl = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = 0; i < n; ++i) {
            const double ak = __builtin_fabs(nk[i]), al = __builtin_fabs(nl[i]);
            const bool tRk = i > k && __builtin_fabs(vRk) < ak, tCk = i < k && __builtin_fabs(vCk) < ak;
            const bool tRl = i > l && __builtin_fabs(vRl) < al, tCl = i < l && __builtin_fabs(vCl) < al;
            vRk = tRk ? nk[i] : vRk; mRk = tRk ? i : mRk;
            vCk = tCk ? nk[i] : vCk; mCk = tCk ? i : mCk;
            vRl = tRl ? nl[i] : vRl; mRl = tRl ? i : mRl;
            vCl = tCl ? nl[i] : vCl; mCl = tCl ? i : mCl;
        }
        if (k < n - 1) indR = eig_set_nib(indR, k, mRk);
        if (k > 0) indC = eig_set_nib(indC, k - 1, mCk);
        if (l < n - 1) indR = eig_set_nib(indR, l, mRl);
        indC = eig_set_nib(indC, l - 1, mCl);   // l >= 1
    }
    if (iters) *iters = logOk ? it : -1;
    // descending selection sort, rows of V swapped along (tracked as a permutation)
    int perm[n];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < n; ++i) {
        w[i] = ws[kEigW + i];
        perm[i] = i;
    }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int k = 0; k < n - 1; ++k) {
        int m = k;
        double wm = w[k];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = k + 1; i < n; ++i)
            if (wm < w[i]) m = i, wm = w[i];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int i = k + 1; i < n; ++i)
            if (i == m) {
                const double tw = w[k]; w[k] = w[i]; w[i] = tw;
                const int tp = perm[k]; perm[k] = perm[i]; perm[i] = tp;
            }
    }
    int r = 0;
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int i = 0; i < n; ++i)
        if (i == pos) r = perm[i];
    return r;
}

// Pass 2 of the split solve: V (the 81-double slice v, row-major) rebuilt from pass 1's rotation log,
// rotation by rotation exactly as eig9_jacobi rotates it (rows k and l, the same products and sums).
// The columns of V rotate independently, so C columns from c0 can run on one lane (C = 9: the whole
// matrix; C = 3: three lanes per hypothesis). The log entries stream through a ring of D loads in
// flight (one load ahead waited out the HBM latency every rotation: 2.1 ms per 2^20 hypotheses).
// The caller initialises V to the identity.
// TR: V stored transposed (element (i, c) at 9 c + i: a lane's columns are contiguous).
template <int C, int D, bool TR = false, class WS>
MCV_HD void eig9_replay_cols(WS& v, int c0, const EigRot* log, int64_t logStride, int nrot) {
    EigRot q[D];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
    for (int u = 0; u < D; ++u) q[u] = u < nrot ? log[(int64_t)u * logStride] : EigRot{0.0, 0.0};
    for (int t0 = 0; t0 < nrot; t0 += D) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
        for (int u = 0; u < D; ++u) {
            const EigRot e = q[u];
            const int tn = t0 + u + D;
            if (tn < nrot) q[u] = log[(int64_t)tn * logStride];
            if (t0 + u < nrot) {
                int k, l;
                const double c = eig_rot_c(e.c, k, l), s = e.s;
                // element (row, c0 + i): row-major 9 row + c0 + i, transposed 9 (c0 + i) + row
                const int vk = TR ? 9 * c0 + k : (k << 3) + k + c0, vl = TR ? 9 * c0 + l : (l << 3) + l + c0;
                constexpr int st = TR ? 9 : 1;
                double va[C], vb[C];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
                for (int i = 0; i < C; ++i) {
                    va[i] = v[vk + st * i];
                    vb[i] = v[vl + st * i];
                }
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
#endif
                for (int i = 0; i < C; ++i) {
                    v[vk + st * i] = va[i] * c - vb[i] * s;
                    v[vl + st * i] = va[i] * s + vb[i] * c;
                }
            }
        }
    }
}

template <class WS>
MCV_HD void eig9_replay(WS& v, const EigRot* log, int64_t logStride, int nrot) {
    for (int i = 0; i < 81; ++i) v[i] = (i / 9 == i % 9) ? 1.0 : 0.0;
    eig9_replay_cols<9, 4>(v, 0, log, logStride, nrot);
}

}  // namespace mcv
