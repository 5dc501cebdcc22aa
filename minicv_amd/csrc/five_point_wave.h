// five_point_wave.h — the five-point solve of hyp_essential.h spread over a group of G lanes of
// one wave64 (G = 16, 32 or 64; device only).
//
// e_solve5 run by one lane per hypothesis is latency-bound: ~2.7 ms per call on gfx950 (its
// 5 x 9 / 10 x 20 working matrices and root lists are indexed dynamically, so they live in
// scratch, and one lane runs every step). Here G lanes solve one hypothesis (64 / G hypotheses
// per wave): the working matrices sit in LDS, and the lanes split each step by element — the
// null-space elimination by (row, column), the 10 x 20 coefficient matrix by (row, monomial), the
// Gauss-Jordan elimination by (row, column), the root bracketing by derivative interval (at most
// 11, hence G >= 16), the model recovery by root.
//
// Every element still sees exactly e_solve5's operation sequence, so the result is bit-identical
// to the host twin and the oracle:
//   * pivot searches are arg-max reductions keyed (|v|, position) with the first position winning
//     ties, which is the serial loop's "first strict maximum" (NaN never wins, as in the loop);
//   * maxima (matrix scales, Cauchy bound) are order-independent;
//   * each coefficient-matrix entry accumulates its (at most 3 per product) contributions in
//     e_acc21's loop order, from a compile-time table;
//   * dot products (Gram-Schmidt) stay serial, evaluated redundantly by every lane of the group;
//   * each derivative level runs a Horner specialised to its degree;
//   * the root list keeps the serial de-duplication rule (an exact zero at b is dropped when it
//     equals the last kept root), evaluated by comparing each candidate with the previous one.
// Groups of one wave may take different branches (degenerate samples, root counts); the wave
// runs both sides, and the block is one wave, so the barriers never wait on another wave.
#pragma once

#if !defined(__HIPCC__)
#error "five_point_wave.h is device code (include it from .hip sources only)"
#endif

#include "mcv_common.h"
#include "hyp_essential.h"
#include "kernels.h"   // EStage

namespace mcv {

struct EWave {
    double pt[4][5];     // the sample: x1, y1, x2, y2
    double a[5][9];      // 5 x 9 epipolar system (original column order; perm holds the pivots)
    double nb[4][9];     // orthonormal null basis
    double v[9];         // Gram-Schmidt working vector
    double eet[6][10];   // E E^T (upper triangle, pairs 00 01 02 11 12 22) as quadratics
    double tr[10];
    double lam[9][10];   // Lambda(i, k) = 2 (E E^T)_ik - tr [i == k]
    double A[10][20];    // cubic constraint matrix, reduced in place
    double det[11];      // det(B(z))
    double c[11];        // det(B(z)) made monic
    double rp[10];       // roots of the previous level (ascending)
    int perm[9];
    int inv[9];
};

// e_acc21's contributions per cubic monomial t, in its (a, b >= a, c) loop order: (pair, c).
struct EAccTab {
    int n[20];
    int p[20][3];
    int c[20][3];
};
constexpr int ew_pair_c(int a, int b) { return a == 0 ? b : (a == 1 ? 3 + b : (a == 2 ? 5 + b : 9)); }
constexpr int ew_triple_c(int a, int b, int c) {
    const int code = a * 16 + b * 4 + c;
    const int codes[20] = {0,  21, 1,  5,  2,  3,  22, 23, 6,  7,
                           10, 11, 15, 26, 27, 31, 42, 43, 47, 63};
    for (int t = 0; t < 20; ++t)
        if (codes[t] == code) return t;
    return 19;
}
constexpr EAccTab ew_acc_tab() {
    EAccTab T{};
    for (int a = 0; a < 4; ++a)
        for (int b = a; b < 4; ++b)
            for (int c = 0; c < 4; ++c) {
                const int lo = c < a ? c : a;
                const int hi = c > b ? c : b;
                const int mid = c < a ? a : (c > b ? b : c);
                const int t = ew_triple_c(lo, mid, hi);
                T.p[t][T.n[t]] = ew_pair_c(a, b);
                T.c[t][T.n[t]] = c;
                ++T.n[t];
            }
    return T;
}
__device__ constexpr EAccTab kEAccTab = ew_acc_tab();
// pair index -> (a, b)
__device__ constexpr int kEPairA[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
__device__ constexpr int kEPairB[10] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};

__device__ __forceinline__ void ew_sync() { __syncthreads(); }

// Lanes [base, base + G) of the wave work on one hypothesis; sub = lane - base.
template <int G>
struct EGroup {
    // 8-lane groups serve the matrix phases only (ew_stage_hypothesis); the root bracketing by
    // interval needs >= 11 lanes (ew_real_roots), so a full solve takes 16, 32 or 64
    static_assert(G == 8 || G == 16 || G == 32 || G == 64, "group of 8, 16, 32 or 64 lanes");
    int sub, base;
    __device__ explicit EGroup(int lane) : sub(lane & (G - 1)), base(lane & ~(G - 1)) {}
    __device__ uint64_t ballot(bool p) const {
        const uint64_t b = __ballot(p);
        if constexpr (G == 64) return b;
        else return (b >> base) & ((1ull << G) - 1ull);
    }
    __device__ uint64_t below() const { return (1ull << sub) - 1ull; }
    __device__ double shfl(double v, int src) const { return __shfl(v, base + src); }
    // max of non-negative keys over the group
    __device__ double max(double x) const {
#pragma unroll
        for (int o = G / 2; o >= 1; o >>= 1) {
            const double y = __shfl_xor(x, o);
            x = y > x ? y : x;
        }
        return x;
    }
    // arg-max over the group: larger key wins, equal keys -> smaller position
    __device__ void argmax(double& key, int& pos) const {
#pragma unroll
        for (int o = G / 2; o >= 1; o >>= 1) {
            const double k2 = __shfl_xor(key, o);
            const int p2 = __shfl_xor(pos, o);
            const bool take = k2 > key || (k2 == key && p2 < pos);
            key = take ? k2 : key;
            pos = take ? p2 : pos;
        }
    }
};

// Local arg-max candidate update in ascending position order (strict: the first maximum stays).
__device__ __forceinline__ void ew_cand(double& key, int& pos, double v, int p) {
    if (v > key) { key = v; pos = p; }
}

__device__ __forceinline__ double ew_L(const EWave& S, int k, int v) { return S.nb[v][k]; }

// e_mul11(L[u], L[w])[pair]
__device__ __forceinline__ double ew_mul11(const EWave& S, int u, int w, int p) {
    const int a = kEPairA[p], b = kEPairB[p];
    return a == b ? ew_L(S, u, a) * ew_L(S, w, a) : ew_L(S, u, a) * ew_L(S, w, b) + ew_L(S, u, b) * ew_L(S, w, a);
}

// ---- e_null_basis (sample in S.pt) ---------------------------------------------------------------
template <int G>
__device__ __forceinline__ bool ew_null_basis(EWave& S, const EGroup<G>& g) {
    double loc = 0;
    for (int e = g.sub; e < 45; e += G) {
        const int i = e / 9, k = e - 9 * (e / 9);
        const double X1 = S.pt[0][i], Y1 = S.pt[1][i], X2 = S.pt[2][i], Y2 = S.pt[3][i];
        double val = 1.0;
        val = k == 0 ? X1 * X2 : val;
        val = k == 1 ? Y1 * X2 : val;
        val = k == 2 ? X2 : val;
        val = k == 3 ? X1 * Y2 : val;
        val = k == 4 ? Y1 * Y2 : val;
        val = k == 5 ? Y2 : val;
        val = k == 6 ? X1 : val;
        val = k == 7 ? Y1 : val;
        S.a[i][k] = val;
        const double av = fabs(val);
        loc = av > loc ? av : loc;
    }
    for (int e = g.sub; e < 9; e += G) S.perm[e] = e;
    const double scale = g.max(loc);
    ew_sync();
    if (!(scale > 0) || !isfinite(scale)) return false;
    for (int r = 0; r < 5; ++r) {
        double key = -2.0;
        int pos = 1 << 30;
        for (int e = g.sub; e < 45; e += G) {
            const int li = e / 9, lj = e - 9 * (e / 9);
            if (li >= r && lj >= r) {
                const double v = fabs(S.a[li][S.perm[lj]]);
                ew_cand(key, pos, v == v ? v : -1.0, e);
            }
        }
        g.argmax(key, pos);
        if (!(key > 1e-12 * scale)) return false;
        const int pr = pos / 9, pc = pos - 9 * (pos / 9);
        for (int e = g.sub; e < 9; e += G) {
            const double t0 = S.a[r][e], t1 = S.a[pr][e];
            S.a[r][e] = t1;
            S.a[pr][e] = t0;
        }
        if (g.sub == 0) {
            const int tp = S.perm[r];
            S.perm[r] = S.perm[pc];
            S.perm[pc] = tp;
        }
        ew_sync();
        const int pcol = S.perm[r];
        const double piv = S.a[r][pcol];
        for (int e = g.sub; e < 9; e += G)
            if (e > r) {
                const int col = S.perm[e];
                S.a[r][col] = S.a[r][col] / piv;
            }
        ew_sync();
        // rows i != r, columns j > r: every lane reads only its own elements, row r and column
        // pcol, none of which this step writes; column pcol is reset after a barrier.
        for (int e = g.sub; e < 45; e += G) {
            const int li = e / 9, lj = e - 9 * (e / 9);
            if (li != r && lj > r) {
                const int col = S.perm[lj];
                const double f = S.a[li][pcol];
                S.a[li][col] = S.a[li][col] - f * S.a[r][col];
            }
        }
        ew_sync();
        for (int e = g.sub; e < 5; e += G) S.a[e][pcol] = e == r ? 1.0 : 0.0;
        ew_sync();
    }
    for (int e = g.sub; e < 9; e += G) S.inv[S.perm[e]] = e;
    ew_sync();
    constexpr int kPer = (9 + G - 1) / G;
    double vk[kPer];
    for (int b = 0; b < 4; ++b) {
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
            const int k = g.sub + G * u;
            vk[u] = 0.0;
            if (k < 9) {
                const int jj = S.inv[k];
                vk[u] = jj == 5 + b ? 1.0 : (jj < 5 ? -S.a[jj][S.perm[5 + b]] : 0.0);
            }
        }
        for (int c = 0; c < b; ++c) {   // modified Gram-Schmidt: serial dot product, per-lane update
#pragma unroll
            for (int u = 0; u < kPer; ++u)
                if (g.sub + G * u < 9) S.v[g.sub + G * u] = vk[u];
            ew_sync();
            double d = 0;
#pragma unroll
            for (int k = 0; k < 9; ++k) d = d + S.nb[c][k] * S.v[k];
#pragma unroll
            for (int u = 0; u < kPer; ++u)
                if (g.sub + G * u < 9) vk[u] = vk[u] - d * S.nb[c][g.sub + G * u];
            ew_sync();
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u)
            if (g.sub + G * u < 9) S.v[g.sub + G * u] = vk[u];
        ew_sync();
        double s = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) s = s + S.v[k] * S.v[k];
        const double nrm = sqrt(s);
        if (!(nrm > 0)) return false;
#pragma unroll
        for (int u = 0; u < kPer; ++u)
            if (g.sub + G * u < 9) S.nb[b][g.sub + G * u] = vk[u] / nrm;
        ew_sync();
    }
    return true;
}

// ---- e_coeffs -----------------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ void ew_coeffs(EWave& S, const EGroup<G>& g) {
    for (int e = g.sub; e < 60; e += G) {   // E E^T: (pair of rows, quadratic monomial)
        const int pp = e / 10, t = e - 10 * (e / 10);
        const int ri = pp < 3 ? 0 : (pp < 5 ? 1 : 2);
        const int rj = pp < 3 ? pp : (pp < 5 ? pp - 2 : 2);
        double v = ew_mul11(S, 3 * ri + 0, 3 * rj + 0, t);
        v = v + ew_mul11(S, 3 * ri + 1, 3 * rj + 1, t);
        v = v + ew_mul11(S, 3 * ri + 2, 3 * rj + 2, t);
        S.eet[pp][t] = v;
    }
    ew_sync();
    for (int e = g.sub; e < 10; e += G) S.tr[e] = S.eet[0][e] + S.eet[3][e] + S.eet[5][e];
    ew_sync();
    for (int e = g.sub; e < 90; e += G) {
        const int ik = e / 10, t = e - 10 * (e / 10);
        const int i = ik / 3, k = ik - 3 * (ik / 3);
        const int lo = i < k ? i : k, hi = i < k ? k : i;
        const int pp = lo == 0 ? hi : (lo == 1 ? 2 + hi : 5);
        S.lam[ik][t] = 2.0 * S.eet[pp][t] - (i == k ? S.tr[t] : 0.0);
    }
    ew_sync();
    const int cof[3][4] = {{4, 8, 5, 7}, {5, 6, 3, 8}, {3, 7, 4, 6}};
    for (int e = g.sub; e < 200; e += G) {
        const int row = e / 20, t = e - 20 * (e / 20);
        const int n = kEAccTab.n[t];
        double acc = 0.0;
        if (row == 0) {
#pragma unroll
            for (int i = 0; i < 3; ++i)
                for (int u = 0; u < n; ++u) {
                    const int p = kEAccTab.p[t][u], c = kEAccTab.c[t][u];
                    const double m = ew_mul11(S, cof[i][0], cof[i][1], p) - ew_mul11(S, cof[i][2], cof[i][3], p);
                    acc = acc + m * ew_L(S, i, c);
                }
        } else {
            const int i = (row - 1) / 3, j = row - 1 - 3 * ((row - 1) / 3);
#pragma unroll
            for (int k = 0; k < 3; ++k)
                for (int u = 0; u < n; ++u) {
                    const int p = kEAccTab.p[t][u], c = kEAccTab.c[t][u];
                    acc = acc + S.lam[3 * i + k][p] * ew_L(S, 3 * k + j, c);
                }
        }
        S.A[row][t] = acc;
    }
    ew_sync();
}

// ---- e_eliminate (in place; C = A[:, 10:]) -------------------------------------------------------
template <int G>
__device__ __forceinline__ bool ew_eliminate(EWave& S, const EGroup<G>& g) {
    double loc = 0;
    for (int e = g.sub; e < 200; e += G) {
        const double v = fabs(S.A[e / 20][e - 20 * (e / 20)]);
        loc = v > loc ? v : loc;
    }
    const double scale = g.max(loc);
    if (!(scale > 0) || !isfinite(scale)) return false;
    for (int c = 0; c < 10; ++c) {
        const double lead = fabs(S.A[c][c]);
        double key = -2.0;
        int pos = 1 << 30;
        for (int e = g.sub; e < 10; e += G) {
            if (e == c) ew_cand(key, pos, lead, c);
            else if (e > c) {
                const double v = fabs(S.A[e][c]);
                ew_cand(key, pos, v == v ? v : -1.0, e);
            }
        }
        g.argmax(key, pos);
        const double best = lead == lead ? key : lead;
        if (!(best > 1e-13 * scale)) return false;
        const int p = pos;
        if (p != c)
            for (int e = g.sub; e < 20; e += G)
                if (e >= c) {
                    const double t0 = S.A[c][e], t1 = S.A[p][e];
                    S.A[c][e] = t1;
                    S.A[p][e] = t0;
                }
        ew_sync();
        const double piv = S.A[c][c];
        for (int e = g.sub; e < 20; e += G)
            if (e > c) S.A[c][e] = S.A[c][e] / piv;
        ew_sync();
        // each lane reads only its own elements, column c and row c (not written in this step)
        for (int e = g.sub; e < 200; e += G) {
            const int r = e / 20, k = e - 20 * (e / 20);
            if (r != c && k > c) S.A[r][k] = S.A[r][k] - S.A[r][c] * S.A[c][k];
        }
        ew_sync();
    }
    return true;
}

// Horner of fixed degree D (e_poly_eval's loop, unrolled: q stays in registers).
template <int D>
struct EPolyD {
    double q[D + 1];
    __device__ __forceinline__ double operator()(double x) const {
        double f = q[D];
#pragma unroll
        for (int k = D - 1; k >= 0; --k) f = f * x + q[k];
        return f;
    }
};

// One level of e_poly_real_roots at derivative degree D: lane s <= np brackets interval
// (a_s, b_s] (a_0 = -R, a_s = rp[s-1], b_s = rp[s], b_np = R); the kept roots replace S.rp.
template <int D, int G>
__device__ __forceinline__ int ew_level(EWave& S, const EGroup<G>& g, int j, int np, double R) {
    EPolyD<D> P;
#pragma unroll
    for (int k = 0; k <= D; ++k) P.q[k] = S.c[k + j] * e_falling(k + j, j);
    int type = 0;   // 1: exact zero at b, 2: bracketed root
    double val = 0.0, b = 0.0;
    if (g.sub <= np) {
        const double a = g.sub == 0 ? -R : S.rp[g.sub - 1];
        b = g.sub < np ? S.rp[g.sub] : R;
        const double fa = P(a), fb = P(b);
        if (fb == 0) {
            type = 1;
            val = b;
        } else if (fa != 0 && ((fa < 0) != (fb < 0))) {
            type = 2;
            val = e_root_bracketed_f(P, a, b, fa, fb);
        }
    }
    // serial rule: an exact zero at b is kept unless it equals the last kept root; a dropped
    // duplicate equals that root, so comparing with the previous candidate is the same test
    const uint64_t cand = g.ballot(type != 0);
    const uint64_t below = cand & g.below();
    const int prevSub = below ? 63 - __clzll(below) : g.sub;
    const double prevVal = g.shfl(val, prevSub);
    const bool keep = type == 2 || (type == 1 && (below == 0 || prevVal != b));
    const uint64_t km = g.ballot(keep);
    ew_sync();
    if (keep) S.rp[__popcll(km & g.below())] = val;
    ew_sync();
    return __popcll(km);
}

// ---- e_poly_real_roots on S.det (degree <= 10): roots land in S.rp, count returned -------------
template <int G>
__device__ __forceinline__ int ew_real_roots(EWave& S, const EGroup<G>& g) {
    int n = 0;
#pragma unroll
    for (int k = 1; k <= 10; ++k) n = S.det[k] != 0 ? k : n;
    if (n < 1) return 0;
    const double lead = S.det[n];
    double loc = 0.0;
    if (g.sub <= n) {
        const double ck = S.det[g.sub] / lead;
        S.c[g.sub] = ck;
        if (g.sub < n) {
            const double a = fabs(ck);
            loc = a > loc ? a : loc;
        }
    }
    const double R = 1.0 + g.max(loc);
    if (!isfinite(R)) return 0;
    ew_sync();
    int np = 0;
    for (int j = n - 1; j >= 0; --j) {
        switch (n - j) {
            case 1: np = ew_level<1>(S, g, j, np, R); break;
            case 2: np = ew_level<2>(S, g, j, np, R); break;
            case 3: np = ew_level<3>(S, g, j, np, R); break;
            case 4: np = ew_level<4>(S, g, j, np, R); break;
            case 5: np = ew_level<5>(S, g, j, np, R); break;
            case 6: np = ew_level<6>(S, g, j, np, R); break;
            case 7: np = ew_level<7>(S, g, j, np, R); break;
            case 8: np = ew_level<8>(S, g, j, np, R); break;
            case 9: np = ew_level<9>(S, g, j, np, R); break;
            default: np = ew_level<10>(S, g, j, np, R); break;
        }
    }
    return np;
}

// ---- e_solve5 on the sample in S.pt: lane sub < count ends with model sub in E (row-major) -------
template <int G>
__device__ __forceinline__ int ew_solve5(EWave& S, const EGroup<G>& g, double (&E)[9]) {
    if (!ew_null_basis(S, g)) return 0;
    ew_coeffs(S, g);
    if (!ew_eliminate(S, g)) return 0;
    double bx[3][4], by[3][4], bc[3][5];
    e_bz(&S.A[0][10], 20, bx, by, bc);
    {
        double det[11];
        e_detpoly(bx, by, bc, det);
        if (g.sub == 0)
#pragma unroll
            for (int k = 0; k < 11; ++k) S.det[k] = det[k];
        ew_sync();
    }
    const int nr = ew_real_roots(S, g);
    bool ok = false;
    if (g.sub < nr) ok = e_model_at(bx, by, bc, S.nb[0], S.nb[1], S.nb[2], S.nb[3], S.rp[g.sub], E);
    // compact in root order: slot t takes the model of the t-th successful root
    const uint64_t m = g.ballot(ok);
    uint64_t mm = m;
#pragma unroll
    for (int t = 0; t < kEMaxModels; ++t) mm = t < g.sub ? mm & (mm - 1) : mm;
    const int src = mm ? __ffsll((unsigned long long)mm) - 1 : 0;
    double out[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) out[k] = g.shfl(E[k], src);
#pragma unroll
    for (int k = 0; k < 9; ++k) E[k] = out[k];
    return __popcll(m);
}

// Stage a sample (four arrays of 5) into S.pt.
template <int G>
__device__ __forceinline__ void ew_stage(EWave& S, const EGroup<G>& g, const double* x1, const double* y1,
                                         const double* x2, const double* y2) {
    for (int e = g.sub; e < 20; e += G) {
        const int c = e / 5, i = e - 5 * (e / 5);
        const double* src = c == 0 ? x1 : (c == 1 ? y1 : (c == 2 ? x2 : y2));
        S.pt[c][i] = src[i];
    }
    ew_sync();
}

// One hypothesis (e_hypothesis): every lane of the group runs the Philox sampler (same values),
// lanes 0..19 fetch the sample. Returns the model count (0 = no model) or kStatusNoSample; lane
// sub < count holds model sub.
template <int G>
__device__ __forceinline__ int ew_hypothesis(EWave& S, const EGroup<G>& g, const double* pts4, int N,
                                             const Sampler& smp, uint64_t hyp, double (&E)[9], int* idx_out) {
    SubsetSrc<5> src(smp, hyp);
    int idx[5];
    bool found = false;   // search and solve apart (h_hypothesis): one solve pass per wave
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, idx);
        if (got < 0) break;
        if (got == 0) continue;
        found = true;
        break;
    }
    if (!found) return kStatusNoSample;
    if (idx_out)
        for (int i = 0; i < 5; ++i) idx_out[i] = idx[i];
    for (int e = g.sub; e < 20; e += G) {
        const int c = e / 5, i = e - 5 * (e / 5);
        int id = idx[0];
#pragma unroll
        for (int k = 1; k < 5; ++k) id = i == k ? idx[k] : id;
        S.pt[c][i] = pts4[4 * (int64_t)id + c];
    }
    ew_sync();
    return ew_solve5(S, g, E);
}

// ---- split path: the matrix phases per 16-lane group, the root finder on fewer lanes -------------
// With many hypotheses in flight the root finder (~400 Illinois steps on the critical path of
// one solve, a few active lanes per 16-lane group) dominates; the split path runs it on a small
// lane group per hypothesis (ew_group_roots, below; the default) or on one lane (ew_lane_roots),
// with the matrix phases' results (EStage) handed over through HBM.

// Matrix phases of hypothesis `hyp` -> EStage (lanes of the group share the writes).
template <int G>
__device__ __forceinline__ void ew_stage_hypothesis(EWave& S, const EGroup<G>& g, const double* pts4, int N,
                                                    const Sampler& smp, uint64_t hyp, EStage* out) {
    SubsetSrc<5> src(smp, hyp);
    int idx[5];
    int status = kStatusNoSample;
    bool found = false;   // search and solve apart (h_hypothesis): one solve pass per wave
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        const int got = src.next(N, idx);
        if (got < 0) break;
        if (got == 0) continue;
        found = true;
        break;
    }
    if (found) {
        for (int e = g.sub; e < 20; e += G) {
            const int c = e / 5, i = e - 5 * (e / 5);
            int id = idx[0];
#pragma unroll
            for (int k = 1; k < 5; ++k) id = i == k ? idx[k] : id;
            S.pt[c][i] = pts4[4 * (int64_t)id + c];
        }
        ew_sync();
        status = 0;
        if (ew_null_basis(S, g)) {
            ew_coeffs(S, g);
            if (ew_eliminate(S, g)) status = 1;
        }
    }
    if (status == 1) {
        for (int e = g.sub; e < 36; e += G) out->nb[e / 9][e - 9 * (e / 9)] = S.nb[e / 9][e - 9 * (e / 9)];
        if (g.sub == 0) {
            double bx[3][4], by[3][4], bc[3][5], det[11];
            e_bz(&S.A[0][10], 20, bx, by, bc);
            e_detpoly(bx, by, bc, det);
#pragma unroll
            for (int i = 0; i < 3; ++i) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    out->bx[i][k] = bx[i][k];
                    out->by[i][k] = by[i][k];
                }
#pragma unroll
                for (int k = 0; k < 5; ++k) out->bc[i][k] = bc[i][k];
            }
#pragma unroll
            for (int k = 0; k < 11; ++k) out->det[k] = det[k];
        }
    }
    if (g.sub == 0) out->status = status;
}

// One level of e_poly_real_roots for this lane, degree D: roots of the previous level in rp,
// new ones to rc (LDS columns [k][lane]).
template <int D>
__device__ __forceinline__ int ew_lane_level(const double (*Lc)[64], const double (*rp)[64], double (*rc)[64],
                                             int lane, int j, int np, double R) {
    EPolyD<D> P;
#pragma unroll
    for (int k = 0; k <= D; ++k) P.q[k] = Lc[k + j][lane] * e_falling(k + j, j);
    int nc = 0;
    double a = -R;
    double fa = P(a);
    for (int s = 0; s <= np; ++s) {
        const double b = s < np ? rp[s][lane] : R;
        const double fb = P(b);
        if (fb == 0) {
            if (nc == 0 || rc[nc - 1][lane] != b) rc[nc++][lane] = b;
        } else if (fa != 0 && ((fa < 0) != (fb < 0))) {
            rc[nc++][lane] = e_root_bracketed_f(P, a, b, fa, fb);
        }
        a = b;
        fa = fb;
    }
    return nc;
}

// e_poly_real_roots of cin (degree <= 10) for this lane; the roots end in L[*which][k][lane].
// (A flattened one-evaluation-per-trip state machine, which keeps lanes in different intervals
// in step, measured slower on gfx950: ~300 instructions per trip against the loop's ~160.)
__device__ __forceinline__ int ew_lane_roots(const double* cin, double (*Lc)[64], double (*L)[10][64], int lane,
                                             int* which) {
    *which = 0;
    int n = 10;
    while (n > 0 && cin[n] == 0) --n;
    if (n < 1) return 0;
    const double lead = cin[n];
    for (int k = 0; k <= n; ++k) Lc[k][lane] = cin[k] / lead;
    double R = 0;
    for (int k = 0; k < n; ++k) {
        const double a = fabs(Lc[k][lane]);
        R = a > R ? a : R;
    }
    R = 1.0 + R;
    if (!isfinite(R)) return 0;
    int np = 0, cur = 0;
    for (int j = n - 1; j >= 0; --j) {
        const double (*rp)[64] = L[cur];
        double (*rc)[64] = L[cur ^ 1];
        switch (n - j) {
            case 1: np = ew_lane_level<1>(Lc, rp, rc, lane, j, np, R); break;
            case 2: np = ew_lane_level<2>(Lc, rp, rc, lane, j, np, R); break;
            case 3: np = ew_lane_level<3>(Lc, rp, rc, lane, j, np, R); break;
            case 4: np = ew_lane_level<4>(Lc, rp, rc, lane, j, np, R); break;
            case 5: np = ew_lane_level<5>(Lc, rp, rc, lane, j, np, R); break;
            case 6: np = ew_lane_level<6>(Lc, rp, rc, lane, j, np, R); break;
            case 7: np = ew_lane_level<7>(Lc, rp, rc, lane, j, np, R); break;
            case 8: np = ew_lane_level<8>(Lc, rp, rc, lane, j, np, R); break;
            case 9: np = ew_lane_level<9>(Lc, rp, rc, lane, j, np, R); break;
            default: np = ew_lane_level<10>(Lc, rp, rc, lane, j, np, R); break;
        }
        cur ^= 1;
    }
    *which = cur;
    return np;
}


// ---- split path, root finder over a small lane group (GR = 4 or 8 lanes per hypothesis) ----------
// One hypothesis per GR lanes: each level's intervals are dealt round-robin to the group's lanes
// (lane sub brackets s = sub, sub + GR, ...), so a level costs the longest per-lane sum of
// Illinois runs rather than the sum over all intervals, and 64 / GR hypotheses share a wave. The
// kept-root list is rebuilt by the group's first lane in interval order (the serial rule).
struct ERootLds {
    double c[11];
    double rp[10];
    double val[11], b[11];
    int type[11];
    int np;
};

template <int D, int GR>
__device__ __forceinline__ int ew_group_level(ERootLds& S, int sub, int j, int np, double R) {
    EPolyD<D> P;
#pragma unroll
    for (int k = 0; k <= D; ++k) P.q[k] = S.c[k + j] * e_falling(k + j, j);
    for (int s = sub; s <= np; s += GR) {
        const double a = s == 0 ? -R : S.rp[s - 1];
        const double b = s < np ? S.rp[s] : R;
        const double fa = P(a), fb = P(b);
        int type = 0;
        double val = 0.0;
        if (fb == 0) {
            type = 1;
            val = b;
        } else if (fa != 0 && ((fa < 0) != (fb < 0))) {
            type = 2;
            val = e_root_bracketed_f(P, a, b, fa, fb);
        }
        S.type[s] = type;
        S.val[s] = val;
        S.b[s] = b;
    }
    ew_sync();
    if (sub == 0) {
        int nc = 0;
        for (int s = 0; s <= np; ++s) {
            const int t = S.type[s];
            if (t == 1) {
                if (nc == 0 || S.rp[nc - 1] != S.b[s]) S.rp[nc++] = S.b[s];
            } else if (t == 2) {
                S.rp[nc++] = S.val[s];
            }
        }
        S.np = nc;
    }
    ew_sync();
    return S.np;
}

// e_poly_real_roots of cin for one group; the roots end in S.rp (count returned).
template <int GR>
__device__ __forceinline__ int ew_group_roots(ERootLds& S, const double* cin, int sub) {
    int n = 10;
    while (n > 0 && cin[n] == 0) --n;
    if (n < 1) return 0;
    const double lead = cin[n];
    for (int k = sub; k <= n; k += GR) S.c[k] = cin[k] / lead;
    ew_sync();
    double R = 0;
    for (int k = 0; k < n; ++k) {
        const double a = fabs(S.c[k]);
        R = a > R ? a : R;
    }
    R = 1.0 + R;
    if (!isfinite(R)) return 0;
    int np = 0;
    for (int j = n - 1; j >= 0; --j) {
        switch (n - j) {
            case 1: np = ew_group_level<1, GR>(S, sub, j, np, R); break;
            case 2: np = ew_group_level<2, GR>(S, sub, j, np, R); break;
            case 3: np = ew_group_level<3, GR>(S, sub, j, np, R); break;
            case 4: np = ew_group_level<4, GR>(S, sub, j, np, R); break;
            case 5: np = ew_group_level<5, GR>(S, sub, j, np, R); break;
            case 6: np = ew_group_level<6, GR>(S, sub, j, np, R); break;
            case 7: np = ew_group_level<7, GR>(S, sub, j, np, R); break;
            case 8: np = ew_group_level<8, GR>(S, sub, j, np, R); break;
            case 9: np = ew_group_level<9, GR>(S, sub, j, np, R); break;
            default: np = ew_group_level<10, GR>(S, sub, j, np, R); break;
        }
    }
    return np;
}

}  // namespace mcv
