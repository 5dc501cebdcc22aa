// san_driver.cpp — host-side AddressSanitizer / UBSan run (sanitizers on host code;
// GPU ASan is not available on this pool). Built by tests/test_sanitizers.py with
//   g++ -fsanitize=address,undefined -fno-sanitize-recover=all -ffp-contract=off
// together with the oracle's C sources, it drives
//   * the host-compiled copy of the per-hypothesis code the kernels run (hyp_*.h: sampler, subset
//     checks, minimal solvers) and checks it bit for bit against the oracle;
//   * the oracle entry points the tests use, on small inputs (RANSAC loops and replay, matchers,
//     findScaled),
// so out-of-bounds accesses, signed overflow or invalid shifts in either fail the run.
// Prints "san ok <checks>" on success, exits non-zero otherwise.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "hyp_essential.h"
#include "five_point_ref.h"
#include "hyp_fundamental.h"
#include "hyp_homography.h"
#include "hyp_pnp.h"
#include "hyp_scaled.h"
#include "sqpnp.h"

extern "C" {
int orc_h_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* H, float* hf, int* idx_out);
int orc_f_hypothesis(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F, int* idx_out);
int orc_e_hypothesis(const double* pts4, int N, uint64_t seed, int64_t hyp, double* E90, int* idx_out);
int orc_pnp_hypothesis(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R, double* t,
                       int* idx_out);
int orc_pnp_hypothesis_epnp(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R,
                            double* t, int* idx_out);
int orc_solve_pnp_ransac_k(const double* img, const double* world, int N, const double* K9, const double* dist4,
                           double thr, double conf, int maxIters, uint64_t seed, int flags, int kind, double* rvec,
                           double* tvec, uint8_t* mask, int64_t* bestOut, int nthreads);
int orc_solve_pnp(const double* img, const double* world, int N, const double* K9, const double* dist4, int kind,
                  double* rvec, double* tvec);
int orc_sqpnp_pose(const double* img, const double* world, int n, const double* cam8, double* rh9, double* t3);
int orc_e_solve5_ref(const double* x1, const double* y1, const double* x2, const double* y2, double* Eout);
void orc_set_fast_minimal(int v);
int orc_find_homography(const double* src, const double* dst, int N, double thr, double conf, int maxIters, int method,
                        uint64_t seed, int flags, double* H, uint8_t* mask, int64_t* bestHypOut, int nthreads);
int orc_find_fundamental(const double* a, const double* b, int N, double thr, double conf, int maxIters, int method,
                         uint64_t seed, int flags, int errorKind, double* F, uint8_t* mask, int64_t* bestHypOut,
                         int nthreads);
int orc_find_essential(const double* a, const double* b, int N, double focal, double ppx, double ppy, double thr,
                       double conf, int maxIters, uint64_t seed, int flags, double* E, uint8_t* mask,
                       int64_t* bestSlotOut, int nthreads);
int orc_solve_pnp_ransac(const double* img, const double* world, int N, const double* K9, const double* dist4,
                         double thr, double conf, int maxIters, uint64_t seed, int flags, double* rvec, double* tvec,
                         uint8_t* mask, int64_t* bestOut, int nthreads);
void orc_match_hamming(const uint8_t* q, int nq, const uint8_t* t, int nt, int bytes, int* idx, int* dist, int* idx2,
                       int* dist2, int nthreads);
void orc_match_l2(const float* q, int nq, const float* t, int nt, int dim, int* idx, double* dist, int* idx2,
                  double* dist2, int nthreads);
int orc_find_scaled(const double* cam14, const double* W, const double* O, int N, const double* R9, const double* T3,
                    double* scales, double* costs, unsigned char* used, double* cost, double* scale, int nthreads);
}

static int g_checks = 0;
static int g_fail = 0;

static void expect(bool ok, const char* what, long a, long b) {
    ++g_checks;
    if (!ok && g_fail++ < 10) std::fprintf(stderr, "mismatch: %s (%ld, %ld)\n", what, a, b);
}

template <class T>
static bool same_bits(const T* a, const T* b, int n) {
    return std::memcmp(a, b, sizeof(T) * (size_t)n) == 0;
}

int main() {
    std::mt19937_64 rng(20261016);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const int threads = 2;

    // ---- homography / fundamental hypotheses on float4 {x, y, x', y'}
    for (int N : {4, 5, 8, 9, 64, 301}) {
        std::vector<float> pts(4 * (size_t)N);
        for (auto& v : pts) v = (float)U(rng);
        for (int h = 0; h < 64; ++h) {
            double H1[9] = {0}, H2[9] = {0};
            mcv::HModelF m1;
            float hf2[8] = {0};
            std::memset(&m1, 0, sizeof(m1));
            int i1[4] = {-1, -1, -1, -1}, i2[4] = {-1, -1, -1, -1};
            mcv::EigWsLocal ws;
            const int s1 = mcv::h_hypothesis(pts.data(), N, mcv::Sampler{7, nullptr}, (uint64_t)h, H1, &m1, i1, ws);
            const int s2 = orc_h_hypothesis(pts.data(), N, 7, h, H2, hf2, i2);
            expect(s1 == s2, "h status", s1, s2);
            if (s1 == 1 && s2 == 1) {
                expect(same_bits(H1, H2, 9), "h model", h, N);
                expect(same_bits(m1.h, hf2, 8), "h fp32 model", h, N);
            }
            if (N >= 8) {
                double F1[9] = {0}, F2[9] = {0};
                int j1[8], j2[8];
                const int t1 = mcv::f_hypothesis(pts.data(), N, mcv::Sampler{9, nullptr}, (uint64_t)h, F1, j1, ws);
                const int t2 = orc_f_hypothesis(pts.data(), N, 9, h, F2, j2);
                expect(t1 == t2, "f status", t1, t2);
                if (t1 == 1 && t2 == 1) expect(same_bits(F1, F2, 9), "f model", h, N);
            }
        }
    }

    // ---- essential hypotheses on double4 normalised points (two-view geometry, some noise)
    for (int N : {5, 6, 50, 200}) {
        std::vector<double> pts(4 * (size_t)N);
        const double c = std::cos(0.2), s = std::sin(0.2);
        for (int i = 0; i < N; ++i) {
            const double X = U(rng), Y = U(rng), Z = 4.0 + U(rng);
            const double X2 = c * X + s * Z + 0.5, Z2 = -s * X + c * Z + 0.1;
            pts[4 * i] = X / Z;
            pts[4 * i + 1] = Y / Z;
            pts[4 * i + 2] = X2 / Z2 + (i % 3 == 0 ? 0.01 * U(rng) : 0.0);
            pts[4 * i + 3] = Y / Z2;
        }
        for (int h = 0; h < 24; ++h) {
            double E1[mcv::kEMaxModels][9], E2[mcv::kEMaxModels * 9];
            std::memset(E1, 0, sizeof(E1));
            std::memset(E2, 0, sizeof(E2));
            int i1[5], i2[5];
            orc_set_fast_minimal(1);   // e_hypothesis = the opt-in replacement solver
            const int n1 = mcv::e_hypothesis(pts.data(), N, mcv::Sampler{11, nullptr}, (uint64_t)h, E1, i1);
            const int n2 = orc_e_hypothesis(pts.data(), N, 11, h, E2, i2);
            orc_set_fast_minimal(0);
            expect(n1 == n2, "e count", n1, n2);
            if (n1 > 0 && n1 == n2) expect(same_bits(&E1[0][0], E2, 9 * n1), "e models", h, N);
            if (h < 6) {   // the cvFivePoint export path on the first five points
                double x1[5], y1[5], x2[5], y2[5];
                for (int i = 0; i < 5; ++i) {
                    x1[i] = pts[4 * i]; y1[i] = pts[4 * i + 1]; x2[i] = pts[4 * i + 2]; y2[i] = pts[4 * i + 3];
                }
                std::memset(E1, 0, sizeof(E1));
                std::memset(E2, 0, sizeof(E2));
                const int r1 = mcv::fpr_solve5(x1, y1, x2, y2, E1);
                const int r2 = orc_e_solve5_ref(x1, y1, x2, y2, E2);
                expect(r1 == r2, "e ref count", r1, r2);
                if (r1 > 0 && r1 == r2) expect(same_bits(&E1[0][0], E2, 9 * r1), "e ref models", h, N);
            }
        }
    }

    // ---- PnP hypotheses (AP3P) on packed PnpPoint
    {
        const int N = 120;
        std::vector<mcv::PnpPoint> pts(N);
        const double cam8[8] = {800, 820, 640, 360, -0.1, 0.02, 0.001, -0.002};
        mcv::PnpCamera cam{cam8[0], cam8[1], cam8[2], cam8[3], cam8[4], cam8[5], cam8[6], cam8[7]};
        for (int i = 0; i < N; ++i) {
            const double X = U(rng), Y = U(rng), Z = U(rng);
            const double x = (X + 0.1) / (Z + 6.0), y = (Y - 0.2) / (Z + 6.0);
            pts[i] = mcv::PnpPoint{(float)X, (float)Y, (float)Z, (float)(x * cam8[0] + cam8[2] + U(rng)),
                                   (float)(y * cam8[1] + cam8[3] + U(rng)), 0.f, 0.f, 0.f};
        }
        for (int h = 0; h < 48; ++h) {
            mcv::PnpPose p1;
            std::memset(&p1, 0, sizeof(p1));
            double R2[9] = {0}, t2[3] = {0};
            int i1[4], i2[4];
            const int s1 = mcv::pnp_hypothesis(pts.data(), N, cam, mcv::Sampler{5, nullptr}, (uint64_t)h, p1, i1);
            const int s2 = orc_pnp_hypothesis(reinterpret_cast<const float*>(pts.data()), N, cam8, 5, h, R2, t2, i2);
            expect(s1 == s2, "pnp status", s1, s2);
            if (s1 == 1 && s2 == 1) expect(same_bits(p1.R, R2, 9) && same_bits(p1.t, t2, 3), "pnp pose", h, N);
            // EPnP hypotheses (epnp.h: JacobiSVD, SVBkSb, Gauss-Newton); every 4th on a planar copy
            std::vector<mcv::PnpPoint> q = pts;
            if (h % 4 == 3)
                for (auto& p : q) p.Z = 0.f;
            mcv::PnpPose e1;
            std::memset(&e1, 0, sizeof(e1));
            double R3[9] = {0}, t3[3] = {0};
            int j1[5], j2[5];
            const int u1 = mcv::pnp_hypothesis_epnp(q.data(), N, cam, mcv::Sampler{6, nullptr}, (uint64_t)h, e1, j1);
            const int u2 = orc_pnp_hypothesis_epnp(reinterpret_cast<const float*>(q.data()), N, cam8, 6, h, R3, t3, j2);
            expect(u1 == u2, "epnp status", u1, u2);
            if (u1 == 1 && u2 == 1) expect(same_bits(e1.R, R3, 9) && same_bits(e1.t, t3, 3), "epnp pose", h, N);
        }
    }

    // ---- oracle entry points end to end (small sizes)
    {
        const int N = 300;
        std::vector<double> a(2 * N), b(2 * N), w3(3 * N);
        for (int i = 0; i < N; ++i) {
            a[2 * i] = U(rng);
            a[2 * i + 1] = U(rng);
            b[2 * i] = 1.02 * a[2 * i] + 0.05 * a[2 * i + 1] + 0.01 + (i % 2 ? 0.2 * U(rng) : 0.0);
            b[2 * i + 1] = -0.03 * a[2 * i] + 0.98 * a[2 * i + 1] - 0.02;
            w3[3 * i] = U(rng);
            w3[3 * i + 1] = U(rng);
            w3[3 * i + 2] = U(rng);
        }
        std::vector<uint8_t> mask(N);
        double M[9];
        int64_t best;
        int k = orc_find_homography(a.data(), b.data(), N, 5e-3, 0.995, 500, 8, 3, 0, M, mask.data(), &best, threads);
        expect(k >= 0, "find_homography", k, 0);
        k = orc_find_fundamental(a.data(), b.data(), N, 5e-3, 0.99, 300, 8, 4, 0, 0, M, mask.data(), &best, threads);
        expect(k >= 0, "find_fundamental", k, 0);
        k = orc_find_essential(a.data(), b.data(), N, 1.0, 0.0, 0.0, 5e-3, 0.999, 100, 0, 0, M, mask.data(), &best,
                               threads);
        expect(k >= 0, "find_essential", k, 0);
        const double K9[9] = {800, 0, 640, 0, 820, 360, 0, 0, 1}, d4[4] = {0, 0, 0, 0};
        std::vector<double> img(2 * N);
        for (int i = 0; i < N; ++i) {
            img[2 * i] = 640 + 80 * w3[3 * i] / (w3[3 * i + 2] + 5);
            img[2 * i + 1] = 360 + 80 * w3[3 * i + 1] / (w3[3 * i + 2] + 5);
        }
        double rv[3], tv[3];
        k = orc_solve_pnp_ransac(img.data(), w3.data(), N, K9, d4, 8.0, 0.99, 100, 1, 0, rv, tv, mask.data(), &best,
                                 threads);
        expect(k >= 0, "solve_pnp_ransac", k, 0);
        for (int kind : {0, 1}) {
            k = orc_solve_pnp_ransac_k(img.data(), w3.data(), N, K9, d4, 8.0, 0.99, 100, 1, 0, kind, rv, tv, mask.data(),
                                       &best, threads);
            expect(k >= 0, "solve_pnp_ransac_k", k, kind);
        }
        k = orc_solve_pnp(img.data(), w3.data(), N, K9, d4, 1, rv, tv);
        expect(k >= 0, "solve_pnp", k, 0);
        // SQPnP: sqpnp.h's host solve over the same sums (sequential: N <= 1024) equals oracle_sqpnp.c
        for (int n : {3, 4, 7, N}) {
            const double cam8[8] = {800, 820, 640, 360, 0, 0, 0, 0};
            double sums[mcv::kSqpSums] = {0};
            for (int i = 0; i < n; ++i) {
                mcv::PnpCamera pc;
                pc.fx = 800; pc.fy = 820; pc.cx = 640; pc.cy = 360; pc.k1 = pc.k2 = pc.p1 = pc.p2 = 0;
                double x, y;
                mcv::pnp_undistort(pc, img[2 * i], img[2 * i + 1], x, y);
                for (int a = 0; a < mcv::kSqpSums; ++a)
                    sums[a] += mcv::sqpnp_term(x, y, w3[3 * i], w3[3 * i + 1], w3[3 * i + 2], a);
            }
            auto npos = [&](const double* rh, const double* t) {
                int c = 0;
                for (int i = 0; i < n; ++i)
                    c += rh[6] * w3[3 * i] + rh[7] * w3[3 * i + 1] + rh[8] * w3[3 * i + 2] + t[2] > 0;
                return c;
            };
            double rh[9], t[3], ro[9], to[3];
            const int c1 = mcv::sqpnp_from_sums(sums, n, npos, rh, t);
            const int c2 = orc_sqpnp_pose(img.data(), w3.data(), n, cam8, ro, to);
            expect(c1 == c2, "sqpnp code", c1, c2);
            if (c1 > 0 && c1 == c2) expect(same_bits(rh, ro, 9) && same_bits(t, to, 3), "sqpnp pose", n, 0);
        }
        // matchers
        std::vector<uint8_t> qb(64 * 32), tb(80 * 32);
        for (auto& v : qb) v = (uint8_t)(rng() & 0xFF);
        for (auto& v : tb) v = (uint8_t)(rng() & 0xFF);
        std::vector<int> idx(64), dist(64), idx2(64), dist2(64);
        orc_match_hamming(qb.data(), 64, tb.data(), 80, 32, idx.data(), dist.data(), idx2.data(), dist2.data(), threads);
        expect(idx[0] >= 0 && idx[0] < 80, "match_hamming", idx[0], 80);
        std::vector<float> qf(64 * 128), tf(80 * 128);
        for (auto& v : qf) v = (float)U(rng);
        for (auto& v : tf) v = (float)U(rng);
        std::vector<double> df(64), df2(64);
        orc_match_l2(qf.data(), 64, tf.data(), 80, 128, idx.data(), df.data(), idx2.data(), df2.data(), threads);
        expect(idx[0] >= 0 && idx[0] < 80, "match_l2", idx[0], 80);
        // findScaled
        const double cam14[14] = {0, -10, 1, 0, 0.995037, -0.0995037, 0, 0.0995037, 0.995037, 1, 0, 0, 1, 1};
        const double R9[9] = {0.99, -0.14, 0.0, 0.14, 0.99, 0.0, 0.0, 0.0, 1.0}, T3[3] = {0.6, 0.1, -0.2};
        std::vector<double> sc(2 * N), co(2 * N);
        std::vector<unsigned char> used(N);
        double cost, scale;
        k = orc_find_scaled(cam14, w3.data(), a.data(), N, R9, T3, sc.data(), co.data(), used.data(), &cost, &scale,
                            threads);
        expect(k >= 0 && k <= 2 * N, "find_scaled", k, 2 * N);
    }

    if (g_fail) {
        std::fprintf(stderr, "san FAILED: %d of %d checks\n", g_fail, g_checks);
        return 1;
    }
    std::printf("san ok %d checks\n", g_checks);
    return 0;
}
