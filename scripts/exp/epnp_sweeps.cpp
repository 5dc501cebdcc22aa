// Sweep-count statistics of EPnP's 12 x 12 Jacobi SVD over bench-like 5-point hypotheses (host build of
// epnp.h): how many sweeps, how many rotating pairs per sweep, and the max over groups of 64 lanes.
#include "hyp_pnp.h"
#include <cstdio>
#include <random>
#include <vector>
#include <algorithm>
using namespace mcv;

static int sweeps_of(double (&A)[12][12], std::vector<long>& rotPerSweep) {
    double W[12];
    for (int i = 0; i < 12; ++i) { double sd = 0; for (int k = 0; k < 12; ++k) sd += A[i][k] * A[i][k]; W[i] = sd; }
    const double eps = kDblEpsilon * 10;
    int iter = 0;
    for (; iter < 30; ++iter) {
        int rot = 0;
        for (int i = 0; i < 11; ++i)
            for (int j = i + 1; j < 12; ++j) {
                double a = W[i], b = W[j], p = 0;
                for (int k = 0; k < 12; ++k) p += A[i][k] * A[j][k];
                if (std::fabs(p) <= eps * std::sqrt(a * b)) continue;
                p *= 2;
                const double beta = a - b, gamma = cv_hypot(p, beta);
                double c, s;
                if (beta < 0) { const double delta = (gamma - beta) * 0.5; s = std::sqrt(delta / gamma); c = p / (gamma * s * 2); }
                else { c = std::sqrt((gamma + beta) / (gamma * 2)); s = p / (gamma * c * 2); }
                a = b = 0;
                for (int k = 0; k < 12; ++k) {
                    const double t0 = c * A[i][k] + s * A[j][k], t1 = -s * A[i][k] + c * A[j][k];
                    A[i][k] = t0; A[j][k] = t1; a += t0 * t0; b += t1 * t1;
                }
                W[i] = a; W[j] = b; ++rot;
            }
        if ((int)rotPerSweep.size() <= iter) rotPerSweep.resize(iter + 1);
        rotPerSweep[iter] += rot;
        if (!rot) { ++iter; break; }
    }
    return iter;
}

int main() {
    std::mt19937_64 g(7);
    std::normal_distribution<double> nd;
    std::uniform_real_distribution<double> ud(-1, 1);
    const int N = 20000;
    std::vector<PnpPoint> pts(N);
    const double f = 800, cx = 640, cy = 360;
    for (int i = 0; i < N; ++i) {
        double X = ud(g) * 2, Y = ud(g) * 2, Z = 6 + ud(g) * 2;
        double u = f * X / Z + cx + nd(g) * 0.5, v = f * Y / Z + cy + nd(g) * 0.5;
        if (i % 2) { u = cx + ud(g) * 640; v = cy + ud(g) * 360; }
        pts[i] = PnpPoint{(float)X, (float)Y, (float)Z, (float)u, (float)v, 0, 0, 0};
    }
    PnpCamera c{};
    c.fx = f; c.fy = f; c.cx = cx; c.cy = cy;
    const int H = 1 << 16;
    std::vector<int> sw(H);
    std::vector<long> rot;
    std::uniform_int_distribution<int> pick(0, N - 1);
    for (int h = 0; h < H; ++h) {
        PnpPoint p5[5];
        for (int k = 0; k < 5; ++k) p5[k] = pts[pick(g)];
        double pw[5][3], us[5][2], al[5][4], mtm[kMtmSums];
        pnp_epnp5_points(c, p5, pw, us);
        EpnpCtrl C;
        epnp_small_mtm<5>(pw, us, EpnpCam{c.fx, c.fy, c.cx, c.cy}, C, al, mtm);
        double A[12][12];
        for (int a = 0; a < 12; ++a) for (int b = a; b < 12; ++b) A[a][b] = A[b][a] = mtm[mtm_index(a, b)];
        sw[h] = sweeps_of(A, rot);
    }
    std::vector<int> hist(31);
    double mean = 0, wmax = 0;
    for (int h = 0; h < H; ++h) { hist[sw[h]]++; mean += sw[h]; }
    for (int w = 0; w < H / 64; ++w) wmax += *std::max_element(sw.begin() + 64 * w, sw.begin() + 64 * w + 64);
    printf("mean sweeps %.3f, mean of per-64 max %.3f\n", mean / H, wmax / (H / 64));
    for (int s = 0; s <= 30; ++s) if (hist[s]) printf("sweeps %2d: %6d\n", s, hist[s]);
    for (size_t s = 0; s < rot.size(); ++s) printf("sweep %zu: rotating pairs per hyp %.2f of 66\n", s, rot[s] / (double)H);
}
