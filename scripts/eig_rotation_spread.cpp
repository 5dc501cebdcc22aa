// Rotation-count spread of the restated JacobiImpl_ over H hypotheses (host twin), per 40-lane wave.
// g++ -O2 -std=c++17 -ffp-contract=off -Iminicv_amd/csrc -Iinclude scripts/eig_rotation_spread.cpp -o /tmp/spread
#include "mcv_common.h"
#include "jacobi_eig.h"
#include "hyp_homography.h"
#include <vector>
#include <random>
#include <algorithm>
#include <cstdio>
using namespace mcv;
struct CountWs {
    double d[kEigWs];
    long n = 0;
    double& operator[](int e) { if (e >= kEigW && e < kEigV) ++n; return d[e]; }
};
int main() {
    const int N = 100000;
    std::vector<float> pts(4 * (size_t)N);
    std::mt19937 g(7);
    std::uniform_real_distribution<float> u(0.f, 640.f), nz(-1.f, 1.f), o(0.f, 1.f);
    const double Ht[9] = {1.02, 0.03, 12.0, -0.02, 0.98, -7.0, 1e-5, -2e-5, 1.0};
    for (int i = 0; i < N; ++i) {
        float x = u(g), y = u(g);
        double w = Ht[6] * x + Ht[7] * y + Ht[8];
        float X = (float)((Ht[0] * x + Ht[1] * y + Ht[2]) / w), Y = (float)((Ht[3] * x + Ht[4] * y + Ht[5]) / w);
        if (o(g) < 0.3f) X = u(g), Y = u(g); else X += nz(g), Y += nz(g);
        pts[4 * i] = x; pts[4 * i + 1] = y; pts[4 * i + 2] = X; pts[4 * i + 3] = Y;
    }
    const int H = 40 * 2000;
    std::vector<int> it(H);
    long sum = 0;
    for (int h = 0; h < H; ++h) {
        CountWs ws;
        double Hm[9]; HModelF mf;
        h_hypothesis(pts.data(), N, 12345, (uint64_t)h, Hm, &mf, nullptr, ws);
        it[h] = ws.n > 18 ? (int)((ws.n - 18) / 4) : 0;
        sum += it[h];
    }
    long waveMax = 0;
    for (int w = 0; w < H / 40; ++w) waveMax += *std::max_element(it.begin() + 40 * w, it.begin() + 40 * w + 40);
    std::vector<int> s = it; std::sort(s.begin(), s.end());
    printf("hyps %d mean %.1f p10 %d p50 %d p90 %d max %d; mean per-wave max %.1f -> lane efficiency %.3f\n", H,
           (double)sum / H, s[H / 10], s[H / 2], s[9 * H / 10], s.back(), (double)waveMax / (H / 40),
           (double)sum / H / ((double)waveMax / (H / 40)));
}
