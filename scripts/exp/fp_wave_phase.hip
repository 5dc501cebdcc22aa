// Experiment (not product): per-phase cycle counts of the wave-cooperative five-point solve
// (five_point_wave.h), and whole-kernel time for 1 / 1024 / 65536 hypotheses.
#include "five_point_wave.h"
#include <cstdio>
#include <random>
#include <vector>
using namespace mcv;

__global__ __launch_bounds__(64) void phases(const double* P, int n, long long* T, int* out) {
    __shared__ EWave S;
    const EGroup<64> g(threadIdx.x);
    const int h = blockIdx.x;
    if (h >= n) return;
    long long t[8];
    int nr = -1;
    t[0] = clock64();
    ew_stage(S, g, P + 20 * h, P + 20 * h + 5, P + 20 * h + 10, P + 20 * h + 15);
    bool ok = ew_null_basis(S, g);
    t[1] = clock64();
    if (ok) ew_coeffs(S, g);
    t[2] = clock64();
    if (ok) ok = ew_eliminate(S, g);
    t[3] = clock64();
    double bx[3][4], by[3][4], bc[3][5], det[11];
    if (ok) {
        e_bz(&S.A[0][10], 20, bx, by, bc);
        e_detpoly(bx, by, bc, det);
        if (g.sub == 0)
            for (int k = 0; k < 11; ++k) S.det[k] = det[k];
        ew_sync();
    }
    t[4] = clock64();
    if (ok) nr = ew_real_roots(S, g);
    t[5] = clock64();
    double E[9];
    bool m = false;
    if (ok && g.sub < nr) m = e_model_at(bx, by, bc, S.nb[0], S.nb[1], S.nb[2], S.nb[3], S.rp[g.sub], E);
    const int cnt = __popcll(__ballot(m));
    t[6] = clock64();
    if (g.sub == 0) {
        out[h] = cnt;
        for (int k = 0; k < 6; ++k) T[6 * h + k] = t[k + 1] - t[k];
    }
}

template <int G>
__global__ __launch_bounds__(64) void full(const double* P, int n, int* out) {
    __shared__ EWave S[64 / G];
    const EGroup<G> g(threadIdx.x);
    const int h = blockIdx.x * (64 / G) + g.base / G;
    if (h >= n) return;
    EWave& W = S[g.base / G];
    ew_stage(W, g, P + 20 * h, P + 20 * h + 5, P + 20 * h + 10, P + 20 * h + 15);
    double E[9];
    const int c = ew_solve5(W, g, E);
    if (g.sub == 0) out[h] = c;
}

template <int G>
void run_full(const double* d, int* o, int cnt) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a); (void)hipEventCreate(&b);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(full<G>, dim3((cnt + 64 / G - 1) / (64 / G)), dim3(64), 0, 0, d, cnt, o);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    printf("full solve G=%2d, %6d hypotheses: %.3f ms\n", G, cnt, ms);
}

int main() {
    const int n = 65536;
    std::vector<double> h(20 * n);
    std::mt19937_64 g(1);
    std::normal_distribution<double> nd;
    for (auto& v : h) v = 0.3 * nd(g);
    double* d; int* o; long long* T;
    (void)hipMalloc(&d, h.size() * 8); (void)hipMalloc(&o, n * 4); (void)hipMalloc(&T, 6 * 64 * 8);
    (void)hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(phases, dim3(64), dim3(64), 0, 0, d, 64, T, o);
    (void)hipDeviceSynchronize();
    std::vector<long long> th(6 * 64);
    std::vector<int> oh(64);
    (void)hipMemcpy(th.data(), T, th.size() * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(oh.data(), o, 64 * 4, hipMemcpyDeviceToHost);
    double s[6] = {0};
    for (int i = 0; i < 64; ++i)
        for (int k = 0; k < 6; ++k) s[k] += th[6 * i + k] / 64.0;
    printf("cycles/phase (mean of 64 waves, 1 wave per CU): null %.0f coeffs %.0f elim %.0f det %.0f roots %.0f models %.0f\n",
           s[0], s[1], s[2], s[3], s[4], s[5]);
    for (int i = 0; i < 4; ++i)
        printf("  wave %d: %lld %lld %lld %lld %lld %lld models %d\n", i, th[6 * i], th[6 * i + 1], th[6 * i + 2],
               th[6 * i + 3], th[6 * i + 4], th[6 * i + 5], oh[i]);
    std::vector<int> r64(n), r16(n);
    for (int cnt : {1, 1024, 8192, n}) {
        run_full<64>(d, o, cnt);
        if (cnt == n) (void)hipMemcpy(r64.data(), o, n * 4, hipMemcpyDeviceToHost);
        run_full<32>(d, o, cnt);
        run_full<16>(d, o, cnt);
        if (cnt == n) (void)hipMemcpy(r16.data(), o, n * 4, hipMemcpyDeviceToHost);
    }
    int diff = 0;
    for (int i = 0; i < n; ++i) diff += r64[i] != r16[i];
    printf("model-count mismatches G=64 vs G=16: %d\n", diff);
    return 0;
}
