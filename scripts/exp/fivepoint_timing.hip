// Experiment (not product): where does the five-point solve spend its time on gfx950?
#include "hyp_essential.h"
#include <cstdio>
#include <vector>
#include <random>
using namespace mcv;

__device__ int stage_solve(const double* p, double (*E)[9], int stage) {
    const double* x1 = p; const double* y1 = p + 5; const double* x2 = p + 10; const double* y2 = p + 15;
    double nb[4][9];
    if (!e_null_basis(x1, y1, x2, y2, nb)) return 0;
    if (stage == 0) return (int)(nb[0][0] * 1000);
    double C[10][10];
    {
        double A[10][20];
        e_coeffs(nb, A);
        if (stage == 1) return (int)(A[3][7] * 1000);
        if (!e_eliminate(A, C)) return 0;
    }
    if (stage == 2) return (int)(C[4][3] * 1000);
    return e_solve5(x1, y1, x2, y2, E);
}

__global__ void k(const double* P, int n, int stage, int* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double E[10][9];
    out[i] = stage_solve(P + 20 * i, E, stage);
}

int main() {
    const int n = 65536;
    std::vector<double> h(20 * n);
    std::mt19937_64 g(1); std::normal_distribution<double> nd;
    for (auto& v : h) v = 0.3 * nd(g);
    double* d; int* o;
    hipMalloc(&d, h.size() * 8); hipMalloc(&o, n * 4);
    hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int stage = 0; stage < 4; ++stage)
        for (int cnt : {1, 64, n}) {
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(a);
                hipLaunchKernelGGL(k, dim3((cnt + 63) / 64), dim3(64), 0, 0, d, cnt, stage, o);
                hipEventRecord(b); hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                if (rep == 2) printf("stage %d (0 null,1 coeffs,2 elim,3 full) count %6d: %.3f ms\n", stage, cnt, ms);
            }
        }
    return 0;
}
