// Micro-benchmark of the L2 split prep's shape (cfg5 8-rank share: 6250 queries + 50000 train rows of
// 128 floats): hi / lo f16 split + norms, with and without the per-block atomic maxima.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

template <int MODE, int STRIDE = 1>   // 0: float4 per lane, no atomics; 1: + per-block atomicMax into 16 slots
                                      // STRIDE words apart; 2: row per wave scalar
__global__ __launch_bounds__(256) void prep(const float* src, int nrows, _Float16* hi, _Float16* lo, float* norms,
                                            unsigned* slot) {
    __shared__ unsigned red[4];
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    unsigned m = 0;
    if (MODE == 2) {
        for (int r = wave; r < nrows; r += nw) {
            float acc = 0.f;
            for (int k = lane; k < 128; k += 64) {
                const float v = src[(size_t)r * 128 + k];
                const _Float16 h = (_Float16)v;
                hi[(size_t)r * 128 + k] = h;
                lo[(size_t)r * 128 + k] = (_Float16)(v - (float)h);
                acc = fmaf(v, v, acc);
                m = max(m, __float_as_uint(fabsf(v)));
            }
            for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
            if (lane == 0) norms[r] = acc;
        }
    } else {
        const int sub = lane >> 5, c = lane & 31;
        for (int r0 = wave * 2; r0 < nrows; r0 += nw * 2) {
            const int r = r0 + sub;
            const float4 v = reinterpret_cast<const float4*>(src + (size_t)r * 128)[c];
            const float x[4] = {v.x, v.y, v.z, v.w};
            _Float16 hx[4], lx[4];
            float acc = 0.f;
            for (int e = 0; e < 4; ++e) {
                hx[e] = (_Float16)x[e];
                lx[e] = (_Float16)(x[e] - (float)hx[e]);
                acc = fmaf(x[e], x[e], acc);
                m = max(m, __float_as_uint(fabsf(x[e])));
            }
            for (int off = 16; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
            *reinterpret_cast<f16x4*>(hi + (size_t)r * 128 + 4 * c) = f16x4{hx[0], hx[1], hx[2], hx[3]};
            *reinterpret_cast<f16x4*>(lo + (size_t)r * 128 + 4 * c) = f16x4{lx[0], lx[1], lx[2], lx[3]};
            if (c == 0) norms[r] = acc;
        }
    }
    for (int off = 32; off >= 1; off >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, off, 64));
    if (lane == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned r = max(max(red[0], red[1]), max(red[2], red[3]));
        if (MODE == 1) atomicMax(slot + (blockIdx.x % 16) * STRIDE, r);
        else slot[16 * 4096 + blockIdx.x] = r;
    }
}

int main() {
    const int rows = 56250;
    float* src; _Float16 *hi, *lo; float* nrm; unsigned* slot;
    hipMalloc(&src, (size_t)rows * 128 * 4);
    hipMalloc(&hi, (size_t)rows * 128 * 2);
    hipMalloc(&lo, (size_t)rows * 128 * 2);
    hipMalloc(&nrm, rows * 4);
    hipMalloc(&slot, (16 * 4096 + 65536) * 4);
    std::vector<float> h((size_t)rows * 128);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) * 0.25f;
    hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, auto kern, int blocks) {
        for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, src, rows, hi, lo, nrm, slot);
        hipEventRecord(a);
        for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, src, rows, hi, lo, nrm, slot);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        printf("%-28s blocks %6d: %7.2f us\n", name, blocks, ms * 1e3 / 50);
    };
    for (int blocks : {256, 1024, 3516, 7032, 14063}) {
        run("vec, no atomics", prep<0>, blocks);
        run("vec, atomic slots", prep<1>, blocks);
    }
    for (int blocks : {3516, 14063}) run("row per wave (scalar)", prep<2>, blocks);
    for (int blocks : {1024, 3516}) {
        run("atomic slots stride 64", prep<1, 64>, blocks);
        run("atomic slots stride 1024", prep<1, 1024>, blocks);
        run("atomic slots stride 4096", prep<1, 4096>, blocks);
    }
    return 0;
}
