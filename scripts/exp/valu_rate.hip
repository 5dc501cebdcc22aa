// Micro-benchmark: issue cost of VALU instruction forms on gfx950, in shader cycles measured
// in-kernel (s_memtime). 8 waves per SIMD on every CU, 8 independent chains per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned long long u64;
#define CHAIN8(OP, C)                                 \
    asm volatile(OP : "+v"(a0) : C(s));               \
    asm volatile(OP : "+v"(a1) : C(s));               \
    asm volatile(OP : "+v"(a2) : C(s));               \
    asm volatile(OP : "+v"(a3) : C(s));               \
    asm volatile(OP : "+v"(a4) : C(s));               \
    asm volatile(OP : "+v"(a5) : C(s));               \
    asm volatile(OP : "+v"(a6) : C(s));               \
    asm volatile(OP : "+v"(a7) : C(s));

__global__ __launch_bounds__(256) void k0(u64* cyc, unsigned* out, int iters, unsigned s) {
    unsigned a0 = (unsigned)threadIdx.x, a1 = a0 + (unsigned)1, a2 = a0 + (unsigned)2, a3 = a0 + (unsigned)3, a4 = a0 + (unsigned)4, a5 = a0 + (unsigned)5, a6 = a0 + (unsigned)6, a7 = a0 + (unsigned)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_xor_b32 %0, %1, %0", "v") CHAIN8("v_xor_b32 %0, %1, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k1(u64* cyc, unsigned* out, int iters, unsigned s) {
    unsigned a0 = (unsigned)threadIdx.x, a1 = a0 + (unsigned)1, a2 = a0 + (unsigned)2, a3 = a0 + (unsigned)3, a4 = a0 + (unsigned)4, a5 = a0 + (unsigned)5, a6 = a0 + (unsigned)6, a7 = a0 + (unsigned)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_bcnt_u32_b32 %0, %1, %0", "v") CHAIN8("v_bcnt_u32_b32 %0, %1, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k2(u64* cyc, unsigned* out, int iters, unsigned s) {
    unsigned a0 = (unsigned)threadIdx.x, a1 = a0 + (unsigned)1, a2 = a0 + (unsigned)2, a3 = a0 + (unsigned)3, a4 = a0 + (unsigned)4, a5 = a0 + (unsigned)5, a6 = a0 + (unsigned)6, a7 = a0 + (unsigned)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_med3_u32 %0, %1, %0, %0", "v") CHAIN8("v_med3_u32 %0, %1, %0, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k3(u64* cyc, unsigned* out, int iters, unsigned s) {
    unsigned a0 = (unsigned)threadIdx.x, a1 = a0 + (unsigned)1, a2 = a0 + (unsigned)2, a3 = a0 + (unsigned)3, a4 = a0 + (unsigned)4, a5 = a0 + (unsigned)5, a6 = a0 + (unsigned)6, a7 = a0 + (unsigned)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_lshl_or_b32 %0, %0, 22, %1", "v") CHAIN8("v_lshl_or_b32 %0, %0, 22, %1", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k4(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_fmac_f32 %0, %1, %0", "s") CHAIN8("v_fmac_f32 %0, %1, %0", "s") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k5(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_fma_f32 %0, %1, %0, 1.0", "s") CHAIN8("v_fma_f32 %0, %1, %0, 1.0", "s") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k6(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_mul_f32 %0, %1, %0", "v") CHAIN8("v_mul_f32 %0, %1, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k7(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_rcp_f32 %0, %0", "v") CHAIN8("v_rcp_f32 %0, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k8(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_cmp_ge_f32_e32 vcc, %1, %0", "s") CHAIN8("v_cmp_ge_f32_e32 vcc, %1, %0", "s") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k9(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_cmp_ge_f32_e64 vcc, %1, %0", "s") CHAIN8("v_cmp_ge_f32_e64 s[20:21], %1, %0", "s") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k10(u64* cyc, unsigned* out, int iters, float s) {
    float a0 = (float)threadIdx.x, a1 = a0 + (float)1, a2 = a0 + (float)2, a3 = a0 + (float)3, a4 = a0 + (float)4, a5 = a0 + (float)5, a6 = a0 + (float)6, a7 = a0 + (float)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_cmp_class_f32_e32 vcc, %0, %1", "v") CHAIN8("v_cmp_class_f32_e32 vcc, %0, %1", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k11(u64* cyc, unsigned* out, int iters, double s) {
    double a0 = (double)threadIdx.x, a1 = a0 + (double)1, a2 = a0 + (double)2, a3 = a0 + (double)3, a4 = a0 + (double)4, a5 = a0 + (double)5, a6 = a0 + (double)6, a7 = a0 + (double)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_pk_fma_f32 %0, %1, %0, %1", "v") CHAIN8("v_pk_fma_f32 %0, %1, %0, %1", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k12(u64* cyc, unsigned* out, int iters, double s) {
    double a0 = (double)threadIdx.x, a1 = a0 + (double)1, a2 = a0 + (double)2, a3 = a0 + (double)3, a4 = a0 + (double)4, a5 = a0 + (double)5, a6 = a0 + (double)6, a7 = a0 + (double)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_pk_fma_f32 %0, %1, %0, %0 op_sel_hi:[0,1,1]", "s") CHAIN8("v_pk_fma_f32 %0, %1, %0, %0 op_sel_hi:[0,1,1]", "s") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k13(u64* cyc, unsigned* out, int iters, double s) {
    double a0 = (double)threadIdx.x, a1 = a0 + (double)1, a2 = a0 + (double)2, a3 = a0 + (double)3, a4 = a0 + (double)4, a5 = a0 + (double)5, a6 = a0 + (double)6, a7 = a0 + (double)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_pk_mul_f32 %0, %1, %0", "v") CHAIN8("v_pk_mul_f32 %0, %1, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k14(u64* cyc, unsigned* out, int iters, double s) {
    double a0 = (double)threadIdx.x, a1 = a0 + (double)1, a2 = a0 + (double)2, a3 = a0 + (double)3, a4 = a0 + (double)4, a5 = a0 + (double)5, a6 = a0 + (double)6, a7 = a0 + (double)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_fma_f64 %0, %1, %0, %1", "v") CHAIN8("v_fma_f64 %0, %1, %0, %1", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k15(u64* cyc, unsigned* out, int iters, double s) {
    double a0 = (double)threadIdx.x, a1 = a0 + (double)1, a2 = a0 + (double)2, a3 = a0 + (double)3, a4 = a0 + (double)4, a5 = a0 + (double)5, a6 = a0 + (double)6, a7 = a0 + (double)7;
    __syncthreads();
    const u64 t0 = __builtin_readcyclecounter();
    for (int i = 0; i < iters; ++i) { CHAIN8("v_mul_f64 %0, %1, %0", "v") CHAIN8("v_mul_f64 %0, %1, %0", "v") }
    const u64 t1 = __builtin_readcyclecounter();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    out[blockIdx.x * 256 + threadIdx.x] = (unsigned)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 8 waves per SIMD
    unsigned* out;
    u64* cyc;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&cyc, blocks * 8);
    u64* h = new u64[blocks];
    const int iters = 2000;
    auto report = [&](const char* name) {
        hipDeviceSynchronize();
        hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; ++i) s += (double)h[i];
        s /= blocks;  // mean wave duration in shader cycles (s_memtime)
        printf("%-24s %.2f cyc per wave-instr per SIMD\n", name, s / (8.0 * iters * 16));
    };
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k0, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (unsigned)5u);
    report("v_xor_b32 (VOP2)");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k1, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (unsigned)5u);
    report("v_bcnt_u32_b32");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k2, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (unsigned)5u);
    report("v_med3_u32");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k3, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (unsigned)5u);
    report("v_lshl_or_b32");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k4, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_fmac_f32 s (VOP2)");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k5, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_fma_f32 s (VOP3)");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k6, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_mul_f32 (VOP2)");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k7, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_rcp_f32");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k8, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_cmp_ge_f32_e32 vcc");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k9, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_cmp_ge_f32_e64 sgpr");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k10, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (float)1.0000001f);
    report("v_cmp_class_f32_e32");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k11, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (double)1.0000001);
    report("v_pk_fma_f32 vvv");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k12, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (double)1.0000001);
    report("v_pk_fma_f32 s-bcast");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k13, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (double)1.0000001);
    report("v_pk_mul_f32");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k14, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (double)1.0000001);
    report("v_fma_f64");
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k15, dim3(blocks), dim3(256), 0, 0, cyc, out, iters, (double)1.0000001);
    report("v_mul_f64");
    return 0;
}
