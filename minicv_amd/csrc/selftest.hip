// selftest.hip — device self-tests exported as test hooks (never on a product path).
//   mcvTestRcpExhaustive: counts, over every 32-bit pattern, where the reciprocals the inlier sweeps
//   use (rcp_newton: v_rcp_f32 + one FMA Newton step; rcp_exact) differ from the correctly rounded
//   IEEE quotient 1.f / w — the property that lets the host oracle reproduce them with a division.
#include "mcv_common.h"
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"

namespace mcv {

// mode 0: rcp_exact; 1 / 3: rcp_newton (everywhere / on its domain only); 2: rcp_newton with
// v_div_fixup_f32 (the special-value fixup alone does not repair denormal inputs); 4: raw v_rcp_f32
__device__ __forceinline__ float rcp_variant(float w, int mode) {
    if (mode == 0) return rcp_exact(w);
    if (mode == 5) return rcp_exact_bounded(w);
    if (mode == 1 || mode == 3) return rcp_newton(w);
    const float r = __builtin_amdgcn_rcpf(w);
    if (mode == 4) return r;
    const float e = __builtin_fmaf(-w, r, 1.0f);
    return __builtin_amdgcn_div_fixupf(__builtin_fmaf(e, r, r), w, 1.0f);
}

__global__ __launch_bounds__(256) void mcv_rcp_check(uint64_t begin, uint64_t count, int mode,
                                                     unsigned long long* mism, uint32_t* first) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += stride) {
        const uint32_t bits = (uint32_t)(begin + i);
        const float w = __uint_as_float(bits);
        if (mode == 3) {   // the sweep's domain: |w| in [2^-126, 2^126)
            const float aw = fabsf(w);
            if (!(aw >= 0x1p-126f && aw < 0x1p126f)) continue;
        }
        if (mode == 5 && fabsf(w) >= 0x1p126f) continue;   // rcp_exact_bounded's domain: |w| < 2^126, NaN
        const float a = rcp_variant(w, mode);
        const float b = 1.0f / w;
        const uint32_t ua = __float_as_uint(a), ub = __float_as_uint(b);
        const bool same = (ua == ub) || (a != a && b != b);
        if (!same) {
            ++local;
            const unsigned long long slot = atomicAdd(mism + 1, 1ull);
            if (slot < 16) first[slot] = bits;
        }
    }
    if (local) atomicAdd(mism, local);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// fp64 with a random sign and mantissa and a binary exponent uniform in [lo, hi] (normal range).
__device__ __forceinline__ double random_f64(uint64_t bits, uint64_t ebits, int lo, int hi) {
    const int e = lo + (int)(ebits % (uint64_t)(hi - lo + 1));
    return __longlong_as_double((long long)((bits & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(e + 1023) << 52)));
}

// Samples (n, d) with d in +-[2^-64, 2^64] and compares div_f64_refined against n / d.
//   mode 0: |n| in [2^-900, 2^699]      mode 1: n = 1 (the reciprocal)
//   mode 2: n = d * k, k a small integer (exact quotients)   mode 3: d at the domain ends
//   mode 4: sqrt_f64_1to2(x) against sqrt(x), x in [1, 2] (the pair records (x, 0))
//   mode 5: the same for x in [0.5, 1] (the cosines / sines of JacobiSVDImpl_'s rotation)
__global__ __launch_bounds__(256) void mcv_div_check(uint64_t seed, uint64_t count, int mode,
                                                     unsigned long long* mism, double* first) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < count; i += stride) {
        const uint64_t a = splitmix64(seed ^ (i * 4 + 0)), b = splitmix64(seed ^ (i * 4 + 1));
        const uint64_t c = splitmix64(seed ^ (i * 4 + 2)), g = splitmix64(seed ^ (i * 4 + 3));
        if (mode == 4 || mode == 5) {
            const double x = (g & 0xFFFF) == 0 ? (mode == 4 ? 2.0 : 1.0)
                                               : random_f64(a & 0x000FFFFFFFFFFFFFull, b, mode == 4 ? 0 : -1,
                                                            mode == 4 ? 0 : -1);
            const double r = sqrt_f64_1to2(x), ref = __builtin_sqrt(x);
            if (__double_as_longlong(r) != __double_as_longlong(ref)) {
                ++local;
                const unsigned long long slot = atomicAdd(mism + 1, 1ull);
                if (slot < 16) {
                    first[2 * slot] = x;
                    first[2 * slot + 1] = 0.0;
                }
            }
            continue;
        }
        double d = random_f64(a, b, -64, 63);
        if (mode == 3) d = (g & 1) ? random_f64(a, b, -64, -64) : random_f64(a, b, 63, 63);
        double n;
        if (mode == 1) n = 1.0;
        else if (mode == 2) n = d * (double)(int)(g % 2001 - 1000);
        else n = random_f64(c, g, -900, 699);
        const double q = div_f64_refined(n, d, rcp_f64_refined(d));
        const double ref = n / d;
        const bool same = __double_as_longlong(q) == __double_as_longlong(ref) || (q == 0.0 && ref == 0.0);
        if (!same) {
            ++local;
            const unsigned long long slot = atomicAdd(mism + 1, 1ull);
            if (slot < 16) {
                first[2 * slot] = n;
                first[2 * slot + 1] = d;
            }
        }
    }
    if (local) atomicAdd(mism, local);
}

}  // namespace mcv

using namespace mcv;

extern "C" MCV_API long long mcvTestRcpExhaustive(int mode, uint32_t* firstMismatches16) {
    MCV_GUARD(-1, {
        require_device();
        DevBuf<unsigned long long> m;
        DevBuf<uint32_t> f;
        m.ensure(2);
        f.ensure(16);
        MCV_HIP(hipMemset(m.p, 0, 16));
        MCV_HIP(hipMemset(f.p, 0, 64));
        hipLaunchKernelGGL(mcv_rcp_check, dim3(8192), dim3(256), 0, 0, (uint64_t)0, (uint64_t)1 << 32, mode, m.p, f.p);
        MCV_HIP(hipGetLastError());
        unsigned long long h[2];
        MCV_HIP(hipMemcpy(h, m.p, 16, hipMemcpyDeviceToHost));
        if (firstMismatches16) MCV_HIP(hipMemcpy(firstMismatches16, f.p, 64, hipMemcpyDeviceToHost));
        return (long long)h[0];
    })
}

extern "C" MCV_API long long mcvTestDivF64(int mode, unsigned long long seed, long long count,
                                           double* firstMismatches32) {
    MCV_GUARD(-1, {
        require_device();
        if (count < 0) return -1LL;
        DevBuf<unsigned long long> m;
        DevBuf<double> f;
        m.ensure(2);
        f.ensure(32);
        MCV_HIP(hipMemset(m.p, 0, 16));
        MCV_HIP(hipMemset(f.p, 0, 256));
        hipLaunchKernelGGL(mcv_div_check, dim3(8192), dim3(256), 0, 0, (uint64_t)seed, (uint64_t)count, mode, m.p,
                           f.p);
        MCV_HIP(hipGetLastError());
        unsigned long long h[2];
        MCV_HIP(hipMemcpy(h, m.p, 16, hipMemcpyDeviceToHost));
        if (firstMismatches32) MCV_HIP(hipMemcpy(firstMismatches32, f.p, 256, hipMemcpyDeviceToHost));
        return (long long)h[0];
    })
}

// Run the homography inlier sweep on caller-supplied fp32 models (host arrays): exercises the
// rare exact-division paths of mcv_h_verify with crafted models (zero / denormal / huge
// denominators) that random hypotheses practically never produce. fused: 0 = op-by-op error,
// 1 = fused error (scalar sweep), 2 = fused error through the packed sweep mcv_h_verify_pk,
// 3 = op-by-op error through the certified sweep mcv_h_verify_cert (the default path).
extern "C" MCV_API int mcvTestHomographySweep(const float* pts4, int N, const float* models8, int nModels,
                                              float thr2, int fused, int* counts) {
    MCV_GUARD(0, {
        require_device();
        if (N <= 0 || nModels <= 0) fail("bad sizes");
        DevBuf<float> p, m, bb;
        DevBuf<int> c;
        p.ensure((size_t)N * 4);
        m.ensure((size_t)nModels * 8);
        c.ensure((size_t)nModels);
        bb.ensure(4);
        MCV_HIP(hipMemcpy(p.p, pts4, (size_t)N * 16, hipMemcpyHostToDevice));
        MCV_HIP(hipMemcpy(m.p, models8, (size_t)nModels * 32, hipMemcpyHostToDevice));
        MCV_HIP(hipMemset(c.p, 0, (size_t)nModels * 4));
        launch_bbox(p.p, N, bb.p, 0);
        if (fused == 3) {   // certified op-by-op sweep + exact recount of the slots it marks kStatusRedo
            DevBuf<float> pairs;
            DevBuf<double> b4;
            pairs.ensure((size_t)(N + 1) / 2 * 8);
            b4.ensure(4);
            launch_h_pair(p.p, N, pairs.p, 0);
            launch_abs_bound4(p.p, false, N, b4.p, nullptr, 0);
            launch_h_verify_certified(p.p, pairs.p, N, m.p, c.p, nModels, thr2, b4.p, 0);
            MCV_HIP(hipDeviceSynchronize());
        } else if (fused == 2) {   // packed sweep + exact recount of the slots it marks kStatusRedo
            DevBuf<float> pairs;
            pairs.ensure((size_t)(N + 1) / 2 * 8);
            launch_h_pair(p.p, N, pairs.p, 0);
            launch_h_verify_packed(p.p, pairs.p, N, m.p, c.p, nModels, thr2, bb.p, 0);
            MCV_HIP(hipDeviceSynchronize());
        } else {
            launch_h_verify(p.p, N, m.p, c.p, nModels, thr2, fused != 0, bb.p, 0);
        }
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipMemcpy(counts, c.p, (size_t)nModels * 4, hipMemcpyDeviceToHost));
        return 1;
    })
}
