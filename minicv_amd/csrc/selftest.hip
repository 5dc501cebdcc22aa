// selftest.hip — device self-tests exported as test hooks (never on a product path).
//   mcvTestRcpExhaustive: checks, over every 32-bit pattern, that the fused reciprocal used by the
//   inlier sweep (v_rcp_f32 + one FMA Newton step + v_div_fixup) equals the correctly rounded
//   IEEE quotient 1.f / w — the property that lets the host oracle reproduce it with a division.
#include "mcv_common.h"
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"

namespace mcv {

__device__ __forceinline__ float rcp_variant(float w, int mode) {
    if (mode == 0) return rcp_rn(w);
    if (mode == 3) return rcp_newton(w);
    const float r = __builtin_amdgcn_rcpf(w);
    if (mode == 2) return r;
    const float e = __builtin_fmaf(-w, r, 1.0f);
    return __builtin_fmaf(e, r, r);
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

// Run the homography inlier sweep on caller-supplied fp32 models (host arrays): exercises the
// rare exact-division paths of mcv_h_verify with crafted models (zero / denormal / huge
// denominators) that random hypotheses practically never produce. fused: 0 = op-by-op error,
// 1 = fused error (scalar sweep), 2 = fused error through the packed sweep mcv_h_verify_pk.
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
        if (fused == 2) {   // packed sweep + exact recount of the slots it marks kStatusRedo
            DevBuf<float> pairs;
            pairs.ensure((size_t)(N + 1) / 2 * 8);
            launch_h_pair(p.p, N, pairs.p, 0);
            if (!launch_h_verify_packed(p.p, pairs.p, N, m.p, c.p, nModels, thr2, bb.p, 0))
                fail("packed sweep disabled by MCV_SWEEP_VARIANT");
            MCV_HIP(hipDeviceSynchronize());
        } else {
            launch_h_verify(p.p, N, m.p, c.p, nModels, thr2, fused != 0, bb.p, 0);
        }
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipMemcpy(counts, c.p, (size_t)nModels * 4, hipMemcpyDeviceToHost));
        return 1;
    })
}
