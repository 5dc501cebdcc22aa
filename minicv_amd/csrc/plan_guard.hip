// plan_guard.hip — fingerprints of device point buffers for the plan's stale-buffer guards.
//
// The device API hands the library raw pointers: a caller may rewrite a point buffer in place (same
// pointer, same N) between mcvRansacEvaluate and mcvRansacFinalize, or between two evaluates of one
// CV-sampler search. The plan therefore keys what it caches on the buffer's content: the last chunk's
// models (finalize takes the winner from them) and OpenCV's subset table (built from the points'
// checkSubset) each carry the fingerprint of the points they came from (mcv_common.h fp_term), and
// a mismatch re-solves / rebuilds. One pass over 16-32 B per correspondence: a few microseconds.
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "mcv_common.h"
#include "kernels.h"

#include <algorithm>

namespace mcv {

__global__ __launch_bounds__(256) void mcv_fingerprint(const uint32_t* __restrict__ w, uint64_t n,
                                                       unsigned long long* __restrict__ out) {
    uint64_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) acc += fp_term(i, w[i]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor((unsigned long long)acc, o);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

void launch_fingerprint(const void* d_buf, size_t bytes, uint64_t* d_out, hipStream_t s) {
    MCV_HIP(hipMemsetAsync(d_out, 0, sizeof(uint64_t), s));
    const uint64_t n = bytes / 4;
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>(std::max<uint64_t>((n + 2047) / 2048, 1), 1024);
    mcv_fingerprint<<<(unsigned)blocks, 256, 0, s>>>((const uint32_t*)d_buf, n, (unsigned long long*)d_out);
}

uint64_t host_fingerprint(const void* h_buf, size_t bytes) {
    const uint32_t* w = (const uint32_t*)h_buf;
    uint64_t acc = 0;
    for (uint64_t i = 0, n = bytes / 4; i < n; ++i) acc += fp_term(i, w[i]);
    return acc;
}

}  // namespace mcv

// Test hooks: the fingerprint of a host buffer, and the device kernel's on a device buffer (d_out:
// one uint64; synchronous). The two must agree.
extern "C" MCV_API uint64_t mcvHostFingerprint(const void* buf, size_t bytes) { return mcv::host_fingerprint(buf, bytes); }

extern "C" MCV_API int mcvTestFingerprint(const void* d_buf, size_t bytes, uint64_t* d_out) {
    MCV_GUARD(0, {
        if (!d_buf || !d_out) mcv::fail("mcvTestFingerprint: null argument");
        mcv::launch_fingerprint(d_buf, bytes, d_out, nullptr);
        MCV_HIP(hipGetLastError());
        MCV_HIP(hipDeviceSynchronize());
        return 1;
    })
}
