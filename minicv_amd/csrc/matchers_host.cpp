// matchers_host.cpp — host-pointer exports of the brute-force matchers (new exports, same
// conventions as the reference: caller-allocated outputs, int return, failure = -1 + message).
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include <cstring>
#include <climits>

using namespace mcv;

namespace {
struct MatchWork {
    DevBuf<uint8_t> q, t;
    DevBuf<int> idx, idx2, di, di2;
    DevBuf<float> df, df2;
    hipStream_t s = nullptr;
    hipStream_t stream() {
        if (!s) MCV_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        return s;
    }
    ~MatchWork() {
        if (s) (void)hipStreamDestroy(s);
    }
};
MatchWork& work() {
    thread_local MatchWork w;
    return w;
}
}  // namespace

extern "C" MCV_API int cvMatchHamming(const uint8_t* q, const int nq, const uint8_t* t, const int nt,
                                      const int bytesPerDesc, int* idx, int* dist, int* idx2, int* dist2) {
    MCV_GUARD(-1, {
        if (nq < 0 || nt < 0 || (nq > 0 && (!q || !idx || !dist)) || (nt > 0 && !t))
            fail("cvMatchHamming: bad argument");
        if (nq == 0) return 0;
        require_device();
        MatchWork& w = work();
        hipStream_t s = w.stream();
        const size_t qb = (size_t)nq * bytesPerDesc, tb = (size_t)nt * bytesPerDesc;
        w.q.ensure(qb);
        w.t.ensure(tb ? tb : 1);
        w.idx.ensure(nq); w.di.ensure(nq); w.idx2.ensure(nq); w.di2.ensure(nq);
        MCV_HIP(hipMemcpyAsync(w.q.p, q, qb, hipMemcpyHostToDevice, s));
        if (tb) MCV_HIP(hipMemcpyAsync(w.t.p, t, tb, hipMemcpyHostToDevice, s));
        launch_match_hamming(w.q.p, nq, w.t.p, nt, bytesPerDesc, w.idx.p, w.di.p, w.idx2.p, w.di2.p, s);
        MCV_HIP(hipMemcpyAsync(idx, w.idx.p, nq * sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipMemcpyAsync(dist, w.di.p, nq * sizeof(int), hipMemcpyDeviceToHost, s));
        if (idx2) MCV_HIP(hipMemcpyAsync(idx2, w.idx2.p, nq * sizeof(int), hipMemcpyDeviceToHost, s));
        if (dist2) MCV_HIP(hipMemcpyAsync(dist2, w.di2.p, nq * sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        return nq;
    })
}

extern "C" MCV_API int cvMatchL2(const float* q, const int nq, const float* t, const int nt, const int dim, int* idx,
                                 float* dist, int* idx2, float* dist2) {
    MCV_GUARD(-1, {
        if (nq < 0 || nt < 0 || dim <= 0 || (nq > 0 && (!q || !idx || !dist)) || (nt > 0 && !t))
            fail("cvMatchL2: bad argument");
        if (nq == 0) return 0;
        require_device();
        MatchWork& w = work();
        hipStream_t s = w.stream();
        const size_t qb = (size_t)nq * dim * sizeof(float), tb = (size_t)nt * dim * sizeof(float);
        w.q.ensure(qb);
        w.t.ensure(tb ? tb : 1);
        w.idx.ensure(nq); w.idx2.ensure(nq); w.df.ensure(nq); w.df2.ensure(nq);
        MCV_HIP(hipMemcpyAsync(w.q.p, q, qb, hipMemcpyHostToDevice, s));
        if (tb) MCV_HIP(hipMemcpyAsync(w.t.p, t, tb, hipMemcpyHostToDevice, s));
        launch_match_l2((const float*)w.q.p, nq, (const float*)w.t.p, nt, dim, w.idx.p, w.df.p, w.idx2.p, w.df2.p, s);
        MCV_HIP(hipMemcpyAsync(idx, w.idx.p, nq * sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipMemcpyAsync(dist, w.df.p, nq * sizeof(float), hipMemcpyDeviceToHost, s));
        if (idx2) MCV_HIP(hipMemcpyAsync(idx2, w.idx2.p, nq * sizeof(int), hipMemcpyDeviceToHost, s));
        if (dist2) MCV_HIP(hipMemcpyAsync(dist2, w.df2.p, nq * sizeof(float), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
        return nq;
    })
}

extern "C" MCV_API int mcvMatchHammingDeviceForm(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt,
                                                 int bytesPerDesc, int* d_idx, int* d_dist, int* d_idx2, int* d_dist2,
                                                 int form, void* stream) {
    MCV_GUARD(-1, {
        if (nq < 0 || nt < 0 || (nq > 0 && (!d_q || !d_idx || !d_dist))) fail("mcvMatchHammingDevice: bad argument");
        if (form != kHammingFormGemm && form != kHammingFormPopcount)
            fail("mcvMatchHammingDeviceForm: form %d is neither 0 (int8 GEMM) nor 1 (popcount)", form);
        return launch_match_hamming(d_q, nq, d_t, nt, bytesPerDesc, d_idx, d_dist, d_idx2, d_dist2,
                                    (hipStream_t)stream, form);
    })
}

extern "C" MCV_API int mcvMatchHammingDevice(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int bytesPerDesc,
                                             int* d_idx, int* d_dist, int* d_idx2, int* d_dist2, void* stream) {
    return mcvMatchHammingDeviceForm(d_q, nq, d_t, nt, bytesPerDesc, d_idx, d_dist, d_idx2, d_dist2,
                                     kHammingFormGemm, stream);
}

extern "C" MCV_API int mcvMatchL2Device(const float* d_q, int nq, const float* d_t, int nt, int dim, int* d_idx,
                                        float* d_dist, int* d_idx2, float* d_dist2, void* stream) {
    MCV_GUARD(-1, {
        if (nq < 0 || nt < 0 || dim <= 0 || (nq > 0 && (!d_q || !d_idx || !d_dist)))
            fail("mcvMatchL2Device: bad argument");
        return launch_match_l2(d_q, nq, d_t, nt, dim, d_idx, d_dist, d_idx2, d_dist2, (hipStream_t)stream);
    })
}

extern "C" MCV_API int mcvL2LastExactScans(void) {
    MCV_GUARD(-1, { return l2_last_exact_scans(); })
}

extern "C" MCV_API int mcvL2LastGemmForm(void) {
    MCV_GUARD(-1, { return l2_last_gemm_form(); })
}
