// matchers_host.cpp — host-pointer exports of the brute-force matchers (new exports, same
// conventions as the reference: caller-allocated outputs, int return, failure = -1 + message).
//
// Query sharding inside one call: cvMatchHammingMulti / cvMatchL2Multi split
// the queries into D contiguous blocks (the cut of minicv_amd/dist.py's shard(): the first nq % D
// blocks one query longer), block k on device (home + k) mod visible devices, home = the calling
// thread's device. The train set is uploaded once to the home device and replicated to every other
// device by one peer copy over xGMI; each block's queries go straight from the caller's array to its
// device and its outputs straight back into the caller's arrays at the block's offset. Queries are
// independent, so the answer is the one-device answer bit for bit. Blocks that land on one device (a
// one-GPU box) share the home train copy and take turns on that device's matcher workspace
// (StreamFence). The single-device exports are D = 1. The host-side caller is one synchronous
// P/Invoke per call, as the reference's (OpenCV.fs:339-382).
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "kernels.h"
#include <algorithm>
#include <type_traits>
#include <cstring>
#include <climits>

using namespace mcv;

namespace {
constexpr int kMaxMatchShards = 16;

struct MatchWork {
    DevBuf<uint8_t> q, t;
    DevBuf<int> idx, idx2, di, di2;
    DevBuf<float> df, df2;
    hipStream_t s = nullptr;
    hipEvent_t ev = nullptr;   // home shard: its train upload finished (the peer copies wait on it)
    int dev = -1;
    // buffers, stream and event belong to one device: a shard slot that moves to another device
    // (the calling thread switched devices) starts over
    void bind(int d) {
        if (dev == d) return;
        release();
        dev = d;
    }
    hipStream_t stream() {
        if (!s) MCV_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        return s;
    }
    hipEvent_t event() {
        if (!ev) MCV_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        return ev;
    }
    void release() {
        q.reset(); t.reset();
        idx.reset(); idx2.reset(); di.reset(); di2.reset(); df.reset(); df2.reset();
        if (s) (void)hipStreamDestroy(s);
        if (ev) (void)hipEventDestroy(ev);
        s = nullptr;
        ev = nullptr;
    }
    ~MatchWork() { release(); }
};
MatchWork& work(int k) {
    thread_local MatchWork w[kMaxMatchShards];
    return w[k];
}

// One matcher call over D query blocks. Elem: the descriptor element type; Dist: the distance type
// (int for Hamming, float for L2); launch(shard work, d_q, nq, d_t, d_idx, d_dist, d_idx2, d_dist2, s).
template <class Dist, class Launch>
int match_sharded(const char* name, const void* q, int nq, const void* t, int nt, size_t rowBytes, int deviceCount,
                  int* idx, Dist* dist, int* idx2, Dist* dist2, Launch&& launch) {
    if (deviceCount < 1 || deviceCount > kMaxMatchShards)
        fail("%s: deviceCount %d outside [1, %d]", name, deviceCount, kMaxMatchShards);
    if (nq == 0) return 0;
    require_device();
    int ndev = 1, home = 0;
    MCV_HIP(hipGetDeviceCount(&ndev));
    MCV_HIP(hipGetDevice(&home));
    struct DeviceRestore {
        int dev;
        ~DeviceRestore() { (void)hipSetDevice(dev); }
    } restore{home};
    const int D = std::min(deviceCount, nq);
    const size_t tb = (size_t)nt * rowBytes;
    // home shard: the train set once from the host
    MatchWork& w0 = work(0);
    w0.bind(home);
    hipStream_t s0 = w0.stream();
    w0.t.ensure(tb ? tb : 1);
    if (tb) MCV_HIP(hipMemcpyAsync(w0.t.p, t, tb, hipMemcpyHostToDevice, s0));
    if (D > 1) MCV_HIP(hipEventRecord(w0.event(), s0));
    const int base = nq / D, rem = nq % D;
    for (int k = 0; k < D; ++k) {
        const int b = k * base + std::min(k, rem), c = base + (k < rem ? 1 : 0);
        const int dev = (home + k) % ndev;
        MCV_HIP(hipSetDevice(dev));
        MatchWork& w = work(k);
        w.bind(dev);
        hipStream_t s = w.stream();
        const uint8_t* d_t = w0.t.p;
        if (k > 0) {
            MCV_HIP(hipStreamWaitEvent(s, w0.event(), 0));   // the home copy of the train set is complete
            if (dev != home) {   // replicate it to this device (xGMI peer copy)
                w.t.ensure(tb ? tb : 1);
                if (tb) MCV_HIP(hipMemcpyPeerAsync(w.t.p, dev, w0.t.p, home, tb, s));
                d_t = w.t.p;
            }
        }
        const size_t qb = (size_t)c * rowBytes;
        w.q.ensure(qb);
        w.idx.ensure(c); w.idx2.ensure(c);
        MCV_HIP(hipMemcpyAsync(w.q.p, (const uint8_t*)q + (size_t)b * rowBytes, qb, hipMemcpyHostToDevice, s));
        Dist* dd;
        Dist* dd2;
        if constexpr (sizeof(Dist) == sizeof(int) && !std::is_floating_point<Dist>::value) {
            w.di.ensure(c); w.di2.ensure(c);
            dd = w.di.p; dd2 = w.di2.p;
        } else {
            w.df.ensure(c); w.df2.ensure(c);
            dd = w.df.p; dd2 = w.df2.p;
        }
        launch(w.q.p, c, d_t, w.idx.p, dd, w.idx2.p, dd2, s);
        MCV_HIP(hipMemcpyAsync(idx + b, w.idx.p, c * sizeof(int), hipMemcpyDeviceToHost, s));
        MCV_HIP(hipMemcpyAsync(dist + b, dd, c * sizeof(Dist), hipMemcpyDeviceToHost, s));
        if (idx2) MCV_HIP(hipMemcpyAsync(idx2 + b, w.idx2.p, c * sizeof(int), hipMemcpyDeviceToHost, s));
        if (dist2) MCV_HIP(hipMemcpyAsync(dist2 + b, dd2, c * sizeof(Dist), hipMemcpyDeviceToHost, s));
    }
    for (int k = 0; k < D; ++k) {
        MCV_HIP(hipSetDevice(work(k).dev));
        MCV_HIP(hipStreamSynchronize(work(k).s));
    }
    return nq;
}
}  // namespace

extern "C" MCV_API int cvMatchHammingMulti(const uint8_t* q, const int nq, const uint8_t* t, const int nt,
                                           const int bytesPerDesc, const int deviceCount, int* idx, int* dist,
                                           int* idx2, int* dist2) {
    MCV_GUARD(-1, {
        if (nq < 0 || nt < 0 || (nq > 0 && (!q || !idx || !dist)) || (nt > 0 && !t))
            fail("cvMatchHamming: bad argument");
        if (bytesPerDesc < 1 || bytesPerDesc > 64) fail("cvMatchHamming: bytesPerDesc %d outside [1, 64]", bytesPerDesc);
        return match_sharded<int>("cvMatchHamming", q, nq, t, nt, (size_t)bytesPerDesc, deviceCount, idx, dist, idx2,
                                  dist2, [&](const uint8_t* dq, int c, const uint8_t* dt, int* i1, int* d1, int* i2,
                                             int* d2, hipStream_t s) {
                                      launch_match_hamming(dq, c, dt, nt, bytesPerDesc, i1, d1, i2, d2, s);
                                  });
    })
}

extern "C" MCV_API int cvMatchHamming(const uint8_t* q, const int nq, const uint8_t* t, const int nt,
                                      const int bytesPerDesc, int* idx, int* dist, int* idx2, int* dist2) {
    return cvMatchHammingMulti(q, nq, t, nt, bytesPerDesc, 1, idx, dist, idx2, dist2);
}

extern "C" MCV_API int cvMatchL2Multi(const float* q, const int nq, const float* t, const int nt, const int dim,
                                      const int deviceCount, int* idx, float* dist, int* idx2, float* dist2) {
    MCV_GUARD(-1, {
        if (nq < 0 || nt < 0 || dim <= 0 || (nq > 0 && (!q || !idx || !dist)) || (nt > 0 && !t))
            fail("cvMatchL2: bad argument");
        return match_sharded<float>("cvMatchL2", q, nq, t, nt, (size_t)dim * sizeof(float), deviceCount, idx, dist,
                                    idx2, dist2, [&](const uint8_t* dq, int c, const uint8_t* dt, int* i1, float* d1,
                                                     int* i2, float* d2, hipStream_t s) {
                                        launch_match_l2((const float*)dq, c, (const float*)dt, nt, dim, i1, d1, i2, d2,
                                                        s);
                                    });
    })
}

extern "C" MCV_API int cvMatchL2(const float* q, const int nq, const float* t, const int nt, const int dim, int* idx,
                                 float* dist, int* idx2, float* dist2) {
    return cvMatchL2Multi(q, nq, t, nt, dim, 1, idx, dist, idx2, dist2);
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
