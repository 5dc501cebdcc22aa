// mcv_runtime.h — host runtime helpers for the C-ABI shim: per-thread last error, HIP error
// checking, device-buffer RAII. No exception crosses an extern "C" boundary: every export wraps
// its body in MCV_GUARD, which records the message and returns the export's failure value.
#pragma once

#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <cstdio>
#include <cstdarg>

namespace mcv {

struct Error : std::runtime_error {
    explicit Error(const std::string& m) : std::runtime_error(m) {}
};

void set_last_error(const char* msg);
void clear_last_error();

[[noreturn]] inline void fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    throw Error(buf);
}

#define MCV_HIP(call)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess) ::mcv::fail("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                                          __LINE__);                                                    \
    } while (0)

// Throws unless a HIP device is usable: the product path has no CPU fallback.
void require_device();

#define MCV_GUARD(failval, ...)                                                     \
    try {                                                                           \
        ::mcv::clear_last_error();                                                  \
        __VA_ARGS__                                                                 \
    } catch (const std::exception& ex) {                                            \
        ::mcv::set_last_error(ex.what());                                           \
        return failval;                                                             \
    } catch (...) {                                                                 \
        ::mcv::set_last_error("unknown exception");                                 \
        return failval;                                                             \
    }

// Device allocation that grows on demand (never shrinks) and is freed on destruction.
template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t count) {
        if (count <= n) return;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        MCV_HIP(hipMalloc((void**)&p, (count ? count : 1) * sizeof(T)));
        n = count;
    }
    void reset() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

template <class T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    void ensure(size_t count) {
        if (count <= n) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        MCV_HIP(hipHostMalloc((void**)&p, (count ? count : 1) * sizeof(T), hipHostMallocPortable));
        n = count;
    }
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
};

// Orders the uses of one per-thread workspace across streams: the device-level matchers are
// asynchronous on the caller's stream, so a call on stream B right after one on stream A would race on
// the shared buffers (and on their finish counters). enter(s) makes s wait for the previous use when
// that ran on another stream; leave(s) records this use's completion.
struct StreamFence {
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;
    bool used = false;
    // The null stream and the per-thread default stream live as long as the process; a caller's own
    // stream may be destroyed right after the call.
    static bool persistent(hipStream_t s) { return s == nullptr || s == hipStreamPerThread; }
    // A call on another stream than the previous one waits for the previous call's completion event.
    // A call on a caller-created stream records that event when it leaves (one reused event), so a
    // stream the caller destroys after the call is never touched again. A call on the null / per-thread
    // stream defers the record to the next call that switches streams (an event record costs the stream
    // a marker packet, ~3 us per call, which back-to-back calls on the default stream would otherwise
    // pay on every call): those streams cannot be destroyed, so the deferred record is always valid.
    void enter(hipStream_t s) {
        if (!used || last == s) return;
        if (persistent(last)) {
            if (!ev) MCV_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            MCV_HIP(hipEventRecord(ev, last));
        }
        MCV_HIP(hipStreamWaitEvent(s, ev, 0));
    }
    void leave(hipStream_t s) {
        if (!persistent(s)) {
            if (!ev) MCV_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            MCV_HIP(hipEventRecord(ev, s));
        }
        last = s;
        used = true;
    }
    ~StreamFence() {
        if (ev) (void)hipEventDestroy(ev);
    }
};

// Waves of `kernel` (blocks of `threads`) the current device holds at once: its occupancy x the CUs.
template <class K>
inline int64_t resident_waves(K kernel, int threads) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess || per <= 0) per = 1;
    return (int64_t)per * cus * (threads / 64);
}

// Point chunks of a (model waves) x (point chunks) sweep: with c chunks the launch takes
// ceil(waves c / resident) rounds of waves 1 / c as long, so the idle tail of the last round is what
// the count changes. Returns the smallest c in [1, hi] within 1 % of the fewest one-chunk-wave
// durations (more chunks cost per-wave model setup and count atomics).
inline int tail_chunks(int64_t waves, int64_t resident, int hi) {
    if (waves <= 0 || resident <= 0 || hi <= 1) return 1;
    double best = 1e300;
    for (int c = 1; c <= hi; ++c) {
        const double cost = (double)((waves * c + resident - 1) / resident) / c;
        if (cost < best) best = cost;
    }
    for (int c = 1; c <= hi; ++c)
        if ((double)((waves * c + resident - 1) / resident) / c <= best * 1.01) return c;
    return 1;
}

}  // namespace mcv
