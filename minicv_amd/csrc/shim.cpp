// shim.cpp — the rest of the MiniCVNative C-ABI surface: error reporting, device query, and the
// reference exports that are outside the hot path (they bind, and fail loudly with a message).
//   cvDetectFeatures / cvFreeFeatures   MiniCVNative.cpp:221-365  (feature detection: out of scope)
//   cvDetectQRCode / cvDetectArucoMarkers MiniCVNative.cpp:384-502 (fiducials: out of scope)
//   cvTest                               MiniCVNative.cpp:504      (debug print: no-op)
#include "minicv_native.h"
#include "mcv_runtime.h"
#include <string>
#include <cstring>

namespace mcv {
static thread_local std::string g_last_error;
void set_last_error(const char* msg) { g_last_error = msg ? msg : ""; }
void clear_last_error() { g_last_error.clear(); }
}  // namespace mcv

using namespace mcv;

// ---- kernel timing (opt-in) ----
#include "plan.h"
#include <mutex>
#include <vector>
namespace {
struct ProfRec { std::string name; hipEvent_t a, b; };
std::mutex g_prof_mu;
std::vector<ProfRec> g_prof;
std::vector<hipEvent_t> g_prof_free;   // events of earlier records, reused (hipEventCreate per launch
                                       // costs microseconds of host time inside a timed loop)
int g_prof_on = 0;   // 0 off, else the sampling stride
std::vector<std::pair<std::string, long>> g_prof_ticks;   // launches seen per scope name
}  // namespace
namespace mcv {
bool prof_enabled() { return g_prof_on != 0; }
bool prof_sample(const char* name) {
    if (!g_prof_on) return false;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto& t : g_prof_ticks)
        if (t.first == name) return t.second++ % g_prof_on == 0;
    g_prof_ticks.push_back({name, 1});
    return true;
}
hipEvent_t prof_event() {
    {
        std::lock_guard<std::mutex> lk(g_prof_mu);
        if (!g_prof_free.empty()) {
            hipEvent_t e = g_prof_free.back();
            g_prof_free.pop_back();
            return e;
        }
    }
    hipEvent_t e = nullptr;
    return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
void prof_record(const char* name, hipEvent_t a, hipEvent_t b) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    g_prof.push_back({name, a, b});
}
}  // namespace mcv

extern "C" MCV_API void mcvProfileEnable(int on) { g_prof_on = on > 0 ? on : 0; }

extern "C" MCV_API void mcvProfileReset(void) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    for (auto& r : g_prof) {
        (void)hipEventSynchronize(r.b);
        g_prof_free.push_back(r.a);
        g_prof_free.push_back(r.b);
    }
    g_prof.clear();
    g_prof_ticks.clear();
}

extern "C" MCV_API int mcvProfileRead(const char* name, double* total_ms) {
    std::lock_guard<std::mutex> lk(g_prof_mu);
    int n = 0;
    double tot = 0;
    for (auto& r : g_prof) {
        if (r.name != name) continue;
        if (hipEventSynchronize(r.b) != hipSuccess) return -1;
        float ms = 0;
        if (hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) return -1;
        tot += ms;
        ++n;
    }
    if (total_ms) *total_ms = tot;
    return n;
}

extern "C" MCV_API const char* mcvGetLastError(void) { return g_last_error.c_str(); }

extern "C" MCV_API const char* mcvVersion(void) { return "minicv-mi355x 0.3.0 (gfx950)"; }
extern "C" MCV_API int mcvAbiVersion(void) { return MCV_ABI_VERSION; }

extern "C" MCV_API int mcvDeviceCount(void) {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) return 0;
    if (e != hipSuccess) {
        set_last_error(hipGetErrorString(e));
        return -1;
    }
    return n;
}

#define MCV_NOT_IN_SCOPE(name, why) set_last_error(name ": " why)

extern "C" MCV_API DetectorResult* cvDetectFeatures(char*, int, int, int, int, void*) {
    MCV_NOT_IN_SCOPE("cvDetectFeatures", "feature detection is outside the MI355X hot path (SURVEY 2 row 4)");
    return nullptr;
}

extern "C" MCV_API void cvFreeFeatures(DetectorResult* res) {
    // Frees a DetectorResult allocated with new[] members (fixes the reference's delete/new[]
    // mismatch and the PointCount == 0 leak, MiniCVNative.cpp:349-358).
    if (!res) return;
    delete[] res->Descriptors;
    delete[] res->Points;
    delete res;
}

extern "C" MCV_API void cvTest(void) {}

extern "C" MCV_API mcvBool cvDetectQRCode(char*, int, int, int, int*, int* count) {
    if (count) *count = 0;
    MCV_NOT_IN_SCOPE("cvDetectQRCode", "QR detection is outside the MI355X hot path (SURVEY 2 row 7)");
    return false;
}

extern "C" MCV_API mcvBool cvDetectArucoMarkers(char*, int, int, int, int* infoCount, ArucoMarkerInfo*) {
    if (infoCount) *infoCount = 0;
    MCV_NOT_IN_SCOPE("cvDetectArucoMarkers", "ArUco detection is outside the MI355X hot path (SURVEY 2 row 8)");
    return false;
}
