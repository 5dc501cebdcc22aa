// scaled_pose_host.cpp — exports of CameraPose.findScaled (CameraPose.fs:39-134):
// the per-call setup (camera frames of CameraPose.fs:45-61, Camera.fs:35-70) on the host in fp64,
// the O(N^2) candidate verify on the GPU (scaled_pose.hip), and the host twin for the CPU tests.
#include "minicv_native.h"
#include "mcv_runtime.h"
#include "hyp_scaled.h"
#include "kernels.h"
#include <cmath>
#include <limits>

using namespace mcv;

namespace {

void normalize3(const double (&v)[3], double (&out)[3]) {   // Vec.normalize (see hyp_scaled.h)
    const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    if (l == 0.0) {
        out[0] = out[1] = out[2] = 0.0;
        return;
    }
    const double r = 1.0 / l;
    for (int i = 0; i < 3; ++i) out[i] = v[i] * r;
}

// Inverse of the affine M44d.FromBasis(x, y, z, o): [A | o]^-1 = [A^-1 | -A^-1 o], A^-1 by the
// adjugate (Aardvark's general M44d.Inverse rounds differently: equal to ~1e-16 relative).
void affine_inverse(const double (&A)[3][3], const double (&o)[3], double (&m)[3][4]) {
    const double c00 = A[1][1] * A[2][2] - A[1][2] * A[2][1];
    const double c01 = A[1][2] * A[2][0] - A[1][0] * A[2][2];
    const double c02 = A[1][0] * A[2][1] - A[1][1] * A[2][0];
    const double det = A[0][0] * c00 + A[0][1] * c01 + A[0][2] * c02;
    const double r = 1.0 / det;
    double inv[3][3];
    inv[0][0] = c00 * r;
    inv[0][1] = (A[0][2] * A[2][1] - A[0][1] * A[2][2]) * r;
    inv[0][2] = (A[0][1] * A[1][2] - A[0][2] * A[1][1]) * r;
    inv[1][0] = c01 * r;
    inv[1][1] = (A[0][0] * A[2][2] - A[0][2] * A[2][0]) * r;
    inv[1][2] = (A[0][2] * A[1][0] - A[0][0] * A[1][2]) * r;
    inv[2][0] = c02 * r;
    inv[2][1] = (A[0][1] * A[2][0] - A[0][0] * A[2][1]) * r;
    inv[2][2] = (A[0][0] * A[1][1] - A[0][1] * A[1][0]) * r;
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 3; ++j) m[i][j] = inv[i][j];
        m[i][3] = -(inv[i][0] * o[0] + inv[i][1] * o[1] + inv[i][2] * o[2]);
    }
}

ScaledSetup make_setup(const mcvCamera& c, const mcvM33d& Rm, const mcvV3d& Tv) {
    ScaledSetup S;
    const double right[3] = {c.right.X, c.right.Y, c.right.Z}, up[3] = {c.up.X, c.up.Y, c.up.Z};
    const double fwd[3] = {c.forward.X, c.forward.Y, c.forward.Z}, loc[3] = {c.location.X, c.location.Y, c.location.Z};
    for (int i = 0; i < 3; ++i) {   // toWorld = M44d.FromBasis(c.right, c.up, -c.forward, c.location)
        S.tw[i][0] = right[i];
        S.tw[i][1] = up[i];
        S.tw[i][2] = -fwd[i];
        S.tw[i][3] = loc[i];
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) S.R[i][j] = Rm.M[3 * i + j];
    S.T[0] = Tv.X;
    S.T[1] = Tv.Y;
    S.T[2] = Tv.Z;
    // toRotWorld = toWorld * transformation(pose): columns 0..2 are toWorld * R (T[3][j] = 0)
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            S.rot[i][j] = S.tw[i][0] * S.R[0][j] + S.tw[i][1] * S.R[1][j] + S.tw[i][2] * S.R[2][j] + S.tw[i][3] * 0.0;
    // TransformDir of the unit axes (Camera.fs:66-68)
    double dx[3], dy[3], dz[3];
    for (int i = 0; i < 3; ++i) {
        dx[i] = S.rot[i][0] * 1.0 + S.rot[i][1] * 0.0 + S.rot[i][2] * 0.0;
        dy[i] = S.rot[i][0] * 0.0 + S.rot[i][1] * 1.0 + S.rot[i][2] * 0.0;
        dz[i] = -(S.rot[i][0] * 0.0 + S.rot[i][1] * 0.0 + S.rot[i][2] * 1.0);
    }
    normalize3(dx, S.right);
    normalize3(dy, S.up);
    normalize3(dz, S.fwd);
    S.fx = c.focal.X;
    S.fy = c.focal.Y;
    // dstCam0 = transformedView (transformation (scale 0.0 pose)) srcCam; dst0View.Forward
    double loc0[3];
    scaled_location(S, 0.0, loc0);
    double A[3][3];
    for (int i = 0; i < 3; ++i) {
        A[i][0] = S.right[i];
        A[i][1] = S.up[i];
        A[i][2] = -S.fwd[i];
    }
    affine_inverse(A, loc0, S.minv);
    // dst0Translation = normalize (dst0View.Forward.TransformDir (srcView.Backward.TransformDir (R * T)))
    double rt[3], u[3], v[3];
    for (int i = 0; i < 3; ++i) rt[i] = S.R[i][0] * S.T[0] + S.R[i][1] * S.T[1] + S.R[i][2] * S.T[2];
    for (int i = 0; i < 3; ++i) u[i] = S.tw[i][0] * rt[0] + S.tw[i][1] * rt[1] + S.tw[i][2] * rt[2];
    for (int i = 0; i < 3; ++i) v[i] = S.minv[i][0] * u[0] + S.minv[i][1] * u[1] + S.minv[i][2] * u[2];
    normalize3(v, S.t);
    return S;
}

struct ScaledWork {
    DevBuf<double> w, o, soa, scales, costs;
    DevBuf<uint8_t> used;
    DevBuf<long long> out;
    hipStream_t s = nullptr;
    hipStream_t stream() {
        if (!s) MCV_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        return s;
    }
    ~ScaledWork() {
        if (s) (void)hipStreamDestroy(s);
    }
};
ScaledWork& work() {
    thread_local ScaledWork w;
    return w;
}

// Device part shared by the host-pointer and device-pointer exports. Synchronises s.
int scaled_device(const ScaledSetup& S, const double* d_w3, const double* d_o2, int N, double* outCost,
                  double* outScale, hipStream_t s, double* h_scales = nullptr, double* h_costs = nullptr) {
    ScaledWork& w = work();
    w.soa.ensure((size_t)N * 5);
    w.scales.ensure((size_t)N * 2);
    w.costs.ensure((size_t)N * 2);
    w.used.ensure((size_t)N);
    w.out.ensure(2);
    launch_scaled(S, d_w3, d_o2, N, w.soa.p, w.scales.p, w.used.p, w.costs.p, w.out.p, s);
    MCV_HIP(hipGetLastError());
    long long out[2];
    MCV_HIP(hipMemcpyAsync(out, w.out.p, sizeof(out), hipMemcpyDeviceToHost, s));
    if (h_scales) MCV_HIP(hipMemcpyAsync(h_scales, w.scales.p, (size_t)N * 2 * 8, hipMemcpyDeviceToHost, s));
    if (h_costs) MCV_HIP(hipMemcpyAsync(h_costs, w.costs.p, (size_t)N * 2 * 8, hipMemcpyDeviceToHost, s));
    MCV_HIP(hipStreamSynchronize(s));
    double cost = std::numeric_limits<double>::infinity(), scale = 0.0;
    if (out[0] >= 0) {
        MCV_HIP(hipMemcpyAsync(&cost, w.costs.p + out[0], 8, hipMemcpyDeviceToHost, s));
        MCV_HIP(hipMemcpyAsync(&scale, w.scales.p + out[0], 8, hipMemcpyDeviceToHost, s));
        MCV_HIP(hipStreamSynchronize(s));
    }
    if (outCost) *outCost = cost;
    if (outScale) *outScale = scale;
    return (int)out[1];
}

void check_args(const mcvCamera* c, const void* w, const void* o, int N, const mcvM33d* R, const mcvV3d* T) {
    if (!c || !R || !T || N < 0 || (N > 0 && (!w || !o))) fail("cvFindScaledPose: bad argument");
    if (N > (1 << 28)) fail("cvFindScaledPose: N = %d too large", N);
}

}  // namespace

extern "C" MCV_API int cvFindScaledPose(double inlierThreshold, const mcvCamera* srcCam, const mcvV3d* worldPoints,
                                        const mcvV2d* observations, int N, const mcvM33d* rotation,
                                        const mcvV3d* translation, double* outCost, double* outScale) {
    (void)inlierThreshold;   // unused by the reference too (CameraPose.fs:39; only countInliers reads it)
    MCV_GUARD(-1, {
        check_args(srcCam, worldPoints, observations, N, rotation, translation);
        if (N == 0) {   // CameraPose.fs:42: [] -> +inf, CameraPose()
            if (outCost) *outCost = std::numeric_limits<double>::infinity();
            if (outScale) *outScale = 0.0;
            return 0;
        }
        require_device();
        const ScaledSetup S = make_setup(*srcCam, *rotation, *translation);
        ScaledWork& w = work();
        hipStream_t s = w.stream();
        w.w.ensure((size_t)N * 3);
        w.o.ensure((size_t)N * 2);
        MCV_HIP(hipMemcpyAsync(w.w.p, worldPoints, (size_t)N * 24, hipMemcpyHostToDevice, s));
        MCV_HIP(hipMemcpyAsync(w.o.p, observations, (size_t)N * 16, hipMemcpyHostToDevice, s));
        return scaled_device(S, w.w.p, w.o.p, N, outCost, outScale, s);
    })
}

extern "C" MCV_API int cvFindScaledPoseCosts(const mcvCamera* srcCam, const mcvV3d* worldPoints,
                                             const mcvV2d* observations, int N, const mcvM33d* rotation,
                                             const mcvV3d* translation, double* scales, double* costs) {
    MCV_GUARD(-1, {
        check_args(srcCam, worldPoints, observations, N, rotation, translation);
        if (N == 0) return 0;
        if (!scales || !costs) fail("cvFindScaledPoseCosts: bad argument");
        require_device();
        const ScaledSetup S = make_setup(*srcCam, *rotation, *translation);
        ScaledWork& w = work();
        hipStream_t s = w.stream();
        w.w.ensure((size_t)N * 3);
        w.o.ensure((size_t)N * 2);
        MCV_HIP(hipMemcpyAsync(w.w.p, worldPoints, (size_t)N * 24, hipMemcpyHostToDevice, s));
        MCV_HIP(hipMemcpyAsync(w.o.p, observations, (size_t)N * 16, hipMemcpyHostToDevice, s));
        scaled_device(S, w.w.p, w.o.p, N, nullptr, nullptr, s, scales, costs);
        return N;
    })
}

extern "C" MCV_API int mcvFindScaledPoseDevice(const mcvCamera* srcCam, const mcvV3d* d_world, const mcvV2d* d_obs,
                                               int N, const mcvM33d* rotation, const mcvV3d* translation,
                                               double* outCost, double* outScale, void* stream) {
    MCV_GUARD(-1, {
        check_args(srcCam, d_world, d_obs, N, rotation, translation);
        if (N == 0) {
            if (outCost) *outCost = std::numeric_limits<double>::infinity();
            if (outScale) *outScale = 0.0;
            return 0;
        }
        require_device();
        const ScaledSetup S = make_setup(*srcCam, *rotation, *translation);
        return scaled_device(S, (const double*)d_world, (const double*)d_obs, N, outCost, outScale,
                             (hipStream_t)stream);
    })
}

extern "C" MCV_API int mcvHostScaledCosts(const mcvCamera* srcCam, const mcvV3d* worldPoints,
                                          const mcvV2d* observations, int N, const mcvM33d* rotation,
                                          const mcvV3d* translation, double* scales, double* costs) {
    MCV_GUARD(-1, {
        check_args(srcCam, worldPoints, observations, N, rotation, translation);
        const ScaledSetup S = make_setup(*srcCam, *rotation, *translation);
        const double inf = std::numeric_limits<double>::infinity();
        for (int i = 0; i < N; ++i) {
            double sx, sy;
            const mcvV3d& p = worldPoints[i];
            const mcvV2d& q = observations[i];
            if (!scaled_candidate(S, p.X, p.Y, p.Z, q.X, q.Y, sx, sy)) {
                scales[2 * i] = scales[2 * i + 1] = std::numeric_limits<double>::quiet_NaN();
                costs[2 * i] = costs[2 * i + 1] = inf;
                continue;
            }
            for (int h = 0; h < 2; ++h) {
                const double sc = h ? sy : sx;
                double loc[3];
                scaled_location(S, sc, loc);
                double sum = 0.0;
                int cnt = 0;
                for (int j = 0; j < N; ++j) {   // avgReprojectionError: list order, sequential sum
                    double e;
                    if (scaled_term(S, loc, worldPoints[j].X, worldPoints[j].Y, worldPoints[j].Z, observations[j].X,
                                    observations[j].Y, e)) {
                        sum += e;
                        cnt += 1;
                    }
                }
                scales[2 * i + h] = sc;
                costs[2 * i + h] = cnt == 0 ? inf : sum / (double)cnt;
            }
        }
        return N;
    })
}
