// ransac_pnp.hip — gfx950 kernels of the PnP-RANSAC path behind cvSolvePnPRansac
// (reference MiniCVNative.cpp:93-139, ap3p.cpp:123-317).
//
//   mcv_pnp_pack         V2d image + V3d world -> PnpPoint (fp32, 32 B) on the device.
//   mcv_pnp_generate     one lane per hypothesis: Philox sample of 4 -> undistort -> AP3P
//                        (3 points) + 4th-point selection (fp64) -> PnpPose (96 B) + status.
//   mcv_pnp_verify<K,F>  inlier sweep, 2-D grid: a wave holds K poses (fp64, VGPRs) and one chunk
//                        of the correspondences; projectPoints (k1, k2, p1, p2) in fp64, fp32
//                        squared pixel error, ballot + popcount; chunk partial counts are added
//                        with integer atomics (order-free, exact). The 2-D split keeps the chip
//                        busy at the reference's default 100 iterations.
//   mcv_pnp_one / _mask  winner recompute, inlier mask.
//   OpPnpLM / OpPnpVVS   fixed-order fp64 reductions for the LM refit / VVS refinement.
//   mcv_pnp_ap3p         solveAp3p export: one AP3P solve (3 points).
#include "mcv_common.h"
#include "hyp_pnp.h"
#include "reduce.h"
#include "kernels.h"
#include <cstdlib>

namespace mcv {

__global__ __launch_bounds__(256) void mcv_pnp_pack(const double* __restrict__ img, const double* __restrict__ world,
                                                    int N, PnpPoint* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    PnpPoint p;
    p.X = (float)world[3 * (size_t)i];
    p.Y = (float)world[3 * (size_t)i + 1];
    p.Z = (float)world[3 * (size_t)i + 2];
    p.u = (float)img[2 * (size_t)i];
    p.v = (float)img[2 * (size_t)i + 1];
    p.pad0 = p.pad1 = p.pad2 = 0.f;
    out[i] = p;
}

__global__ __launch_bounds__(64) void mcv_pnp_generate(const PnpPoint* __restrict__ pts, int N, PnpCamera cam,
                                                       uint64_t seed, int64_t hypBegin, int hypCount,
                                                       PnpPose* __restrict__ models, int* __restrict__ counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= hypCount) return;
    PnpPose p;
    const int st = pnp_hypothesis(pts, N, cam, seed, (uint64_t)(hypBegin + i), p, nullptr);
    if (st == 1) {
        models[i] = p;
        counts[i] = 0;
    } else {
        counts[i] = st;
    }
}

template <int K, bool FUSED>
__global__ __launch_bounds__(256) void mcv_pnp_verify(const PnpPoint* __restrict__ pts, int N, int chunk,
                                                      PnpCamera cam, const PnpPose* __restrict__ models,
                                                      int* __restrict__ counts, int hypCount, float thr2) {
    const int wave = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * 256u + threadIdx.x) >> 6));
    const int lane = threadIdx.x & 63;
    const int h0 = wave * K;
    if (h0 >= hypCount) return;
    double R[K][9], t[K][3];
    bool valid[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int hk = h0 + k;
        valid[k] = hk < hypCount && counts[hk] >= 0;
        const PnpPose m = models[valid[k] ? hk : h0];
#pragma unroll
        for (int j = 0; j < 9; ++j) R[k][j] = valid[k] ? m.R[j] : (j % 4 == 0 ? 1.0 : 0.0);
#pragma unroll
        for (int j = 0; j < 3; ++j) t[k][j] = valid[k] ? m.t[j] : 1e30;
        // poses in VGPRs: 4 x 12 doubles in SGPRs spill into VGPR lanes (v_readlane per use)
#pragma unroll
        for (int j = 0; j < 9; ++j) asm volatile("" : "+v"(R[k][j]));
#pragma unroll
        for (int j = 0; j < 3; ++j) asm volatile("" : "+v"(t[k][j]));
    }
    const int p0 = blockIdx.y * chunk;
    const int p1 = min(N, p0 + chunk);
    uint32_t cnt[K];
#pragma unroll
    for (int k = 0; k < K; ++k) cnt[k] = 0;
    for (int base = p0; base < p1; base += 64) {
        const int p = base + lane;
        const bool v = p < p1;
        const PnpPoint q = pts[v ? p : p0];
        // every lane evaluates (the padding lanes re-read point p0): `v && err <= thr2` would
        // short-circuit into a divergent branch around the whole projection
        const uint64_t vm = __builtin_amdgcn_ballot_w64(v);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float e = pnp_error(cam, R[k], t[k], q.X, q.Y, q.Z, q.u, q.v, FUSED);
            cnt[k] += (uint32_t)__popcll(vm & __builtin_amdgcn_ballot_w64(e <= thr2));
        }
    }
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (valid[k] && cnt[k]) atomicAdd(counts + h0 + k, (int)cnt[k]);
    }
}

__global__ void mcv_pnp_one(const PnpPoint* __restrict__ pts, int N, PnpCamera cam, uint64_t seed, int64_t hyp,
                            PnpOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    PnpPose p;
    for (int k = 0; k < 9; ++k) p.R[k] = 0;
    for (int k = 0; k < 3; ++k) p.t[k] = 0;
    int idx[4] = {-1, -1, -1, -1};
    out->status = pnp_hypothesis(pts, N, cam, seed, (uint64_t)hyp, p, idx);
    for (int k = 0; k < 9; ++k) out->R[k] = p.R[k];
    for (int k = 0; k < 3; ++k) out->t[k] = p.t[k];
    for (int k = 0; k < 4; ++k) out->idx[k] = idx[k];
}

// Direct four-point solve on given normalised points (N == 4 path of solvePnPRansac / solvePnP).
__global__ void mcv_pnp_solve4(const PnpPoint* __restrict__ pts, PnpCamera cam, PnpOneOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double x[4], y[4], W[4][3];
    for (int i = 0; i < 4; ++i) {
        const PnpPoint p = pts[i];
        pnp_undistort(cam, (double)p.u, (double)p.v, x[i], y[i]);
        W[i][0] = p.X; W[i][1] = p.Y; W[i][2] = p.Z;
    }
    PnpPose p;
    for (int k = 0; k < 9; ++k) p.R[k] = 0;
    for (int k = 0; k < 3; ++k) p.t[k] = 0;
    out->status = pnp_ap3p4(cam, x, y, W, p) ? 1 : kStatusNoModel;
    for (int k = 0; k < 9; ++k) out->R[k] = p.R[k];
    for (int k = 0; k < 3; ++k) out->t[k] = p.t[k];
    for (int k = 0; k < 4; ++k) out->idx[k] = k;
}

__global__ __launch_bounds__(256) void mcv_pnp_mask(const PnpPoint* __restrict__ pts, int N, PnpCamera cam,
                                                    PnpPose m, float thr2, bool fused, uint8_t* __restrict__ mask,
                                                    int* __restrict__ count) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool in = false;
    if (i < N) {
        const PnpPoint q = pts[i];
        in = pnp_error(cam, m.R, m.t, q.X, q.Y, q.Z, q.u, q.v, fused) <= thr2;
        mask[i] = in ? 1 : 0;
    }
    const uint64_t b = __ballot(in);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(count, (int)__popcll(b));
}

// The reference's solveAp3p (ap3p.cpp:282-317): bearings from (inv_fx u - cx_fx, ...), all solutions.
__global__ void mcv_pnp_ap3p(Ap3pIn in, Ap3pOut* __restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double b[3][3], w[3][3];
    for (int i = 0; i < 3; ++i) {
        double mu = in.inv_fx * in.mu[i] - in.cx_fx;
        double mv = in.inv_fy * in.mv[i] - in.cy_fy;
        const double nrm = sqrt(mu * mu + mv * mv + 1);
        const double mk = 1. / nrm;
        mu = mu * mk;
        mv = mv * mk;
        b[i][0] = mu; b[i][1] = mv; b[i][2] = mk;
        for (int k = 0; k < 3; ++k) w[i][k] = in.W[i][k];
    }
    double Rr[kPnpMaxSolutions][9], tr[kPnpMaxSolutions][3];
    const int n = ap3p_compute_poses(b, w, Rr, tr);
    out->count = n;
    for (int s = 0; s < kPnpMaxSolutions; ++s) {
        for (int k = 0; k < 9; ++k) out->R[s][k] = s < n ? Rr[s][k] : 0.0;
        for (int k = 0; k < 3; ++k) out->t[s][k] = s < n ? tr[s][k] : 0.0;
    }
}

// ---- LM / VVS reductions ---------------------------------------------------------------------
// Per correspondence: residual r = projectPoints(X) - observed (pixels, fp64) and its Jacobian
// w.r.t. (rvec, t) through dR/drvec (host Rodrigues derivative). 28 sums: J^T J upper (21),
// J^T r (6), |r|^2 (1).
struct OpPnpLM {
    const PnpPoint* pts; const uint8_t* mask; PnpCamera c; double R[9]; double t[3]; double dR[27]; bool wantJ;
    __device__ void operator()(int i, double (&a)[28]) const {
        if (mask && !mask[i]) return;
        const PnpPoint q = pts[i];
        const double X = q.X, Y = q.Y, Z = q.Z;
        const double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
        const double Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        const double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        const double iz = Zc != 0 ? 1.0 / Zc : 1.0;
        const double x = Xc * iz, y = Yc * iz;
        const double r2 = x * x + y * y, r4 = r2 * r2;
        const double cdist = 1.0 + c.k1 * r2 + c.k2 * r4;
        const double xd = x * cdist + c.p1 * (2.0 * x * y) + c.p2 * (r2 + 2.0 * x * x);
        const double yd = y * cdist + c.p1 * (r2 + 2.0 * y * y) + c.p2 * (2.0 * x * y);
        const double ru = xd * c.fx + c.cx - (double)q.u;
        const double rv = yd * c.fy + c.cy - (double)q.v;
        a[27] += ru * ru + rv * rv;
        if (!wantJ) return;
        const double dcr = c.k1 + 2.0 * c.k2 * r2;              // d cdist / d r2
        const double dxdx = cdist + x * dcr * 2.0 * x + 2.0 * c.p1 * y + 6.0 * c.p2 * x;
        const double dxdy = x * dcr * 2.0 * y + 2.0 * c.p1 * x + 2.0 * c.p2 * y;
        const double dydx = y * dcr * 2.0 * x + 2.0 * c.p1 * x + 2.0 * c.p2 * y;
        const double dydy = cdist + y * dcr * 2.0 * y + 6.0 * c.p1 * y + 2.0 * c.p2 * x;
        // d(x, y) / d(Xc, Yc, Zc) = iz [[1, 0, -x], [0, 1, -y]]
        const double du[3] = {c.fx * dxdx * iz, c.fx * dxdy * iz, c.fx * (-dxdx * x - dxdy * y) * iz};
        const double dv[3] = {c.fy * dydx * iz, c.fy * dydy * iz, c.fy * (-dydx * x - dydy * y) * iz};
        double Ju[6], Jv[6];
#pragma unroll
        for (int j = 0; j < 3; ++j) {   // dXc/drvec_j = dR/dr_j * X
            const double* d = dR + 9 * j;
            const double gx = d[0] * X + d[1] * Y + d[2] * Z;
            const double gy = d[3] * X + d[4] * Y + d[5] * Z;
            const double gz = d[6] * X + d[7] * Y + d[8] * Z;
            Ju[j] = du[0] * gx + du[1] * gy + du[2] * gz;
            Jv[j] = dv[0] * gx + dv[1] * gy + dv[2] * gz;
            Ju[3 + j] = du[j];
            Jv[3 + j] = dv[j];
        }
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j)
#pragma unroll
            for (int k = j; k < 6; ++k) a[o++] += Ju[j] * Ju[k] + Jv[j] * Jv[k];
#pragma unroll
        for (int j = 0; j < 6; ++j) a[21 + j] += Ju[j] * ru + Jv[j] * rv;
    }
};

// VVS (solvePnPRefineVVS, [ext]): normalised-plane feature error e = (x, y) - undistorted observed
// point, interaction matrix L (2 x 6, camera-frame twist (v, w)); sums L^T L (21), L^T e (6), |e|^2.
struct OpPnpVVS {
    const PnpPoint* pts; const uint8_t* mask; PnpCamera c; double R[9]; double t[3];
    __device__ void operator()(int i, double (&a)[28]) const {
        if (mask && !mask[i]) return;
        const PnpPoint q = pts[i];
        const double X = q.X, Y = q.Y, Z = q.Z;
        const double Xc = R[0] * X + R[1] * Y + R[2] * Z + t[0];
        const double Yc = R[3] * X + R[4] * Y + R[5] * Z + t[1];
        const double Zc = R[6] * X + R[7] * Y + R[8] * Z + t[2];
        const double iz = Zc != 0 ? 1.0 / Zc : 1.0;
        const double x = Xc * iz, y = Yc * iz;
        double xo, yo;
        pnp_undistort(c, (double)q.u, (double)q.v, xo, yo);
        const double ex = x - xo, ey = y - yo;
        const double Lx[6] = {-iz, 0.0, x * iz, x * y, -(1.0 + x * x), y};
        const double Ly[6] = {0.0, -iz, y * iz, 1.0 + y * y, -x * y, -x};
        int o = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j)
#pragma unroll
            for (int k = j; k < 6; ++k) a[o++] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
#pragma unroll
        for (int j = 0; j < 6; ++j) a[21 + j] += Lx[j] * ex + Ly[j] * ey;
        a[27] += ex * ex + ey * ey;
    }
};

// ---- launchers --------------------------------------------------------------------------------
static PnpCamera to_cam(const double* cam8) {
    PnpCamera c;
    c.fx = cam8[0]; c.fy = cam8[1]; c.cx = cam8[2]; c.cy = cam8[3];
    c.k1 = cam8[4]; c.k2 = cam8[5]; c.p1 = cam8[6]; c.p2 = cam8[7];
    return c;
}

void launch_pnp_pack(const double* d_img, const double* d_world, int N, void* d_pts, hipStream_t s) {
    if (N <= 0) return;
    hipLaunchKernelGGL(mcv_pnp_pack, dim3((N + 255) / 256), dim3(256), 0, s, d_img, d_world, N, (PnpPoint*)d_pts);
}

void launch_pnp_generate(const void* d_pts, int N, const double* cam8, uint64_t seed, int64_t hypBegin, int hypCount,
                         void* d_models, int* d_counts, hipStream_t s) {
    hipLaunchKernelGGL(mcv_pnp_generate, dim3((hypCount + 63) / 64), dim3(64), 0, s, (const PnpPoint*)d_pts, N,
                       to_cam(cam8), seed, hypBegin, hypCount, (PnpPose*)d_models, d_counts);
}

template <int K>
static void launch_pnp_verify_k(const void* d_pts, int N, const double* cam8, const void* d_models, int* d_counts,
                                int hypCount, float thr2, bool fused, hipStream_t s) {
    const int waves = (hypCount + K - 1) / K;
    // split the correspondences so that waves x chunks >= ~8 waves per SIMD, chunks >= 2048 points
    int chunks = (8192 + waves - 1) / waves;
    const int maxChunks = (N + 2047) / 2048;
    if (chunks > maxChunks) chunks = maxChunks;
    if (chunks < 1) chunks = 1;
    int chunk = (N + chunks - 1) / chunks;
    chunk = (chunk + 63) & ~63;
    chunks = (N + chunk - 1) / chunk;
    if (chunks < 1) chunks = 1;
    const dim3 grid((waves + 3) / 4, chunks);
    const PnpPoint* p = (const PnpPoint*)d_pts;
    const PnpPose* m = (const PnpPose*)d_models;
    if (fused)
        hipLaunchKernelGGL((mcv_pnp_verify<K, true>), grid, dim3(256), 0, s, p, N, chunk, to_cam(cam8), m, d_counts,
                           hypCount, thr2);
    else
        hipLaunchKernelGGL((mcv_pnp_verify<K, false>), grid, dim3(256), 0, s, p, N, chunk, to_cam(cam8), m, d_counts,
                           hypCount, thr2);
}

// Poses per wave; MCV_PNP_K selects alternatives for the variant screen only.
void launch_pnp_verify(const void* d_pts, int N, const double* cam8, const void* d_models, int* d_counts, int hypCount,
                       float thr2, bool fused, hipStream_t s) {
    static const int k = [] {
        const char* e = getenv("MCV_PNP_K");
        return e ? atoi(e) : kVerifyPnpPosesPerWave;
    }();
    switch (k) {
        case 2: launch_pnp_verify_k<2>(d_pts, N, cam8, d_models, d_counts, hypCount, thr2, fused, s); break;
        case 6: launch_pnp_verify_k<6>(d_pts, N, cam8, d_models, d_counts, hypCount, thr2, fused, s); break;
        case 8: launch_pnp_verify_k<8>(d_pts, N, cam8, d_models, d_counts, hypCount, thr2, fused, s); break;
        default: launch_pnp_verify_k<kVerifyPnpPosesPerWave>(d_pts, N, cam8, d_models, d_counts, hypCount, thr2, fused, s);
    }
}

void launch_pnp_one(const void* d_pts, int N, const double* cam8, uint64_t seed, int64_t hyp, PnpOneOut* d_out,
                    hipStream_t s) {
    hipLaunchKernelGGL(mcv_pnp_one, dim3(1), dim3(64), 0, s, (const PnpPoint*)d_pts, N, to_cam(cam8), seed, hyp, d_out);
}

void launch_pnp_solve4(const void* d_pts, const double* cam8, PnpOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_pnp_solve4, dim3(1), dim3(64), 0, s, (const PnpPoint*)d_pts, to_cam(cam8), d_out);
}

void launch_pnp_mask(const void* d_pts, int N, const double* cam8, const double* R9, const double* t3, float thr2,
                     bool fused, uint8_t* d_mask, int* d_count, hipStream_t s) {
    PnpPose m;
    for (int k = 0; k < 9; ++k) m.R[k] = R9[k];
    for (int k = 0; k < 3; ++k) m.t[k] = t3[k];
    hipLaunchKernelGGL(mcv_pnp_mask, dim3((N + 255) / 256), dim3(256), 0, s, (const PnpPoint*)d_pts, N, to_cam(cam8),
                       m, thr2, fused, d_mask, d_count);
}

void launch_pnp_ap3p(const Ap3pIn& in, Ap3pOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_pnp_ap3p, dim3(1), dim3(64), 0, s, in, d_out);
}

void pnp_reduce_lm(const void* d_pts, int N, const uint8_t* d_mask, const double* cam8, const double* R9,
                   const double* t3, const double* dR27, bool wantJ, double* d_part, double* d_out, hipStream_t s) {
    OpPnpLM op;
    op.pts = (const PnpPoint*)d_pts;
    op.mask = d_mask;
    op.c = to_cam(cam8);
    for (int k = 0; k < 9; ++k) op.R[k] = R9[k];
    for (int k = 0; k < 3; ++k) op.t[k] = t3[k];
    for (int k = 0; k < 27; ++k) op.dR[k] = dR27 ? dR27[k] : 0.0;
    op.wantJ = wantJ;
    run_reduce<28>(N, op, d_part, d_out, s);
}

void pnp_reduce_vvs(const void* d_pts, int N, const uint8_t* d_mask, const double* cam8, const double* R9,
                    const double* t3, double* d_part, double* d_out, hipStream_t s) {
    OpPnpVVS op;
    op.pts = (const PnpPoint*)d_pts;
    op.mask = d_mask;
    op.c = to_cam(cam8);
    for (int k = 0; k < 9; ++k) op.R[k] = R9[k];
    for (int k = 0; k < 3; ++k) op.t[k] = t3[k];
    run_reduce<28>(N, op, d_part, d_out, s);
}

}  // namespace mcv
