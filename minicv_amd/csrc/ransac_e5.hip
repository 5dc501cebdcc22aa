// ransac_e5.hip — the reference's own five-point solver (five_point_ref.h) on gfx950: the default
// minimal solver of the essential-matrix RANSAC behind cvRecoverPose(s) / cvFindEssentialMat, and the
// cvFivePoint export (reference fivepoint.cpp:233-339; MiniCVNative.cpp:177,204,368-382).
// Kept apart from ransac_e.hip: the generated getCoeffMat / c[] term code makes this unit slow to build.
#include "mcv_common.h"
#include "hyp_essential.h"
#include "five_point_ref.h"
#include "kernels.h"
#include "mcv_runtime.h"
#include "minicv_native.h"

namespace mcv {

// ---- the reference's five-point solver over many hypotheses (default RANSAC path) --------------
// Three kernels, one lane per hypothesis, every step from registers (five_point_ref.h), the staging
// between them in HBM as structure-of-arrays (entry-major, so a wave's 64 lanes touch 512 contiguous
// bytes per access):
//   mcv_e5_coeffs  sample -> JacobiSVD null basis (5 x 9, FULL_UV) -> getCoeffMat's 200 entries
//   mcv_e5_lu      cv::solve(A(:, 0:10), A(:, 10:20), DECOMP_LU) -> B (3 x 13) -> c[0..10] of det B(z)
//   mcv_e5_roots   cv::solvePoly (300 Durand-Kerner sweeps) -> per real root Bz, solveZ, E -> statuses +
//                  models appended to the dense list (one atomic per wave, slots in root order)
// Staging per hypothesis: A 200, null basis 36, B 39, c 11 doubles, status int (E5Stage below).
struct E5StageView {
    double* A;     // [200][H]
    double* nb;    // [36][H]
    double* bc;    // [50][H]: B (39) then c (11)
    int* status;   // [H]: -2 no sample, 0 degenerate, 1 solved
    int H;
    MCV_HD static size_t bytes(int H) { return (size_t)H * (286 * sizeof(double) + sizeof(int)); }
    MCV_HD static E5StageView at(void* base, int H) {
        E5StageView v;
        double* d = (double*)base;
        v.A = d;
        v.nb = d + (size_t)200 * H;
        v.bc = d + (size_t)236 * H;
        v.status = (int*)(d + (size_t)286 * H);
        v.H = H;
        return v;
    }
};

struct E5StoreGlobal {
    double* A;
    int H, i;
    __device__ void operator()(int r, int c, double v) { A[(size_t)(20 * r + c) * H + i] = v; }
};

__global__ __launch_bounds__(64) void mcv_e5_coeffs(const double* __restrict__ pts4, int N, Sampler smp,
                                                    int64_t hypBegin, int hypCount, E5StageView st) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= hypCount) return;
    SubsetSrc<5> src(smp, (uint64_t)(hypBegin + i));
    int idx[5];
    int got = 0;
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {   // no checkSubset (EMEstimatorCallback)
        got = src.next(N, idx);
        if (got != 0) break;
    }
    if (got <= 0) {
        st.status[i] = kStatusNoSample;
        return;
    }
    double x1[5], y1[5], x2[5], y2[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const double4 p = ((const double4*)pts4)[idx[k]];
        x1[k] = p.x; y1[k] = p.y; x2[k] = p.z; y2[k] = p.w;
    }
    double e[36];
    fpr_null_basis(x1, y1, x2, y2, e);
#pragma unroll
    for (int k = 0; k < 36; ++k) st.nb[(size_t)k * hypCount + i] = e[k];
    E5StoreGlobal store{st.A, hypCount, i};
    fpr_coeff_matrix(e, store);
    st.status[i] = 1;
}

// cv::solve(A(:, 0:10), A(:, 10:20), DECOMP_LU) on 32-lane groups (two hypotheses per wave): lane c < 20
// of a group holds column c of [A(:, 0:10) | A(:, 10:20)] in registers. Every element takes LUImpl's own
// operations in its order (fpr_lu_solve): the pivot row and value come from the pivot column's lane, the
// multipliers alpha_j = A[j][i] * d are formed by every lane from the broadcast A[j][i], a row swap is a
// per-lane register swap, and back substitution subtracts A[i][q] b[q] for q ascending with A[i][q]
// broadcast from lane q. The group then gathers B's rows (fpr_b_matrix) and every lane forms c[]; lane 0
// stores them.
__global__ __launch_bounds__(64) void mcv_e5_lu(E5StageView st) {
    const int lane = threadIdx.x, base = lane & 32, c = lane & 31;
    const int h = blockIdx.x * 2 + (lane >> 5);
    const bool act = h < st.H && st.status[h] == 1;   // uniform per group; both groups run every step
    const double eps = kDblEpsilon * 100;
    double col[10];
#pragma unroll
    for (int r = 0; r < 10; ++r) col[r] = (act && c < 20) ? st.A[(size_t)(20 * r + c) * st.H + h] : 0.0;
    bool singular = false;
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        int k = i;
        double ak = __builtin_fabs(col[i]);
#pragma unroll
        for (int j = i + 1; j < 10; ++j)
            if (__builtin_fabs(col[j]) > ak) { k = j; ak = __builtin_fabs(col[j]); }
        k = __shfl(k, base + i);
        ak = __shfl(ak, base + i);
        singular = singular || ak < eps;
        if (c >= i) {
#pragma unroll
            for (int r = i + 1; r < 10; ++r)
                if (r == k) { const double t = col[i]; col[i] = col[r]; col[r] = t; }
        }
        const double d = -1 / __shfl(col[i], base + i);
#pragma unroll
        for (int j = i + 1; j < 10; ++j) {
            const double alpha = __shfl(col[j], base + i) * d;
            if (c > i) col[j] += alpha * col[i];
        }
        if (c == i) col[i] = -d;
    }
#pragma unroll
    for (int i = 9; i >= 0; --i) {
        double s = col[i];
#pragma unroll
        for (int q = i + 1; q < 10; ++q) s -= __shfl(col[i], base + q) * col[q];
        const double aii = __shfl(col[i], base + i);
        if (c >= 10) col[i] = s * aii;
    }
    // B = row1 - row2 from the solution rows 4..9 (columns in lanes 10..19)
    double b[39];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double r1[10], r2[10];
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            r1[k] = __shfl(col[2 * i + 4], base + 10 + k);
            r2[k] = __shfl(col[2 * i + 5], base + 10 + k);
        }
        double row1[13], row2[13];
#pragma unroll
        for (int k = 0; k < 13; ++k) row1[k] = row2[k] = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            row1[1 + k] = r1[k] * 1.0; row1[5 + k] = r1[3 + k] * 1.0;
            row2[k] = r2[k] * 1.0; row2[4 + k] = r2[3 + k] * 1.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) { row1[9 + k] = r1[6 + k] * 1.0; row2[8 + k] = r2[6 + k] * 1.0; }
#pragma unroll
        for (int k = 0; k < 13; ++k) b[13 * i + k] = row1[k] - row2[k];
    }
    if (!act) return;
    if (singular) {
        if (c == 0) st.status[h] = 0;
        return;
    }
    double cf[11];
    fpr_det_coeffs(b, cf);
    if (c == 0) {
#pragma unroll
        for (int k = 0; k < 39; ++k) st.bc[(size_t)k * st.H + h] = b[k];
#pragma unroll
        for (int k = 0; k < 11; ++k) st.bc[(size_t)(39 + k) * st.H + h] = cf[k];
    }
}

// Two waves per SIMD (amdgpu_waves_per_eu: 324 -> 256 VGPRs, ~50 spilled): the 300-sweep Durand-Kerner
// chain is latency-bound at one wave, 29.5 -> 25.8 ms per 2^20 hypotheses. Splitting solvePoly into a
// kernel of its own (roots through the stage) measured 24.0 + 2.3 ms: solvePoly itself holds the
// registers; three / four waves per SIMD spill 58 / 121 VGPRs and lose.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) void mcv_e5_roots(E5StageView st, EModel* __restrict__ dense,
                                                   int* __restrict__ denseSlot, int* __restrict__ nDense,
                                                   int* __restrict__ counts) {
    const int lane = threadIdx.x;
    const int i = blockIdx.x * 64 + lane;
    const bool act = i < st.H;
    const int status = act ? st.status[i] : 0;
    FprCplx roots[10];
    double b[39];
    if (status == 1) {
        double c[11];
#pragma unroll
        for (int k = 0; k < 11; ++k) c[k] = st.bc[(size_t)(39 + k) * st.H + i];
        fpr_solve_poly(c, roots);
#pragma unroll
        for (int k = 0; k < 39; ++k) b[k] = st.bc[(size_t)k * st.H + i];
    }
    // pass 1: which roots give a model (count only), pass 2: write them
    uint32_t okm = 0;
    int m = 0;
    if (status == 1) {
        double e[36];
#pragma unroll
        for (int k = 0; k < 36; ++k) e[k] = st.nb[(size_t)k * st.H + i];
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (__builtin_fabs(roots[r].im) > 1e-10) continue;
            double E[9];
            if (fpr_model(b, e, roots[r].re, E)) {
                okm |= 1u << r;
                ++m;
            }
        }
    }
    if (act)
        for (int s2 = 0; s2 < kEMaxModels; ++s2)
            counts[(int64_t)i * kEMaxModels + s2] =
                s2 < m ? 0 : (s2 == 0 && status == kStatusNoSample ? kStatusNoSample : kStatusNoModel);
    int incl = m;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        incl += lane >= o ? y : 0;
    }
    const int total = __shfl(incl, 63);
    int base = 0;
    if (lane == 63 && total > 0) base = atomicAdd(nDense, total);
    base = __shfl(base, 63) + incl - m;
    if (okm) {
        double e[36];
#pragma unroll
        for (int k = 0; k < 36; ++k) e[k] = st.nb[(size_t)k * st.H + i];
        int t = 0;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (!((okm >> r) & 1u)) continue;
            EModel em;
            (void)fpr_model(b, e, roots[r].re, em.e);
            dense[base + t] = em;
            denseSlot[base + t] = i * kEMaxModels + t;
            ++t;
        }
    }
}

// Winner re-solve with the reference's solver (one lane): all models of hypothesis `hyp`.
__global__ __launch_bounds__(64) void mcv_e5_one(const double* __restrict__ pts4, int N, Sampler smp, int64_t hyp,
                                                 EOneOut* __restrict__ out) {
    if (threadIdx.x != 0) return;
    SubsetSrc<5> src(smp, (uint64_t)hyp);
    int idx[5] = {-1, -1, -1, -1, -1};
    int got = 0;
    for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
        got = src.next(N, idx);
        if (got != 0) break;
    }
    int n = kStatusNoSample;
    if (got > 0) {
        double x1[5], y1[5], x2[5], y2[5];
        for (int k = 0; k < 5; ++k) {
            const double4 p = ((const double4*)pts4)[idx[k]];
            x1[k] = p.x; y1[k] = p.y; x2[k] = p.z; y2[k] = p.w;
        }
        n = fpr_solve5(x1, y1, x2, y2, out->E);
    }
    out->status = n;
    for (int k = 0; k < 5; ++k) out->idx[k] = idx[k];
    for (int s2 = n > 0 ? n : 0; s2 < kEMaxModels; ++s2)
        for (int k = 0; k < 9; ++k) out->E[s2][k] = 0.0;
}

// cvFivePoint: the reference's own solver (five_point_ref.h fpr_solve5), one lane.
__global__ __launch_bounds__(64) void mcv_e_fivepoint(EFiveIn in, EOneOut* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const int n = fpr_solve5(in.x1, in.y1, in.x2, in.y2, out->E);   // models straight to the record
    out->status = n;
    for (int s = n > 0 ? n : 0; s < kEMaxModels; ++s)
        for (int k = 0; k < 9; ++k) out->E[s][k] = 0.0;
}

// ---- launchers ---------------------------------------------------------------------------------
size_t e5_stage_bytes(int hypCount) { return E5StageView::bytes(hypCount); }

void launch_e5_generate(const double* d_pts4, int N, Sampler smp, int64_t hypBegin, int hypCount, void* d_dense,
                        int* d_denseSlot, int* d_nDense, int* d_counts, void* d_stage, hipStream_t s) {
    (void)hipMemsetAsync(d_nDense, 0, sizeof(int), s);
    if (hypCount <= 0) return;
    const E5StageView st = E5StageView::at(d_stage, hypCount);
    const dim3 g((hypCount + 63) / 64);
    hipLaunchKernelGGL(mcv_e5_coeffs, g, dim3(64), 0, s, d_pts4, N, smp, hypBegin, hypCount, st);
    hipLaunchKernelGGL(mcv_e5_lu, dim3((hypCount + 1) / 2), dim3(64), 0, s, st);
    hipLaunchKernelGGL(mcv_e5_roots, g, dim3(64), 0, s, st, (EModel*)d_dense, d_denseSlot, d_nDense, d_counts);
}

void launch_e5_one(const double* d_pts4, int N, Sampler smp, int64_t hyp, EOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_e5_one, dim3(1), dim3(64), 0, s, d_pts4, N, smp, hyp, d_out);
}

void launch_e_fivepoint(const EFiveIn& in, EOneOut* d_out, hipStream_t s) {
    hipLaunchKernelGGL(mcv_e_fivepoint, dim3(1), dim3(64), 0, s, in, d_out);
}

}  // namespace mcv

// ---- host twins (test hooks) -------------------------------------------------------------------
using namespace mcv;

// Host twin of one RANSAC hypothesis with the reference's solver (the default GPU path).
extern "C" MCV_API int mcvHostEssential(const double* pts4, int N, uint64_t seed, int64_t hyp, double* E90,
                                        int* sampleIdx) {
    MCV_GUARD(kStatusNoSample - 1, {
        if (!pts4 || !E90 || N < 5) fail("mcvHostEssential: bad argument");
        double E[kEMaxModels][9];
        SubsetSrc<5> src(Sampler{seed, nullptr}, (uint64_t)hyp);
        int idx[5];
        int got = 0;
        for (int attempt = 0; attempt < kMaxAttempts; ++attempt) {
            got = src.next(N, idx);
            if (got != 0) break;
        }
        if (got <= 0) return kStatusNoSample;
        double x1[5], y1[5], x2[5], y2[5];
        for (int k = 0; k < 5; ++k) {
            x1[k] = pts4[4 * idx[k]]; y1[k] = pts4[4 * idx[k] + 1]; x2[k] = pts4[4 * idx[k] + 2]; y2[k] = pts4[4 * idx[k] + 3];
        }
        if (sampleIdx) for (int k = 0; k < 5; ++k) sampleIdx[k] = idx[k];
        const int n = fpr_solve5(x1, y1, x2, y2, E);
        for (int s = 0; s < kEMaxModels; ++s)
            for (int k = 0; k < 9; ++k) E90[9 * s + k] = s < n ? E[s][k] : 0.0;
        return n;
    })
}

extern "C" MCV_API int mcvHostFivePointRef(const double* p20, double* E90) {
    MCV_GUARD(-1, {
        if (!p20 || !E90) fail("mcvHostFivePointRef: null argument");
        double E[kEMaxModels][9];
        const int n = fpr_solve5(p20, p20 + 5, p20 + 10, p20 + 15, E);
        for (int s = 0; s < kEMaxModels; ++s)
            for (int k = 0; k < 9; ++k) E90[9 * s + k] = s < n ? E[s][k] : 0.0;
        return n;
    })
}

