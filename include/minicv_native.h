/*
 * minicv_native.h — C-ABI of the MI355X-native MiniCVNative drop-in.
 *
 * The managed host (F# `module OpenCV.Native`, /root/reference/src/MiniCV/OpenCV.fs:339-382)
 * binds `[<DllImport("MiniCVNative")>]` entry points. This header declares
 *   (1) the 13 existing exports of the reference library, byte-compatible signatures
 *       (definitions: /root/reference/src/MiniCVNative/MiniCVNative.cpp:48-548, ap3p.cpp:282);
 *   (2) the new hot-path exports (findHomography / findFundamentalMat RANSAC, brute-force
 *       Hamming / L2 matching), written in the conventions of the existing ones
 *       (AoS fp64 point arrays + separate N, caller-allocated byte mask, M33d& out, int return);
 *   (3) a device-level API (plain device pointers + hipStream_t passed as void*) used by
 *       bench.py / multi-GPU ranks that keep inputs resident in HBM.
 *
 * Conventions:
 *   V2d  = 2 x double (x, y)            <-> Aardvark V2d / cv::Point2d
 *   V3d  = 3 x double                   <-> Aardvark V3d / cv::Vec3d
 *   M33d = 9 x double, row-major        <-> Aardvark M33d / cv::Matx33d
 *   masks are caller-allocated uint8[N], values 0/1
 *   no exception crosses the boundary: failure = false / 0 / NULL; mcvGetLastError() says why.
 */
#ifndef MINICV_NATIVE_H
#define MINICV_NATIVE_H

#include <stdint.h>
#include <stdbool.h>
#include <stddef.h>

#if defined(_WIN32)
#define MCV_API __declspec(dllexport)
#else
#define MCV_API __attribute__((visibility("default")))
#endif

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double X, Y; } mcvV2d;
typedef struct { double X, Y, Z; } mcvV3d;
typedef struct { double M[9]; } mcvM33d;       /* row-major */
typedef struct { float X, Y; } mcvV2f;
/* The reference's `bool` exports (MiniCVNative.cpp:48,93,165,384,439) return a 1-byte C++ bool,
 * while the F# P/Invoke side (OpenCV.fs:343-382, no MarshalAs) reads a 4-byte Win32 BOOL: only the
 * low byte is defined there. This library returns them as a 32-bit 0/1, so the upper bytes are
 * zero and both readings agree. */
typedef int32_t mcvBool;

/* ------------------------------------------------------------------------------------------
 * (1) Existing exports of the reference (same names, same argument meaning).
 * ---------------------------------------------------------------------------------------- */

/* RecoverPoseConfig — MiniCVNative.cpp:39-46, OpenCV.fs:16-36 (40 bytes). */
typedef struct {
    double FocalLength;
    mcvV2d PrincipalPoint;
    double Probability;
    double InlierThreshold;
} RecoverPoseConfig;

/* KeyPoint2d / DetectorResult — MiniCVNative.h:14-29, OpenCV.fs:300-337. */
typedef struct {
    mcvV2f pt;
    float size;
    float angle;
    float response;
    int octave;
    int class_id;
} KeyPoint2d;

typedef struct {
    int PointCount;
    int DescriptorEntries;
    int DescriptorElementType;   /* OpenCV depth code (0 = u8, 5 = f32) */
    KeyPoint2d* Points;
    uint8_t* Descriptors;        /* row-major [PointCount][dim] */
} DetectorResult;

typedef struct {
    int Id;
    mcvV2f P0, P1, P2, P3;
} ArucoMarkerInfo;

/* Essential-matrix RANSAC + pose — MiniCVNative.cpp:197-215 (on the GPU):
 * findEssentialMat(pa, pb, f, pp, RANSAC, Probability, InlierThreshold) -> ms = RANSAC mask ->
 * recoverPose(E, ..., mask) (cheirality over the inliers, distance 50). Returns the number of
 * inliers passing the cheirality test of the chosen (R, t); 0 on failure (ms untouched). */
MCV_API int  cvRecoverPose(const RecoverPoseConfig* config, const int N, const mcvV2d* pa, const mcvV2d* pb,
                           mcvM33d* rMat, mcvV3d* tVec, uint8_t* ms);
/* MiniCVNative.cpp:165-194: findEssentialMat -> ms -> decomposeEssentialMat(E) -> R1, R2, t.
 * false if N < 5 or no model (ms untouched then). */
MCV_API mcvBool cvRecoverPoses(const RecoverPoseConfig* config, const int N, const mcvV2d* pa, const mcvV2d* pb,
                            mcvM33d* rMat1, mcvM33d* rMat2, mcvV3d* tVec, uint8_t* ms);
/* Feature detection — MiniCVNative.cpp:221-365 (out of scope: returns NULL). */
MCV_API DetectorResult* cvDetectFeatures(char* data, int width, int height, int channels, int mode, void* config);
MCV_API void cvFreeFeatures(DetectorResult* res);
/* Debug export — MiniCVNative.cpp:504 (no-op). */
MCV_API void cvTest(void);
/* Five-point minimal solver — MiniCVNative.cpp:368-382 / fivepoint.cpp:233-339 (one GPU solve of
 * the reference's own path: SVD null space, solvePoly roots with |Im| <= 1e-10 in its order):
 * Es: caller-allocated 10 x M33d, unit-Frobenius-norm E with pb^T E pa = 0. Returns the count. */
MCV_API int  cvFivePoint(const mcvV2d* pa, const mcvV2d* pb, mcvM33d* Es);
/* PnP — MiniCVNative.cpp:48-163 (on the GPU). K passed by value as in the
 * reference; distortion = 4 doubles (k1, k2, p1, p2; MiniCVNative.cpp:78,120).
 * cvSolvePnPRansac (OpenCV 4.x solvePnPRansac): solverKind 2 / 5 (P3P / AP3P) sample 4 points
 * for AP3P, kinds 0 / 1 / 3 / 4 (ITERATIVE / EPNP / DLS / UPNP) sample 5 points for EPnP (other
 * values act as 0); N == model points -> one solve on all points. fp32 reprojection error of
 * projectPoints, inlier iff err <= reprojectionError^2, sequential-RANSAC semantics with seed 0;
 * final pose on the inliers: LM from the RANSAC pose (kind 0), EPnP (every other kind).
 * outInliers (caller: N ints) = RANSAC inlier indices.
 * cvSolvePnP: kinds 2 / 5 need N == 4 (AP3P, the 4th point picks the solution); 1 / 3 / 4:
 * EPnP on all points; 0 (ITERATIVE) and values outside 0..6: EPnP, then LM over all points;
 * 6 (SQPNP, N >= 3): OpenCV's sqpnp::PoseSolver on the undistorted normalised points (computeOmega's
 * sums on the GPU, the SQP search on the host; its assertion failures return false with the reason,
 * no solution in front of the camera returns false). */
MCV_API mcvBool cvSolvePnP(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                        const double* distortionCoeffs, const int solverKind, mcvV3d* tVec, mcvV3d* rVec);
MCV_API mcvBool cvSolvePnPRansac(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                              const double* distortionCoeffs, const int solverKind, const int iterationsCount,
                              const float reprojectionError, const double confidence, mcvV3d* tVec, mcvV3d* rVec,
                              int* inlierCount, int* outInliers);
/* In/out pose (t, r): 20 LM iterations over all points (solvePnPRefineLM) / 20 VVS iterations with
 * lambda 1 on the normalised image plane (solvePnPRefineVVS). */
MCV_API void cvRefinePnPLM(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                           const double* distortionCoeffs, mcvV3d* tVec, mcvV3d* rVec);
MCV_API void cvRefinePnPVVS(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                            const double* distortionCoeffs, mcvV3d* tVec, mcvV3d* rVec);
/* AP3P — ap3p.cpp:282-317, double arguments as the reference defines them and the F# P/Invoke
 * passes them (OpenCV.fs:373-374: F# `float` is System.Double). The reference's quartic path:
 * Ferrari (std::complex) + two Newton polish passes, every root with |cos| <= 1 in its order,
 * complex roots' real parts included. Rs/ts: caller arrays of 4; R as the reference returns it
 * (ap3p.cpp:245-250). Returns the count. */
MCV_API int  solveAp3p(mcvM33d* Rs, mcvV3d* ts, double mu0, double mv0, double X0, double Y0, double Z0,
                       double mu1, double mv1, double X1, double Y1, double Z1,
                       double mu2, double mv2, double X2, double Y2, double Z2,
                       double inv_fx, double inv_fy, double cx_fx, double cy_fy);
/* Fiducials — MiniCVNative.cpp:384-502 (out of scope: return false). */
MCV_API mcvBool cvDetectQRCode(char* data, int width, int height, int channels, int* positions, int* count);
MCV_API mcvBool cvDetectArucoMarkers(char* data, int width, int height, int channels, int* infoCount,
                                  ArucoMarkerInfo* infos);

/* ------------------------------------------------------------------------------------------
 * (2) New hot-path exports (replace the OpenCV calls a maintainer would otherwise add:
 *     cv::findHomography, cv::findFundamentalMat, cv::BFMatcher(NORM_HAMMING / NORM_L2)).
 * ---------------------------------------------------------------------------------------- */

/* method codes (OpenCV numbering) */
#define MCV_METHOD_LSQ     0   /* all points, no RANSAC (OpenCV method 0) */
#define MCV_METHOD_RANSAC  8   /* cv::RANSAC */

/* flags */
#define MCV_FLAG_FIXED_ITERS  1   /* evaluate exactly maxIters hypotheses (no adaptive stop) */
#define MCV_FLAG_NO_REFINE    2   /* return the best hypothesis' model (skip inlier refit + LM) */
#define MCV_FLAG_RETIRED_4    4   /* retired: meant "unfused error" in the round-1 header (now the default);
                                     rejected with an error so an old caller cannot silently get the
                                     opposite definition */
#define MCV_FLAG_SEVEN_POINT  8   /* fundamental only: OpenCV FM_RANSAC's minimal solver (run7Point: 7-point
                                     samples, up to 3 models each, model slots 3h .. 3h+2 in the device
                                     API) instead of the 8-point default; with errorKind EPIPOLAR it is
                                     cv::findFundamentalMat(FM_RANSAC). Needs N >= 15 (OpenCV switches to
                                     LMeDS below that, not provided) or N == 7 (one solve, first model). */
#define MCV_FLAG_CV_SAMPLER   32  /* OpenCV's own sample stream instead of the counter-based Philox one:
                                     cv::RNG((uint64)-1) per call, getSubset's duplicate rejection and
                                     checkSubset, 10000 attempts (RANSACPointSetRegistrator::run), generated
                                     on the host before the GPU evaluates the hypotheses; cfg->seed is then
                                     unused. The default of cvRecoverPose(s) / cvSolvePnPRansac and of the
                                     NULL-config defaults; sequential by definition: <= 2^24 hypotheses */
#define MCV_FLAG_FUSED_ERROR  64  /* opt-in: FMA-contracted inlier error (what a compiler contracting
                                     OpenCV's computeError produces, e.g. clang on arm64). Default:
                                     op-by-op, every operation rounded as written = OpenCV's x86-64
                                     (SSE baseline) build, the reference's Linux/AMD64 target. */
#define MCV_FLAG_FAST_MINIMAL 16  /* opt-in replacement minimal solvers. Essential: Gauss-Jordan null space,
                                     polynomial-product constraints, Illinois real roots (default: the
                                     reference's fivepoint.cpp solver). Homography / 8-point fundamental:
                                     minimal solve by 8x8 Gaussian
                                     elimination with h22 = 1 / f22 = 1 (no eigenvalue check for F).
                                     Default: OpenCV's own runKernel / run8Point, the 9x9 cv::eigen
                                     (JacobiImpl_) of LtL / A^T A. The two agree to ~1e-11 relative; the
                                     default costs ~50x more per hypothesis on the GPU. */

/* F error metric (cfg->errorKind, fundamental only) */
#define MCV_FERR_SAMPSON   0   /* first-order geometric (Sampson) distance^2 (north_star) */
#define MCV_FERR_EPIPOLAR  1   /* OpenCV FM_RANSAC: max of the two squared point-to-epipolar-line distances */

typedef struct {
    double threshold;     /* max reprojection / epipolar distance of an inlier (point units) */
    double confidence;    /* RANSAC confidence in (0,1) */
    int    maxIters;      /* hypothesis budget */
    int    method;        /* MCV_METHOD_* */
    uint64_t seed;        /* counter-based sampler key: hypothesis i depends only on (seed, i) */
    int    deviceCount;   /* 0/1: one GPU; >1 shard hypotheses over that many local GPUs */
    int    flags;         /* MCV_FLAG_* */
    int    errorKind;     /* MCV_FERR_* (fundamental only) */
    int    pnpKind;       /* PnP only: the reference's solverKind (0 ITERATIVE, 1 EPNP, 2 P3P, 3 DLS, 4 UPNP,
                             5 AP3P; others = 0). 2 / 5: AP3P on 4-point sets; else EPnP on 5-point sets.
                             Final pose on the inliers: LM from the RANSAC pose (0), EPnP (1-5). */
} RansacConfig;           /* 48 bytes */

/* findHomography. src/dst: N AoS fp64 points (converted to fp32 like OpenCV's convertTo(CV_32F)).
 * H: out, row-major, H[8] == 1. mask: caller-allocated uint8[N] (RANSAC inliers of the best
 * hypothesis; all 1 for METHOD_LSQ / N == 4). Returns the inlier count (>= 4), 0 on failure. */
MCV_API int cvFindHomography(const mcvV2d* src, const mcvV2d* dst, const int N, const RansacConfig* cfg,
                             mcvM33d* H, uint8_t* mask);

/* findFundamentalMat, 8-point minimal sets. a/b: N AoS fp64 points. F: out, scaled so that F[8] = 1 when
 * |F[8]| > FLT_EPSILON (run8Point's normalisation), otherwise as solved.
 * mask: caller-allocated uint8[N]. Returns inlier count (>= 8), 0 on failure. */
MCV_API int cvFindFundamentalMat(const mcvV2d* a, const mcvV2d* b, const int N, const RansacConfig* cfg,
                                 mcvM33d* F, uint8_t* mask);

/* findEssentialMat (OpenCV focal/pp overload): a/b pixel points, normalised (x - pp) / focal in
 * fp64; five-point minimal sets (<= 10 models per hypothesis), Sampson error, inlier iff
 * err <= (float)(threshold / focal)^2. cfg NULL: threshold 1, confidence 0.999, maxIters 1000,
 * seed 0. E: out, unit Frobenius norm. mask: uint8[N]. Returns the inlier count, 0 on failure.
 * N == 5 runs one solve on all points (mask all 1) and succeeds only with a single solution. */
MCV_API int cvFindEssentialMat(const mcvV2d* a, const mcvV2d* b, const int N, double focal, mcvV2d pp,
                               const RansacConfig* cfg, mcvM33d* E, uint8_t* mask);

/* cvSolvePnPRansac with a full RansacConfig (threshold = reprojection error in pixels; seed, fixed iterations, fused error, NO_REFINE). */
MCV_API mcvBool cvSolvePnPRansacCfg(const mcvV2d* imgPoints, const mcvV3d* worldPoints, const int N, const mcvM33d K,
                                 const double* distortionCoeffs, const RansacConfig* cfg, mcvV3d* tVec, mcvV3d* rVec,
                                 int* inlierCount, int* outInliers);

/* Device-resident match -> RANSAC hand-off. Inputs are the reference's
 * DetectorResult (MiniCVNative.h:23-29: KeyPoint2d[PointCount] + row-major descriptors,
 * DescriptorElementType 0 = uint8 -> Hamming, 5 = float32 -> L2). Matching a -> b (knn 2), then
 * on the GPU: Lowe ratio test (d1 < ratio d2; ratio <= 0: off), mutual-nearest check, max
 * distance (<= 0: off), order-preserving compaction, keypoint gather into the RANSAC layout. */
typedef struct {
    float ratio;
    int   crossCheck;
    float maxDistance;
    int   model;        /* MCV_MODEL_HOMOGRAPHY or MCV_MODEL_FUNDAMENTAL (cvMatchAndFindModel) */
} MatchConfig;          /* 16 bytes */

/* Matches only: pairs[2k] = index in a, pairs[2k+1] = index in b (ascending in a), dist[k]
 * (Hamming distance or L2 distance; may be NULL). Returns the match count, -1 on failure
 * (maxPairs >= a->PointCount is always enough). */
MCV_API int cvMatchFeatures(const DetectorResult* a, const DetectorResult* b, const MatchConfig* cfg, int* pairs,
                            float* dist, int maxPairs);
/* Matches + RANSAC on the matched keypoints (cvFindHomography / cvFindFundamentalMat semantics,
 * cfg->method RANSAC) without leaving the GPU. M: model; pairs as above; mask[k]: inlier flag of
 * match k; *matchCount: number of matches written. Returns the inlier count, 0 on failure. */
MCV_API int cvMatchAndFindModel(const DetectorResult* a, const DetectorResult* b, const MatchConfig* mcfg,
                                const RansacConfig* rcfg, mcvM33d* M, int* pairs, uint8_t* mask, int maxPairs,
                                int* matchCount);

/* Brute-force Hamming matcher (BFMatcher NORM_HAMMING, knn k = 2). q: [nq][bytesPerDesc],
 * t: [nt][bytesPerDesc] row-major bytes; bytesPerDesc in [1, 64]; nt < 2^22.
 * Outputs per query: best train index / distance and second best (idx2/dist2 may be NULL;
 * -1 / INT_MAX when nt < 2). Ties -> lowest train index. Returns nq, or -1 on failure. */
MCV_API int cvMatchHamming(const uint8_t* q, const int nq, const uint8_t* t, const int nt, const int bytesPerDesc,
                           int* idx, int* dist, int* idx2, int* dist2);

/* Brute-force L2 matcher (BFMatcher NORM_L2, knn k = 2) on fp32 descriptors [n][dim].
 * dist = sqrt of the squared distance (fp32). Returns nq, or -1 on failure. */
MCV_API int cvMatchL2(const float* q, const int nq, const float* t, const int nt, const int dim,
                      int* idx, float* dist, int* idx2, float* dist2);

/* Multi-GPU forms of the two matchers (query blocks Nq / D per GPU, train set
 * replicated), for a host that calls one synchronous export from one process like the reference's
 * P/Invoke layer (OpenCV.fs:339-382). The queries are split into deviceCount contiguous blocks (the
 * first nq % deviceCount one query longer), block k runs on visible device (current + k) mod count,
 * the train set is uploaded once and peer-copied over xGMI to the other devices, and every block's
 * outputs land in the caller's arrays at its offset. Results are identical to deviceCount = 1.
 * deviceCount in [1, 16]; the other arguments and the return are cvMatchHamming's / cvMatchL2's. */
MCV_API int cvMatchHammingMulti(const uint8_t* q, const int nq, const uint8_t* t, const int nt,
                                const int bytesPerDesc, const int deviceCount, int* idx, int* dist, int* idx2,
                                int* dist2);
MCV_API int cvMatchL2Multi(const float* q, const int nq, const float* t, const int nt, const int dim,
                           const int deviceCount, int* idx, float* dist, int* idx2, float* dist2);

/* Diagnostics of the exact L2 re-rank: queries the calling thread's last L2 match sent to the exact
 * full scan (near-ties the GEMM form cannot separate); synchronises that match's stream. */
MCV_API int mcvL2LastExactScans(void);
/* GEMM form of the calling thread's last L2 match: 16 = f16 split (every |x| < 2^15, dim <= 128),
 * 32 = f32; synchronises that match's stream. */
MCV_API int mcvL2LastGemmForm(void);

/* Last error message of the calling thread ("" if none). */
MCV_API const char* mcvGetLastError(void);
/* Library / device info: number of visible HIP devices (0 when none), -1 on runtime error. */
MCV_API int mcvDeviceCount(void);
MCV_API const char* mcvVersion(void);
/* ABI revision of this header: 3 (round 3: MCV_FLAG_FUSED_ERROR moved from 4 to 64, bit 4 rejected,
 * MCV_FLAG_CV_SAMPLER added, RansacConfig unchanged at 48 bytes). */
#define MCV_ABI_VERSION 3
MCV_API int mcvAbiVersion(void);

/* CameraPose.findScaled — src/MiniCV/CameraPose.fs:39-134, the managed
 * O(N^2) scale hypothesize-and-verify, moved onto the GPU behind a new export. The F# wrapper keeps
 * its signature `findScaled inlierThreshold srcCam worldObservations pose` and passes the tuple
 * list as two arrays; it builds `scale bestScale pose` itself from *outScale.
 *   candidates: for observation i (list order), the pose scales s = -z / n from the dst0 frame
 *     (CameraPose.fs:103-117), s.X then s.Y; skipped when |n.X| or |n.Y| < 1e-5 (Fun.IsTiny);
 *   cost(s) = avgReprojectionError s (CameraPose.fs:71-87): mean of |project1 dstCam(s) w - obs|^2
 *     over the observations visible in dstCam(s) (Camera.fs:72-83), +inf if none;
 *   selection: first strictly smaller cost wins (CameraPose.fs:119-125).
 * inlierThreshold is accepted and unused, as in the reference (only the dead countInliers uses it).
 * Writes *outCost = best cost (+inf when no candidate improves on +inf) and *outScale = its scale
 * (0 then). Returns the number of candidate scales evaluated (2 per non-tiny observation), -1 on
 * failure. N == 0 returns 0 with *outCost = +inf, *outScale = 0 (the reference's empty-list case). */
typedef struct {             /* Camera.fs:7-14, F# record field order: 13 doubles */
    mcvV3d location;
    mcvV3d forward;
    mcvV3d up;
    mcvV3d right;
    mcvV2d focal;
} mcvCamera;
MCV_API int cvFindScaledPose(double inlierThreshold, const mcvCamera* srcCam, const mcvV3d* worldPoints,
                             const mcvV2d* observations, int N, const mcvM33d* rotation, const mcvV3d* translation,
                             double* outCost, double* outScale);
/* Per-candidate costs of cvFindScaledPose (test / analysis helper): scales[2N] and costs[2N] in
 * candidate order (slot 2i = s.X, 2i+1 = s.Y of observation i; a skipped observation has NaN scales
 * and +inf costs). Returns N, -1 on failure. */
MCV_API int cvFindScaledPoseCosts(const mcvCamera* srcCam, const mcvV3d* worldPoints, const mcvV2d* observations,
                                  int N, const mcvM33d* rotation, const mcvV3d* translation, double* scales,
                                  double* costs);

/* ------------------------------------------------------------------------------------------
 * (3) Device-level API: device pointers, caller's stream (hipStream_t as void*), current device.
 *     Points on device are packed fp32 correspondences float4 {x, y, x', y'} (16 B each).
 * ---------------------------------------------------------------------------------------- */

typedef struct mcvRansacPlan_ mcvRansacPlan;

#define MCV_MODEL_HOMOGRAPHY   0
#define MCV_MODEL_FUNDAMENTAL  1
#define MCV_MODEL_ESSENTIAL    2   /* points: double4 {x1, y1, x2, y2} normalised (mcvPackEssential);
                                      hypothesis h owns model slots 10h .. 10h+9: keys, counts and
                                      indices below are slot indices for this model */
#define MCV_MODEL_PNP          3   /* points: PnpPoint {X, Y, Z, u, v, pad[3]} fp32 (mcvPackPnP); camera
                                      via mcvRansacPlanSetCamera; threshold in pixels; cfg->pnpKind
                                      picks the minimal solver; finalize writes model9 = {rvec[3],
                                      tvec[3], 0, 0, 0}, the inlier solve of cfg->pnpKind unless
                                      MCV_FLAG_NO_REFINE */

/* Workspace for problems up to maxN correspondences and maxHyps hypotheses per evaluate call. */
MCV_API mcvRansacPlan* mcvRansacPlanCreate(int model, int maxN, int64_t maxHyps);
MCV_API void mcvRansacPlanDestroy(mcvRansacPlan* plan);

/* Pack host AoS fp64 pairs into the device float4 layout (synchronous H2D on `stream`). */
MCV_API int mcvPackCorrespondences(const mcvV2d* a, const mcvV2d* b, int N, float* d_pts4, void* stream);
/* PnP model: upload image V2d[N] + world V3d[N] and pack them on the device (32 B each). */
MCV_API int mcvPackPnP(const mcvV2d* img, const mcvV3d* world, int N, void* d_pts, void* stream);
/* PnP plans: camera matrix (row-major 3x3; fx = K[0], fy = K[4], cx = K[2], cy = K[5]) and
 * distortion (k1, k2, p1, p2; NULL = none). */
MCV_API int mcvRansacPlanSetCamera(mcvRansacPlan* plan, const double* K9, const double* dist4);
/* Essential model: upload host pairs and normalise on the device into double4 (32 B each). */
MCV_API int mcvPackEssential(const mcvV2d* a, const mcvV2d* b, int N, double focal, mcvV2d pp, double* d_pts4,
                             void* stream);

/* Evaluate hypotheses [hypBegin, hypBegin + hypCount) against all N correspondences:
 * sample + minimal solve + inlier count, then reduce to the best packed key
 *   key = (count << 32) | (0xFFFFFFFF - hypIndex)     (0 when no hypothesis has >= m inliers)
 * written to d_key[0]; d_key[1] = first hypothesis index whose sampler failed (or INT64 max).
 * d_counts (optional, may be NULL): per-hypothesis status/count (int32, -1 no model, -2 no sample).
 * Asynchronous on `stream`, except with MCV_FLAG_CV_SAMPLER: OpenCV's subset stream is generated on
 * the host, so the call synchronises `stream` (to check the plan's table against N and the points'
 * fingerprint, and to rebuild it when hypBegin == 0 or either differs). The plan fingerprints the
 * points of every evaluated chunk; mcvRansacFinalize re-solves the winner when the buffer's content
 * changed since (a rewrite in place, same pointer and N). Returns 1 on successful launch, 0 on error. */
MCV_API int mcvRansacEvaluate(mcvRansacPlan* plan, const void* d_pts4, int N, const RansacConfig* cfg,
                              int64_t hypBegin, int64_t hypCount, uint64_t* d_key, int* d_counts, void* stream);

/* Recompute the best hypothesis' model (hypIndex), write the inlier mask (d_mask, uint8[N]),
 * optionally refit on the inliers + LM refine (per cfg->flags), model out to host `model9`.
 * Synchronises `stream`. Returns the inlier count, 0 on failure. */
MCV_API int mcvRansacFinalize(mcvRansacPlan* plan, const void* d_pts4, int N, const RansacConfig* cfg,
                              int64_t hypIndex, double* model9, uint8_t* d_mask, void* stream);

/* Sequential-RANSAC replay over per-hypothesis counts (host arrays), OpenCV semantics:
 * improvement iff count > max(best, m-1); niters <- RANSACUpdateNumIters(conf, 1-count/N, m, niters);
 * loop stops at iter >= niters or at the first sampler failure. State carried across chunks.
 * Returns 1 when the replay stopped inside this chunk (no more hypotheses needed), else 0. */
typedef struct {
    int64_t niters;      /* current iteration budget */
    int64_t bestIndex;   /* -1 if none */
    int32_t bestCount;
    int32_t stopped;
} mcvReplayState;
MCV_API void mcvReplayInit(mcvReplayState* st, int maxIters);
MCV_API int  mcvReplayChunk(mcvReplayState* st, const int* counts, int64_t hypBegin, int64_t hypCount,
                            int N, int modelPoints, double confidence, int fixedIters);
/* Multi-model hypotheses (essential: slotsPerHyp = 10): counts[h * slotsPerHyp + s], -2 at slot 0 =
 * sampler failure, -1 = no model; models of one hypothesis are tried in slot order, niters is
 * checked per hypothesis (RANSACPointSetRegistrator::run). bestIndex is the slot index. */
MCV_API int  mcvReplayChunkModels(mcvReplayState* st, const int* counts, int64_t hypBegin, int64_t hypCount,
                                  int slotsPerHyp, int N, int modelPoints, double confidence, int fixedIters);

/* Device-level matchers: d_q/d_t device arrays, outputs device arrays. Asynchronous on stream. */
MCV_API int mcvMatchHammingDevice(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int bytesPerDesc,
                                  int* d_idx, int* d_dist, int* d_idx2, int* d_dist2, void* stream);
/* The same with the kernel form chosen explicitly: 0 = fp4 GEMM on the matrix cores (the default of
 * every other Hamming entry point), 1 = the XOR / popcount sweep. Identical results. */
MCV_API int mcvMatchHammingDeviceForm(const uint8_t* d_q, int nq, const uint8_t* d_t, int nt, int bytesPerDesc,
                                      int* d_idx, int* d_dist, int* d_idx2, int* d_dist2, int form, void* stream);
MCV_API int mcvMatchL2Device(const float* d_q, int nq, const float* d_t, int nt, int dim,
                             int* d_idx, float* d_dist, int* d_idx2, float* d_dist2, void* stream);

/* Device-level CameraPose.findScaled: d_world V3d[N], d_obs V2d[N] on the device. Synchronises
 * `stream`; same outputs and return value as cvFindScaledPose. */
MCV_API int mcvFindScaledPoseDevice(const mcvCamera* srcCam, const mcvV3d* d_world, const mcvV2d* d_obs, int N,
                                    const mcvM33d* rotation, const mcvV3d* translation, double* outCost,
                                    double* outScale, void* stream);

/* Opt-in kernel timing: HIP events recorded around the inlier-sweep launches on their stream.
 * mcvProfileRead returns the number of launches of `kernel` ("h_verify", "f_verify") and their
 * summed duration in ms (synchronises the recorded events). */
MCV_API void mcvProfileEnable(int on);
MCV_API void mcvProfileReset(void);
MCV_API int  mcvProfileRead(const char* kernel, double* total_ms);

/* ------------------------------------------------------------------------------------------
 * Test hooks: the host-compiled copy of the per-hypothesis code that the kernels run
 * (sampler + subset check + minimal solver + error), so CPU tests can check it against the
 * oracle bit for bit without a GPU. Never on a product path.
 * ---------------------------------------------------------------------------------------- */
#define MCV_HOST_FAST_MINIMAL 0x100   /* or-ed into mcvHostHypothesis' model: the elimination solver */
MCV_API int mcvHostHypothesis(int model, const float* pts4, int N, uint64_t seed, int64_t hyp,
                              double* model9, float* modelf9, int* sampleIdx);
/* Device self-test: number of 32-bit patterns w where a reciprocal differs from 1.f/w (mode 0 =
 * rcp_exact; 1 = rcp_newton everywhere; 2 = rcp_newton + v_div_fixup; 3 = rcp_newton on its domain
 * |w| in [2^-126, 2^126) only; 4 = raw v_rcp_f32; 5 = rcp_exact_bounded on |w| < 2^126 and NaN). */
MCV_API long long mcvTestRcpExhaustive(int mode, uint32_t* firstMismatches16);
/* Device self-test: number of sampled (n, d), d in +-[2^-64, 2^64], where the unscaled fp64
 * division (rcp_f64_refined + div_f64_refined) differs from n / d (mode 0: 2^-900 <= |n| < 2^700;
 * 1: n = 1; 2: n = k d, |k| <= 1000; 3: d at the domain ends); first 16 (n, d) pairs returned.
 * Mode 4: sampled x in [1, 2] where the rotation's unscaled sqrt_f64_1to2 differs from sqrt (pairs (x, 0)). */
MCV_API long long mcvTestDivF64(int mode, unsigned long long seed, long long count, double* firstMismatches32);
/* Device self-test: run the homography inlier sweep on caller-supplied fp32 models (8 floats each);
 * fused: 0 = op-by-op error (scalar sweep), 1 = fused (scalar sweep), 2 = fused through the packed-f32
 * sweep, 3 = op-by-op through the certified division-free sweep (the default path). */
MCV_API int mcvTestHomographySweep(const float* pts4, int N, const float* models8, int nModels, float thr2, int fused,
                                   int* counts);
/* Host twins of the essential path: hypothesis (double4 normalised points; E90 = 10 x 9; the reference's
 * solver, as the default GPU path) and the raw five-point solves (x1[5], y1[5], x2[5], y2[5] packed in
 * p20): mcvHostFivePoint = the opt-in replacement solver, mcvHostFivePointRef = the reference's.
 * Return the model count / status. */
MCV_API int mcvHostEssential(const double* pts4, int N, uint64_t seed, int64_t hyp, double* E90, int* sampleIdx);
/* mcvHostEssential with the opt-in replacement solver (MCV_FLAG_FAST_MINIMAL). */
MCV_API int mcvHostEssentialFast(const double* pts4, int N, uint64_t seed, int64_t hyp, double* E90, int* sampleIdx);
MCV_API int mcvHostFivePoint(const double* p20, double* E90);
/* Host build of the cvFivePoint export's own path (e_solve5_ref), same packing as mcvHostFivePoint. */
MCV_API int mcvHostFivePointRef(const double* p20, double* E90);
/* Host twin of one 7-point fundamental hypothesis (MCV_FLAG_SEVEN_POINT): F27 = up to 3 models,
 * idx7 = the accepted sample (may be NULL). Returns the model count or the kStatus code. */
MCV_API int mcvHostF7(const float* pts4, int N, uint64_t seed, int64_t hyp, double* F27, int* idx7);
MCV_API void mcvHostDecomposeEssential(const double* E9, double* R1, double* R2, double* t3);
/* Host twin of the real-root finder (Rolle brackets + Illinois) of sum c[k] x^k, deg <= 10;
 * fixed = 1 (deg == 4 only) runs the register-resident fixed-size form the AP3P quartic uses.
 * Writes the ascending roots, returns their count (-1 on bad arguments). */
MCV_API int mcvHostRealRoots(const double* c, int deg, int fixed, double* roots);
/* Host twins of the PnP path: one hypothesis on packed PnpPoint[N] (cam8 = fx, fy, cx, cy, k1, k2,
 * p1, p2), and the Rodrigues maps used by the LM refit. */
MCV_API int mcvHostPnP(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R9, double* t3,
                       int* idx4);
/* mcvHostPnP with the opt-in real-root-finder AP3P quartic (MCV_FLAG_FAST_MINIMAL). */
MCV_API int mcvHostPnPFast(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R9,
                           double* t3, int* idx4);
/* EPnP twins: a 5-point EPnP hypothesis (idx5: the sample), and epnp_solve_small<5> on given world
 * points pw15 (5 x 3) and pixel observations us10 (5 x 2), cam4 = fu, fv, uc, vc. */
MCV_API int mcvHostPnPEpnp(const void* pts, int N, const double* cam8, uint64_t seed, int64_t hyp, double* R9,
                           double* t3, int* idx5);
MCV_API void mcvHostEpnp5(const double* pw15, const double* us10, const double* cam4, double* R9, double* t3);
/* Device self-test: the PnP generate kernel's poses for hypotheses [hypBegin, hypBegin + hypCount) on
 * host PnpPoint[N] (kind: solverKind, EPnP kernel unless 2 / 5; | MCV_HOST_FAST_MINIMAL: the opt-in
 * real-root-finder AP3P quartic). poses12[h] = {R (9), t (3)},
 * status[h] = 1 or -1 / -2. Returns hypCount, -1 on failure. */
MCV_API int mcvTestPnpHypotheses(const float* pts, int N, const double* cam8, uint64_t seed, int64_t hypBegin,
                                 int hypCount, int kind, double* poses12, int* status);
/* Device self-test: the PnP inlier sweep on caller-supplied poses (poses12[h] = {R (9), t (3)}) over
 * host PnpPoint[N]; mode 0 = the certified packed-fp32 sweep (the default path), 1 = the all-fp64
 * sweep. counts[h] = inliers. Returns nPoses, -1 on failure. */
MCV_API int mcvTestPnpSweep(const float* pts, int N, const double* cam8, const double* poses12, int nPoses,
                            float thr2, int fused, int mode, int* counts);
/* Host twin of the certified PnP prefilter (pnp_pk.h) for one pose over host PnpPoint[N]: decision[i]
 * = 1 certified inlier, 0 certified outlier, -1 undecided; exact[i] = the fp64 test (pnp_error).
 * fused: bit 0 = the FMA-contracted error; bit 1 = the cheap tier alone (default: the cheap tier, then
 * the exact per-lane bound for what it leaves undecided: MCV_PNP_TIERS=2's order; the default sweep
 * runs the exact bound alone, whose decisions are a superset of the cheap tier's on its domain).
 * Returns the number of decided points whose decision differs from the exact test (must be 0). */
MCV_API int mcvHostPnpCert(const float* pts, int N, const double* cam8, const double* R9, const double* t3,
                           float thr2, int fused, int* decision, int* exact);
/* Host twin of the certified Sampson prefilter (sampson_pk.h) for one fp64 model F9 over host float4
 * points {x1, y1, x2, y2}: decision[i] = 1 certified inlier, 0 certified outlier, -1 undecided; exact[i]
 * = the fp64 Sampson test (kind 0 fused, 1 op-by-op). Returns the number of decided points whose decision
 * differs from the exact test (must be 0). */
MCV_API int mcvHostSampsonCert(const float* pts4, int N, const double* F9, float thr2, int kind, int* decision,
                               int* exact);
/* Host build of solveAp3p's computation (mu3 / mv3 pixels, W9 = 3 world points), R36 / t12 out. */
MCV_API int mcvHostSolveAp3p(const double* mu3, const double* mv3, const double* W9, double inv_fx, double inv_fy,
                             double cx_fx, double cy_fy, double* R36, double* t12);
/* Host twin of cvSolvePnP kind 6 (SQPnP) on double img (N x 2) / world (N x 3), cam8 as above: the
 * computeOmega sums in the device passes' block order, then the same host solve. R9 / t3 = the first
 * solution; returns the solution count, 0 (none), or -1 / -2 / -3 (computeOmega's assertions). */
MCV_API int mcvHostSqpnp(const double* img, const double* world, int N, const double* cam8, double* R9, double* t3);
MCV_API void mcvHostRodrigues(const double* r, double* R, double* dR27);
MCV_API void mcvHostRodriguesInv(const double* R, double* r);
/* OpenCV's sample stream (MCV_FLAG_CV_SAMPLER) on the host: rows [0, rows) of m indices each for the
 * model family (homography / fundamental: pts4 = the float4 points their checkSubset reads; essential /
 * PnP: no check, pts4 may be NULL). Rows from the first failed getSubset on are -1. Returns the number
 * of accepted rows, -1 on bad arguments. */
MCV_API int64_t mcvCvSubsets(int model, int m, const float* pts4, int N, int64_t rows, int* out);
/* glibc_math.h's restatements over arrays: fn 0 cbrt(a), 1 hypot(a, b), 2 the real part of clog(a + i b),
 * 3 a^2 + b^2 - 1 (glibc's __x2y2m1), 4 exp(a), 5 log(a), 6 log1p(a), 7 cos(a), 8 atan2(a, b) — glibc
 * 2.35's x86_64 (FMA multiarch) code paths, restated so the device computes AP3P's complex cube root
 * bit-identically to the reference's std::pow. Returns n, -1 on bad arguments. */
MCV_API int mcvHostGlibcMath(int fn, const double* a, const double* b, int n, double* out);
/* The plan guards' fingerprint (mcv_common.h fp_term summed over the 32-bit words) of a host buffer:
 * the device kernel gives the same value for the same bytes. */
MCV_API uint64_t mcvHostFingerprint(const void* buf, size_t bytes);
/* The device kernel's fingerprint of a device buffer into d_out[0] (synchronous). Returns 1, 0 on error. */
MCV_API int mcvTestFingerprint(const void* d_buf, size_t bytes, uint64_t* d_out);
/* Round 6: the homography generate's split eigen-solve logs at most `cap` rotations per hypothesis
 * (default and maximum 192; a cfg3 LtL takes 110-157); a hypothesis needing more is solved again by
 * the one-pass kernel. Lowering the cap sends lanes down that path (tests). Returns the previous cap. */
MCV_API int mcvTestEigLogCap(int cap);
MCV_API void mcvHostPhilox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                           uint32_t* out4);
/* Host twin of CameraPose.findScaled: the same candidates and costs as cvFindScaledPoseCosts,
 * computed by the host-compiled kernel code with the reference's sequential sums (list order). */
MCV_API int mcvHostScaledCosts(const mcvCamera* srcCam, const mcvV3d* worldPoints, const mcvV2d* observations, int N,
                               const mcvM33d* rotation, const mcvV3d* translation, double* scales, double* costs);

#ifdef __cplusplus
}
#endif

#endif /* MINICV_NATIVE_H */
