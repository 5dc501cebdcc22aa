// hyp_scaled.h — CameraPose.findScaled (src/MiniCV/CameraPose.fs:39-134) restated for the GPU:
// the per-candidate destination camera and the per-observation reprojection term of
// avgReprojectionError (CameraPose.fs:71-87), compiled for gfx950 (kernels) and x86-64 (host
// setup + the mcvHostScaledCosts twin). Every expression is written in the evaluation order of
// the managed code (C#/F# left-to-right, no FMA contraction: files are built -ffp-contract=off),
// so a term computed here is bit-identical on the host and on the GPU.
//
// Aardvark.Base semantics restated [ext: Aardvark.Base, not in /root/reference, unverifiable
// here]: M44d.FromBasis(x, y, z, o) has columns x, y, z, o; TransformPos(p) = M (p, 1) without
// a perspective divide, TransformDir(v) = M3x3 v, each row summed left to right; M33d * V3d
// row-wise left to right; Vec.normalize(v) = v * (1 / |v|) (zero vector -> zero); V2d / s
// divides each component; Fun.IsTiny(x, e) = |x| < e.
#pragma once

#include "mcv_common.h"

namespace mcv {

// Everything of a findScaled call that does not depend on the candidate scale s. Host-built
// (scaled_pose_host.cpp) from srcCam, pose.Rotation R and pose.Translation T.
struct ScaledSetup {
    double tw[3][4];    // rows of toWorld = M44d.FromBasis(right, up, -forward, location)  (Camera.fs:62)
    double rot[3][3];   // toRotWorld = toWorld * transformation(pose) 3x3 part             (Camera.fs:63)
    double R[3][3], T[3];
    double right[3], up[3], fwd[3];   // dstCam(s) axes: independent of s (Camera.fs:66-68)
    double fx, fy;                    // focal (unchanged by transformedView, Camera.fs:69)
    double minv[3][4];  // dst0View.Forward rows (CameraPose.fs:48-49)
    double t[3];        // dst0Translation (CameraPose.fs:57-61)
};

// location of dstCam(s) = transformedView (transformation (scale s pose)) srcCam
// (CameraPose.fs:31-37 scale / transformation, Camera.fs:60-70): toRotWorld.TransformPos(V3d.Zero).
MCV_HD void scaled_location(const ScaledSetup& S, double s, double (&loc)[3]) {
    const double st0 = s * S.T[0], st1 = s * S.T[1], st2 = s * S.T[2];   // f * pose.Translation
    double rt[3];                                                          // m * pose.Translation
    for (int i = 0; i < 3; ++i) rt[i] = S.R[i][0] * st0 + S.R[i][1] * st1 + S.R[i][2] * st2;
    for (int i = 0; i < 3; ++i) {
        // toRotWorld[i][3] = sum_k toWorld[i][k] * T[k][3], T[3][3] = 1
        const double m3 = S.tw[i][0] * rt[0] + S.tw[i][1] * rt[1] + S.tw[i][2] * rt[2] + S.tw[i][3] * 1.0;
        loc[i] = S.rot[i][0] * 0.0 + S.rot[i][1] * 0.0 + S.rot[i][2] * 0.0 + m3;   // TransformPos(V3d.Zero)
    }
}

// One observation against dstCam(s): Camera.project1 (Camera.fs:72-83) and the squared distance
// to the observation (CameraPose.fs:80-82). Returns false when the point is not visible; err is
// computed either way (no branch: the caller selects it), meaningful only when visible.
MCV_HD bool scaled_term(const ScaledSetup& S, const double (&loc)[3], double wx, double wy, double wz, double ox,
                        double oy, double& err) {
    const double o0 = wx - loc[0], o1 = wy - loc[1], o2 = wz - loc[2];
    const double p0 = o0 * S.right[0] + o1 * S.right[1] + o2 * S.right[2];
    const double p1 = o0 * S.up[0] + o1 * S.up[1] + o2 * S.up[2];
    const double p2 = o0 * S.fwd[0] + o1 * S.fwd[1] + o2 * S.fwd[2];
#if defined(__HIP_DEVICE_COMPILE__)
    // Both quotients share one refined reciprocal (mcv_common.h): equal to the IEEE divisions for
    // p2 in [2^-64, 2^64] and every numerator whose quotient can be visible (|c| <= 1); a numerator
    // below 2^-900 gives |c| < 2^-836 either way, and c - o then rounds identically (to -o, or to
    // a value whose square is +0). A visible p2 outside that range takes the IEEE divisions.
    const double rp2 = rcp_f64_refined(p2);
    double cx = div_f64_refined(S.fx * p0, p2, rp2), cy = div_f64_refined(S.fy * p1, p2, rp2);
    if (p2 >= 0.0 && !div_f64_refined_domain(p2)) {
        cx = S.fx * p0 / p2;
        cy = S.fy * p1 / p2;
    }
#else
    const double cx = S.fx * p0 / p2, cy = S.fy * p1 / p2;
#endif
    const double dx = cx - ox, dy = cy - oy;
    err = dx * dx + dy * dy;
    return p2 >= 0.0 && cx >= -1.0 && cy >= -1.0 && cx <= 1.0 && cy <= 1.0;
}

// Candidate scales of observation (w, obs) (CameraPose.fs:103-117). Returns false when the
// observation is skipped (IsTiny(n.X, 1e-5) || IsTiny(n.Y, 1e-5)).
MCV_HD bool scaled_candidate(const ScaledSetup& S, double wx, double wy, double wz, double ox, double oy,
                             double& sx, double& sy) {
    double p[3];
    for (int i = 0; i < 3; ++i) p[i] = S.minv[i][0] * wx + S.minv[i][1] * wy + S.minv[i][2] * wz + S.minv[i][3];
    const double zx = ox * p[2] - p[0], zy = oy * p[2] - p[1];       // obs * point.Z - point.XY
    const double nx = S.t[0] - ox * S.t[2], ny = S.t[1] - oy * S.t[2];   // t.XY - obs * t.Z
    if (fabs(nx) < 1e-5 || fabs(ny) < 1e-5) return false;
    sx = -zx / nx;
    sy = -zy / ny;
    return true;
}

}  // namespace mcv
