// Device math for the BA kernels (gfx950, float64 throughout like the reference, bundle_adjustment.py:73,83,98).
//
// Camera rows follow TorchBA's packing (bundle_adjustment.py:70-80): [t(3), q_xyzw(4), intrinsics-without-pp].
// Projection restates cost_function.py:32-177 per model; the pose action restates bae.utils.ba.rotate_quat
// (un-vendored) as p_c = p + 2w (qv x p) + 2 qv x (qv x p) + t.  Jacobians are analytic:
// pose tangent is pypose se3 [rho, phi] under left perturbation X <- Exp(d) X (dp_c/drho = I, dp_c/dphi = -[p_c]x).
#pragma once
#include <hip/hip_runtime.h>

namespace insfm {

// Number of intrinsics after the principal point is removed, and of focal lengths, per CameraModelId.
template <int M> struct Model;
template <> struct Model<0> { static constexpr int NI = 1, NF = 1; };   // SIMPLE_PINHOLE  [f]
template <> struct Model<1> { static constexpr int NI = 2, NF = 2; };   // PINHOLE         [fx, fy]
template <> struct Model<2> { static constexpr int NI = 2, NF = 1; };   // SIMPLE_RADIAL   [f, k]
template <> struct Model<3> { static constexpr int NI = 3, NF = 1; };   // RADIAL          [f, k1, k2]
template <> struct Model<4> { static constexpr int NI = 6, NF = 2; };   // OPENCV          [fx, fy, k1, k2, p1, p2]
template <> struct Model<5> { static constexpr int NI = 6, NF = 2; };   // OPENCV_FISHEYE  [fx, fy, k1, k2, k3, k4]
template <> struct Model<6> { static constexpr int NI = 10, NF = 2; };  // FULL_OPENCV     [fx, fy, k1, k2, p1, p2, k3..k6]
template <> struct Model<8> { static constexpr int NI = 2, NF = 1; };   // SIMPLE_RADIAL_FISHEYE [f, k]
template <> struct Model<9> { static constexpr int NI = 3, NF = 1; };   // RADIAL_FISHEYE  [f, k1, k2]

// Global positioning (TorchGP, global_positioning.py:45-206): the "camera" is its position c (3 values), no rotation
// or intrinsics; kernels that depend on the camera parametrization specialise on this id.
constexpr int kGP = 100;
template <> struct Model<kGP> { static constexpr int NI = 0, NF = 0; };

template <int M> constexpr int kD = M == kGP ? 3 : 6 + Model<M>::NI;       // camera block dimension
template <int M> constexpr int kStride = M == kGP ? 3 : 7 + Model<M>::NI;  // stored camera row

// atan(r)/r and d/dr2 (series near 0 for the derivative; value as the reference computes it).
__device__ __forceinline__ void fisheye_g(double r2, double& g, double& dg) {
    if (r2 == 0.0) { g = 1.0; dg = -1.0 / 3.0; return; }
    const double r = sqrt(r2);
    g = atan(r) / r;
    if (r2 < 1e-3) {
        double s = 0.0, pw = 1.0;
#pragma unroll
        for (int n = 1; n <= 8; ++n) { s += ((n & 1) ? -1.0 : 1.0) * n * pw / (2 * n + 1); pw *= r2; }
        dg = s;
    } else {
        dg = (1.0 / (1.0 + r2) - g) / (2.0 * r2);
    }
}

// Distortion of normalized coordinates for model M.  k points at the distortion params (after the focal(s)).
// Outputs distorted (du, dv), Jd = d(du,dv)/d(u,v) row-major 2x2, Jk[2][NK] = d(du,dv)/dk.
template <int M>
__device__ __forceinline__ void distort(const double* k, double u, double v, double& du, double& dv, double Jd[4],
                                        double (*Jk)[(Model<M>::NI - Model<M>::NF) > 0 ? (Model<M>::NI - Model<M>::NF) : 1]) {
    constexpr int NK = Model<M>::NI - Model<M>::NF;
    const double r2 = u * u + v * v;
    if constexpr (M == 0 || M == 1) {
        du = u; dv = v; Jd[0] = 1.0; Jd[1] = 0.0; Jd[2] = 0.0; Jd[3] = 1.0;
    } else if constexpr (M == 4 || M == 6) {
        const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3];
        double rad, radp;
        double dr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if constexpr (M == 4) {
            rad = k1 * r2 + k2 * r2 * r2;
            radp = k1 + 2.0 * k2 * r2;
            dr[0] = r2; dr[1] = r2 * r2;
        } else {
            const double k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
            const double r4 = r2 * r2, r6 = r4 * r2;
            const double Nn = 1.0 + k1 * r2 + k2 * r4 + k3 * r6, Dn = 1.0 + k4 * r2 + k5 * r4 + k6 * r6;
            rad = Nn / Dn - 1.0;
            const double Np = k1 + 2.0 * k2 * r2 + 3.0 * k3 * r4, Dp = k4 + 2.0 * k5 * r2 + 3.0 * k6 * r4;
            const double iD2 = 1.0 / (Dn * Dn);
            radp = (Np * Dn - Nn * Dp) * iD2;
            dr[0] = r2 / Dn; dr[1] = r4 / Dn; dr[4] = r6 / Dn;
            dr[5] = -Nn * r2 * iD2; dr[6] = -Nn * r4 * iD2; dr[7] = -Nn * r6 * iD2;
        }
        const double uv = u * v;
        du = u + u * rad + 2.0 * p1 * uv + p2 * (r2 + 2.0 * u * u);
        dv = v + v * rad + 2.0 * p2 * uv + p1 * (r2 + 2.0 * v * v);
        Jd[0] = 1.0 + rad + 2.0 * u * u * radp + 2.0 * p1 * v + 6.0 * p2 * u;
        Jd[1] = 2.0 * uv * radp + 2.0 * p1 * u + 2.0 * p2 * v;
        Jd[2] = 2.0 * uv * radp + 2.0 * p2 * v + 2.0 * p1 * u;
        Jd[3] = 1.0 + rad + 2.0 * v * v * radp + 2.0 * p2 * u + 6.0 * p1 * v;
#pragma unroll
        for (int j = 0; j < NK; ++j) {
            const bool radial = (j < 2) || (j >= 4);
            Jk[0][j] = radial ? u * dr[j] : 0.0;
            Jk[1][j] = radial ? v * dr[j] : 0.0;
        }
        Jk[0][2] = 2.0 * uv;            Jk[1][2] = r2 + 2.0 * v * v;   // p1
        Jk[0][3] = r2 + 2.0 * u * u;    Jk[1][3] = 2.0 * uv;           // p2
    } else {
        // radial-h family: (du, dv) = h(r2) (u, v)
        double h, hp;
        double dh[NK];
        if constexpr (M == 2) {
            h = 1.0 + k[0] * r2; hp = k[0]; dh[0] = r2;
        } else if constexpr (M == 3) {
            h = 1.0 + k[0] * r2 + k[1] * r2 * r2; hp = k[0] + 2.0 * k[1] * r2; dh[0] = r2; dh[1] = r2 * r2;
        } else {
            double g, gp, P, Pp;
            fisheye_g(r2, g, gp);
            if constexpr (M == 5) {
                P = 1.0 + k[0] * r2 + k[1] * r2 * r2 + k[2] * r2 * r2 * r2;
                Pp = k[0] + 2.0 * k[1] * r2 + 3.0 * k[2] * r2 * r2;
                dh[0] = g * r2; dh[1] = g * r2 * r2; dh[2] = g * r2 * r2 * r2; dh[3] = 0.0;  // k4 ignored (cost_function.py:95)
            } else if constexpr (M == 8) {
                P = 1.0 + k[0] * r2; Pp = k[0]; dh[0] = g * r2;
            } else {
                P = 1.0 + k[0] * r2 + k[1] * r2 * r2; Pp = k[0] + 2.0 * k[1] * r2; dh[0] = g * r2; dh[1] = g * r2 * r2;
            }
            h = g * P; hp = gp * P + g * Pp;
        }
        du = u * h; dv = v * h;
        Jd[0] = h + 2.0 * u * u * hp; Jd[1] = 2.0 * u * v * hp;
        Jd[2] = 2.0 * u * v * hp;     Jd[3] = h + 2.0 * v * v * hp;
#pragma unroll
        for (int j = 0; j < NK; ++j) { Jk[0][j] = u * dh[j]; Jk[1][j] = v * dh[j]; }
    }
}

// Residual (projection - uv) and optionally the analytic Jacobians of one observation.
// cam: kStride<M> doubles; Jc[2][D]: pose [rho(3), phi(3)] then intrinsics; Jp[2][3].
template <int M, bool WANT_J>
__device__ __forceinline__ void eval_obs(const double* __restrict__ cam, const double X[3], const double pp[2],
                                         const double uvobs[2], double r[2], double (*Jc)[kD<M>], double (*Jp)[3]) {
    constexpr int NF = Model<M>::NF;
    constexpr int NK = Model<M>::NI - NF;
    constexpr int D = kD<M>;
    const double tx = cam[0], ty = cam[1], tz = cam[2];
    const double qx = cam[3], qy = cam[4], qz = cam[5], qw = cam[6];
    const double c1x = qy * X[2] - qz * X[1], c1y = qz * X[0] - qx * X[2], c1z = qx * X[1] - qy * X[0];
    const double c2x = qy * c1z - qz * c1y, c2y = qz * c1x - qx * c1z, c2z = qx * c1y - qy * c1x;
    const double px = X[0] + 2.0 * (qw * c1x + c2x) + tx;
    const double py = X[1] + 2.0 * (qw * c1y + c2y) + ty;
    const double pz = X[2] + 2.0 * (qw * c1z + c2z) + tz;
    const double iz = 1.0 / pz;
    const double u = px * iz, v = py * iz;
    double du, dv, Jd[4];
    double Jk[2][NK > 0 ? NK : 1];
    distort<M>(cam + 7 + NF, u, v, du, dv, Jd, Jk);
    const double fx = cam[7];
    const double fy = (NF == 2) ? cam[8] : cam[7];
    r[0] = fx * du + pp[0] - uvobs[0];
    r[1] = fy * dv + pp[1] - uvobs[1];
    if constexpr (WANT_J) {
        // A = diag(f) Jd d(u,v)/dp_c  (2x3)
        const double duv0[3] = {iz, 0.0, -u * iz};
        const double duv1[3] = {0.0, iz, -v * iz};
        double A[2][3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            A[0][c] = fx * (Jd[0] * duv0[c] + Jd[1] * duv1[c]);
            A[1][c] = fy * (Jd[2] * duv0[c] + Jd[3] * duv1[c]);
        }
        // dp_c/dX = M = I + 2w[q]x + 2[q]x[q]x
        const double K[3][3] = {{0.0, -qz, qy}, {qz, 0.0, -qx}, {-qy, qx, 0.0}};
        double Mq[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
                Mq[i][j] = (i == j ? 1.0 : 0.0) + 2.0 * qw * K[i][j] + 2.0 * kk;
            }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int j = 0; j < 3; ++j) Jp[a][j] = A[a][0] * Mq[0][j] + A[a][1] * Mq[1][j] + A[a][2] * Mq[2][j];
        // pose: rho -> A ; phi_k -> A (e_k x p_c)
        const double ex[3][3] = {{0.0, -pz, py}, {pz, 0.0, -px}, {-py, px, 0.0}};
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            Jc[a][0] = A[a][0]; Jc[a][1] = A[a][1]; Jc[a][2] = A[a][2];
#pragma unroll
            for (int kk = 0; kk < 3; ++kk) Jc[a][3 + kk] = A[a][0] * ex[kk][0] + A[a][1] * ex[kk][1] + A[a][2] * ex[kk][2];
        }
        if constexpr (NF == 1) {
            Jc[0][6] = du; Jc[1][6] = dv;
        } else {
            Jc[0][6] = du; Jc[0][7] = 0.0; Jc[1][6] = 0.0; Jc[1][7] = dv;
        }
#pragma unroll
        for (int j = 0; j < NK; ++j) { Jc[0][6 + NF + j] = fx * Jk[0][j]; Jc[1][6 + NF + j] = fy * Jk[1][j]; }
        (void)D;
    }
}

// pypose se3 Exp (left) composed with a stored pose [t, q_xyzw]: out = Exp([rho, phi]) * x.
__device__ __forceinline__ void retract_pose(const double* x, const double* d, double* out) {
    const double r0 = d[0], r1 = d[1], r2 = d[2];
    const double px = d[3], py = d[4], pz = d[5];
    const double th2 = px * px + py * py + pz * pz;
    double sh, ch, A, B;
    if (th2 < 1e-10) {  // th < 1e-5
        sh = 0.5 - th2 / 48.0 + th2 * th2 / 3840.0;
        ch = 1.0 - th2 / 8.0 + th2 * th2 / 384.0;
        A = 0.5 - th2 / 24.0 + th2 * th2 / 720.0;
        B = 1.0 / 6.0 - th2 / 120.0 + th2 * th2 / 5040.0;
    } else {
        const double th = sqrt(th2);
        sh = sin(0.5 * th) / th;
        ch = cos(0.5 * th);
        A = (1.0 - cos(th)) / th2;
        B = (th - sin(th)) / (th2 * th);
    }
    const double qdx = sh * px, qdy = sh * py, qdz = sh * pz, qdw = ch;
    const double cx = py * r2 - pz * r1, cy = pz * r0 - px * r2, cz = px * r1 - py * r0;
    const double c2x = py * cz - pz * cy, c2y = pz * cx - px * cz, c2z = px * cy - py * cx;
    const double taux = r0 + A * cx + B * c2x, tauy = r1 + A * cy + B * c2y, tauz = r2 + A * cz + B * c2z;
    const double t0 = x[0], t1 = x[1], t2 = x[2];
    const double e1x = qdy * t2 - qdz * t1, e1y = qdz * t0 - qdx * t2, e1z = qdx * t1 - qdy * t0;
    const double e2x = qdy * e1z - qdz * e1y, e2y = qdz * e1x - qdx * e1z, e2z = qdx * e1y - qdy * e1x;
    out[0] = t0 + 2.0 * (qdw * e1x + e2x) + taux;
    out[1] = t1 + 2.0 * (qdw * e1y + e2y) + tauy;
    out[2] = t2 + 2.0 * (qdw * e1z + e2z) + tauz;
    const double bx = x[3], by = x[4], bz = x[5], bw = x[6];
    out[3] = qdw * bx + qdx * bw + qdy * bz - qdz * by;
    out[4] = qdw * by - qdx * bz + qdy * bw + qdz * bx;
    out[5] = qdw * bz + qdx * by - qdy * bx + qdz * bw;
    out[6] = qdw * bw - qdx * bx - qdy * by - qdz * bz;
}

__device__ __forceinline__ double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

// Inverse of an SPD 3x3 given as [xx, xy, xz, yy, yz, zz] via Cholesky (same operation order as the oracle).
// Returns false if not positive definite.  Output in the same packed layout.
// The same Cholesky steps as spd3_inverse (bitwise the same inverse o), also returning the factor R (s = R R^T, lower)
// and R^-1, packed (00, 10, 20, 11, 21, 22).  On failure nothing is written.
__device__ __forceinline__ bool spd3_factor(const double s[6], double o[6], double R[6], double Ri[6]) {
    const double a00 = s[0], a10 = s[1], a20 = s[2], a11 = s[3], a21 = s[4], a22 = s[5];
    if (!(a00 > 0.0)) return false;
    const double l00 = sqrt(a00);
    const double l10 = a10 / l00;
    const double l20 = a20 / l00;
    const double d11 = a11 - l10 * l10;
    if (!(d11 > 0.0)) return false;
    const double l11 = sqrt(d11);
    const double l21 = (a21 - l20 * l10) / l11;
    const double d22 = a22 - l20 * l20 - l21 * l21;
    if (!(d22 > 0.0)) return false;
    const double l22 = sqrt(d22);
    const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
    const double i10 = (-l10 * i00) / l11;
    const double i20 = (-(l20 * i00) - l21 * i10) / l22;
    const double i21 = (-l21 * i11) / l22;
    o[0] = i00 * i00 + i10 * i10 + i20 * i20;
    o[1] = i10 * i11 + i20 * i21;
    o[2] = i20 * i22;
    o[3] = i11 * i11 + i21 * i21;
    o[4] = i21 * i22;
    o[5] = i22 * i22;
    R[0] = l00; R[1] = l10; R[2] = l20; R[3] = l11; R[4] = l21; R[5] = l22;
    Ri[0] = i00; Ri[1] = i10; Ri[2] = i20; Ri[3] = i11; Ri[4] = i21; Ri[5] = i22;
    return true;
}

__device__ __forceinline__ bool spd3_inverse(const double s[6], double o[6]) {
    const double a00 = s[0], a10 = s[1], a20 = s[2], a11 = s[3], a21 = s[4], a22 = s[5];
    if (!(a00 > 0.0)) return false;
    const double l00 = sqrt(a00);
    const double l10 = a10 / l00;
    const double l20 = a20 / l00;
    const double d11 = a11 - l10 * l10;
    if (!(d11 > 0.0)) return false;
    const double l11 = sqrt(d11);
    const double l21 = (a21 - l20 * l10) / l11;
    const double d22 = a22 - l20 * l20 - l21 * l21;
    if (!(d22 > 0.0)) return false;
    const double l22 = sqrt(d22);
    // Li = L^-1
    const double i00 = 1.0 / l00, i11 = 1.0 / l11, i22 = 1.0 / l22;
    const double i10 = (-l10 * i00) / l11;
    const double i20 = (-(l20 * i00) - l21 * i10) / l22;
    const double i21 = (-l21 * i11) / l22;
    // Ainv = Li^T Li
    o[0] = i00 * i00 + i10 * i10 + i20 * i20;
    o[1] = i10 * i11 + i20 * i21;
    o[2] = i20 * i22;
    o[3] = i11 * i11 + i21 * i21;
    o[4] = i21 * i22;
    o[5] = i22 * i22;
    return true;
}

}  // namespace insfm
