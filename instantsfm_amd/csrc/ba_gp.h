// Global positioning (TorchGP.Optimize, instantsfm/processors/global_positioning.py:45-206) on the BA core.
//
// Parameters: camera positions c [C,3], track points X [P,3], one scale s_o per observation (fixed where the
// observation has a valid depth: TorchGP's scale_indices).  Residual (utils/cost_function.py:23-29):
//     r_o = f_o (t_o - s_o (X_p - c_i)),   f_o = 1 (calibrated camera) or 0.5.
// With Huber/Triggs weight sqrt(w) the weighted Jacobian rows of an observation are
//     J_c = beta I,  J_X = -beta I,  J_s = a = -f (X - c) sqrt(w),   beta = s f sqrt(w).
// The scale blocks (1x1, damped h_ss = clamp(a.a) f) are eliminated first, per observation; what is left has exactly
// the bundle-adjustment shape with D = 3 (W_o = -beta^2 (I - a a^T / h_ss) per observation, 3x3 point and camera
// blocks), so the same k_schur / PCG / two-level kernels solve it.  The oracle is oracle/ba_oracle.c ora_gp_*.
//
//   linearize   k_gp_lin        : per observation: beta, a, r~ -> one 64-byte record
//               k_gp_lin_cams   : per camera (one wave): h_c = sum beta^2, g_c = -sum beta r~   (all-reduced)
//   per trial   k_gp_prep_points: per track: W_o, V_p (scale-eliminated, damped), g'_p, V^-1, y = V^-1 g'_p
//               k_gp_prep_cams  : per camera (one wave): U'_c, g'_c (this rank's observations; rank 0 adds the
//                                 damped diagonal and g_c, so summing S over ranks is exact)
//               k_schur<3>, k_cg_*, k_tl_* (basis [I | c_i])
//               k_gp_backsub    : per track: dp, trial points, scale steps, trial scales, model decrease
//               k_gp_update_cams: c + dc
//               k_gp_cost       : Huber loss + sum ||r||^2
#pragma once
#include "ba_common.h"
#include "ba_device.h"

namespace insfm {

// per local observation: {a0, a1, a2, beta} {r~0, r~1, r~2, free}
constexpr int kGO = 8;

__device__ __forceinline__ double gp_hss(const double4& A, const double4& R, double f, double cmin, double cmax) {
    return R.w != 0.0 ? clampd(A.x * A.x + A.y * A.y + A.z * A.z, cmin, cmax) * f : 0.0;
}

__global__ __launch_bounds__(kThreads) void k_gp_lin(int Nl, const int* __restrict__ cam, const int* __restrict__ ptl,
                                                     const double* __restrict__ trans, const double* __restrict__ fcam,
                                                     const int* __restrict__ sfree, const double* __restrict__ cams,
                                                     const double* __restrict__ pts, const double* __restrict__ scl,
                                                     double delta, double* __restrict__ gobs) {
    const int o = blockIdx.x * kThreads + threadIdx.x;
    if (o >= Nl) return;
    const int c = cam[o], p = ptl[o];
    const double f = fcam[c], s = scl[o];
    double e[3], r[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        e[k] = pts[3 * (size_t)p + k] - cams[3 * (size_t)c + k];
        r[k] = f * (trans[3 * (size_t)o + k] - s * e[k]);
    }
    const double rs = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    const double sw = sqrt(rs < delta ? 1.0 : delta / rs);
    const bool fr = sfree[o] != 0;
    double4* g = reinterpret_cast<double4*>(gobs + (size_t)o * kGO);
    g[0] = make_double4(fr ? -f * e[0] * sw : 0.0, fr ? -f * e[1] * sw : 0.0, fr ? -f * e[2] * sw : 0.0, s * f * sw);
    g[1] = make_double4(sw * r[0], sw * r[1], sw * r[2], fr ? 1.0 : 0.0);
}

// One wave per camera: h_c -> U[c][0], g_c -> gc[c] (summed over ranks afterwards, like the BA's U / g_c).
__global__ __launch_bounds__(kThreads) void k_gp_lin_cams(int C, const int* __restrict__ cam_ptr, const int* __restrict__ cam_obs,
                                                          const double* __restrict__ gobs, double* __restrict__ U,
                                                          double* __restrict__ gc) {
    const int c = blockIdx.x * kWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (c >= C) return;
    double h = 0.0, g0 = 0.0, g1 = 0.0, g2 = 0.0;
    for (int e = cam_ptr[c] + lane; e < cam_ptr[c + 1]; e += 64) {
        const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)cam_obs[e] * kGO);
        const double4 A = q[0], R = q[1];
        h += A.w * A.w;
        g0 -= A.w * R.x; g1 -= A.w * R.y; g2 -= A.w * R.z;
    }
    h = wave_sum(h); g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
    if (lane == 0) {
        double* u = U + (size_t)c * 9;
        u[0] = h;
#pragma unroll
        for (int k = 1; k < 9; ++k) u[k] = 0.0;
        gc[3 * (size_t)c] = g0; gc[3 * (size_t)c + 1] = g1; gc[3 * (size_t)c + 2] = g2;
    }
}

// One thread per local track: scale-eliminated W_o (symmetric, [o][3][3]), damped V_p (packed), g'_p, V^-1, y.
__global__ __launch_bounds__(kThreads) void k_gp_prep_points(int Pl, const int* __restrict__ pt_ptr, const double* __restrict__ gobs,
                                                             double f, double cmin, double cmax, double* __restrict__ W,
                                                             double* __restrict__ V, double* __restrict__ gp,
                                                             double* __restrict__ Vinv, double* __restrict__ y,
                                                             int* __restrict__ flags) {
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= Pl) return;
    double hx = 0.0, g[3] = {0.0, 0.0, 0.0}, Vc[6] = {0, 0, 0, 0, 0, 0};
    for (int o = pt_ptr[p]; o < pt_ptr[p + 1]; ++o) {
        const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)o * kGO);
        const double4 A = q[0], R = q[1];
        const double b = A.w, b2 = b * b;
        hx += b2;
        g[0] += b * R.x; g[1] += b * R.y; g[2] += b * R.z;
        const double hss = gp_hss(A, R, f, cmin, cmax);
        const double a[3] = {A.x, A.y, A.z};
        const double ih = hss > 0.0 ? 1.0 / hss : 0.0;
        double* Wo = W + (size_t)o * 9;
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) Wo[i * 3 + j] = -b2 * ((i == j ? 1.0 : 0.0) - (hss > 0.0 ? a[i] * a[j] / hss : 0.0));
        if (hss > 0.0) {
            const double c2 = b2 * ih, cg = -b * (A.x * R.x + A.y * R.y + A.z * R.z) * ih;
            Vc[0] -= c2 * a[0] * a[0]; Vc[1] -= c2 * a[0] * a[1]; Vc[2] -= c2 * a[0] * a[2];
            Vc[3] -= c2 * a[1] * a[1]; Vc[4] -= c2 * a[1] * a[2]; Vc[5] -= c2 * a[2] * a[2];
            g[0] += cg * a[0]; g[1] += cg * a[1]; g[2] += cg * a[2];
        }
    }
    const double d = clampd(hx, cmin, cmax) * f;
    double s[6] = {d + Vc[0], Vc[1], Vc[2], d + Vc[3], Vc[4], d + Vc[5]};
#pragma unroll
    for (int k = 0; k < 6; ++k) V[6 * (size_t)p + k] = s[k];
    double iv[6];
    if (!spd3_inverse(s, iv)) {
        atomicOr(flags, 1);
#pragma unroll
        for (int k = 0; k < 6; ++k) iv[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) Vinv[6 * (size_t)p + k] = iv[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) gp[3 * (size_t)p + k] = g[k];
    y[3 * (size_t)p + 0] = iv[0] * g[0] + iv[1] * g[1] + iv[2] * g[2];
    y[3 * (size_t)p + 1] = iv[1] * g[0] + iv[3] * g[1] + iv[4] * g[2];
    y[3 * (size_t)p + 2] = iv[2] * g[0] + iv[4] * g[1] + iv[5] * g[2];
}

// One wave per camera: U'_c = [rank 0] clamp(h_c) f I - sum c2 a a^T,  g'_c = [rank 0] g_c - sum cg a.
__global__ __launch_bounds__(kThreads) void k_gp_prep_cams(int C, const int* __restrict__ cam_ptr, const int* __restrict__ cam_obs,
                                                           const double* __restrict__ gobs, const double* __restrict__ U,
                                                           const double* __restrict__ gc, double f, double cmin, double cmax,
                                                           int add_diag, double* __restrict__ Up, double* __restrict__ gpc) {
    const int c = blockIdx.x * kWaves + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (c >= C) return;
    double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // packed sym U correction (6) | g correction (3)
    for (int e = cam_ptr[c] + lane; e < cam_ptr[c + 1]; e += 64) {
        const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)cam_obs[e] * kGO);
        const double4 A = q[0], R = q[1];
        const double hss = gp_hss(A, R, f, cmin, cmax);
        if (!(hss > 0.0)) continue;
        const double b = A.w, c2 = b * b / hss, cg = -b * (A.x * R.x + A.y * R.y + A.z * R.z) / hss;
        v[0] -= c2 * A.x * A.x; v[1] -= c2 * A.x * A.y; v[2] -= c2 * A.x * A.z;
        v[3] -= c2 * A.y * A.y; v[4] -= c2 * A.y * A.z; v[5] -= c2 * A.z * A.z;
        v[6] -= cg * A.x; v[7] -= cg * A.y; v[8] -= cg * A.z;
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0) {
        const double d = add_diag ? clampd(U[(size_t)c * 9], cmin, cmax) * f : 0.0;
        double* u = Up + (size_t)c * 9;
        u[0] = d + v[0]; u[1] = v[1]; u[2] = v[2];
        u[3] = v[1]; u[4] = d + v[3]; u[5] = v[4];
        u[6] = v[2]; u[7] = v[4]; u[8] = d + v[5];
#pragma unroll
        for (int k = 0; k < 3; ++k) gpc[3 * (size_t)c + k] = (add_diag ? gc[3 * (size_t)c + k] : 0.0) + v[6 + k];
    }
}

// dp = V^-1 (g'_p - sum W_o dc), trial points; per observation ds = (g_s - beta a.(dc - dp)) / h_ss, trial scales;
// model decrease -sum (J d).(2 r~ + J d) as a block partial.
__global__ __launch_bounds__(kThreads) void k_gp_backsub(int Pl, const int* __restrict__ pt_ptr, const int* __restrict__ cam,
                                                         const double* __restrict__ gobs, const double* __restrict__ W,
                                                         const double* __restrict__ dc, const double* __restrict__ Vinv,
                                                         const double* __restrict__ gp, const double* __restrict__ pts,
                                                         const double* __restrict__ scl, double f, double cmin, double cmax,
                                                         double* __restrict__ dp, double* __restrict__ pts_new,
                                                         double* __restrict__ scl_new, double* __restrict__ ds_out,
                                                         double* __restrict__ part) {
    __shared__ double red[kThreads];
    const int p = blockIdx.x * kThreads + threadIdx.x;
    double gain[1] = {0.0};
    if (p < Pl) {
        const int ob = pt_ptr[p], oe = pt_ptr[p + 1];
        double t0 = gp[3 * (size_t)p], t1 = gp[3 * (size_t)p + 1], t2 = gp[3 * (size_t)p + 2];
        for (int o = ob; o < oe; ++o) {
            const double* Wo = W + (size_t)o * 9;
            const double* d = dc + 3 * (size_t)cam[o];
            t0 -= Wo[0] * d[0] + Wo[1] * d[1] + Wo[2] * d[2];
            t1 -= Wo[3] * d[0] + Wo[4] * d[1] + Wo[5] * d[2];
            t2 -= Wo[6] * d[0] + Wo[7] * d[1] + Wo[8] * d[2];
        }
        const double* vi = Vinv + 6 * (size_t)p;
        const double x0 = vi[0] * t0 + vi[1] * t1 + vi[2] * t2;
        const double x1 = vi[1] * t0 + vi[3] * t1 + vi[4] * t2;
        const double x2 = vi[2] * t0 + vi[4] * t1 + vi[5] * t2;
        dp[3 * (size_t)p] = x0; dp[3 * (size_t)p + 1] = x1; dp[3 * (size_t)p + 2] = x2;
        pts_new[3 * (size_t)p] = pts[3 * (size_t)p] + x0;
        pts_new[3 * (size_t)p + 1] = pts[3 * (size_t)p + 1] + x1;
        pts_new[3 * (size_t)p + 2] = pts[3 * (size_t)p + 2] + x2;
        double dec = 0.0;
        for (int o = ob; o < oe; ++o) {
            const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)o * kGO);
            const double4 A = q[0], R = q[1];
            const double* d = dc + 3 * (size_t)cam[o];
            const double e0 = d[0] - x0, e1 = d[1] - x1, e2 = d[2] - x2;
            const double hss = gp_hss(A, R, f, cmin, cmax);
            double ds = 0.0;
            if (hss > 0.0) {
                const double gs = -(A.x * R.x + A.y * R.y + A.z * R.z);
                ds = (gs - A.w * (A.x * e0 + A.y * e1 + A.z * e2)) / hss;
            }
            scl_new[o] = scl[o] + ds;
            ds_out[o] = ds;
            const double j0 = A.w * e0 + A.x * ds, j1 = A.w * e1 + A.y * ds, j2 = A.w * e2 + A.z * ds;
            dec += j0 * (2.0 * R.x + j0) + j1 * (2.0 * R.y + j1) + j2 * (2.0 * R.z + j2);
        }
        gain[0] = -dec;
    }
    // block_sum<1> lives in ba_kernels.hip; a plain fixed-order tree here
    red[threadIdx.x] = gain[0];
    __syncthreads();
    for (int s = kThreads / 2; s >= 1; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ __launch_bounds__(kThreads) void k_gp_update_cams(int n, const double* __restrict__ cams, const double* __restrict__ dc,
                                                             double* __restrict__ cams_new) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k < n) cams_new[k] = cams[k] + dc[k];
}

// Huber loss and sum ||r||^2 (block partials {loss, sq}).
__global__ __launch_bounds__(kThreads) void k_gp_cost(int Nl, const int* __restrict__ cam, const int* __restrict__ ptl,
                                                      const double* __restrict__ trans, const double* __restrict__ fcam,
                                                      const double* __restrict__ cams, const double* __restrict__ pts,
                                                      const double* __restrict__ scl, double delta, double* __restrict__ part) {
    __shared__ double red[2 * kThreads];
    const int o = blockIdx.x * kThreads + threadIdx.x;
    double v0 = 0.0, v1 = 0.0;
    if (o < Nl) {
        const int c = cam[o], p = ptl[o];
        const double f = fcam[c], s = scl[o];
        double q = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double r = f * (trans[3 * (size_t)o + k] - s * (pts[3 * (size_t)p + k] - cams[3 * (size_t)c + k]));
            q += r * r;
        }
        const double rs = sqrt(q);
        v0 = rs < delta ? q : 2.0 * delta * rs - delta * delta;
        v1 = q;
    }
    red[threadIdx.x] = v0;
    red[kThreads + threadIdx.x] = v1;
    __syncthreads();
    for (int s = kThreads / 2; s >= 1; s >>= 1) {
        if (threadIdx.x < s) {
            red[threadIdx.x] += red[threadIdx.x + s];
            red[kThreads + threadIdx.x] += red[kThreads + threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) { part[2 * (size_t)blockIdx.x] = red[0]; part[2 * (size_t)blockIdx.x + 1] = red[kThreads]; }
}

// scales in the caller's observation order <-> the library's local order (tracks re-sorted by camera)
__global__ __launch_bounds__(kThreads) void k_gp_gather(int Nl, const int* __restrict__ osrc, const double* __restrict__ src,
                                                        double* __restrict__ dst) {
    const int o = blockIdx.x * kThreads + threadIdx.x;
    if (o < Nl) dst[o] = src[osrc[o]];
}

__global__ __launch_bounds__(kThreads) void k_gp_scatter(int Nl, const int* __restrict__ osrc, const double* __restrict__ src,
                                                         double* __restrict__ dst) {
    const int o = blockIdx.x * kThreads + threadIdx.x;
    if (o < Nl) dst[osrc[o]] = src[o];
}

}  // namespace insfm
