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
//   per trial   k_gp_prep_points: per track (a group of kGPG lanes): W_o, V_p (scale-eliminated, damped), g'_p, V^-1, y = V^-1 g'_p
//               k_gp_prep_cams  : per camera (one wave): U'_c, g'_c (this rank's observations; rank 0 adds the
//                                 damped diagonal and g_c, so summing S over ranks is exact)
//               k_schur<3>, k_cg_*, k_tl_* (basis [I | c_i])
//               k_gp_backsub    : per track (kGPG lanes): dp, trial points, scale steps, trial scales, model decrease
//               k_gp_update_cams: c + dc
//               k_gp_cost       : Huber loss + sum ||r||^2
#pragma once
#include "ba_common.h"
#include "ba_device.h"

namespace insfm {

// per local observation: {a0, a1, a2, beta} {r~0, r~1, r~2, free}
constexpr int kGO = 8;
constexpr int kGPG = 8;  // lanes per track in the per-track kernels
constexpr int kVY = 9;   // per-point record {V^-1 packed (6), y (3)}
#ifndef INSFM_GPS_G
#define INSFM_GPS_G 8
#endif
constexpr int kGPSG = INSFM_GPS_G;  // lanes per own observation in k_schur_gp (they split its partners)

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
// Sum NV per-thread values over the workgroup (wave butterflies, then the waves' sums in wave order through LDS);
// thread 0 gets the totals.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double (*red)[NV]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = wave_sum(v[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) red[wv][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            double t = red[0][k];
            for (int w = 1; w < kWaves; ++w) t += red[w][k];
            v[k] = t;
        }
}

// One workgroup per camera (its observations strided over the workgroup, two records in flight per thread).
__global__ __launch_bounds__(kThreads) void k_gp_lin_cams(int C, const int* __restrict__ cam_ptr, const int* __restrict__ cam_obs,
                                                          const double* __restrict__ gobs, double* __restrict__ U,
                                                          double* __restrict__ gc) {
    __shared__ double red[kWaves][4];
    const int c = blockIdx.x;
    double v[4] = {0.0, 0.0, 0.0, 0.0};  // h | g
    const int e0 = cam_ptr[c], e1 = cam_ptr[c + 1];
    for (int e = e0 + (int)threadIdx.x; e < e1; e += 2 * kThreads) {
        const int e2 = e + kThreads;
        const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)cam_obs[e] * kGO);
        const double4* q2 = reinterpret_cast<const double4*>(gobs + (size_t)cam_obs[min(e2, e1 - 1)] * kGO);
        const double4 A = q[0], R = q[1], A2 = q2[0], R2 = q2[1];
        v[0] += A.w * A.w;
        v[1] -= A.w * R.x; v[2] -= A.w * R.y; v[3] -= A.w * R.z;
        if (e2 < e1) {
            v[0] += A2.w * A2.w;
            v[1] -= A2.w * R2.x; v[2] -= A2.w * R2.y; v[3] -= A2.w * R2.z;
        }
    }
    block_sum<4>(v, red);
    if (threadIdx.x == 0) {
        double* u = U + (size_t)c * 9;
        u[0] = v[0];
#pragma unroll
        for (int k = 1; k < 9; ++k) u[k] = 0.0;
        gc[3 * (size_t)c] = v[1]; gc[3 * (size_t)c + 1] = v[2]; gc[3 * (size_t)c + 2] = v[3];
    }
}

// Reduce NV values over the G lanes of a lane group (xor butterfly: every lane of the group gets the sum).
template <int G, int NV>
__device__ __forceinline__ void group_sum(double (&v)[NV]) {
#pragma unroll
    for (int off = G / 2; off >= 1; off >>= 1)
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] += __shfl_xor(v[k], off, 64);
}

// A group of G lanes per local track (CSR-vector): lane l takes observations ob + l, ob + l + G, ... so a group reads
// G consecutive 64-byte records per round.  Scale-eliminated W_o (as {u, beta^2}, see load_wcol in ba_kernels.hip),
// damped V_p (packed), g'_p, V^-1, y.
template <int G>
__global__ __launch_bounds__(kThreads) void k_gp_prep_points(int Pl, const int* __restrict__ pt_ptr, const double* __restrict__ gobs,
                                                             double f, double cmin, double cmax, double* __restrict__ W,
                                                             double* __restrict__ V, double* __restrict__ gp,
                                                             double* __restrict__ Vinv, double* __restrict__ y,
                                                             double* __restrict__ VY, int* __restrict__ flags) {
    const int p = (blockIdx.x * kThreads + threadIdx.x) / G, l = threadIdx.x % G;
    const bool on = p < Pl;
    double v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // hx | g (3) | V correction (6, packed)
    if (on) {
        for (int o = pt_ptr[p] + l; o < pt_ptr[p + 1]; o += G) {
            const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)o * kGO);
            const double4 A = q[0], R = q[1];
            const double b = A.w, b2 = b * b;
            v[0] += b2;
            v[1] += b * R.x; v[2] += b * R.y; v[3] += b * R.z;
            const double hss = gp_hss(A, R, f, cmin, cmax);
            const double a[3] = {A.x, A.y, A.z};
            // W_o = -beta^2 (I - u u^T), u = a / sqrt(h_ss): the 32-byte record k_schur / k_gp_backsub expand
            const double ru = hss > 0.0 ? 1.0 / sqrt(hss) : 0.0;
            reinterpret_cast<double4*>(W)[o] = make_double4(a[0] * ru, a[1] * ru, a[2] * ru, b2);
            if (hss > 0.0) {
                const double c2 = b2 / hss, cg = -b * (A.x * R.x + A.y * R.y + A.z * R.z) / hss;
                v[4] -= c2 * a[0] * a[0]; v[5] -= c2 * a[0] * a[1]; v[6] -= c2 * a[0] * a[2];
                v[7] -= c2 * a[1] * a[1]; v[8] -= c2 * a[1] * a[2]; v[9] -= c2 * a[2] * a[2];
                v[1] += cg * a[0]; v[2] += cg * a[1]; v[3] += cg * a[2];
            }
        }
    }
    group_sum<G, 10>(v);
    if (!on || l != 0) return;
    const double d = clampd(v[0], cmin, cmax) * f;
    double s[6] = {d + v[4], v[5], v[6], d + v[7], v[8], d + v[9]};
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
    const double g[3] = {v[1], v[2], v[3]};
#pragma unroll
    for (int k = 0; k < 3; ++k) gp[3 * (size_t)p + k] = g[k];
    const double y0 = iv[0] * g[0] + iv[1] * g[1] + iv[2] * g[2];
    const double y1 = iv[1] * g[0] + iv[3] * g[1] + iv[4] * g[2];
    const double y2 = iv[2] * g[0] + iv[4] * g[1] + iv[5] * g[2];
    y[3 * (size_t)p + 0] = y0; y[3 * (size_t)p + 1] = y1; y[3 * (size_t)p + 2] = y2;
    // {V^-1 (packed 6), y (3)} in one 9-double record: k_schur_gp's lane group loads it with one instruction
    double* r = VY + (size_t)p * kVY;
#pragma unroll
    for (int k = 0; k < 6; ++k) r[k] = iv[k];
    r[6] = y0; r[7] = y1; r[8] = y2;
}

// One wave per camera: U'_c = [rank 0] clamp(h_c) f I - sum c2 a a^T,  g'_c = [rank 0] g_c - sum cg a.
__global__ __launch_bounds__(kThreads) void k_gp_prep_cams(int C, const int* __restrict__ cam_ptr, const int* __restrict__ cam_obs,
                                                           const double* __restrict__ gobs, const double* __restrict__ U,
                                                           const double* __restrict__ gc, double f, double cmin, double cmax,
                                                           int add_diag, double* __restrict__ Up, double* __restrict__ gpc) {
    __shared__ double red[kWaves][9];
    const int c = blockIdx.x;
    double v[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // packed sym U correction (6) | g correction (3)
    const int e0 = cam_ptr[c], e1 = cam_ptr[c + 1];
    auto add = [&](const double4& A, const double4& R) {
        const double hss = gp_hss(A, R, f, cmin, cmax);
        if (!(hss > 0.0)) return;
        const double b = A.w, c2 = b * b / hss, cg = -b * (A.x * R.x + A.y * R.y + A.z * R.z) / hss;
        v[0] -= c2 * A.x * A.x; v[1] -= c2 * A.x * A.y; v[2] -= c2 * A.x * A.z;
        v[3] -= c2 * A.y * A.y; v[4] -= c2 * A.y * A.z; v[5] -= c2 * A.z * A.z;
        v[6] -= cg * A.x; v[7] -= cg * A.y; v[8] -= cg * A.z;
    };
    for (int e = e0 + (int)threadIdx.x; e < e1; e += 2 * kThreads) {
        const int e2 = e + kThreads;
        const double4* q = reinterpret_cast<const double4*>(gobs + (size_t)cam_obs[e] * kGO);
        const double4* q2 = reinterpret_cast<const double4*>(gobs + (size_t)cam_obs[min(e2, e1 - 1)] * kGO);
        const double4 A = q[0], R = q[1], A2 = q2[0], R2 = q2[1];
        add(A, R);
        if (e2 < e1) add(A2, R2);
    }
    block_sum<9>(v, red);
    if (threadIdx.x == 0) {
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
// model decrease -sum (J d).(2 r~ + J d) as a block partial.  G lanes per track as in k_gp_prep_points; W_o dc is
// formed from the 32-byte {a, beta} half of the record (W_o = -beta^2 (I - a a^T / h_ss)) instead of reading W.
template <int G>
__global__ __launch_bounds__(kThreads) void k_gp_backsub(int Pl, const int* __restrict__ pt_ptr, const int* __restrict__ cam,
                                                         const double* __restrict__ gobs, const double* __restrict__ dc,
                                                         const double* __restrict__ Vinv, const double* __restrict__ gp,
                                                         const double* __restrict__ pts, const double* __restrict__ scl,
                                                         double f, double cmin, double cmax, double* __restrict__ dp,
                                                         double* __restrict__ pts_new, double* __restrict__ scl_new,
                                                         double* __restrict__ ds_out, double* __restrict__ part) {
    __shared__ double red[kThreads];
    const int p = (blockIdx.x * kThreads + threadIdx.x) / G, l = threadIdx.x % G;
    const bool on = p < Pl;
    const int ob = on ? pt_ptr[p] : 0, oe = on ? pt_ptr[p + 1] : 0;
    double t[3] = {0.0, 0.0, 0.0};
    for (int o = ob + l; o < oe; o += G) {
        const double4 A = reinterpret_cast<const double4*>(gobs + (size_t)o * kGO)[0];
        const double fr = gobs[(size_t)o * kGO + 7];
        const double* d = dc + 3 * (size_t)cam[o];
        const double d0 = d[0], d1 = d[1], d2 = d[2];
        const double b2 = A.w * A.w;
        const double hss = fr != 0.0 ? clampd(A.x * A.x + A.y * A.y + A.z * A.z, cmin, cmax) * f : 0.0;
        const double ad = hss > 0.0 ? (A.x * d0 + A.y * d1 + A.z * d2) / hss : 0.0;
        // W_o d = -beta^2 (d - a (a.d) / h_ss)
        t[0] += b2 * (d0 - A.x * ad); t[1] += b2 * (d1 - A.y * ad); t[2] += b2 * (d2 - A.z * ad);
    }
    group_sum<G, 3>(t);
    double x0 = 0.0, x1 = 0.0, x2 = 0.0;
    if (on) {
        t[0] += gp[3 * (size_t)p]; t[1] += gp[3 * (size_t)p + 1]; t[2] += gp[3 * (size_t)p + 2];
        const double* vi = Vinv + 6 * (size_t)p;
        x0 = vi[0] * t[0] + vi[1] * t[1] + vi[2] * t[2];
        x1 = vi[1] * t[0] + vi[3] * t[1] + vi[4] * t[2];
        x2 = vi[2] * t[0] + vi[4] * t[1] + vi[5] * t[2];
        if (l < 3) {
            const double xv = l == 0 ? x0 : (l == 1 ? x1 : x2);
            dp[3 * (size_t)p + l] = xv;
            pts_new[3 * (size_t)p + l] = pts[3 * (size_t)p + l] + xv;
        }
    }
    double dec = 0.0;
    for (int o = ob + l; o < oe; o += G) {
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
    red[threadIdx.x] = -dec;
    __syncthreads();
    for (int s = kThreads / 2; s >= 1; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// Schur complement for global positioning (D = 3): like k_schur (one workgroup per camera row chunk, the chunk of S's
// row accumulated in LDS with f64 atomics, descriptors {o, p, partner begin, end} prefetched), but ONE lane per own
// observation: a 3x3 block needs 9 products per partner, so a lane holds the whole W^_o = W_o V_p^-1 and the wave
// covers 64 own observations per round instead of 21 three-lane groups -- the round chain (descriptor -> V^-1, W ->
// partner records -> slot lookup) is what bounds this kernel, not the atomics.
template <int WAVES, int G>
__global__ __launch_bounds__(WAVES * 64) void k_schur_gp(const int4* __restrict__ work, const int* __restrict__ row_ptr,
                                                         const int* __restrict__ col, int C, const int* __restrict__ cam_ptr,
                                                         const int4* __restrict__ sdesc, const int* __restrict__ cam,
                                                         const double* __restrict__ W, const double* __restrict__ VY,
                                                         const double* __restrict__ Up,
                                                         const double* __restrict__ gpc, double* __restrict__ S,
                                                         double* __restrict__ b) {
    constexpr int NT = WAVES * 64, BS = 9, NGW = NT / G;
    static_assert(64 % G == 0, "lane groups must tile a wave");
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const int4 wk = work[blockIdx.x];
    const int i = wk.x, kb = wk.y, ke = wk.z, nb = ke - kb;
    double* acc = sh;
    double* bacc = acc + (size_t)nb * BS;
    int* slot = reinterpret_cast<int*>(bacc + 4);
    const int t = threadIdx.x, lane = t & 63, g = t / G, l = t % G;
    for (int k = t; k < nb * BS; k += NT) acc[k] = 0.0;
    for (int k = t; k < C; k += NT) slot[k] = -1;
    if (t < 3) bacc[t] = 0.0;
    __syncthreads();
    for (int e = kb + t; e < ke; e += NT) slot[col[e]] = e - kb;
    __syncthreads();
    const bool diag_chunk = (kb == row_ptr[i]);
    const double4* Wr = reinterpret_cast<const double4*>(W);
    double br[3] = {0.0, 0.0, 0.0};
    const int ob = cam_ptr[i], oe = cam_ptr[i + 1];
    // software pipeline: descriptors two rounds ahead, the own record {V^-1, y | u, beta^2} and the lane's first
    // partner record one round ahead -- every round's chain of dependent gathers overlaps the previous round's work
    struct Own {
        double v[6], yv[3];
        double4 r, q;
        int cq;
    };
    auto load_own = [&](const int4& d, Own& w) {
        const double* vy = VY + (size_t)d.y * kVY;
#pragma unroll
        for (int k = 0; k < 6; ++k) w.v[k] = vy[k];
        w.yv[0] = vy[6]; w.yv[1] = vy[7]; w.yv[2] = vy[8];
        w.r = Wr[d.x];
        const int q = d.z + l;
        w.cq = -1;
        if (q < d.w) { w.q = Wr[q]; w.cq = cam[q]; }
    };
    const int eend = oe;
    int4 dcur = make_int4(0, 0, 0, 0), dnext = make_int4(0, 0, 0, 0);
    Own cur, nxt;
    if (ob + g < eend) { dcur = sdesc[ob + g]; load_own(dcur, cur); }
    if (ob + g + NGW < eend) dnext = sdesc[ob + g + NGW];
    for (int e = ob + g; e < eend; e += NGW) {
        int4 dnn = make_int4(0, 0, 0, 0);
        if (e + 2 * NGW < eend) dnn = sdesc[e + 2 * NGW];
        if (e + NGW < eend) load_own(dnext, nxt);
        const double* v = cur.v;
        const double* yv = cur.yv;
        const double u[3] = {cur.r.x, cur.r.y, cur.r.z};
        const double rw = cur.r.w;
        double w[3][3], wh[3][3];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int m = 0; m < 3; ++m) w[k][m] = -rw * ((k == m ? 1.0 : 0.0) - u[k] * u[m]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            wh[k][0] = w[k][0] * v[0] + w[k][1] * v[1] + w[k][2] * v[2];
            wh[k][1] = w[k][0] * v[1] + w[k][1] * v[3] + w[k][2] * v[4];
            wh[k][2] = w[k][0] * v[2] + w[k][1] * v[4] + w[k][2] * v[5];
        }
        if (diag_chunk && l == 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k) br[k] -= w[k][0] * yv[0] + w[k][1] * yv[1] + w[k][2] * yv[2];
        }
        for (int q = dcur.z + l; q < dcur.w; q += G) {
            const bool first = q == dcur.z + l;
            const double4 rq = first ? cur.q : Wr[q];
            const int sl = slot[first ? cur.cq : cam[q]];
            if (sl < 0) continue;
            // W_q = -beta_q^2 (I - u_q u_q^T):  -(W^_o W_q^T)[k][m] = beta_q^2 (wh[k][m] - (wh[k] . u_q) u_q[m])
            const double uq[3] = {rq.x, rq.y, rq.z};
            double* dst = acc + (size_t)sl * BS;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double wu = wh[k][0] * uq[0] + wh[k][1] * uq[1] + wh[k][2] * uq[2];
#pragma unroll
                for (int m = 0; m < 3; ++m) {
                    const double val = rq.w * (wh[k][m] - wu * uq[m]);
                    atomicAdd(dst + k * 3 + m, val);
                }
            }
        }
        cur = nxt;
        dcur = dnext;
        dnext = dnn;
    }
    if (diag_chunk) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double s = wave_sum(br[k]);
            if (lane == 0) atomicAdd(bacc + k, s);
        }
    }
    __syncthreads();
    double* Sout = S + (size_t)kb * 9;
    for (int k = t; k < nb * 9; k += NT) {
        double val = acc[k];
        if (diag_chunk && k < 9) val += Up[(size_t)i * 9 + k];
        Sout[k] = val;
    }
    if (diag_chunk && t < 3) b[(size_t)i * 3 + t] = gpc[(size_t)i * 3 + t] + bacc[t];
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


// insfm_gp_step's parameter exchange with the caller's buffers in one launch: positions (3C), the shard's points
// (3Pl) and the per-observation scales (caller order <-> track order through osrc); `in` = 1 loads the LM state
// from the caller, 0 writes it back.
__global__ __launch_bounds__(kThreads) void k_gp_io(int in, long long n3c, double* __restrict__ pos, double* __restrict__ cams,
                                                    long long n3p, double* __restrict__ upts, double* __restrict__ pts,
                                                    long long nl, const int* __restrict__ osrc, double* __restrict__ uscl,
                                                    double* __restrict__ scl) {
    const long long tot = n3c + n3p + nl;
    for (long long k = (long long)blockIdx.x * kThreads + threadIdx.x; k < tot; k += (long long)gridDim.x * kThreads) {
        if (k < n3c) {
            if (in) cams[k] = pos[k]; else pos[k] = cams[k];
        } else if (k < n3c + n3p) {
            const long long q = k - n3c;
            if (in) pts[q] = upts[q]; else upts[q] = pts[q];
        } else {
            const long long o = k - n3c - n3p;
            if (in) scl[o] = uscl[osrc[o]]; else uscl[osrc[o]] = scl[o];
        }
    }
}

}  // namespace insfm
