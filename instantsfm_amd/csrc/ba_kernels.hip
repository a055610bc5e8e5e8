// MI355X (gfx950) sparse bundle-adjustment core: HIP kernels + host LM driver behind include/insfm_ba.h.
//
// One LM step (bae.optim.LM.step as reconstructed in SURVEY.md 3.3, options of bundle_adjustment.py:115-119):
//   linearize (per step)   k_lin_points  : per track, residual + analytic J + Huber/Triggs weight  -> W_o, V_p, g_p
//                          k_lin_cams    : per camera, J~c^T J~c and -J~c^T r~ (LDS-staged batch)  -> U_c, g_c
//   per trial (damping f)  k_point_prep  : V_p clamp/damp + 3x3 SPD inverse                          -> V^-1, y = V^-1 g_p
//                          k_schur       : per camera row, LDS-resident row of S (upper blocks), b
//                          k_cg_factor / k_cg_scale : S_ii = L L^T, S~ = L^-1 S L^-T, r0 = L^-1 b
//                          k_cg_iter x k : Chronopoulos-Gear CG on S~, ONE launch per iteration
//                          k_cg_finish   : dc = L^-T x~
//                          k_backsub_rc  : dp = V^-1 (g_p - W^T dc), trial points, gain terms; its last blocks the
//                                          SE3 left retraction of the cameras, intrinsics +=, gain terms
//                          k_cost        : Huber loss + sum ||r||^2 at the trial parameters
//                          k_final       : fixed-order reduction of all partials -> 64 B to the host
// Every cross-workgroup reduction is a fixed-order partial sum (no float atomics in global memory), so a step is
// bitwise reproducible when desc.deterministic = 1 (the Schur row accumulation then uses one wave per row).
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <unordered_map>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/insfm_ba.h"
#include "../../include/insfm_gp.h"
#include "ba_device.h"
#include "ba_common.h"
#include "ba_twolevel.h"
#include "ba_cgp.h"
#include "ba_gp.h"
#include "cg_poll.h"
#include "create_host.h"

using namespace insfm;

namespace {

constexpr int kLdsBudget = 96 * 1024;  // dynamic LDS cap for one k_schur workgroup
#ifndef SCHUR_LDS_KB
#define SCHUR_LDS_KB 96  // k_schur row-chunk LDS target (rows with more upper blocks are split into chunks)
#endif
constexpr int kLdsTarget = SCHUR_LDS_KB * 1024;
#ifndef SCHUR_LDS_KB_DET
#define SCHUR_LDS_KB_DET 52  // deterministic mode's k_schur row-chunk LDS target (3 four-wave workgroups per CU)
#endif
constexpr int kLdsTargetDet = SCHUR_LDS_KB_DET * 1024;
#ifndef INSFM_SCHUR_WAVES
#define INSFM_SCHUR_WAVES 8
#endif
constexpr int kSchurWaves = INSFM_SCHUR_WAVES;  // waves per k_schur workgroup (non-deterministic mode)
constexpr int kSchurChunk = 4;  // k_schur rounds per chunk of a camera's observation list (create)
#ifndef LIN_CAMS_NT
#define LIN_CAMS_NT 128  // k_lin_cams_reg threads per camera (measured 128 / 192 / 256 / 320: 0.156 / 0.161 / 0.167 / 0.194 ms linearize)
#endif
#ifndef COST_THREADS
#define COST_THREADS 256
#endif
constexpr int kCostThreads = COST_THREADS;  // k_cost workgroup size (64 / 128 / 512: same time, 25-26 us; 1024: trial cost 0.045 -> 0.055 ms)
#ifndef SCHUR_MINW
#define SCHUR_MINW 1  // k_schur launch bound: minimum waves per SIMD (caps VGPRs: 4 -> 128)
#endif
#ifndef SCHUR_SLOTPRE
#define SCHUR_SLOTPRE 1  // k_schur: a round's partner slots looked up before its LDS adds
#endif
// the persistent CG's solves form the factorization and the coarse basis in one launch (k_cg_factor_basis; 0: the
// separate k_cg_factor and k_tl_basis launches, for A/B builds)
#ifndef FACTOR_BASIS
#define FACTOR_BASIS 1
#endif
#ifndef SCHUR_UP
#define SCHUR_UP 10
#endif
#ifndef LIN_NT_STORE
// k_lin_points: the 384-MB Y-record stream stored with the nontemporal hint (global_store_dwordx4 ... nt).  Config 3
// (profiles/r6_v10/nt_ab.txt, same box): back-to-back launches 152-153 -> 85 us, LM step 1.046-1.050 -> 1.013-1.033
// ms; k_schur, which reads the records next, unchanged (440-448 us).
#define LIN_NT_STORE 1
#endif
#ifndef SCHUR_NT_STORE
#define SCHUR_NT_STORE 0  // k_schur: S blocks stored with the nontemporal hint (A/B builds)
#endif
// deterministic mode's k_schur: waves per workgroup; with more than one the waves take their LDS adds in turn.
// Measured on config 3 (profiles/r6_v7/det_ab*.txt, k_schur per trial): 1 wave (round 5) 1.15 ms; 2 / 3 / 4 / 6 / 8
// waves 1.06 / 0.97 / 0.90 / 1.68 / 1.36 ms (4 waves at 5 partners in flight: 148 VGPRs, three workgroups per CU;
// 3 / 4 / 10 partners in flight 0.98 / 0.93 / 1.10 ms; row chunks of 40 / 52 / 64 KB 1.33 / 0.90 / 1.03 ms)
#ifndef SCHUR_DET_WAVES
#define SCHUR_DET_WAVES 4
#endif
#ifndef SCHUR_UP_DET
#define SCHUR_UP_DET 5  // partners in flight per group in the turn-taking form
#endif
#define SCHUR_DET_ORD (SCHUR_DET_WAVES > 1)
constexpr int kDetWaves = SCHUR_DET_WAVES;

// ------------------------------------------------------------------------------------------------------------
// reductions
// ------------------------------------------------------------------------------------------------------------
// Fixed-order block reduction of NV values per thread, returned to every thread: a butterfly per wave, then the wave
// sums in wave order (one barrier instead of one per tree level).
template <int NV, int NT = kThreads>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* sh /* >= NV * NT / 64 doubles */) {
    constexpr int NW = NT / 64;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const double s = wave_sum(v[k]);
        if (lane == 0) sh[k * NW + wv] = s;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = sh[k * NW];
#pragma unroll
        for (int w = 1; w < NW; ++w) s += sh[k * NW + w];
        v[k] = s;
    }
    __syncthreads();
}

// Sum n partial records of NV doubles (record-major) in a fixed order; every thread gets the result.
template <int NV, int NT = kThreads>
__device__ __forceinline__ void sum_partials(const double* __restrict__ part, int n, double (&out)[NV], double* sh) {
    double v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] = 0.0;
#pragma unroll 8
    for (int i = threadIdx.x; i < n; i += NT)  // unrolled: 8 loads in flight, the adds in order
#pragma unroll
        for (int k = 0; k < NV; ++k) v[k] += part[(size_t)i * NV + k];
    block_sum<NV, NT>(v, sh);
#pragma unroll
    for (int k = 0; k < NV; ++k) out[k] = v[k];
}

__device__ __forceinline__ double huber_weight_sqrt(double s, double delta) {
    const double rs = sqrt(s);
    const double w = rs < delta ? 1.0 : delta / rs;
    return sqrt(w);
}

// ------------------------------------------------------------------------------------------------------------
// linearization
// ------------------------------------------------------------------------------------------------------------
// Every observation's weighted J gives W_o = J~c^T J~p (stored [o][3][D]: a group of D lanes reads each column of W_o
// as one contiguous segment in k_schur); each track reduces V_p = sum J~p^T J~p (packed sym) and g_p = -sum J~p^T r~.
constexpr int kLinThreads = 128;  // k_lin_points workgroup (LDS: W staging + V/g terms of its observations)

// Symmetric camera-point records (round 4).  With R_p the Cholesky factor of point p's damped block at the first
// trial's damping (V_p,d = R_p R_p^T; f = 1 + damping is known when the linearization is enqueued) and L_p = R_p^-T,
// L_p L_p^T = V_p,d^-1, so every observation's record is stored as Y_o = W_o L_p (D x 3, [o][3][D] like W) and
//   S_ij -= sum_p Y_ip Y_jp^T,   b_i -= sum Y_o z_p,  z_p = L_p^T g_p = R_p^-1 g_p:
// k_schur's first trial needs no per-observation V^-1 loads or W V^-1 products.  A retried trial at another damping
// factor f' uses M_p = L_p^-1 V'_p^-1 L_p^-T = R_p^T V'_p^-1 R_p (symmetric) between the records and z'_p = R_p^T y'_p
// (y'_p = V'_p^-1 g_p), formed per point by k_point_prep: the same k_schur with M_p where the GP build has V^-1.
// The first trial's point preparation itself is fused into k_lin_points: per track the damped V_p (diagonal clamped,
// times f), its 3x3 inverse (bitwise k_point_prep's: the same Cholesky steps), R_p and z_p, and the CG status words
// cleared.
struct PointPrep {
    double f = 1.0, cmin = 0.0, cmax = 0.0;
    double* Vinv = nullptr;
    double* y = nullptr;   // z_p = R_p^-1 g_p (with R), else y_p = V_p^-1 g_p
    double* R = nullptr;   // R_p packed (00, 10, 20, 11, 21, 22); null: no records (points-only solves)
    int* flags = nullptr;
    int* status = nullptr;
};
// Returns R_p^-1 (packed) in Ri; all zero when the damped block is not positive definite (flag raised).
__device__ __forceinline__ void point_prep_first(int p, const double V[6], const double g[3], const PointPrep& a,
                                                 double Ri[6]) {
    double s[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) s[k] = V[k];
    s[0] = clampd(s[0], a.cmin, a.cmax) * a.f;
    s[3] = clampd(s[3], a.cmin, a.cmax) * a.f;
    s[5] = clampd(s[5], a.cmin, a.cmax) * a.f;
    double o[6], R[6];
    if (!spd3_factor(s, o, R, Ri)) {
        atomicOr(a.flags, 1);
#pragma unroll
        for (int k = 0; k < 6; ++k) o[k] = R[k] = Ri[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) a.Vinv[6 * (size_t)p + k] = o[k];
    if (a.R) {
#pragma unroll
        for (int k = 0; k < 6; ++k) a.R[6 * (size_t)p + k] = R[k];
        a.y[3 * (size_t)p + 0] = Ri[0] * g[0];
        a.y[3 * (size_t)p + 1] = Ri[1] * g[0] + Ri[3] * g[1];
        a.y[3 * (size_t)p + 2] = Ri[2] * g[0] + Ri[4] * g[1] + Ri[5] * g[2];
    } else {
        a.y[3 * (size_t)p + 0] = o[0] * g[0] + o[1] * g[1] + o[2] * g[2];
        a.y[3 * (size_t)p + 1] = o[1] * g[0] + o[3] * g[1] + o[4] * g[2];
        a.y[3 * (size_t)p + 2] = o[2] * g[0] + o[4] * g[1] + o[5] * g[2];
    }
}

// One observation's weighted linearization: the V / g_p terms (cv: V packed sym 6, J~p^T r~ 3) and W_o (w[k * D + a] =
// (J~c^T J~p)[a][k]).
template <int M>
__device__ __forceinline__ void lin_obs(int o, const int* __restrict__ cam, const int* __restrict__ ptl,
                                        const double* __restrict__ uv, const double* __restrict__ pp,
                                        const double* __restrict__ cams, const double* __restrict__ pts, double delta,
                                        double cv[9], double w[3 * kD<M>]) {
    constexpr int D = kD<M>, ST = kStride<M>;
    const int c = cam[o], p = ptl[o];
    const double X[3] = {pts[3 * (size_t)p], pts[3 * (size_t)p + 1], pts[3 * (size_t)p + 2]};
    const double2 z = reinterpret_cast<const double2*>(uv)[o];
    const double uvo[2] = {z.x, z.y};
    const double ppc[2] = {pp[2 * c], pp[2 * c + 1]};
    double r[2], Jc[2][D], Jp[2][3];
    eval_obs<M, true>(cams + (size_t)c * ST, X, ppc, uvo, r, Jc, Jp);
    const double sw = huber_weight_sqrt(r[0] * r[0] + r[1] * r[1], delta);
    r[0] *= sw; r[1] *= sw;
#pragma unroll
    for (int a = 0; a < D; ++a) { Jc[0][a] *= sw; Jc[1][a] *= sw; }
#pragma unroll
    for (int k = 0; k < 3; ++k) { Jp[0][k] *= sw; Jp[1][k] *= sw; }
    cv[0] = Jp[0][0] * Jp[0][0] + Jp[1][0] * Jp[1][0];
    cv[1] = Jp[0][0] * Jp[0][1] + Jp[1][0] * Jp[1][1];
    cv[2] = Jp[0][0] * Jp[0][2] + Jp[1][0] * Jp[1][2];
    cv[3] = Jp[0][1] * Jp[0][1] + Jp[1][1] * Jp[1][1];
    cv[4] = Jp[0][1] * Jp[0][2] + Jp[1][1] * Jp[1][2];
    cv[5] = Jp[0][2] * Jp[0][2] + Jp[1][2] * Jp[1][2];
#pragma unroll
    for (int k = 0; k < 3; ++k) cv[6 + k] = Jp[0][k] * r[0] + Jp[1][k] * r[1];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k * D + a] = Jc[0][a] * Jp[0][k] + Jc[1][a] * Jp[1][k];
}

// Y_o = W_o L_p in place (w[k * D + a] as lin_obs), L_p = R_p^-T: Y[a][j] = sum_{k <= j} W[a][k] (R_p^-1)[j][k].
template <int D>
__device__ __forceinline__ void y_from_w(double w[3 * D], const double Ri[6]) {
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const double w0 = w[a], w1 = w[D + a], w2 = w[2 * D + a];
        w[a] = w0 * Ri[0];
        w[D + a] = w0 * Ri[1] + w1 * Ri[3];
        w[2 * D + a] = w0 * Ri[2] + w1 * Ri[4] + w2 * Ri[5];
    }
}

// Records of observations [base, base + n) from the LDS staging rows (odd stride WRP) to HBM, consecutive lanes storing
// consecutive 16-B pairs when the record length is even (a pair never crosses a record; every record starts 16-B
// aligned).
template <int WR, int WRP>
__device__ __forceinline__ void store_records(const double* wst, double* __restrict__ Y, int base, int n) {
    const int t = threadIdx.x;
    if constexpr ((WR & 1) == 0) {
        double2* dst = reinterpret_cast<double2*>(Y + (size_t)base * WR);
        for (int k2 = t; k2 < n * (WR / 2); k2 += kLinThreads) {
            const int k = 2 * k2, rec = k / WR, e = k - rec * WR;
            const double* src = wst + rec * WRP + e;
#if LIN_NT_STORE
            typedef double nt_d2 __attribute__((ext_vector_type(2)));
            nt_d2 v2 = {src[0], src[1]};
            __builtin_nontemporal_store(v2, reinterpret_cast<nt_d2*>(dst + k2));
#else
            dst[k2] = make_double2(src[0], src[1]);
#endif
        }
    } else {
        double* dst = Y + (size_t)base * WR;
        for (int k = t; k < n * WR; k += kLinThreads) dst[k] = wst[(k / WR) * WRP + k % WR];
    }
}

template <int M>
__global__ __launch_bounds__(kLinThreads) void k_lin_points(const int* __restrict__ blk, const int* __restrict__ pt_ptr,
                                                         const int* __restrict__ cam, const int* __restrict__ ptl,
                                                         const double* __restrict__ uv, const double* __restrict__ pp,
                                                         const double* __restrict__ cams, const double* __restrict__ pts,
                                                         double delta, double* __restrict__ Y, double* __restrict__ V,
                                                         double* __restrict__ gp, PointPrep pp1, long long* stp) {
    // One workgroup per run of whole tracks (blk, built at create: at most kLinThreads observations unless a single track
    // is longer), one thread per observation: coalesced uv / cam / point loads.  Each observation's V / g terms go to
    // LDS and one thread per track adds them in observation order -- the same sequence of additions as a thread walking
    // its track; that thread then prepares the point (damped V^-1, R_p, z_p) and puts R_p^-1 in LDS, and every
    // observation turns its W_o (kept in registers) into Y_o, staged in LDS (odd row stride) and stored coalesced in
    // 16-B pairs (192-B records for D = 8).  A run that is one track longer than the workgroup evaluates its
    // observations twice (once for the sums, once for the records).  One 25.6-KB LDS buffer serves the terms, the
    // R_p^-1 table and the record staging (6 workgroups per CU).  Y null (points-only solves): no records.
    constexpr int D = kD<M>, WR = 3 * D, WRP = WR | 1;  // odd LDS row stride
    static_assert(WRP >= 9, "the V / g terms reuse a record staging row");
    const StampScope stamp_(stp);
    __shared__ double wst[kLinThreads * WRP];
    const int t = threadIdx.x;
    const int tb = blk[blockIdx.x], te = blk[blockIdx.x + 1];
    const int ob = pt_ptr[tb], oe = pt_ptr[te];
    const bool one = oe - ob <= kLinThreads;  // (uniform) the run's observations fit one pass
    double Vs[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    const int tr = tb + t;  // the track this thread sums (tracks of the run)
    const int tlo = tr < te ? pt_ptr[tr] : 0, thi = tr < te ? pt_ptr[tr + 1] : 0;
    double w[WR];
    for (int base = ob; base < oe; base += kLinThreads) {
        const int o = base + t;
        double cv[9];
        if (o < oe) {
            lin_obs<M>(o, cam, ptl, uv, pp, cams, pts, delta, cv, w);
#pragma unroll
            for (int k = 0; k < 9; ++k) wst[(size_t)t * 9 + k] = cv[k];
        }
        __syncthreads();
        if (tr < te) {
            const int lo = max(tlo, base), hi = min(thi, base + kLinThreads);
            for (int q = lo; q < hi; ++q) {
                const double* cq = wst + (size_t)(q - base) * 9;
#pragma unroll
                for (int k = 0; k < 6; ++k) Vs[k] += cq[k];
#pragma unroll
                for (int k = 0; k < 3; ++k) g[k] -= cq[6 + k];
            }
        }
        __syncthreads();
    }
    double Ri[6];
    if (tr < te) {
#pragma unroll
        for (int k = 0; k < 6; ++k) V[6 * (size_t)tr + k] = Vs[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) gp[3 * (size_t)tr + k] = g[k];
        point_prep_first(tr, Vs, g, pp1, Ri);
        if (Y) {
#pragma unroll
            for (int k = 0; k < 6; ++k) wst[(size_t)t * 6 + k] = Ri[k];
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < 4) pp1.status[threadIdx.x] = 0;  // (k_point_prep's status clear)
    if (!Y) return;
    __syncthreads();
    if (one) {
        const int o = ob + t;
        if (o < oe) {
            const double* rq = wst + (size_t)(ptl[o] - tb) * 6;
            double r6[6];
#pragma unroll
            for (int k = 0; k < 6; ++k) r6[k] = rq[k];
            y_from_w<D>(w, r6);
        }
        __syncthreads();  // (every R^-1 read before the staging overwrites the table)
        if (o < oe) {
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int k = 0; k < 3; ++k) wst[(size_t)t * WRP + k * D + a] = w[k * D + a];
        }
        __syncthreads();
        store_records<WR, WRP>(wst, Y, ob, oe - ob);
        return;
    }
    // one track longer than the workgroup: its R^-1 from the table, then the records chunk by chunk
    double r6[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) r6[k] = wst[k];
    __syncthreads();
    for (int base = ob; base < oe; base += kLinThreads) {
        const int o = base + t;
        if (o < oe) {
            double cv[9];
            lin_obs<M>(o, cam, ptl, uv, pp, cams, pts, delta, cv, w);
            y_from_w<D>(w, r6);
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int k = 0; k < 3; ++k) wst[(size_t)t * WRP + k * D + a] = w[k * D + a];
        }
        __syncthreads();
        store_records<WR, WRP>(wst, Y, base, min(kLinThreads, oe - base));
        __syncthreads();
    }
}

// One workgroup per camera: 256 observations at a time are evaluated (one per thread) into an LDS batch
// [obs][J~c row0 | J~c row1 | r~0 r~1]; then thread e owns entry e of [U (DxD) | g_c (D)] and sums the batch in
// observation order (the oracle's order).  The camera-major point index and uv of each observation (cm_pt, cm_uv,
// built at create) are read coalesced; the next batch's point is fetched while the current batch is reduced and
// the indices two batches ahead, so no batch waits on a dependent load chain.
template <int M>
__global__ __launch_bounds__(kThreads) void k_lin_cams(const int* __restrict__ cam_ptr, const int* __restrict__ cm_pt,
                                                       const double* __restrict__ cm_uv, const double* __restrict__ pp,
                                                       const double* __restrict__ cams, const double* __restrict__ pts,
                                                       double delta, double* __restrict__ U, double* __restrict__ gc) {
    constexpr int D = kD<M>, ST = kStride<M>;
    constexpr int RW = 2 * D + 2;
    constexpr int E = D * D + D;
    constexpr int EPT = (E + kThreads - 1) / kThreads;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const int c = blockIdx.x, t = threadIdx.x;
    const int eb = cam_ptr[c], ee = cam_ptr[c + 1];
    const double2* uv2 = reinterpret_cast<const double2*>(cm_uv);
    double camv[ST];
#pragma unroll
    for (int k = 0; k < ST; ++k) camv[k] = cams[(size_t)c * ST + k];
    const double ppc[2] = {pp[2 * c], pp[2 * c + 1]};
    double acc[EPT];
#pragma unroll
    for (int m = 0; m < EPT; ++m) acc[m] = 0.0;
    // pipeline registers: current batch (X, z), next batch (pn, zn), two ahead (pnn, znn)
    double X[3] = {0.0, 0.0, 0.0};
    double2 z = make_double2(0.0, 0.0), zn = z, znn = z;
    int pn = 0, pnn = 0;
    {
        const int e0 = eb + t, e1 = e0 + kThreads;
        if (e0 < ee) {
            const int p0 = cm_pt[e0];
            z = uv2[e0];
            X[0] = pts[3 * (size_t)p0]; X[1] = pts[3 * (size_t)p0 + 1]; X[2] = pts[3 * (size_t)p0 + 2];
        }
        if (e1 < ee) { pn = cm_pt[e1]; zn = uv2[e1]; }
    }
    for (int base = eb; base < ee; base += kThreads) {
        const int e = base + t;
        const bool has = e < ee, hn = e + kThreads < ee, hnn = e + 2 * kThreads < ee;
        double Xn[3] = {0.0, 0.0, 0.0};
        if (hn) { Xn[0] = pts[3 * (size_t)pn]; Xn[1] = pts[3 * (size_t)pn + 1]; Xn[2] = pts[3 * (size_t)pn + 2]; }
        if (hnn) { pnn = cm_pt[e + 2 * kThreads]; znn = uv2[e + 2 * kThreads]; }
        double* row = sh + (size_t)t * RW;
        if (has) {
            const double uvo[2] = {z.x, z.y};
            double r[2], Jc[2][D], Jp[2][3];
            eval_obs<M, true>(camv, X, ppc, uvo, r, Jc, Jp);
            const double sw = huber_weight_sqrt(r[0] * r[0] + r[1] * r[1], delta);
#pragma unroll
            for (int a = 0; a < D; ++a) { row[a] = Jc[0][a] * sw; row[D + a] = Jc[1][a] * sw; }
            row[2 * D] = r[0] * sw;
            row[2 * D + 1] = r[1] * sw;
        }
        __syncthreads();
        const int n = min(kThreads, ee - base);
#pragma unroll
        for (int m = 0; m < EPT; ++m) {
            const int ent = t + m * kThreads;
            if (ent < D * D) {
                const int a = ent / D, b = ent % D;
                double s = acc[m];
                for (int i = 0; i < n; ++i) {
                    const double* rw = sh + (size_t)i * RW;
                    s += rw[a] * rw[b] + rw[D + a] * rw[D + b];
                }
                acc[m] = s;
            } else if (ent < E) {
                const int a = ent - D * D;
                double s = acc[m];
                for (int i = 0; i < n; ++i) {
                    const double* rw = sh + (size_t)i * RW;
                    s -= rw[a] * rw[2 * D] + rw[D + a] * rw[2 * D + 1];
                }
                acc[m] = s;
            }
        }
        __syncthreads();
        X[0] = Xn[0]; X[1] = Xn[1]; X[2] = Xn[2];
        z = zn; pn = pnn; zn = znn;
    }
#pragma unroll
    for (int m = 0; m < EPT; ++m) {
        const int ent = t + m * kThreads;
        if (ent < D * D) U[(size_t)c * D * D + ent] = acc[m];
        else if (ent < E) gc[(size_t)c * D + (ent - D * D)] = acc[m];
    }
}

// Register form of k_lin_cams for D <= 9 (D(D+1)/2 + D accumulators per thread): one workgroup per camera, thread t
// evaluates observations t, t + 256, ... of the camera and keeps its own partial sums of the upper triangle of U and
// of g_c in registers (no per-batch LDS round trip, no 256-long dependent add chain per entry); the partials are then
// summed by a fixed butterfly per wave and the 4 wave sums in wave order, and U is written with both triangles from
// the upper one (a product commutes exactly, so U stays exactly symmetric).  Same point / uv pipeline as k_lin_cams.
template <int M, int NT = LIN_CAMS_NT>
__global__ __launch_bounds__(NT) void k_lin_cams_reg(const int* __restrict__ cam_ptr, const int* __restrict__ cm_pt,
                                                           const double* __restrict__ cm_uv, const double* __restrict__ pp,
                                                           const double* __restrict__ cams, const double* __restrict__ pts,
                                                           double delta, double* __restrict__ U, double* __restrict__ gc) {
    constexpr int D = kD<M>, ST = kStride<M>, NU = D * (D + 1) / 2, NE = NU + D;
    static_assert(D <= 9, "register accumulation is sized for D <= 9");
    constexpr int NW = NT / 64;
    __shared__ double red[NW][NE];
    const int c = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int eb = cam_ptr[c], ee = cam_ptr[c + 1];
    const double2* uv2 = reinterpret_cast<const double2*>(cm_uv);
    double camv[ST];
#pragma unroll
    for (int k = 0; k < ST; ++k) camv[k] = cams[(size_t)c * ST + k];
    const double ppc[2] = {pp[2 * c], pp[2 * c + 1]};
    double acc[NE];
#pragma unroll
    for (int m = 0; m < NE; ++m) acc[m] = 0.0;
    double X[3] = {0.0, 0.0, 0.0};
    double2 z = make_double2(0.0, 0.0), zn = z, znn = z;
    int pn = 0, pnn = 0;
    {
        const int e0 = eb + t, e1 = e0 + NT;
        if (e0 < ee) {
            const int p0 = cm_pt[e0];
            z = uv2[e0];
            X[0] = pts[3 * (size_t)p0]; X[1] = pts[3 * (size_t)p0 + 1]; X[2] = pts[3 * (size_t)p0 + 2];
        }
        if (e1 < ee) { pn = cm_pt[e1]; zn = uv2[e1]; }
    }
    for (int e = eb + t; e < ee; e += NT) {
        const bool hn = e + NT < ee, hnn = e + 2 * NT < ee;
        double Xn[3] = {0.0, 0.0, 0.0};
        if (hn) { Xn[0] = pts[3 * (size_t)pn]; Xn[1] = pts[3 * (size_t)pn + 1]; Xn[2] = pts[3 * (size_t)pn + 2]; }
        if (hnn) { pnn = cm_pt[e + 2 * NT]; znn = uv2[e + 2 * NT]; }
        const double uvo[2] = {z.x, z.y};
        double r[2], Jc[2][D], Jp[2][3];
        eval_obs<M, true>(camv, X, ppc, uvo, r, Jc, Jp);
        const double sw = huber_weight_sqrt(r[0] * r[0] + r[1] * r[1], delta);
#pragma unroll
        for (int a = 0; a < D; ++a) { Jc[0][a] *= sw; Jc[1][a] *= sw; }
        r[0] *= sw; r[1] *= sw;
        int m = 0;
#pragma unroll
        for (int a = 0; a < D; ++a)
#pragma unroll
            for (int b = a; b < D; ++b, ++m) acc[m] += Jc[0][a] * Jc[0][b] + Jc[1][a] * Jc[1][b];
#pragma unroll
        for (int a = 0; a < D; ++a) acc[NU + a] -= Jc[0][a] * r[0] + Jc[1][a] * r[1];
        X[0] = Xn[0]; X[1] = Xn[1]; X[2] = Xn[2];
        z = zn; pn = pnn; zn = znn;
    }
#pragma unroll
    for (int m = 0; m < NE; ++m) {
        const double v = wave_sum(acc[m]);
        if (lane == 0) red[wv][m] = v;
    }
    __syncthreads();
    for (int m = t; m < NE; m += NT) {
        double s = red[0][m];
#pragma unroll
        for (int w = 1; w < NW; ++w) s += red[w][m];
        if (m < NU) {
            int a = 0, rem = m;
            while (rem >= D - a) { rem -= D - a; ++a; }
            const int b = a + rem;
            U[(size_t)c * D * D + a * D + b] = s;
            U[(size_t)c * D * D + b * D + a] = s;
        } else {
            gc[(size_t)c * D + (m - NU)] = s;
        }
    }
}

// ------------------------------------------------------------------------------------------------------------
// per-trial point preparation
// ------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kThreads) void k_point_prep(int Pl, const double* __restrict__ V, const double* __restrict__ gp,
                                                         double f, double cmin, double cmax, double* __restrict__ Vinv,
                                                         double* __restrict__ y, int* __restrict__ flags,
                                                         int* __restrict__ status, const double* __restrict__ R,
                                                         double* __restrict__ Mp) {
    // R non-null (a retried trial on the symmetric records, see PointPrep): M_p = R^T V'^-1 R (packed sym) and
    // z'_p = R^T y'_p into y; else y'_p = V'^-1 g_p (global positioning's re-prep, points-only solves)
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x < 4) status[threadIdx.x] = 0;  // the CG status word of this solve
    if (p >= Pl) return;
    double s[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) s[k] = V[6 * (size_t)p + k];
    s[0] = clampd(s[0], cmin, cmax) * f;
    s[3] = clampd(s[3], cmin, cmax) * f;
    s[5] = clampd(s[5], cmin, cmax) * f;
    double o[6];
    if (!spd3_inverse(s, o)) {
        atomicOr(flags, 1);
#pragma unroll
        for (int k = 0; k < 6; ++k) o[k] = 0.0;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) Vinv[6 * (size_t)p + k] = o[k];
    const double g0 = gp[3 * (size_t)p], g1 = gp[3 * (size_t)p + 1], g2 = gp[3 * (size_t)p + 2];
    const double y0 = o[0] * g0 + o[1] * g1 + o[2] * g2;
    const double y1 = o[1] * g0 + o[3] * g1 + o[4] * g2;
    const double y2 = o[2] * g0 + o[4] * g1 + o[5] * g2;
    if (!R) {
        y[3 * (size_t)p + 0] = y0;
        y[3 * (size_t)p + 1] = y1;
        y[3 * (size_t)p + 2] = y2;
        return;
    }
    const double* r = R + 6 * (size_t)p;
    const double r00 = r[0], r10 = r[1], r20 = r[2], r11 = r[3], r21 = r[4], r22 = r[5];
    // T = V'^-1 R (columns of R: (r00, r10, r20), (0, r11, r21), (0, 0, r22))
    const double Rm[3][3] = {{r00, 0.0, 0.0}, {r10, r11, 0.0}, {r20, r21, r22}};
    const double O[3][3] = {{o[0], o[1], o[2]}, {o[1], o[3], o[4]}, {o[2], o[4], o[5]}};
    double T[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c) T[a][c] = O[a][0] * Rm[0][c] + O[a][1] * Rm[1][c] + O[a][2] * Rm[2][c];
    double Mq[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int c = 0; c < 3; ++c) Mq[a][c] = Rm[0][a] * T[0][c] + Rm[1][a] * T[1][c] + Rm[2][a] * T[2][c];
    double* mo = Mp + 6 * (size_t)p;
    mo[0] = Mq[0][0]; mo[1] = Mq[0][1]; mo[2] = Mq[0][2]; mo[3] = Mq[1][1]; mo[4] = Mq[1][2]; mo[5] = Mq[2][2];
    y[3 * (size_t)p + 0] = r00 * y0 + r10 * y1 + r20 * y2;
    y[3 * (size_t)p + 1] = r11 * y1 + r21 * y2;
    y[3 * (size_t)p + 2] = r22 * y2;
}

// ------------------------------------------------------------------------------------------------------------
// Schur complement: one workgroup per (camera row i, chunk of its upper blocks); the chunk of S's row lives in LDS.
// A group of D lanes owns one of camera i's observations o (64/D observations in flight per wave); lane b of the
// group owns column b.  The group stages the rows of its own record (row b per lane, shared through LDS) -- the BA's
// symmetric record Y_o as it is on the first trial, Y_o M_p on a retried one (PointPrep), global positioning's
// W^_o = W_o V_p^-1 -- then walks the upper partners q of track p -- tracks are sorted by camera at create, so they
// are exactly [ustart[o], end) -- and adds column b of -Y^_o Y_q^T into slot(cam[q]) with LDS f64 atomics
// (ds_add_f64).  b_i -= Y_o z_p (z_p, z'_p: PointPrep) alongside.  Each camera's
// observation list is in point order cut into chunks sorted by partner count (create: the groups of a wave stay
// balanced, and the rows walk the tracks in step).  The kernel is bound by the
// chain of dependent loads per round, not by bytes (cache-resident partner data: no faster): every own-observation
// index comes from one descriptor {o, p, partner range} prefetched a round ahead.  Measured and rejected: a
// precomputed per-pair block position (36 MB streamed per trial, slower than cam[] from cache + an LDS lookup).
// ------------------------------------------------------------------------------------------------------------
// LDS strides of k_schur.  The D groups of a wave add into D different blocks at the same (row, column): with a
// block stride that is a multiple of the 64-bank period (D*D = 64 doubles = 512 B for D = 8) every group lands on the
// same banks (8-way conflicts, SQ_LDS_BANK_CONFLICT ~1.6x the busy cycles); 8 extra doubles spread the groups over 4
// bank quarters.  The W^ staging of each group gets an odd stride for the same reason.
__host__ __device__ constexpr int schur_bs(int D) { return D * D + ((D * D) % 16 == 0 ? 8 : 0); }
__host__ __device__ constexpr int schur_ws(int D) { return D * 4 + 1; }

// Column cb of W_o: the BA stores W [o][3][D]; global positioning (GPW) stores the 32-byte record {u, beta^2} of
// W_o = -beta^2 (I - u u^T) (u = a / sqrt(h_ss), 0 for a fixed scale; symmetric, D = 3) written by k_gp_prep_points.
template <int D, bool GPW>
__device__ __forceinline__ void load_wcol(const double* __restrict__ W, int o, int cb, double& w0, double& w1, double& w2) {
    if constexpr (GPW) {
        const double4 r = reinterpret_cast<const double4*>(W)[o];
        const double uc = cb == 0 ? r.x : (cb == 1 ? r.y : r.z);
        w0 = -r.w * ((cb == 0 ? 1.0 : 0.0) - r.x * uc);
        w1 = -r.w * ((cb == 1 ? 1.0 : 0.0) - r.y * uc);
        w2 = -r.w * ((cb == 2 ? 1.0 : 0.0) - r.z * uc);
    } else {
        const double* wo = W + (size_t)o * D * 3 + cb;
        w0 = wo[0]; w1 = wo[D]; w2 = wo[2 * D];
    }
}

// SCHUR_PROBE (timing-only builds for the floor model of DESIGN.md section 8, tools/schur_variants.sh; wrong results):
//   1  the partner products summed in a register instead of the LDS atomics (gathers + FMAs, no ds_add_f64)
//   2  the partner walk's loads only (records + camera indices; no slot lookup, no FMA, no LDS add)
//   3  no partner-record gathers: the own record stands in for the partner's (camera index, slot lookup, FMAs and
//      LDS adds as usual)
#ifndef SCHUR_PROBE
#define SCHUR_PROBE 0
#endif
template <int D, int WAVES, bool GPW = false, bool RETRY = false, bool ORD = false>
__global__ __launch_bounds__(WAVES * 64, SCHUR_MINW) void k_schur(const int4* __restrict__ work, const int* __restrict__ row_ptr,
                                                      const int* __restrict__ col, int C, const int* __restrict__ cam_ptr,
                                                      const int* __restrict__ cam_obs, const int* __restrict__ ptl,
                                                      const int* __restrict__ pt_ptr, const int* __restrict__ ustart,
                                                      const int4* __restrict__ sdesc,
                                                      const int* __restrict__ cam, const double* __restrict__ W,
                                                      const double* __restrict__ Vinv, const double* __restrict__ y,
                                                      const double* __restrict__ U, const double* __restrict__ gc, double f,
                                                      double cmin, double cmax, int add_diag, double* __restrict__ S,
                                                      double* __restrict__ b, long long* stp) {
    const StampScope stamp_(stp);
    constexpr int DD = D * D;
    constexpr int BS = schur_bs(D);  // LDS stride of an accumulated block (padded off the 64-bank period)
    constexpr int WS = schur_ws(D);  // LDS stride of a group's W^ staging
    constexpr int NG = 64 / D;  // observation groups per wave
    constexpr int NT = WAVES * 64;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    __shared__ int rnd_sh[ORD ? 2 * WAVES : 1];  // (ORD) partner-round counts of the waves, by own-round parity
    const int4 wk = work[blockIdx.x];
    const int i = wk.x, kb = wk.y, ke = wk.z, nb = ke - kb;
    double* acc = sh;
    double* wsh = acc + (size_t)nb * BS;           // [WAVES][NG][WS]  W^ rows ([D][4], padded group stride)
    double* bacc = wsh + (size_t)WAVES * NG * WS;  // [D]
    int* slot = reinterpret_cast<int*>(bacc + D + 12);  // [C]
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int k = t; k < nb * BS; k += NT) acc[k] = 0.0;
    for (int k = t; k < C; k += NT) slot[k] = -1;
    if (t < D) bacc[t] = 0.0;
    __syncthreads();
    for (int e = kb + t; e < ke; e += NT) slot[col[e]] = e - kb;
    __syncthreads();
    const bool diag_chunk = (kb == row_ptr[i]);
    const int g = lane / D, cb = lane - g * D;
    const bool active = g < NG;
    double* my_wh = wsh + (size_t)(wv * NG + (active ? g : 0)) * WS;
    double breg = 0.0;
    double probe_sum = 0.0;  // (SCHUR_PROBE 1 / 2: keeps the probed work alive)
    const int ob = cam_ptr[i], oe = cam_ptr[i + 1];
    // per own observation one descriptor {o, p, partner begin, partner end}: one load gives every index, and the next
    // round's descriptor is loaded while the current round runs (the round chain is latency-bound, not byte-bound)
    int4 dnext = make_int4(0, 0, 0, 0);
    constexpr int UP = ORD ? SCHUR_UP_DET : SCHUR_UP;  // partners in flight per group
    {
        const int e0 = ob + wv * NG + g;
        if (active && e0 < oe) dnext = sdesc[e0];
        if constexpr (ORD) {  // the first own round's partner-round count of each wave
            const int n0 = (active && e0 < oe) ? dnext.w - dnext.z : 0;
            int nr0 = 0;
            while (__builtin_amdgcn_ballot_w64(nr0 * UP < n0) != 0) ++nr0;
            if (lane == 0) rnd_sh[wv] = nr0;
            __syncthreads();
        }
    }
    // ORD (deterministic mode): every wave runs the same number of rounds (own observations, and per own round the
    // workgroup's partner rounds), and in each partner round the waves make their LDS adds in turn (wave 0 first, a
    // barrier between turns), so each slot sees its additions in a fixed order
    // -- lanes of one wave adding into one address within one instruction are ordered by the hardware -- while the
    // waves' gathers stay in flight together
    const int nround = ORD ? (oe - ob + WAVES * NG - 1) / (WAVES * NG) : 0;
    for (int base = ob + wv * NG, rd = 0; ORD ? rd < nround : base < oe; base += WAVES * NG, ++rd) {
        const int e = base + g;
        const bool has = active && e < oe;
        const int4 dcur = dnext;
        {
            const int en = e + WAVES * NG;
            if (active && en < oe) dnext = sdesc[en];
        }
        const int qs = has ? dcur.z : 0, qe = has ? dcur.w : 0;
        const int n = qe - qs;
        // issue order = wait order (vmcnt retires in order): the own record first, then the first UP partner records,
        // so the W^ staging waits only for the own record while the partner loads stay in flight
        double w0 = 0.0, w1 = 0.0, w2 = 0.0, v00 = 0.0, v01 = 0.0, v02 = 0.0, v11 = 0.0, v12 = 0.0, v22 = 0.0;
        if (has) {
            if constexpr (GPW || RETRY) {  // V^-1 (global positioning) or M_p (a retried trial on the Y records)
                const double* vi = Vinv + 6 * (size_t)dcur.y;
                v00 = vi[0]; v01 = vi[1]; v02 = vi[2]; v11 = vi[3]; v12 = vi[4]; v22 = vi[5];
            }
            load_wcol<D, GPW>(W, dcur.x, cb, w0, w1, w2);
        }
        double x[UP][3];
        int cj[UP];
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            cj[u] = -1;
            if (u < n) {
                if (SCHUR_PROBE == 3) { x[u][0] = w0; x[u][1] = w1; x[u][2] = w2; }
                else load_wcol<D, GPW>(W, qs + u, cb, x[u][0], x[u][1], x[u][2]);
                cj[u] = cam[qs + u];
            }
        }
        if (has) {
            // staged negated: the partner products below then come out with the sign S_ij needs (sign-symmetric
            // rounding: bitwise the negation of the positive products) and need no v_xor per row
            if constexpr (GPW || RETRY) {
                my_wh[cb * 4 + 0] = -(w0 * v00 + w1 * v01 + w2 * v02);
                my_wh[cb * 4 + 1] = -(w0 * v01 + w1 * v11 + w2 * v12);
                my_wh[cb * 4 + 2] = -(w0 * v02 + w1 * v12 + w2 * v22);
            } else {  // the first trial on the Y records: S_ij -= Y_o Y_q^T directly
                my_wh[cb * 4 + 0] = -w0;
                my_wh[cb * 4 + 1] = -w1;
                my_wh[cb * 4 + 2] = -w2;
            }
            if (diag_chunk) {
                const double* yp = y + 3 * (size_t)dcur.y;
                breg -= w0 * yp[0] + w1 * yp[1] + w2 * yp[2];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double wh[D][3];
        if (has) {
#pragma unroll
            for (int a2 = 0; a2 < D; ++a2) {
                wh[a2][0] = my_wh[a2 * 4 + 0];
                wh[a2][1] = my_wh[a2 * 4 + 1];
                wh[a2][2] = my_wh[a2 * 4 + 2];
            }
        }
        // rounds while any lane of the wave has partners left: a ballot (scalar compare) instead of a shuffle max of n,
        // which cost six ds_bpermute per own-observation round on the LDS pipe the accumulation already saturates
        // ORD: the workgroup's partner-round count, the most any wave needs.  Each wave writes the next own round's
        // count (from the prefetched descriptor, by round parity) before this round's last barrier: the readers of
        // that buffer slot, two rounds back, have all passed the previous round's last barrier.
        int nrd = 0;
        if constexpr (ORD) {
#pragma unroll
            for (int w2 = 0; w2 < WAVES; ++w2) nrd = max(nrd, rnd_sh[(rd & 1) * WAVES + w2]);
            const int en = e + WAVES * NG;
            const int nn = (active && en < oe) ? dnext.w - dnext.z : 0;
            int nrn = 0;
            while (__builtin_amdgcn_ballot_w64(nrn * UP < nn) != 0) ++nrn;
            if (lane == 0) rnd_sh[((rd + 1) & 1) * WAVES + wv] = nrn;
        }
        for (int k0 = 0; ORD ? k0 < nrd * UP : __builtin_amdgcn_ballot_w64(k0 < n) != 0; k0 += UP) {
            if (k0 > 0) {
#pragma unroll
                for (int u = 0; u < UP; ++u) {
                    cj[u] = -1;
                    if (k0 + u < n) {
                        const int q = qs + k0 + u;
                        if (SCHUR_PROBE == 3) { x[u][0] = w0 + k0; x[u][1] = w1; x[u][2] = w2; }
                        else load_wcol<D, GPW>(W, q, cb, x[u][0], x[u][1], x[u][2]);
                        cj[u] = cam[q];
                    }
                }
            }
#if SCHUR_PROBE == 2
#pragma unroll
            for (int u = 0; u < UP; ++u)
                if (cj[u] >= 0) probe_sum += x[u][0] + x[u][1] + x[u][2] + (double)cj[u];
            continue;
#endif
#if SCHUR_SLOTPRE
            // every slot of the round looked up before the first ds_add_f64: one LDS wait per round instead of one
            // per partner (a slot read issued behind the previous partner's adds waits for them to retire)
            int slv[UP];
#pragma unroll
            for (int u = 0; u < UP; ++u) slv[u] = slot[cj[u] >= 0 ? cj[u] : 0];
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) (vmcnt, expcnt unconstrained): all slots read
            __builtin_amdgcn_sched_barrier(0);
#endif
            // ORD: wave w adds between the w-th and the (w+1)-th of the round's WAVES barriers
            if constexpr (ORD)
                for (int k = 0; k < wv; ++k) __syncthreads();
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                if (cj[u] >= 0) {
#if SCHUR_SLOTPRE
                    const int sl = slv[u];
#else
                    const int sl = slot[cj[u]];
#endif
                    if (sl >= 0) {
                        double* dst = acc + (size_t)sl * BS + cb;
                        const double y0 = x[u][0], y1 = x[u][1], y2 = x[u][2];
#pragma unroll
                        for (int a2 = 0; a2 < D; ++a2) {
                            if (SCHUR_PROBE == 1) probe_sum += wh[a2][0] * y0 + wh[a2][1] * y1 + wh[a2][2] * y2;
                            else atomicAdd(dst + a2 * D, wh[a2][0] * y0 + wh[a2][1] * y1 + wh[a2][2] * y2);
                        }
                    }
                }
            }
            if constexpr (ORD)
                for (int k = wv; k < WAVES; ++k) __syncthreads();
        }
        if (ORD && nrd == 0) __syncthreads();  // (a round without partners: its one barrier)
        __builtin_amdgcn_wave_barrier();
    }
    if constexpr (ORD)
        for (int k = 0; k < wv; ++k) __syncthreads();
    if (diag_chunk && active) atomicAdd(bacc + cb, breg);
    if constexpr (ORD)
        for (int k = wv; k < WAVES; ++k) __syncthreads();
    if (SCHUR_PROBE != 0 && probe_sum == 1.2345e-300) acc[0] = probe_sum;  // (never true: a use of the probed sums)
    __syncthreads();
    double* Sout = S + (size_t)kb * DD;
    const double* Ui = U + (size_t)i * DD;
    for (int k = t; k < nb * DD; k += NT) {
        double v = acc[(k / DD) * BS + k % DD];
        if (diag_chunk && add_diag && k < DD) {
            const int a2 = k / D, bb = k % D;
            double u = Ui[k];
            if (a2 == bb) u = clampd(u, cmin, cmax) * f;
            v += u;
        }
#if SCHUR_NT_STORE
        __builtin_nontemporal_store(v, Sout + k);
#else
        Sout[k] = v;
#endif
    }
    if (diag_chunk && t < D) b[(size_t)i * D + t] = (add_diag ? gc[(size_t)i * D + t] : 0.0) + bacc[t];
}

// ------------------------------------------------------------------------------------------------------------
// PCG on the reduced camera system
// ------------------------------------------------------------------------------------------------------------
// One wave per camera, in registers: lane r holds row r of S_ii and factors it right-looking (pivot and column
// entries broadcast with readlane), so S_ii = L L^T costs D short steps instead of a lane-0 loop over LDS; lane c
// then forms column c of L^-1 by forward substitution, and r0 = L^-1 b, zero p/x/s.  Same operations in the same
// order as the left-looking entry-wise loops (a[c] -= L[r][j] L[c][j] for j ascending, L[r][c] = s / L[c][c],
// I[r][c] = -sum_k L[r][k] I[k][c] / L[r][r]).
// U / g_c (`Ul` non-null): k_schur built S_ii and b_i without the camera terms (k_lin_cams ran beside it on another
// stream), so they are added here -- S_ii += U_i with the diagonal clamped and scaled by the damping factor, b_i =
// g_c + b_i, the same single additions k_schur makes -- and the completed block and right-hand side are written back.
// One camera's factorization on one wave (k_cg_factor's work for camera i).  On return lane r < D holds row r of L_i in
// a[] (zero above the diagonal) and column r of L_i^-1 in x[], and r0 = (L_i^-1 b_i)[lane] (0 when S_ii is not positive
// definite: *ok false, the CG status raised to 2).
template <int D>
__device__ __forceinline__ void factor_camera(int i, int lane, const int* __restrict__ row_ptr, double* __restrict__ S,
                                              double* __restrict__ b, double* __restrict__ Lf, double* __restrict__ Li,
                                              CgBufs& cg, const double* __restrict__ Ul, const double* __restrict__ gcl,
                                              double f, double cmin, double cmax, double (&a)[D], double (&x)[D],
                                              double& r0out, bool& okout) {
    constexpr int DD = D * D;
    const int rl = min(lane, D - 1);
    double* blk = S + (size_t)row_ptr[i] * DD;
#pragma unroll
    for (int c = 0; c < D; ++c) a[c] = blk[rl * D + c];
    double bl = b[(size_t)i * D + rl];
    if (Ul) {
        const double* Ui = Ul + (size_t)i * DD + rl * D;
#pragma unroll
        for (int c = 0; c < D; ++c) {
            double u = Ui[c];
            if (c == rl) u = clampd(u, cmin, cmax) * f;
            a[c] += u;
        }
        bl = gcl[(size_t)i * D + rl] + bl;
        if (lane < D) {
#pragma unroll
            for (int c = 0; c < D; ++c) blk[rl * D + c] = a[c];
            b[(size_t)i * D + rl] = bl;
        }
    }
    bool ok = true;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        double piv = readlane_d(a[j], j);
        if (!(piv > 0.0)) { ok = false; piv = 1.0; }
        const double ljj = sqrt(piv);
        const double lrj = (lane == j) ? ljj : ((lane > j) ? a[j] / ljj : 0.0);
        a[j] = lrj;
#pragma unroll
        for (int c = j + 1; c < D; ++c) {
            const double lcj = readlane_d(lrj, c);
            if (lane >= c) a[c] -= lrj * lcj;
        }
    }
#pragma unroll
    for (int c = 0; c < D; ++c)
        if (c > lane) a[c] = 0.0;
    // column `lane` of L^-1: x[r] = (delta_rc - sum_{k<r} L[r][k] x[k]) / L[r][r]
#pragma unroll
    for (int r = 0; r < D; ++r) {
        double s = 0.0;  // (x[k] = 0 for k < lane: those terms leave s unchanged)
#pragma unroll
        for (int k = 0; k < r; ++k) s -= readlane_d(a[k], r) * x[k];
        x[r] = (r >= lane) ? ((r == lane) ? 1.0 / readlane_d(a[r], r) : s / readlane_d(a[r], r)) : 0.0;
    }
    if (!ok && lane == 0) atomicMax(cg.status, 2);
    if (lane < D) {
#pragma unroll
        for (int c = 0; c < D; ++c) {
            Lf[(size_t)i * DD + lane * D + c] = a[c];
            Li[(size_t)i * DD + c * D + lane] = ok ? x[c] : 0.0;
        }
    }
    // r0 = L^-1 b: row a of L^-1 is (x[a] of lanes 0..a)
    double r0 = 0.0;
#pragma unroll
    for (int aa = 0; aa < D; ++aa) {
        double sacc = 0.0;
#pragma unroll
        for (int k = 0; k <= aa; ++k) sacc += readlane_d(x[aa], k) * readlane_d(bl, k);
        if (lane == aa) r0 = sacc;
    }
    if (lane < D) {
        const size_t idx = (size_t)i * D + lane;
        cg.r[0][idx] = ok ? r0 : 0.0;
        cg.r[1][idx] = 0.0;
        cg.w[0][idx] = 0.0; cg.w[1][idx] = 0.0;
        cg.s[0][idx] = 0.0; cg.s[1][idx] = 0.0;
        cg.p[idx] = 0.0; cg.x[idx] = 0.0;
    }
    okout = ok;
    r0out = ok ? r0 : 0.0;
}

template <int D>
__global__ __launch_bounds__(kThreads) void k_cg_factor(int C, const int* __restrict__ row_ptr, double* __restrict__ S,
                                                        double* __restrict__ b, double* __restrict__ Lf,
                                                        double* __restrict__ Li, CgBufs cg, const double* __restrict__ Ul,
                                                        const double* __restrict__ gcl, double f, double cmin, double cmax,
                                                        long long* stp = nullptr) {
    const StampScope stamp_(stp);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = blockIdx.x * kWaves + wv;
    if (i >= C) return;
    double a[D], x[D], r0;
    bool ok;
    factor_camera<D>(i, lane, row_ptr, S, b, Lf, Li, cg, Ul, gcl, f, cmin, cmax, a, x, r0, ok);
}

// k_cg_factor and k_tl_basis in one launch (round 6), for the persistent CG (k_tl_cgp): the waves take the cameras in
// cluster order -- workgroup g the four cameras k_tl_cgp's workgroup g holds -- and after its factorization each wave
// forms its camera's basis (k_tl_basis's tl_basis_entry: lane k < D + 1 the column k of G_i, Z~_i = L_i^T G_i, the
// restriction partial Z~_i[:,k]^T r0_i) from the factor still in its registers.  The restriction of r0 is summed per
// cluster run of the workgroup (rows in order) into slots 3..11 of the run records `runs` (k_tl_cgp's parity-1 records,
// which it sums per cluster in run order, det_cluster_sums) instead of k_tl_basis's per-cluster tl.Rc: one launch and
// its gap less per solve.
template <int D>
__global__ __launch_bounds__(kThreads) void k_cg_factor_basis(int C, const int* __restrict__ row_ptr, double* __restrict__ S,
                                                              double* __restrict__ b, double* __restrict__ Lf,
                                                              double* __restrict__ Li, CgBufs cg,
                                                              const double* __restrict__ Ul, const double* __restrict__ gcl,
                                                              double f, double cmin, double cmax,
                                                              const double* __restrict__ cams, TlBufs tl,
                                                              double* __restrict__ runs, long long* stp = nullptr) {
    static_assert(kWaves == kCgpRows, "k_cg_factor_basis's workgroups are k_tl_cgp's");
    const StampScope stamp_(stp);
    constexpr int MC = D + 1, ST = D + 1;  // (a BA camera row: pose [t, q] and D - 6 intrinsics)
    __shared__ double prt[kWaves][MC];
    __shared__ int pcl[kWaves];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int pos = blockIdx.x * kWaves + wv;
    const bool has = pos < C;
    const int i = has ? tl.cl_cams[pos] : 0;
    double rr = 0.0;
    if (has) {
        double a[D], x[D], r0;
        bool ok;
        factor_camera<D>(i, lane, row_ptr, S, b, Lf, Li, cg, Ul, gcl, f, cmin, cmax, a, x, r0, ok);
        const int k = min(lane, MC - 1);
        double col[D];
        basis_column<D>(k, cams + (size_t)i * ST, tl.alone[i] != 0, col);
        const bool st = lane < MC;
        const int cp = tl.cpos[i];
#pragma unroll
        for (int aa = 0; aa < D; ++aa) {
            double sz = 0.0;  // Z~[aa][k] = sum_{l >= aa} L[l][aa] G[l][k] (tl_basis_entry's order)
#pragma unroll
            for (int l = aa; l < D; ++l) sz += readlane_d(a[aa], l) * col[l];
            if (st) {
                tl.Zt[((size_t)i * D + aa) * MC + k] = sz;
                if (tl.Gb) tl.Gb[((size_t)i * D + aa) * MC + k] = col[aa];
                tl.Ztc[((size_t)cp * D + aa) * MC + k] = sz;
            }
            rr += sz * readlane_d(r0, aa);
        }
        if (st) tl.rowR[(size_t)cp * MC + k] = rr;
        if (lane < D) tl.vc[(size_t)cp * D + lane] = r0;
    }
    if (lane < MC) prt[wv][lane] = rr;
    if (lane == 0) pcl[wv] = has ? tl.clab[i] : -1;
    __syncthreads();
    if (has && (wv == 0 || pcl[wv - 1] != pcl[wv]) && lane < MC) {
        double v = prt[wv][lane];
        for (int r2 = wv + 1; r2 < kWaves && pcl[r2] == pcl[wv]; ++r2) v += prt[r2][lane];
        runs[(size_t)pos * 12 + 3 + lane] = v;
    }
}

// One wave per scale_nb(D) upper blocks: S~_ij = L_i^-1 S_ij L_j^-T (diagonal blocks -> I).  Off-diagonal blocks are also
// written, padded to DP = D + (D & 1) columns, into the row-contiguous neighbour copy Sn: S~_ij at slot pos_up[e]
// of row i and S~_ij^T at slot pos_lo[e] of row j, so the CG iteration reads every row's blocks as one
// contiguous, 16-byte-coalesced stream.
// Blocks per wave: their loads are issued together (one memory latency per NB blocks); fewer for large D so that the
// staging (3 NB D^2 doubles per wave) leaves several workgroups per CU.
__host__ __device__ constexpr int scale_nb(int D) { return D * D <= 64 ? 4 : (D * D <= 144 ? 2 : 1); }
template <int D>
__global__ __launch_bounds__(kThreads) void k_cg_scale(int nnzb, const int* __restrict__ blk_row, const int* __restrict__ col,
                                                       const int* __restrict__ row_ptr, const int* __restrict__ pos_up,
                                                       const int* __restrict__ pos_lo, const double* __restrict__ Li,
                                                       double* __restrict__ S, double* __restrict__ Sn, int keep_S) {
    constexpr int DD = D * D;
    constexpr int DP = D + (D & 1);
    constexpr int NB = scale_nb(D);
    constexpr int UL = (DD + 63) / 64;  // elements of a block per lane
    __shared__ double T[kWaves][DD];
    __shared__ double Sb[kWaves][NB][DD];
    __shared__ double La[kWaves][NB][DD];
    __shared__ double Lb[kWaves][NB][DD];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int e0 = (blockIdx.x * kWaves + wv) * NB;
    if (e0 >= nnzb) return;
    // every block of the wave and both factors' inverses staged together (all loads in flight at once; indices past
    // the end clamped to the last block, whose products are then not stored)
    int ei[NB], ii[NB], jj[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        ei[u] = min(e0 + u, nnzb - 1);
        ii[u] = blk_row[ei[u]];
        jj[u] = col[ei[u]];
    }
    double sv[NB][UL], av[NB][UL], bv[NB][UL];
#pragma unroll
    for (int u = 0; u < NB; ++u)
#pragma unroll
        for (int q = 0; q < UL; ++q) {
            const int k = min(lane + 64 * q, DD - 1);
            sv[u][q] = S[(size_t)ei[u] * DD + k];
            av[u][q] = Li[(size_t)ii[u] * DD + k];
            bv[u][q] = Li[(size_t)jj[u] * DD + k];
        }
#pragma unroll
    for (int u = 0; u < NB; ++u)
#pragma unroll
        for (int q = 0; q < UL; ++q) {
            const int k = lane + 64 * q;
            if (k < DD) { Sb[wv][u][k] = sv[u][q]; La[wv][u][k] = av[u][q]; Lb[wv][u][k] = bv[u][q]; }
        }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int e = e0 + u;
        if (e >= nnzb) break;
        const int i = ii[u];
        double* blk = S + (size_t)e * DD;
        if (e == row_ptr[i]) {
            if (keep_S)
                for (int k = lane; k < DD; k += 64) blk[k] = (k / D == k % D) ? 1.0 : 0.0;
            continue;
        }
        // same products in the same order as entry-wise loops over global memory
        for (int k = lane; k < DD; k += 64) {
            const int a = k / D, bb = k % D;
            double s = 0.0;
            for (int m = 0; m <= a; ++m) s += La[wv][u][a * D + m] * Sb[wv][u][m * D + bb];
            T[wv][k] = s;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        double* up = Sn + (size_t)pos_up[e] * D * DP;
        double* lo = Sn + (size_t)pos_lo[e] * D * DP;
        for (int k = lane; k < D * DP; k += 64) {
            const int a = k / DP, bb = k % DP;
            double v = 0.0;
            if (bb < D) {
                for (int m = 0; m <= bb; ++m) v += T[wv][a * D + m] * Lb[wv][u][bb * D + m];
                if (keep_S) blk[a * D + bb] = v;  // the scaled upper S is only read by the debug getters
                Sb[wv][u][a * D + bb] = v;
            }
            up[k] = v;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        // transpose: lo[a][bb] = S~_ij[bb][a]
        for (int k = lane; k < D * DP; k += 64) {
            const int a = k / DP, bb = k % DP;
            lo[k] = (bb < D) ? Sb[wv][u][bb * D + a] : 0.0;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

// CG iteration kernel `it` (Chronopoulos-Gear on S~; diagonal blocks of S~ are I).  it = 0 computes w0 = S~ r0 and
// the first dots.  it >= 1 performs recurrence step i = it-1: reads dots_i (per-row partials of kernel it-1), decides
// convergence on the true residual rho_i = ||L r~_i||^2 <= tol^2 ||b||^2, then for its camera row
//   p = r + beta p; s = w + beta s; x += alpha p; r' = r - alpha s; w' = S~ r'
// where every neighbour's r'_j is recomputed from its previous-iteration (r, w, s), so one iteration = ONE launch.
// One 512-thread workgroup per camera row.  The row's neighbour blocks are contiguous in Sn (padded D x DP); lane l of
// a wave owns 16-byte piece (l mod PPB) of block (l / PPB): every load instruction is a contiguous 1 KiB stream.
// Loads that do not depend on alpha / beta (blocks, neighbour vectors, partials, history, own row) are issued first.
// Recurrence scalars for step i = it-1: ONE wave sums the per-row partial dots of launch it-1 in a fixed order
// (16 independent loads in flight per lane per quantity, butterfly across lanes; no barriers), tests convergence on the
// true residual and publishes {alpha, beta, flag} (+ history) for k_cg_iter.
__global__ __launch_bounds__(64) void k_cg_dots(int it, int C, int maxit, double tol2_rel, CgBufs cg) {
    const int lane = threadIdx.x;
    if (cg.status[0] != 0) return;
    const int i = it - 1;
    const double* P0 = cg.part[it & 1 ? 0 : 1];
    const double* P1 = P0 + C;
    const double* P2 = P1 + C;
    double g0 = 0.0, g1 = 0.0, g2 = 0.0;
    for (int base = lane; base < C; base += 64 * 16) {
        double a0[16], a1[16], a2[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int k = base + 64 * u;
            const bool ok = k < C;
            a0[u] = ok ? P0[k] : 0.0;
            a1[u] = ok ? P1[k] : 0.0;
            a2[u] = ok ? P2[k] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) { g0 += a0[u]; g1 += a1[u]; g2 += a2[u]; }
    }
    g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
    const double h_alpha = (i >= 1) ? cg.hist[2 * (i - 1)] : 1.0;
    const double h_gam = (i >= 1) ? cg.hist[2 * (i - 1) + 1] : 1.0;
    const double h_bb = cg.hist[2 * (maxit + 1)];
    if (lane == 0) {
        const double gam = g0, del = g1, rho = g2;
        const double bb = (i == 0) ? rho : h_bb;
        double flag = 0.0, al = 0.0, be = 0.0;
        if (rho <= tol2_rel * bb || i >= maxit) {
            flag = 1.0;
            cg.status[0] = 1; cg.status[1] = i;
        } else {
            double den;
            if (i == 0) { be = 0.0; den = del; }
            else {
                be = gam / h_gam;
                den = del - be * gam / h_alpha;
            }
            if (!(den > 0.0)) {
                flag = 2.0;
                cg.status[0] = 2; cg.status[1] = i;
            } else {
                al = gam / den;
                cg.hist[2 * i] = al;
                cg.hist[2 * i + 1] = gam;
                if (i == 0) cg.hist[2 * (maxit + 1)] = bb;
            }
        }
        cg.scal[0] = al; cg.scal[1] = be; cg.scal[2] = flag;
    }
}

template <int D>
__global__ __launch_bounds__(kCgThreads) void k_cg_iter(int it, int C, int maxit, double tol2_rel,
                                                        const int* __restrict__ nbr_ptr, const int* __restrict__ nbr_j,
                                                        const double* __restrict__ Sn, const double* __restrict__ Lf,
                                                        CgBufs cg) {
    using G = CgGeom<D>;
    constexpr int DD = D * D;
    constexpr int DP = G::DP, HP = G::HP, PPB = G::PPB, BPW = G::BPW, PPL = G::PPL, BPR = G::BPR;
    __shared__ double red[kCgWaves][BPW][PPB];
    __shared__ double rsh[D];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int row = blockIdx.x;
    const int pin = (it + 1) & 1;
    const int pout = it & 1;
    const double* r_old = cg.r[it == 0 ? 0 : pin];
    const double* w_old = cg.w[pin];
    const double* s_old = cg.s[pout];
    const int bw = (PPB <= 64) ? lane / PPB : 0;     // block slot within the wave
    const int pc0 = (PPB <= 64) ? lane - bw * PPB : lane;
    const bool lane_on = (PPB <= 64) ? (bw < BPW) : true;
    const int slot = wv * BPW + bw;                  // block slot within the round
    // ======== phase 1: loads independent of alpha / beta ========
    const int status = cg.status[0];
    const int n0 = nbr_ptr[row], n1 = nbr_ptr[row + 1];
    double acc[PPL];
#pragma unroll
    for (int m = 0; m < PPL; ++m) acc[m] = 0.0;
    // first round prefetch
    double s0[PPL], s1[PPL], xr0[PPL], xr1[PPL], xw0[PPL], xw1[PPL], xs0[PPL], xs1[PPL];
    const int nfirst = n0 + slot;
    const bool have = lane_on && nfirst < n1;
    auto load_piece = [&](int nn, int m, double& a0, double& a1, double& r0, double& r1, double& w0, double& w1, double& q0,
                          double& q1) {
        const int pc = pc0 + 64 * m;
        a0 = a1 = r0 = r1 = w0 = w1 = q0 = q1 = 0.0;
        if (pc >= PPB) return;
        const int b = 2 * (pc % HP);
        const double2 sv = *reinterpret_cast<const double2*>(Sn + ((size_t)nn * D * DP + 2 * (size_t)pc));
        a0 = sv.x; a1 = sv.y;
        const int j = nbr_j[nn];
        const size_t jx = (size_t)j * D + b;
        if constexpr ((D & 1) == 0) {
            const double2 rv = *reinterpret_cast<const double2*>(r_old + jx);
            r0 = rv.x; r1 = rv.y;
            if (it > 0) {
                const double2 wv2 = *reinterpret_cast<const double2*>(w_old + jx);
                const double2 sv2 = *reinterpret_cast<const double2*>(s_old + jx);
                w0 = wv2.x; w1 = wv2.y; q0 = sv2.x; q1 = sv2.y;
            }
        } else {
            r0 = r_old[jx];
            if (b + 1 < D) r1 = r_old[jx + 1];
            if (it > 0) {
                w0 = w_old[jx]; q0 = s_old[jx];
                if (b + 1 < D) { w1 = w_old[jx + 1]; q1 = s_old[jx + 1]; }
            }
        }
    };
    if (have) {
#pragma unroll
        for (int m = 0; m < PPL; ++m) load_piece(nfirst, m, s0[m], s1[m], xr0[m], xr1[m], xw0[m], xw1[m], xs0[m], xs1[m]);
    }
    // wave 0: own row and the row of L (for the true-residual norm)
    double own_r = 0.0, own_w = 0.0, own_s = 0.0, own_p = 0.0;
    double lrow[D];
    const size_t own = (size_t)row * D + (lane < D ? lane : 0);
    if (wv == 0 && lane < D) {
        own_r = r_old[own];
        if (it > 0) { own_w = w_old[own]; own_s = s_old[own]; own_p = cg.p[own]; }
        const double* L = Lf + (size_t)row * DD + lane * D;
#pragma unroll
        for (int k = 0; k < D; ++k) lrow[k] = (k <= lane) ? L[k] : 0.0;
    }
    // recurrence scalars published by k_cg_dots (uniform loads)
    double alpha = 0.0, beta = 0.0;
    if (it > 0) {
        if (cg.scal[2] != 0.0) return;
        alpha = cg.scal[0];
        beta = cg.scal[1];
    }
    if (status != 0) return;
    // ======== phase 3: own row update (wave 0, lanes < D) ========
    double rn = 0.0;
    if (wv == 0 && lane < D) {
        if (it == 0) {
            rn = own_r;
        } else {
            const double sn = own_w + beta * own_s;
            const double pn = own_r + beta * own_p;
            cg.x[own] += alpha * pn;
            cg.p[own] = pn;
            cg.s[pin][own] = sn;
            rn = own_r - alpha * sn;
            cg.r[pout][own] = rn;
        }
        rsh[lane] = rn;
    }
    // ======== phase 4: neighbour blocks, streamed one round (BPR blocks) at a time ========
    auto consume = [&](int m, double a0, double a1, double r0, double r1, double w0, double w1, double q0, double q1) {
        const double v0 = (it == 0) ? r0 : r0 - alpha * (w0 + beta * q0);
        const double v1 = (it == 0) ? r1 : r1 - alpha * (w1 + beta * q1);
        acc[m] += a0 * v0 + a1 * v1;
    };
    if (have) {
#pragma unroll
        for (int m = 0; m < PPL; ++m) consume(m, s0[m], s1[m], xr0[m], xr1[m], xw0[m], xw1[m], xs0[m], xs1[m]);
    }
    for (int nn = nfirst + BPR; lane_on && nn < n1; nn += BPR) {
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            load_piece(nn, m, s0[m], s1[m], xr0[m], xr1[m], xw0[m], xw1[m], xs0[m], xs1[m]);
            consume(m, s0[m], s1[m], xr0[m], xr1[m], xw0[m], xw1[m], xs0[m], xs1[m]);
        }
    }
    if (lane_on) {
#pragma unroll
        for (int m = 0; m < PPL; ++m) {
            const int pc = pc0 + 64 * m;
            if (pc < PPB) red[wv][bw][pc] = acc[m];
        }
    }
    __syncthreads();
    // ======== phase 5: w' for the row and the partial dots (wave 0) ========
    if (wv == 0) {
        double g0 = 0.0, g1 = 0.0, g2 = 0.0;
        if (lane < D) {
            const int a = lane;
            double tot = 0.0;
            for (int w = 0; w < kCgWaves; ++w)
#pragma unroll
                for (int bb = 0; bb < BPW; ++bb)
#pragma unroll
                    for (int k = 0; k < HP; ++k) tot += red[w][bb][a * HP + k];
            const double wn = rn + tot;
            cg.w[pout][own] = wn;
            double lr = 0.0;
#pragma unroll
            for (int k = 0; k < D; ++k) lr += lrow[k] * rsh[k];
            g0 = rn * rn;
            g1 = wn * rn;
            g2 = lr * lr;
        }
        g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
        if (lane == 0) {
            double* pp = cg.part[pout];
            pp[row] = g0; pp[C + row] = g1; pp[2 * (size_t)C + row] = g2;
        }
    }
}

// dc = L^-T x~
template <int D>
__global__ __launch_bounds__(kThreads) void k_cg_finish(int C, const double* __restrict__ Li, const double* __restrict__ xt,
                                                        double* __restrict__ dc, long long* stp) {
    const StampScope stamp_(stp);
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= C * D) return;
    const int i = k / D, a = k % D;
    const double* L = Li + (size_t)i * D * D;
    double s = 0.0;
    for (int m = a; m < D; ++m) s += L[m * D + a] * xt[(size_t)i * D + m];
    dc[k] = s;
}

// ------------------------------------------------------------------------------------------------------------
// back-substitution, parameter update, cost
// ------------------------------------------------------------------------------------------------------------
// Cameras: X <- Exp(dc_pose) X, intrinsics += dc_intr; gain part 2 g_c.dc - dc^T U dc (rank 0 only).  One block of NT
// cameras per call; the block's gain partial goes to part[blk].
template <int M, int NT>
__device__ __forceinline__ void update_cams_block(int blk, int C, const double* __restrict__ cams,
                                                  const double* __restrict__ dc, const double* __restrict__ U,
                                                  const double* __restrict__ gc, int with_gain,
                                                  double* __restrict__ cams_new, double* __restrict__ part,
                                                  double* red /* >= NT / 64 doubles */) {
    constexpr int D = kD<M>, ST = kStride<M>, NI = Model<M>::NI;
    const int c = blk * NT + threadIdx.x;
    double gain[1] = {0.0};
    if (c < C) {
        const double* x = cams + (size_t)c * ST;
        double* o = cams_new + (size_t)c * ST;
        if (dc) {
            const double* d = dc + (size_t)c * D;
            retract_pose(x, d, o);
#pragma unroll
            for (int k = 0; k < NI; ++k) o[7 + k] = x[7 + k] + d[6 + k];
            if (with_gain) {
                const double* Uc = U + (size_t)c * D * D;
                double quad = 0.0, lin = 0.0;
                for (int a = 0; a < D; ++a) {
                    double s = 0.0;
                    for (int bb = 0; bb < D; ++bb) s += Uc[a * D + bb] * d[bb];
                    quad += d[a] * s;
                    lin += gc[(size_t)c * D + a] * d[a];
                }
                gain[0] = 2.0 * lin - quad;
            }
        } else {
#pragma unroll
            for (int k = 0; k < ST; ++k) o[k] = x[k];
        }
    }
    block_sum<1, NT>(gain, red);
    if (threadIdx.x == 0) part[blk] = gain[0];
}

// Back-substitution: dp = V^-1 (g_p - sum_o W_o^T dc_cam(o)) per track, trial points, gain part 2 g_p.dp - dp^T V dp
// (block partial).  Same runs of whole tracks as k_lin_points, one thread per observation; W_o^T dc is re-derived
// instead of read from W: J~ is evaluated again at the linearization point exactly as k_lin_points does (same inputs,
// same code: the same J~c, J~p) and q_o = J~p^T (J~c dc); one thread per track subtracts its q_o in observation order.
// It reads ~50 B per observation (uv, camera / point index, the run's points) instead of the 192-B W record, and the
// evaluation costs less than the record's HBM time (the W-reading form measured 107 vs 64 us on config 3).
template <int M>
__global__ __launch_bounds__(kLinThreads) void k_backsub_rc(const int* __restrict__ blk, const int* __restrict__ pt_ptr,
                                                            const int* __restrict__ cam, const int* __restrict__ ptl,
                                                            const double* __restrict__ uv, const double* __restrict__ pp,
                                                            const double* __restrict__ cams, double delta,
                                                            const double* __restrict__ dc, const double* __restrict__ V,
                                                            const double* __restrict__ Vinv, const double* __restrict__ gp,
                                                            const double* __restrict__ pts, double* __restrict__ dp,
                                                            double* __restrict__ pts_new, double* __restrict__ part,
                                                            int nrun, int C, const double* __restrict__ U,
                                                            const double* __restrict__ gc, int with_gain,
                                                            double* __restrict__ cams_new, double* __restrict__ part_gc,
                                                            long long* stp = nullptr) {
    const StampScope stamp_(stp);
    constexpr int D = kD<M>, ST = kStride<M>;
    __shared__ double red[kLinThreads];
    __shared__ double q[kLinThreads][3];
    if ((int)blockIdx.x >= nrun) {  // the camera update rides along as the launch's last blocks (no separate launch)
        update_cams_block<M, kLinThreads>(blockIdx.x - nrun, C, cams, dc, U, gc, with_gain, cams_new, part_gc, red);
        return;
    }
    const int t = threadIdx.x;
    const int tb = blk[blockIdx.x], te = blk[blockIdx.x + 1];
    const int p = tb + t;
    const bool own = p < te;
    double gain[1] = {0.0};
    double t0 = 0.0, t1 = 0.0, t2 = 0.0;
    if (own) { t0 = gp[3 * (size_t)p]; t1 = gp[3 * (size_t)p + 1]; t2 = gp[3 * (size_t)p + 2]; }
    if (dc) {
        const int ob = pt_ptr[tb], oe = pt_ptr[te];
        const int lo = own ? pt_ptr[p] : 0, hi = own ? pt_ptr[p + 1] : 0;
        for (int base = ob; base < oe; base += kLinThreads) {
            const int n = min(kLinThreads, oe - base);
            if (t < n) {
                const int o = base + t;
                const int c = cam[o], pl = ptl[o];
                const double X[3] = {pts[3 * (size_t)pl], pts[3 * (size_t)pl + 1], pts[3 * (size_t)pl + 2]};
                const double2 z = reinterpret_cast<const double2*>(uv)[o];
                const double uvo[2] = {z.x, z.y};
                const double ppc[2] = {pp[2 * c], pp[2 * c + 1]};
                double d[D];
                const double* dr = dc + (size_t)c * D;
#pragma unroll
                for (int a = 0; a < D; ++a) d[a] = dr[a];
                double r[2], Jc[2][D], Jp[2][3];
                eval_obs<M, true>(cams + (size_t)c * ST, X, ppc, uvo, r, Jc, Jp);
                const double sw = huber_weight_sqrt(r[0] * r[0] + r[1] * r[1], delta);
                double e0 = 0.0, e1 = 0.0;
#pragma unroll
                for (int a = 0; a < D; ++a) { e0 += (Jc[0][a] * sw) * d[a]; e1 += (Jc[1][a] * sw) * d[a]; }
#pragma unroll
                for (int k = 0; k < 3; ++k) q[t][k] = (Jp[0][k] * sw) * e0 + (Jp[1][k] * sw) * e1;
            }
            __syncthreads();
            for (int o = max(lo, base); o < min(hi, base + n); ++o) {
                t0 -= q[o - base][0]; t1 -= q[o - base][1]; t2 -= q[o - base][2];
            }
            __syncthreads();
        }
    }
    if (own) {
        const double* vi = Vinv + 6 * (size_t)p;
        const double d0 = vi[0] * t0 + vi[1] * t1 + vi[2] * t2;
        const double d1 = vi[1] * t0 + vi[3] * t1 + vi[4] * t2;
        const double d2 = vi[2] * t0 + vi[4] * t1 + vi[5] * t2;
        dp[3 * (size_t)p] = d0; dp[3 * (size_t)p + 1] = d1; dp[3 * (size_t)p + 2] = d2;
        pts_new[3 * (size_t)p] = pts[3 * (size_t)p] + d0;
        pts_new[3 * (size_t)p + 1] = pts[3 * (size_t)p + 1] + d1;
        pts_new[3 * (size_t)p + 2] = pts[3 * (size_t)p + 2] + d2;
        const double* v = V + 6 * (size_t)p;
        const double Vd0 = v[0] * d0 + v[1] * d1 + v[2] * d2;
        const double Vd1 = v[1] * d0 + v[3] * d1 + v[4] * d2;
        const double Vd2 = v[2] * d0 + v[4] * d1 + v[5] * d2;
        gain[0] = 2.0 * (t0 * d0 + t1 * d1 + t2 * d2) - (d0 * Vd0 + d1 * Vd1 + d2 * Vd2);
    }
    block_sum<1, kLinThreads>(gain, red);
    if (threadIdx.x == 0) part[blockIdx.x] = gain[0];
}

// Huber loss and sum ||r||^2 (block partials).  (Measured: 4 observations per thread, loads hoisted, ran 25 -> 33 us.)
template <int M>
__global__ __launch_bounds__(kCostThreads) void k_cost(int Nl, const int* __restrict__ cam, const int* __restrict__ ptl,
                                                       const double* __restrict__ uv, const double* __restrict__ pp,
                                                       const double* __restrict__ cams, const double* __restrict__ pts,
                                                       double delta, double* __restrict__ part,
                                                       long long* stp = nullptr) {
    const StampScope stamp_(stp);
    constexpr int ST = kStride<M>;
    __shared__ double red[2 * (kCostThreads / 64)];
    const int o = blockIdx.x * kCostThreads + threadIdx.x;
    double v[2] = {0.0, 0.0};
    if (o < Nl) {
        const int c = cam[o], p = ptl[o];
        const double X[3] = {pts[3 * (size_t)p], pts[3 * (size_t)p + 1], pts[3 * (size_t)p + 2]};
        const double2 z = reinterpret_cast<const double2*>(uv)[o];
        const double uvo[2] = {z.x, z.y};
        const double ppc[2] = {pp[2 * c], pp[2 * c + 1]};
        double r[2];
        eval_obs<M, false>(cams + (size_t)c * ST, X, ppc, uvo, r, nullptr, nullptr);
        const double s = r[0] * r[0] + r[1] * r[1];
        const double rs = sqrt(s);
        v[0] = rs < delta ? s : 2.0 * delta * rs - delta * delta;
        v[1] = s;
    }
    block_sum<2, kCostThreads>(v, red);
    if (threadIdx.x == 0) { part[2 * (size_t)blockIdx.x] = v[0]; part[2 * (size_t)blockIdx.x + 1] = v[1]; }
}

// result[0..4] = {loss, sum ||r||^2, gain_points, gain_cams, #non-PD point blocks}; fixed-order sums of the partials.
// All five are summed across ranks, so every rank takes the same accept / reject / fail branch.
// one 1024-thread workgroup (16 waves: four times the loads in flight of a 256-thread one; 11 -> 5 us on config 3's
// ~40k partials)
constexpr int kFinalThreads = 1024;
__global__ __launch_bounds__(kFinalThreads) void k_final(const double* __restrict__ cost_part, int ncost,
                                                    const double* __restrict__ gp_part, int ngp,
                                                    const double* __restrict__ gc_part, int ngc, int* __restrict__ flags,
                                                    double* __restrict__ result, const int* __restrict__ cgst,
                                                    long long* stp = nullptr) {
    const StampScope stamp_(stp);
    // the three partial arrays in one pass (every load of a round in flight together), each array still summed by
    // each thread in index order and then by the same butterfly and wave order: bitwise the sums of three separate
    // sum_partials passes, with one latency chain instead of three
    __shared__ double red[4 * kFinalThreads / 64];
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    const int ng1 = gp_part ? ngp : 0, ng2 = gc_part ? ngc : 0;
    const int nmax = max(ncost, max(ng1, ng2));
#pragma unroll 4
    for (int i = threadIdx.x; i < nmax; i += kFinalThreads) {
        if (i < ncost) { v[0] += cost_part[2 * (size_t)i]; v[1] += cost_part[2 * (size_t)i + 1]; }
        if (i < ng1) v[2] += gp_part[i];
        if (i < ng2) v[3] += gc_part[i];
    }
    block_sum<4, kFinalThreads>(v, red);
    const double c2[2] = {v[0], v[1]}, a[1] = {v[2]}, b[1] = {v[3]};
    if (threadIdx.x == 0) {
        result[0] = c2[0]; result[1] = c2[1]; result[2] = a[0]; result[3] = b[0];
        result[4] = (double)flags[0];
        // a k_tl_cgp solve whose status the host reads after the cost: 1 when it aborted at a grid barrier (status 4).
        // All-reduced with the other scalars, so every rank of a replicated CG sees whether any rank aborted.
        result[5] = (cgst != nullptr && cgst[0] == 4) ? 1.0 : 0.0;
        flags[0] = 0;  // consumed: the next solve's point preparation starts from a clear flag
    }
}

// flags[0..3] = 0, status[0..3] = 0
// ---- create: structure derived on the device --------------------------------------------------------------------
// Per local track p (observations sorted by camera): each observation's track and the start of its camera run, i.e.
// of its upper partners (the tail of the track from there on).
__global__ __launch_bounds__(kThreads) void k_derive_tracks(int Pl, const int* __restrict__ pt_ptr, const int* __restrict__ cam,
                                                            int* __restrict__ ptl, int* __restrict__ ustart) {
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= Pl) return;
    const int b0 = pt_ptr[p], b1 = pt_ptr[p + 1];
    int u = b0, prev = -1;
    for (int o = b0; o < b1; ++o) {
        const int c = cam[o];
        if (c != prev) { u = o; prev = c; }
        ptl[o] = p;
        ustart[o] = u;
    }
}
// Per camera-major entry e (observation o = cam_obs[e]): the Schur descriptor {o, p, partner begin, partner end} and,
// for the BA, the point and uv the camera linearization reads.
__global__ __launch_bounds__(kThreads) void k_derive_cm(int Nl, const int* __restrict__ cam_obs, const int* __restrict__ ptl,
                                                        const int* __restrict__ ustart, const int* __restrict__ pt_ptr,
                                                        const double* __restrict__ uv, int4* __restrict__ sdesc,
                                                        int* __restrict__ cm_pt, double* __restrict__ cm_uv) {
    const int e = blockIdx.x * kThreads + threadIdx.x;
    if (e >= Nl) return;
    const int o = cam_obs[e], p = ptl[o];
    sdesc[e] = make_int4(o, p, ustart[o], pt_ptr[p + 1]);
    if (uv) {
        cm_pt[e] = p;
        reinterpret_cast<double2*>(cm_uv)[e] = reinterpret_cast<const double2*>(uv)[o];
    }
}

// Upper block pattern of S and the co-visibility weights on the device (create, single rank; the host pass in create
// is the multi-rank / INSFM_DIAG=pattern_host path and gives the same lists): one workgroup per camera row i counts, in
// LDS, for every camera j the (observation of i, observation of j) pairs sharing a track, walking each own
// observation's upper partners [ustart, track end) exactly like k_schur.  `off` null: cnt[i] = #{j > i with pairs};
// else the j > i in increasing order and their pair counts go to nb / wt from off[i] (the second pass recounts).
constexpr int kPatternMaxC = 16384;  // the row's counters in <= 64 KB of LDS
__global__ __launch_bounds__(256) void k_pattern(int C, const int* __restrict__ cam_ptr, const int* __restrict__ cam_obs,
                                                 const int* __restrict__ ustart, const int* __restrict__ ptl,
                                                 const int* __restrict__ pt_ptr, const int* __restrict__ cam,
                                                 int* __restrict__ cnt, const int* __restrict__ off, int* __restrict__ nb,
                                                 int* __restrict__ wt) {
    extern __shared__ int acc[];  // [C]
    __shared__ int wsum[4];
    const int i = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int j = t; j < C; j += 256) acc[j] = 0;
    __syncthreads();
    for (int e = cam_ptr[i] + t; e < cam_ptr[i + 1]; e += 256) {
        const int o = cam_obs[e];
        const int q1 = pt_ptr[ptl[o] + 1];
        for (int q = ustart[o]; q < q1; ++q) {
            const int j = cam[q];
            if (j != i) atomicAdd(&acc[j], 1);  // (the run of camera i itself: the observation and its duplicates)
        }
    }
    __syncthreads();
    if (!off) {
        int c = 0;
        for (int j = i + 1 + t; j < C; j += 256) c += acc[j] > 0;
        for (int d = 32; d > 0; d >>= 1) c += __shfl_xor(c, d);
        if (lane == 0) wsum[w] = c;
        __syncthreads();
        if (t == 0) cnt[i] = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        return;
    }
    int base = off[i];
    for (int j0 = i + 1; j0 < C; j0 += 256) {  // ordered compaction, 256 columns at a time
        const int j = j0 + t;
        const int v = j < C ? acc[j] : 0;
        const unsigned long long bal = __ballot(v > 0);
        if (lane == 0) wsum[w] = __popcll(bal);
        __syncthreads();
        int wo = 0;
        for (int k = 0; k < w; ++k) wo += wsum[k];
        if (v > 0) {
            const int at = base + wo + __popcll(bal & ((1ull << lane) - 1));
            nb[at] = j;
            wt[at] = v;
        }
        base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
    }
}

__global__ void k_zero_words(int* __restrict__ flags, int* __restrict__ status) {
    const int t = threadIdx.x;
    if (t < 4) flags[t] = 0;
    else if (t < 8) status[t - 4] = 0;
}

// After k_final (and the cross-rank sum): result[0..4] into host-mapped memory for the host's spin-wait, then
// sequence word `seq` (system-scope release), so the host reads the trial's cost without a stream synchronization or a
// copy launch.  With `cams_cur` set (insfm_ba_step: the caller's buffers hold the current parameters) the accepted
// trial is copied there in the same launch; the test is lm_step's accept rule on the same doubles (not SPD -> fail;
// last < loss with rejects left -> reject; otherwise accept), and the decision is published in pub[5] for the host to
// check against its own.
__global__ __launch_bounds__(kThreads) void k_publish(const double* __restrict__ result, const int* __restrict__ cgst,
                                                      double* pub, unsigned seq, double last,
                                                      int can_reject, const double* __restrict__ cams_new,
                                                      double* __restrict__ cams_cur, long long ncam,
                                                      const double* __restrict__ pts_new, double* __restrict__ pts_cur,
                                                      long long npts, long long* stp) {
    const StampScope stamp_(stp);
    const double loss = result[0];
    // cgst (a k_tl_cgp solve whose status the host reads afterwards): only a converged CG's trial can be accepted
    // (result[5]: a k_tl_cgp abort on any rank -- every rank then repeats the trial on the launch path)
    const bool acc = result[4] == 0.0 && !(last < loss && can_reject) && (cgst == nullptr || cgst[0] == 1) &&
                     result[5] == 0.0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        for (int k = 0; k < 5; ++k) pub[k] = result[k];
        pub[5] = acc ? 1.0 : 0.0;
        pub[6] = result[5];
        __threadfence_system();
        __hip_atomic_store(reinterpret_cast<unsigned*>(pub + 8), seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (!acc || cams_cur == nullptr) return;
    const long long g = (long long)blockIdx.x * kThreads + threadIdx.x, G = (long long)gridDim.x * kThreads;
    for (long long k = g; k < ncam; k += G) cams_cur[k] = cams_new[k];
    // points: 16-byte pieces (both buffers 16-B aligned: allocations and the shard offset are whole points of 24 B,
    // so the pair path is taken only when both pointers are)
    const bool al = ((reinterpret_cast<uintptr_t>(pts_new) | reinterpret_cast<uintptr_t>(pts_cur)) & 15) == 0;
    if (al) {
        const long long n2 = npts / 2;
        const double2* s2 = reinterpret_cast<const double2*>(pts_new);
        double2* d2 = reinterpret_cast<double2*>(pts_cur);
        for (long long k = g; k < n2; k += G) d2[k] = s2[k];
        if (g == 0 && (npts & 1)) pts_cur[npts - 1] = pts_new[npts - 1];
    } else {
        for (long long k = g; k < npts; k += G) pts_cur[k] = pts_new[k];
    }
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace

// ============================================================================================================
// host side
// ============================================================================================================
struct insfm_ba {
    insfm_ba_desc d{};
    int model = 0, ni = 0, D = 0, stride = 0;
    int C = 0, P = 0, N = 0;
    int p0 = 0, p1 = 0, Pl = 0, o0 = 0, Nl = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // structure (device)
    double *uv = nullptr, *pp = nullptr;
    int *cam = nullptr, *ptl = nullptr, *pt_ptr = nullptr, *cam_ptr = nullptr, *cam_obs = nullptr;
    int *row_ptr = nullptr, *col = nullptr, *blk_row = nullptr, *ustart = nullptr;
    int *nbr_ptr = nullptr, *nbr_j = nullptr, *pos_up = nullptr, *pos_lo = nullptr;
    int4* sdesc = nullptr;  // k_schur: per camera-major own observation {o, p, partner begin, partner end}
    int* cm_pt = nullptr;    // k_lin_cams: per camera-major observation, its (local) point
    int* lin_blk = nullptr;  // k_lin_points: track runs of at most kThreads observations (or one longer track)
    int n_lin = 0;
    double* cm_uv = nullptr; // k_lin_cams: per camera-major observation, its uv
    double* Sn = nullptr;  // row-contiguous scaled neighbour blocks for the CG (both triangles, padded rows)
    int64_t n_nbr = 0;
    int nbr_stride = 0;  // > 0: every CG row has exactly nbr_stride neighbour slots (padded), row r starts at r * stride
    bool flags_dirty = false;  // a solve's point preparation ran and no k_final has consumed (cleared) its flag yet
    int keep_S = 0;      // debug entry points: every solve forms the scaled copy Sn (insfm_ba_debug_get(5) reads S~ from it;
                         // S itself stays unscaled -- k_tl_cgp reads it)
    std::vector<int> pos_up_host;  // [nnzb] Sn slot of each upper block (debug_get(5))
    int4* work = nullptr;
    int nwork = 0, nnzb = 0, max_chunk = 0;
    size_t schur_lds = 0;
    // numeric (device)
    // W: the BA's symmetric records Y_o = W_o L_p (PointPrep; global positioning: its {u, beta^2} records); y: z_p
    // (BA) / y_p (GP); Rf: R_p of the first trial's damped point blocks; Mp: M_p of a retried trial
    double *W = nullptr, *V = nullptr, *gp = nullptr, *Vinv = nullptr, *y = nullptr, *dp = nullptr;
    double *Rf = nullptr, *Mp = nullptr;
    double *xbuf = nullptr;  // [S | b | U | gc | scal]
    double *S = nullptr, *b = nullptr, *U = nullptr, *gc = nullptr, *scal = nullptr;
    int64_t xcount = 0;
    double *Lf = nullptr, *Li = nullptr, *dc = nullptr;
    double* cgmem = nullptr;
    CgBufs cg{};
    int cg_nwg = 0;
    double *cams_cur = nullptr, *cams_new = nullptr, *pts_cur = nullptr, *pts_new = nullptr;
    bool ext_cur = false;  // during insfm_ba_step: cams_cur / pts_cur are the caller's buffers
    bool trial_copied = false;  // the last trial cost's k_publish copied the accepted trial into cams_cur / pts_cur
    double *part_cost = nullptr, *part_gp = nullptr, *part_gc = nullptr;
    int n_cost = 0, n_gp = 0, n_gc = 0;
    int n_gp_grp = 0;  // global positioning: k_gp_backsub blocks (kGPG lanes per track)
    double* result = nullptr;
    int* flags = nullptr;
    double* host_res = nullptr;  // pinned 128 B: result[0..4] (doubles) | cg status (ints, from double slot 8)
    int* prog_host = nullptr;    // pinned, device-mapped: progress of the two-level CG (CgBufs::prog)
    // the last linearization already prepared the points (Vinv, y, status) for damping factor prep_f (PointPrep)
    bool prep_valid = false;
    double prep_f = 0.0;
    double* pub_host = nullptr;  // pinned, device-mapped: k_publish's result[0..4], decision, sequence word (double 8)
    double* pub_dev = nullptr;
    unsigned pub_seq = 0;
    std::vector<void*> allocs;
    // LM state
    double damping = 0.0, down = 0.0, loss = 0.0;
    bool have_loss = false;
    int last_cg_iters = 16;
    hipEvent_t ev[18]{};  // 0-9 phase markers, 10-11 debug timing, 12-15 the side chain's start / end by slot,
                          // 16-17 the chunked exchange's span on the exchange stream
    bool chain_timed[2]{};  // set_timing: the side chain of that slot has timing events not yet harvested
    bool timing = false;
    // device time of the current step, accumulated per phase (ms): see insfm_ba_stats.time_ms
    double tms[8]{};
    int cg_launches = 0;
    bool want_timing = false;       // insfm_ba_set_timing: hipEvent phase timing inside insfm_ba_step
    // two-level preconditioner (desc.precond == 1)
    bool tlon = false;
    TlBufs tl{};
    std::vector<int> clab_host;
    size_t erow_lds = 0, pc_lds = 0;
    int pc_rows = 0;  // k_tl_pc rows per restriction pass
    // the register-resident persistent CG (ba_cgp.h k_tl_cgp): blocks per row (0: not eligible), grid, the w exchange
    // [C][8], the coarse vector [kCoarseMax], the grid-barrier words; cgp_defer: the side chain of slot cgp_slot is
    // issued behind the CG (k_tl_cgp holds every SIMD of its CUs, so a chain beside it would crawl on the rest)
    int cgp_nb = 0, cgp_grid = 0, cgp_slot = 0;
    bool cgp_det = false;                // fixed-order partial sums (deterministic mode, multi-rank replicated CG)
    bool adef2 = false;                  // precond 2: k_tl_cgp applies the coarse correction as A-DEF2 (ba_cgp.h)
    bool basis_by_factor = false;        // this solve's coarse basis was formed by k_cg_factor_basis
    int adef2_fallbacks = 0;             // A-DEF2 solves that broke down and were repeated additively (adef2_fallback)
    double* cgp_runs = nullptr;               // [2][grid * 4][12] the cluster runs' partials by parity (cgp_det)
    int* cgp_src = nullptr;     // [n_nbr] S block of each CG slot: e (upper), ~e (lower, transposed), INT_MIN (pad)
    bool sn_valid = false;      // Sn holds the scaled S~ of the current solve (k_cg_scale ran for it)
    long long* stamps = nullptr;  // INSFM_DIAG=stamps: [kStampSteps][kStKinds][2] kernel entry / exit (wall_clock64)
    long long stamp_step = 0;     // LM steps stamped so far
    unsigned cgp_epochs = 0;  // grid barriers the counters in cgp_sync have counted (reset with them)
    bool cgp_defer = false;
    int cgp_slots = 0;            // workgroups of k_tl_cgp the device holds at once
    bool cg_async = false;        // lm_step: a k_tl_cgp solve's status is read after the trial's k_publish
    bool cgp_pending = false;     // a k_tl_cgp launch whose status the host has not read yet (cgp_complete)
    bool dc_by_cgp = false;       // this solve's k_tl_cgp writes dc itself (cg_tail launches no k_cg_finish)
    bool cgp_lost = false;        // the last k_tl_cgp timed out at a grid barrier (another process holds CUs)
    double* cgp_trace = nullptr;  // INSFM_DIAG=cgp_trace: [64][4] of the last solve, printed to stderr
    // row-partitioned multi-rank CG (ba_xpart.h; insfm_ba_cg_window / insfm_ba_cg_attach)
    bool xpart = false;
    double* xwin = nullptr;            // own window (uncached): 2 x [vc C*D | gd 3C | rowR C*MC + 2], xg C*D, flags
    size_t xwin_bytes = 0;
    long long xoff_region[2]{}, xoff_xg = 0, xoff_flags = 0;  // in doubles from the window base
    std::vector<void*> xopened;        // IPC-opened peer windows (closed at destroy)
    double** xbases = nullptr;         // device [world] window bases (own included)
    unsigned** xpflags = nullptr;      // device [world] flag blocks
    unsigned* xcnt = nullptr;          // device exchange counters [2]
    std::vector<int> xq;               // [world + 1] cluster-ordered row ranges of the ranks
    double* cgp_wx = nullptr;           // [2][C][8]
    unsigned long long* cgp_yg = nullptr;  // [kCoarseMax][2] tagged granules of y
    unsigned cgp_tag = 1;               // tag of the next launch's first iteration
    unsigned* cgp_sync = nullptr;
    bool chain_oseg = false;  // the side chain of slot cgp_slot builds E from k_tl_cgp's segments (reissue_chain)
    // the coarse factorization of solve n runs on `side` while the CG of solve n uses slot (n-1)&1
    double *Ebuf[2]{}, *Einvbuf[2]{};
    double* gjW = nullptr;  // Gauss-Jordan ping-pong buffer [ldE][ldE]
    double* gjP = nullptr;  // Gauss-Jordan pivot-block inverses [2][64][64]
    int* okbuf = nullptr;  // [2]
    hipStream_t side = nullptr;
    hipEvent_t ev_E = nullptr, ev_built = nullptr, ev_fact[2]{};
    // chunked [S | b] exchange (desc.allreduce_async): work-item / row boundaries of the chunks, the exchange stream
    std::vector<int> xw, xr, rptr_host;
    hipStream_t xstream = nullptr;
    // u_late: k_lin_cams runs on `aux` beside k_lin_points / k_schur; k_schur builds S / b without U / g_c and
    // k_cg_factor adds them after waiting for ev_lc (lin_join).  Single-rank W-path only.
    bool u_late = false, lin_pending = false;
    hipStream_t aux = nullptr;
    hipEvent_t ev_lin0 = nullptr, ev_lc = nullptr;
    hipEvent_t ev_x = nullptr, ev_xdone = nullptr;
    hipEvent_t ev_pre = nullptr;  // multi-rank: recorded in front of the CG (its stall deadline starts after it)
    bool built_pending = false;
    long long tl_solves = 0;
    bool tl_fresh = false;  // no solve since the last linearization (the lag rule applies to that solve only)
    int coarse_used = 0;
    // global positioning (kind 1, insfm_gp_*): per local observation ray / scale-free flag / source index, camera
    // factors, the linearization records and the scale-eliminated camera blocks of the current trial
    int kind = 0;
    double *trans = nullptr, *fcam = nullptr, *gobs = nullptr, *Up = nullptr, *gpc = nullptr, *VY = nullptr;
    int *sfree = nullptr, *osrc = nullptr;
    double *scl_cur = nullptr, *scl_new = nullptr, *ds = nullptr;
    std::vector<int> osrc_host;
    std::vector<std::pair<const char*, double>> hmarks;  // INSFM_HOST_TRACE=2
};

namespace {

#define HIPCHK(expr)                                                                              \
    do {                                                                                          \
        hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            h->err = std::string(#expr) + " failed: " + hipGetErrorString(e_);                    \
            return INSFM_BA_EHIP;                                                                 \
        }                                                                                         \
    } while (0)

// INSFM_DIAG: comma-separated diagnostics, read once per process (none is on by default):
//   poison        every buffer dalloc hands out is first filled with 0xff bytes (NaN doubles, -1 ints), so a read of
//                 something never written shows up instead of a fresh allocation's zero pages
//   pattern_host  create builds the block pattern by the host pass (the multi-rank path) on a single rank too
//   trace         per solve, host microseconds spent enqueueing CG iterations (stderr)
//   trace2        per LM step, host timestamps of the step's API calls (stderr)
//   create        host milliseconds of create's phases (stderr)
//   no_cgp        the two-level CG runs as two launches per iteration (k_tl_pc_cl + k_tl_pspmv) even where the
//                 persistent register-resident k_tl_cgp is eligible (A/B and parity of the two paths)
//   cgp_trace     k_tl_cgp records gamma, delta, rho and its stop flag per iteration; printed after each solve
//   cgp128        k_tl_cgp with 128 register blocks per row even for shorter rows (tests the wide variant)
//   own_streams   per-handle side / linearization streams instead of the process-wide ones (A/B)
//   chain_hold    timing only: the lagged coarse-inverse chain is never issued (later solves keep an older E^-1)
//   side_hi / side_normal   the coarse-inverse side stream at the high / normal stream priority (default: lowest)
bool diag(const char* name) {
    static const std::string v = [] { const char* e = std::getenv("INSFM_DIAG"); return std::string(e ? e : ""); }();
    const size_t n = std::strlen(name);
    for (size_t a = 0; a <= v.size();) {
        size_t b = v.find(',', a);
        if (b == std::string::npos) b = v.size();
        if (b - a == n && v.compare(a, n, name) == 0) return true;
        a = b + 1;
    }
    return false;
}

// Process-wide cache of the device buffers of destroyed handles.  TorchBA creates a handle per Solve (the mapper
// solves 4-5 times per reconstruction), and freeing config 3's ~1 GB of buffers took ~7 ms per destroy (hipFree
// synchronizes the device) plus the allocations of the next create.  insfm_ba_destroy waits for the handle's streams
// and parks its buffers here, keyed by their HIP device; dalloc takes the smallest parked buffer of the current device
// of at least the requested size and at most twice it.  Bounded by INSFM_DEVICE_CACHE_MB (default 4096; 0 disables
// it): beyond that, buffers are freed.  The parked memory is invisible to PyTorch's caching allocator, so
// insfm_ba_release_cache() frees it all (TorchBA calls it when torch reports an out-of-memory error, the mapper at the
// end of a reconstruction); a failing hipMalloc inside dalloc releases it too.
struct DeviceCache {
    struct Buf {
        size_t bytes;
        int dev;
        bool uc;  // uncached device memory (hipDeviceMallocUncached)
    };
    std::mutex m;
    std::map<std::pair<int, size_t>, std::vector<void*>> free;  // (2 * device + uncached, size) -> pointers
    size_t bytes = 0;
    std::unordered_map<void*, Buf> info;  // every pointer dalloc handed out (cached or fresh)
};
DeviceCache& device_cache() {
    static DeviceCache* c = new DeviceCache();  // (never destroyed: buffers may be parked until process exit)
    return *c;
}
size_t device_cache_cap() {
    static const size_t v = [] {
        const char* e = std::getenv("INSFM_DEVICE_CACHE_MB");
        return (size_t)(e ? std::max(0LL, std::atoll(e)) : 4096LL) << 20;
    }();
    return v;
}

// frees every parked buffer (any device); returns the bytes released
size_t release_cache() {
    DeviceCache& c = device_cache();
    std::vector<std::pair<void*, int>> drop;
    size_t n = 0;
    {
        std::lock_guard<std::mutex> lk(c.m);
        for (auto& kv : c.free)
            for (void* q : kv.second) {
                drop.emplace_back(q, kv.first.first / 2);
                c.info.erase(q);
            }
        c.free.clear();
        n = c.bytes;
        c.bytes = 0;
    }
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto& d : drop) {
        if (d.second != cur) (void)hipSetDevice(d.second);
        (void)hipFree(d.first);
        if (d.second != cur) (void)hipSetDevice(cur);
    }
    (void)hipGetLastError();
    return n;
}

// Process-wide helper streams, one per (HIP device, role): the side stream of the coarse-inverse chain (role 0, low
// priority) and the camera-linearization stream (role 1).  Every handle of a device shares them, so the number of
// hardware queues a process uses does not grow with the handles alive at once.  With per-handle streams, a TorchBA.Solve
// run while another config-3 handle was alive (bench.py's solve_end_to_end beside its main engine) took 1.9-2.0 ms per
// LM step instead of 1.17: its side chain landed on a queue that the dispatcher served behind k_schur, k_gj_step ran
// 2-4x longer, and the main stream waited ~330 us per step for the lagged coarse inverse (profiles/r5_v1/).  Handles
// on one device are driven one at a time (the reference builds a TorchBA per Solve, global_mapper.py:115), and all
// cross-stream ordering is by the handle's own events, so sharing only serializes what would compete anyway.
// INSFM_DIAG=own_streams restores per-handle streams (A/B).
std::mutex& stream_pool_mutex() {
    static std::mutex* m = new std::mutex();
    return *m;
}
std::map<std::pair<int, int>, hipStream_t>& stream_pool() {
    static auto* p = new std::map<std::pair<int, int>, hipStream_t>();  // (never destroyed, like the device cache)
    return *p;
}
hipError_t helper_stream(int role, int prio, hipStream_t* out) {
    if (diag("own_streams")) return hipStreamCreateWithPriority(out, hipStreamNonBlocking, prio);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(stream_pool_mutex());
    auto& pool = stream_pool();
    auto it = pool.find(std::make_pair(dev, role));
    if (it != pool.end()) {
        *out = it->second;
        return hipSuccess;
    }
    const hipError_t e = hipStreamCreateWithPriority(out, hipStreamNonBlocking, prio);
    if (e == hipSuccess) pool[std::make_pair(dev, role)] = *out;
    return e;
}
void release_helper_stream(hipStream_t s) {
    if (!s) return;
    {
        std::lock_guard<std::mutex> lk(stream_pool_mutex());
        for (auto& kv : stream_pool())
            if (kv.second == s) return;  // pooled: stays for the next handle
    }
    (void)hipStreamDestroy(s);
}

// uc: uncached device memory (the CG's cross-workgroup hand-off buffers: their loads, stores and atomics skip the L2s,
// config 3: 10.4-11.0 -> 9.3-9.7 us per k_tl_cgp iteration; profiles/r4_v7/)
int dalloc(insfm_ba* h, void** p, size_t bytes, bool uc = false) {
    if (bytes == 0) bytes = 16;
    bytes = (bytes + 255) & ~(size_t)255;
    DeviceCache& c = device_cache();
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const int key = 2 * dev + (uc ? 1 : 0);
    bool hit = false;
    {
        std::lock_guard<std::mutex> lk(c.m);
        auto it = c.free.lower_bound(std::make_pair(key, bytes));
        if (it != c.free.end() && it->first.first == key && it->first.second <= 2 * bytes && !it->second.empty()) {
            *p = it->second.back();
            it->second.pop_back();
            c.bytes -= it->first.second;
            if (it->second.empty()) c.free.erase(it);
            hit = true;
        }
    }
    if (hit) {
        h->allocs.push_back(*p);
        if (diag("poison")) (void)hipMemset(*p, 0xff, bytes);
        return 0;
    }
    auto alloc = [&] { return uc ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached) : hipMalloc(p, bytes); };
    hipError_t e = alloc();
    if (e == hipErrorOutOfMemory) {  // give the parked buffers back and try once more
        (void)hipGetLastError();
        release_cache();
        e = alloc();
    }
    if (e != hipSuccess) {
        h->err = std::string("hipMalloc(") + std::to_string(bytes) + ") failed: " + hipGetErrorString(e);
        return INSFM_BA_ENOMEM;
    }
    {
        std::lock_guard<std::mutex> lk(c.m);
        c.info[*p] = DeviceCache::Buf{bytes, dev, uc};
    }
    h->allocs.push_back(*p);
    if (diag("poison")) (void)hipMemset(*p, 0xff, bytes);
    return 0;
}

// the handle's buffers back to the cache (the caller has synchronized every stream that used them)
void dfree_all(insfm_ba* h) {
    DeviceCache& c = device_cache();
    const size_t cap = device_cache_cap();
    std::vector<void*> drop;
    {
        std::lock_guard<std::mutex> lk(c.m);
        for (void* q : h->allocs) {
            auto it = c.info.find(q);
            if (it == c.info.end()) { drop.push_back(q); continue; }
            const DeviceCache::Buf b = it->second;
            if (c.bytes + b.bytes > cap) {
                c.info.erase(it);
                drop.push_back(q);
            } else {
                c.free[std::make_pair(2 * b.dev + (b.uc ? 1 : 0), b.bytes)].push_back(q);
                c.bytes += b.bytes;
            }
        }
    }
    for (void* q : drop) (void)hipFree(q);  // (hipFree takes a pointer of any device)
    h->allocs.clear();
}

template <typename T>
int upload(insfm_ba* h, T** dst, const T* src, size_t n) {
    int rc = dalloc(h, (void**)dst, n * sizeof(T));
    if (rc) return rc;
    if (n) HIPCHK(hipMemcpyAsync(*dst, src, n * sizeof(T), hipMemcpyHostToDevice, h->stream));
    return 0;
}

int model_ni(int m) {
    switch (m) {
        case 0: return 1; case 1: return 2; case 2: return 2; case 3: return 3; case 4: return 6;
        case 5: return 6; case 6: return 10; case 8: return 2; case 9: return 3;
        default: return -1;
    }
}

// ---- model / D dispatch ----------------------------------------------------------------------------------------
template <typename F>
int with_model(int m, F&& f) {
    switch (m) {
        case 0: return f(std::integral_constant<int, 0>{});
        case 1: return f(std::integral_constant<int, 1>{});
        case 2: return f(std::integral_constant<int, 2>{});
        case 3: return f(std::integral_constant<int, 3>{});
        case 4: return f(std::integral_constant<int, 4>{});
        case 5: return f(std::integral_constant<int, 5>{});
        case 6: return f(std::integral_constant<int, 6>{});
        case 8: return f(std::integral_constant<int, 8>{});
        case 9: return f(std::integral_constant<int, 9>{});
        default: return INSFM_BA_EINVAL;
    }
}
template <typename F>
int with_D(int D, F&& f) {
    switch (D) {
        case 3: return f(std::integral_constant<int, 3>{});  // global positioning
        case 7: return f(std::integral_constant<int, 7>{});
        case 8: return f(std::integral_constant<int, 8>{});
        case 9: return f(std::integral_constant<int, 9>{});
        case 12: return f(std::integral_constant<int, 12>{});
        case 16: return f(std::integral_constant<int, 16>{});
        default: return INSFM_BA_EINVAL;
    }
}

int launch_err(insfm_ba* h, const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        h->err = std::string(what) + ": " + hipGetErrorString(e);
        return INSFM_BA_EHIP;
    }
    return 0;
}

int allreduce(insfm_ba* h, double* buf, int64_t n) {
    // a single rank skips the exchange unless a callback is installed (tests drive the RCCL path with one rank)
    if (h->d.world_size <= 1 && !h->d.allreduce) return 0;
    if (!h->d.allreduce) { h->err = "world_size > 1 needs an allreduce callback"; return INSFM_BA_ECOMM; }
    int rc = h->d.allreduce(h->d.allreduce_ctx, buf, n);
    if (rc) { h->err = "allreduce callback failed (" + std::to_string(rc) + ")"; return INSFM_BA_ECOMM; }
    return 0;
}

int allreduce_async(insfm_ba* h, double* buf, int64_t n) {
    int rc = h->d.allreduce_async(h->d.allreduce_ctx, buf, n, h->xstream);
    if (rc) { h->err = "allreduce_async callback failed (" + std::to_string(rc) + ")"; return INSFM_BA_ECOMM; }
    return 0;
}

long long* stamp_ptr(const insfm_ba* h, int kind) {
    if (!h->stamps) return nullptr;
    return h->stamps + ((size_t)(h->stamp_step % kStampSteps) * kStKinds + kind) * 2;
}

void rec(insfm_ba* h, int k) {
    if (h->timing) (void)hipEventRecord(h->ev[k], h->stream);
}

// INSFM_DIAG=trace2: host timestamps of one LM step's API calls (labels + microseconds since the step began),
// printed to stderr when the step ends -- where the host, not the GPU, sets the pace
bool host_trace2() {
    static const bool v = diag("trace2");
    return v;
}
void hmark(insfm_ba* h, const char* what) {
    if (host_trace2()) h->hmarks.emplace_back(what, wall_seconds());
}

// after a stream sync: add the device time between events a and b to phase `slot`
void acc_time(insfm_ba* h, int a, int b, int slot) {
    if (!h->timing) return;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, h->ev[a], h->ev[b]) == hipSuccess) h->tms[slot] += ms;
}

// ---- camera clusters of the two-level preconditioner (same rules as oracle/ba_oracle.c: ora_aggregate) ----------
// Co-visibility weight w(i,j) = number of (obs of i, obs of j) pairs sharing a track.  Greedy aggregation from seeds
// in increasing id, growing by the most-connected unassigned camera (ties: smallest id) up to K members; aggregates
// smaller than K/2 are dissolved into the most-connected aggregate of size >= K/2 (ties: smallest aggregate id);
// labels renumbered by first appearance.
// (built in create's block-pattern pass)
struct CovisGraph {
    std::vector<int> ptr, nb;
    std::vector<long long> w;
};

int aggregate(const CovisGraph& g, int C, int K, std::vector<int>& lab) {
    lab.assign(C, -1);
    std::vector<long long> score(C, 0);
    std::vector<char> incand(C, 0);
    std::vector<int> cand, asize;
    int nagg = 0;
    for (int seed = 0; seed < C; ++seed) {
        if (lab[seed] >= 0) continue;
        cand.clear();
        int size = 0, cur = seed;
        for (;;) {
            lab[cur] = nagg;
            ++size;
            for (int e = g.ptr[cur]; e < g.ptr[cur + 1]; ++e) {
                const int j = g.nb[e];
                if (lab[j] >= 0) continue;
                if (!incand[j]) { incand[j] = 1; score[j] = 0; cand.push_back(j); }
                score[j] += g.w[e];
            }
            if (size >= K) break;
            int best = -1;
            long long bs = 0;
            for (int j : cand) {
                if (lab[j] >= 0) continue;
                if (score[j] > bs || (score[j] == bs && bs > 0 && j < best)) { bs = score[j]; best = j; }
            }
            if (best < 0) break;
            cur = best;
        }
        for (int j : cand) incand[j] = 0;
        asize.push_back(size);
        ++nagg;
    }
    const int minsz = K / 2 > 1 ? K / 2 : 1;
    std::vector<long long> to(nagg, 0);
    std::vector<int> nl(lab);
    for (int i = 0; i < C; ++i) {
        if (asize[lab[i]] >= minsz) continue;
        for (int e = g.ptr[i]; e < g.ptr[i + 1]; ++e) {
            const int a = lab[g.nb[e]];
            if (asize[a] >= minsz) to[a] += g.w[e];
        }
        int best = -1;
        long long bs = 0;
        for (int e = g.ptr[i]; e < g.ptr[i + 1]; ++e) {
            const int a = lab[g.nb[e]];
            if (asize[a] >= minsz && to[a] > 0 && (to[a] > bs || (to[a] == bs && a < best))) { bs = to[a]; best = a; }
        }
        for (int e = g.ptr[i]; e < g.ptr[i + 1]; ++e) to[lab[g.nb[e]]] = 0;
        if (best >= 0) nl[i] = best;
    }
    std::vector<int> ren(nagg, -1);
    int nc = 0;
    for (int i = 0; i < C; ++i) {
        if (ren[nl[i]] < 0) ren[nl[i]] = nc++;
        lab[i] = ren[nl[i]];
    }
    return nc;
}

// ---- phases --------------------------------------------------------------------------------------------------
// The main stream waits for the camera linearization on `aux` (before anything reads U / g_c).
int lin_join(insfm_ba* h) {
    if (!h->lin_pending) return 0;
    HIPCHK(hipStreamWaitEvent(h->stream, h->ev_lc, 0));
    h->lin_pending = false;
    return 0;
}

// The first trial's point preparation of a BA linearization (PointPrep): damping factor f = 1 + damping, records Y
// (and R_p) only when the poses are optimized (points-only solves have no Schur complement).
PointPrep first_trial_prep(insfm_ba* h) {
    PointPrep pp1;
    pp1.f = 1.0 + h->damping;
    pp1.cmin = h->d.clamp_min;
    pp1.cmax = h->d.clamp_max;
    pp1.Vinv = h->Vinv;
    pp1.y = h->y;
    pp1.R = h->d.optimize_poses ? h->Rf : nullptr;
    pp1.flags = h->flags;
    pp1.status = h->cg.status;
    return pp1;
}

template <int M>
void launch_lin_points_w(insfm_ba* h, const double* cams, const double* pts_local, const PointPrep& pp1) {
    k_lin_points<M><<<h->n_lin, kLinThreads, 0, h->stream>>>(h->lin_blk, h->pt_ptr, h->cam, h->ptl, h->uv, h->pp, cams,
                                                         pts_local, h->d.huber_delta, pp1.R ? h->W : nullptr, h->V, h->gp,
                                                         pp1, stamp_ptr(h, kStLinPoints));
}

int run_linearize(insfm_ba* h, const double* cams, const double* pts_local) {
    h->tl_fresh = true;
    if (h->kind == 1) {
        if (h->Nl > 0)
            k_gp_lin<<<cdiv(h->Nl, kThreads), kThreads, 0, h->stream>>>(h->Nl, h->cam, h->ptl, h->trans, h->fcam, h->sfree,
                                                                       cams, pts_local, h->scl_cur, h->d.huber_delta, h->gobs);
        k_gp_lin_cams<<<h->C, kThreads, 0, h->stream>>>(h->C, h->cam_ptr, h->cam_obs, h->gobs, h->U, h->gc);
        int rc = launch_err(h, "k_gp_lin");
        if (rc) return rc;
        return allreduce(h, h->U, (int64_t)h->C * h->D * h->D + (int64_t)h->C * h->D);
    }
    if (int rc0 = lin_join(h)) return rc0;  // (the previous linearization's U / g_c writes come first)
    // The first trial's point preparation rides along with k_lin_points (PointPrep): lm_step's first trial runs at
    // f = 1 + damping (config 3, same box, 3 runs each: 725 / 722 / 701 -> 733 / 725 / 734 LM it/s against a separate
    // k_point_prep launch; profiles/r3_v13/prep_fuse_ab.log).  The records Y_o depend on it (R_p).
    const PointPrep pp1 = first_trial_prep(h);
    h->prep_valid = false;
    if (h->kind == 0 && h->Pl > 0) {
        if (h->flags_dirty) {  // a solve without a cost left the flags / status set: clear them first (k_zero_words)
            k_zero_words<<<1, 64, 0, h->stream>>>(h->flags, h->cg.status);
            if (int e = launch_err(h, "k_zero_words")) return e;
            h->flags_dirty = false;
        }
        h->prep_valid = true;
        h->prep_f = pp1.f;
    }
    hipStream_t cst = h->aux;
    int rc = with_model(h->model, [&](auto mc) -> int {
        constexpr int M = decltype(mc)::value;
        constexpr int D = kD<M>;
        // k_lin_cams (compute-bound) forks after k_lin_points (HBM-bound) so that it overlaps k_schur (bound by
        // gather latency) instead of competing with k_lin_points for bandwidth
        if (h->u_late && h->Pl > 0) launch_lin_points_w<M>(h, cams, pts_local, pp1);
        if (h->u_late) {
            HIPCHK(hipEventRecord(h->ev_lin0, h->stream));
            HIPCHK(hipStreamWaitEvent(h->aux, h->ev_lin0, 0));
            if constexpr (D <= 9) {
                k_lin_cams_reg<M><<<h->C, LIN_CAMS_NT, 0, cst>>>(h->cam_ptr, h->cm_pt, h->cm_uv, h->pp, cams, pts_local,
                                                              h->d.huber_delta, h->U, h->gc);
            } else {
                const size_t lds = sizeof(double) * kThreads * (2 * D + 2);
                k_lin_cams<M><<<h->C, kThreads, lds, cst>>>(h->cam_ptr, h->cm_pt, h->cm_uv, h->pp, cams, pts_local,
                                                            h->d.huber_delta, h->U, h->gc);
            }
            if (int e = launch_err(h, "k_lin_cams")) return e;
            HIPCHK(hipEventRecord(h->ev_lc, h->aux));
            h->lin_pending = true;
            return launch_err(h, "k_lin_points");
        }
        if (h->Pl > 0) launch_lin_points_w<M>(h, cams, pts_local, pp1);
        if constexpr (D <= 9) {
            k_lin_cams_reg<M><<<h->C, LIN_CAMS_NT, 0, h->stream>>>(h->cam_ptr, h->cm_pt, h->cm_uv, h->pp, cams,
                                                                pts_local, h->d.huber_delta, h->U, h->gc);
            return launch_err(h, "linearize");
        }
        const size_t lds = sizeof(double) * kThreads * (2 * D + 2);
        k_lin_cams<M><<<h->C, kThreads, lds, h->stream>>>(h->cam_ptr, h->cm_pt, h->cm_uv, h->pp, cams, pts_local,
                                                          h->d.huber_delta, h->U, h->gc);
        return launch_err(h, "linearize");
    });
    if (rc) return rc;
    return allreduce(h, h->U, (int64_t)h->C * h->D * h->D + (int64_t)h->C * h->D);
}

// Two-level setup, part 1: coarse basis Z~ (on `basis_stream`, the CG needs it) and E into slot `slot` (on
// `build_stream`, which must already be ordered after the basis).
int run_tl_basis(insfm_ba* h, const double* cams, hipStream_t stream) {
    const int C = h->C;
    if (h->kind == 1) {
        k_tl_basis<kGP><<<h->tl.nc, kThreads, 0, stream>>>(C, cams, h->Lf, h->tl, h->cg.r[0]);
        return launch_err(h, "k_tl_basis");
    }
    return with_model(h->model, [&](auto mc) -> int {
        constexpr int M = decltype(mc)::value;
        constexpr int MC = kD<M> + 1;
        k_tl_basis<M><<<h->tl.nc, kThreads, 0, stream>>>(C, cams, h->Lf, h->tl, h->cg.r[0], stamp_ptr(h, kStBasis));
        (void)MC;
        return launch_err(h, "k_tl_basis");
    });
}

// The side stream's E build runs with at most kErowGrid workgroups (rows strided over the grid): with one workgroup
// per row it held CU / LDS slots the overlapping CG launches needed (config 3, round 1: grid 1000 / 512 / 384 / 256 /
// 192 / 128 -> 593 / 616 / 612-615 / 603 / 594 LM it/s).
constexpr int kErowGrid = 256;
int run_tl_build(insfm_ba* h, int slot, hipStream_t stream, bool have_oseg = false) {
    const int C = h->C, m = h->tl.m;
    TlBufs tl = h->tl;
    tl.E = h->Ebuf[slot];
    return with_D(h->D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        const int grid = stream != h->stream ? std::min(C, kErowGrid) : C;
        if (!have_oseg)  // (k_tl_cgp wrote the segments of this solve)
            k_tl_erow<DV><<<grid, kThreads, h->erow_lds, stream>>>(C, h->nbr_ptr, h->nbr_j, h->Sn, tl);
        k_tl_ereduce<DV><<<cdiv(m * m, kThreads), kThreads, 0, stream>>>(tl);
        return launch_err(h, "k_tl_erow/ereduce");
    });
}

// Two-level setup, part 2: unit u of E_slot's Gauss-Jordan inversion on `stream` (launch_gj_unit; the last writes
// Einvbuf[slot]).
int run_tl_gj_unit(insfm_ba* h, int slot, int u, hipStream_t stream) {
    launch_gj_unit(u, h->tl.m, h->Ebuf[slot], h->gjW, h->gjP, h->tl.Ed, h->Einvbuf[slot], h->okbuf + slot, stream);
    return launch_err(h, "k_gj_pinv0/k_gj_step");
}

// Per solve (after k_cg_factor / k_cg_scale on the main stream): the basis Z~ on the main stream, then E_n's build
// (reads S~ and Z~) and factorization on the side stream.  The CG is pointed at the coarse inverse of the previous
// solve when this is the first solve after a linearization (it starts right away), otherwise at its own (it waits
// for the factorization) -- the oracle's lag rule (ora_pcg).  The next solve's k_cg_scale / k_tl_basis overwrite
// S~ / Z~, so they wait for ev_built (run_solve).
// CG iterations the host keeps queued ahead of the device: 1 since late round 3 (config 3, same box, 3 runs each:
// 2 / 1 / 0 -> 714-721 / 722-726 / 720-727 LM it/s; every queued iteration a converged CG still runs costs ~9 us;
// profiles/r3_v12/cg_ahead_ab.log)
#ifndef CG_AHEAD
#define CG_AHEAD 1
#endif
#ifndef CG_INIT_BACK
#define CG_INIT_BACK 2
#endif
constexpr int kCgAhead = CG_AHEAD;

// The side-stream chain of solve `slot`: wait for the basis (ev_E), the E build (k_tl_erow, k_tl_ereduce), ev_built,
// then the Gauss-Jordan launches, the last followed by ev_fact[slot].  The whole chain (~20 launches) is issued at the
// solve's setup, while the GPU is still in k_lin_points / k_schur: the host is then ~0.6 ms ahead of the GPU, the
// launches cost the GPU nothing, and the chain overlaps the CG.  (Round 2 issued it piecemeal from the CG poll loop,
// and a chain deferred past the CG was measured too: both slower)
// set_timing: the device time of finished side chains (start after the wait on ev_E, end after the last Gauss-Jordan
// unit) into phase slot 6 of the current step.  A chain issued behind the CG usually finishes during the next step, so
// it is counted there; summed over the steps of a run every chain is counted once (but the last one).
void harvest_chain_time(insfm_ba* h) {
    for (int sl = 0; sl < 2; ++sl) {
        if (!h->chain_timed[sl] || hipEventQuery(h->ev[14 + sl]) != hipSuccess) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, h->ev[12 + sl], h->ev[14 + sl]) == hipSuccess) h->tms[6] += ms;
        h->chain_timed[sl] = false;
    }
}

int issue_side_chain(insfm_ba* h, int slot, bool have_oseg = false) {
    hipStream_t fs = h->side;
    HIPCHK(hipStreamWaitEvent(fs, h->ev_E, 0));
    const bool tm = h->timing && !h->chain_timed[slot];
    if (tm) HIPCHK(hipEventRecord(h->ev[12 + slot], fs));
    if (int rc = run_tl_build(h, slot, fs, have_oseg)) return rc;
    h->chain_oseg = have_oseg;
    HIPCHK(hipEventRecord(h->ev_built, fs));
    h->built_pending = true;
    for (int u = 0; u <= gj_steps(h->tl.m); ++u)
        if (int rc = run_tl_gj_unit(h, slot, u, fs)) return rc;
    HIPCHK(hipEventRecord(h->ev_fact[slot], fs));
    if (tm) {
        HIPCHK(hipEventRecord(h->ev[14 + slot], fs));
        h->chain_timed[slot] = true;
    }
    return 0;
}

// Everything of the side chain finished (debug getters, kernel timing, destroy, reset).
int side_flush(insfm_ba* h) {
    if (h->side) HIPCHK(hipStreamSynchronize(h->side));
    return 0;
}

// Per-solve setup on the main stream: the basis, then this solve's side chain; the CG uses the previous solve's
// E^-1 under the lag rule, else its own (the main stream waits for the factorization).
int run_tl_setup(insfm_ba* h, const double* cams) {
    const int slot = (int)(h->tl_solves & 1);
    if (h->timing) harvest_chain_time(h);
    int rc = h->basis_by_factor ? 0 : run_tl_basis(h, cams, h->stream);  // (k_cg_factor_basis formed it)
    if (rc) return rc;
    const int use = (h->tl_solves > 0 && h->tl_fresh) ? (slot ^ 1) : slot;
    h->tl_fresh = false;
    // k_tl_cgp under the lag rule: this solve's chain runs after the CG (run_tl_cg records ev_E behind the CG; an
    // event record here as well would only cost the main queue a marker); else it runs now and the CG waits
    h->cgp_defer = h->cgp_nb && use != slot;
    h->cgp_slot = slot;
    if (!h->cgp_defer) {
        HIPCHK(hipEventRecord(h->ev_E, h->stream));
        if ((rc = issue_side_chain(h, slot))) return rc;
    }
    // a lagged solve's coarse inverse normally finished long ago: a completed event needs no wait marker in the main
    // queue (each one idles it a few us; always queueing it measured 659-665 vs 659-664 LM it/s, round 2)
    if (use == slot || hipEventQuery(h->ev_fact[use]) != hipSuccess)
        HIPCHK(hipStreamWaitEvent(h->stream, h->ev_fact[use], 0));
    h->tl.Einv = h->Einvbuf[use];
    h->tl.ok = h->okbuf + use;
    ++h->tl_solves;
    return 0;
}

// Launch `it` of the two-level CG: update (recurrence step it-1 when it >= 1; restriction always), coarse
// correction, S~ u.
template <int D>
void launch_tl_iter(insfm_ba* h, int it, int maxit, double tol2) {
    if (it == 0) {  // setup: restriction of r0, u0 = M~^-1 r0, w0 = S~ u0 and the partials of iteration 0
        // (the restriction of r0 was formed by k_tl_basis)
        k_tl_pc<D><<<h->tl.nc, kPcThreads, h->pc_lds, h->stream>>>(-1, h->C, maxit, tol2, h->pc_rows, h->cg, h->tl,
                                                                   h->tl.Einv);
        k_tl_pspmv<D><<<h->C, kPspmvThreads, 0, h->stream>>>(-1, h->C, h->nbr_stride, h->nbr_ptr, h->nbr_j, h->Sn, h->Lf,
                                                              h->cg, h->tl, XPart{});
    }
    if (h->tl.Racc)  // per-cluster atomic sums of the row partials (single rank, non-deterministic)
        k_tl_pc_cl<D><<<h->tl.nc, kPcThreads, 0, h->stream>>>(it, h->C, maxit, tol2, h->cg, h->tl, h->tl.Einv);
    else
        k_tl_pc<D><<<h->tl.nc, kPcThreads, h->pc_lds, h->stream>>>(it, h->C, maxit, tol2, h->pc_rows, h->cg, h->tl,
                                                                   h->tl.Einv);
    k_tl_pspmv<D><<<h->C, kPspmvThreads, 0, h->stream>>>(it, h->C, h->nbr_stride, h->nbr_ptr, h->nbr_j, h->Sn, h->Lf,
                                                          h->cg, h->tl, XPart{});
}

// TlBufs whose exchanged buffers (vc, gd, rowR) are window region q of a partitioned handle
TlBufs tl_region(const insfm_ba* h, int q) {
    TlBufs t = h->tl;
    const int C = h->C, D = h->D, MC = D + 1;
    double* base = h->xwin + h->xoff_region[q];
    t.vc = base;
    t.gd = base + (size_t)C * D;
    t.rowR = base + (size_t)C * D + 3 * (size_t)C;
    (void)MC;
    return t;
}

XPart xpart_region(const insfm_ba* h, int q) {
    XPart xp;
    xp.win = h->xbases;
    xp.world = h->d.world_size;
    xp.q0 = h->xq[h->d.rank];
    xp.off_vc = h->xoff_region[q];
    xp.off_gd = xp.off_vc + (long long)h->C * h->D;
    xp.off_rowR = xp.off_gd + 3LL * h->C;
    return xp;
}

// One exchange of the partitioned CG (slot 0: iterations, skipped once the CG status is set; 1: solution gather)
void launch_xchg(insfm_ba* h, int slot) {
    k_xsignal<<<1, 64, 0, h->stream>>>(h->cg.status, h->xcnt, h->xpflags, h->d.world_size, h->d.rank, slot);
    k_xwait<<<1, 64, 0, h->stream>>>(h->cg.status, h->cg.prog, h->xcnt,
                                     reinterpret_cast<unsigned*>(h->xwin + h->xoff_flags), h->d.world_size, slot);
}

// launch_tl_iter for a row-partitioned handle: k_tl_pc replicated on region it & 1, this rank's rows of k_tl_pspmv
// writing region (it + 1) & 1 of every window, then the exchange
template <int D>
void launch_tl_iter_x(insfm_ba* h, int it, int maxit, double tol2) {
    const int nrows = h->xq[h->d.rank + 1] - h->xq[h->d.rank];
    auto pspmv = [&](int i) {
        if (nrows > 0)
            k_tl_pspmv<D><<<nrows, kPspmvThreads, 0, h->stream>>>(i, h->C, h->nbr_stride, h->nbr_ptr, h->nbr_j, h->Sn,
                                                                  h->Lf, h->cg, tl_region(h, i & 1),
                                                                  xpart_region(h, (i + 1) & 1));
        launch_xchg(h, 0);
    };
    if (it == 0) {  // setup (k_tl_basis wrote r0 and its restriction into region 1)
        k_tl_pc<D><<<h->tl.nc, kPcThreads, h->pc_lds, h->stream>>>(-1, h->C, maxit, tol2, h->pc_rows, h->cg,
                                                                   tl_region(h, 1), h->tl.Einv);
        pspmv(-1);
    }
    k_tl_pc<D><<<h->tl.nc, kPcThreads, h->pc_lds, h->stream>>>(it, h->C, maxit, tol2, h->pc_rows, h->cg,
                                                               tl_region(h, it & 1), h->tl.Einv);
    pspmv(it);
}

// The k_tl_cgp instantiation for NB blocks per row (64 / 128), the fixed-order form (det) and A-DEF2 (adef).
using CgpKernel = void (*)(int, const int*, const int*, const double*, const int*, const double*, const double*, CgBufs,
                           TlBufs, const double*, int, double, double*, unsigned long long*, unsigned, unsigned*, unsigned,
                           int, double*, double*, double*, long long*);
CgpKernel cgp_kernel(int nb, bool det, bool adef) {
    if (nb == 64) {
        if (det) return adef ? k_tl_cgp<64, true, true> : k_tl_cgp<64, true, false>;
        return adef ? k_tl_cgp<64, false, true> : k_tl_cgp<64, false, false>;
    }
    if (det) return adef ? k_tl_cgp<128, true, true> : k_tl_cgp<128, true, false>;
    return adef ? k_tl_cgp<128, false, true> : k_tl_cgp<128, false, false>;
}

// The whole two-level CG of a solve on the persistent k_tl_cgp (D = 8, h->cgp_nb > 0): one launch for the coarse
// solve of r0 (u0 = M~^-1 r0, formerly k_tl_pc's setup launch), the setup's operator product and every iteration.
int launch_tl_cgp(insfm_ba* h, int maxit, double tol2) {
    if (h->cgp_epochs > (1u << 24)) {  // (counter headroom: zero them now and then; an abort zeroes them too)
        HIPCHK(hipMemsetAsync(h->cgp_sync, 0, sizeof(unsigned) * kCgpSyncWords, h->stream));
        h->cgp_epochs = 0;
    }
    // INSFM_DIAG=cgp_fault (tests): the first launch of the process aborts at iteration 2
    static std::atomic<int> faults{diag("cgp_fault") ? 1 : 0};
    const bool fault = faults.load() > 0 && faults.fetch_sub(1) > 0;
    // INSFM_DIAG=adef2_breakdown (tests): the first A-DEF2 launch of the process reports a breakdown at iteration 2
    static std::atomic<int> bkdn{diag("adef2_breakdown") ? 1 : 0};
    const bool breakdown = h->adef2 && bkdn.load() > 0 && bkdn.fetch_sub(1) > 0;
    hipLaunchKernelGGL(cgp_kernel(h->cgp_nb, h->cgp_det, h->adef2), dim3(h->cgp_grid), dim3(kCgpThreads), 0, h->stream,
                       h->C, h->nbr_ptr, h->nbr_j, (const double*)h->S, (const int*)h->cgp_src, (const double*)h->Li,
                       (const double*)h->Lf, h->cg, h->tl, (const double*)h->tl.Einv, maxit, tol2, h->cgp_wx, h->cgp_yg,
                       h->cgp_tag, h->cgp_sync, h->cgp_epochs,
                       (h->cgp_defer ? 1 : 0) | (fault ? 2 : 0) | (breakdown ? 4 : 0) | (h->basis_by_factor ? 0 : 8),
                       h->cgp_runs, h->cgp_trace, h->dc,
                       stamp_ptr(h, kStCgp));
    return launch_err(h, "k_tl_cgp");
}

// k_schur for the handle's kind (BA: template on D; global positioning: D = 3 with the compact W record).
int launch_schur(insfm_ba* h, const double* Uin, const double* gcin, double sf, double smin, double smax, int sdiag,
                 bool retry, int w0 = 0, int w1 = -1) {
    const bool det = h->d.deterministic != 0;
    if (w1 < 0) w1 = h->nwork;
    const int nt = det ? kDetWaves * 64 : kSchurWaves * 64;
    if (h->kind == 1) {
        if (det)
            k_schur<3, kDetWaves, true, false, SCHUR_DET_ORD><<<h->nwork, nt, h->schur_lds, h->stream>>>(
                h->work, h->row_ptr, h->col, h->C, h->cam_ptr, h->cam_obs, h->ptl, h->pt_ptr, h->ustart, h->sdesc, h->cam, h->W,
                h->Vinv, h->y, Uin, gcin, sf, smin, smax, sdiag, h->S, h->b, nullptr);
        else
            k_schur_gp<kSchurWaves, kGPSG><<<h->nwork, nt, h->schur_lds, h->stream>>>(
                h->work, h->row_ptr, h->col, h->C, h->cam_ptr, h->sdesc, h->cam, h->W, h->VY, Uin, gcin, h->S, h->b);
        return launch_err(h, "k_schur");
    }
    return with_D(h->D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        if (w1 <= w0) return 0;
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3(w1 - w0), dim3(nt), h->schur_lds, h->stream,
                h->work + w0, h->row_ptr, h->col, h->C, h->cam_ptr, h->cam_obs, h->ptl, h->pt_ptr, h->ustart, h->sdesc, h->cam,
                h->W, h->Mp, h->y, Uin, gcin, sf, smin, smax, sdiag, h->S, h->b, stamp_ptr(h, kStSchur));
        };
        if (det) retry ? go(k_schur<DV, kDetWaves, false, true, SCHUR_DET_ORD>) : go(k_schur<DV, kDetWaves, false, false, SCHUR_DET_ORD>);
        else retry ? go(k_schur<DV, kSchurWaves, false, true>) : go(k_schur<DV, kSchurWaves>);
        return launch_err(h, "k_schur");
    });
}

// The k_tl_cgp launch of this solve has finished (the host saw its status word, or the trial's k_publish behind
// it): its status {status, iterations, coarse used} into st, the barrier bookkeeping, an abort's fallback, the trace.
int cgp_complete(insfm_ba* h, int* st) {
    std::atomic_thread_fence(std::memory_order_seq_cst);
    volatile int* pg = h->prog_host;
    st[0] = pg[1]; st[1] = pg[2]; st[2] = pg[3];
    {  // the barriers this launch counted: one per completed iteration; an abort restarts the counters
        if (st[0] == 1 || st[0] == 2) {
            // (the setup's two barriers and one per completed iteration; A-DEF2: three and two)
            h->cgp_epochs += h->adef2 ? 2u * (unsigned)st[1] + 3u : (unsigned)st[1] + 2u;
        } else {
            HIPCHK(hipStreamSynchronize(h->stream));
            HIPCHK(hipMemsetAsync(h->cgp_sync, 0, sizeof(unsigned) * kCgpSyncWords, h->stream));
            h->cgp_epochs = 0;
            // a barrier timed out: the grid was not resident at once (another process's kernels held CUs).  A single
            // rank drops the persistent CG for good and run_solve repeats this solve on the launch path; a rank of a
            // replicated multi-rank CG cannot (its peers would compute a dc that differs in rounding) and reports it.
            if (st[0] == 4 && h->d.world_size <= 1 && !h->xpart) {
                std::fprintf(stderr, "[insfm] k_tl_cgp: a grid barrier timed out (the GPU is shared with another "
                                     "process?); this handle continues on the launch-per-iteration CG\n");
                h->cgp_nb = 0;
                h->cgp_lost = true;
            }
        }
    }
    if (h->cgp_trace) {
        double tr[kCgpTraceLen];
        HIPCHK(hipMemcpy(tr, h->cgp_trace, sizeof(tr), hipMemcpyDeviceToHost));
        const int n = std::min(st[1], 63);
        std::fprintf(stderr, "[insfm cgp] status %d iterations %d coarse %d: setup %.1f us (blocks + tables %.1f, A %.1f, "
                     "rest %.1f), iterations %.1f us (%.2f us each)\n",
                     st[0], st[1], st[2], 0.01 * (tr[257] - tr[256]), 0.01 * (tr[578] - tr[256]),
                     0.01 * (tr[579] - tr[578]), 0.01 * (tr[257] - tr[579]), 0.01 * (tr[258 + n] - tr[257]),
                     n > 0 ? 0.01 * (tr[258 + n] - tr[258]) / n : 0.0);
        for (int k = 0; k <= n; ++k) {
            std::fprintf(stderr, "[insfm cgp]   it %d gamma %.17g delta %.17g rho %.17g done %g t %.1f us | loads %.2f P1 %.2f y %.2f "
                         "P2 %.2f B2 %.2f\n", k, tr[4 * k], tr[4 * k + 1], tr[4 * k + 2], tr[4 * k + 3], 0.01 * (tr[258 + k] - tr[256]),
                         k > 0 ? 0.01 * (tr[258 + k] - tr[322 + 4 * (k - 1) + 3]) : 0.0,
                         0.01 * (tr[322 + 4 * k] - tr[258 + k]), 0.01 * (tr[323 + 4 * k] - tr[322 + 4 * k]),
                         0.01 * (tr[324 + 4 * k] - tr[323 + 4 * k]), 0.01 * (tr[325 + 4 * k] - tr[324 + 4 * k]));
            if (k < n)
                std::fprintf(stderr, "[insfm cgp]        P1 split: fills + workgroup barrier %.2f, y %.2f, S~w %.2f; "
                             "scalar partials in %.2f after the barrier\n",
                             0.01 * (tr[580 + 3 * k] - tr[258 + k]), 0.01 * (tr[581 + 3 * k] - tr[580 + 3 * k]),
                             0.01 * (tr[322 + 4 * k] - tr[581 + 3 * k]),
                             k > 0 ? 0.01 * (tr[582 + 3 * k] - tr[322 + 4 * (k - 1) + 3]) : 0.0);
        }
        const int G = std::min(h->cgp_grid, 256);
        if (st[1] > kCgpTraceIt + 1 && G > 0) {  // every workgroup's start and end of iteration kCgpTraceIt
            double s0 = tr[772], s1 = tr[772];
            for (int b = 0; b < G; ++b) { s0 = std::min(s0, tr[772 + b]); s1 = std::max(s1, tr[772 + b]); }
            std::vector<int> ord(G);
            for (int b = 0; b < G; ++b) ord[b] = b;
            std::sort(ord.begin(), ord.end(), [&](int a, int b) { return tr[1028 + a] > tr[1028 + b]; });
            std::fprintf(stderr, "[insfm cgp] it %d per workgroup: starts within %.2f us; arrival at the barrier "
                         "(us after the first start): median %.2f, last %.2f; latest:", kCgpTraceIt, 0.01 * (s1 - s0),
                         0.01 * (tr[1028 + ord[G / 2]] - s0), 0.01 * (tr[1028 + ord[0]] - s0));
            for (int q = 0; q < std::min(G, 8); ++q)
                std::fprintf(stderr, " wg %d (%.2f, start %.2f)", ord[q], 0.01 * (tr[1028 + ord[q]] - s0),
                             0.01 * (tr[772 + ord[q]] - s0));
            std::fprintf(stderr, "\n");
        }
    }
    return 0;
}


// The two-level CG (precond 1): iterations enqueued from a host poll loop, no stream sync inside the CG.  k_tl_pc's
// lead workgroup publishes its progress into host-mapped memory; more iterations are enqueued while the GPU has fewer
// than kCgAhead pending, and the loop ends when the status word turns non-zero.  The few iterations enqueued past
// convergence exit at the device status flag.  Returns 0 with st[0..2] = {status, iterations, coarse used}.
int run_tl_cg(insfm_ba* h, int* st) {
    const int D = h->D, maxit = h->d.pcg_max_iter;
    h->dc_by_cgp = h->cgp_nb != 0;
    const double tol2 = h->d.pcg_tol * h->d.pcg_tol;
    volatile int* pg = h->prog_host;
    pg[0] = pg[1] = pg[2] = pg[3] = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    // INSFM_DIAG=trace: per solve, host microseconds spent enqueueing CG iterations and the longest single call
    static const bool htrace = diag("trace");
    double t_enq = 0.0, m_enq = 0.0, t_sol0 = htrace ? wall_seconds() : 0.0;
    int n_enq = 0;
    auto enqueue = [&](int from, int to) -> int {
        const double t0 = htrace ? wall_seconds() : 0.0;
        if (h->cgp_nb) return from == 0 ? launch_tl_cgp(h, maxit, tol2) : 0;
        const int r = with_D(D, [&](auto dc_) -> int {
            constexpr int DV = decltype(dc_)::value;
            for (int k = from; k < to; ++k) {
                if (h->xpart) launch_tl_iter_x<DV>(h, k, maxit, tol2);
                else launch_tl_iter<DV>(h, k, maxit, tol2);
            }
            return launch_err(h, "k_tl_pc/k_tl_pspmv");
        });
        if (htrace) { const double dt = wall_seconds() - t0; t_enq += dt; m_enq = std::max(m_enq, dt / std::max(1, to - from)); n_enq += to - from; }
        return r;
    };
    rec(h, 8);
    // multi-rank: the CG's first launch waits for the exchange (the slowest peer); the stall deadline starts once
    // everything queued in front of the CG has completed (ev_pre), and that gate has its own longer deadline
    const bool gated = h->d.world_size > 1 || h->d.allreduce;
    if (gated) HIPCHK(hipEventRecord(h->ev_pre, h->stream));
    // first batch: a little less than the last solve's count (counts drift by a few iterations per LM step); the loop
    // below tops up one iteration at a time
    int enq = std::min(std::max(kCgAhead + 2, h->last_cg_iters - CG_INIT_BACK), maxit + 2);
    if (h->cgp_nb) enq = maxit + 2;  // k_tl_cgp: one launch runs every iteration
    if (int rc = enqueue(0, enq)) return rc;
    if (h->cgp_nb) h->cgp_tag += (unsigned)maxit + 3u;  // (the tags of this launch are never reused)
    if (h->cgp_defer) {  // the side chain of this solve behind the CG (run_tl_setup), from k_tl_cgp's segments
        // (INSFM_DIAG=chain_hold, timing only: no lagged chain at all -- later solves keep an older coarse inverse --
        // to measure what the chain's overlap costs the kernels it runs beside)
        static const bool hold = diag("chain_hold");
        if (!hold) {
            HIPCHK(hipEventRecord(h->ev_E, h->stream));
            if (int rc = issue_side_chain(h, h->cgp_slot, true)) return rc;
        } else {
            h->chain_oseg = false;
        }
        h->cgp_defer = false;
    }
    if (h->cgp_nb && h->cg_async) {
        // one launch runs the whole CG and the kernels behind it need no host decision: the host queues them at once
        // and reads the CG status after the trial's k_publish (cgp_complete), which accepts the trial only for a
        // converged CG.  (Waiting here for the status word cost a host round trip and a launch from an idle queue
        // between the CG and k_cg_finish.)
        rec(h, 9);
        h->cg_launches += 1;
        h->cgp_pending = true;
        st[0] = 1; st[1] = 0; st[2] = 1;
        return 0;
    }
    CgPoll poll;
    poll.enq = enq;
    static const double stall_s = cg_stall_limit_s(std::getenv("INSFM_CG_STALL_S"));
    int erc = 0;
    const int pr = cg_poll(
        poll, maxit + 2, kCgAhead, stall_s, cg_gate_limit_s(stall_s), [&] { return (int)pg[1]; },
        [&] { return (int)pg[0]; }, enqueue,
        [&] {
            const hipError_t q = hipStreamQuery(h->stream);
            if (q == hipSuccess) { std::atomic_thread_fence(std::memory_order_seq_cst); return 0; }
            return q == hipErrorNotReady ? 1 : -1;
        },
        wall_seconds,
        [] {
#if defined(__x86_64__)
            __builtin_ia32_pause();
#endif
        },
        [&] { return !gated || hipEventQuery(h->ev_pre) != hipErrorNotReady; }, &erc);
    hmark(h, "cg converged");
    if (htrace)
        std::fprintf(stderr, "[insfm host] solve %.1f us: %d iterations enqueued in %.1f us (max %.1f per iteration)\n",
                     1e6 * (wall_seconds() - t_sol0), n_enq, 1e6 * t_enq, 1e6 * m_enq);
    enq = poll.enq;
    if (pr == CgPoll::kEnqueueError) return erc;
    if (pr == CgPoll::kStreamError) {
        h->err = std::string("PCG: ") + hipGetErrorString(hipStreamQuery(h->stream));
        return INSFM_BA_EHIP;
    }
    if (pr == CgPoll::kStalled || pr == CgPoll::kGateStalled) {
        h->err = std::string(pr == CgPoll::kGateStalled ? "PCG: the cross-rank exchange in front of the CG did not "
                                                          "complete within "
                                                        : "PCG: no progress from the device for ") +
                 std::to_string(poll.stalled_s) + " s (iterations started " + std::to_string(pg[0]) + ", status " +
                 std::to_string(pg[1]) + ", enqueued " + std::to_string(enq) +
                 "); set INSFM_CG_STALL_S to change the limit";
        return INSFM_BA_EHIP;
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);
    rec(h, 9);
    if (h->timing) {
        HIPCHK(hipStreamSynchronize(h->stream));
        acc_time(h, 8, 9, 5);
    }
    h->cg_launches += h->cgp_nb ? 1 : enq;
    if (h->cgp_nb) return cgp_complete(h, st);
    st[0] = pg[1]; st[1] = pg[2]; st[2] = pg[3];
    return 0;
}

// The block-Jacobi CG (precond 0, or the two-level path without host-mapped memory): launches in chunks, a status
// copy and a stream sync per chunk.
int run_bj_cg(insfm_ba* h, int* st) {
    const int D = h->D, maxit = h->d.pcg_max_iter;
    const double tol2 = h->d.pcg_tol * h->d.pcg_tol;
    int it = 0;
    for (;;) {
        // the count grows by a few iterations per LM step as the damping drops: launch past the last count so most
        // solves need one host poll (a converged iteration costs ~1 us per launch: its kernels exit at the flag)
        const int chunk = (it == 0) ? std::max(8, h->last_cg_iters + 6) : 8;
        const int stop = std::min(it + chunk, maxit + 2);
        const int first = it;
        rec(h, 8);
        const int rc = with_D(D, [&](auto dc_) -> int {
            constexpr int DV = decltype(dc_)::value;
            for (int k = it; k < stop; ++k) {
                if (h->tlon) {
                    if (h->xpart) launch_tl_iter_x<DV>(h, k, maxit, tol2);
                    else launch_tl_iter<DV>(h, k, maxit, tol2);
                    continue;
                }
                if (k > 0) k_cg_dots<<<1, 64, 0, h->stream>>>(k, h->C, maxit, tol2, h->cg);
                k_cg_iter<DV><<<h->C, kCgThreads, 0, h->stream>>>(k, h->C, maxit, tol2, h->nbr_ptr, h->nbr_j, h->Sn,
                                                                h->Lf, h->cg);
            }
            return launch_err(h, "k_cg_iter");
        });
        if (rc) return rc;
        rec(h, 9);
        it = stop;
        HIPCHK(hipMemcpyAsync(st, h->cg.status, sizeof(int) * 3, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        acc_time(h, 8, 9, 5);
        h->cg_launches += stop - first;
        if (st[0] != 0 || it >= maxit + 2) break;
    }
    return 0;
}

// Build S/b for factor f, solve, back-substitute and form the trial parameters.  Returns PCG iterations (>= 0),
// INSFM_BA_ESOLVER on breakdown, or another negative code.
// After the CG of a solve: its status (breakdown -> ESOLVER), the partitioned CG's solution gather, dc = L^-T x.
// Returns the PCG iterations (0 while a k_tl_cgp status is still pending) or an error.
int cg_tail(insfm_ba* h, int* st) {
    const int D = h->D;
    int rc = 0;
    if (st[0] != 1) {
        h->err = std::string("PCG ") +
                 (st[0] == 2 ? "breakdown"
                  : st[0] == 4 ? "timed out (a k_tl_cgp grid barrier or a cross-rank exchange of the partitioned CG)"
                               : "did not finish") +
                 " at iteration " +
                 std::to_string(st[1]) + " (status " + std::to_string(st[0]) + ", coarse " +
                 (h->tlon ? std::to_string(st[2]) : std::string("off")) + ")";
        return st[0] == 4 ? INSFM_BA_EHIP : INSFM_BA_ESOLVER;
    }
    if (!h->cgp_pending) {
        h->coarse_used = h->tlon ? st[2] : 0;
        h->last_cg_iters = st[1];
    }
    if (h->xpart) {  // partitioned CG: every rank's solution rows into every window, then into cg.x
        const int n = h->xq[h->d.rank + 1] - h->xq[h->d.rank];
        if (n > 0)
            k_xput_x<<<cdiv((long long)n * D, 256), 256, 0, h->stream>>>(n, D, h->tl.cl_cams, h->cg.x,
                                                                        xpart_region(h, 0), h->xoff_xg);
        launch_xchg(h, 1);
        HIPCHK(hipMemcpyAsync(h->cg.x, h->xwin + h->xoff_xg, sizeof(double) * (size_t)h->C * D,
                              hipMemcpyDeviceToDevice, h->stream));
        if ((rc = launch_err(h, "partitioned CG gather"))) return rc;
        int sw[2] = {0, 0};  // (prototype path: one synchronization to see a gather that timed out)
        HIPCHK(hipMemcpyAsync(sw, h->cg.status, sizeof(sw), hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        if (sw[0] == 4) {
            h->err = "partitioned CG: the solution gather across ranks timed out";
            return INSFM_BA_EHIP;
        }
    }
    if (h->dc_by_cgp) return h->cgp_pending ? 0 : st[1];  // (k_tl_cgp wrote dc; an abort's launch-path repeat clears it)
    rc = with_D(D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        k_cg_finish<DV><<<cdiv((long long)h->C * DV, kThreads), kThreads, 0, h->stream>>>(h->C, h->Li, h->cg.x,
                                                                                        h->dc, stamp_ptr(h, kStCgFinish));
        return launch_err(h, "k_cg_finish");
    });
    if (rc) return rc;
    hmark(h, "cg_finish");
    return h->cgp_pending ? 0 : st[1];
}

int solve_tail(insfm_ba* h, double f, const double* cams, const double* pts_local, const double* dcp);

// The scaled copy Sn of the current solve's S~ (k_cg_scale), for consumers that read it when the solve skipped it
// (k_tl_cgp's lagged solves): the launch-path CG after an abort, the debug timing of launch-path kernels.
int ensure_sn(insfm_ba* h) {
    if (h->sn_valid || h->kind != 0 || !h->d.optimize_poses) return 0;
    const int rc = with_D(h->D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        k_cg_scale<DV><<<cdiv(h->nnzb, kWaves * scale_nb(DV)), kThreads, 0, h->stream>>>(
            h->nnzb, h->blk_row, h->col, h->row_ptr, h->pos_up, h->pos_lo, h->Li, h->S, h->Sn, 0);
        return launch_err(h, "k_cg_scale");
    });
    if (!rc) h->sn_valid = true;
    return rc;
}

// After a k_tl_cgp abort: the basis was formed again on the main stream; a side chain issued from the launch's coarse
// segments (incomplete when a workgroup never got past the A build) is issued once more from S~ / Z~ (k_tl_erow),
// behind the first on the side stream, so the next solve's coarse inverse is this solve's.
int reissue_chain(insfm_ba* h) {
    if (!h->chain_oseg) return 0;
    h->chain_oseg = false;
    HIPCHK(hipEventRecord(h->ev_E, h->stream));
    return issue_side_chain(h, h->cgp_slot);
}

int run_solve(insfm_ba* h, double f, const double* cams, const double* pts_local) {
    const int D = h->D;
    // the point preparation of the linearization covers this solve when it runs at the prepared damping factor
    const bool prepared = h->prep_valid && h->prep_f == f && h->kind == 0;
    h->prep_valid = false;
    // The non-PD flag is cleared by the k_final that consumed it and the CG status word by k_point_prep; one tiny
    // launch clears both only when that chain is broken (a solve not followed by a cost, or no local points).
    if (h->flags_dirty || h->Pl == 0 || h->kind == 1) {
        k_zero_words<<<1, 64, 0, h->stream>>>(h->flags, h->cg.status);
        const int rc0 = launch_err(h, "k_zero_words");
        if (rc0) return rc0;
    }
    h->flags_dirty = true;
    const bool gpk = h->kind == 1;
    // global positioning: the scale-eliminated blocks are already damped, so k_schur takes U'/g'_c as they are
    const double* Uin = gpk ? h->Up : h->U;
    const double* gcin = gpk ? h->gpc : h->gc;
    const double sf = gpk ? 1.0 : f;
    const double smin = gpk ? -1.0e308 : h->d.clamp_min, smax = gpk ? 1.0e308 : h->d.clamp_max;
    const int sdiag = gpk ? 1 : (h->u_late ? 0 : (h->d.rank == 0));  // u_late: U / g_c added by k_cg_factor
    if (gpk) {
        if (h->Pl > 0)
            k_gp_prep_points<kGPG><<<cdiv((long long)h->Pl * kGPG, kThreads), kThreads, 0, h->stream>>>(h->Pl, h->pt_ptr, h->gobs, f, h->d.clamp_min,
                                                                               h->d.clamp_max, h->W, h->V, h->gp, h->Vinv,
                                                                               h->y, h->VY, h->flags);
        k_gp_prep_cams<<<h->C, kThreads, 0, h->stream>>>(h->C, h->cam_ptr, h->cam_obs, h->gobs, h->U, h->gc, f,
                                                                     h->d.clamp_min, h->d.clamp_max, h->d.rank == 0, h->Up,
                                                                     h->gpc);
    } else if (h->Pl > 0 && !prepared && (hmark(h, "point_prep"), true))
        k_point_prep<<<cdiv(h->Pl, kThreads), kThreads, 0, h->stream>>>(h->Pl, h->V, h->gp, f, h->d.clamp_min, h->d.clamp_max,
                                                                       h->Vinv, h->y, h->flags, h->cg.status,
                                                                       h->d.optimize_poses ? h->Rf : nullptr, h->Mp);
    int iters = 0;
    const double* dcp = nullptr;
    if (h->d.optimize_poses) {
        rec(h, 6);
        int rc = 0;
        if (h->xstream) {
            // chunked exchange: each row chunk's blocks of S are summed across ranks on the exchange stream while the
            // next chunk's Schur rows are built; b (filled by every row) after the last chunk
            const int K = (int)h->xw.size() - 1;
            for (int c = 0; c < K; ++c) {
                if ((rc = launch_schur(h, Uin, gcin, sf, smin, smax, sdiag, !prepared, h->xw[c], h->xw[c + 1]))) return rc;
                const int64_t b0 = h->rptr_host[h->xr[c]], b1 = h->rptr_host[h->xr[c + 1]];
                HIPCHK(hipEventRecord(h->ev_x, h->stream));
                HIPCHK(hipStreamWaitEvent(h->xstream, h->ev_x, 0));
                // set_timing: the exchange's span on its stream, from the first chunk's start to b's end (phase 7)
                if (h->timing && c == 0) HIPCHK(hipEventRecord(h->ev[16], h->xstream));
                if (b1 > b0 && (rc = allreduce_async(h, h->S + b0 * D * D, (b1 - b0) * D * D))) return rc;
            }
            if ((rc = allreduce_async(h, h->b, (int64_t)h->C * D))) return rc;
            HIPCHK(hipEventRecord(h->ev_xdone, h->xstream));
            if (h->timing) HIPCHK(hipEventRecord(h->ev[17], h->xstream));
            HIPCHK(hipStreamWaitEvent(h->stream, h->ev_xdone, 0));
            rec(h, 7);
        } else {
            rc = launch_schur(h, Uin, gcin, sf, smin, smax, sdiag, !prepared);
            if (rc) return rc;
            hmark(h, "schur");
            rec(h, 7);
            rc = allreduce(h, h->S, (int64_t)h->nnzb * D * D + (int64_t)h->C * D);
            if (rc) return rc;
        }
        if (h->built_pending) {  // the side stream's E build of the previous solve still reads S~ / Z~
            HIPCHK(hipStreamWaitEvent(h->stream, h->ev_built, 0));
            h->built_pending = false;
        }
        if ((rc = lin_join(h))) return rc;
        const bool ul = h->u_late && !gpk;
        // k_tl_cgp holds S unscaled and scales the vectors (ba_cgp.h): a lagged solve on it (whose E build behind
        // the CG takes the coarse segments k_tl_cgp writes) needs no scaled copy Sn; the first solve after a
        // linearization that factorizes its own E (k_tl_erow reads Sn), the launch-path CG and the debug getters do
        const bool scale = !(h->tlon && h->cgp_nb && h->tl_solves > 0 && h->tl_fresh && !h->keep_S);
        // the persistent CG's solves: the factorization and the coarse basis in one launch (k_cg_factor_basis)
        h->basis_by_factor = FACTOR_BASIS && h->tlon && h->cgp_nb && !gpk;
        rc = with_D(D, [&](auto dc_) -> int {
            constexpr int DV = decltype(dc_)::value;
            if constexpr (DV != 3) {
                if (h->basis_by_factor) {
                    k_cg_factor_basis<DV><<<cdiv(h->C, kWaves), kThreads, 0, h->stream>>>(
                        h->C, h->row_ptr, h->S, h->b, h->Lf, h->Li, h->cg, ul ? h->U : nullptr, ul ? h->gc : nullptr,
                        f, h->d.clamp_min, h->d.clamp_max, cams, h->tl, h->cgp_runs + (size_t)h->cgp_grid * kCgpRows * 12,
                        stamp_ptr(h, kStFactor));
                }
            }
            if (!h->basis_by_factor)
                k_cg_factor<DV><<<cdiv(h->C, kWaves), kThreads, 0, h->stream>>>(
                    h->C, h->row_ptr, h->S, h->b, h->Lf, h->Li, h->cg, ul ? h->U : nullptr, ul ? h->gc : nullptr, f,
                    h->d.clamp_min, h->d.clamp_max, stamp_ptr(h, kStFactor));
            if (scale)
                k_cg_scale<DV><<<cdiv(h->nnzb, kWaves * scale_nb(DV)), kThreads, 0, h->stream>>>(
                    h->nnzb, h->blk_row, h->col, h->row_ptr, h->pos_up, h->pos_lo, h->Li, h->S, h->Sn, 0);
            return launch_err(h, "k_cg_factor/scale");
        });
        h->sn_valid = scale;
        if (rc) return rc;
        hmark(h, "factor/scale");
        if (h->tlon && (rc = run_tl_setup(h, cams))) return rc;
        hmark(h, "tl setup");
        int* st = reinterpret_cast<int*>(h->host_res + 8);
        rc = (h->tlon && h->prog_host) ? run_tl_cg(h, st) : run_bj_cg(h, st);
        if (rc) return rc;
        if (h->cgp_lost) {  // k_tl_cgp aborted (it left r0 alone): the CG again from the basis, launch path
            h->cgp_lost = false;
            HIPCHK(hipMemsetAsync(h->cg.status, 0, sizeof(int) * 4, h->stream));
            if ((rc = ensure_sn(h)) || (rc = run_tl_basis(h, cams, h->stream)) || (rc = reissue_chain(h)) ||
                (rc = run_tl_cg(h, st)))
                return rc;
        }
        const int ci = cg_tail(h, st);
        if (ci < 0) return ci;
        iters = ci;
        dcp = h->dc;
    }
    if (int rb = solve_tail(h, f, cams, pts_local, dcp)) return rb;
    return iters;
}

// The back-substitution and the trial parameters of a solve (dcp: the camera step, null for a points-only solve).
int solve_tail(insfm_ba* h, double f, const double* cams, const double* pts_local, const double* dcp) {
    const bool gpk = h->kind == 1;
    rec(h, 3);
    if (gpk) {
        if (h->Pl > 0)
            k_gp_backsub<kGPG><<<h->n_gp_grp, kThreads, 0, h->stream>>>(h->Pl, h->pt_ptr, h->cam, h->gobs, dcp, h->Vinv, h->gp,
                                                              pts_local, h->scl_cur, f, h->d.clamp_min, h->d.clamp_max, h->dp,
                                                              h->pts_new, h->scl_new, h->ds, h->part_gp);
        k_gp_update_cams<<<cdiv(3 * h->C, kThreads), kThreads, 0, h->stream>>>(3 * h->C, cams, dcp, h->cams_new);
        int rc = launch_err(h, "k_gp_backsub/update");
        if (rc) return rc;
        return 0;
    }
    if (int rc0 = lin_join(h)) return rc0;  // the camera update reads U / g_c (points-only solves skip the factor)
    const int rc = with_model(h->model, [&](auto mc) -> int {
        constexpr int M = decltype(mc)::value;
        const int nrun = h->Pl > 0 ? h->n_lin : 0;  // point runs, then the camera-update blocks
        k_backsub_rc<M><<<nrun + h->n_gc, kLinThreads, 0, h->stream>>>(
            h->lin_blk, h->pt_ptr, h->cam, h->ptl, h->uv, h->pp, cams, h->d.huber_delta, dcp, h->V, h->Vinv, h->gp,
            pts_local, h->dp, h->pts_new, h->part_gp, nrun, h->C, h->U, h->gc, h->d.rank == 0, h->cams_new, h->part_gc,
            stamp_ptr(h, kStBacksub));
        return launch_err(h, "k_backsub_rc");
    });
    if (rc) return rc;
    hmark(h, "backsub");
    return 0;
}

// A step that ended in an error with a k_tl_cgp status unread: wait for the launch and restart the barrier counters
// (the next launch's epochs would otherwise not match what this one counted).
void cgp_drop_pending(insfm_ba* h) {
    if (!h->cgp_pending) return;
    h->cgp_pending = false;
    (void)hipStreamSynchronize(h->stream);
    (void)hipMemsetAsync(h->cgp_sync, 0, sizeof(unsigned) * kCgpSyncWords, h->stream);
    h->cgp_epochs = 0;
}

// Multi-rank: every rank leaves k_tl_cgp after an abort on any rank (own status `st0`).  A rank whose k_tl_cgp
// converged left its final CG vectors in place of r0, so r0 = L^-1 b is formed again from the completed S / b
// (k_cg_factor without U / g_c: the same L, L^-1 and r0) before the basis / restriction and the launch-path CG.
int cgp_collective_fallback(insfm_ba* h, int st0) {
    std::fprintf(stderr, "[insfm] rank %d: a k_tl_cgp grid barrier timed out on %s rank; every rank continues on the "
                         "launch-per-iteration CG\n", h->d.rank, st0 == 4 ? "this" : "another");
    h->cgp_nb = 0;
    h->cgp_lost = false;
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipMemsetAsync(h->cgp_sync, 0, sizeof(unsigned) * kCgpSyncWords, h->stream));
    h->cgp_epochs = 0;
    HIPCHK(hipMemsetAsync(h->cg.status, 0, sizeof(int) * 4, h->stream));
    const int rc = with_D(h->D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        k_cg_factor<DV><<<cdiv(h->C, kWaves), kThreads, 0, h->stream>>>(h->C, h->row_ptr, h->S, h->b, h->Lf, h->Li, h->cg,
                                                                       nullptr, nullptr, 1.0, 0.0, 0.0);
        return launch_err(h, "k_cg_factor");
    });
    if (rc) return rc;
    if (int r2 = ensure_sn(h)) return r2;
    if (int r3 = run_tl_basis(h, h->cams_cur, h->stream)) return r3;
    return reissue_chain(h);
}

// The persistent CG's factorization and coarse basis again on the completed S / b (no U / g_c added: the same L,
// L^-1 and r0 = L^-1 b): k_cg_factor_basis, or (FACTOR_BASIS=0 builds) k_cg_factor and k_tl_basis.
int refactor_for_cgp(insfm_ba* h, const double* cams) {
    const int rc = with_D(h->D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        if constexpr (DV != 3) {
            if (h->basis_by_factor) {
                k_cg_factor_basis<DV><<<cdiv(h->C, kWaves), kThreads, 0, h->stream>>>(
                    h->C, h->row_ptr, h->S, h->b, h->Lf, h->Li, h->cg, nullptr, nullptr, 1.0, 0.0, 0.0, cams, h->tl,
                    h->cgp_runs + (size_t)h->cgp_grid * kCgpRows * 12);
                return launch_err(h, "k_cg_factor_basis");
            }
        }
        k_cg_factor<DV><<<cdiv(h->C, kWaves), kThreads, 0, h->stream>>>(h->C, h->row_ptr, h->S, h->b, h->Lf, h->Li, h->cg,
                                                                       nullptr, nullptr, 1.0, 0.0, 0.0);
        return launch_err(h, "k_cg_factor");
    });
    if (rc) return rc;
    return h->basis_by_factor ? 0 : run_tl_basis(h, cams, h->stream);
}

// An A-DEF2 solve that broke down (k_tl_cgp status 2).  Its soundness rests on the coarse start x0 making
// Z~^T r exactly zero, which holds only with the solve's own coarse inverse; under the lag rule E^-1 is the previous
// solve's, the preconditioner is not symmetric on the iterates, and the single-reduction recurrence can break down.
// The trial's solve is then repeated with the additive coarse correction (precond 1, symmetric for any SPD E^-1) on
// the same handle: r0 = L^-1 b, the basis and the restriction of r0 again from the completed S / b
// (refactor_for_cgp), one additive k_tl_cgp launch.  Every rank of a replicated
// multi-rank CG sees the same status (bitwise-equal fixed-order arithmetic), so every rank repeats it.
int adef2_fallback(insfm_ba* h, int it_failed, int* st) {
    std::fprintf(stderr, "[insfm] A-DEF2 PCG breakdown at iteration %d: the trial's solve is repeated with the additive "
                         "coarse correction\n", it_failed);
    ++h->adef2_fallbacks;
    HIPCHK(hipMemsetAsync(h->cg.status, 0, sizeof(int) * 4, h->stream));
    int rc = refactor_for_cgp(h, h->cams_cur);
    if (rc) return rc;
    h->adef2 = false;
    rc = run_tl_cg(h, st);
    h->adef2 = true;
    return rc;
}

// lm_step's accept rule for the trial being costed (k_publish copies an accepted trial into the caller's buffers)
struct TrialAccept {
    double last;     // the loss before the step
    int can_reject;  // rejects < max_rejects
};

// The cost result to the host: k_publish into host-mapped memory and a spin on its sequence word; without the mapped
// block, a copy and a stream synchronization.
// Sets h->trial_copied when k_publish also copied an accepted trial (h->pub_host[5] holds its decision).
int finish_cost(insfm_ba* h, const TrialAccept* ta) {
    h->trial_copied = false;
    if (!h->pub_host) {
        HIPCHK(hipMemcpyAsync(h->host_res, h->result, sizeof(double) * 6, hipMemcpyDeviceToHost, h->stream));
        HIPCHK(hipStreamSynchronize(h->stream));
        return 0;
    }
    if (++h->pub_seq == 0) h->pub_seq = 1;
    const unsigned seq = h->pub_seq;
    const bool copy = ta != nullptr && h->ext_cur && h->kind == 0;
    const long long ncam = copy ? (long long)h->C * h->stride : 0, npts = copy ? (long long)h->Pl * 3 : 0;
    const int grid = copy ? std::max(1, std::min(1024, cdiv(std::max(ncam, npts / 2 + 1), kThreads))) : 1;
    k_publish<<<grid, kThreads, 0, h->stream>>>(h->result, h->cgp_pending ? h->cg.status : nullptr, h->pub_dev, seq,
                                               ta ? ta->last : 0.0, ta ? ta->can_reject : 0,
                                               h->cams_new, copy ? h->cams_cur : nullptr, ncam, h->pts_new, h->pts_cur, npts,
                                               stamp_ptr(h, kStPublish));
    if (int rc = launch_err(h, "k_publish")) return rc;
    hmark(h, "publish");
    const unsigned* w = reinterpret_cast<const unsigned*>(h->pub_host + 8);
    // bounded like the CG poll: a device that neither publishes nor reports an error ends the step with EHIP
    static const double stall_s = 6.0 * cg_stall_limit_s(std::getenv("INSFM_CG_STALL_S"));
    const double t_wait = wall_seconds();
    for (unsigned n = 1;; ++n) {
        if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) break;
        if ((n & 255) == 0) {
            const hipError_t q = hipStreamQuery(h->stream);
            if (q != hipSuccess && q != hipErrorNotReady) {
                h->err = std::string("cost: ") + hipGetErrorString(q);
                return INSFM_BA_EHIP;
            }
            if (q == hipSuccess && __atomic_load_n(w, __ATOMIC_ACQUIRE) != seq) {
                h->err = "cost: the stream drained without publishing the result";
                return INSFM_BA_EHIP;
            }
            if (wall_seconds() - t_wait > stall_s) {
                h->err = "cost: no result from the device for " + std::to_string(stall_s) +
                         " s (INSFM_CG_STALL_S scales the limit)";
                return INSFM_BA_EHIP;
            }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    hmark(h, "published");
    const volatile double* pv = h->pub_host;
    for (int k = 0; k < 5; ++k) h->host_res[k] = pv[k];
    h->host_res[5] = pv[6];  // k_tl_cgp aborts (summed over the ranks)
    h->trial_copied = copy;
    return 0;
}

// cost at (cams, pts_local) -> h->result[0..1]; with gain partials when `gains` (after a solve).
int run_cost(insfm_ba* h, const double* cams, const double* pts_local, bool gains, const double* scl = nullptr,
             const TrialAccept* ta = nullptr) {
    if (h->kind == 1) {
        if (h->Nl > 0)
            k_gp_cost<<<h->n_cost, kThreads, 0, h->stream>>>(h->Nl, h->cam, h->ptl, h->trans, h->fcam, cams, pts_local, scl,
                                                             h->d.huber_delta, h->part_cost);
        k_final<<<1, kFinalThreads, 0, h->stream>>>(h->part_cost, h->Nl > 0 ? h->n_cost : 0, gains && h->Pl > 0 ? h->part_gp : nullptr,
                                               h->n_gp, nullptr, 0, h->flags, h->result, nullptr);
        int rc = launch_err(h, "k_gp_cost/k_final");
        if (rc) return rc;
        h->flags_dirty = false;
        rc = allreduce(h, h->result, 6);
        if (rc) return rc;
        return finish_cost(h, nullptr);
    }
    int rc = with_model(h->model, [&](auto mc) -> int {
        constexpr int M = decltype(mc)::value;
        if (h->Nl > 0)
            k_cost<M><<<h->n_cost, kCostThreads, 0, h->stream>>>(h->Nl, h->cam, h->ptl, h->uv, h->pp, cams, pts_local,
                                                             h->d.huber_delta, h->part_cost,
                                                             gains ? stamp_ptr(h, kStCost) : nullptr);
        k_final<<<1, kFinalThreads, 0, h->stream>>>(h->part_cost, h->Nl > 0 ? h->n_cost : 0, gains && h->Pl > 0 ? h->part_gp : nullptr,
                                               h->n_gp, gains ? h->part_gc : nullptr, h->n_gc, h->flags, h->result,
                                               h->cgp_pending ? h->cg.status : nullptr,
                                               gains ? stamp_ptr(h, kStFinal) : nullptr);
        return launch_err(h, "k_cost/k_final");
    });
    if (rc) return rc;
    h->flags_dirty = false;
    rc = allreduce(h, h->result, 6);
    if (rc) return rc;
    return finish_cost(h, ta);
}

// One LM step on the parameters loaded into cams_cur / pts_cur (/ scl_cur): bae.optim.LM.step semantics (SURVEY.md
// 3.3): cumulative damping, TrustRegion radius update, up to max_rejects rejected trials.
int lm_step(insfm_ba* h, insfm_ba_stats* st) {
    h->timing = st != nullptr && h->want_timing;
    for (auto& v : h->tms) v = 0.0;
    h->cg_launches = 0;
    int rc;
    if (!h->have_loss) {
        if ((rc = run_cost(h, h->cams_cur, h->pts_cur, false, h->scl_cur))) return rc;
        h->loss = h->host_res[0];
        h->have_loss = true;
    }
    const double last = h->loss;
    h->hmarks.clear();
    hmark(h, "step");
    if (h->stamps)  // (this step's slot of the ring: a kernel not launched in the step reads 0, not a stamp of 1024 ago)
        HIPCHK(hipMemsetAsync(stamp_ptr(h, 0), 0, sizeof(long long) * kStKinds * 2, h->stream));
    rec(h, 0);
    if ((rc = run_linearize(h, h->cams_cur, h->pts_cur))) return rc;
    hmark(h, "linearize enqueued");
    if (h->timing && (rc = lin_join(h))) return rc;  // (the phase split times both linearization kernels)
    rec(h, 1);
    double f = 1.0;
    int rejects = 0, trials = 0, pcg_total = 0, pcg_last = 0, failed = 0;
    cgp_drop_pending(h);
    for (;;) {
        f *= (1.0 + h->damping);
        ++trials;
        h->cg_async = true;  // (a k_tl_cgp solve: its status is read after the trial's cost, below)
        int it = run_solve(h, f, h->cams_cur, h->pts_cur);
        h->cg_async = false;
        if (it == INSFM_BA_ESOLVER) { failed = 1; h->loss = last; break; }
        if (it < 0) return it;
        rec(h, 4);
        const TrialAccept ta{last, rejects < h->d.max_rejects ? 1 : 0};
        if ((rc = run_cost(h, h->cams_new, h->pts_new, true, h->scl_new, &ta))) return rc;  // waits for the result
        if (h->cgp_pending) {  // the k_tl_cgp launch finished before the k_publish the host just saw
            h->cgp_pending = false;
            int cst[3];
            if ((rc = cgp_complete(h, cst))) return rc;
            if (h->timing) acc_time(h, 8, 9, 5);
            if (h->host_res[4] != 0.0) { failed = 1; h->loss = last; break; }  // a damped point block was not SPD
            const bool multi = h->d.world_size > 1 || h->d.allreduce;
            if (multi && h->host_res[5] != 0.0) {
                // a replicated multi-rank CG: some rank's k_tl_cgp timed out at a grid barrier (the all-reduced flag,
                // the same on every rank, and k_publish accepted nowhere).  Every rank leaves the persistent CG for
                // good and repeats this trial's solve on the launch path from r0 -- the same fixed-order arithmetic
                // everywhere, so the ranks' dc stay bitwise equal -- then its back-substitution and cost.
                if ((rc = cgp_collective_fallback(h, cst[0]))) return rc;
                int* st = reinterpret_cast<int*>(h->host_res + 8);
                if ((rc = run_tl_cg(h, st))) return rc;
                it = cg_tail(h, st);
                if (it == INSFM_BA_ESOLVER) { failed = 1; h->loss = last; break; }
                if (it < 0) return it;
                if ((rc = solve_tail(h, f, h->cams_cur, h->pts_cur, h->dc))) return rc;
                if ((rc = run_cost(h, h->cams_new, h->pts_new, true, h->scl_new, &ta))) return rc;
            } else if (cst[0] == 4 && h->cgp_lost) {
                // single rank: a grid barrier timed out (cgp_complete switched the handle to the launch path); this
                // trial's CG again from the basis, then its back-substitution and cost (k_publish rejected the first)
                h->cgp_lost = false;
                HIPCHK(hipMemsetAsync(h->cg.status, 0, sizeof(int) * 4, h->stream));
                int* st = reinterpret_cast<int*>(h->host_res + 8);
                if ((rc = ensure_sn(h)) || (rc = run_tl_basis(h, h->cams_cur, h->stream)) || (rc = reissue_chain(h)) ||
                    (rc = run_tl_cg(h, st)))
                    return rc;
                it = cg_tail(h, st);
                if (it == INSFM_BA_ESOLVER) { failed = 1; h->loss = last; break; }
                if (it < 0) return it;
                if ((rc = solve_tail(h, f, h->cams_cur, h->pts_cur, h->dc))) return rc;
                if ((rc = run_cost(h, h->cams_new, h->pts_new, true, h->scl_new, &ta))) return rc;
            } else if (cst[0] == 2 && h->adef2) {
                // A-DEF2 breakdown: this trial's solve again with the additive coarse correction (adef2_fallback),
                // then its back-substitution and cost (k_publish rejected the first: its CG did not converge)
                int* st = reinterpret_cast<int*>(h->host_res + 8);
                if ((rc = adef2_fallback(h, cst[1], st))) return rc;
                it = cg_tail(h, st);
                if (it == INSFM_BA_ESOLVER) { failed = 1; h->loss = last; break; }
                if (it < 0) return it;
                if ((rc = solve_tail(h, f, h->cams_cur, h->pts_cur, h->dc))) return rc;
                if ((rc = run_cost(h, h->cams_new, h->pts_new, true, h->scl_new, &ta))) return rc;
            } else if (cst[0] != 1) {
                h->err = std::string("PCG ") + (cst[0] == 2 ? "breakdown" : "timed out (a k_tl_cgp grid barrier)") +
                         " at iteration " + std::to_string(cst[1]) + " (status " + std::to_string(cst[0]) + ")";
                if (cst[0] == 2) { failed = 1; h->loss = last; break; }
                return INSFM_BA_EHIP;
            } else {
                it = cst[1];
                h->coarse_used = cst[2];
                h->last_cg_iters = it;
            }
        }
        rec(h, 5);
        if (h->timing) {
            (void)hipEventSynchronize(h->ev[5]);
            if (trials == 1) acc_time(h, 0, 1, 0);
            if (h->d.optimize_poses) {
                acc_time(h, 6, 7, 1);
                acc_time(h, 1, 3, 2);
                if (h->xstream) acc_time(h, 16, 17, 7);
            }
            acc_time(h, 3, 4, 3);
            acc_time(h, 4, 5, 4);
            rec(h, 1);  // the next trial starts here
        }
        if (h->trial_copied && (h->host_res[4] != 0.0 || (last < h->host_res[0] && rejects < h->d.max_rejects)) &&
            h->pub_host[5] != 0.0) {  // (cannot happen: the same rule on the same doubles)
            h->err = "k_publish accepted a trial the host rejects";
            return INSFM_BA_EHIP;
        }
        if (h->host_res[4] != 0.0) { failed = 1; h->loss = last; break; }  // a damped point block was not SPD
        pcg_last = it;
        pcg_total += it;
        const double loss_new = h->host_res[0];
        const double denom = h->host_res[2] + h->host_res[3];
        const double quality = (last - loss_new) / denom;
        double radius = 1.0 / h->damping;
        if (quality > h->d.tr_high) { radius = h->d.tr_up * radius; h->down = h->d.tr_down; }
        else if (quality > h->d.tr_low) { h->down = h->d.tr_down; }
        else { radius = radius * h->down; h->down = h->down * h->d.tr_factor; }
        radius = std::min(std::max(radius, h->d.tr_min), h->d.tr_max);
        h->damping = 1.0 / radius;
        if (last < loss_new && rejects < h->d.max_rejects) {
            ++rejects;
            h->loss = last;
            continue;
        }
        if (h->trial_copied) {  // k_publish already copied the accepted trial into the caller's buffers
            if (h->pub_host[5] != 1.0) {
                h->err = "accept decision of k_publish differs from the host's";
                return INSFM_BA_EHIP;
            }
        } else if (h->ext_cur) {  // the current parameters live in the caller's buffers: copy the accepted trial there
            HIPCHK(hipMemcpyAsync(h->cams_cur, h->cams_new, sizeof(double) * (size_t)h->C * h->stride,
                                  hipMemcpyDeviceToDevice, h->stream));
            if (h->Pl)
                HIPCHK(hipMemcpyAsync(h->pts_cur, h->pts_new, sizeof(double) * (size_t)h->Pl * 3, hipMemcpyDeviceToDevice,
                                      h->stream));
        } else {
            std::swap(h->cams_cur, h->cams_new);
            std::swap(h->pts_cur, h->pts_new);
        }
        std::swap(h->scl_cur, h->scl_new);
        h->loss = loss_new;
        break;
    }
    if (h->timing) harvest_chain_time(h);
    if (st) {
        st->loss = h->loss;
        st->loss_before = last;
        st->damping = h->damping;
        st->trials = trials;
        st->rejects = rejects;
        st->pcg_iters_last = pcg_last;
        st->pcg_iters_total = pcg_total;
        st->solver_failed = failed;
        for (int k = 0; k < 8; ++k) st->time_ms[k] = h->tms[k];
        st->cg_launches = h->cg_launches;
        st->coarse_used = h->coarse_used;
    }
    h->timing = false;
    if (h->stamps) ++h->stamp_step;
    if (host_trace2() && !h->hmarks.empty()) {
        hmark(h, "step end");
        std::string line = "[insfm host2]";
        for (auto& m : h->hmarks) line += " " + std::string(m.first) + "=" + std::to_string((int)(1e6 * (m.second - h->hmarks[0].second)));
        std::fprintf(stderr, "%s\n", line.c_str());
    }
    return 0;
}

}  // namespace

// ============================================================================================================
// C ABI
// ============================================================================================================
extern "C" {

void insfm_ba_default_desc(insfm_ba_desc* d) {
    std::memset(d, 0, sizeof(*d));
    d->cam_model = 2;
    d->optimize_poses = 1;
    d->deterministic = 0;
    d->huber_delta = 1.0;
    d->tr_radius = 1e4; d->tr_max = 1e10; d->tr_min = 1e-6; d->tr_up = 2.0; d->tr_down = 1.0 / 16.0;
    d->tr_factor = 0.25; d->tr_high = 0.5; d->tr_low = 1e-3;
    d->clamp_min = 1e-6; d->clamp_max = 1e32;
    d->max_rejects = 30;
    d->pcg_max_iter = 500;
    d->pcg_tol = 1e-5;
    d->world_size = 1; d->rank = 0;
    d->shard_point_begin = 0; d->shard_point_end = -1;
    d->precond = 2;
    d->cluster_size = 24;
    d->exchange_chunks = 4;
}

const char* insfm_ba_last_error(const insfm_ba* h) { return h ? h->err.c_str() : "null handle"; }

void insfm_ba_destroy(insfm_ba* h) {
    if (!h) return;
    if (h->side) (void)side_flush(h);
    // every stream that may still use the buffers, before they are parked for the next handle
    for (hipStream_t st : {h->stream, h->side, h->xstream, h->aux})
        if (st) (void)hipStreamSynchronize(st);
    if (!h->stream) (void)hipDeviceSynchronize();
    for (void* q : h->xopened) (void)hipIpcCloseMemHandle(q);  // (peers must be done writing: the caller's barrier)
    if (h->xwin) (void)hipFree(h->xwin);
    dfree_all(h);
    if (h->host_res) (void)hipHostFree(h->host_res);
    if (h->prog_host) (void)hipHostFree(h->prog_host);
    if (h->pub_host) (void)hipHostFree(h->pub_host);
    for (auto& e : h->ev)
        if (e) (void)hipEventDestroy(e);
    if (h->side) {
        (void)hipStreamSynchronize(h->side);
        release_helper_stream(h->side);
    }
    if (h->xstream) {
        (void)hipStreamSynchronize(h->xstream);
        (void)hipStreamDestroy(h->xstream);
    }
    if (h->aux) {
        (void)hipStreamSynchronize(h->aux);
        release_helper_stream(h->aux);
    }
    if (h->ev_lin0) (void)hipEventDestroy(h->ev_lin0);
    if (h->ev_lc) (void)hipEventDestroy(h->ev_lc);
    if (h->ev_x) (void)hipEventDestroy(h->ev_x);
    if (h->ev_xdone) (void)hipEventDestroy(h->ev_xdone);
    if (h->ev_pre) (void)hipEventDestroy(h->ev_pre);
    if (h->ev_E) (void)hipEventDestroy(h->ev_E);
    if (h->ev_built) (void)hipEventDestroy(h->ev_built);
    for (auto& e : h->ev_fact)
        if (e) (void)hipEventDestroy(e);
    delete h;
}

int64_t insfm_ba_nnzb(const insfm_ba* h) { return h ? h->nnzb : -1; }

int64_t insfm_ba_release_cache(void) { return (int64_t)release_cache(); }

}  // extern "C"

namespace {

// Shared creation of a BA (kind 0: obs = uv [N,2], cpar = pp [C,2]) or global-positioning (kind 1: obs = rays [N,3],
// cpar = camera factors [C], sfree = scale-free flags [N] or NULL) handle.
int create_impl(const insfm_ba_desc* desc, int kind, const double* obs, const int32_t* cam_idx, const int32_t* pt_idx,
                const double* cpar, const int32_t* sfree_in, void* stream, insfm_ba** out) {
    if (!desc || !out) return INSFM_BA_EINVAL;
    *out = nullptr;
    insfm_ba* h = new insfm_ba();
    h->d = *desc;
    h->kind = kind;
    h->stream = reinterpret_cast<hipStream_t>(stream);
    auto fail = [&](int rc, const std::string& msg) {
        if (!msg.empty()) h->err = msg;
        *out = h;  // handle returned so the caller can read the error; caller destroys it
        return rc;
    };
    if (kind == 1) {
        h->model = kGP;
        h->ni = 0;
        h->D = 3;
        h->stride = 3;
        h->d.optimize_poses = 1;
    } else {
        h->model = desc->cam_model;
        h->ni = model_ni(h->model);
        if (h->ni < 0) return fail(INSFM_BA_EINVAL, "unsupported camera model " + std::to_string(h->model));
        h->D = 6 + h->ni;
        h->stride = 7 + h->ni;
    }
    h->C = desc->n_cams; h->P = desc->n_points; h->N = desc->n_obs;
    if (h->C <= 0 || h->P <= 0 || h->N < 0) return fail(INSFM_BA_EINVAL, "empty problem");
    if (!obs || !cam_idx || !pt_idx || !cpar) return fail(INSFM_BA_EINVAL, "null input pointer");
    if (desc->world_size < 1 || desc->rank < 0 || desc->rank >= desc->world_size) return fail(INSFM_BA_EINVAL, "bad rank");
    if (desc->world_size > 1 && !desc->allreduce) return fail(INSFM_BA_EINVAL, "world_size > 1 needs allreduce");
    if (h->C > 30000) return fail(INSFM_BA_EINVAL, "n_cams > 30000 not supported (LDS slot table)");
    // desc.schur_variant: only 0 (the W-reading k_schur) remains.  Variants 1 / 2 (camera-point blocks re-derived per
    // pair, LDS-atomic rows / MFMA register accumulation) and 3 (compact W records) were built, parity-tested and
    // measured slower or even in rounds 2-3; they live in the git history.
    if (desc->schur_variant != 0) return fail(INSFM_BA_EINVAL, "schur_variant must be 0");
    const int C = h->C, P = h->P, N = h->N, D = h->D;
    // every pass over the observations below runs on this pool (create_host.h); joined when create returns
    HostPool pool(host_pool_size());
    {
        // input checks, first failing index wins (the lowest slice with a failure holds it)
        std::vector<int> bad(pool.size(), 0);
        pool.ranges(N, [&](int t, long long a, long long b) {
            for (long long i = a; i < b; ++i) {
                if (cam_idx[i] < 0 || cam_idx[i] >= C) { bad[t] = 1; return; }
                if (pt_idx[i] < 0 || pt_idx[i] >= P) { bad[t] = 2; return; }
                if (i && pt_idx[i] < pt_idx[i - 1]) { bad[t] = 3; return; }
            }
        });
        for (int e : bad) {
            if (e == 1) return fail(INSFM_BA_EINVAL, "cam_idx out of range");
            if (e == 2) return fail(INSFM_BA_EINVAL, "pt_idx out of range");
            if (e == 3) return fail(INSFM_BA_EINVAL, "observations must be track-major (pt_idx nondecreasing)");
        }
    }
    h->p0 = std::max(0, desc->shard_point_begin);
    h->p1 = desc->shard_point_end < 0 ? P : std::min(P, desc->shard_point_end);
    if (h->p1 < h->p0) return fail(INSFM_BA_EINVAL, "bad shard range");
    h->Pl = h->p1 - h->p0;
    // INSFM_DIAG=create: host milliseconds of create's phases (stderr)
    static const bool ctrace = diag("create");
    const double ct0 = wall_seconds();
    auto tick = [&](const char* what) {
        if (ctrace) std::fprintf(stderr, "[insfm create] %-28s %8.1f ms\n", what, 1e3 * (wall_seconds() - ct0));
    };
    // global track pointers (pt_idx is nondecreasing: one binary search per track)
    std::vector<int> gptr(P + 1, 0);
    pool.ranges(P + 1, [&](int, long long a, long long b) {
        for (long long p = a; p < b; ++p) gptr[p] = (int)(std::lower_bound(pt_idx, pt_idx + N, (int32_t)p) - pt_idx);
    });
    h->o0 = gptr[h->p0];
    h->Nl = gptr[h->p1] - h->o0;
    const int o0 = h->o0, Nl = h->Nl, Pl = h->Pl;
    // local arrays; each track's observations are reordered by camera (stable insertion sort: tracks are short) so
    // that the upper-triangle partners of an observation are the contiguous tail [ustart[o], track end) of its track;
    // key = that tail's length (the observation's upper-partner count)
    std::vector<int> lptr(Pl + 1);
    nivec<int> lptl(Nl), lcam(Nl), lsrc(Nl), lust(Nl), key(Nl);
    for (int p = 0; p <= Pl; ++p) lptr[p] = gptr[h->p0 + p] - o0;
    std::vector<int> kmax_t(pool.size(), 0);
    pool.ranges(Pl, [&](int t, long long pa, long long pb) {
        int km = 0;
        for (long long p = pa; p < pb; ++p) {
            const int b0 = lptr[p], b1 = lptr[p + 1];
            for (int o = b0; o < b1; ++o) {
                const int x = o0 + o, cx = cam_idx[x];
                int u = o;
                while (u > b0 && cam_idx[lsrc[u - 1]] > cx) { lsrc[u] = lsrc[u - 1]; --u; }
                lsrc[u] = x;
            }
            int u = b0;
            for (int o = b0; o < b1; ++o) {
                lcam[o] = cam_idx[lsrc[o]];
                lptl[o] = (int)p;
                if (o > b0 && lcam[o] != lcam[o - 1]) u = o;
                lust[o] = u;
                key[o] = b1 - u;
                km = std::max(km, key[o]);
            }
        }
        kmax_t[t] = km;
    });
    const int kmax = *std::max_element(kmax_t.begin(), kmax_t.end());
    tick("local track order");
    // camera-major lists: within a camera the observations in point order, cut into chunks of kSchurChunk k_schur
    // rounds (4 x 64 own observations for D = 8), each chunk sorted by descending upper-partner count (stable;
    // balances the Schur groups of a wave: 2.8 % more wave partner slots than a global count sort, 10.8 % with
    // one-round chunks).  Every k_schur row then walks the points in the same global order at about the same pace, so
    // rows running together read a shared track's partner W records close together in time.  Config 3, k_schur:
    // 491 us (count sort over the whole camera) -> 467 us (chunks of 4 rounds; 1 / 2 / 8 / 16 rounds: 541 / 499 / 471 /
    // 483 us -- the wave partner slots cost more than the locality buys below 4).  Measured and dropped in round 3
    // (DESIGN.md section 8): the chunk's slices dealt to the waves in snake order (480-484 vs 473-475 us) and runs of
    // consecutive rows per XCD (L2 hit 4 -> 54 %, yet 469-515 us).
    std::vector<int> cptr;
    nivec<int> cobs;
    {
        // observations are track-major (point order), so a stable counting sort by camera leaves each list in point
        // order; then a stable sort of each chunk by descending partner count
        pcount_sort(pool, Nl, C, nullptr, [&](int o) { return lcam[o]; }, cobs, cptr);
        const int NG = 64 / D, K = kSchurChunk * kSchurWaves * NG;
        pool.ranges(C, [&](int, long long i0, long long i1) {
            for (long long i = i0; i < i1; ++i)
                for (int a = cptr[i]; a < cptr[i + 1]; a += K) {
                    const int e = std::min(a + K, cptr[i + 1]);
                    std::stable_sort(cobs.data() + a, cobs.data() + e, [&](int x, int y) { return key[x] > key[y]; });
                }
        });
    }
    (void)kmax;
    tick("camera-major lists");
    // the per-observation arrays go to the device now: the block pattern below is derived there (single rank)
    int rc;
    if (kind == 1) {
        nivec<double> tl((size_t)3 * Nl);
        nivec<int> sl(Nl);
        pool.ranges(Nl, [&](int, long long a, long long b) {
            for (long long o = a; o < b; ++o) {
                for (int k = 0; k < 3; ++k) tl[3 * (size_t)o + k] = obs[3 * (size_t)lsrc[o] + k];
                sl[o] = sfree_in ? (sfree_in[lsrc[o]] != 0) : 1;
            }
        });
        if ((rc = upload(h, &h->trans, tl.data(), tl.size()))) return fail(rc, "");
        if ((rc = upload(h, &h->sfree, sl.data(), sl.size()))) return fail(rc, "");
        if ((rc = upload(h, &h->fcam, cpar, (size_t)C))) return fail(rc, "");
        if ((rc = upload(h, &h->osrc, lsrc.data(), lsrc.size()))) return fail(rc, "");
        h->osrc_host.assign(lsrc.begin(), lsrc.end());
        auto dd1 = [&](double** p, size_t n) { return dalloc(h, (void**)p, n * sizeof(double)); };
        if ((rc = dd1(&h->gobs, (size_t)Nl * kGO))) return fail(rc, "");
        if ((rc = dd1(&h->Up, (size_t)C * 9))) return fail(rc, "");
        if ((rc = dd1(&h->VY, (size_t)std::max(Pl, 1) * kVY))) return fail(rc, "");
        if ((rc = dd1(&h->gpc, (size_t)C * 3))) return fail(rc, "");
        if ((rc = dd1(&h->scl_cur, (size_t)std::max(Nl, 1)))) return fail(rc, "");
        if ((rc = dd1(&h->scl_new, (size_t)std::max(Nl, 1)))) return fail(rc, "");
        if ((rc = dd1(&h->ds, (size_t)std::max(Nl, 1)))) return fail(rc, "");
    } else {
        nivec<double> uvl((size_t)2 * Nl);
        pool.ranges(Nl, [&](int, long long a, long long b) {
            for (long long o = a; o < b; ++o) {
                uvl[2 * (size_t)o] = obs[2 * (size_t)lsrc[o]];
                uvl[2 * (size_t)o + 1] = obs[2 * (size_t)lsrc[o] + 1];
            }
        });
        if ((rc = upload(h, &h->uv, uvl.data(), uvl.size()))) return fail(rc, "");
        if ((rc = upload(h, &h->pp, cpar, (size_t)2 * C))) return fail(rc, "");
    }
    if ((rc = upload(h, &h->cam, lcam.data(), lcam.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->pt_ptr, lptr.data(), lptr.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->cam_ptr, cptr.data(), cptr.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->cam_obs, cobs.data(), cobs.size()))) return fail(rc, "");
    // derived on the device from the four arrays above instead of uploaded (88 of 140 MB for config 3):
    // per observation its track and the start of its upper partners; per camera-major entry the Schur descriptor and
    // (BA) the linearization's point / uv gathers
    if ((rc = dalloc(h, (void**)&h->ptl, sizeof(int) * (size_t)std::max(Nl, 1)))) return fail(rc, "");
    if ((rc = dalloc(h, (void**)&h->ustart, sizeof(int) * (size_t)std::max(Nl, 1)))) return fail(rc, "");
    if ((rc = dalloc(h, (void**)&h->sdesc, sizeof(int4) * (size_t)std::max(Nl, 1)))) return fail(rc, "");
    if (kind != 1) {
        if ((rc = dalloc(h, (void**)&h->cm_pt, sizeof(int) * (size_t)std::max(Nl, 1)))) return fail(rc, "");
        if ((rc = dalloc(h, (void**)&h->cm_uv, sizeof(double) * 2 * (size_t)std::max(Nl, 1)))) return fail(rc, "");
    }
    if (Pl > 0) k_derive_tracks<<<cdiv(Pl, kThreads), kThreads, 0, h->stream>>>(Pl, h->pt_ptr, h->cam, h->ptl, h->ustart);
    if (Nl > 0)
        k_derive_cm<<<cdiv(Nl, kThreads), kThreads, 0, h->stream>>>(Nl, h->cam_obs, h->ptl, h->ustart, h->pt_ptr,
                                                                    kind != 1 ? h->uv : nullptr, h->sdesc, h->cm_pt,
                                                                    h->cm_uv);
    if ((rc = launch_err(h, "k_derive"))) return fail(rc, "");
    tick("uploads (observations)");
    // The upper block pattern of S (row i: i, then the cameras j > i sharing a track) and the co-visibility graph (per
    // camera every other camera sharing a track, weighted by the number of (obs of i, obs of j) pairs sharing one:
    // the two-level clustering's weights).  Single rank: on the device (k_pattern, two passes), the lower half of the
    // graph transposed from the upper on the host.  Multi-rank (every rank needs the global pattern, and holds only its
    // shard's observations on the device) or INSFM_DIAG=pattern_host: one host pass over the global camera-major list.
    std::vector<int> gcptr;
    CovisGraph g;
    std::vector<int> rptr(C + 1, 0), cols;
    static const bool pattern_host = diag("pattern_host");
    const bool gpu_pattern = !pattern_host && Pl == P && o0 == 0 && Nl == N && C <= kPatternMaxC && Nl > 0;
    std::vector<int> upw;  // (device pattern) the pair count of every upper block, indexed like cols
    if (gpu_pattern) {
        gcptr = cptr;  // (single rank: the local camera-major list is the global one)
        // (scratch from dalloc: a hipFree here would synchronize the device; it goes back with the handle's buffers)
        int *dcnt = nullptr, *doff = nullptr, *dnb = nullptr, *dwt = nullptr;
        const size_t lds = sizeof(int) * (size_t)C;
        std::vector<int> ulen(C), uoff(C + 1, 0);
        if ((rc = dalloc(h, (void**)&dcnt, sizeof(int) * (size_t)C))) return fail(rc, "");
        if ((rc = dalloc(h, (void**)&doff, sizeof(int) * (size_t)(C + 1)))) return fail(rc, "");
        hipError_t e = hipSuccess;
        {
            k_pattern<<<C, 256, lds, h->stream>>>(C, h->cam_ptr, h->cam_obs, h->ustart, h->ptl, h->pt_ptr, h->cam, dcnt,
                                                  nullptr, nullptr, nullptr);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(ulen.data(), dcnt, sizeof(int) * (size_t)C, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        for (int i = 0; i < C && e == hipSuccess; ++i) uoff[i + 1] = uoff[i] + ulen[i];
        const int U = uoff[C];
        std::vector<int> unb(std::max(U, 1)), uwt(std::max(U, 1));
        if (e == hipSuccess && ((rc = dalloc(h, (void**)&dnb, sizeof(int) * (size_t)std::max(U, 1))) ||
                                (rc = dalloc(h, (void**)&dwt, sizeof(int) * (size_t)std::max(U, 1)))))
            return fail(rc, "");
        if (e == hipSuccess) e = hipMemcpyAsync(doff, uoff.data(), sizeof(int) * (size_t)(C + 1), hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) {
            k_pattern<<<C, 256, lds, h->stream>>>(C, h->cam_ptr, h->cam_obs, h->ustart, h->ptl, h->pt_ptr, h->cam, nullptr,
                                                  doff, dnb, dwt);
            e = hipGetLastError();
        }
        if (e == hipSuccess && U > 0) e = hipMemcpyAsync(unb.data(), dnb, sizeof(int) * (size_t)U, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess && U > 0) e = hipMemcpyAsync(uwt.data(), dwt, sizeof(int) * (size_t)U, hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return fail(INSFM_BA_EHIP, std::string("k_pattern: ") + hipGetErrorString(e));
        for (int i = 0; i < C; ++i) rptr[i + 1] = rptr[i] + 1 + ulen[i];
        cols.resize(rptr[C]);
        upw.assign(rptr[C], 0);
        for (int i = 0; i < C; ++i) {
            cols[rptr[i]] = i;
            for (int k = 0; k < ulen[i]; ++k) {
                cols[rptr[i] + 1 + k] = unb[uoff[i] + k];
                upw[rptr[i] + 1 + k] = uwt[uoff[i] + k];
            }
        }
    } else {
    nivec<int> gcpt;  // the point of every observation, camera-major (global)
    pcount_sort(pool, N, C, nullptr, [&](int i) { return cam_idx[i]; }, gcpt, gcptr, [&](int i) { return pt_idx[i]; });
    {
        const int T = pool.size();
        std::vector<std::vector<int>> pnb(T);
        std::vector<std::vector<long long>> pw(T);
        std::vector<int> nlen(C, 0), ulen(C, 0);
        pool.ranges(C, [&](int t, long long i0, long long i1) {
            std::vector<int> mark(C, -1), buf;
            std::vector<long long> acc(C, 0);
            for (int i = (int)i0; i < (int)i1; ++i) {
                buf.clear();
                for (int e = gcptr[i]; e < gcptr[i + 1]; ++e) {
                    const int p = gcpt[e];
                    for (int q = gptr[p]; q < gptr[p + 1]; ++q) {
                        const int j = cam_idx[q];
                        if (j == i) continue;  // (the observation itself and same-camera duplicates)
                        if (mark[j] != i) { mark[j] = i; acc[j] = 0; buf.push_back(j); }
                        acc[j] += 1;
                    }
                }
                std::sort(buf.begin(), buf.end());
                int up = 0;
                for (int j : buf) { pnb[t].push_back(j); pw[t].push_back(acc[j]); up += j > i; }
                nlen[i] = (int)buf.size();
                ulen[i] = up;
            }
        });
        g.ptr.assign(C + 1, 0);
        for (int i = 0; i < C; ++i) {
            g.ptr[i + 1] = g.ptr[i] + nlen[i];
            rptr[i + 1] = rptr[i] + 1 + ulen[i];
        }
        g.nb.reserve(g.ptr[C]);
        g.w.reserve(g.ptr[C]);
        for (int t = 0; t < T; ++t) {
            g.nb.insert(g.nb.end(), pnb[t].begin(), pnb[t].end());
            g.w.insert(g.w.end(), pw[t].begin(), pw[t].end());
        }
        cols.resize(rptr[C]);
        pool.ranges(C, [&](int, long long i0, long long i1) {
            for (int i = (int)i0; i < (int)i1; ++i) {
                int k = rptr[i];
                cols[k++] = i;
                for (int e = g.ptr[i]; e < g.ptr[i + 1]; ++e)
                    if (g.nb[e] > i) cols[k++] = g.nb[e];
            }
        });
    }
    }
    h->nnzb = rptr[C];
    std::vector<int> brow(h->nnzb);
    for (int i = 0; i < C; ++i)
        for (int e = rptr[i]; e < rptr[i + 1]; ++e) brow[e] = i;
    std::vector<int> lop(C + 1, 0);
    for (int i = 0; i < C; ++i)
        for (int e = rptr[i] + 1; e < rptr[i + 1]; ++e) lop[cols[e] + 1]++;
    for (int c = 0; c < C; ++c) lop[c + 1] += lop[c];
    std::vector<int> locol(std::max(1, lop[C])), loblk(std::max(1, lop[C]));
    {
        std::vector<int> fill(lop.begin(), lop.end() - 1);
        for (int i = 0; i < C; ++i)
            for (int e = rptr[i] + 1; e < rptr[i + 1]; ++e) {
                const int k = fill[cols[e]]++;
                locol[k] = i;
                loblk[k] = e;
            }
    }
    if (gpu_pattern) {  // the graph: per row the lower neighbours (transposed, ascending), then the upper ones
        g.ptr.assign(C + 1, 0);
        for (int i = 0; i < C; ++i) g.ptr[i + 1] = g.ptr[i] + (lop[i + 1] - lop[i]) + (rptr[i + 1] - rptr[i] - 1);
        g.nb.resize(g.ptr[C]);
        g.w.resize(g.ptr[C]);
        for (int i = 0; i < C; ++i) {
            int k = g.ptr[i];
            for (int q = lop[i]; q < lop[i + 1]; ++q, ++k) { g.nb[k] = locol[q]; g.w[k] = upw[loblk[q]]; }
            for (int e2 = rptr[i] + 1; e2 < rptr[i + 1]; ++e2, ++k) { g.nb[k] = cols[e2]; g.w[k] = upw[e2]; }
        }
    }
    tick("block pattern + covisibility");
    if (desc->precond < 0 || desc->precond > 2) return fail(INSFM_BA_EINVAL, "precond must be 0, 1 or 2");
    // ---- two-level preconditioner: clusters ----
    // Target cluster size 14 by default (config 3, same box, 3 x 3 runs: K = 16 / 14 / 12 -> 703-711 / 716-720 /
    // 713-720 LM it/s, CG iterations per 10 steps 225 / 213 / 208; profiles/r3_v10/cluster_size_probe_*.log).
    // While the coarse dimension exceeds kCoarseMax the target grows in proportion to the excess (at least by one),
    // rounded up to even (aggregates below K / 2 are dissolved: an odd K would keep singletons):
    // K' = max(K + 1, ceil(K nc MC / kCoarseMax)) rounded up to even, at most C -- the oracle's ora_cluster_cameras.
    // With K = C the clusters are the co-visibility components: if even those do not fit (more components than
    // kCoarseMax / MC), the solver runs the block-Jacobi PCG (precond 0) instead.
    const int MC = D + 1;
    int nc = 0;
    bool coarse_ok = false;
    std::vector<int>& lab = h->clab_host;
    if (desc->precond >= 1 && h->d.optimize_poses) {
        int K = std::min(desc->cluster_size > 0 ? desc->cluster_size : 24, C);
        nc = aggregate(g, C, K, lab);
        while (nc * MC > kCoarseMax && K < C) {
            K = (int)std::min<long long>(C, std::max<long long>(K + 1, ((long long)K * nc * MC + kCoarseMax - 1) / kCoarseMax));
            K += K & 1;
            K = std::min(K, C);
            nc = aggregate(g, C, K, lab);
        }
        coarse_ok = nc * MC <= kCoarseMax;
    }
    tick("clusters");
    // flattened CG neighbour list per row: upper blocks then lower (transposed) ones -- with the two-level
    // preconditioner each row's list is sorted by (cluster of the neighbour, neighbour), so that a row's
    // neighbour-cluster segments are contiguous runs of its blocks (the register-resident CG kernel k_tl_cgp walks
    // them in block order); pos_up/pos_lo give each upper
    // block's two slots in the row-contiguous copy Sn
    std::vector<int> nptr(C + 1, 0), nj, pup(std::max(1, h->nnzb), -1), plo(std::max(1, h->nnzb), -1);
    nj.reserve(2 * (size_t)h->nnzb);
    {
        // per row entries (neighbour j, block e, 0 = upper slot / 1 = lower slot), in cluster order when the coarse
        // space exists (stable: within a cluster the upper-then-lower order)
        std::vector<int4> ent;
        for (int i = 0; i < C; ++i) {
            ent.clear();
            for (int e = rptr[i] + 1; e < rptr[i + 1]; ++e) ent.push_back(make_int4(cols[e], e, 0, 0));
            for (int k = lop[i]; k < lop[i + 1]; ++k) ent.push_back(make_int4(locol[k], loblk[k], 1, 0));
            if (coarse_ok)
                std::stable_sort(ent.begin(), ent.end(), [&](const int4& x, const int4& y) { return lab[x.x] < lab[y.x]; });
            for (const int4& q : ent) {
                (q.z ? plo : pup)[q.y] = (int)nj.size();
                nj.push_back(q.x);
            }
            nptr[i + 1] = (int)nj.size();
        }
    }
    // Equal-length rows (every row padded to the longest with zero blocks of neighbour = the row itself) when that
    // costs at most 10 % more slots: the CG's product kernel then derives a row's range from its index instead of
    // loading nbr_ptr first (one dependent memory round trip less per iteration).  The padded blocks stay zero (Sn is
    // cleared at create and k_cg_scale never writes them), so every consumer of the lists may walk them unchanged.
    {
        int stride = 0;
        for (int i = 0; i < C; ++i) stride = std::max(stride, nptr[i + 1] - nptr[i]);
        const int64_t nn = (int64_t)nj.size();
        if (stride > 0 && nn > 0 && (int64_t)C * stride * 10 <= nn * 11) {
            // the pad slots of a row (neighbour = the row itself) go behind the row's own-cluster entries when the
            // list is in cluster order, so that it stays in cluster order; else at the end
            std::vector<int> nj2((size_t)C * stride), nptr2(C + 1), ins(C);
            for (int i = 0; i < C; ++i) {
                const int n = nptr[i + 1] - nptr[i], pad = stride - n;
                int at = n;
                if (coarse_ok) {
                    at = 0;
                    while (at < n && lab[nj[nptr[i] + at]] <= lab[i]) ++at;
                }
                ins[i] = at;
                nptr2[i] = i * stride;
                int* dst = nj2.data() + (size_t)i * stride;
                for (int q = 0; q < n; ++q) dst[q < at ? q : q + pad] = nj[nptr[i] + q];
                for (int q = 0; q < pad; ++q) dst[at + q] = i;
            }
            nptr2[C] = C * stride;
            // remap the Sn slots of every upper block (row i = brow[e] for pos_up, row cols[e] for pos_lo)
            auto slot = [&](int r, int p) {
                const int q = p - nptr[r];
                return r * stride + (q < ins[r] ? q : q + stride - (nptr[r + 1] - nptr[r]));
            };
            for (int e = 0; e < h->nnzb; ++e) {
                if (e == rptr[brow[e]]) continue;  // diagonal block: no slot
                const int i = brow[e], j = cols[e];
                pup[e] = slot(i, pup[e]);
                plo[e] = slot(j, plo[e]);
            }
            nj.swap(nj2);
            nptr.swap(nptr2);
            h->nbr_stride = stride;
        }
    }
    h->n_nbr = (int64_t)nj.size();
    for (int i = 0; i < C; ++i) { pup[rptr[i]] = 0; plo[rptr[i]] = 0; }  // diagonal blocks: unused slots
    if (nj.empty()) nj.push_back(0);
    tick("CG neighbour lists");
    // Schur work items: split long rows so a chunk fits the LDS budget
    // Deterministic mode's k_schur runs kDetWaves waves per workgroup taking their LDS adds in turn (round 6; one wave
    // in round 5): its workgroups stage kDetWaves waves' W^ and take row chunks of <= kLdsTargetDet, so that three
    // share a CU.  (With the 96-KB chunks of the 8-wave form one wave held a whole CU: k_schur 2.1 ms per trial on
    // config 3 in deterministic mode.)
    const bool det_schur = desc->deterministic != 0;
    const size_t wsh_lds = sizeof(double) * (det_schur ? kDetWaves : kSchurWaves) * (64 / D) * schur_ws(D);  // W^ staging
    const size_t fixed_lds = sizeof(double) * (D + 12) + sizeof(int) * (size_t)C + wsh_lds + 64;
    if (fixed_lds + sizeof(double) * D * D > (size_t)kLdsBudget) return fail(INSFM_BA_EINVAL, "too many cameras for LDS");
    // chunk target: kLdsTarget (deterministic mode kLdsTargetDet) when at least 8 blocks fit under it, else the hard
    // budget
    const size_t tgt0 = det_schur ? (size_t)kLdsTargetDet : (size_t)kLdsTarget;
    const size_t tgt = tgt0 >= fixed_lds + 8 * sizeof(double) * schur_bs(D) ? tgt0 : (size_t)kLdsBudget;
    const int cap = (int)((tgt - fixed_lds) / (sizeof(double) * schur_bs(D)));
    std::vector<int4> work;
    int maxc = 1;
    for (int i = 0; i < C; ++i) {
        if (gcptr[i + 1] == gcptr[i] && rptr[i + 1] - rptr[i] == 1) {
            work.push_back(make_int4(i, rptr[i], rptr[i + 1], 0));
            continue;
        }
        for (int kb = rptr[i]; kb < rptr[i + 1]; kb += cap) {
            const int ke = std::min(kb + cap, rptr[i + 1]);
            work.push_back(make_int4(i, kb, ke, 0));
            maxc = std::max(maxc, ke - kb);
        }
    }
    h->nwork = (int)work.size();
    h->max_chunk = maxc;
    if (kind == 0 && desc->allreduce_async && (desc->world_size > 1 || desc->allreduce) && desc->exchange_chunks > 1 &&
        desc->optimize_poses) {
        // chunk boundaries at rows splitting the blocks into about equal counts (geometric series of chunk sizes
        // were measured in round 3 and do not pay: the all-reduces run back to back on one stream; DESIGN.md section
        // 5), and the first work item of each boundary row
        const int K = std::min(desc->exchange_chunks, C);
        h->rptr_host = rptr;
        h->xr.assign(1, 0);
        h->xw.assign(1, 0);
        for (int c = 1; c < K; ++c) {
            const int64_t target = (int64_t)rptr[C] * c / K;
            const int r = (int)(std::upper_bound(rptr.begin(), rptr.end(), (int)target) - rptr.begin()) - 1;
            if (r <= h->xr.back() || r >= C) continue;
            int w = h->xw.back();
            while (w < (int)work.size() && work[w].x < r) ++w;
            h->xr.push_back(r);
            h->xw.push_back(w);
        }
        h->xr.push_back(C);
        h->xw.push_back((int)work.size());
        hipError_t e = hipStreamCreateWithFlags(&h->xstream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_x, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_xdone, hipEventDisableTiming);
        if (e != hipSuccess) return fail(INSFM_BA_EHIP, std::string("exchange stream: ") + hipGetErrorString(e));
    }
    // Work order: natural (row order), so the 256 rows running at once are 256 consecutive cameras that share tracks
    // in the Infinity Cache.
    h->schur_lds = sizeof(double) * ((size_t)maxc * schur_bs(D) + D + 12) + wsh_lds + sizeof(int) * (size_t)C;
    h->schur_lds = (h->schur_lds + 15) & ~(size_t)15;
    // Camera linearization beside k_lin_points / k_schur (u_late), single rank (multi-rank, U / g_c are all-reduced
    // before the Schur build adds them).
    {
        if (kind == 0 && desc->world_size <= 1 && !desc->allreduce) {
            hipError_t e = helper_stream(1, 0, &h->aux);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_lin0, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_lc, hipEventDisableTiming);
            if (e != hipSuccess) return fail(INSFM_BA_EHIP, std::string("linearization stream: ") + hipGetErrorString(e));
            h->u_late = true;
        }
    }

    if (kind != 1) {
        std::vector<int> lb(1, 0);
        for (int p = 0; p < Pl; ++p)  // close the run before a track that would overflow it
            if (p > lb.back() && (lptr[p + 1] - lptr[lb.back()] > kLinThreads || p - lb.back() >= kLinThreads))
                lb.push_back(p);
        if (Pl > 0) lb.push_back(Pl);
        h->n_lin = (int)lb.size() - 1;
        if ((rc = upload(h, &h->lin_blk, lb.data(), lb.size()))) return fail(rc, "");
    }
    if ((rc = upload(h, &h->row_ptr, rptr.data(), rptr.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->col, cols.data(), cols.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->blk_row, brow.data(), brow.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->nbr_ptr, nptr.data(), nptr.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->nbr_j, nj.data(), nj.size()))) return fail(rc, "");
    if ((rc = upload(h, &h->pos_up, pup.data(), pup.size()))) return fail(rc, "");
    h->pos_up_host = pup;
    if ((rc = upload(h, &h->pos_lo, plo.data(), plo.size()))) return fail(rc, "");
    {
        const int DPd = D + (D & 1);
        const size_t snb = sizeof(double) * (size_t)std::max<int64_t>(h->n_nbr, 1) * D * DPd;
        if ((rc = dalloc(h, (void**)&h->Sn, snb))) return fail(rc, "");
        if (hipMemsetAsync(h->Sn, 0, snb, h->stream) != hipSuccess) return fail(INSFM_BA_EHIP, "Sn clear");
    }
    if ((rc = upload(h, &h->work, work.data(), work.size()))) return fail(rc, "");
    auto dd = [&](double** p, size_t n) { return dalloc(h, (void**)p, n * sizeof(double)); };
    // the CG's cross-workgroup hand-off buffers (atomic partial sums, exchanged w, tagged granules, barrier words) in
    // uncached device memory (INSFM_DIAG=cgp_cached: ordinary memory, for A/B runs)
    const bool uc = !diag("cgp_cached");
    auto hand = [&](void** p, size_t bytes) { return dalloc(h, p, bytes, uc); };
    // W: [3][D] records per observation (global positioning: its 32-B {u, beta^2} records fit in the same buffer)
    if ((rc = dd(&h->W, (size_t)Nl * D * 3 + 2))) return fail(rc, "");
    if ((rc = dd(&h->V, (size_t)Pl * 6))) return fail(rc, "");
    if ((rc = dd(&h->gp, (size_t)Pl * 3))) return fail(rc, "");
    if ((rc = dd(&h->Vinv, (size_t)Pl * 6))) return fail(rc, "");
    if ((rc = dd(&h->y, (size_t)Pl * 3))) return fail(rc, "");
    if (kind == 0) {
        if ((rc = dd(&h->Rf, (size_t)Pl * 6))) return fail(rc, "");
        if ((rc = dd(&h->Mp, (size_t)Pl * 6))) return fail(rc, "");
    }
    if ((rc = dd(&h->dp, (size_t)Pl * 3))) return fail(rc, "");
    h->xcount = (int64_t)h->nnzb * D * D + (int64_t)C * D + (int64_t)C * D * D + (int64_t)C * D + 8;
    if ((rc = dd(&h->xbuf, (size_t)h->xcount))) return fail(rc, "");
    h->S = h->xbuf;
    h->b = h->S + (size_t)h->nnzb * D * D;
    h->U = h->b + (size_t)C * D;
    h->gc = h->U + (size_t)C * D * D;
    h->scal = h->gc + (size_t)C * D;
    if ((rc = dd(&h->Lf, (size_t)C * D * D))) return fail(rc, "");
    if ((rc = dd(&h->Li, (size_t)C * D * D))) return fail(rc, "");
    if ((rc = dd(&h->dc, (size_t)C * D))) return fail(rc, "");
    h->cg_nwg = C;  // one workgroup (and one partial record) per camera row
    const size_t cd = (size_t)C * D;
    const size_t cgn = 8 * cd + 2 * 3 * (size_t)h->cg_nwg + 2 * ((size_t)desc->pcg_max_iter + 2) + 16;
    if ((rc = dd(&h->cgmem, cgn))) return fail(rc, "");
    {
        double* m = h->cgmem;
        h->cg.r[0] = m; m += cd; h->cg.r[1] = m; m += cd;
        h->cg.w[0] = m; m += cd; h->cg.w[1] = m; m += cd;
        h->cg.s[0] = m; m += cd; h->cg.s[1] = m; m += cd;
        h->cg.p = m; m += cd; h->cg.x = m; m += cd;
        h->cg.part[0] = m; m += 3 * (size_t)h->cg_nwg; h->cg.part[1] = m; m += 3 * (size_t)h->cg_nwg;
        h->cg.hist = m; m += 2 * ((size_t)desc->pcg_max_iter + 2);
        h->cg.scal = m; m += 4;
    }
    if ((rc = dalloc(h, (void**)&h->cg.status, sizeof(int) * 4))) return fail(rc, "");
    const int ST = h->stride;
    if ((rc = dd(&h->cams_cur, (size_t)C * ST))) return fail(rc, "");
    if ((rc = dd(&h->cams_new, (size_t)C * ST))) return fail(rc, "");
    if ((rc = dd(&h->pts_cur, (size_t)std::max(Pl, 1) * 3))) return fail(rc, "");
    if ((rc = dd(&h->pts_new, (size_t)std::max(Pl, 1) * 3))) return fail(rc, "");
    h->n_cost = std::max(1, cdiv(Nl, kind == 1 ? kThreads : kCostThreads));
    h->n_gp = std::max(1, cdiv(Pl, kThreads));
    h->n_gp_grp = std::max(1, cdiv((long long)Pl * kGPG, kThreads));
    if (kind == 1) h->n_gp = h->n_gp_grp;  // the gain partials of k_gp_backsub
    else h->n_gp = std::max(1, h->n_lin);   // one per run of k_backsub
    h->n_gc = std::max(1, cdiv(C, kLinThreads));  // camera-update blocks (ride along with k_backsub_rc)
    if ((rc = dd(&h->part_cost, 2 * (size_t)h->n_cost))) return fail(rc, "");
    if ((rc = dd(&h->part_gp, (size_t)h->n_gp))) return fail(rc, "");
    if ((rc = dd(&h->part_gc, (size_t)h->n_gc))) return fail(rc, "");
    h->result = h->scal;  // the 4 result scalars are all-reduced in place with the exchange buffer
    if ((rc = dalloc(h, (void**)&h->flags, sizeof(int) * 4))) return fail(rc, "");
    {
        hipError_t e = hipHostMalloc((void**)&h->host_res, 128, hipHostMallocDefault);
        if (e != hipSuccess) return fail(INSFM_BA_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
        // the published cost block (without it, or with a cross-rank sum installed, costs come back by copy + sync)
        void* pm = nullptr;
        if (hipHostMalloc(&pm, 16 * sizeof(double), hipHostMallocMapped) == hipSuccess) {
            void* dp = nullptr;
            if (hipHostGetDevicePointer(&dp, pm, 0) == hipSuccess) {
                h->pub_host = static_cast<double*>(pm);
                h->pub_dev = static_cast<double*>(dp);
                std::memset(pm, 0, 16 * sizeof(double));
            } else {
                (void)hipHostFree(pm);
            }
        }
    }
    for (auto& e : h->ev) {
        hipError_t x = hipEventCreate(&e);
        if (x != hipSuccess) return fail(INSFM_BA_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(x));
    }
    if (desc->world_size > 1 || desc->allreduce) {
        const hipError_t x = hipEventCreateWithFlags(&h->ev_pre, hipEventDisableTiming);
        if (x != hipSuccess) return fail(INSFM_BA_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(x));
    }
    {
        hipError_t e = hipMemsetAsync(h->part_gp, 0, sizeof(double) * h->n_gp, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(h->part_gc, 0, sizeof(double) * h->n_gc, h->stream);
        if (e == hipSuccess) e = hipMemsetAsync(h->flags, 0, sizeof(int) * 4, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return fail(INSFM_BA_EHIP, std::string("init: ") + hipGetErrorString(e));
    }
    // the Schur kernels may need more than the default dynamic-LDS limit
    with_D(D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        (void)hipFuncSetAttribute((const void*)k_schur<DV, kDetWaves, false, false, SCHUR_DET_ORD>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->schur_lds);
        (void)hipFuncSetAttribute((const void*)k_schur<DV, kSchurWaves>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)h->schur_lds);
        (void)hipFuncSetAttribute((const void*)k_schur<DV, kDetWaves, false, true, SCHUR_DET_ORD>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->schur_lds);
        (void)hipFuncSetAttribute((const void*)k_schur<DV, kSchurWaves, false, true>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->schur_lds);
        if constexpr (DV == 3) {
            (void)hipFuncSetAttribute((const void*)k_schur<3, kDetWaves, true, false, SCHUR_DET_ORD>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->schur_lds);
            (void)hipFuncSetAttribute((const void*)k_schur<3, kSchurWaves, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)h->schur_lds);
            (void)hipFuncSetAttribute((const void*)k_schur_gp<kSchurWaves, kGPSG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)h->schur_lds);
        }
        return 0;
    });
    tick("uploads + allocations");
    if (coarse_ok) {
        // ---- two-level preconditioner: source lists of E, buffers ----
        const int m = nc * MC;
        tick("covisibility + clusters");
        std::vector<int> clp(nc + 1, 0), clc(C), alone(C);
        for (int i = 0; i < C; ++i) clp[lab[i] + 1]++;
        for (int c = 0; c < nc; ++c) clp[c + 1] += clp[c];
        {
            std::vector<int> fill(clp.begin(), clp.end() - 1);
            for (int i = 0; i < C; ++i) clc[fill[lab[i]]++] = i;
        }
        int maxmem = 1;
        for (int c = 0; c < nc; ++c) maxmem = std::max(maxmem, clp[c + 1] - clp[c]);
        for (int i = 0; i < C; ++i) alone[i] = (clp[lab[i] + 1] - clp[lab[i]]) < 2;
        // per row: neighbour slots ordered by (cluster of the neighbour, slot) and one segment per neighbour cluster
        // (the row's own cluster always has one: it carries the diagonal term)
        std::vector<int> sperm(std::max<int64_t>(h->n_nbr, 1), 0), rsp(C + 1, 0);
        std::vector<int4> segs;
        int maxseg = 1;
        {
            // rows in parallel (each row's segments into its own list), then concatenated in row order
            std::vector<std::vector<int4>> rsegs(C);
            pool.ranges(C, [&](int, long long i0, long long i1) {
                std::vector<int> ord;
                for (int i = (int)i0; i < (int)i1; ++i) {
                    const int n0 = nptr[i], n1 = nptr[i + 1];
                    ord.resize(n1 - n0);
                    for (int q = 0; q < n1 - n0; ++q) ord[q] = n0 + q;
                    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return lab[nj[x]] < lab[nj[y]]; });
                    for (int q = 0; q < n1 - n0; ++q) sperm[n0 + q] = ord[q];
                    const int own = lab[i];
                    bool own_done = false;
                    int q = 0;
                    std::vector<int4>& out = rsegs[i];
                    while (q < n1 - n0 || !own_done) {
                        const int cq = q < n1 - n0 ? lab[nj[ord[q]]] : nc;
                        if (!own_done && own < cq) {  // own cluster without neighbours in it
                            out.push_back(make_int4(own, q, q, 1));
                            own_done = true;
                            continue;
                        }
                        int qe = q;
                        while (qe < n1 - n0 && lab[nj[ord[qe]]] == cq) ++qe;
                        out.push_back(make_int4(cq, q, qe, cq == own ? 1 : 0));
                        if (cq == own) own_done = true;
                        q = qe;
                    }
                }
            });
            for (int i = 0; i < C; ++i) {
                segs.insert(segs.end(), rsegs[i].begin(), rsegs[i].end());
                rsp[i + 1] = (int)segs.size();
                maxseg = std::max(maxseg, (int)rsegs[i].size());
            }
        }
        // E source lists per cluster pair (row cluster c', column cluster c): the segments of c's rows, rows ascending
        std::vector<int> eptr((size_t)nc * nc + 1, 0), eseg;
        eseg.reserve(segs.size());
        {
            std::vector<std::vector<int>> bucket(nc);
            for (int cr = 0; cr < nc; ++cr) {
                for (auto& v : bucket) v.clear();
                for (int e = clp[cr]; e < clp[cr + 1]; ++e) {
                    const int i = clc[e];
                    for (int sidx = rsp[i]; sidx < rsp[i + 1]; ++sidx) bucket[segs[sidx].x].push_back(sidx);
                }
                for (int c = 0; c < nc; ++c) {
                    eseg.insert(eseg.end(), bucket[c].begin(), bucket[c].end());
                    eptr[(size_t)cr * nc + c + 1] = (int)eseg.size();
                }
            }
        }
        tick("coarse segments");
        TlBufs& tl = h->tl;
        tl.nc = nc;
        tl.m = m;
        tl.maxmem = maxmem;
        const int ldE = gj_steps(m) * kGB;
        tl.ldE = ldE;
        int* ip = nullptr;
        if ((rc = upload(h, &ip, clp.data(), clp.size()))) return fail(rc, "");
        tl.cl_ptr = ip;
        if ((rc = upload(h, &ip, clc.data(), clc.size()))) return fail(rc, "");
        tl.cl_cams = ip;
        {
            std::vector<int> cpos(C);
            for (int q = 0; q < C; ++q) cpos[clc[q]] = q;
            if ((rc = upload(h, &ip, cpos.data(), cpos.size()))) return fail(rc, "");
            tl.cpos = ip;
        }
        if ((rc = upload(h, &ip, alone.data(), alone.size()))) return fail(rc, "");
        tl.alone = ip;
        if ((rc = upload(h, &ip, sperm.data(), sperm.size()))) return fail(rc, "");
        tl.sperm = ip;
        if ((rc = upload(h, &ip, rsp.data(), rsp.size()))) return fail(rc, "");
        tl.rseg_ptr = ip;
        if ((rc = upload(h, &ip, eptr.data(), eptr.size()))) return fail(rc, "");
        tl.ered_ptr = ip;
        if (eseg.empty()) eseg.push_back(0);
        if ((rc = upload(h, &ip, eseg.data(), eseg.size()))) return fail(rc, "");
        tl.ered_seg = ip;
        {
            int4* sp = nullptr;
            if ((rc = upload(h, &sp, segs.data(), segs.size()))) return fail(rc, "");
            tl.seg = sp;
        }
        if ((rc = dd(&tl.u, cd))) return fail(rc, "");
        if ((rc = dd(&tl.Zt, cd * MC))) return fail(rc, "");
        if ((rc = dd(&tl.Ztc, cd * MC))) return fail(rc, "");
        if ((rc = dd(&tl.vc, cd))) return fail(rc, "");
        if ((rc = dd(&tl.Rc, (size_t)m))) return fail(rc, "");
        if ((rc = dd(&tl.gd, 3 * (size_t)C))) return fail(rc, "");
        {
            if ((rc = upload(h, &ip, lab.data(), lab.size()))) return fail(rc, "");
            tl.clab = ip;
            // atomic cluster sums of the CG partials: single GPU, non-deterministic mode only -- the replicated
            // multi-rank CG needs bitwise-equal inputs on every rank (config 3: CG iteration 23.9 -> 22.3 us, round 3)
            tl.Racc = nullptr;
            tl.Gacc = nullptr;
            if (!desc->deterministic && desc->world_size <= 1 && !desc->allreduce) {
                if ((rc = hand((void**)&tl.Racc, sizeof(double) * 3 * (size_t)m))) return fail(rc, "");
                if ((rc = hand((void**)&tl.Gacc, sizeof(double) * 3 * 3 * (size_t)nc))) return fail(rc, "");
                if (hipMemsetAsync(tl.Racc, 0, sizeof(double) * 3 * (size_t)m, h->stream) != hipSuccess ||
                    hipMemsetAsync(tl.Gacc, 0, sizeof(double) * 9 * (size_t)nc, h->stream) != hipSuccess)
                    return fail(INSFM_BA_EHIP, "Racc clear");
            }
        }
        if ((rc = dd(&tl.rowR, (size_t)C * MC + 2))) return fail(rc, "");  // +2: k_tl_pc reads it in 16-B pairs
        if ((rc = dd(&tl.Oseg, segs.size() * MC * MC))) return fail(rc, "");
        {
            // E is kept padded to whole blocks; the pad is the identity (k_tl_ereduce writes only the m x m part and
            // the Gauss-Jordan steps keep the pad an identity)
            std::vector<double> eye((size_t)ldE * ldE, 0.0);
            for (int q = m; q < ldE; ++q) eye[(size_t)q * ldE + q] = 1.0;
            for (int sl = 0; sl < 2; ++sl) {
                if ((rc = upload(h, &h->Ebuf[sl], eye.data(), eye.size()))) return fail(rc, "");
                if ((rc = dd(&h->Einvbuf[sl], (size_t)m * m))) return fail(rc, "");
            }
        }
        if ((rc = dd(&h->gjW, (size_t)ldE * ldE))) return fail(rc, "");
        if ((rc = dd(&h->gjP, (size_t)2 * kGB * kGB))) return fail(rc, "");
        {
            std::vector<double> ones(ldE, 1.0);   // equilibration of the pad (k_tl_ereduce writes the first m)
            if ((rc = upload(h, &tl.Ed, ones.data(), ones.size()))) return fail(rc, "");
        }
        if ((rc = dalloc(h, (void**)&h->okbuf, sizeof(int) * 2))) return fail(rc, "");
        tl.E = h->Ebuf[0];
        tl.Einv = h->Einvbuf[0];
        tl.ok = h->okbuf;
        hipError_t e = hipMemsetAsync(h->okbuf, 0, sizeof(int) * 2, h->stream);
        // The side stream (E build + factorization, off the critical path) at the lowest priority (ROCm exposes only
        // normal and high: no measured effect either way, round 1)
        int prio_lo = 0, prio_hi = 0;
        if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
        // (INSFM_DIAG=side_hi / side_normal: the side stream at the high / normal priority instead, for A/B runs)
        const int side_prio = diag("side_hi") ? prio_hi : diag("side_normal") ? 0 : prio_lo;
        if (e == hipSuccess) e = helper_stream(0, side_prio, &h->side);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_E, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_built, hipEventDisableTiming);
        for (int sl = 0; sl < 2 && e == hipSuccess; ++sl) e = hipEventCreateWithFlags(&h->ev_fact[sl], hipEventDisableTiming);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return fail(INSFM_BA_EHIP, std::string("two-level init: ") + hipGetErrorString(e));
        h->erow_lds = 0;  // (k_tl_erow's LDS is static: a few KB)
        (void)maxseg;
        {
            const size_t fixed = sizeof(double) * ((size_t)MC * m + (size_t)m), budget = 144 * 1024;
            h->pc_rows = (int)std::min<size_t>((size_t)C, (budget - fixed) / (sizeof(double) * MC));
            h->pc_lds = fixed + sizeof(double) * (size_t)h->pc_rows * MC;
        }
        if (h->erow_lds > 160 * 1024 || h->pc_lds > 150 * 1024)
            return fail(INSFM_BA_EINVAL, "two-level preconditioner: scene too connected for the LDS budget (use precond 0)");
        with_D(D, [&](auto dc_) -> int {
            constexpr int DV = decltype(dc_)::value;
            (void)hipFuncSetAttribute((const void*)k_tl_pc<DV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)h->pc_lds);
            return 0;
        });
        h->tlon = true;
        void* pm = nullptr;
        if (hipHostMalloc(&pm, sizeof(int) * 8, hipHostMallocMapped) == hipSuccess) {
            h->prog_host = static_cast<int*>(pm);
            void* dp = nullptr;
            if (hipHostGetDevicePointer(&dp, pm, 0) == hipSuccess) h->cg.prog = static_cast<int*>(dp);
            else { (void)hipHostFree(pm); h->prog_host = nullptr; }
        }
        // the persistent register-resident CG (ba_cgp.h): D = 8, atomic cluster sums, host-mapped progress, rows of
        // at most NB = 128 blocks in cluster order, at most kCgpSegMax neighbour clusters per row, and the whole grid
        // resident at once
        int maxlen = 0;
        for (int i = 0; i < C; ++i) maxlen = std::max(maxlen, nptr[i + 1] - nptr[i]);
        bool in_order = true;
        for (int64_t q = 0; q < h->n_nbr && in_order; ++q) in_order = sperm[q] == q;
        const int nb = (maxlen <= 64 && !diag("cgp128")) ? 64 : maxlen <= 128 ? 128 : 0;
        const int grid = (C + kCgpRows - 1) / kCgpRows;
        if (diag("create"))
            std::fprintf(stderr, "[insfm create] k_tl_cgp eligibility: D %d, atomic sums %d, progress %d, max row %d, "
                         "cluster order %d, max segments %d\n", D, tl.Racc != nullptr, h->prog_host != nullptr, maxlen,
                         (int)in_order, maxseg);
        // non-deterministic single rank: per-cluster atomic sums (tl.Racc); otherwise (deterministic mode, or every
        // rank of a replicated multi-rank CG) the fixed-order variant
        // (INSFM_DIAG=cgp_det: the fixed-order variant on a non-deterministic handle too, for A/B runs)
        const bool det = tl.Racc == nullptr || diag("cgp_det");
        // precond 2 (A-DEF2) in either form (round 6: the fixed-order DET form too); the launch path runs the additive
        // form of precond 1
        const bool adef = desc->precond == 2;
        if (D == 8 && h->prog_host && nb && in_order && maxseg <= kCgpSegMax && !diag("no_cgp")) {
            int dev = 0, ncu = 0, per_cu = 0;
            hipError_t ce = hipGetDevice(&dev);
            if (ce == hipSuccess) ce = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
            if (ce == hipSuccess)
                ce = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)cgp_kernel(nb, det, adef), kCgpThreads,
                                                                  0);
            if (ce == hipSuccess && per_cu >= 1 && grid <= ncu) {
                if ((rc = hand((void**)&h->cgp_wx, sizeof(double) * 2 * cd))) return fail(rc, "");
                if ((rc = hand((void**)&h->cgp_yg, sizeof(unsigned long long) * 2 * kCoarseMax))) return fail(rc, "");
                if (hipMemsetAsync(h->cgp_yg, 0, sizeof(unsigned long long) * 2 * kCoarseMax, h->stream) != hipSuccess)
                    return fail(INSFM_BA_EHIP, "cgp granules");
                if ((rc = hand((void**)&h->cgp_sync, sizeof(unsigned) * kCgpSyncWords))) return fail(rc, "");
                if (hipMemsetAsync(h->cgp_sync, 0, sizeof(unsigned) * kCgpSyncWords, h->stream) != hipSuccess)
                    return fail(INSFM_BA_EHIP, "cgp barrier words");
                if (diag("cgp_trace") && (rc = dd(&h->cgp_trace, kCgpTraceLen))) return fail(rc, "");
                // the run records: DET's partials by parity, and (every form) the restriction of r0 that
                // k_cg_factor_basis writes for the setup
                if ((rc = hand((void**)&h->cgp_runs, sizeof(double) * 2 * 12 * (size_t)grid * kCgpRows)))
                    return fail(rc, "");
                // k_tl_cgp holds S unscaled: the S block (and orientation) of every slot, and the unscaled basis
                {
                    std::vector<int> src((size_t)std::max<int64_t>(h->n_nbr, 1), kCgpPadSlot);
                    for (int e = 0; e < h->nnzb; ++e) {
                        if (e == rptr[brow[e]]) continue;  // diagonal block: no slot
                        src[pup[e]] = e;
                        src[plo[e]] = ~e;
                    }
                    if ((rc = upload(h, &h->cgp_src, src.data(), src.size()))) return fail(rc, "");
                    if ((rc = dd(&tl.Gb, cd * MC))) return fail(rc, "");
                }
                h->cgp_det = det;
                h->adef2 = adef;
                h->cgp_nb = nb;
                h->cgp_grid = grid;
                h->cgp_slots = per_cu * ncu;
                if (diag("create"))
                    std::fprintf(stderr, "[insfm create] k_tl_cgp<%d>: %d workgroups, %d CUs, %d per CU\n", nb, grid, ncu,
                                 per_cu);
            }
        }
    }
    tick("two-level setup (end)");
    if (kind == 0 && diag("stamps")) {
        const size_t n = (size_t)kStampSteps * kStKinds * 2;
        if ((rc = dalloc(h, (void**)&h->stamps, sizeof(long long) * n))) return fail(rc, "");
        if (hipMemsetAsync(h->stamps, 0, sizeof(long long) * n, h->stream) != hipSuccess) return fail(INSFM_BA_EHIP, "stamps");
    }
    h->damping = 1.0 / desc->tr_radius;
    h->down = desc->tr_down;
    *out = h;
    return INSFM_BA_OK;
}

}  // namespace

extern "C" {

int insfm_ba_create(const insfm_ba_desc* desc, const double* obs_uv, const int32_t* cam_idx, const int32_t* pt_idx,
                    const double* pp, void* stream, insfm_ba** out) {
    return create_impl(desc, 0, obs_uv, cam_idx, pt_idx, pp, nullptr, stream, out);
}

int insfm_ba_set_timing(insfm_ba* h, int32_t on) {
    if (!h) return INSFM_BA_EINVAL;
    h->want_timing = on != 0;
    return INSFM_BA_OK;
}

int64_t insfm_ba_exchange_count(const insfm_ba* h) { return h ? h->xcount : -1; }

int insfm_ba_set_exchange(insfm_ba* h, double* buf, int64_t count) {
    if (!h || !buf || count < h->xcount) return INSFM_BA_EINVAL;
    const int C = h->C, D = h->D;
    h->xbuf = buf;
    h->S = h->xbuf;
    h->b = h->S + (size_t)h->nnzb * D * D;
    h->U = h->b + (size_t)C * D;
    h->gc = h->U + (size_t)C * D * D;
    h->scal = h->gc + (size_t)C * D;
    h->result = h->scal;
    return INSFM_BA_OK;
}

int insfm_ba_set_ranks_per_device(insfm_ba* h, int32_t ranks) {
    if (!h || ranks < 1) return INSFM_BA_EINVAL;
    if (h->cgp_nb && (long long)ranks * h->cgp_grid > (long long)h->cgp_slots) {
        if (diag("create"))
            std::fprintf(stderr, "[insfm create] %d ranks per GPU: k_tl_cgp would need %lld of %d workgroup slots; "
                         "launch path\n", ranks, (long long)ranks * h->cgp_grid, h->cgp_slots);
        h->cgp_nb = 0;
    }
    return INSFM_BA_OK;
}

int insfm_ba_cg_info(const insfm_ba* h, int32_t* out) {
    if (!h || !out) return INSFM_BA_EINVAL;
    out[0] = h->xpart ? 3 : h->cgp_nb ? (h->cgp_det ? (h->adef2 ? 5 : 2) : (h->adef2 ? 4 : 1)) : 0;
    out[1] = h->cgp_grid;
    out[2] = h->cgp_slots;
    out[3] = h->cgp_nb;
    return INSFM_BA_OK;
}

int32_t insfm_ba_cg_fallbacks(const insfm_ba* h) {
    if (!h) return INSFM_BA_EINVAL;
    return h->adef2_fallbacks;
}

int32_t insfm_ba_debug_stamps(insfm_ba* h, int64_t* host_out, int32_t max_steps) {
    if (!h || !host_out || max_steps < 0) return INSFM_BA_EINVAL;
    if (!h->stamps) return 0;
    HIPCHK(hipStreamSynchronize(h->stream));
    const long long n = std::min<long long>(std::min<long long>(h->stamp_step, kStampSteps), max_steps);
    std::vector<long long> ring((size_t)kStampSteps * kStKinds * 2);
    HIPCHK(hipMemcpy(ring.data(), h->stamps, sizeof(long long) * ring.size(), hipMemcpyDeviceToHost));
    const long long first = h->stamp_step - n;  // the oldest of the last n steps
    for (long long q = 0; q < n; ++q) {
        const size_t src = (size_t)((first + q) % kStampSteps) * kStKinds * 2;
        std::memcpy(host_out + (size_t)q * kStKinds * 2, ring.data() + src, sizeof(long long) * kStKinds * 2);
    }
    return (int32_t)n;
}

int insfm_ba_set_persistent_cg(insfm_ba* h, int32_t on) {
    if (!h) return INSFM_BA_EINVAL;
    if (on) return h->cgp_nb ? INSFM_BA_OK : INSFM_BA_EINVAL;  // (cannot turn on what create found ineligible)
    cgp_drop_pending(h);
    h->cgp_nb = 0;
    return INSFM_BA_OK;
}

int insfm_ba_cg_window(insfm_ba* h, void* ipc_handle) {
    if (!h || !ipc_handle) return INSFM_BA_EINVAL;
    if (h->kind != 0 || h->d.world_size < 2 || !h->tlon || h->tl.Racc || h->xwin) {
        h->err = "cg_window: needs a multi-rank two-level handle (precond 1) that has no window yet";
        return INSFM_BA_EINVAL;
    }
    h->cgp_nb = 0;  // (the partitioned launch path replaces the replicated persistent CG)
    const int C = h->C, D = h->D, MC = D + 1, W = h->d.world_size;
    const long long region = (long long)C * D + 3LL * C + (long long)C * MC + 2;
    h->xoff_region[0] = 0;
    h->xoff_region[1] = region;
    h->xoff_xg = 2 * region;
    h->xoff_flags = h->xoff_xg + (long long)C * D;
    h->xwin_bytes = sizeof(double) * (size_t)h->xoff_flags + sizeof(unsigned) * kXFlagStride * 2 * (size_t)W;
    // uncached device memory: peers write into it over their mappings, and no cache of this device keeps a stale line
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&h->xwin), h->xwin_bytes, hipDeviceMallocUncached);
    if (e == hipSuccess) e = hipMemsetAsync(h->xwin, 0, h->xwin_bytes, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(ipc_handle), h->xwin);
    if (e != hipSuccess) {
        h->err = std::string("cg_window: ") + hipGetErrorString(e);
        return INSFM_BA_EHIP;
    }
    return INSFM_BA_OK;
}

int insfm_ba_cg_attach(insfm_ba* h, const void* handles) {
    if (!h || !handles || !h->xwin || h->xpart) return INSFM_BA_EINVAL;
    const int W = h->d.world_size, C = h->C;
    std::vector<double*> bases(W, nullptr);
    std::vector<unsigned*> flags(W, nullptr);
    for (int r = 0; r < W; ++r) {
        if (r == h->d.rank) {
            bases[r] = h->xwin;
        } else {
            void* q = nullptr;
            hipIpcMemHandle_t hd;
            std::memcpy(&hd, static_cast<const char*>(handles) + (size_t)r * sizeof(hipIpcMemHandle_t), sizeof(hd));
            const hipError_t e = hipIpcOpenMemHandle(&q, hd, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) {
                h->err = std::string("cg_attach: rank ") + std::to_string(r) + ": " + hipGetErrorString(e);
                return INSFM_BA_EHIP;
            }
            h->xopened.push_back(q);
            bases[r] = static_cast<double*>(q);
        }
        flags[r] = reinterpret_cast<unsigned*>(bases[r] + h->xoff_flags);
    }
    int rc = 0;
    if ((rc = dalloc(h, reinterpret_cast<void**>(&h->xbases), sizeof(double*) * W))) return rc;
    if ((rc = dalloc(h, reinterpret_cast<void**>(&h->xpflags), sizeof(unsigned*) * W))) return rc;
    if ((rc = dalloc(h, reinterpret_cast<void**>(&h->xcnt), sizeof(unsigned) * 2))) return rc;
    HIPCHK(hipMemcpyAsync(h->xbases, bases.data(), sizeof(double*) * W, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemcpyAsync(h->xpflags, flags.data(), sizeof(unsigned*) * W, hipMemcpyHostToDevice, h->stream));
    HIPCHK(hipMemsetAsync(h->xcnt, 0, sizeof(unsigned) * 2, h->stream));
    // rows: the cluster-ordered positions split at cluster boundaries, rank r from the boundary nearest r C / W
    const std::vector<int>& lab = h->clab_host;
    std::vector<int> bnd;  // cluster-ordered boundaries (positions where a cluster starts), incl. 0 and C
    {
        std::vector<int> size(h->tl.nc, 0);
        for (int i = 0; i < C; ++i) size[lab[i]]++;
        int q = 0;
        for (int c = 0; c < h->tl.nc; ++c) { bnd.push_back(q); q += size[c]; }
        bnd.push_back(q);
    }
    h->xq.assign(W + 1, C);
    h->xq[0] = 0;
    for (int r = 1; r < W; ++r) {
        const long long target = (long long)r * C / W;
        int best = bnd[0];
        for (int b : bnd)
            if (std::llabs(b - target) < std::llabs(best - target)) best = b;
        h->xq[r] = std::max(best, h->xq[r - 1]);
    }
    // the basis writes r0 and its restriction into region 1 (what the setup k_tl_pc reads)
    h->tl = tl_region(h, 1);
    HIPCHK(hipStreamSynchronize(h->stream));
    h->xpart = true;
    return INSFM_BA_OK;
}

int insfm_ba_debug_time_xchg(insfm_ba* h, int32_t reps, double* us) {
    if (!h || !us || !h->xpart || reps < 1) return INSFM_BA_EINVAL;
    HIPCHK(hipEventRecord(h->ev[10], h->stream));
    for (int r = 0; r < reps; ++r) launch_xchg(h, 1);  // (slot 1: not gated by the CG status)
    HIPCHK(hipEventRecord(h->ev[11], h->stream));
    HIPCHK(hipEventSynchronize(h->ev[11]));
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, h->ev[10], h->ev[11]));
    *us = 1e3 * ms / reps;
    return INSFM_BA_OK;
}

int insfm_ba_cg_partition(const insfm_ba* h, int32_t* rows_begin_end) {
    if (!h || !rows_begin_end || !h->xpart) return INSFM_BA_EINVAL;
    rows_begin_end[0] = h->xq[h->d.rank];
    rows_begin_end[1] = h->xq[h->d.rank + 1];
    return INSFM_BA_OK;
}

int insfm_ba_reset(insfm_ba* h) {
    if (!h) return INSFM_BA_EINVAL;
    h->damping = 1.0 / h->d.tr_radius;
    h->down = h->d.tr_down;
    h->have_loss = false;
    // a fresh LM: the first solve after the reset factorizes its own coarse matrix (no lagged E^-1 of an earlier solve
    // survives) and the CG's first batch is sized as for a new handle
    cgp_drop_pending(h);
    if (int rc = side_flush(h)) return rc;
    h->tl_solves = 0;
    h->tl_fresh = false;
    h->last_cg_iters = 16;
    h->chain_timed[0] = h->chain_timed[1] = false;
    return INSFM_BA_OK;
}

int insfm_ba_cost(insfm_ba* h, const double* cams, const double* pts, double* loss, double* rmse) {
    if (!h || !cams || !pts || h->kind != 0) return INSFM_BA_EINVAL;
    cgp_drop_pending(h);
    HIPCHK(hipMemsetAsync(h->flags, 0, sizeof(int) * 4, h->stream));
    int rc = run_cost(h, cams, pts + 3 * (size_t)h->p0, false);
    if (rc) return rc;
    if (loss) *loss = h->host_res[0];
    if (rmse) *rmse = h->N > 0 ? std::sqrt(h->host_res[1] / h->N) : 0.0;
    return INSFM_BA_OK;
}

int insfm_ba_step(insfm_ba* h, double* cams_user, double* pts_user, insfm_ba_stats* st) {
    if (!h || !cams_user || !pts_user || h->kind != 0) return INSFM_BA_EINVAL;
    // The caller's buffers are the linearization point of this step (read in place, no copy-in); trials go to the
    // internal cams_new / pts_new, and an accepted trial is copied back into the caller's buffers (stream-ordered, no
    // host wait: the step's loss is already on the host).
    double* const ic = h->cams_cur;
    double* const ip = h->pts_cur;
    h->cams_cur = cams_user;
    h->pts_cur = pts_user + 3 * (size_t)h->p0;
    h->ext_cur = true;
    const int rc = lm_step(h, st);
    h->cams_cur = ic;
    h->pts_cur = ip;
    h->ext_cur = false;
    return rc;
}

int insfm_ba_debug_linearize(insfm_ba* h, const double* cams, const double* pts) {
    if (!h || !cams || !pts || h->kind != 0) return INSFM_BA_EINVAL;
    cgp_drop_pending(h);
    h->keep_S = 1;
    HIPCHK(hipMemcpyAsync(h->cams_cur, cams, sizeof(double) * (size_t)h->C * h->stride, hipMemcpyDeviceToDevice, h->stream));
    if (h->Pl)
        HIPCHK(hipMemcpyAsync(h->pts_cur, pts + 3 * (size_t)h->p0, sizeof(double) * (size_t)h->Pl * 3, hipMemcpyDeviceToDevice,
                              h->stream));
    int rc = run_linearize(h, h->cams_cur, h->pts_cur);
    if (!rc) rc = lin_join(h);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
}

int insfm_ba_debug_solve(insfm_ba* h, double f) {
    if (!h) return INSFM_BA_EINVAL;
    cgp_drop_pending(h);
    h->keep_S = 1;
    // solves around the parameters last passed to insfm_ba_debug_linearize
    int it = run_solve(h, f, h->cams_cur, h->pts_cur);
    HIPCHK(hipStreamSynchronize(h->stream));
    return it;
}

int insfm_ba_debug_spd_inverse(int32_t m, const double* E, double* Einv, void* stream, int32_t reps,
                               double* us_per_inverse) {
    if (m < 1 || m > 4096 || !E || !Einv) return INSFM_BA_EINVAL;
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int nB = gj_steps(m), ld = nB * kGB;
    const int n = reps > 0 && us_per_inverse ? reps : 1;
    // the padded, identity-extended copy and the equilibration d = 1 / sqrt(diag E) are built on the host
    std::vector<double> Eh((size_t)m * m), Ep((size_t)ld * ld, 0.0), dh(ld, 1.0);
    if (hipMemcpy(Eh.data(), E, sizeof(double) * Eh.size(), hipMemcpyDeviceToHost) != hipSuccess) return INSFM_BA_EHIP;
    for (int r = 0; r < ld; ++r)
        for (int c = 0; c < ld; ++c)
            Ep[(size_t)r * ld + c] = (r < m && c < m) ? Eh[(size_t)r * m + c] : (r == c ? 1.0 : 0.0);
    for (int r = 0; r < m; ++r) dh[r] = 1.0 / std::sqrt(Eh[(size_t)r * m + r]);
    double *Ew = nullptr, *Ww = nullptr, *dd = nullptr, *Pw = nullptr;
    int* ok = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int okh = 0;
    float ms = 0.f;
    hipError_t e = hipMalloc(&Ew, sizeof(double) * (size_t)ld * ld);
    if (e == hipSuccess) e = hipMalloc(&Ww, sizeof(double) * (size_t)ld * ld);
    if (e == hipSuccess) e = hipMalloc(&dd, sizeof(double) * ld);
    if (e == hipSuccess) e = hipMalloc(&Pw, sizeof(double) * 2 * kGB * kGB);
    if (e == hipSuccess) e = hipMalloc(&ok, sizeof(int));
    if (e == hipSuccess) e = hipMemcpy(dd, dh.data(), sizeof(double) * ld, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    for (int r = 0; r < n && e == hipSuccess; ++r) {
        e = hipMemcpyAsync(Ew, Ep.data(), sizeof(double) * Ep.size(), hipMemcpyHostToDevice, st);
        if (e == hipSuccess) e = hipEventRecord(e0, st);
        for (int u = 0; u <= nB && e == hipSuccess; ++u) {
            launch_gj_unit(u, m, Ew, Ww, Pw, dd, Einv, ok, st);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(e1, st);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float t = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
        ms += t;
    }
    if (e == hipSuccess) e = hipMemcpy(&okh, ok, sizeof(int), hipMemcpyDeviceToHost);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(Ew); (void)hipFree(Ww); (void)hipFree(dd); (void)hipFree(Pw); (void)hipFree(ok);
    if (e != hipSuccess) return INSFM_BA_EHIP;
    if (us_per_inverse) *us_per_inverse = 1e3 * ms / n;
    return okh ? 1 : 0;
}

int insfm_ba_debug_time_kernel(insfm_ba* h, int32_t which, int32_t reps, double* us_per_launch) {
    if (!h || reps <= 0 || !us_per_launch || !h->d.optimize_poses) return INSFM_BA_EINVAL;
    // re-run one kernel `reps` times back to back on the data of the last solve; the CG state it overwrites is
    // scratch once the solve has finished (dc already extracted).  0: k_cg_iter  1: k_schur (damping factor 1)
    // 2: one two-level CG iteration  3: k_tl_pspmv  4: the two-level setup  5: k_lin_points (overwrites W / V / g_p)
    HIPCHK(hipMemsetAsync(h->cg.status, 0, sizeof(int) * 4, h->stream));
    HIPCHK(hipMemsetAsync(h->cg.scal, 0, sizeof(double) * 4, h->stream));
    if (((which >= 2 && which <= 4) || which == 6 || which == 7) && !h->tlon) return INSFM_BA_EINVAL;
    if (which == 5 && (h->kind != 0 || !h->W)) return INSFM_BA_EINVAL;
    if (which < 0 || which > 7) return INSFM_BA_EINVAL;
    if (int rc0 = side_flush(h)) return rc0;  // its pending E build / factorization must not interleave
    if (int rc0 = lin_join(h)) return rc0;
    if (which != 1 && which != 5 && which != 6)
        if (int rc0 = ensure_sn(h)) return rc0;  // (kernels that read the scaled copy Sn)
    if (which == 2 && h->tl.Racc) {
        // atomic cluster sums: iteration 1's k_tl_pc reads buffer 1 every repetition (its k_tl_pspmv adds into buffer
        // 0, which the next repetition clears), so fill buffer 1 once from a k_tl_pspmv of iteration 0
        HIPCHK(hipMemsetAsync(h->tl.Racc + h->tl.m, 0, sizeof(double) * h->tl.m, h->stream));
        HIPCHK(hipMemsetAsync(h->tl.Gacc + 3 * h->tl.nc, 0, sizeof(double) * 3 * h->tl.nc, h->stream));
        with_D(h->D, [&](auto dc_) -> int {
            constexpr int DV = decltype(dc_)::value;
            k_tl_pspmv<DV><<<h->C, kPspmvThreads, 0, h->stream>>>(0, h->C, h->nbr_stride, h->nbr_ptr, h->nbr_j, h->Sn,
                                                                 h->Lf, h->cg, h->tl, XPart{});
            return 0;
        });
    }
    HIPCHK(hipEventRecord(h->ev[10], h->stream));
    int rc = with_D(h->D, [&](auto dc_) -> int {
        constexpr int DV = decltype(dc_)::value;
        for (int r = 0; r < reps; ++r) {
            if (which == 2) {
                launch_tl_iter<DV>(h, 1, h->d.pcg_max_iter, 0.0);
            } else if (which == 3) {
                k_tl_pspmv<DV><<<h->C, kPspmvThreads, 0, h->stream>>>(1, h->C, h->nbr_stride, h->nbr_ptr, h->nbr_j, h->Sn, h->Lf, h->cg,
                                                                   h->tl, XPart{});
            } else if (which == 4) {
                int rc2 = run_tl_basis(h, h->cams_cur, h->stream);
                if (!rc2) rc2 = run_tl_build(h, 0, h->stream);
                for (int u = 0; u <= gj_steps(h->tl.m) && !rc2; ++u) rc2 = run_tl_gj_unit(h, 0, u, h->stream);
                if (rc2) return rc2;
            } else if (which == 6) {  // the coarse inverse alone: k_gj_pinv0 + nB x k_gj_step on slot 0's E
                for (int u = 1; u <= gj_steps(h->tl.m) + 1; ++u)
                    if (int rc2 = run_tl_gj_unit(h, 0, u - 1, h->stream)) return rc2;
            } else if (which == 7) {  // the E build alone: k_tl_erow + k_tl_ereduce
                if (int rc2 = run_tl_build(h, 0, h->stream)) return rc2;
            } else if (which == 5 && h->kind == 0 && h->W) {  // k_lin_points at the last trial's parameters
                with_model(h->model, [&](auto mc) -> int {
                    constexpr int M = decltype(mc)::value;
                    if (h->Pl > 0) launch_lin_points_w<M>(h, h->cams_new, h->pts_new, first_trial_prep(h));
                    return 0;
                });
            } else if (which == 0)
                k_cg_iter<DV><<<h->C, kCgThreads, 0, h->stream>>>(1, h->C, h->d.pcg_max_iter, 0.0, h->nbr_ptr, h->nbr_j, h->Sn,
                                                                h->Lf, h->cg);
            else {  // the k_schur form this handle runs (deterministic mode: one wave per workgroup, its LDS layout)
                const int rc2 = launch_schur(h, h->kind ? h->Up : h->U, h->kind ? h->gpc : h->gc, 1.0,
                                             h->kind ? -1e308 : h->d.clamp_min, h->kind ? 1e308 : h->d.clamp_max,
                                             h->kind ? 1 : h->d.rank == 0, false);
                if (rc2) return rc2;
            }
        }
        return launch_err(h, "debug_time_kernel");
    });
    if (rc) return rc;
    HIPCHK(hipEventRecord(h->ev[11], h->stream));
    HIPCHK(hipEventSynchronize(h->ev[11]));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, h->ev[10], h->ev[11]));
    *us_per_launch = 1e3 * ms / reps;
    return INSFM_BA_OK;
}

int insfm_ba_debug_time_cgp(insfm_ba* h, int32_t reps, double* out) {
    // the persistent CG of the last solve again, `reps` times: k_cg_factor_basis on the completed S / b (no U / g_c
    // added: the same L, L^-1 and r0 = L^-1 b; Z~ and the restriction of r0), then the timed part -- the k_tl_cgp
    // launch, bracketed by events -- with the coarse segments written as in a lagged solve.  out[0] us per
    // k_tl_cgp launch, out[1] 0 (the setup launch k_tl_pc that preceded it until round 4 is folded in), out[2]
    // iterations (mean).
    if (!h || reps <= 0 || !out || !h->cgp_nb || h->kind != 0 || !h->prog_host) return INSFM_BA_EINVAL;
    cgp_drop_pending(h);
    if (int rc0 = side_flush(h)) return rc0;
    if (int rc0 = lin_join(h)) return rc0;
    const int maxit = h->d.pcg_max_iter;
    const double tol2 = h->d.pcg_tol * h->d.pcg_tol;
    double t_cg = 0.0, t_pc = 0.0, iters = 0.0;
    for (int r = 0; r < reps; ++r) {
        HIPCHK(hipMemsetAsync(h->cg.status, 0, sizeof(int) * 4, h->stream));
        if (int rc = refactor_for_cgp(h, h->cams_new)) return rc;  // (the last trial's cameras)
        volatile int* pg = h->prog_host;
        pg[0] = pg[1] = pg[2] = pg[3] = 0;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        h->cgp_defer = true;  // (oseg: the segments are written, as in the lagged solves that are most of a run)
        HIPCHK(hipEventRecord(h->ev[10], h->stream));
        if (int rc2 = launch_tl_cgp(h, maxit, tol2)) { h->cgp_defer = false; return rc2; }
        h->cgp_defer = false;
        h->cgp_tag += (unsigned)maxit + 3u;
        HIPCHK(hipEventRecord(h->ev[11], h->stream));
        HIPCHK(hipEventSynchronize(h->ev[11]));
        int st[3];
        if (int rc2 = cgp_complete(h, st)) return rc2;
        if (st[0] != 1) {
            h->err = "debug_time_cgp: the CG ended with status " + std::to_string(st[0]);
            return st[0] == 2 ? INSFM_BA_ESOLVER : INSFM_BA_EHIP;
        }
        float ms = 0.f;
        HIPCHK(hipEventElapsedTime(&ms, h->ev[10], h->ev[11]));
        t_cg += ms;
        iters += st[1];
    }
    // (round 5: the coarse solve of r0 runs inside k_tl_cgp; no setup launch in front of it)
    out[1] = t_pc;
    out[0] = 1e3 * t_cg / reps;
    out[2] = iters / reps;
    return INSFM_BA_OK;
}

int32_t insfm_ba_debug_clusters(const insfm_ba* h, int32_t* labels) {
    if (!h) return INSFM_BA_EINVAL;
    if (!h->tlon) return 0;
    if (labels) std::memcpy(labels, h->clab_host.data(), sizeof(int32_t) * h->C);
    return h->tl.nc;
}

int64_t insfm_ba_debug_get(insfm_ba* h, int32_t which, double* host) {
    if (!h || !host) return INSFM_BA_EINVAL;
    const size_t C = h->C, Pl = h->Pl, Nl = h->Nl, D = h->D;
    const double* src = nullptr;
    size_t n = 0;
    switch (which) {
        case 0: src = h->W; n = Nl * D * 3; break;
        case 1: src = h->V; n = Pl * 6; break;
        case 2: src = h->gp; n = Pl * 3; break;
        case 3: src = h->U; n = C * D * D; break;
        case 4: src = h->gc; n = C * D; break;
        case 5: {  // the scaled upper blocks S~ (diagonal: I), assembled from the row-contiguous copy Sn
            if (h->kind != 0 && h->kind != 1) return INSFM_BA_EINVAL;
            if (int rc0 = side_flush(h)) return rc0;
            if (int rc0 = ensure_sn(h)) return rc0;
            const size_t DP = D + (D & 1), nb = (size_t)h->nnzb;
            std::vector<double> sn((size_t)std::max<int64_t>(h->n_nbr, 1) * D * DP);
            if (h->n_nbr) HIPCHK(hipMemcpyAsync(sn.data(), h->Sn, sizeof(double) * h->n_nbr * D * DP, hipMemcpyDeviceToHost, h->stream));
            HIPCHK(hipStreamSynchronize(h->stream));
            std::vector<int> rp(C + 1);
            HIPCHK(hipMemcpy(rp.data(), h->row_ptr, sizeof(int) * (C + 1), hipMemcpyDeviceToHost));
            std::vector<char> diag_blk(nb, 0);
            for (size_t i = 0; i < C; ++i) diag_blk[rp[i]] = 1;
            for (size_t e = 0; e < nb; ++e)
                for (size_t a = 0; a < D; ++a)
                    for (size_t c = 0; c < D; ++c)
                        host[(e * D + a) * D + c] = diag_blk[e] ? (a == c ? 1.0 : 0.0)
                                                                : sn[((size_t)h->pos_up_host[e] * D + a) * DP + c];
            return (int64_t)(nb * D * D);
        }
        case 6: src = h->b; n = C * D; break;
        case 7: src = h->dc; n = C * D; break;
        case 8: src = h->dp; n = Pl * 3; break;
        // two-level internals (debug): 9 u, 10 w, 11 rowR, 12/13 E^-1 slot 0/1, 14 row partials [r.u | w.u], 15 r
        case 9: src = h->tl.u; n = h->tlon ? C * D : 0; break;
        case 10: src = h->cg.w[0]; n = C * D; break;
        case 11: src = h->tl.rowR; n = h->tlon ? C * (D + 1) : 0; break;  // restriction row partials
        case 12: src = h->Einvbuf[0]; n = h->tlon ? (size_t)h->tl.m * h->tl.m : 0; break;
        case 13: src = h->Einvbuf[1]; n = h->tlon ? (size_t)h->tl.m * h->tl.m : 0; break;
        case 14: src = h->tl.gd; n = h->tlon ? 2 * C : 0; break;
        case 15: src = h->cg.r[0]; n = C * D; break;
        // 16/17 E slot 0/1 padded to whole blocks [ldE][ldE] (E^-1 once the slot's inversion has run)
        case 16: case 17: src = h->Ebuf[which - 16]; n = h->tlon ? (size_t)h->tl.ldE * h->tl.ldE : 0; break;
        default: return INSFM_BA_EINVAL;
    }
    if (int rc0 = side_flush(h)) return rc0;
    if (int rc0 = lin_join(h)) return rc0;
    if (n) HIPCHK(hipMemcpyAsync(host, src, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return (int64_t)n;
}

// ---- global positioning (include/insfm_gp.h) -------------------------------------------------------------------
void insfm_gp_default_desc(insfm_ba_desc* d) {
    insfm_ba_default_desc(d);
    d->cam_model = -1;
    d->huber_delta = 0.1;  // GLOBAL_POSITIONER_OPTIONS['thres_loss_function'] (config/colmap.py:41-46)
    d->tr_radius = 1e3;    // TrustRegion(radius=1e3, max=1e8, up=2.0, down=0.5**4) (global_positioning.py:158)
    d->tr_max = 1e8;
}

int insfm_gp_create(const insfm_ba_desc* desc, const double* trans, const int32_t* cam_idx, const int32_t* pt_idx,
                    const double* cam_factor, const int32_t* scale_free, void* stream, insfm_ba** out) {
    return create_impl(desc, 1, trans, cam_idx, pt_idx, cam_factor, scale_free, stream, out);
}

// Positions, the shard's points and the scales between the caller's buffers and the LM state (one k_gp_io launch).
static int gp_io(insfm_ba* h, int in, const double* pos, const double* pts, const double* scales) {
    const long long n3c = 3LL * h->C, n3p = 3LL * h->Pl, nl = h->Nl, tot = n3c + n3p + nl;
    if (tot == 0) return 0;
    const int grid = std::max(1, std::min(2048, cdiv(tot, kThreads)));
    k_gp_io<<<grid, kThreads, 0, h->stream>>>(in, n3c, const_cast<double*>(pos), h->cams_cur, n3p,
                                              const_cast<double*>(pts) + 3 * (size_t)h->p0, h->pts_cur, nl, h->osrc,
                                              const_cast<double*>(scales), h->scl_cur);
    return launch_err(h, "k_gp_io");
}

int insfm_gp_step(insfm_ba* h, double* pos, double* pts, double* scales, insfm_ba_stats* st) {
    if (!h || !pos || !pts || !scales || h->kind != 1) return INSFM_BA_EINVAL;
    int rc = gp_io(h, 1, pos, pts, scales);
    if (rc) return rc;
    if ((rc = lm_step(h, st))) return rc;
    // written back in stream order (no host wait: the step's loss is already on the host), like insfm_ba_step
    return gp_io(h, 0, pos, pts, scales);
}

int insfm_gp_cost(insfm_ba* h, const double* pos, const double* pts, const double* scales, double* loss, double* rmse) {
    if (!h || !pos || !pts || !scales || h->kind != 1) return INSFM_BA_EINVAL;
    HIPCHK(hipMemsetAsync(h->flags, 0, sizeof(int) * 4, h->stream));
    // scratch copies (the LM's current state is untouched: cams_new / pts_new / scl_new are trial buffers)
    HIPCHK(hipMemcpyAsync(h->cams_new, pos, sizeof(double) * 3 * (size_t)h->C, hipMemcpyDeviceToDevice, h->stream));
    if (h->Nl) k_gp_gather<<<cdiv(h->Nl, kThreads), kThreads, 0, h->stream>>>(h->Nl, h->osrc, scales, h->scl_new);
    int rc = launch_err(h, "k_gp_gather");
    if (rc) return rc;
    if ((rc = run_cost(h, h->cams_new, pts + 3 * (size_t)h->p0, false, h->scl_new))) return rc;
    if (loss) *loss = h->host_res[0];
    if (rmse) *rmse = h->N > 0 ? std::sqrt(h->host_res[1] / h->N) : 0.0;
    return INSFM_BA_OK;
}

int insfm_gp_debug_linearize(insfm_ba* h, const double* pos, const double* pts, const double* scales) {
    if (!h || !pos || !pts || !scales || h->kind != 1) return INSFM_BA_EINVAL;
    h->keep_S = 1;
    int rc = gp_io(h, 1, pos, pts, scales);
    if (rc) return rc;
    if ((rc = run_linearize(h, h->cams_cur, h->pts_cur))) return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
    return 0;
}

int64_t insfm_gp_debug_get_ds(insfm_ba* h, double* host_out) {
    if (!h || !host_out || h->kind != 1) return INSFM_BA_EINVAL;
    std::vector<double> loc(h->Nl);
    if (h->Nl) HIPCHK(hipMemcpyAsync(loc.data(), h->ds, sizeof(double) * h->Nl, hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    std::memset(host_out, 0, sizeof(double) * (size_t)h->N);
    for (int o = 0; o < h->Nl; ++o) host_out[h->osrc_host[o]] = loc[o];
    return h->N;
}

}  // extern "C"

