// Schur complement with the camera-point blocks re-derived instead of read (BA, non-deterministic mode).
//
// S_ij = U_i [i = j] - sum_{tracks p seen by i and j} W_ip V_p^-1 W_jp^T, with W_o = J~c_o^T J~p_o.  Each observation's
// weighted Jacobian is a function of (camera row, point, Huber weight), so instead of storing W (192 B / observation,
// re-read ~4.5x by the rows that share its track: 1.55 GB of gathers per launch on config 3) the kernel stores per
// observation only {sqrt(w), camera} (16 B, written by k_lin_points) and per point {V^-1, y, X} (96 B, written by
// k_point_prep), and evaluates J~ again from a per-row LDS table of the row's neighbour cameras (rotation matrix,
// translation, intrinsics: 12 + NI doubles each).
//
// Because every residual is 2-dimensional, a pair's block is rank 2:
//   W^_a W_q^T = J~c_a^T (A_a J~p_q^T) J~c_q,   A_a = J~p_a V_p^-1 (2x3, once per own observation),
// i.e. M = A_a J~p_q^T (2x2, 12 FMA), T = M J~c_q (2xD), block += J~c_a^T T (2 D^2 FMA).
//
// Work mapping: one workgroup per (camera row i, chunk of its upper blocks), as k_schur; ONE LANE per own observation
// a of camera i, walking a's upper partners q (the contiguous camera-sorted tail of its track, a itself first) and
// adding each D x D block into the LDS row with ds_add_f64.  Same-address collisions are spread two ways: each lane
// starts its partner walk at (lane mod n), and walks the block's rows in a lane-rotated order (row (k + lane) mod D
// at step k), so lanes that hit the same partner camera in the same step still add to different rows.  The block
// stride is odd, so different partner slots fall on different LDS banks.
#pragma once
#include <hip/hip_runtime.h>

#include "ba_common.h"
#include "ba_device.h"

#ifndef SCHUR_RC_PROBE
#define SCHUR_RC_PROBE 0  // timing-only variants (results wrong): 1 no LDS adds, 2 no partner Jacobian, 3 both
#endif
#ifndef SCHUR_RC_UP
#define SCHUR_RC_UP 10  // partner records in flight per own observation (longer partner lists: more batches)
#endif
#ifndef SCHUR_RC_ROT
#define SCHUR_RC_ROT 1  // lane-rotated partner start and block rows
#endif

namespace insfm {

template <int M> constexpr int kCamTab = 12 + Model<M>::NI;  // per camera in LDS: R (row-major 3x3), t, intrinsics
// LDS block layout.  D = 8: blocks of exactly 64 doubles (every block starts on the same bank) with row a's columns
// XOR-swizzled by 4 (a >> 2): a lane-rotated row order then puts the 8 lanes of each 8-lane run on 8 distinct bank
// pairs in every add, whatever partner slots they hit.  Other D: an odd block stride (slots spread over the banks).
__host__ __device__ constexpr int schur_rc_bs(int D) { return D == 8 ? 64 : ((D * D) | 1); }
__host__ __device__ constexpr int schur_rc_swz(int D, int a) { return D == 8 ? 4 * (a >> 2) : 0; }

// R = I + 2w[q]x + 2[q]x^2 (the matrix of the action eval_obs applies), t, intrinsics -> dst[kCamTab<M>]
template <int M>
__device__ __forceinline__ void camtab_fill(const double* __restrict__ cam, double* dst) {
    constexpr int NI = Model<M>::NI;
    const double qx = cam[3], qy = cam[4], qz = cam[5], qw = cam[6];
    const double K[3][3] = {{0.0, -qz, qy}, {qz, 0.0, -qx}, {-qy, qx, 0.0}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const double kk = K[i][0] * K[0][j] + K[i][1] * K[1][j] + K[i][2] * K[2][j];
            dst[3 * i + j] = (i == j ? 1.0 : 0.0) + 2.0 * qw * K[i][j] + 2.0 * kk;
        }
    dst[9] = cam[0]; dst[10] = cam[1]; dst[11] = cam[2];
#pragma unroll
    for (int k = 0; k < NI; ++k) dst[12 + k] = cam[7 + k];
}

// Weighted Jacobians of one observation from a camera table entry (same formulas as eval_obs<M, true>, with the
// rotation given as a matrix; pp does not enter the Jacobian).  sw = sqrt of the Huber weight.
template <int M>
__device__ __forceinline__ void eval_jac_tab(const double* __restrict__ ct, const double X[3], double sw,
                                             double (*Jc)[kD<M>], double (*Jp)[3]) {
    constexpr int NF = Model<M>::NF;
    constexpr int NK = Model<M>::NI - NF;
    const double px = ct[0] * X[0] + ct[1] * X[1] + ct[2] * X[2] + ct[9];
    const double py = ct[3] * X[0] + ct[4] * X[1] + ct[5] * X[2] + ct[10];
    const double pz = ct[6] * X[0] + ct[7] * X[1] + ct[8] * X[2] + ct[11];
    const double iz = 1.0 / pz;
    const double u = px * iz, v = py * iz;
    double du, dv, Jd[4];
    double Jk[2][NK > 0 ? NK : 1];
    distort<M>(ct + 12 + NF, u, v, du, dv, Jd, Jk);
    const double fx = ct[12] * sw;
    const double fy = ((NF == 2) ? ct[13] : ct[12]) * sw;
    const double duv0[3] = {iz, 0.0, -u * iz};
    const double duv1[3] = {0.0, iz, -v * iz};
    double A[2][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        A[0][c] = fx * (Jd[0] * duv0[c] + Jd[1] * duv1[c]);
        A[1][c] = fy * (Jd[2] * duv0[c] + Jd[3] * duv1[c]);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 3; ++j) Jp[a][j] = A[a][0] * ct[j] + A[a][1] * ct[3 + j] + A[a][2] * ct[6 + j];
    const double ex[3][3] = {{0.0, -pz, py}, {pz, 0.0, -px}, {-py, px, 0.0}};
#pragma unroll
    for (int a = 0; a < 2; ++a) {
        Jc[a][0] = A[a][0]; Jc[a][1] = A[a][1]; Jc[a][2] = A[a][2];
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) Jc[a][3 + kk] = A[a][0] * ex[kk][0] + A[a][1] * ex[kk][1] + A[a][2] * ex[kk][2];
    }
    if constexpr (NF == 1) {
        Jc[0][6] = du * sw; Jc[1][6] = dv * sw;
    } else {
        Jc[0][6] = du * sw; Jc[0][7] = 0.0; Jc[1][6] = 0.0; Jc[1][7] = dv * sw;
    }
#pragma unroll
    for (int j = 0; j < NK; ++j) { Jc[0][6 + NF + j] = fx * Jk[0][j]; Jc[1][6 + NF + j] = fy * Jk[1][j]; }
}

// LDS layout of one work item: acc [nb][BS] | camera table [(nb + 1)][CT] (slot nb = the row's own camera) |
// b [D] | slot [C] (ints)
template <int M>
inline size_t schur_rc_lds_bytes(int nb, int C) {
    constexpr int D = kD<M>;
    const size_t dbl = (size_t)nb * schur_rc_bs(D) + (size_t)(nb + 1) * kCamTab<M> + D;
    return ((sizeof(double) * dbl + sizeof(int) * (size_t)C) + 15) & ~(size_t)15;
}

template <int M, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_schur_rc(const int4* __restrict__ work, const int* __restrict__ row_ptr,
                                                         const int* __restrict__ col, int C, const int* __restrict__ cam_ptr,
                                                         const int4* __restrict__ sdesc, const double2* __restrict__ obrec,
                                                         const double* __restrict__ ptrec, const double* __restrict__ cams,
                                                         const double* __restrict__ U, const double* __restrict__ gc,
                                                         double f, double cmin, double cmax, int add_diag,
                                                         double* __restrict__ S, double* __restrict__ b) {
    constexpr int D = kD<M>, ST = kStride<M>, DD = D * D, BS = schur_rc_bs(D), CT = kCamTab<M>;
    constexpr int NT = WAVES * 64;
    constexpr int UP = SCHUR_RC_UP;
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const int4 wk = work[blockIdx.x];
    const int i = wk.x, kb = wk.y, ke = wk.z, nb = ke - kb;
    double* acc = sh;
    double* ctab = acc + (size_t)nb * BS;
    double* bacc = ctab + (size_t)(nb + 1) * CT;
    int* slot = reinterpret_cast<int*>(bacc + D);
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int k = t; k < nb * BS; k += NT) acc[k] = 0.0;
    for (int k = t; k < C; k += NT) slot[k] = -1;
    if (t < D) bacc[t] = 0.0;
    for (int e = t; e <= nb; e += NT) camtab_fill<M>(cams + (size_t)(e < nb ? col[kb + e] : i) * ST, ctab + (size_t)e * CT);
    __syncthreads();
    for (int e = kb + t; e < ke; e += NT) slot[col[e]] = e - kb;
    __syncthreads();
    const bool diag_chunk = (kb == row_ptr[i]);
    const double* own = ctab + (size_t)nb * CT;
    const int rot = SCHUR_RC_ROT ? lane % D : 0;
    int rowoff[D], colx[D];  // this lane's row order: row (k + rot) mod D at step k, and its column swizzle
#pragma unroll
    for (int k = 0; k < D; ++k) {
        rowoff[k] = ((k + rot) % D) * D;
        colx[k] = schur_rc_swz(D, (k + rot) % D);
    }
    double breg[D];
#pragma unroll
    for (int a = 0; a < D; ++a) breg[a] = 0.0;
    double probe_sum = 0.0;
    const int ob = cam_ptr[i], oe = cam_ptr[i + 1];
    // own-observation inputs of the NEXT round are loaded while the current round's partners are processed
    int4 dn = make_int4(0, 0, 0, 0);
    double2 pn[6];
    double san = 0.0;
    auto load_own = [&](int e) {
        if (e < oe) {
            dn = sdesc[e];
            const double2* pr = reinterpret_cast<const double2*>(ptrec + 12 * (size_t)dn.y);
#pragma unroll
            for (int k = 0; k < 6; ++k) pn[k] = pr[k];
            san = obrec[dn.x].x;
        }
    };
    load_own(ob + wv * 64 + lane);
    for (int base = ob + wv * 64; base < oe; base += NT) {
        const int e = base + lane;
        const bool has = e < oe;
        const int4 dsc = has ? dn : make_int4(0, 0, 0, 0);
        double X[3] = {0.0, 0.0, 1.0}, vi[6] = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0}, yv[3] = {0.0, 0.0, 0.0}, sa = 0.0;
        if (has) {
            vi[0] = pn[0].x; vi[1] = pn[0].y; vi[2] = pn[1].x; vi[3] = pn[1].y; vi[4] = pn[2].x; vi[5] = pn[2].y;
            yv[0] = pn[3].x; yv[1] = pn[3].y; yv[2] = pn[4].x;
            X[0] = pn[4].y; X[1] = pn[5].x; X[2] = pn[5].y;
            sa = san;
        }
        // every partner record of this round in flight at once (the tail of one track: one or two cache lines), in
        // the lane's rotated order
        const int qs = dsc.z, n = has ? dsc.w - dsc.z : 0;
        const int start = (SCHUR_RC_ROT && n > 0) ? lane % n : 0;
        double psw[UP];
        int pcam[UP];
#pragma unroll
        for (int u = 0; u < UP; ++u) {
            pcam[u] = -1;
            psw[u] = 0.0;
            if (u < n) {
                int j = start + u;
                if (j >= n) j -= n;
                const double2 r = obrec[qs + j];
                psw[u] = r.x;
                pcam[u] = (int)r.y;
            }
        }
        load_own(e + NT);
        double Jc[2][D], Jp[2][3];
        eval_jac_tab<M>(own, X, sa, Jc, Jp);
        // A = J~p V^-1 (V^-1 packed symmetric)
        double A[2][3];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            A[r][0] = Jp[r][0] * vi[0] + Jp[r][1] * vi[1] + Jp[r][2] * vi[2];
            A[r][1] = Jp[r][0] * vi[1] + Jp[r][1] * vi[3] + Jp[r][2] * vi[4];
            A[r][2] = Jp[r][0] * vi[2] + Jp[r][1] * vi[4] + Jp[r][2] * vi[5];
        }
        if (diag_chunk && has) {  // b_i -= W_a y_p = J~c^T (J~p y)
            const double j0 = Jp[0][0] * yv[0] + Jp[0][1] * yv[1] + Jp[0][2] * yv[2];
            const double j1 = Jp[1][0] * yv[0] + Jp[1][1] * yv[1] + Jp[1][2] * yv[2];
#pragma unroll
            for (int a = 0; a < D; ++a) breg[a] -= Jc[0][a] * j0 + Jc[1][a] * j1;
        }
        // the own Jacobian's columns in this lane's rotated row order (one dynamic index per own observation)
        double Jr[2][D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const int a = (k + rot) % D;
            double v0 = 0.0, v1 = 0.0;
#pragma unroll
            for (int m = 0; m < D; ++m)
                if (m == a) { v0 = Jc[0][m]; v1 = Jc[1][m]; }
            Jr[0][k] = v0; Jr[1][k] = v1;
        }
        // rounds while any lane has partners left (ballot: no ds_bpermute on the LDS pipe, as in k_schur)
        for (int k0 = 0; __builtin_amdgcn_ballot_w64(k0 < n) != 0; k0 += UP) {
            if (k0 > 0) {  // tracks longer than UP + 1 observations: the next batch of partners
#pragma unroll
                for (int u = 0; u < UP; ++u) {
                    pcam[u] = -1;
                    if (k0 + u < n) {
                        int j = start + k0 + u;
                        while (j >= n) j -= n;
                        const double2 r = obrec[qs + j];
                        psw[u] = r.x;
                        pcam[u] = (int)r.y;
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < UP; ++u) {
                if (pcam[u] < 0) continue;
                const int sl = slot[pcam[u]];
                if (sl < 0) continue;
                double Jcq[2][D], Jpq[2][3];
                if constexpr ((SCHUR_RC_PROBE & 2) != 0) {
                    const double* ctp = ctab + (size_t)sl * CT;
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
#pragma unroll
                        for (int m = 0; m < D; ++m) Jcq[r][m] = Jc[r][m] * psw[u] + ctp[m];
#pragma unroll
                        for (int m = 0; m < 3; ++m) Jpq[r][m] = Jp[r][m] * psw[u];
                    }
                } else {
                    eval_jac_tab<M>(ctab + (size_t)sl * CT, X, psw[u], Jcq, Jpq);
                }
                double M2[2][2];
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
                        M2[r][s2] = A[r][0] * Jpq[s2][0] + A[r][1] * Jpq[s2][1] + A[r][2] * Jpq[s2][2];
                double T[2][D];
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int bb = 0; bb < D; ++bb) T[r][bb] = M2[r][0] * Jcq[0][bb] + M2[r][1] * Jcq[1][bb];
                double* dst = acc + (size_t)sl * BS;
                if constexpr ((SCHUR_RC_PROBE & 1) != 0) {
                    double sum = 0.0;
#pragma unroll
                    for (int k = 0; k < D; ++k)
#pragma unroll
                        for (int bb = 0; bb < D; ++bb) sum += Jr[0][k] * T[0][bb] + Jr[1][k] * T[1][bb];
                    probe_sum += sum;
                } else {
#pragma unroll
                    for (int k = 0; k < D; ++k)
#pragma unroll
                        for (int bb = 0; bb < D; ++bb)
                            atomicAdd(dst + rowoff[k] + (bb ^ colx[k]), -(Jr[0][k] * T[0][bb] + Jr[1][k] * T[1][bb]));
                }
            }
        }
    }
    if constexpr ((SCHUR_RC_PROBE & 1) != 0) atomicAdd(acc + lane % (nb > 0 ? nb : 1), probe_sum);
    if (diag_chunk) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double s = wave_sum(breg[a]);
            if (lane == 0) atomicAdd(bacc + a, s);
        }
    }
    __syncthreads();
    double* Sout = S + (size_t)kb * DD;
    const double* Ui = U + (size_t)i * DD;
    for (int k = t; k < nb * DD; k += NT) {
        const int a2_ = (k % DD) / D, b2_ = k % D;
        double v = acc[(k / DD) * BS + a2_ * D + (b2_ ^ schur_rc_swz(D, a2_))];
        if (diag_chunk && add_diag && k < DD) {
            const int a2 = k / D, bb = k % D;
            double u = Ui[k];
            if (a2 == bb) u = clampd(u, cmin, cmax) * f;
            v += u;
        }
        Sout[k] = v;
    }
    if (diag_chunk && t < D) b[(size_t)i * D + t] = (add_diag ? gc[(size_t)i * D + t] : 0.0) + bacc[t];
}

}  // namespace insfm
