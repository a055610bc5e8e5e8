// Two-level preconditioner for the reduced camera system (included by ba_kernels.hip and tools/bench_dense.hip).
//
// In the scaled space of the block-Jacobi CG (S~ = L^-1 S L^-T, diag blocks I) the preconditioner is
//     M~^-1 = I + Z~ E^-1 Z~^T,   Z~_i = L_i^T G_i,   E = Z~^T S~ Z~            (oracle/ba_oracle.c: ora_coarse_setup)
// where G_i (D x MC, MC = D + 1) spans camera i's response to an infinitesimal similarity of the world (3 translation,
// 3 rotation, 1 scale) plus one unit column per intrinsic, and the columns of a camera cluster share coarse unknowns.
// These are the smooth, low-energy modes that block-Jacobi cannot reduce (a cluster of cameras moving rigidly together
// barely changes the reprojection error), so the coarse correction removes the slow tail of the CG.
//
// Setup per trial (after k_cg_factor / k_cg_scale):
//   k_tl_basis   : Z~ per (camera, coarse column)
//   k_tl_erow    : per camera row and neighbour cluster, sum of Z~_i^T S~_ij Z~_j (+ Z~_i^T Z~_i), LDS-staged
//   k_tl_ereduce : E[(c',k),(c,l)] = fixed-order sum of the row segments of cluster pair (c', c)
//   k_gj_step    : E^-1 by blocked Gauss-Jordan inversion, one launch per 64-wide block step (f64 MFMA)
// Per CG iteration (pipelined PCG, same stopping rule as block-Jacobi; see the section below):
//   k_tl_pc      : per cluster: recurrence scalars from the row partials, restriction, y = E^-1 R (its MC rows),
//                  m_i = w_i + Z~_i y_c
//   k_tl_pspmv   : n = S~ m (row-contiguous Sn stream), the row's vector updates, its partials for the next iteration
#pragma once
#include <algorithm>
#include <utility>

#include "ba_common.h"

#ifndef COARSE_MAX_DIM
#define COARSE_MAX_DIM 768
#endif
#include "ba_device.h"
#include "ba_xpart.h"

namespace insfm {

constexpr int kCoarseMax = COARSE_MAX_DIM;  // nclust * (D + 1) cap (k_tl_pc keeps a cluster's E^-1 rows in registers)

struct TlBufs {
    double* u;           // [C*D]  preconditioned residual
    double* Zt;          // [C][D][MC]
    double* Ztc;         // [C][D][MC] the same rows in cluster-member order (cpos)
    double* Gb;          // [C][D][MC] the unscaled basis G_i (Z~_i = L_i^T G_i; k_tl_cgp's A_ic); nullptr: not kept
    double* vc;          // [C][D] the vector k_tl_pc reads (r0 at setup, w after), rows in cluster-member order
    double* Rc;          // [m]   (debug) restriction
    double* gd;          // [3][C] row partials r_i.u_i | w_i.u_i | ||L_i r_i||^2 (k_tl_pspmv), rows in cluster-member order
    double* rowR;        // [C][MC] row partials of the restriction Z~_i^T w_i, rows in cluster-member order (cpos)
    // atomic cluster sums (single GPU, non-deterministic mode; nullptr otherwise): k_tl_pspmv adds each row's
    // restriction and scalar partials into its cluster's entries with no-return f64 atomics, double-buffered by
    // iteration parity (k_tl_pc of iteration i reads buffer i & 1 and clears buffer (i + 1) & 1 for k_tl_pspmv);
    // k_tl_cgp uses three buffers (i mod 3)
    double* Racc;        // [3][m]
    double* Gacc;        // [3][3][nc]
    double* Oseg;        // [nseg][MC][MC] per (row, neighbour cluster) sums of Z~_i^T S~_ij Z~_j
    double* E;           // [ldE][ldE] coarse matrix padded to whole kGB blocks (pad: identity), inverted in place
    double* Einv;        // [m][m] compact E^-1 (k_tl_pc reads its cluster's rows)
    double* Ed;          // [ldE] 1 / sqrt(E_kk) (pad: 1): E is inverted as diag(Ed) E diag(Ed) (symmetric equilibration)
    int* ok;             // coarse correction usable (E positive definite)
    const int* cl_ptr;   // [nc+1]
    const int* cl_cams;  // cluster members, ascending camera id
    const int* cpos;     // [C] position of camera i in cl_cams
    const int* clab;     // [C] cluster of camera i
    const int* alone;    // [C] camera is alone in its cluster -> basis [I_D | 0]
    const int* sperm;    // [n_nbr] neighbour slots of each row ordered by (cluster of the neighbour, slot)
    const int4* seg;     // [nseg] (cluster, sorted begin, sorted end, own-cluster flag) per (row, neighbour cluster)
    const int* rseg_ptr; // [C+1] segments of each row
    const int* ered_ptr; // [nc*nc+1]
    const int* ered_seg; // segment ids of each cluster pair, rows ascending
    int nc, m, maxmem, ldE;
};

// Hand-off of the row partials to the cluster's last-arriving workgroup inside one k_tl_pspmv launch: every partial is
// stored write-through (sc1), the storing wave waits for its stores (vmcnt(0)) before its one agent-scope counter add,
// and the last arriver reads them with sc1 loads (MI355X_MICROARCH.md, hand-off table row 1: no L2 write-back, no
// acquire).  Relaxed agent-scope atomic load / store lower to global_load / global_store ... sc1 on gfx950.
__device__ __forceinline__ void st_sc1(double* p, double v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ double ld_sc1(const double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// ---- setup ---------------------------------------------------------------------------------------------------
// One workgroup per camera cluster c, one thread per (member camera i, coarse column k): column k of G_i at the
// linearization point and Z~_i[:,k] = L_i^T G_i[:,k], the row partial Z~_i[:,k]^T r0_i of the restriction of the CG's
// starting residual; then the cluster's restriction R_c[k] = sum of its members' partials in cluster order (k_tl_pc's
// order of additions) into tl.Rc (k_tl_cgp's coarse solve of r0 reads it; k_tl_pc sums the partials itself).
template <int M>
__device__ __forceinline__ void tl_basis_entry(int i, int k, const double* __restrict__ cams, const double* __restrict__ Lf,
                                               const TlBufs& tl, const double* __restrict__ r0);

template <int M>
__global__ __launch_bounds__(kThreads) void k_tl_basis(int C, const double* __restrict__ cams, const double* __restrict__ Lf,
                                                       TlBufs tl, const double* __restrict__ r0,
                                                       long long* stp = nullptr) {
    const StampScope stamp_(stp);
    constexpr int D = kD<M>, MC = D + 1;
    const int c = blockIdx.x, e0 = tl.cl_ptr[c], ne = tl.cl_ptr[c + 1] - e0;
    for (int g = threadIdx.x; g < ne * MC; g += kThreads) tl_basis_entry<M>(tl.cl_cams[e0 + g / MC], g % MC, cams, Lf, tl, r0);
    __syncthreads();  // (the block's rowR stores are visible to the block behind the barrier)
    if (threadIdx.x < MC) {
        const int k = threadIdx.x;
        double v = 0.0;
        for (int e = 0; e < ne; ++e) v += tl.rowR[(size_t)(e0 + e) * MC + k];
        tl.Rc[(size_t)c * MC + k] = v;
    }
    (void)D;
    (void)C;
}

// Column k of a BA camera's G_i (D x (D + 1)): the response of its pose [rho, phi] and intrinsics to an infinitesimal
// similarity of the world -- 3 translations (k < 3), 3 rotations (k < 6), scale (k = 6) -- then one unit column per
// intrinsic; a camera alone in its cluster gets [I_D | 0].  cp: the camera row [t, q_xyzw, intrinsics].
template <int D>
__device__ __forceinline__ void basis_column(int k, const double* __restrict__ cp, bool alone, double (&col)[D]) {
#pragma unroll
    for (int a = 0; a < D; ++a) col[a] = 0.0;
    if (alone) {
        if (k < D) col[k] = 1.0;
        return;
    }
    const double t0 = cp[0], t1 = cp[1], t2 = cp[2];
    const double qx = cp[3], qy = cp[4], qz = cp[5], w = cp[6];
    // R = I + 2w[q]x + 2[q]x^2 (same form as the retraction / projection)
    const double K[9] = {0, -qz, qy, qz, 0, -qx, -qy, qx, 0};
    double R[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            double kk = 0.0;
#pragma unroll
            for (int l = 0; l < 3; ++l) kk += K[r * 3 + l] * K[l * 3 + c];
            R[r * 3 + c] = (r == c ? 1.0 : 0.0) + 2.0 * w * K[r * 3 + c] + 2.0 * kk;
        }
    const double tx[9] = {0, -t2, t1, t2, 0, -t0, -t1, t0, 0};
    if (k < 3) {
#pragma unroll
        for (int a = 0; a < 3; ++a) col[a] = -R[a * 3 + k];
    } else if (k < 6) {
        const int kk = k - 3;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double s = 0.0;
#pragma unroll
            for (int l = 0; l < 3; ++l) s += tx[a * 3 + l] * R[l * 3 + kk];
            col[a] = -s;
            col[3 + a] = -R[a * 3 + kk];
        }
    } else if (k == 6) {
        col[0] = t0; col[1] = t1; col[2] = t2;
    } else {
        col[6 + (k - 7)] = 1.0;
    }
}

template <int M>
__device__ __forceinline__ void tl_basis_entry(int i, int k, const double* __restrict__ cams, const double* __restrict__ Lf,
                                               const TlBufs& tl, const double* __restrict__ r0) {
    constexpr int D = kD<M>, MC = D + 1, ST = kStride<M>;
    double col[D];
    if constexpr (M == kGP) {  // global positioning: translation (I) and scaling about the origin (c_i)
#pragma unroll
        for (int a = 0; a < D; ++a) col[a] = 0.0;
        if (tl.alone[i]) {
            if (k < D) col[k] = 1.0;
        } else {
            const double* cp = cams + (size_t)i * ST;
            if (k < 3) col[k] = 1.0;
            else { col[0] = cp[0]; col[1] = cp[1]; col[2] = cp[2]; }
        }
    } else {
        basis_column<D>(k, cams + (size_t)i * ST, tl.alone[i] != 0, col);
    }
    const double* L = Lf + (size_t)i * D * D;
    const double* r = r0 + (size_t)i * D;
    double rr = 0.0;  // restriction partial of the CG's starting residual sum_a Z~[a][k] r0_a, a ascending
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double s = 0.0;
#pragma unroll
        for (int l = a; l < D; ++l) s += L[l * D + a] * col[l];
        tl.Zt[((size_t)i * D + a) * MC + k] = s;
        if (tl.Gb) tl.Gb[((size_t)i * D + a) * MC + k] = col[a];
        tl.Ztc[((size_t)tl.cpos[i] * D + a) * MC + k] = s;
        rr += s * r[a];
    }
    tl.rowR[(size_t)tl.cpos[i] * MC + k] = rr;
    if (k < D) tl.vc[(size_t)tl.cpos[i] * D + k] = r[k];
}

// One workgroup per camera row i (rows strided over the grid), its 4 waves taking the row's neighbour-cluster
// segments round-robin.  Per segment c: A = sum over the segment's neighbours j (slot order) of S~_ij Z~_j (D x MC,
// one output entry per lane and round, the block and Z~_j staged through the wave's own LDS slice), then
// Oseg = [c == c_i] Z~_i^T Z~_i + Z~_i^T A (MC x MC).  The next block's loads are issued before the current block's
// products, so each wave keeps one block in flight while it computes.  No workgroup-wide barrier after the start:
// a wave's LDS slice is private and LDS operations of one wave complete in order.
template <int D>
struct ErowGeom {
    static constexpr int MC = D + 1;
    static constexpr int DP = D + (D & 1);
    static constexpr int SB = D * DP, ZB = D * MC, MM = MC * MC;
    static constexpr int NS = (SB + 63) / 64, NZ = (ZB + 63) / 64, NO = (MM + 63) / 64;
};

template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_erow(int C, const int* __restrict__ nbr_ptr, const int* __restrict__ nbr_j,
                                                      const double* __restrict__ Sn, TlBufs tl) {
    using G = ErowGeom<D>;
    constexpr int MC = G::MC, DP = G::DP, SB = G::SB, ZB = G::ZB, MM = G::MM, NS = G::NS, NZ = G::NZ, NO = G::NO;
    constexpr int NWV = kThreads / 64;
    __shared__ __attribute__((aligned(16))) double Zi[ZB];         // Z~_i, a-major
    __shared__ __attribute__((aligned(16))) double Sb[NWV][SB];    // the wave's current block, row-major (stride DP)
    __shared__ __attribute__((aligned(16))) double Zs[NWV][ZB];    // Z~_j transposed: Zs[l * D + b] = Z~_j[b][l]
    __shared__ __attribute__((aligned(16))) double As[NWV][ZB];    // the segment's A, a-major
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int i = blockIdx.x; i < C; i += gridDim.x) {
        __syncthreads();
        for (int e = t; e < ZB; e += kThreads) Zi[e] = tl.Zt[(size_t)i * ZB + e];
        __syncthreads();
        const int n0 = nbr_ptr[i];
        const int s0 = tl.rseg_ptr[i], s1 = tl.rseg_ptr[i + 1];
        for (int s = s0 + wv; s < s1; s += NWV) {
            const int4 sg = tl.seg[s];
            double acc[NZ];
#pragma unroll
            for (int u = 0; u < NZ; ++u) acc[u] = 0.0;
            double sv[NS], zv[NZ];
            auto load = [&](int q) {
                const int nb = tl.sperm[n0 + q];
                const int j = nbr_j[nb];
#pragma unroll
                for (int u = 0; u < NS; ++u) sv[u] = Sn[(size_t)nb * SB + min(lane + 64 * u, SB - 1)];
#pragma unroll
                for (int u = 0; u < NZ; ++u) zv[u] = tl.Zt[(size_t)j * ZB + min(lane + 64 * u, ZB - 1)];
            };
            if (sg.y < sg.z) load(sg.y);
            for (int q = sg.y; q < sg.z; ++q) {
#pragma unroll
                for (int u = 0; u < NS; ++u) {
                    const int e = lane + 64 * u;
                    if (e < SB) Sb[wv][e] = sv[u];
                }
#pragma unroll
                for (int u = 0; u < NZ; ++u) {
                    const int e = lane + 64 * u;
                    if (e < ZB) Zs[wv][(e % MC) * D + e / MC] = zv[u];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (q + 1 < sg.z) load(q + 1);
#pragma unroll
                for (int u = 0; u < NZ; ++u) {
                    const int o = min(lane + 64 * u, ZB - 1), a = o / MC, l = o % MC;
                    double v = 0.0;
                    if constexpr ((D & 1) == 0) {  // 16-byte LDS reads (row a of the block, column l of Z~_j)
                        const double2* sr = reinterpret_cast<const double2*>(&Sb[wv][a * DP]);
                        const double2* zc = reinterpret_cast<const double2*>(&Zs[wv][l * D]);
#pragma unroll
                        for (int b = 0; b < D / 2; ++b) {
                            const double2 x = sr[b], y = zc[b];
                            v += x.x * y.x;
                            v += x.y * y.y;
                        }
                    } else {
#pragma unroll
                        for (int b = 0; b < D; ++b) v += Sb[wv][a * DP + b] * Zs[wv][l * D + b];
                    }
                    acc[u] += v;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
#pragma unroll
            for (int u = 0; u < NZ; ++u) {
                const int e = lane + 64 * u;
                if (e < ZB) As[wv][e] = acc[u];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int u = 0; u < NO; ++u) {
                const int o = lane + 64 * u;
                if (o < MM) {
                    const int k = o / MC, l = o % MC;
                    double v = 0.0;
                    if (sg.w) {
#pragma unroll
                        for (int a = 0; a < D; ++a) v += Zi[a * MC + k] * Zi[a * MC + l];
                    }
#pragma unroll
                    for (int a = 0; a < D; ++a) v += Zi[a * MC + k] * As[wv][a * MC + l];
                    tl.Oseg[(size_t)s * MM + o] = v;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
}

// One thread per entry of E: fixed-order sum of the cluster pair's segments (rows ascending); an exactly-zero
// diagonal entry (the unused column of a single-camera cluster) becomes 1.
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_ereduce(TlBufs tl) {
    constexpr int MC = D + 1, MM = MC * MC;
    const int m = tl.m, nc = tl.nc;
    const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (g >= (int64_t)m * m) return;
    const int r = (int)(g / m), q = (int)(g % m);
    const int cr = r / MC, k = r % MC, cq = q / MC, l = q % MC;
    const int s0 = tl.ered_ptr[cr * nc + cq], s1 = tl.ered_ptr[cr * nc + cq + 1];
    const double* O = tl.Oseg + k * MC + l;
    double acc = 0.0;
    int e = s0;
    for (; e + 4 <= s1; e += 4) {
        const int a0 = tl.ered_seg[e], a1 = tl.ered_seg[e + 1], a2 = tl.ered_seg[e + 2], a3 = tl.ered_seg[e + 3];
        const double v0 = O[(size_t)a0 * MM], v1 = O[(size_t)a1 * MM], v2 = O[(size_t)a2 * MM], v3 = O[(size_t)a3 * MM];
        acc += v0; acc += v1; acc += v2; acc += v3;
    }
    for (; e < s1; ++e) acc += O[(size_t)tl.ered_seg[e] * MM];
    if (r == q && acc == 0.0) acc = 1.0;
    tl.E[(size_t)r * tl.ldE + q] = acc;
    if (r == q) tl.Ed[r] = 1.0 / sqrt(acc);  // equilibration (k_gj_equil); NaN for a non-positive diagonal
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// ---- E^-1 by blocked Gauss-Jordan inversion (multi-workgroup, f64 MFMA) -------------------------------------------
// E (m x m, SPD) is held padded to ld = nB * kGB (pad: identity), symmetrically equilibrated on the fly
// (d = 1 / sqrt(diag E), from k_tl_ereduce; the pad's d is 1) and inverted by block Gauss-Jordan steps k = 0..nB-1
// with pivot block P = X_kk (no pivoting: every pivot block of an SPD matrix is SPD):
//   Y_kk = P^-1,  Y_kj = P^-1 X_kj,  Y_ik = -X_ik P^-1,  Y_ij = X_ij - X_ik (P^-1 X_kj)      (i, j != k)
// One launch per step (k_gj_step: nB x nB workgroups, one 32 x 32 tile each, v_mfma_f64_16x16x4f64), ping-ponging
// between two buffers so that no workgroup reads a tile another one writes in the same launch.  P^-1 is looked
// ahead: the workgroup that forms the next pivot block Y_{k+1,k+1} inverts it right away (k_gj_pinv0 does P_0) by
// scalar in-place Gauss-Jordan in one wave's registers (lane r = row r, pivot rows broadcast by readlane), so the
// other workgroups only load it.  The last step writes diag(d) Y diag(d) compactly (row stride m) for k_tl_pc.
// 2 m^3 flops in nB + 1 launches; the oracle (ba_oracle.c gj_inverse) runs the same steps, pivots and fused
// multiply-adds.
constexpr int kGB = 32;        // block size
constexpr int kGS = kGB + 1;   // LDS row stride (odd: the A-fragment column reads are conflict-free)
typedef double gj_acc_t __attribute__((ext_vector_type(4)));

// acc += sgn * As[R .. R+15][:] * Bs[:][Cc .. Cc+15] over K = 32 for wave w's subtile (R, Cc) = (16 (w >> 1),
// 16 (w & 1)) (v_mfma_f64_16x16x4f64: A fragment lane l = A[row l & 15][k l >> 4], B fragment = B[k l >> 4]
// [col l & 15], result reg q = D[row (l >> 4) + 4 q][col l & 15]; cdna_hip_programming.md, f64 MFMA layout).
__device__ __forceinline__ gj_acc_t gj_tile_mfma(const double (*As)[kGS], const double (*Bs)[kGS], gj_acc_t acc, double sgn,
                                                 int lane, int w) {
    const int R = (w >> 1) * 16, Cc = (w & 1) * 16, lr = lane & 15, lk = lane >> 4;
#pragma unroll
    for (int s = 0; s < kGB / 4; ++s)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(sgn * As[R + lr][4 * s + lk], Bs[4 * s + lk][Cc + lr], acc, 0, 0, 0);
    return acc;
}

// tile (r0, c0) of X (row stride ld) -> LDS, optionally equilibrated ((x d_r) d_c, the oracle's order)
__device__ __forceinline__ void gj_stage(double (*dst)[kGS], const double* __restrict__ X, int ld, size_t r0, size_t c0,
                                         const double* __restrict__ d) {
    for (int e = threadIdx.x; e < kGB * kGB; e += 256) {
        const int r = e / kGB, c = e % kGB;
        double v = X[(r0 + r) * ld + c0 + c];
        if (d) v = v * d[r0 + r] * d[c0 + c];
        dst[r][c] = v;
    }
}

// In-place scalar Gauss-Jordan inversion of the SPD block in M (LDS) by wave 0 (lane r & 31 = row r), result back into
// M; every thread of the workgroup must call it.  Returns (in wave 0) whether a pivot was not positive.
// GJ_PINV 6 (default since round 5): lane l holds the 4 x 4 sub-block (rows 4 (l & 7) .., columns 4 (l >> 3) ..), the
// pivot column / row entries it needs come by ds_bpermute -- about half the instructions per pivot of variant 4: the
// inversion of E (m = 639) 310 -> 242 us standalone, bitwise equal (tools/bench_dense.hip, profiles/r5_v2/);
// 5: variant 4's layout with the pivot row broadcast by ds_swizzle (294 us);
// GJ_PINV 0: the pivot row is broadcast by readlane (2 x 32 v_readlane per pivot); 1: lane p stores its row in LDS and
// every lane reads it back (one 16-B read per column pair, all lanes the same address); 2: timing only (no inversion,
// results wrong); 3: all 256 threads, four entries each, the matrix ping-ponged through LDS; 4: one wave, 16 entries
// per lane, pivot row / column through LDS without a workgroup barrier.  0, 1, 3 and 4 perform the same arithmetic in
// the same order.  (Round 4: a variant exchanging the pivot row and column by lane permutes instead of LDS was bitwise
// equal and 8-10 % slower at m = 567-747, profiles/r4_v2/gj_pinv4_vs_pinv5.log, and was removed.)
#ifndef GJ_PINV
#define GJ_PINV 6
#endif
// variant 5: lane P of each 32-lane half, broadcast to its half by ds_swizzle (BitMode: and 0, or P, xor 0) -- the LDS
// crossbar without an LDS store, a fence or a read-back
template <int P>
__device__ __forceinline__ double swz_bcast(double v) {
    constexpr int pat = P << 5;
    const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), pat);
    const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), pat);
    return __hiloint2double(hi, lo);
}
// one pivot round of variant 5 (variant 4's arithmetic: the same products and fused multiply-adds in the same order)
template <int P>
__device__ __forceinline__ void gj_p5_round(double (&a)[16], int r, int h, bool& bad) {
    constexpr int hp = P >> 4, jp = P & 15;
    double pr[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) pr[j] = swz_bcast<P>(a[j]);  // row P, this half's columns
    const double mine = a[jp];
    const double other = __shfl_xor(mine, 32, 64);               // row r, column P from the other half
    double piv = readlane_d(mine, P + 32 * hp);
    const double aip = (h == hp) ? mine : other;
    if (!(piv > 0.0)) { bad = true; piv = 1.0; }
    const double inv = 1.0 / piv;
    const int cb = 16 * h;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if (cb + j == P) {
            a[j] = (r == P) ? inv : -aip * inv;
        } else {
            const double rpc = pr[j] * inv;
            a[j] = (r == P) ? rpc : __builtin_fma(-aip, rpc, a[j]);
        }
    }
}
template <int... P>
__device__ __forceinline__ void gj_p5_all(double (&a)[16], int r, int h, bool& bad, std::integer_sequence<int, P...>) {
    (gj_p5_round<P>(a, r, h, bad), ...);
}

// variant 6: lane l holds the 4 x 4 sub-block (rows 4 (l & 7) .., columns 4 (l >> 3) ..); per pivot P the lane fetches
// the 4 pivot-column entries of its rows and the 4 pivot-row entries of its columns by ds_bpermute from the two lanes
// that hold them (16 dword permutes), forms 4 scaled row entries and does 16 fused multiply-adds -- variant 4's values
// for every entry (rpc = row * (1 / piv), fma(-aip, rpc, a), the pivot row / column cases), in half the instructions
__device__ __forceinline__ double bperm_d(int src_lane, double v) {
    const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, __double2hiint(v));
    return __hiloint2double(hi, lo);
}
template <int P>
__device__ __forceinline__ void gj_p6_round(double (&a)[4][4], int rb, int cb, bool& bad) {
    constexpr int PB = P >> 2, PI = P & 3;
    double colv[4], rowv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) colv[i] = bperm_d(PB * 8 + rb, a[i][PI]);  // row 4 rb + i, column P
#pragma unroll
    for (int c = 0; c < 4; ++c) rowv[c] = bperm_d(cb * 8 + PB, a[PI][c]);  // row P, column 4 cb + c
    double piv = readlane_d(a[PI][PI], PB * 8 + PB);
    if (!(piv > 0.0)) { bad = true; piv = 1.0; }
    const double inv = 1.0 / piv;
    double rpc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) rpc[c] = rowv[c] * inv;
    const bool prow = rb == PB, pcol = cb == PB;  // this lane holds part of row P / of column P
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const double up = __builtin_fma(-colv[i], rpc[c], a[i][c]);
            if (c == PI && i == PI) {
                a[i][c] = pcol ? (prow ? inv : -colv[i] * inv) : (prow ? rpc[c] : up);
            } else if (c == PI) {
                a[i][c] = pcol ? -colv[i] * inv : up;
            } else if (i == PI) {
                a[i][c] = prow ? rpc[c] : up;
            } else {
                a[i][c] = up;
            }
        }
}
template <int... P>
__device__ __forceinline__ void gj_p6_all(double (&a)[4][4], int rb, int cb, bool& bad, std::integer_sequence<int, P...>) {
    (gj_p6_round<P>(a, rb, cb, bad), ...);
}

__device__ bool gj_invert_block(double (*M)[kGS]) {
#if GJ_PINV == 2
    __syncthreads();
    return false;
#elif GJ_PINV == 3
    // all 256 threads: thread t owns row t / 8, columns 4 (t % 8) .. +3, in registers; per pivot every thread reads the
    // pivot row's entries of its columns and its row's pivot-column entry from the LDS copy of the previous step and
    // writes its updated entries to the other copy (ping-pong, one barrier per pivot)
    static_assert(kGB == 32 && (kGB & 1) == 0, "256 threads = 32 rows x 8 column quads; an even pivot count ends in M");
    __shared__ double Mb[kGB][kGS];
    __syncthreads();
    const int t = threadIdx.x, r = t >> 3, c0 = (t & 7) * 4;
    double a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = M[r][c0 + j];
    double(*src)[kGS] = M;
    double(*dst)[kGS] = Mb;
    bool bad = false;
    for (int p = 0; p < kGB; ++p) {
        double piv = src[p][p];
        const double aip = src[r][p];
        double pr[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) pr[j] = src[p][c0 + j];
        if (!(piv > 0.0)) { bad = true; piv = 1.0; }
        const double inv = 1.0 / piv;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (c0 + j == p) {
                a[j] = (r == p) ? inv : -aip * inv;
            } else {
                const double rpc = pr[j] * inv;
                a[j] = (r == p) ? rpc : __builtin_fma(-aip, rpc, a[j]);
            }
            dst[r][c0 + j] = a[j];
        }
        __syncthreads();
        double(*tmp)[kGS] = src;
        src = dst;
        dst = tmp;
    }
    return bad;  // (the same pivots in every thread)
#elif GJ_PINV == 4
    // one wave: lane l holds row l & 31, columns 16 (l >> 5) .. +15 in registers.  Per pivot p the two lanes of row p
    // publish it and every lane of the half holding column p publishes its column-p entry through LDS; the wave reads
    // back what it needs.  LDS requests of one wave complete in order, so a wave-level fence replaces the workgroup
    // barrier of variant 3 (the other three waves wait at the closing barrier); the pivot buffers alternate by parity.
    static_assert(kGB == 32, "64 lanes = 32 rows x 2 column halves");
    __shared__ __attribute__((aligned(16))) double prow[2][kGB];
    __shared__ __attribute__((aligned(16))) double pcol[2][kGB];
    __syncthreads();
    bool bad = false;
    if (threadIdx.x < 64) {
        const int l = threadIdx.x, r = l & 31, h = l >> 5, cb = 16 * h;
        double a[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = M[r][cb + j];
#pragma unroll
        for (int p = 0; p < kGB; ++p) {
            const int par = p & 1, hp = p >> 4, jp = p & 15;
            if (r == p) {
#pragma unroll
                for (int j = 0; j < 16; j += 2)
                    *reinterpret_cast<double2*>(&prow[par][cb + j]) = make_double2(a[j], a[j + 1]);
            }
            if (h == hp) pcol[par][r] = a[jp];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double pr[16];
#pragma unroll
            for (int j = 0; j < 16; j += 2) {
                const double2 v = *reinterpret_cast<const double2*>(&prow[par][cb + j]);
                pr[j] = v.x;
                pr[j + 1] = v.y;
            }
            double piv = prow[par][p];
            const double aip = pcol[par][r];
            if (!(piv > 0.0)) { bad = true; piv = 1.0; }
            const double inv = 1.0 / piv;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                if (cb + j == p) {
                    a[j] = (r == p) ? inv : -aip * inv;
                } else {
                    const double rpc = pr[j] * inv;
                    a[j] = (r == p) ? rpc : __builtin_fma(-aip, rpc, a[j]);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) M[r][cb + j] = a[j];
    }
    __syncthreads();
    return bad;
#elif GJ_PINV == 5
    // one wave, variant 4's layout (lane l: row l & 31, columns 16 (l >> 5) .. +15) and arithmetic; per pivot the
    // pivot row goes to each half by ds_swizzle, the pivot by readlane, the other half's pivot-column entry by one
    // permute: no LDS traffic and no fence in the pivot loop
    static_assert(kGB == 32, "64 lanes = 32 rows x 2 column halves");
    __syncthreads();
    bool bad = false;
    if (threadIdx.x < 64) {
        const int l = threadIdx.x, r = l & 31, h = l >> 5, cb = 16 * h;
        double a[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = M[r][cb + j];
        gj_p5_all(a, r, h, bad, std::make_integer_sequence<int, kGB>{});
#pragma unroll
        for (int j = 0; j < 16; ++j) M[r][cb + j] = a[j];
    }
    __syncthreads();
    return bad;
#elif GJ_PINV == 6
    static_assert(kGB == 32, "64 lanes = 8 x 8 sub-blocks of 4 x 4");
    __syncthreads();
    bool bad = false;
    if (threadIdx.x < 64) {
        const int l = threadIdx.x, rb = l & 7, cb = l >> 3;
        double a[4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) a[i][c] = M[4 * rb + i][4 * cb + c];
        gj_p6_all(a, rb, cb, bad, std::make_integer_sequence<int, kGB>{});
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) M[4 * rb + i][4 * cb + c] = a[i][c];
    }
    __syncthreads();
    return bad;
#elif GJ_PINV == 1
    __shared__ __attribute__((aligned(16))) double prow[kGB];
    __syncthreads();
    bool bad = false;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x, r = lane & 31;
        double a[kGB];
#pragma unroll
        for (int c = 0; c < kGB; ++c) a[c] = M[r][c];
#pragma unroll
        for (int p = 0; p < kGB; ++p) {
            if (lane == p) {
#pragma unroll
                for (int c = 0; c < kGB; c += 2) *reinterpret_cast<double2*>(&prow[c]) = make_double2(a[c], a[c + 1]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double pr[kGB];
#pragma unroll
            for (int c = 0; c < kGB; c += 2) {
                const double2 v = *reinterpret_cast<const double2*>(&prow[c]);
                pr[c] = v.x;
                pr[c + 1] = v.y;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double piv = pr[p];
            if (!(piv > 0.0)) { bad = true; piv = 1.0; }
            const double inv = 1.0 / piv;
            const double aip = a[p];
#pragma unroll
            for (int c = 0; c < kGB; ++c) {
                if (c == p) continue;
                const double rpc = pr[c] * inv;
                a[c] = (r == p) ? rpc : __builtin_fma(-aip, rpc, a[c]);
            }
            a[p] = (r == p) ? inv : -aip * inv;
        }
        if (lane < kGB) {
#pragma unroll
            for (int c = 0; c < kGB; ++c) M[lane][c] = a[c];
        }
    }
    __syncthreads();
    return bad;
#else
    __syncthreads();
    bool bad = false;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x, r = lane & 31;
        double a[kGB];
#pragma unroll
        for (int c = 0; c < kGB; ++c) a[c] = M[r][c];
#pragma unroll
        for (int p = 0; p < kGB; ++p) {
            double piv = readlane_d(a[p], p);
            if (!(piv > 0.0)) { bad = true; piv = 1.0; }
            const double inv = 1.0 / piv;
            const double aip = a[p];
#pragma unroll
            for (int c = 0; c < kGB; ++c) {
                if (c == p) continue;
                const double rpc = readlane_d(a[c], p) * inv;
                a[c] = (r == p) ? rpc : __builtin_fma(-aip, rpc, a[c]);
            }
            a[p] = (r == p) ? inv : -aip * inv;
        }
        if (lane < kGB) {
#pragma unroll
            for (int c = 0; c < kGB; ++c) M[lane][c] = a[c];
        }
    }
    __syncthreads();
    return bad;
#endif
}

// P_0^-1 (one workgroup): the equilibrated first pivot block.
__global__ __launch_bounds__(256) void k_gj_pinv0(int ld, const double* __restrict__ X, const double* __restrict__ d,
                                                  double* __restrict__ Pout, int* __restrict__ ok) {
    __shared__ double M[kGB][kGS];
    gj_stage(M, X, ld, 0, 0, d);
    const bool bad = gj_invert_block(M);
    for (int e = threadIdx.x; e < kGB * kGB; e += 256) Pout[e] = M[e / kGB][e % kGB];
    if (threadIdx.x == 0) ok[0] = !bad;
}

__global__ __launch_bounds__(256) void k_gj_step(int k, int nB, int ld, int m, const double* __restrict__ X,
                                                 double* __restrict__ Y, const double* __restrict__ d, int first,
                                                 const double* __restrict__ Pin, double* __restrict__ Pnext,
                                                 double* __restrict__ Eout, int* __restrict__ ok) {
    __shared__ double Ps[kGB][kGS];   // P^-1
    __shared__ double Bk[kGB][kGS];   // X_kj, then P^-1 X_kj
    __shared__ double Ci[kGB][kGS];   // X_ik
    const int i = blockIdx.x / nB, j = blockIdx.x % nB, t = threadIdx.x, lane = t & 63, w = t >> 6;
    const size_t k0 = (size_t)k * kGB, i0 = (size_t)i * kGB, j0 = (size_t)j * kGB;
    const int R = (w >> 1) * 16, Cc = (w & 1) * 16;
    const double* ds = first ? d : nullptr;   // equilibrate while reading E (step 0)
    // Every load of the step is issued before the first one is used (P^-1, X_kj, X_ik: 4 entries each per thread at
    // (row (t >> 5) + 8 q, column t & 31); X_ij: this lane's 4 accumulator entries), so the step waits for one global
    // latency instead of one per staged entry (a load-then-store loop retires its loads one at a time).
    const bool upd = i != k && j != k;
    const int sr = t >> 5, sc = t & 31;
    double pv[4], bv[4], cv[4], xv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        pv[q] = Pin[(sr + 8 * q) * kGB + sc];
        bv[q] = j != k ? X[(k0 + sr + 8 * q) * ld + j0 + sc] : 0.0;
        cv[q] = i != k ? X[(i0 + sr + 8 * q) * ld + k0 + sc] : 0.0;
        xv[q] = upd ? X[(i0 + R + (lane >> 4) + 4 * q) * ld + j0 + Cc + (lane & 15)] : 0.0;
    }
    if (ds) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const size_t rk = k0 + sr + 8 * q, ri = i0 + sr + 8 * q;
            bv[q] = bv[q] * ds[rk] * ds[j0 + sc];
            cv[q] = cv[q] * ds[ri] * ds[k0 + sc];
            xv[q] = xv[q] * ds[i0 + R + (lane >> 4) + 4 * q] * ds[j0 + Cc + (lane & 15)];
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        Ps[sr + 8 * q][sc] = pv[q];
        Bk[sr + 8 * q][sc] = bv[q];
        Ci[sr + 8 * q][sc] = cv[q];
    }
    __syncthreads();
    gj_acc_t acc = {0.0, 0.0, 0.0, 0.0};
    if (i == k && j == k) {
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = Ps[R + (lane >> 4) + 4 * q][Cc + (lane & 15)];
    } else if (i == k) {
        acc = gj_tile_mfma(Ps, Bk, acc, 1.0, lane, w);                // Y_kj = P^-1 X_kj
    } else if (j == k) {
        acc = gj_tile_mfma(Ci, Ps, acc, -1.0, lane, w);               // Y_ik = -X_ik P^-1
    } else {
        acc = gj_tile_mfma(Ps, Bk, acc, 1.0, lane, w);                // P^-1 X_kj ...
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) Bk[R + (lane >> 4) + 4 * q][Cc + (lane & 15)] = acc[q];
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = xv[q];
        acc = gj_tile_mfma(Ci, Bk, acc, -1.0, lane, w);               // ... Y_ij = X_ij - X_ik (P^-1 X_kj)
    }
    const bool last = k == nB - 1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const size_t r = i0 + R + (lane >> 4) + 4 * q, cc = j0 + Cc + (lane & 15);
        Y[r * ld + cc] = acc[q];
        if (last && r < (size_t)m && cc < (size_t)m) Eout[r * m + cc] = acc[q] * d[r] * d[cc];
    }
    if (i == k + 1 && j == k + 1) {
        // look-ahead: this tile is the next step's pivot block; invert it now
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) Ps[R + (lane >> 4) + 4 * q][Cc + (lane & 15)] = acc[q];
        const bool bad = gj_invert_block(Ps);
        for (int e = t; e < kGB * kGB; e += 256) Pnext[e] = Ps[e / kGB][e % kGB];
        if (t == 0 && bad) ok[0] = 0;
    }
}

inline int gj_steps(int m) { return (m + kGB - 1) / kGB; }

// Launch unit u of the inversion of E (padded [ld][ld], equilibration d [ld], pad entries 1), u = 0 .. gj_steps(m):
// 0 = P_0^-1, u >= 1 = step u - 1.  E and W are the ping-pong buffers, P [2][kGB][kGB] the pivot inverses; the last
// step writes the compact E^-1 into Eout [m][m]; ok[0] = 0 when E is not positive definite.  Units run in order on
// one stream.
inline void launch_gj_unit(int u, int m, double* E, double* W, double* P, const double* d, double* Eout, int* ok,
                           hipStream_t st) {
    const int nB = gj_steps(m), ld = nB * kGB;
    if (u == 0) {
        k_gj_pinv0<<<1, 256, 0, st>>>(ld, E, d, P, ok);
        return;
    }
    const int k = u - 1;
    const double* X = (k & 1) ? W : E;
    double* Y = (k & 1) ? E : W;
    k_gj_step<<<nB * nB, 256, 0, st>>>(k, nB, ld, m, X, Y, d, k == 0, P + (size_t)(k & 1) * kGB * kGB,
                                       P + (size_t)((k + 1) & 1) * kGB * kGB, Eout, ok);
}

// ---- per iteration: pipelined PCG (oracle/ba_oracle.c ora_pcg, two-level path) -----------------------------------
// Ghysels & Vanroose's pipelined recurrence: per iteration i, with r, u = M~^-1 r, w = S~ u and the row partials of
// gamma = (r, u), delta = (w, u), rho = ||L r||^2 and of the restriction Z~^T w already in memory:
//   k_tl_pc    (one workgroup per cluster): the scalars (every workgroup sums the partials in the same fixed order;
//              convergence / breakdown test; alpha_i, beta_i recorded by workgroup 0), the full restriction R, the
//              cluster's coarse rows y_c = (E^-1 R)_c and m = w + Z~ y_c for its rows;
//   k_tl_pspmv (one workgroup per camera row): n = S~ m, then z = n + beta z, q = m + beta q, s = w + beta s,
//              p = u + beta p, x += alpha p, r -= alpha s, u -= alpha q, w -= alpha z for the row, and the row's
//              partials for iteration i + 1.
// Two launches per iteration instead of three.  Setup (it = -1): k_tl_basis forms Z~^T r0 per row, k_tl_pc (u0 = r0 + Z~ y),
// k_tl_pspmv (w0 = S~ u0 and the partials of iteration 0).  Buffers: q = cg.r[1], z = cg.w[1], m = cg.s[1].

// Copy n doubles global -> LDS: U loads per thread in flight before their LDS stores (a plain strided loop waits for
// every load before its store).
template <int NT, int U>
__device__ __forceinline__ void stage_lds(double* dst, const double* __restrict__ src, int n) {
    const int t = threadIdx.x;
    for (int b = 0; b < n; b += NT * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = b + t + u * NT;
            if (q < n) v[u] = src[q];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = b + t + u * NT;
            if (q < n) dst[q] = v[u];
        }
    }
}

#ifndef PC_NT
#define PC_NT 512
#endif
constexpr int kPcThreads = PC_NT, kPcWaves = PC_NT / 64;  // k_tl_pc workgroup (256 / 512 / 1024: 11.0 / 8.8 / 9.1 us)

// prows: restriction row partials staged in LDS per pass (rows in cluster order; the host sizes it to the LDS budget)
template <int D>
__global__ __launch_bounds__(kPcThreads) void k_tl_pc(int it, int C, int maxit, double tol2_rel, int prows, CgBufs cg,
                                                      TlBufs tl, const double* __restrict__ Einv) {
    constexpr int MC = D + 1;
    extern __shared__ double lds[];
    double* LR = lds;                         // [prows * MC] restriction row partials of a pass
    double* EL = LR + (size_t)prows * MC;     // [MC][m] this cluster's rows of E^-1
    double* Rs = EL + (size_t)MC * tl.m;      // [m] full restriction
    __shared__ double y[MC];
    __shared__ double red[3][kPcWaves];
    __shared__ double sc[3];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c = blockIdx.x, m = tl.m;
    const bool setup = it < 0;
    // Every global load that does not depend on another is issued before the first wait (s_waitcnt retires loads in
    // issue order): the status word (a launch past convergence returns before any store), the coarse flag, the
    // cluster's member range, its E^-1 rows and the first pass of the restriction partials (registers, stored to LDS
    // below; E^-1 is loaded even when the coarse correction is off -- the buffer always exists), history, member
    // ranges and the scalar partials.  Only the cluster's rows of the source vector and of Z~ wait for the range.
    const int st0 = cg.status[0];
    const int okv = tl.ok[0];
    const int e0 = tl.cl_ptr[c], e1 = tl.cl_ptr[c + 1];
    constexpr int UE = (MC * kCoarseMax + kPcThreads - 1) / kPcThreads, UR = 16384 / kPcThreads, UR2 = UR / 2;
    const int np = (C + prows - 1) / prows;
    const int nlr0 = min(C, prows) * MC;
    // the scalar partials and the history first: the recurrence scalars below wait only for them (loads retire in
    // issue order), so that reduction overlaps the E^-1 / restriction batch still in flight
    // the first GK partials per thread are held in registers and summed at the scalar phase (a summing loop here
    // would wait for them before the batch below is issued); rows past GK * kPcThreads are summed there too
    // with the atomic cluster sums (tl.Racc) k_tl_pspmv left one record per cluster: nc scalar partials and the full
    // restriction (m values) instead of C and C * MC row partials
    const bool usecl = tl.Racc != nullptr && !setup;
    const double* gsrc = usecl ? tl.Gacc + (size_t)(it & 1) * 3 * tl.nc : tl.gd;
    const int gn = usecl ? tl.nc : C;
    const double* rsrc = usecl ? tl.Racc + (size_t)(it & 1) * tl.m : nullptr;
    constexpr int GK = 2;
    double ga0[GK], ga1[GK], ga2[GK];
#pragma unroll
    for (int r = 0; r < GK; ++r) {
        const int k = min(t + r * kPcThreads, gn - 1);
        ga0[r] = gsrc[k]; ga1[r] = gsrc[gn + k]; ga2[r] = gsrc[2 * gn + k];
    }
    const int ih = max(it - 1, 0);
    const double h_alpha = cg.hist[2 * ih], h_gam = cg.hist[2 * ih + 1], h_bb = cg.hist[2 * (maxit + 1)];
    double ev[UE];
    double2 lrv[UR2];  // restriction partials in 16-B pairs (rowR is 16-B aligned and padded by 2)
    constexpr int URC = (kCoarseMax + kPcThreads - 1) / kPcThreads;
    double rcv[URC];   // the cluster restriction (usecl)
    // branch-free: indices past the end are clamped to the last valid element (a load under a divergent branch is
    // waited for at the branch's join, which would serialize the batch)
#pragma unroll
    for (int u = 0; u < UE; ++u) ev[u] = Einv[(size_t)c * MC * m + min(t + u * kPcThreads, MC * m - 1)];
    if (usecl) {
#pragma unroll
        for (int u = 0; u < URC; ++u) rcv[u] = rsrc[min(t + u * kPcThreads, m - 1)];
    } else {
#pragma unroll
        for (int u = 0; u < UR2; ++u)
            lrv[u] = reinterpret_cast<const double2*>(tl.rowR)[min(t + u * kPcThreads, (nlr0 - 1) / 2)];
    }
    const int tc = min(t / MC, tl.nc - 1);
    const int rb0 = tl.cl_ptr[tc], rb1 = tl.cl_ptr[tc + 1];
    const int ne = e1 - e0;
    if (tl.Racc != nullptr && blockIdx.x == 0) {  // clear the buffer this iteration's k_tl_pspmv adds into
        // (setup: buffers 0 and 1 -- k_tl_cgp's first iteration adds into buffer 1 with no barrier before it)
        for (int bq = (it + 1) & 1; bq <= (setup ? 1 : ((it + 1) & 1)); ++bq) {
            double* R = tl.Racc + (size_t)bq * m;
            double* G = tl.Gacc + (size_t)bq * 3 * tl.nc;
            for (int q = t; q < m; q += kPcThreads) R[q] = 0.0;
            for (int q = t; q < 3 * tl.nc; q += kPcThreads) G[q] = 0.0;
        }
    }
    if (st0 != 0 || ne < 0) return;  // (ne < 0 never holds: it makes the branch wait for the range loads as well)
    const bool use = okv != 0;
    if (setup && c == 0 && t == 0) {
        cg.status[2] = okv;  // reported as insfm_ba_stats.coarse_used
        if (cg.prog) __hip_atomic_store(cg.prog + 3, okv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const int tp = min(t, ne * D - 1);
    // the cluster's rows are contiguous in the cluster-ordered copies
    const size_t ci = (size_t)e0 * D + tp;
    const double vp = tl.vc[ci];
    double Zq[MC];
#pragma unroll
    for (int k = 0; k < MC; ++k) Zq[k] = tl.Ztc[ci * MC + k];
    const size_t pidx = (size_t)tl.cl_cams[e0 + tp / D] * D + tp % D;  // only the output store waits for it
    if (!setup) {
        const int i = it;
        double g0 = 0.0, g1 = 0.0, g2 = 0.0;
#pragma unroll
        for (int r = 0; r < GK; ++r)
            if (t + r * kPcThreads < gn) { g0 += ga0[r]; g1 += ga1[r]; g2 += ga2[r]; }
        for (int k = t + GK * kPcThreads; k < gn; k += kPcThreads) { g0 += gsrc[k]; g1 += gsrc[gn + k]; g2 += gsrc[2 * gn + k]; }
        g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
        if (lane == 0) { red[0][wv] = g0; red[1][wv] = g1; red[2][wv] = g2; }
        __syncthreads();
        if (t == 0) {
            double gam = 0.0, del = 0.0, rho = 0.0;
            for (int w = 0; w < kPcWaves; ++w) { gam += red[0][w]; del += red[1][w]; rho += red[2][w]; }
            const double bb = (i == 0) ? rho : h_bb;
            double flag = 0.0;
            const bool lead = blockIdx.x == 0;
            int done = 0;
            if (rho <= tol2_rel * bb || i >= maxit) {
                flag = 1.0;
                done = 1;
            } else {
                const double bev = (i == 0) ? 0.0 : gam / h_gam;
                const double den = (i == 0) ? del : del - bev * gam / h_alpha;
                if (!(den > 0.0)) {
                    flag = 2.0;
                    done = 2;
                } else if (lead) {
                    cg.hist[2 * i] = gam / den;
                    cg.hist[2 * i + 1] = gam;
                    if (i == 0) cg.hist[2 * (maxit + 1)] = bb;
                }
            }
            if (lead) {
                if (done) { cg.status[1] = i; __threadfence(); cg.status[0] = done; }
                // progress for the host, which enqueues more iterations without a stream sync (system-scope stores)
                if (cg.prog) {
                    if (done) {
                        __hip_atomic_store(cg.prog + 2, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __hip_atomic_store(cg.prog + 1, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                    } else {
                        __hip_atomic_store(cg.prog + 0, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                }
            }
            sc[0] = flag;
        }
        __syncthreads();
        if (sc[0] != 0.0) return;
    }
    if (use) {
#pragma unroll
        for (int u = 0; u < UE; ++u) {
            const int q = t + u * kPcThreads;
            if (q < MC * m) EL[q] = ev[u];
        }
        if (usecl) {
#pragma unroll
            for (int u = 0; u < URC; ++u) {
                const int q = t + u * kPcThreads;
                if (q < m) Rs[q] = rcv[u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < UR2; ++u) {
                const int q = 2 * (t + u * kPcThreads);
                if (q < nlr0) LR[q] = lrv[u].x;
                if (q + 1 < nlr0) LR[q + 1] = lrv[u].y;
            }
            if (nlr0 > UR * kPcThreads) stage_lds<kPcThreads, 16>(LR + UR * kPcThreads, tl.rowR + UR * kPcThreads,
                                                                    nlr0 - UR * kPcThreads);
        }
    }
    if (use && !usecl) {
        // full restriction: entry (c', k) sums the row partials of cluster c' in ascending camera order (from LDS)
        for (int pass = 0; pass < np; ++pass) {
            const int r0 = pass * prows, r1 = min(C, r0 + prows);
            if (pass > 0) {
                __syncthreads();
                stage_lds<kPcThreads, 32>(LR, tl.rowR + (size_t)r0 * MC, (r1 - r0) * MC);
            }
            __syncthreads();
            for (int e = t; e < m; e += kPcThreads) {
                const int k = e % MC;
                const int b0 = max(e == t ? rb0 : tl.cl_ptr[e / MC], r0), b1 = min(e == t ? rb1 : tl.cl_ptr[e / MC + 1], r1);
                double v = pass == 0 ? 0.0 : Rs[e];
#pragma unroll 8
                for (int mi = b0; mi < b1; ++mi) v += LR[(mi - r0) * MC + k];
                Rs[e] = v;
            }
        }
    }
    if (use) {
        __syncthreads();
        constexpr int KPW = (MC + kPcWaves - 1) / kPcWaves, LPL = (kCoarseMax + 63) / 64;
        double sy[KPW];
#pragma unroll
        for (int kk = 0; kk < KPW; ++kk) sy[kk] = 0.0;
#pragma unroll
        for (int q = 0; q < LPL; ++q) {
            const int l = lane + 64 * q;
            if (l < m) {
                const double rl = Rs[l];
#pragma unroll
                for (int kk = 0; kk < KPW; ++kk) {
                    const int k = wv + kk * kPcWaves;
                    if (k < MC) sy[kk] += EL[(size_t)k * m + l] * rl;
                }
            }
        }
#pragma unroll
        for (int kk = 0; kk < KPW; ++kk) {
            const int k = wv + kk * kPcWaves;
            const double v = wave_sum(sy[kk]);
            if (lane == 0 && k < MC) y[k] = v;
        }
        __syncthreads();
    }
    double* dst = setup ? tl.u : cg.s[1];
    for (int e = t; e < ne * D; e += kPcThreads) {
        const bool first = e == t;
        const size_t idx = first ? pidx : (size_t)tl.cl_cams[e0 + e / D] * D + e % D;
        double v = first ? vp : tl.vc[(size_t)e0 * D + e];
        if (use) {
            const double* Z = tl.Ztc + ((size_t)e0 * D + e) * MC;
            double sz = 0.0;
#pragma unroll
            for (int k = 0; k < MC; ++k) sz += (first ? Zq[k] : Z[k]) * y[k];
            v += sz;
        }
        dst[idx] = v;
    }
}

// k_tl_pc for iterations it >= 0 when the row partials arrive as per-cluster sums (tl.Racc: atomic cluster sums):
// every wave reduces the nc scalar partials itself (no workgroup barrier before the recurrence scalars), each wave
// keeps its coarse rows of E^-1 in registers, loaded column-per-lane (no LDS staging), and multiplies them with the
// restriction loaded the same way; one barrier publishes the MC entries of y before m = w + Z~ y.  Same arithmetic
// as k_tl_pc's cluster path up to the order of the scalar sums (here: a butterfly over the clusters in every wave).
template <int D>
__global__ __launch_bounds__(kPcThreads) void k_tl_pc_cl(int it, int C, int maxit, double tol2_rel, CgBufs cg,
                                                         TlBufs tl, const double* __restrict__ Einv) {
    constexpr int MC = D + 1, NW = kPcWaves, KPW = (MC + NW - 1) / NW, LPL = (kCoarseMax + 63) / 64;
    __shared__ double y[MC];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c = blockIdx.x, m = tl.m, nc = tl.nc;
    const int st0 = cg.status[0];
    const int okv = tl.ok[0];
    const int e0 = tl.cl_ptr[c], e1 = tl.cl_ptr[c + 1];
    const double* G = tl.Gacc + (size_t)(it & 1) * 3 * nc;
    const double* Rv = tl.Racc + (size_t)(it & 1) * m;
    // every load that does not depend on another is issued before the first wait: the scalar partials, history,
    // E^-1 rows (row k = wv + NW kk, column l = lane + 64 q), the restriction, the cluster's source rows
    double ga[3] = {0.0, 0.0, 0.0};
    constexpr int LNC = (kCoarseMax / 3 + 63) / 64;  // clusters per lane (nc <= m / 3)
    double gl[3][LNC];
#pragma unroll
    for (int q = 0; q < LNC; ++q) {
        const int l = min(lane + 64 * q, nc - 1);
        gl[0][q] = G[l]; gl[1][q] = G[nc + l]; gl[2][q] = G[2 * nc + l];
    }
    const int ih = max(it - 1, 0);
    const double h_alpha = cg.hist[2 * ih], h_gam = cg.hist[2 * ih + 1], h_bb = cg.hist[2 * (maxit + 1)];
    double ev[KPW][LPL], rv[LPL];
#pragma unroll
    for (int kk = 0; kk < KPW; ++kk) {
        const int k = min(wv + NW * kk, MC - 1);
#pragma unroll
        for (int q = 0; q < LPL; ++q) ev[kk][q] = Einv[((size_t)c * MC + k) * m + min(lane + 64 * q, m - 1)];
    }
#pragma unroll
    for (int q = 0; q < LPL; ++q) rv[q] = Rv[min(lane + 64 * q, m - 1)];
    const int ne = e1 - e0;
    if (blockIdx.x == 0) {  // clear the buffer this iteration's k_tl_pspmv adds into
        double* Rn = tl.Racc + (size_t)((it + 1) & 1) * m;
        double* Gn = tl.Gacc + (size_t)((it + 1) & 1) * 3 * nc;
        for (int q = t; q < m; q += kPcThreads) Rn[q] = 0.0;
        for (int q = t; q < 3 * nc; q += kPcThreads) Gn[q] = 0.0;
    }
    if (st0 != 0 || ne < 0) return;
    const bool use = okv != 0;
    // recurrence scalars, in every wave (the same butterfly, so the same doubles everywhere)
#pragma unroll
    for (int q = 0; q < LNC; ++q)
        if (lane + 64 * q < nc) { ga[0] += gl[0][q]; ga[1] += gl[1][q]; ga[2] += gl[2][q]; }
    const double gam = wave_sum(ga[0]), del = wave_sum(ga[1]), rho = wave_sum(ga[2]);
    const int i = it;
    const double bb = (i == 0) ? rho : h_bb;
    int done = 0;
    double alpha = 0.0;
    if (rho <= tol2_rel * bb || i >= maxit) {
        done = 1;
    } else {
        const double bev = (i == 0) ? 0.0 : gam / h_gam;
        const double den = (i == 0) ? del : del - bev * gam / h_alpha;
        if (!(den > 0.0)) done = 2;
        else alpha = gam / den;
    }
    if (blockIdx.x == 0 && t == 0) {
        if (done) {
            cg.status[1] = i;
            __threadfence();
            cg.status[0] = done;
        } else {
            cg.hist[2 * i] = alpha;
            cg.hist[2 * i + 1] = gam;
            if (i == 0) cg.hist[2 * (maxit + 1)] = bb;
        }
        if (cg.prog) {
            if (done) {
                __hip_atomic_store(cg.prog + 2, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(cg.prog + 1, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                __hip_atomic_store(cg.prog + 0, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (done) return;
    if (use) {
#pragma unroll
        for (int kk = 0; kk < KPW; ++kk) {
            double sy = 0.0;
#pragma unroll
            for (int q = 0; q < LPL; ++q)
                if (lane + 64 * q < m) sy += ev[kk][q] * rv[q];
            const double v = wave_sum(sy);
            const int k = wv + NW * kk;
            if (lane == 0 && k < MC) y[k] = v;
        }
    }
    __syncthreads();
    for (int e = t; e < ne * D; e += kPcThreads) {
        const size_t idx = (size_t)tl.cl_cams[e0 + e / D] * D + e % D;
        double v = tl.vc[(size_t)e0 * D + e];
        if (use) {
            const double* Z = tl.Ztc + ((size_t)e0 * D + e) * MC;
            double sz = 0.0;
#pragma unroll
            for (int k = 0; k < MC; ++k) sz += Z[k] * y[k];
            v += sz;
        }
        cg.s[1][idx] = v;
    }
}

// One camera row per 512-thread workgroup: the product with S~ (row-contiguous Sn stream), the row's vector updates
// and its partials for the next iteration (setup: w0 = S~ u0 and the partials of iteration 0).
// NT threads per workgroup: at 256, the 1000 rows of config 3 (4 waves each) are all resident at once at <= 128 VGPRs.
#ifndef PSPMV_NT
#define PSPMV_NT 256
#endif
#ifndef PSPMV_RG
#define PSPMV_RG 8
#endif
constexpr int kPspmvThreads = PSPMV_NT;
template <int D, int NT = kPspmvThreads>
__global__ __launch_bounds__(NT) void k_tl_pspmv(int it, int C, int stride, const int* __restrict__ nbr_ptr,
                                                 const int* __restrict__ nbr_j, const double* __restrict__ Sn,
                                                 const double* __restrict__ Lf, CgBufs cg, TlBufs tl, XPart xp) {
    using G = CgGeom<D>;
    constexpr int NW = NT / 64;
    constexpr int DP = G::DP, HP = G::HP, PPB = G::PPB, BPW = G::BPW, PPL = G::PPL, BPR = BPW * NW, MC = D + 1;
    __shared__ double red[NW][BPW][PPB];
    __shared__ double sv[2][D];  // r and w of the row after the update
    if (cg.status[0] != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    // partitioned across ranks (ba_xpart.h): this rank's rows are the cluster-ordered positions from xp.q0
    const int row = xp.win ? tl.cl_cams[xp.q0 + blockIdx.x] : blockIdx.x;
    const bool setup = it < 0;
    const int bw = (PPB <= 64) ? lane / PPB : 0;
    const int pc0 = (PPB <= 64) ? lane - bw * PPB : lane;
    const bool lane_on = (PPB <= 64) ? (bw < BPW) : true;
    const int slot = wv * BPW + bw;
    // equal-length (padded) rows: the range follows from the row index, no load in front of the stream
    const int n0 = stride > 0 ? row * stride : nbr_ptr[row], n1 = stride > 0 ? n0 + stride : nbr_ptr[row + 1];
    const double* v = setup ? tl.u : cg.s[1];
    // The row's own vector entries and wave 0's tail operands (row a of L for lanes a < D, column k of Z~ for lanes
    // D + k), independent of the product, are loaded by wave 0 under a wave-uniform branch with clamped lane
    // indices: no lane divergence around the loads, so they stay in flight during wave 0's stream instead of being
    // waited for before it.
    const int la = min(lane, D - 1);
    const size_t own = (size_t)row * D + la;
    double vo = 0.0, u_ = 0.0, w_ = 0.0, r_ = 0.0, z_ = 0.0, q_ = 0.0, s_ = 0.0, p_ = 0.0, x_ = 0.0;
    double al = 0.0, hg1 = 1.0, hg0 = 1.0;
    double tailop[D];
#pragma unroll
    for (int k = 0; k < D; ++k) tailop[k] = 0.0;
    if (__builtin_amdgcn_readfirstlane(wv) == 0) {
        const bool isL = lane < D;
        const double* tb = isL ? Lf + (size_t)row * D * D + lane * D
                               : tl.Zt + (size_t)row * D * MC + min(max(lane - D, 0), MC - 1);
        const int ts = isL ? 1 : MC;
#pragma unroll
        for (int k = 0; k < D; ++k) tailop[k] = tb[k * ts];  // (L's upper part is masked at the use)
        vo = v[own]; u_ = tl.u[own]; r_ = cg.r[0][own];
        w_ = cg.w[0][own]; z_ = cg.w[1][own]; q_ = cg.r[1][own]; s_ = cg.s[0][own]; p_ = cg.p[own]; x_ = cg.x[own];
        const int ia = max(it, 0), ib = max(it - 1, 0);
        al = cg.hist[2 * ia]; hg1 = cg.hist[2 * ia + 1]; hg0 = cg.hist[2 * ib + 1];
    }
    double acc[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) acc[q] = 0.0;
    // The lane's blocks are rounds k = 0, 1, ... of the row (nn = n0 + slot + k * BPR), taken RG rounds at a time:
    // the RG neighbour indices are loaded together, then every Sn piece and vector entry of the group, with the indices
    // of rounds past the row's end clamped to its last block (valid addresses, no branch around the loads, so the
    // whole group is in flight at once) and their products dropped by a select.  Sums stay in round order.
    constexpr int RG = PSPMV_RG;
    for (int base = n0 + slot; lane_on && base < n1; base += RG * BPR) {
        int jr[RG];
#pragma unroll
        for (int r = 0; r < RG; ++r) jr[r] = nbr_j[min(base + r * BPR, n1 - 1)];
        double2 sg[RG][PPL], ug[RG][PPL];
#pragma unroll
        for (int r = 0; r < RG; ++r) {
            const size_t nn = (size_t)min(base + r * BPR, n1 - 1);
#pragma unroll
            for (int q = 0; q < PPL; ++q) {
                const int pc = min(pc0 + 64 * q, PPB - 1);
                const int bcol = 2 * (pc % HP);
                sg[r][q] = *reinterpret_cast<const double2*>(Sn + (nn * D * DP + 2 * (size_t)pc));
                const size_t jx = (size_t)jr[r] * D + bcol;
                if constexpr ((D & 1) == 0) {
                    ug[r][q] = *reinterpret_cast<const double2*>(v + jx);
                } else {
                    ug[r][q].x = v[jx];
                    ug[r][q].y = v[jx + (bcol + 1 < D ? 1 : 0)];
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RG; ++r)
#pragma unroll
            for (int q = 0; q < PPL; ++q) {
                const int pc = pc0 + 64 * q;
                const double u1 = ((D & 1) == 0 || 2 * (pc % HP) + 1 < D) ? ug[r][q].y : 0.0;
                const double t2 = sg[r][q].x * ug[r][q].x + sg[r][q].y * u1;
                if (base + r * BPR < n1 && pc < PPB) acc[q] += t2;
            }
    }
    if (lane_on) {
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const int pc = pc0 + 64 * q;
            if (pc < PPB) red[wv][bw][pc] = acc[q];
        }
    }
    __syncthreads();
    if (wv != 0) return;
    double g0 = 0.0, g1 = 0.0;
    if (lane < D) {
        const int a = lane;
        double tot = 0.0;
        for (int w = 0; w < NW; ++w)
#pragma unroll
            for (int bb = 0; bb < BPW; ++bb)
#pragma unroll
                for (int k = 0; k < HP; ++k) tot += red[w][bb][a * HP + k];
        const double prod = vo + tot;  // diagonal block of S~ is I
        if (setup) {
            w_ = prod;
            cg.w[0][own] = w_;
            cg.w[1][own] = 0.0;  // z
            cg.r[1][own] = 0.0;  // q
        } else {
            const double be = (it == 0) ? 0.0 : hg1 / hg0;
            const double zn = prod + be * z_;
            const double qn = vo + be * q_;
            const double sn = w_ + be * s_;
            const double pn = u_ + be * p_;
            x_ += al * pn;
            r_ -= al * sn;
            u_ -= al * qn;
            w_ -= al * zn;
            cg.w[1][own] = zn; cg.r[1][own] = qn; cg.s[0][own] = sn; cg.p[own] = pn; cg.x[own] = x_;
            cg.r[0][own] = r_; tl.u[own] = u_; cg.w[0][own] = w_;
        }
        sv[0][a] = r_;
        sv[1][a] = w_;
        xstore(xp, tl.vc + (size_t)tl.cpos[row] * D + a, xp.off_vc + (size_t)tl.cpos[row] * D + a, w_);
        g0 = r_ * u_;
        g1 = w_ * u_;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double g2 = 0.0, rr = 0.0;
    const int cp = tl.cpos[row];
    if (lane < D) {  // (L r)_a for the true-residual norm
        double lr = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (k <= lane) lr += tailop[k] * sv[0][k];
        g2 = lr * lr;
    } else if (lane < D + MC) {  // restriction of w: sum_a Z~[a][k] w_a
#pragma unroll
        for (int a = 0; a < D; ++a) rr += tailop[a] * sv[1][a];
        if (tl.Racc == nullptr) {
            if (xp.win) xstore(xp, nullptr, xp.off_rowR + (size_t)cp * MC + (lane - D), rr);
            else st_sc1(tl.rowR + (size_t)cp * MC + (lane - D), rr);
        }
    }
    g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
    if (tl.Racc != nullptr) {  // cluster sums by atomics (order varies run to run; single GPU, non-deterministic)
        const int c = tl.clab[row], bsel = (it + 1) & 1;
        if (lane >= D && lane < D + MC)
            unsafeAtomicAdd(tl.Racc + (size_t)bsel * tl.m + (size_t)c * MC + (lane - D), rr);
        if (lane == 0) {
            double* G = tl.Gacc + (size_t)bsel * 3 * tl.nc;
            unsafeAtomicAdd(G + c, g0);
            unsafeAtomicAdd(G + tl.nc + c, g1);
            unsafeAtomicAdd(G + 2 * tl.nc + c, g2);
        }
        return;
    }
    if (lane == 0) {
        if (xp.win) {
            xstore(xp, nullptr, xp.off_gd + cp, g0);
            xstore(xp, nullptr, xp.off_gd + C + cp, g1);
            xstore(xp, nullptr, xp.off_gd + 2 * C + cp, g2);
        } else {
            st_sc1(tl.gd + cp, g0); st_sc1(tl.gd + C + cp, g1); st_sc1(tl.gd + 2 * C + cp, g2);
        }
    }
}

}  // namespace insfm
