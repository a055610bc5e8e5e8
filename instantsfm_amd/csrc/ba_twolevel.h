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
//   k_tl_chol    : one workgroup, blocked right-looking Cholesky of E (diag block in registers, panel in LDS)
//   k_tl_dinv    : inverses of the factor's diagonal blocks
//   k_tl_trinv   : L^-1 by column blocks (block forward substitution, diag-block inverses as GEMMs)
//   k_tl_gram    : E^-1 = L^-T L^-1 (dense tiles)
// Per CG iteration (preconditioned Chronopoulos-Gear, same stopping rule as block-Jacobi):
//   k_tl_update  : per cluster: recurrence scalars from the partials, p/s/x/r update, R_c = sum Z~_i^T r_i, ||L r||^2
//   k_tl_coarse  : per cluster: y = E^-1 R (its MC rows), u_i = r_i + Z~_i y_c
//   k_tl_spmv    : w = S~ u (row-contiguous Sn stream), partial dots r.u and w.u per row
#pragma once
#include "ba_common.h"
#include "ba_device.h"

namespace insfm {

constexpr int kCoarseMax = 288;  // nclust * (D + 1) cap: L^-1's column block + an L strip (2 x 288 x 33 f64) fit LDS
constexpr int kNB = 32;          // block size of the dense coarse factorization
constexpr int kPS = kNB + 1;     // padded LDS row stride (odd: conflict-free column walks)

struct TlBufs {
    double* u;           // [C*D]  preconditioned residual
    double* Zt;          // [C][D][MC]
    double* Rc;          // [m]   restriction Z~^T r per cluster (k_tl_update)
    double* gd;          // [2C]  r_i.u_i | w_i.u_i  (row partials of k_tl_spmv)
    double* rho[2];      // [nc]  ||L r||^2 per cluster of r_k, stored at parity k & 1
    double* Oseg;        // [nseg][MC][MC] per (row, neighbour cluster) sums of Z~_i^T S~_ij Z~_j
    double* E;           // [m][m] coarse matrix, Cholesky factor (lower) in place
    double* Dinv;        // [nB][kNB][kNB] inverses of the diagonal blocks of the factor
    double* Linv;        // [m][m] (lower)
    double* Einv;        // [m][m]
    int* ok;             // coarse correction usable (E positive definite)
    const int* cl_ptr;   // [nc+1]
    const int* cl_cams;  // cluster members, ascending camera id
    const int* alone;    // [C] camera is alone in its cluster -> basis [I_D | 0]
    const int* sperm;    // [n_nbr] neighbour slots of each row ordered by (cluster of the neighbour, slot)
    const int4* seg;     // [nseg] (cluster, sorted begin, sorted end, own-cluster flag) per (row, neighbour cluster)
    const int* rseg_ptr; // [C+1] segments of each row
    const int* ered_ptr; // [nc*nc+1]
    const int* ered_seg; // segment ids of each cluster pair, rows ascending
    int nc, m, maxmem;
};

// ---- setup ---------------------------------------------------------------------------------------------------
// One thread per (camera i, coarse column k): column k of G_i at the linearization point and Z~_i[:,k] = L_i^T G_i[:,k].
template <int M>
__global__ __launch_bounds__(kThreads) void k_tl_basis(int C, const double* __restrict__ cams, const double* __restrict__ Lf,
                                                       TlBufs tl) {
    constexpr int D = kD<M>, MC = D + 1, ST = kStride<M>;
    const int g = blockIdx.x * kThreads + threadIdx.x;
    if (g >= C * MC) return;
    const int i = g / MC, k = g % MC;
    double col[D];
#pragma unroll
    for (int a = 0; a < D; ++a) col[a] = 0.0;
    if (tl.alone[i]) {
        if (k < D) col[k] = 1.0;
    } else if constexpr (M == kGP) {  // global positioning: translation (I) and scaling about the origin (c_i)
        const double* cp = cams + (size_t)i * ST;
        if (k < 3) col[k] = 1.0;
        else { col[0] = cp[0]; col[1] = cp[1]; col[2] = cp[2]; }
    } else {
        const double* cp = cams + (size_t)i * ST;
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
    const double* L = Lf + (size_t)i * D * D;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double s = 0.0;
#pragma unroll
        for (int l = a; l < D; ++l) s += L[l * D + a] * col[l];
        tl.Zt[((size_t)i * D + a) * MC + k] = s;
    }
}

template <int D>
struct ErowGeom {
    static constexpr int MC = D + 1;
    static constexpr int DP = D + (D & 1);
    static constexpr int CH = D <= 9 ? 32 : 16;   // neighbour blocks staged per round
};

// One workgroup per camera row i: per neighbour cluster c, Oseg = [c == c_i] Z~_i^T Z~_i + sum over the row's
// neighbours j in c (slot order) of Z~_i^T S~_ij Z~_j.  Neighbour blocks and Z~_j are staged in rounds of CH through
// LDS; T = S~_ij Z~_j is formed once per block; each (segment, k, l) output is owned by one thread (fixed order).
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_erow(int C, const int* __restrict__ nbr_ptr, const int* __restrict__ nbr_j,
                                                      const double* __restrict__ Sn, TlBufs tl) {
    using G = ErowGeom<D>;
    constexpr int MC = G::MC, DP = G::DP, CH = G::CH, MM = MC * MC;
    extern __shared__ double lds[];
    double* Zi = lds;                         // [D][MC]
    double* Sb = Zi + D * MC;                 // [CH][D][DP]
    double* Zj = Sb + CH * D * DP;            // [CH][D][MC]
    double* T = Zj + CH * D * MC;             // [CH][D][MC]
    double* acc = T + CH * D * MC;            // [nseg_row][MC][MC]
    const int i = blockIdx.x, t = threadIdx.x;
    const int n0 = nbr_ptr[i], n1 = nbr_ptr[i + 1];
    const int s0 = tl.rseg_ptr[i], ns = tl.rseg_ptr[i + 1] - s0;
    const int nout = ns * MM;
    for (int e = t; e < D * MC; e += kThreads) Zi[e] = tl.Zt[(size_t)i * D * MC + e];
    __syncthreads();
    for (int o = t; o < nout; o += kThreads) {
        const int4 sg = tl.seg[s0 + o / MM];
        const int k = (o % MM) / MC, l = o % MC;
        double v = 0.0;
        if (sg.w) {
#pragma unroll
            for (int a = 0; a < D; ++a) v += Zi[a * MC + k] * Zi[a * MC + l];
        }
        acc[o] = v;
    }
    for (int q0 = n0; q0 < n1; q0 += CH) {
        const int nq = min(CH, n1 - q0);
        __syncthreads();
        for (int e = t; e < nq * D * DP; e += kThreads) {
            const int q = e / (D * DP), r = e % (D * DP);
            Sb[e] = Sn[(size_t)tl.sperm[q0 + q] * D * DP + r];
        }
        for (int e = t; e < nq * D * MC; e += kThreads) {
            const int q = e / (D * MC), r = e % (D * MC);
            Zj[e] = tl.Zt[(size_t)nbr_j[tl.sperm[q0 + q]] * D * MC + r];
        }
        __syncthreads();
        for (int e = t; e < nq * D * MC; e += kThreads) {
            const int q = e / (D * MC), r = e % (D * MC), a = r / MC, l = r % MC;
            const double* B = Sb + q * D * DP + a * DP;
            const double* Z = Zj + q * D * MC + l;
            double v = 0.0;
#pragma unroll
            for (int b = 0; b < D; ++b) v += B[b] * Z[b * MC];
            T[e] = v;
        }
        __syncthreads();
        for (int o = t; o < nout; o += kThreads) {
            const int4 sg = tl.seg[s0 + o / MM];
            const int k = (o % MM) / MC, l = o % MC;
            const int qa = max(sg.y, q0 - n0), qb = min(sg.z, q0 - n0 + nq);
            double v = acc[o];
            for (int q = qa; q < qb; ++q) {
                const double* Tq = T + (q - (q0 - n0)) * D * MC + l;
#pragma unroll
                for (int a = 0; a < D; ++a) v += Zi[a * MC + k] * Tq[a * MC];
            }
            acc[o] = v;
        }
    }
    __syncthreads();
    for (int o = t; o < nout; o += kThreads) tl.Oseg[(size_t)s0 * MM + o] = acc[o];
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
    tl.E[g] = acc;
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

constexpr int kCB = 16;          // block size of the Cholesky factorization
constexpr int kCPS = kCB + 1;    // LDS row stride of the Cholesky panel

// One 1024-thread workgroup: blocked right-looking Cholesky of E (m <= kCoarseMax) in place (lower triangle).
// Per block column of kCB:
//   diagonal block : wave 0, lane r holds row r in registers; each pivot column goes through LDS once and is read
//                    back as one batch of independent loads;
//   panel          : one thread per row below, column-oriented forward substitution against the block (LDS);
//   trailing SYRK  : 4x4 register tiles with rows/columns strided by ceil(n/4) (the 64 lanes of a wave read 64
//                    consecutive panel rows: conflict-free LDS; update consecutive columns: coalesced RMW); only the
//                    entries of the lower triangle are computed.
// ok[0] = 0 when a pivot is not positive (the solve then runs without the coarse correction).  `prof` (debug only)
// receives clock64() stamps per block column and phase.
__global__ __launch_bounds__(1024) void k_tl_chol(int m, double* __restrict__ A, int* __restrict__ ok,
                                                  long long* __restrict__ prof = nullptr) {
    extern __shared__ double lds[];
    double* Pn = lds;  // [m][kCPS]; rows [kb, kb+nb) double as the diagonal block of the current step
    __shared__ double colb[2][64];
    __shared__ int bad;
    const int t = threadIdx.x;
    if (t == 0) bad = 0;
    if (prof && t == 0) prof[63] = clock64();
    __syncthreads();
    int step = 0;
    for (int kb = 0; kb < m; kb += kCB, ++step) {
        const int nb = min(kCB, m - kb);
        double* Dg = Pn + (size_t)kb * kCPS;
        if (t < 64) {
            const int r = t;
            double a[kCB];
#pragma unroll
            for (int c = 0; c < kCB; ++c) a[c] = (r < nb && c <= r && c < nb) ? A[(size_t)(kb + r) * m + kb + c] : 0.0;
            int isbad = 0;
#pragma unroll
            for (int j = 0; j < kCB; ++j) {
                if (j < nb) {
                    colb[j & 1][r] = a[j];
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    double d = colb[j & 1][j];
                    if (!(d > 0.0)) { isbad = 1; d = 1.0; }
                    const double inv = 1.0 / sqrt(d);
                    // column j of L: lanes >= j (lane j: sqrt(d))
                    double lc[kCB];
#pragma unroll
                    for (int c = 0; c < kCB; ++c) lc[c] = colb[j & 1][c] * inv;
                    const double l = (r > j) ? a[j] * inv : (r == j ? d * inv : 0.0);
                    a[j] = (r >= j) ? l : 0.0;
#pragma unroll
                    for (int c = j + 1; c < kCB; ++c) a[c] -= l * lc[c];
                }
            }
            if (r == 0 && isbad) bad = 1;
            if (r < nb) {
#pragma unroll
                for (int c = 0; c < kCB; ++c) {
                    if (c < nb) {
                        const double v = (c <= r) ? a[c] : 0.0;
                        Dg[r * kCPS + c] = v;
                        if (c <= r) A[(size_t)(kb + r) * m + kb + c] = v;
                    }
                }
                Dg[r * kCPS + kCB] = 1.0 / a[r];   // reciprocal pivot in the pad column
            }
        }
        __syncthreads();
        if (prof && t == 0 && step < 20) prof[3 * step] = clock64();
        // panel: row i solves x L_kk^T = a, column by column
        const int i = kb + nb + t;
        if (i < m) {
            double x[kCB];
#pragma unroll
            for (int c = 0; c < kCB; ++c) x[c] = (c < nb) ? A[(size_t)i * m + kb + c] : 0.0;
#pragma unroll
            for (int q = 0; q < kCB; ++q) {
                if (q < nb) {
                    double lq[kCB];
#pragma unroll
                    for (int c = q + 1; c < kCB; ++c) lq[c] = Dg[c * kCPS + q];
                    x[q] *= Dg[q * kCPS + kCB];
#pragma unroll
                    for (int c = q + 1; c < kCB; ++c) x[c] -= x[q] * lq[c];
                }
            }
#pragma unroll
            for (int c = 0; c < kCB; ++c)
                if (c < nb) {
                    A[(size_t)i * m + kb + c] = x[c];
                    Pn[(size_t)i * kCPS + c] = x[c];
                }
        }
        __syncthreads();
        if (prof && t == 0 && step < 20) prof[3 * step + 1] = clock64();
        // trailing update: strided 4x4 tiles, entries (u, v) with v <= u (the others are above the diagonal)
        const int base = kb + nb, n = m - base;
        if (n > 0) {
            const int nt = (n + 3) / 4;
            for (int tt = t; tt < nt * nt; tt += 1024) {
                const int I = tt / nt, J = tt - (tt / nt) * nt;
                int rr[4], cc[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) { rr[u] = base + I + nt * u; cc[u] = base + J + nt * u; }
                double acc[10];
#pragma unroll
                for (int e = 0; e < 10; ++e) acc[e] = 0.0;
                for (int k = 0; k < nb; ++k) {
                    double av[4], bq[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) av[u] = (rr[u] < m) ? Pn[(size_t)rr[u] * kCPS + k] : 0.0;
#pragma unroll
                    for (int v = 0; v < 4; ++v) bq[v] = (cc[v] < m) ? Pn[(size_t)cc[v] * kCPS + k] : 0.0;
                    int e = 0;
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v <= u; ++v) acc[e++] += av[u] * bq[v];
                }
                int e = 0;
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v <= u; ++v, ++e)
                        if (rr[u] < m && cc[v] <= rr[u]) A[(size_t)rr[u] * m + cc[v]] -= acc[e];
            }
        }
        __threadfence_block();
        __syncthreads();
        if (prof && t == 0 && step < 20) prof[3 * step + 2] = clock64();
    }
    if (t == 0) ok[0] = !bad;
}

// One wave per diagonal block R of the factor: Dinv_R = L_RR^-1, lane c owns column c (forward substitution).
__global__ __launch_bounds__(64) void k_tl_dinv(int m, const double* __restrict__ Lc, double* __restrict__ Dinv,
                                                const int* __restrict__ ok) {
    __shared__ double Lb[kNB][kPS];
    if (!ok[0]) return;
    const int R = blockIdx.x, c = threadIdx.x;
    const int r0 = R * kNB, nb = min(kNB, m - r0);
    for (int e = c; e < kNB * kNB; e += 64) {
        const int rr = e / kNB, q = e % kNB;
        Lb[rr][q] = (rr < nb && q <= rr) ? Lc[(size_t)(r0 + rr) * m + r0 + q] : (rr == q ? 1.0 : 0.0);
    }
    __syncthreads();
    if (c >= kNB) return;
    double x[kNB];
#pragma unroll
    for (int rr = 0; rr < kNB; ++rr) {
        double s = (rr == c) ? 1.0 : 0.0;
#pragma unroll
        for (int q = 0; q < rr; ++q) s -= Lb[rr][q] * x[q];
        x[rr] = (rr >= c) ? s / Lb[rr][rr] : 0.0;
    }
    double* Dv = Dinv + (size_t)R * kNB * kNB;
#pragma unroll
    for (int rr = 0; rr < kNB; ++rr) Dv[rr * kNB + c] = x[rr];
}

// Workgroup J computes columns [J*kNB, J*kNB + kNB) of L^-1 by block forward substitution:
//   X_R = Dinv_R (I_RJ - sum_{J<=K<R} L_RK X_K), the column block kept in LDS.  The strip L_R[J*kNB, R*kNB) is staged
//   through LDS with coalesced loads; 256 threads, thread (q, c) owns rows q, q+8, q+16, q+24 of column c, so every LDS
//   load of X feeds four FMAs (the strip loads are broadcasts).  Rows past the end of the matrix are never touched.
__global__ __launch_bounds__(256) void k_tl_trinv(int m, const double* __restrict__ Lc, const double* __restrict__ Dinv,
                                                  double* __restrict__ Linv, const int* __restrict__ ok) {
    extern __shared__ double lds[];
    double* X = lds;                          // [m][kPS]
    double* St = lds + (size_t)m * kPS;       // [kNB][m + 1] strip of L (row stride m + 1)
    __shared__ double Tb[kNB][kPS];
    if (!ok[0]) return;
    const int J = blockIdx.x;
    const int t = threadIdx.x, q0 = t / kNB, c = t % kNB;   // q0 in [0, 8)
    const int j0 = J * kNB;
    const int nB = (m + kNB - 1) / kNB;
    const int ls = m + 1;
    for (int R = J; R < nB; ++R) {
        const int r0 = R * kNB, nr = min(kNB, m - r0);
        const int w = r0 - j0;                // strip width
        for (int e = t; e < nr * w; e += 256) {
            const int q = e / w, k = e - q * w;
            St[q * ls + k] = Lc[(size_t)(r0 + q) * m + j0 + k];
        }
        __syncthreads();
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int rr = q0 + 8 * u;
            double a = (R == J && rr == c) ? 1.0 : 0.0;
            if (rr < nr) {
                const double* Sr = St + rr * ls;
                for (int k = 0; k < w; ++k) a -= Sr[k] * X[(size_t)(j0 + k) * kPS + c];
            }
            v[u] = a;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) Tb[q0 + 8 * u][c] = v[u];
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int rr = q0 + 8 * u;
            if (rr < nr) {
                const double* Dv = Dinv + (size_t)R * kNB * kNB + rr * kNB;
                double x = 0.0;
                for (int q = 0; q <= rr; ++q) x += Dv[q] * Tb[q][c];
                X[(size_t)(r0 + rr) * kPS + c] = x;
                if (j0 + c < m) Linv[(size_t)(r0 + rr) * m + j0 + c] = x;
            }
        }
        __syncthreads();
    }
}

// E^-1 = L^-T L^-1 : one 32x32 tile per 256-thread workgroup (4 outputs per thread), rows of L^-1 staged through LDS.
__global__ __launch_bounds__(256) void k_tl_gram(int m, const double* __restrict__ Linv, double* __restrict__ Einv,
                                                 const int* __restrict__ ok) {
    __shared__ double A[kNB][kPS];
    __shared__ double B[kNB][kPS];
    if (!ok[0]) return;
    const int nB = (m + kNB - 1) / kNB;
    const int tk = blockIdx.x / nB, tlb = blockIdx.x % nB;
    const int t = threadIdx.x, k0q = t / kNB, ll = t % kNB;
    const int k0 = tk * kNB, l0 = tlb * kNB;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int r0 = max(k0, l0); r0 < m; r0 += kNB) {
        for (int e = t; e < kNB * kNB; e += 256) {
            const int rr = e / kNB, cc = e % kNB, r = r0 + rr;
            A[rr][cc] = (r < m && k0 + cc < m) ? Linv[(size_t)r * m + k0 + cc] : 0.0;
            B[rr][cc] = (r < m && l0 + cc < m) ? Linv[(size_t)r * m + l0 + cc] : 0.0;
        }
        __syncthreads();
#pragma unroll 8
        for (int q = 0; q < kNB; ++q) {
            const double bq = B[q][ll];
#pragma unroll
            for (int u = 0; u < 4; ++u) acc[u] += A[q][k0q + 8 * u] * bq;
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int kk = k0q + 8 * u;
        if (k0 + kk < m && l0 + ll < m) Einv[(size_t)(k0 + kk) * m + l0 + ll] = acc[u];
    }
}

// ---- per iteration ------------------------------------------------------------------------------------------
// One workgroup per cluster c.  it >= 1: recurrence step i = it - 1 -- every workgroup sums the row partials of
// k_tl_spmv (it-1) and the cluster partials of rho_i in the same fixed order, tests rho_i <= tol^2 ||b||^2 and forms
// alpha_i, beta_i (workgroup 0 records them); then for the cluster's rows p = u + beta p, s = w + beta s,
// x += alpha p, r -= alpha s.  Every it: R_c = sum_i Z~_i^T r_i and rho_c = sum_i ||L_i r_i||^2 over its rows.
// The row data are loaded before the scalar reduction (they do not depend on alpha / beta).
template <int D>
__global__ __launch_bounds__(kCgThreads) void k_tl_update(int it, int C, int maxit, double tol2_rel,
                                                          const double* __restrict__ Lf, CgBufs cg, TlBufs tl) {
    constexpr int MC = D + 1, RPW = kCgThreads / D;
    extern __shared__ double lds[];
    double* rl = lds;                 // [RPW][D]  r of the pass's rows
    double* lq = rl + RPW * D;        // [RPW][D]  (L r)_a^2
    double* Rm = lq + RPW * D;        // [maxmem][MC]
    double* sq = Rm + tl.maxmem * MC; // [maxmem]
    __shared__ double red[3][kCgWaves];
    __shared__ double sc[3];
    if (cg.status[0] != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c = blockIdx.x;
    const int e0 = tl.cl_ptr[c], ne = tl.cl_ptr[c + 1] - e0;
    const int rloc = t / D, a = t % D;
    if (it == 0 && c == 0 && t == 0) cg.status[2] = tl.ok[0];   // reported as insfm_ba_stats.coarse_used
    // first pass row data (prefetch)
    double pu = 0.0, pp = 0.0, pw = 0.0, ps = 0.0, px = 0.0, pr = 0.0;
    size_t idx0 = 0;
    const bool on0 = rloc < RPW && rloc < ne;
    if (on0) {
        idx0 = (size_t)tl.cl_cams[e0 + rloc] * D + a;
        pr = cg.r[0][idx0];
        if (it > 0) { pu = tl.u[idx0]; pp = cg.p[idx0]; pw = cg.w[0][idx0]; ps = cg.s[0][idx0]; px = cg.x[idx0]; }
    }
    // the first pass's L row and Z~ column depend only on the cluster's rows: in flight before the barriers too
    double Lp[D], Zp[D];
    if (on0) {
        const double* L = Lf + idx0 * D;  // row a of L_row (idx0 = row * D + a)
#pragma unroll
        for (int k = 0; k < D; ++k) Lp[k] = (k <= a) ? L[k] : 0.0;
    }
    const bool zon = t < RPW * MC && t / MC < ne;
    if (zon) {
        const double* Z = tl.Zt + (size_t)tl.cl_cams[e0 + t / MC] * D * MC + t % MC;
#pragma unroll
        for (int aa = 0; aa < D; ++aa) Zp[aa] = Z[aa * MC];
    }
    double al = 0.0, be = 0.0;
    if (it > 0) {
        const int i = it - 1;
        const double* G0 = tl.gd;
        const double* G1 = tl.gd + C;
        const double* RH = tl.rho[i & 1];
        double g0 = 0.0, g1 = 0.0, g2 = 0.0;
        for (int k = t; k < C; k += kCgThreads) { g0 += G0[k]; g1 += G1[k]; }
        for (int k = t; k < tl.nc; k += kCgThreads) g2 += RH[k];
        g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
        if (lane == 0) { red[0][wv] = g0; red[1][wv] = g1; red[2][wv] = g2; }
        __syncthreads();
        if (t == 0) {
            double gam = 0.0, del = 0.0, rho = 0.0;
            for (int w = 0; w < kCgWaves; ++w) { gam += red[0][w]; del += red[1][w]; rho += red[2][w]; }
            const double h_alpha = (i >= 1) ? cg.hist[2 * (i - 1)] : 1.0;
            const double h_gam = (i >= 1) ? cg.hist[2 * (i - 1) + 1] : 1.0;
            const double bb = (i == 0) ? rho : cg.hist[2 * (maxit + 1)];
            double flag = 0.0, alv = 0.0, bev = 0.0;
            const bool lead = blockIdx.x == 0;
            if (rho <= tol2_rel * bb || i >= maxit) {
                flag = 1.0;
                if (lead) { cg.status[1] = i; __threadfence(); cg.status[0] = 1; }
            } else {
                bev = (i == 0) ? 0.0 : gam / h_gam;
                const double den = (i == 0) ? del : del - bev * gam / h_alpha;
                if (!(den > 0.0)) {
                    flag = 2.0;
                    if (lead) { cg.status[1] = i; __threadfence(); cg.status[0] = 2; }
                } else {
                    alv = gam / den;
                    if (lead) {
                        cg.hist[2 * i] = alv;
                        cg.hist[2 * i + 1] = gam;
                        if (i == 0) cg.hist[2 * (maxit + 1)] = bb;
                    }
                }
            }
            sc[0] = alv; sc[1] = bev; sc[2] = flag;
        }
        __syncthreads();
        if (sc[2] != 0.0) return;
        al = sc[0];
        be = sc[1];
    }
    for (int pass = 0; pass * RPW < ne; ++pass) {
        const int mi = pass * RPW + rloc;
        const bool on = rloc < RPW && mi < ne;
        const int row = on ? tl.cl_cams[e0 + mi] : 0;
        if (on) {
            const size_t idx = (size_t)row * D + a;
            double u_, p_, w_, s_, x_, r_;
            if (pass == 0) { u_ = pu; p_ = pp; w_ = pw; s_ = ps; x_ = px; r_ = pr; }
            else {
                r_ = cg.r[0][idx];
                if (it > 0) { u_ = tl.u[idx]; p_ = cg.p[idx]; w_ = cg.w[0][idx]; s_ = cg.s[0][idx]; x_ = cg.x[idx]; }
                else { u_ = p_ = w_ = s_ = x_ = 0.0; }
            }
            if (it > 0) {
                const double pn = u_ + be * p_;
                const double sn = w_ + be * s_;
                cg.p[idx] = pn;
                cg.s[0][idx] = sn;
                cg.x[idx] = x_ + al * pn;
                r_ = r_ - al * sn;
                cg.r[0][idx] = r_;
            }
            rl[rloc * D + a] = r_;
        }
        __syncthreads();
        if (on) {
            double lr = 0.0;
            if (pass == 0) {
#pragma unroll
                for (int k = 0; k < D; ++k)
                    if (k <= a) lr += Lp[k] * rl[rloc * D + k];
            } else {
                const double* L = Lf + (size_t)row * D * D + a * D;
#pragma unroll
                for (int k = 0; k < D; ++k)
                    if (k <= a) lr += L[k] * rl[rloc * D + k];
            }
            lq[rloc * D + a] = lr * lr;
        }
        __syncthreads();
        for (int e = t; e < RPW * MC; e += kCgThreads) {
            const int rr = e / MC, k = e % MC, mj = pass * RPW + rr;
            if (mj < ne) {
                double v = 0.0;
                if (pass == 0 && e == t) {
#pragma unroll
                    for (int aa = 0; aa < D; ++aa) v += Zp[aa] * rl[rr * D + aa];
                } else {
                    const double* Z = tl.Zt + (size_t)tl.cl_cams[e0 + mj] * D * MC + k;
#pragma unroll
                    for (int aa = 0; aa < D; ++aa) v += Z[aa * MC] * rl[rr * D + aa];
                }
                Rm[mj * MC + k] = v;
                if (k == 0) {
                    double s2 = 0.0;
#pragma unroll
                    for (int aa = 0; aa < D; ++aa) s2 += lq[rr * D + aa];
                    sq[mj] = s2;
                }
            }
        }
        __syncthreads();
    }
    if (t < MC) {
        double v = 0.0;
        for (int mi = 0; mi < ne; ++mi) v += Rm[mi * MC + t];
        tl.Rc[c * MC + t] = v;
    } else if (t == MC) {
        double v = 0.0;
        for (int mi = 0; mi < ne; ++mi) v += sq[mi];
        tl.rho[it & 1][c] = v;
    }
}

// One workgroup per cluster c: y_c = (E^-1 R) rows of c, u_i = r_i + Z~_i y_c for its rows (u = r without a usable
// coarse matrix).
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_coarse(CgBufs cg, TlBufs tl, const double* __restrict__ Einv) {
    constexpr int MC = D + 1;
    __shared__ double y[MC];
    if (cg.status[0] != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c = blockIdx.x, m = tl.m;
    const bool use = tl.ok[0] != 0;
    const int e0 = tl.cl_ptr[c], ne = tl.cl_ptr[c + 1] - e0;
    // this thread's first row entry (r and its Z~ row) is independent of y: loaded together with E^-1 and R
    const bool pon = t < ne * D;
    size_t pidx = 0;
    double rp = 0.0, Zq[MC];
    if (pon) {
        pidx = (size_t)tl.cl_cams[e0 + t / D] * D + t % D;
        rp = cg.r[0][pidx];
        if (use) {
#pragma unroll
            for (int k = 0; k < MC; ++k) Zq[k] = tl.Zt[pidx * MC + k];
        }
    }
    if (use) {
        // a wave's rows of E^-1 are read together (every load of the wave in flight at once), each row's dot in the
        // same lane order as a row-at-a-time loop
        constexpr int KPW = (MC + kWaves - 1) / kWaves, LPL = (kCoarseMax + 63) / 64;
        double s[KPW];
#pragma unroll
        for (int kk = 0; kk < KPW; ++kk) s[kk] = 0.0;
#pragma unroll
        for (int q = 0; q < LPL; ++q) {
            const int l = lane + 64 * q;
            if (l < m) {
                const double rl = tl.Rc[l];
#pragma unroll
                for (int kk = 0; kk < KPW; ++kk) {
                    const int k = wv + kk * kWaves;
                    if (k < MC) s[kk] += Einv[(size_t)(c * MC + k) * m + l] * rl;
                }
            }
        }
#pragma unroll
        for (int kk = 0; kk < KPW; ++kk) {
            const int k = wv + kk * kWaves;
            const double v = wave_sum(s[kk]);
            if (lane == 0 && k < MC) y[k] = v;
        }
        __syncthreads();
    }
    for (int e = t; e < ne * D; e += kThreads) {
        const bool first = e == t;
        const size_t idx = first ? pidx : (size_t)tl.cl_cams[e0 + e / D] * D + e % D;
        double v = first ? rp : cg.r[0][idx];
        if (use) {
            const double* Z = tl.Zt + idx * MC;
#pragma unroll
            for (int k = 0; k < MC; ++k) v += (first ? Zq[k] : Z[k]) * y[k];
        }
        tl.u[idx] = v;
    }
}

// w = S~ u for one camera row per 512-thread workgroup (Sn streamed as in k_cg_iter), row partials r.u and w.u.
template <int D>
__global__ __launch_bounds__(kCgThreads) void k_tl_spmv(int C, const int* __restrict__ nbr_ptr, const int* __restrict__ nbr_j,
                                                        const double* __restrict__ Sn, CgBufs cg, TlBufs tl) {
    using G = CgGeom<D>;
    constexpr int DP = G::DP, HP = G::HP, PPB = G::PPB, BPW = G::BPW, PPL = G::PPL, BPR = G::BPR;
    __shared__ double red[kCgWaves][BPW][PPB];
    if (cg.status[0] != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int row = blockIdx.x;
    const int bw = (PPB <= 64) ? lane / PPB : 0;
    const int pc0 = (PPB <= 64) ? lane - bw * PPB : lane;
    const bool lane_on = (PPB <= 64) ? (bw < BPW) : true;
    const int slot = wv * BPW + bw;
    const int n0 = nbr_ptr[row], n1 = nbr_ptr[row + 1];
    const double* u = tl.u;
    double acc[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) acc[q] = 0.0;
    for (int nn = n0 + slot; lane_on && nn < n1; nn += BPR) {
        const int j = nbr_j[nn];
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const int pc = pc0 + 64 * q;
            if (pc >= PPB) continue;
            const int bcol = 2 * (pc % HP);
            const double2 sv = *reinterpret_cast<const double2*>(Sn + ((size_t)nn * D * DP + 2 * (size_t)pc));
            const size_t jx = (size_t)j * D + bcol;
            double u0, u1;
            if constexpr ((D & 1) == 0) {
                const double2 uv = *reinterpret_cast<const double2*>(u + jx);
                u0 = uv.x; u1 = uv.y;
            } else {
                u0 = u[jx];
                u1 = (bcol + 1 < D) ? u[jx + 1] : 0.0;
            }
            acc[q] += sv.x * u0 + sv.y * u1;
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
    if (wv == 0) {
        double g0 = 0.0, g1 = 0.0;
        if (lane < D) {
            const int a = lane;
            double tot = 0.0;
            for (int w = 0; w < kCgWaves; ++w)
#pragma unroll
                for (int bb = 0; bb < BPW; ++bb)
#pragma unroll
                    for (int k = 0; k < HP; ++k) tot += red[w][bb][a * HP + k];
            const size_t own = (size_t)row * D + a;
            const double uo = u[own];
            const double wn = uo + tot;
            cg.w[0][own] = wn;
            g0 = cg.r[0][own] * uo;
            g1 = wn * uo;
        }
        g0 = wave_sum(g0); g1 = wave_sum(g1);
        if (lane == 0) { tl.gd[row] = g0; tl.gd[C + row] = g1; }
    }
}

}  // namespace insfm
