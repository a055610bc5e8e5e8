// Two-level preconditioner for the reduced camera system (included by ba_kernels.hip; needs CgBufs, wave_sum,
// kThreads, kD/kStride, CgGeom).
//
// In the scaled space of the block-Jacobi CG (S~ = L^-1 S L^-T, diag blocks I) the preconditioner is
//     M~^-1 = I + Z~ E^-1 Z~^T,   Z~_i = L_i^T G_i,   E = Z~^T S~ Z~            (oracle/ba_oracle.c: ora_coarse_setup)
// where G_i (D x MC, MC = D + 1) spans camera i's response to an infinitesimal similarity of the world (3 translation,
// 3 rotation, 1 scale) plus one unit column per intrinsic, and the columns of a camera cluster share coarse unknowns.
// These are the smooth, low-energy modes that block-Jacobi cannot reduce (a cluster of cameras moving rigidly together
// barely changes the reprojection error), so the coarse correction removes the slow tail of the CG.
//
// Setup per trial (after k_cg_factor / k_cg_scale):
//   k_tl_basis   : Z~ per (camera, coarse column), restriction of r0, rho0 = ||b_i||^2
//   k_tl_opart   : O_ij = Z~_i^T S~_ij Z~_j per neighbour slot (and Z~_i^T Z~_i per camera), written out
//   k_tl_ereduce : E[(c',k),(c,l)] = fixed-order sum of the O blocks of cluster pair (c', c)
//   k_tl_chol    : one workgroup, blocked right-looking Cholesky of E with the panel in LDS; diag-block inverses
//   k_tl_trinv   : L^-1 by column blocks (block forward substitution, diag-block inverses as GEMMs)
//   k_tl_gram    : E^-1 = L^-T L^-1 (dense tiles)
// Per CG iteration (preconditioned Chronopoulos-Gear, same stopping rule as block-Jacobi):
//   k_tl_update  : recurrence scalars from the row partials, p/s/x/r update, restriction R_i = Z~_i^T r_i, ||L r||^2
//   k_tl_coarse  : per cluster: R_c = sum of its rows' R_i, y = E^-1 R (its MC rows), u_i = r_i + Z~_i y_c
//   k_tl_spmv    : w = S~ u (row-contiguous Sn stream), partial dots r.u and w.u per row
#pragma once

constexpr int kCoarseMax = 576;  // nclust * (D + 1) cap: the Cholesky panel (576 x 33 f64 = 152 KB) fits one WG's LDS
constexpr int kNB = 32;          // block size of the dense coarse factorization
constexpr int kPS = kNB + 1;     // padded LDS row stride (odd: conflict-free column walks)

struct TlBufs {
    double* u;           // [C*D]  preconditioned residual
    double* Zt;          // [C][D][MC]
    double* Rp;          // [C][MC] restriction of r per camera row
    double* gd;          // [2C]: r_i.u_i | w_i.u_i  (row partials of k_tl_spmv)
    double* rho[2];      // [C]  ||L_i r_i||^2 of r_k, stored at parity k & 1
    double* Opart;       // [n_nbr][MC][MC]
    double* Odiag;       // [C][MC][MC]
    double* E;           // [m][m] coarse matrix, Cholesky factor (lower) in place
    double* Dinv;        // [nB][kNB][kNB] inverses of the diagonal blocks of the factor
    double* Linv;        // [m][m] (lower)
    double* Einv;        // [m][m]
    int* ok;             // coarse correction usable (E positive definite)
    const int* clab;     // [C]
    const int* cl_ptr;   // [nc+1]
    const int* cl_cams;  // cluster members, ascending camera id
    const int* alone;    // [C] camera is alone in its cluster -> basis [I_D | 0]
    const int* nbr_row;  // [n_nbr] row of each neighbour slot
    const int* ered_ptr; // [nc*nc+1]
    const int* ered_src; // >= 0: neighbour slot (Opart); < 0: -(i+1) diagonal term of camera i (Odiag)
    int nc, m;
};

// ---- setup ---------------------------------------------------------------------------------------------------
// One thread per (camera i, coarse column k): column k of G_i at the linearization point, Z~_i[:,k] = L_i^T G_i[:,k],
// the restriction of r0 and (k == 0) rho0_i = ||b_i||^2 (= ||L_i r0_i||^2).
template <int M>
__global__ __launch_bounds__(kThreads) void k_tl_basis(int C, const double* __restrict__ cams, const double* __restrict__ Lf,
                                                       const double* __restrict__ b, const double* __restrict__ r0,
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
    double rp = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double s = 0.0;
#pragma unroll
        for (int l = a; l < D; ++l) s += L[l * D + a] * col[l];
        tl.Zt[((size_t)i * D + a) * MC + k] = s;
        rp += s * r0[(size_t)i * D + a];
    }
    tl.Rp[(size_t)i * MC + k] = rp;
    if (k == 0) {
        double bb = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) bb += b[(size_t)i * D + a] * b[(size_t)i * D + a];
        tl.rho[0][i] = bb;
    }
}

// One thread per (neighbour slot nn, column l): column l of Z~_i^T S~_ij Z~_j; threads past the slots do the
// diagonal terms Z~_i^T Z~_i (S~_ii = I) per (camera, column).
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_opart(int C, int64_t n_nbr, const int* __restrict__ nbr_j,
                                                       const double* __restrict__ Sn, TlBufs tl) {
    constexpr int MC = D + 1, DP = D + (D & 1);
    const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    const int64_t nslot = n_nbr * MC;
    if (g < nslot) {
        const int64_t nn = g / MC;
        const int l = (int)(g % MC);
        const int i = tl.nbr_row[nn], j = nbr_j[nn];
        const double* B = Sn + (size_t)nn * D * DP;
        const double* Zj = tl.Zt + (size_t)j * D * MC;
        const double* Zi = tl.Zt + (size_t)i * D * MC;
        double zc[D], tcol[D];
#pragma unroll
        for (int bb = 0; bb < D; ++bb) zc[bb] = Zj[bb * MC + l];
#pragma unroll
        for (int a = 0; a < D; ++a) {
            double s = 0.0;
#pragma unroll
            for (int bb = 0; bb < D; ++bb) s += B[a * DP + bb] * zc[bb];
            tcol[a] = s;
        }
        double* O = tl.Opart + (size_t)nn * MC * MC;
#pragma unroll
        for (int k = 0; k < MC; ++k) {
            double s = 0.0;
#pragma unroll
            for (int a = 0; a < D; ++a) s += Zi[a * MC + k] * tcol[a];
            O[k * MC + l] = s;
        }
        return;
    }
    const int64_t h = g - nslot;
    if (h >= (int64_t)C * MC) return;
    const int i = (int)(h / MC), l = (int)(h % MC);
    const double* Zi = tl.Zt + (size_t)i * D * MC;
    double zc[D];
#pragma unroll
    for (int a = 0; a < D; ++a) zc[a] = Zi[a * MC + l];
    double* O = tl.Odiag + (size_t)i * MC * MC;
#pragma unroll
    for (int k = 0; k < MC; ++k) {
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) s += Zi[a * MC + k] * zc[a];
        O[k * MC + l] = s;
    }
}

// One thread per entry of E: fixed-order sum over the cluster pair's source list; an exactly-zero diagonal entry
// (the unused column of a single-camera cluster) becomes 1.
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_ereduce(TlBufs tl) {
    constexpr int MC = D + 1;
    const int m = tl.m, nc = tl.nc;
    const int64_t g = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (g >= (int64_t)m * m) return;
    const int r = (int)(g / m), q = (int)(g % m);
    const int cr = r / MC, k = r % MC, cq = q / MC, l = q % MC;
    const int s0 = tl.ered_ptr[cr * nc + cq], s1 = tl.ered_ptr[cr * nc + cq + 1];
    double acc = 0.0;
    for (int e = s0; e < s1; ++e) {
        const int src = tl.ered_src[e];
        const double* O = src >= 0 ? tl.Opart + (size_t)src * MC * MC : tl.Odiag + (size_t)(-src - 1) * MC * MC;
        acc += O[k * MC + l];
    }
    if (r == q && acc == 0.0) acc = 1.0;
    tl.E[g] = acc;
}

// One 1024-thread workgroup: blocked right-looking Cholesky of E (m <= kCoarseMax) in place (lower triangle).
// Per block column: wave 0 factors the kNB x kNB diagonal block in LDS and inverts it (-> Dinv), every thread solves
// one panel row against it (panel kept in LDS), then 4x4 register tiles apply the trailing SYRK update.
// ok[0] = 0 when a pivot is not positive (the solve then runs without the coarse correction).
__global__ __launch_bounds__(1024) void k_tl_chol(int m, double* __restrict__ A, double* __restrict__ Dinv,
                                                  int* __restrict__ ok) {
    extern __shared__ double lds[];
    double* Pn = lds;  // [m][kPS]; rows [kb, kb+nb) double as the diagonal block of the current step
    __shared__ int bad;
    const int t = threadIdx.x;
    if (t == 0) bad = 0;
    __syncthreads();
    for (int kb = 0; kb < m; kb += kNB) {
        const int nb = min(kNB, m - kb);
        double* Dg = Pn + (size_t)kb * kPS;
        for (int e = t; e < nb * nb; e += 1024) {
            const int r = e / nb, c = e % nb;
            Dg[r * kPS + c] = (c <= r) ? A[(size_t)(kb + r) * m + kb + c] : 0.0;
        }
        __syncthreads();
        if (t < 64) {
            const int r = t;
            for (int j = 0; j < nb; ++j) {
                double djj = Dg[j * kPS + j];
                if (!(djj > 0.0)) {
                    if (r == 0) bad = 1;
                    djj = 1.0;
                }
                const double d = sqrt(djj);
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                double lrj = 0.0;
                if (r < nb && r > j) {
                    lrj = Dg[r * kPS + j] / d;
                    Dg[r * kPS + j] = lrj;
                }
                if (r == j) Dg[j * kPS + j] = d;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                if (r < nb && r > j)
                    for (int c = j + 1; c <= r; ++c) Dg[r * kPS + c] -= lrj * Dg[c * kPS + j];
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            }
            // inverse of the lower-triangular block: lane c owns column c
            if (r < kNB) {
                const int c = r;
                double x[kNB];
#pragma unroll
                for (int q = 0; q < kNB; ++q) x[q] = 0.0;
                double* Dv = Dinv + (size_t)(kb / kNB) * kNB * kNB;
                if (c < nb) {
#pragma unroll
                    for (int rr = 0; rr < kNB; ++rr) {
                        if (rr < nb && rr >= c) {
                            double s = (rr == c) ? 1.0 : 0.0;
#pragma unroll
                            for (int q = 0; q < kNB; ++q)
                                if (q >= c && q < rr) s -= Dg[rr * kPS + q] * x[q];
                            x[rr] = s / Dg[rr * kPS + rr];
                        }
                    }
                }
#pragma unroll
                for (int rr = 0; rr < kNB; ++rr) Dv[rr * kNB + c] = x[rr];
            }
        }
        __syncthreads();
        for (int e = t; e < nb * nb; e += 1024) {
            const int r = e / nb, c = e % nb;
            if (c <= r) A[(size_t)(kb + r) * m + kb + c] = Dg[r * kPS + c];
        }
        // panel: row i solves x L_kk^T = a
        const int i = kb + nb + t;
        if (i < m) {
            double x[kNB];
#pragma unroll
            for (int c = 0; c < kNB; ++c) x[c] = (c < nb) ? A[(size_t)i * m + kb + c] : 0.0;
#pragma unroll
            for (int c = 0; c < kNB; ++c) {
                if (c < nb) {
                    double s = x[c];
#pragma unroll
                    for (int q = 0; q < kNB; ++q)
                        if (q < c) s -= x[q] * Dg[c * kPS + q];
                    x[c] = s / Dg[c * kPS + c];
                }
            }
#pragma unroll
            for (int c = 0; c < kNB; ++c)
                if (c < nb) {
                    A[(size_t)i * m + kb + c] = x[c];
                    Pn[(size_t)i * kPS + c] = x[c];
                }
        }
        __syncthreads();
        // trailing update of the lower triangle, 4x4 tiles
        const int base = kb + nb, n = m - base;
        if (n > 0) {
            const int nt = (n + 3) / 4;
            const int ntiles = nt * (nt + 1) / 2;
            for (int tt = t; tt < ntiles; tt += 1024) {
                int I = (int)((sqrt(8.0 * tt + 1.0) - 1.0) * 0.5);
                while (I * (I + 1) / 2 > tt) --I;
                while ((I + 1) * (I + 2) / 2 <= tt) ++I;
                const int J = tt - I * (I + 1) / 2;
                const int r0 = base + 4 * I, c0 = base + 4 * J;
                double acc[4][4];
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) acc[u][v] = 0.0;
                for (int k = 0; k < nb; ++k) {
                    double a[4], bq[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) a[u] = (r0 + u < m) ? Pn[(size_t)(r0 + u) * kPS + k] : 0.0;
#pragma unroll
                    for (int v = 0; v < 4; ++v) bq[v] = (c0 + v < m) ? Pn[(size_t)(c0 + v) * kPS + k] : 0.0;
#pragma unroll
                    for (int u = 0; u < 4; ++u)
#pragma unroll
                        for (int v = 0; v < 4; ++v) acc[u][v] += a[u] * bq[v];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int r = r0 + u, c = c0 + v;
                        if (r < m && c <= r) A[(size_t)r * m + c] -= acc[u][v];
                    }
            }
        }
        __threadfence_block();
        __syncthreads();
    }
    if (t == 0) ok[0] = !bad;
}

// Workgroup J computes columns [J*kNB, J*kNB + kNB) of L^-1 by block forward substitution:
//   X_R = Dinv_R (I_RJ - sum_{K<R} L_RK X_K), column block kept in LDS.
__global__ __launch_bounds__(1024) void k_tl_trinv(int m, const double* __restrict__ Lc, const double* __restrict__ Dinv,
                                                   double* __restrict__ Linv, const int* __restrict__ ok) {
    extern __shared__ double lds[];
    double* X = lds;                      // [m][kPS]
    double* Tb = lds + (size_t)m * kPS;   // [kNB][kPS]
    if (!ok[0]) return;
    const int J = blockIdx.x;
    const int t = threadIdx.x, rr = t / kNB, c = t % kNB;
    const int j0 = J * kNB;
    const int colv = j0 + c < m;
    const int nB = (m + kNB - 1) / kNB;
    for (int R = J; R < nB; ++R) {
        const int r0 = R * kNB, nr = min(kNB, m - r0);
        double v = 0.0;
        if (rr < nr && colv) {
            v = (R == J && rr == c) ? 1.0 : 0.0;
            const double* Lrow = Lc + (size_t)(r0 + rr) * m;
            for (int k = j0; k < r0; ++k) v -= Lrow[k] * X[(size_t)k * kPS + c];
        }
        Tb[rr * kPS + c] = v;
        __syncthreads();
        double x = 0.0;
        if (rr < nr && colv) {
            const double* Dv = Dinv + (size_t)R * kNB * kNB + rr * kNB;
            for (int q = 0; q <= rr; ++q) x += Dv[q] * Tb[q * kPS + c];
            X[(size_t)(r0 + rr) * kPS + c] = x;
            Linv[(size_t)(r0 + rr) * m + j0 + c] = x;
        }
        __syncthreads();
    }
}

// E^-1 = L^-T L^-1 : one 32x32 tile per workgroup, rows of L^-1 staged through LDS.
__global__ __launch_bounds__(1024) void k_tl_gram(int m, const double* __restrict__ Linv, double* __restrict__ Einv,
                                                  const int* __restrict__ ok) {
    __shared__ double A[kNB][kPS];
    __shared__ double B[kNB][kPS];
    if (!ok[0]) return;
    const int nB = (m + kNB - 1) / kNB;
    const int tk = blockIdx.x / nB, tlb = blockIdx.x % nB;
    const int t = threadIdx.x, kk = t / kNB, ll = t % kNB;
    const int k0 = tk * kNB, l0 = tlb * kNB;
    double acc = 0.0;
    for (int r0 = max(k0, l0); r0 < m; r0 += kNB) {
        const int rr = t / kNB, cc = t % kNB;
        const int r = r0 + rr;
        A[rr][cc] = (r < m && k0 + cc < m) ? Linv[(size_t)r * m + k0 + cc] : 0.0;
        B[rr][cc] = (r < m && l0 + cc < m) ? Linv[(size_t)r * m + l0 + cc] : 0.0;
        __syncthreads();
#pragma unroll 8
        for (int q = 0; q < kNB; ++q) acc += A[q][kk] * B[q][ll];
        __syncthreads();
    }
    if (k0 + kk < m && l0 + ll < m) Einv[(size_t)(k0 + kk) * m + l0 + ll] = acc;
}

// ---- per iteration ------------------------------------------------------------------------------------------
// Recurrence step i = it - 1 (it >= 1): every workgroup sums the row partials of launch it-1 in the same fixed order,
// tests convergence on rho_i = ||L r~_i||^2 <= tol^2 ||b||^2 and forms alpha_i, beta_i; workgroup 0 records them.
// Then, per camera row: p = u + beta p, s = w + beta s, x += alpha p, r -= alpha s, R_i = Z~_i^T r_i, rho_{i+1}.
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_update(int it, int C, int maxit, double tol2_rel,
                                                        const double* __restrict__ Lf, CgBufs cg, TlBufs tl) {
    constexpr int MC = D + 1, RPW = kThreads / D;
    __shared__ double red[3][kWaves];
    __shared__ double rl[RPW][D];
    __shared__ double sq[RPW][D];
    __shared__ double sc[3];
    if (cg.status[0] != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int i = it - 1;
    const double* G0 = tl.gd;
    const double* G1 = tl.gd + C;
    const double* RH = tl.rho[i & 1];
    double g0 = 0.0, g1 = 0.0, g2 = 0.0;
    for (int k = t; k < C; k += kThreads) { g0 += G0[k]; g1 += G1[k]; g2 += RH[k]; }
    g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
    if (lane == 0) { red[0][wv] = g0; red[1][wv] = g1; red[2][wv] = g2; }
    __syncthreads();
    if (t == 0) {
        double gam = 0.0, del = 0.0, rho = 0.0;
        for (int w = 0; w < kWaves; ++w) { gam += red[0][w]; del += red[1][w]; rho += red[2][w]; }
        const double h_alpha = (i >= 1) ? cg.hist[2 * (i - 1)] : 1.0;
        const double h_gam = (i >= 1) ? cg.hist[2 * (i - 1) + 1] : 1.0;
        const double bb = (i == 0) ? rho : cg.hist[2 * (maxit + 1)];
        double flag = 0.0, al = 0.0, be = 0.0;
        const bool lead = blockIdx.x == 0;
        if (rho <= tol2_rel * bb || i >= maxit) {
            flag = 1.0;
            if (lead) { cg.status[1] = i; __threadfence(); cg.status[0] = 1; }
        } else {
            const double den = (i == 0) ? del : del - (gam / h_gam) * gam / h_alpha;
            be = (i == 0) ? 0.0 : gam / h_gam;
            if (!(den > 0.0)) {
                flag = 2.0;
                if (lead) { cg.status[1] = i; __threadfence(); cg.status[0] = 2; }
            } else {
                al = gam / den;
                if (lead) {
                    cg.hist[2 * i] = al;
                    cg.hist[2 * i + 1] = gam;
                    if (i == 0) cg.hist[2 * (maxit + 1)] = bb;
                }
            }
        }
        sc[0] = al; sc[1] = be; sc[2] = flag;
    }
    __syncthreads();
    if (sc[2] != 0.0) return;
    const double al = sc[0], be = sc[1];
    const int rloc = t / D, a = t % D;
    const int row = blockIdx.x * RPW + rloc;
    const bool on = rloc < RPW && row < C;
    if (on) {
        const size_t idx = (size_t)row * D + a;
        const double pn = tl.u[idx] + be * cg.p[idx];
        const double sn = cg.w[0][idx] + be * cg.s[0][idx];
        cg.p[idx] = pn;
        cg.s[0][idx] = sn;
        cg.x[idx] += al * pn;
        const double rn = cg.r[0][idx] - al * sn;
        cg.r[0][idx] = rn;
        rl[rloc][a] = rn;
    }
    __syncthreads();
    if (on) {
        const double* L = Lf + (size_t)row * D * D + a * D;
        double lr = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k)
            if (k <= a) lr += L[k] * rl[rloc][k];
        sq[rloc][a] = lr * lr;
    }
    for (int e = t; e < RPW * MC; e += kThreads) {
        const int rr = e / MC, k = e % MC;
        const int row2 = blockIdx.x * RPW + rr;
        if (row2 < C) {
            const double* Z = tl.Zt + (size_t)row2 * D * MC + k;
            double s = 0.0;
#pragma unroll
            for (int aa = 0; aa < D; ++aa) s += Z[aa * MC] * rl[rr][aa];
            tl.Rp[(size_t)row2 * MC + k] = s;
        }
    }
    __syncthreads();
    if (t < RPW && blockIdx.x * RPW + t < C) {
        double s = 0.0;
#pragma unroll
        for (int aa = 0; aa < D; ++aa) s += sq[t][aa];
        tl.rho[it & 1][blockIdx.x * RPW + t] = s;
    }
}

// One workgroup per cluster c: R (all clusters, fixed member order), y_c = (E^-1 R) rows of c, u_i = r_i + Z~_i y_c.
// Without a usable coarse matrix: u = r.
template <int D>
__global__ __launch_bounds__(kThreads) void k_tl_coarse(CgBufs cg, TlBufs tl, const double* __restrict__ Einv) {
    constexpr int MC = D + 1;
    extern __shared__ double Rs[];  // [m] + y[MC]
    if (cg.status[0] != 0) return;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int c = blockIdx.x, m = tl.m;
    double* y = Rs + m;
    const bool use = tl.ok[0] != 0;
    if (use) {
        for (int q = t; q < m; q += kThreads) {
            const int cc = q / MC, k = q % MC;
            double s = 0.0;
            for (int e = tl.cl_ptr[cc]; e < tl.cl_ptr[cc + 1]; ++e) s += tl.Rp[(size_t)tl.cl_cams[e] * MC + k];
            Rs[q] = s;
        }
        __syncthreads();
        for (int k = wv; k < MC; k += kWaves) {
            const double* Er = Einv + (size_t)(c * MC + k) * m;
            double s = 0.0;
            for (int l = lane; l < m; l += 64) s += Er[l] * Rs[l];
            s = wave_sum(s);
            if (lane == 0) y[k] = s;
        }
        __syncthreads();
    }
    const int e0 = tl.cl_ptr[c], ne = tl.cl_ptr[c + 1] - e0;
    for (int e = t; e < ne * D; e += kThreads) {
        const int i = tl.cl_cams[e0 + e / D], a = e % D;
        const size_t idx = (size_t)i * D + a;
        double v = cg.r[0][idx];
        if (use) {
            const double* Z = tl.Zt + idx * MC;
#pragma unroll
            for (int k = 0; k < MC; ++k) v += Z[k] * y[k];
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
