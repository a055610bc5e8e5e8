// The two-level pipelined PCG of a solve as ONE persistent launch with S~ held in the register file (D = 8).
//
// The launch-per-phase CG (ba_twolevel.h: k_tl_pc_cl + k_tl_pspmv per iteration) streams the 61-MB row copy of S~ from
// the Infinity Cache every iteration (~13 us on config 3) and pays two kernel boundaries.  Here one wave owns one camera
// row for the whole solve: lane l = 8 a + b holds entry (a, b) of each of the row's blocks (one double per block and
// lane; NB blocks, 2 NB registers, most of them AGPRs at one wave per SIMD), so the operator is read from HBM once per
// solve.  With the coarse correction written as  n = S~ m = m_i + sum_j S~_ij w_j + sum_c A_ic y_c  (m = w + Z~ y,
// y = E^-1 Z~^T w, A_ic = sum_{j in c} S~_ij Z~_j over the row's off-diagonal blocks of neighbour cluster c, formed once
// per solve from the register-resident blocks), an iteration needs two grid-wide hand-offs:
//   P1  every wave: gamma, delta, rho from the per-cluster atomic partials -> convergence, alpha, beta (k_tl_pc_cl's
//       butterfly, so the same doubles in every wave); y_k = (E^-1 R)_k, coarse row k on wave k mod (waves of the
//       grid), its row of E^-1 read from L2; every row: S~ w, the neighbours' w (the previous iteration's exchange) gathered
//       eight blocks per load instruction into LDS;
//   ---- grid barrier ----
//   P2  y into LDS; every row: m_i, n_i, the recurrence update of the row (k_tl_pspmv's formulas), the partials of the
//       next iteration (per-cluster atomics) and the row's new w into the exchange buffer;
//   ---- grid barrier ----
// The recurrence is the oracle's (oracle/ba_oracle.c ora_pcg, pipelined two-level branch) and k_tl_pc_cl/k_tl_pspmv's;
// only the summation order inside S~ m differs.  Every handed-off word is stored write-through (sc1) or added by an
// agent-scope atomic and read with sc1 loads; every storing wave drains (vmcnt(0)) before the workgroup barrier behind
// which one lane arrives (MI355X_MICROARCH.md, hand-off table row 1; cdna_hip_programming.md Guideline 16 R1).  The
// grid barrier is two-level: arrivals per group of workgroups (blockIdx % 8: one XCD under round-robin placement, speed
// only), the last of a group arrives at the top counter, the last there releases every group's generation word.  Every
// spin is bounded; a timeout raises the abort word (status 4), which every waiting workgroup checks.
// Host eligibility (ba_kernels.hip, create): single rank, atomic cluster sums (non-deterministic mode), D = 8, rows of at
// most NB = 128 blocks stored in cluster order (tl.sperm the identity), at most kCgpSegMax neighbour clusters per row,
// and every workgroup resident at once (one per CU).
#pragma once
#include "ba_common.h"
#include "ba_twolevel.h"

namespace insfm {

constexpr int kCgpRows = 4;                      // camera rows per workgroup
constexpr int kCgpWaves = kCgpRows;              // one wave per row, one per SIMD (the row's blocks spill into AGPRs)
constexpr int kCgpThreads = 64 * kCgpWaves;
constexpr int kCgpSegMax = 32;                   // neighbour-cluster segments per row (LDS table of A_ic)
constexpr int kCgpGroups = 8;                    // barrier arrival groups
constexpr int kCgpSyncWords = (2 * kCgpGroups + 2) * 32;  // [group x 8][top][generation x 8][abort], 128-B apart
constexpr unsigned kCgpSpinMax = 1u << 22;       // polls before a barrier gives up (~seconds; the host's stall limit is 10 s)

__device__ __forceinline__ unsigned* cgp_grp(unsigned* s, int g) { return s + 32 * g; }
__device__ __forceinline__ unsigned* cgp_top(unsigned* s) { return s + 32 * kCgpGroups; }
__device__ __forceinline__ unsigned* cgp_gen(unsigned* s, int g) { return s + 32 * (kCgpGroups + 1 + g); }
__device__ __forceinline__ unsigned* cgp_abort(unsigned* s) { return s + 32 * (2 * kCgpGroups + 1); }

// Grid barrier number `epoch` (1, 2, ...; the words are zeroed before the launch).  Every wave drains its own stores
// and atomics (vmcnt(0)) before the workgroup barrier that orders them in front of lane 0's arrival.  Returns false in
// every thread when the barrier timed out or another workgroup aborted.
__device__ __forceinline__ bool cgp_barrier(unsigned* sync, unsigned epoch, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const int G = gridDim.x, g = blockIdx.x % kCgpGroups;
        const int ngroups = G < kCgpGroups ? G : kCgpGroups;
        const unsigned gsize = (unsigned)((G - g + kCgpGroups - 1) / kCgpGroups);
        const unsigned a = __hip_atomic_fetch_add(cgp_grp(sync, g), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        if (a == epoch * gsize) {
            const unsigned t = __hip_atomic_fetch_add(cgp_top(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
            if (t == epoch * (unsigned)ngroups)
                for (int q = 0; q < ngroups; ++q)
                    __hip_atomic_store(cgp_gen(sync, q), epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int ok = 1;
        for (unsigned spins = 0;
             __hip_atomic_load(cgp_gen(sync, g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < epoch;) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 255u) == 0u &&
                (spins >= kCgpSpinMax || __hip_atomic_load(cgp_abort(sync), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                __hip_atomic_store(cgp_abort(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
        }
        *flag = ok;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*flag) != 0;
}

// a wave-uniform double (every lane holds the same value) as a scalar: branches on it are scalar branches
__device__ __forceinline__ double uni(double v) {
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}

// NB: blocks per row held in registers (a multiple of 8).  sync: kCgpSyncWords zeroed words; wx: [C][8] the w
// exchange (one buffer: P1 reads it before the barrier behind which P2 rewrites it); yx: [m] the coarse vector;
// trace (diagnostics, normally null): gamma, delta, rho, done of the first 64 iterations.
template <int NB>
__global__ __launch_bounds__(kCgpThreads, 1) void k_tl_cgp(int C, const int* __restrict__ nbr_ptr,
                                                          const int* __restrict__ nbr_j, const double* __restrict__ Sn,
                                                          const double* __restrict__ Lf, CgBufs cg, TlBufs tl,
                                                          const double* __restrict__ Einv, int maxit, double tol2_rel,
                                                          double* wx, double* yx, unsigned* sync, double* trace) {
    static_assert(NB % 8 == 0, "k_tl_cgp gathers eight blocks per load instruction");
    constexpr int D = 8, MC = 9, BS = D * MC, LPL = (kCoarseMax + 63) / 64, LNC = (kCoarseMax / MC + 63) / 64;
    constexpr int NG = NB / 8;                          // gather loads per wave and iteration
    constexpr int RPT = (kCoarseMax + kCgpThreads - 1) / kCgpThreads;  // coarse entries per thread (LDS fills)
    __shared__ double Aseg[kCgpRows][kCgpSegMax][BS];  // A_ic of the row's segments, a-major
    __shared__ double wg[kCgpWaves][NB][D];            // the neighbours' w of the wave's blocks (gathered per iteration)
    __shared__ double rs[kCoarseMax];                  // the restriction R of the iteration, then y
    __shared__ double Lrow[kCgpRows][D * D];           // L_i (row a, column k)
    __shared__ double Zrow[kCgpRows][BS];              // Z~_i (row a, column k)
    __shared__ double vec[kCgpRows][8][D];             // the row's r u w z q s p x
    __shared__ int jn[kCgpWaves][NB];                  // neighbour of each register block
    __shared__ int segc[kCgpRows][kCgpSegMax];         // neighbour cluster of each segment
    __shared__ int bflag;
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);  // (wave-uniform: the row's values live in SGPRs)
    const int a8 = lane >> 3, b8 = lane & 7;           // block entry (a, b) of this lane
    const int rl = wv;                                 // local row
    const int row = blockIdx.x * kCgpRows + rl;
    const bool has_row = row < C;
    const int m = tl.m, nc = tl.nc;
    const int gw = blockIdx.x * kCgpWaves + wv;        // this wave's coarse row of E^-1 (if gw < m)
    const int n0 = has_row ? nbr_ptr[row] : 0;
    const int len = has_row ? nbr_ptr[row + 1] - n0 : 0;
    const int nk = min(len, NB);                       // blocks of the row (the host checks len <= NB)
    const int s0 = has_row ? tl.rseg_ptr[row] : 0, nseg = has_row ? tl.rseg_ptr[row + 1] - s0 : 0;
    double* V = &vec[rl][0][0];
    enum { VR = 0, VU = 8, VW = 16, VZ = 24, VQ = 32, VS = 40, VP = 48, VX = 56 };
    // ---- setup ----
    // the row's blocks (slots past the row: zero, neighbour = the row itself, so the products need no guard)
    double sreg[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) sreg[k] = k < nk ? Sn[(size_t)(n0 + k) * (D * D) + lane] : 0.0;
    for (int k = lane; k < NB; k += 64) jn[wv][k] = k < nk ? nbr_j[n0 + k] : (has_row ? row : 0);
    for (int e = t; e < kCgpRows * kCgpSegMax * BS; e += kCgpThreads) (&Aseg[0][0][0])[e] = 0.0;
    const size_t own = (size_t)(has_row ? row : 0) * D + (lane & 7);
    {
        if (lane < nseg && lane < kCgpSegMax) segc[rl][lane] = tl.seg[s0 + lane].x;
        if (has_row) {
            Lrow[rl][lane] = Lf[(size_t)row * D * D + lane];
            for (int e = lane; e < BS; e += 64) Zrow[rl][e] = tl.Zt[(size_t)row * BS + e];
            const double* src = lane < 8 ? cg.r[0] : lane < 16 ? tl.u : lane < 24 ? cg.w[0] : lane < 32 ? cg.w[1]
                              : lane < 40 ? cg.r[1] : lane < 48 ? cg.s[0] : lane < 56 ? cg.p : cg.x;
            V[lane] = src[own];
        }
    }
    __syncthreads();
    // A_ic: lane (a, b) sums S~_ij[a][b] Z~_j[b][q] over the segment's blocks, then adds them into Aseg (LDS atomics).  Segment boundaries are wave-uniform; the Z~ rows
    // of two blocks are loaded together ahead of their products.
    if (nk > 0) {
        int cur = 0;
        while (cur < nseg && tl.seg[s0 + cur].z <= 0) ++cur;
        int send = cur < nseg ? tl.seg[s0 + cur].z : 1 << 30;
        double za[MC];
#pragma unroll
        for (int q = 0; q < MC; ++q) za[q] = 0.0;
        auto flush = [&]() {
            if (cur < kCgpSegMax) {
#pragma unroll
                for (int q = 0; q < MC; ++q) {
                    __hip_atomic_fetch_add(&Aseg[rl][cur][a8 * MC + q], za[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    za[q] = 0.0;
                }
            }
            ++cur;
            send = cur < nseg ? tl.seg[s0 + cur].z : 1 << 30;
        };
        constexpr int CH = 2;
#pragma unroll
        for (int k0 = 0; k0 < NB; k0 += CH) {
            if (k0 >= nk) continue;
            double zv[CH][MC];
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const double* zr = tl.Zt + ((size_t)jn[wv][k0 + c] * D + b8) * MC;
#pragma unroll
                for (int q = 0; q < MC; ++q) zv[c][q] = zr[q];
            }
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int k = k0 + c;
                if (k < nk) {
                    while (k >= send) flush();
#pragma unroll
                    for (int q = 0; q < MC; ++q) za[q] += sreg[k] * zv[c][q];
                }
            }
        }
        flush();
    }
    const int ci = has_row ? tl.clab[row] : 0;
    const bool use = tl.ok[0] != 0;
    const double* erow = Einv + (size_t)min(gw, m - 1) * m;  // this wave's coarse row of E^-1 (read from L2)
    double h_alpha = 1.0, h_gam = 1.0, h_bb = 1.0;
    unsigned epoch = 0;
    bool alive = true;
    int it = 0;
    __syncthreads();  // Aseg complete
    for (;; ++it) {
        // ======== P1 ========
        // every load of the phase is issued before the first wait: the scalar partials, this wave's gathers (lane
        // (a, b) loads entry b of the w of block 8 g + a), the restriction (all threads, into LDS), the E^-1 row
        const double* G = tl.Gacc + (size_t)(it & 1) * 3 * nc;
        double gl[3][LNC];
#pragma unroll
        for (int q = 0; q < LNC; ++q) {
            const int l = min(lane + 64 * q, nc - 1);
            gl[0][q] = ld_sc1(G + l); gl[1][q] = ld_sc1(G + nc + l); gl[2][q] = ld_sc1(G + 2 * nc + l);
        }
        const double* wsrc = (it == 0 ? cg.w[0] : wx) + b8;
        double wv8[NG];
#pragma unroll
        for (int g = 0; g < NG; ++g) wv8[g] = ld_sc1(wsrc + (size_t)jn[wv][8 * g + a8] * D);
        const double* Rv = tl.Racc + (size_t)(it & 1) * m;
        double rv[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) rv[q] = use ? ld_sc1(Rv + min(t + q * kCgpThreads, m - 1)) : 0.0;
        double ev[LPL];
        if (use && gw < m) {
#pragma unroll
            for (int q = 0; q < LPL; ++q) ev[q] = erow[min(lane + 64 * q, m - 1)];
        }
        double ga0 = 0.0, ga1 = 0.0, ga2 = 0.0;
#pragma unroll
        for (int q = 0; q < LNC; ++q)
            if (lane + 64 * q < nc) { ga0 += gl[0][q]; ga1 += gl[1][q]; ga2 += gl[2][q]; }
        const double gam = uni(wave_sum(ga0)), del = uni(wave_sum(ga1)), rho = uni(wave_sum(ga2));
        const double bb = (it == 0) ? rho : h_bb;
        double alpha = 0.0, be = 0.0;
        int done = 0;
        if (rho <= tol2_rel * bb || it >= maxit) {
            done = 1;
        } else {
            be = (it == 0) ? 0.0 : gam / h_gam;
            const double den = (it == 0) ? del : del - be * gam / h_alpha;
            if (!(den > 0.0)) done = 2;
            else alpha = gam / den;
        }
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) {  // INSFM_DIAG=cgp_trace
            trace[4 * it] = gam; trace[4 * it + 1] = del; trace[4 * it + 2] = rho; trace[4 * it + 3] = done;
        }
        if (blockIdx.x == 0 && t == 0) {
            if (done) {
                cg.status[1] = it;
                cg.status[0] = done;
            } else {
                cg.hist[2 * it] = alpha;
                cg.hist[2 * it + 1] = gam;
                if (it == 0) cg.hist[2 * (maxit + 1)] = bb;
            }
            if (cg.prog) {
                if (done) {
                    __hip_atomic_store(cg.prog + 2, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(cg.prog + 1, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                } else {
                    __hip_atomic_store(cg.prog + 0, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        if (done) break;
        if (it == 0) h_bb = bb;
        h_alpha = alpha;
        h_gam = gam;
        // the partial buffers of iteration it + 1 (last read in P1 of it - 1) are cleared for this iteration's P2
        if (blockIdx.x == 0) {
            double* Rn = tl.Racc + (size_t)((it + 1) & 1) * m;
            double* Gn = tl.Gacc + (size_t)((it + 1) & 1) * 3 * nc;
            for (int q = t; q < m; q += kCgpThreads) st_sc1(Rn + q, 0.0);
            for (int q = t; q < 3 * nc; q += kCgpThreads) st_sc1(Gn + q, 0.0);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) wg[wv][8 * g + a8][b8] = wv8[g];
        if (use) {
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if (t + q * kCgpThreads < m) rs[t + q * kCgpThreads] = rv[q];
        }
        __syncthreads();
        // coarse row gw: y = E^-1 R (k_tl_pc_cl's products and butterfly)
        if (use && gw < m) {
            double sy = 0.0;
#pragma unroll
            for (int q = 0; q < LPL; ++q)
                if (lane + 64 * q < m) sy += ev[q] * rs[lane + 64 * q];
            const double y = wave_sum(sy);
            if (lane == 0) st_sc1(yx + gw, y);
        }
        // more coarse rows than waves (small grids): the rest, E^-1 rows loaded here
        for (int g = gw + gridDim.x * kCgpWaves; use && g < m; g += gridDim.x * kCgpWaves) {
            const double* er = Einv + (size_t)g * m;
            double sy = 0.0;
            for (int l = lane; l < m; l += 64) sy += er[l] * rs[l];
            const double y = wave_sum(sy);
            if (lane == 0) st_sc1(yx + g, y);
        }
        // the row's S~ w (lane a < 8 ends with entry a)
        double sw = 0.0;
        if (has_row) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < NB; ++k) acc += sreg[k] * wg[wv][k][b8];
            acc += __shfl_xor(acc, 1, 64);
            acc += __shfl_xor(acc, 2, 64);
            acc += __shfl_xor(acc, 4, 64);
            sw = __shfl(acc, 8 * (lane & 7), 64);
        }
        if (!(alive = cgp_barrier(sync, ++epoch, &bflag))) break;
        // ======== P2 ========
        if (use) {
            double yv[RPT];
#pragma unroll
            for (int q = 0; q < RPT; ++q) yv[q] = ld_sc1(yx + min(t + q * kCgpThreads, m - 1));
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if (t + q * kCgpThreads < m) rs[t + q * kCgpThreads] = yv[q];
            __syncthreads();
        }
        if (has_row) {
            const int la = lane & 7;
            const double w_ = V[VW + la];
            double mi = w_, ay = 0.0;
            if (use) {
                double sz = 0.0;
#pragma unroll
                for (int k = 0; k < MC; ++k) sz += Zrow[rl][la * MC + k] * rs[ci * MC + k];
                mi += sz;
                const int ns = min(nseg, kCgpSegMax);
                for (int sg = 0; sg < ns; ++sg) {
                    const double* yc = rs + segc[rl][sg] * MC;
                    const double* A = &Aseg[rl][sg][la * MC];
#pragma unroll
                    for (int k = 0; k < MC; ++k) ay += A[k] * yc[k];
                }
            }
            const double prod = mi + (sw + ay);  // (the diagonal block of S~ is I)
            const double zn = prod + be * V[VZ + la];
            const double qn = mi + be * V[VQ + la];
            const double sn = w_ + be * V[VS + la];
            const double pn = V[VU + la] + be * V[VP + la];
            const double xn = V[VX + la] + alpha * pn;
            const double rn = V[VR + la] - alpha * sn;
            const double un = V[VU + la] - alpha * qn;
            const double wn = w_ - alpha * zn;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < D) {
                V[VZ + la] = zn; V[VQ + la] = qn; V[VS + la] = sn; V[VP + la] = pn;
                V[VX + la] = xn; V[VR + la] = rn; V[VU + la] = un; V[VW + la] = wn;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // partials of iteration it + 1: r.u, w.u, ||L r||^2 and the restriction Z~_i^T w (k_tl_pspmv's order)
            double g0 = 0.0, g1 = 0.0, g2 = 0.0, rr = 0.0;
            if (lane < D) {
                g0 = rn * un;
                g1 = wn * un;
                double lr = 0.0;
#pragma unroll
                for (int k = 0; k < D; ++k)
                    if (k <= lane) lr += Lrow[rl][lane * D + k] * V[VR + k];
                g2 = lr * lr;
            }
            if (lane < MC) {
#pragma unroll
                for (int a = 0; a < D; ++a) rr += Zrow[rl][a * MC + lane] * V[VW + a];
            }
            g0 = wave_sum(g0); g1 = wave_sum(g1); g2 = wave_sum(g2);
            const int bsel = (it + 1) & 1;
            if (lane < MC) unsafeAtomicAdd(tl.Racc + (size_t)bsel * m + (size_t)ci * MC + lane, rr);
            if (lane == 0) {
                double* Gq = tl.Gacc + (size_t)bsel * 3 * nc;
                unsafeAtomicAdd(Gq + ci, g0);
                unsafeAtomicAdd(Gq + nc + ci, g1);
                unsafeAtomicAdd(Gq + 2 * nc + ci, g2);
            }
            if (lane < D) st_sc1(wx + (size_t)row * D + lane, wn);
        }
        if (!(alive = cgp_barrier(sync, ++epoch, &bflag))) break;
    }
    if (!alive && blockIdx.x == 0 && t == 0) {
        cg.status[1] = it;
        cg.status[0] = 4;
        if (cg.prog) {
            __hip_atomic_store(cg.prog + 2, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(cg.prog + 1, 4, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // the scaled solution for k_cg_finish, and the vectors as the launch path leaves them
    if (has_row) {
        double* dst = lane < 8 ? cg.r[0] : lane < 16 ? tl.u : lane < 24 ? cg.w[0] : lane < 32 ? cg.w[1]
                    : lane < 40 ? cg.r[1] : lane < 48 ? cg.s[0] : lane < 56 ? cg.p : cg.x;
        dst[own] = V[lane];
    }
}

}  // namespace insfm
