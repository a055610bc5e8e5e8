// The two-level pipelined PCG of a solve as ONE persistent launch with S~ held in the register file (D = 8).
//
// The launch-per-phase CG (ba_twolevel.h: k_tl_pc_cl + k_tl_pspmv per iteration) streams the 61-MB row copy of S~ from
// the Infinity Cache every iteration (~13 us on config 3) and pays two kernel boundaries.  Here one wave owns one camera
// row for the whole solve: lane l = 8 a + b holds entry (a, b) of each of the row's blocks (one double per block and
// lane; NB blocks, 2 NB registers, most of them AGPRs at one wave per SIMD), so the operator is read from HBM once per
// solve.  With the coarse correction written as  n = S~ m = m_i + sum_j S~_ij w_j + sum_c A_ic y_c  (m = w + Z~ y,
// y = E^-1 Z~^T w, A_ic = sum_{j in c} S~_ij Z~_j over the row's off-diagonal blocks of neighbour cluster c, formed once
// per solve from the register-resident blocks), an iteration needs one grid barrier:
//   P1  every wave: gamma, delta, rho from the per-cluster atomic partials -> convergence, alpha, beta (k_tl_pc_cl's
//       butterfly, so the same doubles in every wave); y_k = (E^-1 R)_k, coarse row k on wave k mod (waves of the
//       grid), its row of E^-1 read from L2; every row: S~ w, the neighbours' w (the previous iteration's exchange) gathered
//       eight blocks per load instruction into LDS;
//   P2  y into LDS (each coarse row is published as two tagged 8-byte granules that are their own flag: the workgroups
//       poll them, no grid barrier); every row: m_i, n_i, the recurrence update of the row (k_tl_pspmv's formulas), the
//       partials of the next iteration (summed per cluster run of the workgroup in LDS, then per-cluster atomics into
//       one of three buffers) and the row's new w into the exchange buffer of the next parity;
//   ---- grid barrier ----
// The recurrence is the oracle's (oracle/ba_oracle.c ora_pcg, pipelined two-level branch) and k_tl_pc_cl/k_tl_pspmv's;
// only the summation order inside S~ m differs.  Every handed-off word is stored write-through (sc1) or added by an
// agent-scope atomic and read with sc1 loads; every storing wave drains (vmcnt(0)) before the workgroup barrier behind
// which one lane arrives (MI355X_MICROARCH.md, hand-off table row 1; cdna_hip_programming.md Guideline 16 R1).  The
// grid barrier counts arrivals per group of workgroups (blockIdx % 8: one XCD under round-robin placement, speed only)
// and every workgroup polls the eight counters at once.  Every spin is bounded; a timeout raises the abort word
// (status 4), which every waiting workgroup checks; a single-rank host then repeats the solve on the launch path and
// stays there.
// Two variants: per-cluster atomic partial sums (single rank, non-deterministic), and DET, a fixed summation order
// (deterministic mode and every rank of the replicated multi-rank CG): each workgroup run's partials are stored in a
// parity buffer before the grid barrier, and after it every workgroup sums each cluster's runs itself in run order
// (det_cluster_sums).  Either variant applies the coarse correction additively (precond 1) or as A-DEF2 (ADEF,
// precond 2; round 6 added the DET form of A-DEF2, so the multi-rank and deterministic paths run it too).
// Host eligibility (ba_kernels.hip, create): D = 8, host-mapped progress word, rows of at most NB = 128 blocks stored in
// cluster order (tl.sperm the identity), at most kCgpSegMax neighbour clusters per row, and every workgroup resident at
// once (one per CU) -- for ranks sharing a GPU, all of their grids at once.
#pragma once
#include <climits>

#include "ba_common.h"
#include "ba_twolevel.h"

namespace insfm {

constexpr int kCgpRows = 4;                      // camera rows per workgroup
constexpr int kCgpWaves = kCgpRows;              // one wave per row, one per SIMD (the row's blocks spill into AGPRs)
constexpr int kCgpThreads = 64 * kCgpWaves;
constexpr int kCgpSegMax = 40;                   // neighbour-cluster segments per row (LDS table of A_ic)
constexpr int kCgpGroups = 8;                    // barrier arrival groups
constexpr int kCgpSyncWords = (kCgpGroups + 1) * 32;  // [group counter x 8][abort], 128 B apart
constexpr int kCgpMaxClusters = kCoarseMax / 9;   // clusters of a D = 8 handle (m = 9 nc <= kCoarseMax)
constexpr int kCgpRunBatch = 8;                  // cluster runs (or setup rows) an owner loads at once
constexpr int kCgpTraceIt = 5;                   // INSFM_DIAG=cgp_trace: every workgroup's times of this iteration
constexpr int kCgpTraceLen = 772 + 2 * 256;
constexpr unsigned kCgpSpinMax = 1u << 22;       // polls before a barrier gives up (~seconds; the host's stall limit is 10 s)

__device__ __forceinline__ unsigned* cgp_grp(unsigned* s, int g) { return s + 32 * g; }
__device__ __forceinline__ unsigned* cgp_abort(unsigned* s) { return s + 32 * kCgpGroups; }

// Grid barrier number `epoch` (counting on from the barriers of earlier launches: the counters are zeroed at create
// and after an abort only).  Every wave drains its own stores
// and atomics (vmcnt(0)) before the workgroup barrier that orders them in front of lane 0's arrival, one no-return
// agent-scope add on its group's counter (blockIdx % 8).  Wave 0 then polls all group counters at once (lane g loads
// counter g with an sc1 load) until each has reached epoch x its group size: one atomic and one poll round trip per
// barrier, no release step (a hierarchical arrive / release / generation barrier took ~3.7 us).  Returns false in
// every thread when the spin limit passed or another workgroup aborted.
__device__ __forceinline__ bool cgp_barrier(unsigned* sync, unsigned epoch, int* flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int G = gridDim.x;
    if (threadIdx.x == 0)
        __hip_atomic_fetch_add(cgp_grp(sync, blockIdx.x % kCgpGroups), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x < 64) {
        const int g = threadIdx.x & (kCgpGroups - 1);
        const unsigned need = epoch * (unsigned)((G - g + kCgpGroups - 1) / kCgpGroups);  // (0 for an empty group)
        int ok = 1;
        for (unsigned spins = 0;; ) {
            const unsigned v = __hip_atomic_load(cgp_grp(sync, g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(v >= need)) break;
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 255u) == 0u &&
                (spins >= kCgpSpinMax || __hip_atomic_load(cgp_abort(sync), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                if (threadIdx.x == 0) __hip_atomic_store(cgp_abort(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
        }
        if (threadIdx.x == 0) *flag = ok;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*flag) != 0;
}

// y_k of iteration `tag` as two tagged 8-byte granules {tag, low word} / {tag, high word}: the data is its own flag
// (MI355X_MICROARCH.md hand-offs, R2), written by one lane with agent-scope (sc1) stores.
__device__ __forceinline__ void put_y(unsigned long long* yg, int k, unsigned tag, double y) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(y), hi = (unsigned long long)tag << 32;
    __hip_atomic_store(yg + 2 * k, hi | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(yg + 2 * k + 1, hi | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Every thread of the workgroup: poll the granule pairs of entries t, t + 256, ... (entry k at pair map(k)) until both
// halves carry `tag`, then the value into LDS; the workgroup repeats until all of its threads hold theirs.  Bounded:
// false (abort word raised) past the spin limit or when another workgroup aborted.
template <int CAP = kCoarseMax, class Map>
__device__ __forceinline__ bool poll_tagged(const unsigned long long* yg, Map map, double* ys, int m, unsigned tag,
                                            unsigned* sync) {
    constexpr int RPT = (CAP + kCgpThreads - 1) / kCgpThreads;
    const int t = threadIdx.x;
    unsigned have = 0;
    for (unsigned spins = 0;; ++spins) {
        unsigned long long lo[RPT], hi[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int k = min(t + q * kCgpThreads, m - 1);
            lo[q] = hi[q] = 0;
            if (!(have & (1u << q))) {
                lo[q] = __hip_atomic_load(yg + 2 * map(k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                hi[q] = __hip_atomic_load(yg + 2 * map(k) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        int mine = 1;
#pragma unroll
        for (int q = 0; q < RPT; ++q) {
            const int k = t + q * kCgpThreads;
            if (k >= m || (have & (1u << q))) continue;
            if ((unsigned)(lo[q] >> 32) == tag && (unsigned)(hi[q] >> 32) == tag) {
                ys[k] = __longlong_as_double((long long)(((hi[q] & 0xffffffffull) << 32) | (lo[q] & 0xffffffffull)));
                have |= 1u << q;
            } else {
                mine = 0;
            }
        }
        if (__syncthreads_and(mine)) return true;
        __builtin_amdgcn_s_sleep(1);
        if ((spins & 255u) == 255u) {
            const int stop = spins >= kCgpSpinMax ||
                             (t == 0 && __hip_atomic_load(cgp_abort(sync), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (__syncthreads_or(stop)) {
                if (t == 0) __hip_atomic_store(cgp_abort(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return false;
            }
        }
    }
}

__device__ __forceinline__ bool get_y(const unsigned long long* yg, double* ys, int m, unsigned tag, unsigned* sync) {
    return poll_tagged(yg, [](int k) { return k; }, ys, m, tag, sync);
}

// One wave: poll the granule pairs g[idx[q]] (q < n, lane-varying indices) until every lane's all carry `tag`.
template <int N>
__device__ __forceinline__ bool poll_wave(const unsigned long long* g, const int (&idx)[N], double (&out)[N], unsigned tag,
                                          unsigned* sync, unsigned have = 0) {
    for (unsigned spins = 0;; ++spins) {
        int mine = 1;
#pragma unroll
        for (int q = 0; q < N; ++q) {
            if (have & (1u << q)) continue;
            const unsigned long long lo = __hip_atomic_load(g + 2 * idx[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned long long hi = __hip_atomic_load(g + 2 * idx[q] + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)(lo >> 32) == tag && (unsigned)(hi >> 32) == tag) {
                out[q] = __longlong_as_double((long long)(((hi & 0xffffffffull) << 32) | (lo & 0xffffffffull)));
                have |= 1u << q;
            } else {
                mine = 0;
            }
        }
        if (__all(mine)) return true;
        __builtin_amdgcn_s_sleep(1);
        if ((spins & 255u) == 255u &&
            (spins >= kCgpSpinMax || __hip_atomic_load(cgp_abort(sync), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            __hip_atomic_store(cgp_abort(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
    }
}

// a wave-uniform double (every lane holds the same value) as a scalar: branches on it are scalar branches
__device__ __forceinline__ double uni(double v) {
    const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
    const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
    return __hiloint2double(hi, lo);
}

// DET (fixed summation order): rs[e] for e < NS nc (c = e / NS, k = e % NS) = the sum of slot off + k of the
// 12-slot run records of cluster c (rb + position * 12, one record at the head position of each run), taken in run
// order -- the same doubles in every workgroup, no atomics.  Run heads: the cluster's first position, then every
// multiple of kCgpRows inside it; the first RB heads of each entry are loaded at once.
template <int NS>
__device__ __forceinline__ void det_cluster_sums(const double* rb, int off, const int* clp, int nc, double* rs) {
    constexpr int EPT = (NS * kCgpMaxClusters + kCgpThreads - 1) / kCgpThreads;
    constexpr int RB = 6;  // run heads per cluster loaded at once (clusters with more take a second pass)
    const int t = threadIdx.x, ne = NS * nc;
    double x[EPT][RB];
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
        const int e = min(t + q * kCgpThreads, ne - 1), c = e / NS, k = e - NS * c;
        const int p1 = clp[c + 1];
        int p = clp[c];
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            x[q][r] = ld_sc1(rb + (size_t)max(min(p, p1 - 1), 0) * 12 + off + k);  // (an empty first cluster: 0)
            if (p < p1) p = (p / kCgpRows + 1) * kCgpRows;
        }
    }
#pragma unroll
    for (int q = 0; q < EPT; ++q) {
        const int e0 = t + q * kCgpThreads, e = min(e0, ne - 1), c = e / NS, k = e - NS * c;
        const int p1 = clp[c + 1];
        int p = clp[c];
        double v = 0.0;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
            if (p < p1) {
                v += x[q][r];
                p = (p / kCgpRows + 1) * kCgpRows;
            }
        }
        for (; p < p1; p = (p / kCgpRows + 1) * kCgpRows) v += ld_sc1(rb + (size_t)p * 12 + off + k);
        if (e0 < ne) rs[e0] = v;
    }
}

// NB: blocks per row held in registers (a multiple of 8).  wx: [2][C][8] the w exchange by iteration parity (a
// workgroup's P2 may run while another is still gathering in P1); yg: [m][2] the tagged granules of y, tag0 the tag of
// iteration 0 (tags never repeat on a handle); sync: kCgpSyncWords barrier words, epoch0: the barriers they have
// counted so far (one per iteration of earlier launches); oseg bit 0: also write this solve's coarse segments tl.Oseg
// (the E build behind the CG then skips k_tl_erow), bit 1 (tests, INSFM_DIAG=cgp_fault): the last workgroup leaves
// at iteration 2 as if a barrier had timed out, bit 2 (tests, INSFM_DIAG=adef2_breakdown): an A-DEF2 launch reports a
// breakdown (status 2) at iteration 2, bit 3: the restriction of r0 comes from k_tl_basis (tl.Rc) instead of
// k_cg_factor_basis's run records;
// dcout (non-null): the camera step dc = L^-T x~ written at the end (k_cg_finish's arithmetic);
// trace (diagnostics, normally null): gamma, delta, rho, done of the first 64 iterations, then wall-clock ticks (100 MHz)
// of the launch start, the setup's end and each iteration's start, then per iteration the ticks around its two grid
// barriers (workgroup 0).
constexpr int kCgpPadSlot = INT_MIN;  // ssrc of a pad slot (a zero block)

template <int NB, bool DET, bool ADEF = false>
__global__ __launch_bounds__(kCgpThreads, 1) void k_tl_cgp(int C, const int* __restrict__ nbr_ptr,
                                                          const int* __restrict__ nbr_j, const double* __restrict__ S,
                                                          const int* __restrict__ ssrc, const double* __restrict__ Li,
                                                          const double* __restrict__ Lf, CgBufs cg, TlBufs tl,
                                                          const double* __restrict__ Einv, int maxit, double tol2_rel,
                                                          double* wx, unsigned long long* yg, unsigned tag0,
                                                          unsigned* sync, unsigned epoch0, int oseg, double* runs,
                                                          double* trace, double* __restrict__ dcout, long long* stp) {
    static_assert(NB % 8 == 0, "k_tl_cgp gathers eight blocks per load instruction");
    const StampScope stamp_(stp);
    constexpr int D = 8, MC = 9, BS = D * MC, LPL = (kCoarseMax + 63) / 64, LNC = (kCoarseMax / MC + 63) / 64;
    constexpr int NG = NB / 8;                          // gather loads per wave and iteration
    constexpr int RPT = (kCoarseMax + kCgpThreads - 1) / kCgpThreads;  // coarse entries per thread (LDS fills)
    // B_ic = sum_{j in c} S_ij G_j of the row's segments, a-major (A_ic = S~_i,c Z~_c = L_i^-1 B_ic)
    // (segment stride BS + 1: P2's lanes (a, j) read row a of segments j, j + 8, ... -- an odd stride keeps the 8
    // segments of a row on distinct banks)
    __shared__ double Aseg[kCgpRows][kCgpSegMax][BS + 1];
    __shared__ double wg[kCgpWaves][NB][D];            // the neighbours' w of the wave's blocks (gathered per iteration)
    // the restriction R of the iteration; DET: the 12 cluster sums (gamma, delta, rho partials, R) of every cluster
    __shared__ double rs[DET ? 12 * kCgpMaxClusters : kCoarseMax];
    __shared__ double ys[kCoarseMax];                  // y of the iteration
    __shared__ double Lrow[kCgpRows][D * D];           // L_i (row a, column k)
    __shared__ double Lirow[kCgpRows][D * D];          // L_i^-1 (row a, column k)
    __shared__ double Zrow[kCgpRows][BS];              // Z~_i (row a, column k)
    __shared__ double Grow[kCgpRows][BS];              // G_i, the unscaled basis (row a, column k)
    __shared__ double vec[kCgpRows][8][D];             // the row's r u w z q s p x
    __shared__ int jn[kCgpWaves][NB];                  // neighbour of each register block
    __shared__ int segc[kCgpRows][kCgpSegMax];         // neighbour cluster of each segment
    __shared__ int clp[kCgpMaxClusters + 1];          // the clusters' cluster-ordered position ranges
    __shared__ double prt[kCgpRows][12];               // each row's partials: r.u, w.u, ||L r||^2, Z~_i^T w (9)
    __shared__ int pcl[kCgpRows];                      // each row's cluster (-1: no row)
    __shared__ int bflag;
    __shared__ double dvec[kCgpRows][D];               // ADEF: each row's d = -(off-diagonal part of S~ v)
    const int t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6);  // (wave-uniform: the row's values live in SGPRs)
    const int a8 = lane >> 3, b8 = lane & 7;           // block entry (a, b) of this lane
    const int rl = wv;                                 // local row
    // the workgroup's rows are consecutive in cluster order (tl.cl_cams), so its rows mostly share one cluster and
    // their CG partials are summed in LDS before the cluster's atomics
    const int pos = blockIdx.x * kCgpRows + rl;
    const bool has_row = pos < C;
    const int row = has_row ? tl.cl_cams[pos] : 0;
    const int m = tl.m, nc = tl.nc;
    const int gw = blockIdx.x * kCgpWaves + wv;        // this wave's coarse row of E^-1 (if gw < m)
    const int n0 = has_row ? nbr_ptr[row] : 0;
    const int len = has_row ? nbr_ptr[row + 1] - n0 : 0;
    const int nk = min(len, NB);                       // blocks of the row (the host checks len <= NB)
    const int s0 = has_row ? tl.rseg_ptr[row] : 0, nseg = has_row ? tl.rseg_ptr[row + 1] - s0 : 0;
    const long long t_start = wall_clock64();
    double* V = &vec[rl][0][0];
    enum { VR = 0, VU = 8, VW = 16, VZ = 24, VQ = 32, VS = 40, VP = 48, VX = 56 };
    // The block-Jacobi scaling on the vector side, lane (a, b) = (a8, b8) holding one entry of the 8 x 8 factor
    // L_i^-1 (li_ba = L_i^-1[b][a], li_ab = L_i^-1[a][b], set once per solve below):
    //   lscale: acc = sum of row a of an unscaled product (the value lane (a, *) holds after the butterfly over b) ->
    //           (L_i^-1 sum)[b] = sum_{a <= b} L_i^-1[b][a] sum_a, by a butterfly over a (lane stride 8, 16, 32);
    //   ltscale: x = the row's vector entry of lane a8 -> (L_i^-T x)[b] = sum_{a >= b} L_i^-1[a][b] x_a, the same way.
    // Either way every lane ends with the entry of index b8 = lane & 7 (the lanes < 8 store it).
    double li_ba = 0.0, li_ab = 0.0;
    auto bfly8 = [&](double v) {
        v += __shfl_xor(v, 8, 64);
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        return v;
    };
    auto lscale = [&](double acc) { return bfly8(a8 <= b8 ? li_ba * acc : 0.0); };
    auto ltscale = [&](double xa) { return bfly8(a8 >= b8 ? li_ab * xa : 0.0); };
    // ---- setup ----
    // The operator is held UNSCALED (round 5): slot k of the row keeps S_ij (j = its neighbour) from the upper block
    // pattern of S -- block ssrc >= 0 as stored, or block ~ssrc transposed for a lower neighbour -- and the block-Jacobi
    // scaling S~_ij = L_i^-1 S_ij L_j^-T is applied to the vectors instead: every row publishes v_j = L_j^-T w_j and
    // forms S~ w = L_i^-1 (sum_j S_ij v_j).  So no k_cg_scale launch and no 61-MB Sn copy in front of the CG (the
    // first solve of an LM run, whose own coarse matrix k_tl_erow builds from Sn, still has them).
    // The row's blocks (slots past the row: zero, neighbour = the row itself, so the products need no guard).
    for (int k = lane; k < NB; k += 64) jn[wv][k] = k < nk ? nbr_j[n0 + k] : (has_row ? row : 0);
    // the slots' S blocks, slot k in lane k & 63 of sqa (k < 64) / sqb; read back per slot by readlane (no memory
    // round trip between a slot's index and its block load)
    const int sqa = lane < nk ? ssrc[n0 + lane] : kCgpPadSlot;
    const int sqb = (NB > 64 && lane + 64 < nk) ? ssrc[n0 + 64 + lane] : kCgpPadSlot;
    const int lt = b8 * D + a8;  // this lane's entry of a transposed block
    auto slot_val = [&](int k) {  // entry (a8, b8) of S_ij for register slot k (branch-free: one load per slot)
        const int q = __builtin_amdgcn_readlane(k < 64 ? sqa : sqb, k & 63);
        const bool pad = q == kCgpPadSlot;
        const int e = pad ? 0 : (q >= 0 ? q : ~q);
        const double v = S[(size_t)e * (D * D) + (q >= 0 ? lane : lt)];
        return pad ? 0.0 : v;
    };
    double sreg[NB];
#pragma unroll
    for (int k = 0; k < NB; ++k) sreg[k] = slot_val(k);
    for (int e = t; e < kCgpRows * kCgpSegMax * (BS + 1); e += kCgpThreads) (&Aseg[0][0][0])[e] = 0.0;
    const size_t own = (size_t)(has_row ? row : 0) * D + (lane & 7);
    {
        if (lane < nseg && lane < kCgpSegMax) segc[rl][lane] = tl.seg[s0 + lane].x;
        for (int i = t; i <= nc; i += kCgpThreads) clp[i] = tl.cl_ptr[i];
        if (has_row) {
            Lrow[rl][lane] = Lf[(size_t)row * D * D + lane];
            Lirow[rl][lane] = Li[(size_t)row * D * D + lane];
            li_ab = Li[(size_t)row * D * D + lane];   // L_i^-1[a8][b8]
            li_ba = Li[(size_t)row * D * D + lt];     // L_i^-1[b8][a8]
            for (int e = lane; e < BS; e += 64) {
                Zrow[rl][e] = tl.Zt[(size_t)row * BS + e];
                Grow[rl][e] = tl.Gb[(size_t)row * BS + e];
            }
            const double* src = lane < 8 ? cg.r[0] : lane < 16 ? tl.u : lane < 24 ? cg.w[0] : lane < 32 ? cg.w[1]
                              : lane < 40 ? cg.r[1] : lane < 48 ? cg.s[0] : lane < 56 ? cg.p : cg.x;
            V[lane] = src[own];
        }
    }
    __syncthreads();
    if (trace && blockIdx.x == 0 && t == 0) trace[578] = (double)wall_clock64();  // (blocks issued, LDS tables in)
    // B_ic = sum_{j in c} S_ij G_j (A_ic = S~_i,c Z~_c = L_i^-1 B_ic, since Z~_j = L_j^T G_j, G_j the unscaled basis):
    // lane (a, b) sums S_ij[a][b] G_j[b][q] over the segment's blocks (segment boundaries are wave-uniform); at the
    // segment's end the eight b lanes are summed by a fixed butterfly and lane (a, 0) writes row a of B_ic (one wave
    // per row: each segment is written once, in a fixed order).  L_i^-1 is applied per iteration together with the
    // row's S~ w (P2), and Z~_i^T A_ic = G_i^T B_ic for the coarse segments.  The G_j rows of ZC blocks at a time are
    // staged in the wave's gather buffer by coalesced loads (all in flight together), then read back per lane.
    if (nk > 0) {
        constexpr int ZC = NB * D / BS;            // blocks per staging chunk (14 for NB = 128)
        constexpr int ZU = (ZC * BS + 63) / 64;    // coalesced loads per lane and chunk
        double* zs = &wg[wv][0][0];
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
                    double v = za[q];
                    v += __shfl_xor(v, 1, 64);
                    v += __shfl_xor(v, 2, 64);
                    v += __shfl_xor(v, 4, 64);
                    if (b8 == 0) Aseg[rl][cur][a8 * MC + q] = v;
                    za[q] = 0.0;
                }
            }
            ++cur;
            send = cur < nseg ? tl.seg[s0 + cur].z : 1 << 30;
        };
        // (the blocks are re-read from memory here -- L2 / MALL-hot behind the register loads above: a loop over the
        // register copies would have to be unrolled over all NB blocks, too large with the segment flushes)
        for (int k0 = 0; k0 < nk; k0 += ZC) {
            double zl[ZU], sv[ZC];
#pragma unroll
            for (int u = 0; u < ZU; ++u) {
                const int e = min(lane + 64 * u, ZC * BS - 1), c = e / BS;
                zl[u] = tl.Gb[(size_t)jn[wv][min(k0 + c, NB - 1)] * BS + (e - c * BS)];
            }
#pragma unroll
            for (int c = 0; c < ZC; ++c) sv[c] = slot_val(min(k0 + c, nk - 1));
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int u = 0; u < ZU; ++u)
                if (lane + 64 * u < ZC * BS) zs[lane + 64 * u] = zl[u];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // two blocks' Z~ rows read ahead of their products (see P2)
#pragma unroll
            for (int c = 0; c < ZC; c += 2) {
                const int c1 = min(c + 1, ZC - 1);
                const double* zr0 = zs + c * BS + b8 * MC;
                const double* zr1 = zs + c1 * BS + b8 * MC;
                double z0[MC], z1[MC];
#pragma unroll
                for (int q = 0; q < MC; ++q) { z0[q] = zr0[q]; z1[q] = zr1[q]; }
                __builtin_amdgcn_sched_barrier(0);
                const int kk = k0 + c;
                if (kk >= nk) break;
                while (kk >= send) flush();
#pragma unroll
                for (int q = 0; q < MC; ++q) za[q] += sv[c] * z0[q];
                if (c + 1 >= ZC || kk + 1 >= nk) break;
                while (kk + 1 >= send) flush();
#pragma unroll
                for (int q = 0; q < MC; ++q) za[q] += sv[c1] * z1[q];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        flush();
    }
    const int ci = has_row ? tl.clab[row] : 0;
    if (lane == 0) pcl[rl] = has_row ? ci : -1;
    const bool use = tl.ok[0] != 0;
    // R(r0) into rs: the cluster sums of k_cg_factor_basis's run partials (parity-1 run records, slots 3..11, summed in
    // run order), or with oseg bit 3 k_tl_basis's per-cluster sums tl.Rc (the separate launches; FACTOR_BASIS=0)
    auto r0_restriction = [&]() {
        if (oseg & 8) {
            for (int q = t; q < m; q += kCgpThreads) rs[q] = tl.Rc[q];
        } else {
            det_cluster_sums<MC>(runs + (size_t)gridDim.x * kCgpRows * 12, 3, clp, nc, rs);
        }
    };
    const double* erow = Einv + (size_t)min(gw, m - 1) * m;  // this wave's coarse row of E^-1 (read from L2)
    double h_alpha = 1.0, h_gam = 1.0, h_bb = 1.0;
    unsigned epoch = epoch0;
    bool alive = true;
    int it = 0;
    __syncthreads();  // Aseg complete
    if (trace && blockIdx.x == 0 && t == 0) trace[579] = (double)wall_clock64();  // (A_ic complete)
    // the coarse matrix's row segments of this solve for the E build that runs behind the CG (k_tl_erow's outputs:
    // Z~_i^T A_ic, plus Z~_i^T Z~_i on the own-cluster segment, in k_tl_erow's order of additions)
    if ((oseg & 1) && has_row) {
        const int ns = min(nseg, kCgpSegMax);
        for (int sg = 0; sg < ns; ++sg) {
            const int own_seg = tl.seg[s0 + sg].w;
            for (int o = lane; o < MC * MC; o += 64) {
                const int k = o / MC, l = o % MC;
                double v = 0.0;
                if (own_seg) {
#pragma unroll
                    for (int a = 0; a < D; ++a) v += Zrow[rl][a * MC + k] * Zrow[rl][a * MC + l];
                }
#pragma unroll
                for (int a = 0; a < D; ++a) v += Grow[rl][a * MC + k] * Aseg[rl][sg][a * MC + l];  // Z~_i^T A = G_i^T B
                tl.Oseg[(size_t)(s0 + sg) * MC * MC + o] = v;
            }
        }
    }
    if constexpr (ADEF) {
        // ---- A-DEF2 setup (precond 2; oracle/ba_oracle.c adef2_apply): x0 = Z~ E^-1 R(r0) and r0' = r0 - S~ x0 without
        // an exchange (S~ Z~ = A is this row's B segments scaled by L_i^-1); then d0 = -(the off-diagonal part of
        // S~ r0') from the neighbours' r0' (one exchange), its restriction summed per cluster (atomic buffer 2), y0' =
        // E^-1 R(d0), u0 = r0' + Z~ y0' and w0 = S~ u0 = r0' + off(S~ r0') + Z~ y0' + A y0' again without an exchange.
        // Three grid barriers; the coarse solves under the setup tags tag0 + maxit + 1 and + 2.
        // DET (deterministic mode, every rank of a replicated multi-rank CG): the cluster sums of the restrictions and
        // of the scalar partials come from the run records (det_cluster_sums) instead of atomics -- d0's restriction in
        // slots 3..11 of the parity-1 records (next written by iteration 1, behind three more barriers), iteration 0's
        // scalars in slots 0..2 of parity 0.
        if constexpr (!DET) {
            for (int q = blockIdx.x * kCgpThreads + t; q < 3 * m + 2 * 3 * nc; q += gridDim.x * kCgpThreads)
                st_sc1(q < 3 * m ? tl.Racc + q : tl.Gacc + (q - 3 * m), 0.0);
        }
        if (blockIdx.x == 0 && t == 0) {
            cg.status[2] = use ? 1 : 0;  // reported as insfm_ba_stats.coarse_used
            if (cg.prog) __hip_atomic_store(cg.prog + 3, use ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        // coarse rows of y = E^-1 R (R in rs, LDS) published under `tag`, then collected by every workgroup into ys
        // (the E^-1 row loaded here each time: held across the setup's products it pushed the kernel into spills)
        auto coarse_solve = [&](unsigned tag) -> bool {
            if (gw < m) {
                double ev[LPL];
#pragma unroll
                for (int q = 0; q < LPL; ++q) ev[q] = erow[min(lane + 64 * q, m - 1)];
                double rq[LPL];
#pragma unroll
                for (int q = 0; q < LPL; ++q) rq[q] = rs[min(lane + 64 * q, m - 1)];
                __builtin_amdgcn_sched_barrier(0);
                double sy = 0.0;
#pragma unroll
                for (int q = 0; q < LPL; ++q)
                    if (lane + 64 * q < m) sy += ev[q] * rq[q];
                const double y = wave_sum(sy);
                if (lane == 0) put_y(yg, gw, tag, y);
            }
            for (int g = gw + gridDim.x * kCgpWaves; g < m; g += gridDim.x * kCgpWaves) {
                const double* er = Einv + (size_t)g * m;
                double sy = 0.0;
                for (int l = lane; l < m; l += 64) sy += er[l] * rs[l];
                const double y = wave_sum(sy);
                if (lane == 0) put_y(yg, g, tag, y);
            }
            return get_y(yg, ys, m, tag, sync);
        };
        // row a8's sum over the segments of B_ic y_c (lane (a, j): segments j, j + 8, ...), then over j
        auto seg_ay = [&]() -> double {
            double ay = 0.0;
            const int ns = min(nseg, kCgpSegMax);
            for (int sg = b8; sg < ns; sg += 8) {
                const double* yc = ys + segc[rl][sg] * MC;
                const double* A = &Aseg[rl][sg][a8 * MC];
                double a9[MC], c9[MC];
#pragma unroll
                for (int k = 0; k < MC; ++k) { a9[k] = A[k]; c9[k] = yc[k]; }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < MC; ++k) ay += a9[k] * c9[k];
            }
            ay += __shfl_xor(ay, 1, 64);
            ay += __shfl_xor(ay, 2, 64);
            ay += __shfl_xor(ay, 4, 64);
            return ay;
        };
        auto zy_entry = [&](int la) -> double {  // (Z~_i y_ci)[la]
            double z9[MC], y9[MC];
#pragma unroll
            for (int k = 0; k < MC; ++k) { z9[k] = Zrow[rl][la * MC + k]; y9[k] = ys[ci * MC + k]; }
            __builtin_amdgcn_sched_barrier(0);
            double sz = 0.0;
#pragma unroll
            for (int k = 0; k < MC; ++k) sz += z9[k] * y9[k];
            return sz;
        };
        const unsigned tag_s = tag0 + (unsigned)maxit + 1u, tag_s2 = tag0 + (unsigned)maxit + 2u;
        const int la = lane & 7;
        // x0, r0' (R(r0): k_cg_factor_basis's run partials, summed per cluster in run order)
        if (use) {
            r0_restriction();
            __syncthreads();
            if (!coarse_solve(tag_s)) alive = false;
        }
        if (alive && has_row) {
            double x0 = 0.0, sx = 0.0;
            if (use) {
                x0 = zy_entry(la);
                sx = lscale(seg_ay());  // entry la of off(S~) x0 = L_i^-1 sum_c B_ic y0_c
            }
            const double r0 = V[VR + la];
            const double r0p = r0 - x0 - sx;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // (r0 itself parked in z, zeroed below: the stopping rule's reference ||L r0||^2 = ||b||^2 comes from it)
            if (lane < D) { V[VR + la] = r0p; V[VX + la] = x0; V[VZ + la] = r0; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double v0 = ltscale(V[VR + a8]);  // the neighbours read L_i^-T r0'
            if (lane < D) st_sc1(wx + (size_t)C * D + (size_t)row * D + lane, v0);
        }
        if (alive) alive = cgp_barrier(sync, ++epoch, &bflag);
        // d0 = -off(S~ r0') and its restriction
        double off0 = 0.0;
        if (alive) {
            double uv8[NG];
            {
                int jr[NG];
#pragma unroll
                for (int g = 0; g < NG; ++g) jr[g] = jn[wv][8 * g + a8];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int g = 0; g < NG; ++g) uv8[g] = ld_sc1(wx + (size_t)C * D + (size_t)jr[g] * D + b8);
            }
#pragma unroll
            for (int g = 0; g < NG; ++g) wg[wv][8 * g + a8][b8] = uv8[g];
            __syncthreads();
            if (has_row) {
                double ac4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int k0 = 0; k0 < NB; k0 += 16) {
                    double w16[16];
#pragma unroll
                    for (int c = 0; c < 16; ++c) w16[c] = wg[wv][k0 + c][b8];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int c = 0; c < 16; ++c) ac4[c & 3] += sreg[k0 + c] * w16[c];
                    __builtin_amdgcn_sched_barrier(0);
                }
                double acc = (ac4[0] + ac4[1]) + (ac4[2] + ac4[3]);
                acc += __shfl_xor(acc, 1, 64);
                acc += __shfl_xor(acc, 2, 64);
                acc += __shfl_xor(acc, 4, 64);
                off0 = lscale(acc);
                if (lane < D) dvec[rl][lane] = -off0;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < MC) {
                    double d8[D], z8[D];
#pragma unroll
                    for (int a = 0; a < D; ++a) { d8[a] = dvec[rl][a]; z8[a] = Zrow[rl][a * MC + lane]; }
                    __builtin_amdgcn_sched_barrier(0);
                    double rr = 0.0;
#pragma unroll
                    for (int a = 0; a < D; ++a) rr += z8[a] * d8[a];
                    prt[rl][3 + lane] = rr;
                }
            }
            __syncthreads();
            if (has_row && (rl == 0 || pcl[rl - 1] != ci) && lane >= 3 && lane < 3 + MC) {
                double v = prt[rl][lane];
                for (int r2 = rl + 1; r2 < kCgpRows && pcl[r2] == ci; ++r2) v += prt[r2][lane];
                if constexpr (DET) st_sc1(runs + (size_t)gridDim.x * kCgpRows * 12 + (size_t)pos * 12 + lane, v);
                else unsafeAtomicAdd(tl.Racc + (size_t)2 * m + (size_t)ci * MC + (lane - 3), v);
            }
            alive = cgp_barrier(sync, ++epoch, &bflag);
        }
        // u0, w0 and the partials of iteration 0
        if (alive) {
            if (use) {
                if constexpr (DET) {
                    det_cluster_sums<MC>(runs + (size_t)gridDim.x * kCgpRows * 12, 3, clp, nc, rs);
                } else {
                    double rv[RPT];
#pragma unroll
                    for (int q = 0; q < RPT; ++q) rv[q] = ld_sc1(tl.Racc + (size_t)2 * m + min(t + q * kCgpThreads, m - 1));
#pragma unroll
                    for (int q = 0; q < RPT; ++q)
                        if (t + q * kCgpThreads < m) rs[t + q * kCgpThreads] = rv[q];
                }
                __syncthreads();
                if (!coarse_solve(tag_s2)) alive = false;
            }
            if (alive && has_row) {
                double zy = 0.0, sa = 0.0;
                if (use) {
                    zy = zy_entry(la);
                    sa = lscale(seg_ay());
                }
                const double r0p = V[VR + la];
                const double u0 = r0p + zy;
                const double w0 = r0p + off0 + zy + sa;  // S~ u0 (the diagonal block of S~ is I)
                // the original r0 (parked in z above) for ||L r0||^2: iteration 0's rho, which the stopping rule keeps
                // as its reference -- ||b||^2, as in the oracle (bb2) and the additive form, not ||L r0'||^2
                double l8[D], r8[D];
#pragma unroll
                for (int k = 0; k < D; ++k) { l8[k] = Lrow[rl][la * D + k]; r8[k] = V[VZ + k]; }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < D) { V[VU + la] = u0; V[VW + la] = w0; V[VZ + la] = 0.0; V[VQ + la] = 0.0; }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                double g0 = 0.0, g1 = 0.0, g2 = 0.0;
                {
                    if (lane < D) {
                        g0 = r0p * u0;
                        g1 = w0 * u0;
                        double lr = 0.0;
#pragma unroll
                        for (int k = 0; k < D; ++k)
                            if (k <= lane) lr += l8[k] * r8[k];
                        g2 = lr * lr;
                    }
                    const double v0 = ltscale(V[VW + a8]);  // the neighbours read L_i^-T w0
                    if (lane < D) st_sc1(wx + (size_t)row * D + lane, v0);
                }
                wave_sum3(g0, g1, g2);
                if (lane == 0) { prt[rl][0] = g0; prt[rl][1] = g1; prt[rl][2] = g2; }
            }
            if constexpr (DET) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (w0 before the runs' partials)
            __syncthreads();
            if (has_row && (rl == 0 || pcl[rl - 1] != ci) && lane < 3) {
                double v = prt[rl][lane];
                for (int r2 = rl + 1; r2 < kCgpRows && pcl[r2] == ci; ++r2) v += prt[r2][lane];
                if constexpr (DET) st_sc1(runs + (size_t)pos * 12 + lane, v);  // (parity 0: iteration 0's scalars)
                else unsafeAtomicAdd(tl.Gacc + (size_t)lane * nc + ci, v);
            }
            alive = cgp_barrier(sync, ++epoch, &bflag);
        }
    } else {
    // ---- u0 = M~^-1 r0 (round 5: k_tl_pc's setup launch folded in; config 3 saved its 10-us launch and the gap
    // in front of it).  The restriction R(r0): every workgroup sums k_tl_basis's row partials of each cluster itself,
    // rows in cluster order (k_tl_pc's order, so the same doubles); the wave's own cluster's rows of y0 = E^-1 R
    // (k_tl_pc's products and butterfly); u0_i = r0_i + Z~_i y0_ci.  u0 goes to the neighbours through the w exchange
    // buffer of parity 1 (next written by P2 of iteration 0, two grid barriers later) behind one grid barrier, in
    // front of which the per-cluster atomic buffers 0 and 1 are cleared (the setup's partials go to buffer 0, P2 of
    // iteration 0 adds into buffer 1) and workgroup 0 reports whether the coarse correction is on.
    {
        if (!DET) {
            for (int q = blockIdx.x * kCgpThreads + t; q < 2 * (m + 3 * nc); q += gridDim.x * kCgpThreads)
                st_sc1(q < 2 * m ? tl.Racc + q : tl.Gacc + (q - 2 * m), 0.0);
        }
        if (blockIdx.x == 0 && t == 0) {
            cg.status[2] = use ? 1 : 0;  // reported as insfm_ba_stats.coarse_used
            if (cg.prog) __hip_atomic_store(cg.prog + 3, use ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        // R(r0) = the cluster sums of k_cg_factor_basis's run partials (parity-1 run records, slots 3..11, summed in
        // run order: det_cluster_sums); wave gw forms coarse row gw of y0 = E^-1 R (k_tl_pc's products and butterfly)
        // and publishes it as tagged granules like an iteration's y, under the setup's own tag (tag0 + maxit + 1:
        // never an iteration's); every workgroup polls all of y0
        const unsigned tag_s = tag0 + (unsigned)maxit + 1u;
        if (use) {
            double ev[LPL];
            if (gw < m) {
#pragma unroll
                for (int q = 0; q < LPL; ++q) ev[q] = erow[min(lane + 64 * q, m - 1)];
            }
            r0_restriction();
            __syncthreads();
            if (gw < m) {
                double rq[LPL];
#pragma unroll
                for (int q = 0; q < LPL; ++q) rq[q] = rs[min(lane + 64 * q, m - 1)];
                __builtin_amdgcn_sched_barrier(0);
                double sy = 0.0;
#pragma unroll
                for (int q = 0; q < LPL; ++q)
                    if (lane + 64 * q < m) sy += ev[q] * rq[q];
                const double y = wave_sum(sy);
                if (lane == 0) put_y(yg, gw, tag_s, y);
            }
            for (int g = gw + gridDim.x * kCgpWaves; g < m; g += gridDim.x * kCgpWaves) {
                const double* er = Einv + (size_t)g * m;
                double sy = 0.0;
                for (int l = lane; l < m; l += 64) sy += er[l] * rs[l];
                const double y = wave_sum(sy);
                if (lane == 0) put_y(yg, g, tag_s, y);
            }
            if (!get_y(yg, ys, m, tag_s, sync)) alive = false;
        }
        if (alive && has_row) {
            const int la = lane & 7;
            double v = V[VR + la];
            if (use) {
                double z9[MC], y9[MC];
#pragma unroll
                for (int k = 0; k < MC; ++k) { z9[k] = Zrow[rl][la * MC + k]; y9[k] = ys[ci * MC + k]; }
                __builtin_amdgcn_sched_barrier(0);
                double sz = 0.0;
#pragma unroll
                for (int k = 0; k < MC; ++k) sz += z9[k] * y9[k];
                v += sz;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < D) V[VU + la] = v;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const double v0 = ltscale(V[VU + a8]);  // the neighbours read L_i^-T u0
            if (lane < D) st_sc1(wx + (size_t)C * D + (size_t)row * D + lane, v0);
        }
        if (alive) alive = cgp_barrier(sync, ++epoch, &bflag);
    }
    // ---- iteration 0's operator product (k_tl_pspmv's setup, folded in): w0 = u0 + S~ u0, z0 = q0 = 0; w0 into the
    // exchange buffer of parity 0 and the partials of iteration 0 (r0.u0, w0.u0, ||L r0||^2, Z~^T w0) published like
    // P2's (atomic buffer 0 / runs tagged with iteration 0)
    if (alive) {
        double uv8[NG];
        {
            int jr[NG];
#pragma unroll
            for (int g = 0; g < NG; ++g) jr[g] = jn[wv][8 * g + a8];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int g = 0; g < NG; ++g) uv8[g] = ld_sc1(wx + (size_t)C * D + (size_t)jr[g] * D + b8);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) wg[wv][8 * g + a8][b8] = uv8[g];
        __syncthreads();
        if (has_row) {
            double ac4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k0 = 0; k0 < NB; k0 += 16) {
                double w16[16];
#pragma unroll
                for (int c = 0; c < 16; ++c) w16[c] = wg[wv][k0 + c][b8];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < 16; ++c) ac4[c & 3] += sreg[k0 + c] * w16[c];
                __builtin_amdgcn_sched_barrier(0);
            }
            double acc = (ac4[0] + ac4[1]) + (ac4[2] + ac4[3]);
            acc += __shfl_xor(acc, 1, 64);
            acc += __shfl_xor(acc, 2, 64);
            acc += __shfl_xor(acc, 4, 64);
            const double su = lscale(acc);  // (S~ u0)_i = L_i^-1 sum_j S_ij v0_j
            const int la = lane & 7;
            const double u_ = V[VU + la], r_ = V[VR + la];
            const double w0 = u_ + su;  // (the diagonal block of S~ is I)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < D) { V[VW + la] = w0; V[VZ + la] = 0.0; V[VQ + la] = 0.0; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            double g0 = 0.0, g1 = 0.0, g2 = 0.0, rr = 0.0;
            {
                const int lc = min(lane, MC - 1);
                double l8[D], r8[D], z8[D], w8[D];
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    l8[k] = Lrow[rl][la * D + k];
                    r8[k] = V[VR + k];
                    z8[k] = Zrow[rl][k * MC + lc];
                    w8[k] = V[VW + k];
                }
                __builtin_amdgcn_sched_barrier(0);
                if (lane < D) {
                    g0 = r_ * u_;
                    g1 = w0 * u_;
                    double lr = 0.0;
#pragma unroll
                    for (int k = 0; k < D; ++k)
                        if (k <= lane) lr += l8[k] * r8[k];
                    g2 = lr * lr;
                }
                if (lane < MC) {
#pragma unroll
                    for (int a = 0; a < D; ++a) rr += z8[a] * w8[a];
                }
                const double v0 = ltscale(V[VW + a8]);  // the neighbours read L_i^-T w0
                if (lane < D) st_sc1(wx + (size_t)row * D + lane, v0);
            }
            wave_sum3(g0, g1, g2);
            if (lane == 0) { prt[rl][0] = g0; prt[rl][1] = g1; prt[rl][2] = g2; }
            if (lane < MC) prt[rl][3 + lane] = rr;
        }
        if constexpr (DET) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (w0 before the runs' partials)
        __syncthreads();
        if (has_row && (rl == 0 || pcl[rl - 1] != ci) && lane < 3 + MC) {
            double v = prt[rl][lane];
            for (int r2 = rl + 1; r2 < kCgpRows && pcl[r2] == ci; ++r2) v += prt[r2][lane];
            if constexpr (DET) {
                st_sc1(runs + (size_t)pos * 12 + lane, v);  // (parity 0: iteration 0's run partials)
            } else {
                if (lane < 3) unsafeAtomicAdd(tl.Gacc + (size_t)lane * nc + ci, v);
                else unsafeAtomicAdd(tl.Racc + (size_t)ci * MC + (lane - 3), v);
            }
        }
        alive = cgp_barrier(sync, ++epoch, &bflag);
    }
    }  // (ADEF)
    if (trace && blockIdx.x == 0 && t == 0) {
        trace[256] = (double)t_start;
        trace[257] = (double)wall_clock64();
    }
    for (; alive; ++it) {
        if ((oseg & 2) && it == 2 && blockIdx.x == gridDim.x - 1) {  // (fault injection: see above)
            if (t == 0) __hip_atomic_store(cgp_abort(sync), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            alive = false;
            break;
        }
        if (trace && t == 0 && it == kCgpTraceIt && blockIdx.x < 256) trace[772 + blockIdx.x] = (double)wall_clock64();
        // ======== P1 ========
        // every load of the phase is issued before the first wait: the scalar partials, this wave's gathers (lane
        // (a, b) loads entry b of the w of block 8 g + a), the restriction (all threads, into LDS), the E^-1 row
        const int b0 = it % 3;  // partial sums of this iteration (P2 of it - 1 added them)
        double gl[3][LNC];
        if constexpr (DET) {
            // every workgroup sums each cluster's run partials of this iteration itself, in run order (the runs were
            // stored before the grid barrier that ended the previous iteration, in its parity buffer): the same doubles
            // in every workgroup, in a fixed order, no atomics (A-DEF2: the 3 scalars; the additive form: the scalars
            // and the restriction of w)
            constexpr int NS = ADEF ? 3 : 12;
            det_cluster_sums<NS>(runs + (size_t)(it & 1) * gridDim.x * kCgpRows * 12, 0, clp, nc, rs);
            __syncthreads();
#pragma unroll
            for (int q = 0; q < LNC; ++q) {
                const int c = min(lane + 64 * q, nc - 1);
                gl[0][q] = rs[c * NS]; gl[1][q] = rs[c * NS + 1]; gl[2][q] = rs[c * NS + 2];
            }
        } else {
            const double* G = tl.Gacc + (size_t)b0 * 3 * nc;
#pragma unroll
            for (int q = 0; q < LNC; ++q) {
                const int l = min(lane + 64 * q, nc - 1);
                gl[0][q] = ld_sc1(G + l); gl[1][q] = ld_sc1(G + nc + l); gl[2][q] = ld_sc1(G + 2 * nc + l);
            }
        }
        const double* wsrc = wx + (size_t)(it & 1) * C * D + b8;
        double wv8[NG];
        {
            int jr[NG];  // (the neighbour indices read from LDS as one batch, then every gather issued)
#pragma unroll
            for (int g = 0; g < NG; ++g) jr[g] = jn[wv][8 * g + a8];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int g = 0; g < NG; ++g) wv8[g] = ld_sc1(wsrc + (size_t)jr[g] * D);
        }
        const double* Rv = DET ? nullptr : tl.Racc + (size_t)b0 * m;  // (DET: no atomic buffers)
        double rv[RPT];
#pragma unroll
        for (int q = 0; q < RPT; ++q) rv[q] = (use && !DET && !ADEF) ? ld_sc1(Rv + min(t + q * kCgpThreads, m - 1)) : 0.0;
        double ev[LPL];
        if (!ADEF && use && gw < m) {  // (A-DEF2: loaded with the restriction after the mid-phase barrier)
#pragma unroll
            for (int q = 0; q < LPL; ++q) ev[q] = erow[min(lane + 64 * q, m - 1)];
        }
        double ga0 = 0.0, ga1 = 0.0, ga2 = 0.0;
#pragma unroll
        for (int q = 0; q < LNC; ++q)
            if (lane + 64 * q < nc) { ga0 += gl[0][q]; ga1 += gl[1][q]; ga2 += gl[2][q]; }
        wave_sum3(ga0, ga1, ga2);
        const double gam = uni(ga0), del = uni(ga1), rho = uni(ga2);
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[582 + 3 * it] = (double)wall_clock64();
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
            if (ADEF && (oseg & 4) && it == 2) done = 2;  // (INSFM_DIAG=adef2_breakdown: a breakdown, for the tests)
        }
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) {  // INSFM_DIAG=cgp_trace
            trace[4 * it] = gam; trace[4 * it + 1] = del; trace[4 * it + 2] = rho; trace[4 * it + 3] = done;
            trace[258 + it] = (double)wall_clock64();
        }
        // the status for the host (the progress word only every 8th iteration: it serves the host's stall deadline,
        // and a store to host memory holds the storing wave's next vmcnt(0) for a PCIe round trip)
        if (blockIdx.x == 0 && t == 0) {
            if (done) {
                cg.status[1] = it;
                cg.status[0] = done;
            }
            if (cg.prog) {
                if (done) {
                    __hip_atomic_store(cg.prog + 2, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(cg.prog + 1, done, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                } else if ((it & 7) == 0) {
                    __hip_atomic_store(cg.prog + 0, it + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
        if (done) break;
        if (it == 0) h_bb = bb;
        h_alpha = alpha;
        h_gam = gam;
        // the partial buffers of iteration it + 2 (last read in P1 of it - 1, before the barrier ending P2 of it - 1;
        // first added to in P2 of it + 1, behind the barrier ending this P2) are cleared now
        if (!DET) {  // (spread over the workgroups: at most one store per thread)
            double* Rn = tl.Racc + (size_t)((it + 2) % 3) * m;
            double* Gn = tl.Gacc + (size_t)((it + 2) % 3) * 3 * nc;
            for (int q = blockIdx.x * kCgpThreads + t; q < m + 3 * nc; q += gridDim.x * kCgpThreads)
                st_sc1(q < m ? Rn + q : Gn + (q - m), 0.0);
        }
#pragma unroll
        for (int g = 0; g < NG; ++g) wg[wv][8 * g + a8][b8] = wv8[g];
        if (use && !DET && !ADEF) {
#pragma unroll
            for (int q = 0; q < RPT; ++q)
                if (t + q * kCgpThreads < m) rs[t + q * kCgpThreads] = rv[q];
        }
        __syncthreads();
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[580 + 3 * it] = (double)wall_clock64();
        // coarse row gw: y = E^-1 R (k_tl_pc_cl's products and butterfly; A-DEF2: after the restriction below)
        if (!ADEF && use && gw < m) {
            double rq[LPL];
#pragma unroll
            for (int q = 0; q < LPL; ++q) {  // (DET: entry k of R is record k / 9's value 3 + k % 9)
                const int k = min(lane + 64 * q, m - 1);
                rq[q] = rs[DET ? (k / 9) * 12 + 3 + k % 9 : k];
            }
            __builtin_amdgcn_sched_barrier(0);
            double sy = 0.0;
#pragma unroll
            for (int q = 0; q < LPL; ++q)
                if (lane + 64 * q < m) sy += ev[q] * rq[q];
            const double y = wave_sum(sy);
            if (lane == 0) put_y(yg, gw, tag0 + (unsigned)it, y);
        }
        // more coarse rows than waves (small grids): the rest, E^-1 rows loaded here
        for (int g = gw + gridDim.x * kCgpWaves; !ADEF && use && g < m; g += gridDim.x * kCgpWaves) {
            const double* er = Einv + (size_t)g * m;
            double sy = 0.0;
            for (int l = lane; l < m; l += 64) sy += er[l] * rs[DET ? (l / 9) * 12 + 3 + l % 9 : l];
            const double y = wave_sum(sy);
            if (lane == 0) put_y(yg, g, tag0 + (unsigned)it, y);
        }
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[581 + 3 * it] = (double)wall_clock64();
        // the row's S~ w (lane a < 8 ends with entry a)
        double sw = 0.0;
        if (has_row) {
            // the gathered w read back 16 blocks at a time, all reads in flight before their products (one read
            // per block waited on its own left the LDS latency in series: 2.5 us per iteration)
            double ac4[4] = {0.0, 0.0, 0.0, 0.0};  // four independent chains
#pragma unroll
            for (int k0 = 0; k0 < NB; k0 += 16) {
                double w16[16];
#pragma unroll
                for (int c = 0; c < 16; ++c) w16[c] = wg[wv][k0 + c][b8];
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int c = 0; c < 16; ++c) ac4[c & 3] += sreg[k0 + c] * w16[c];
                __builtin_amdgcn_sched_barrier(0);
            }
            double acc = (ac4[0] + ac4[1]) + (ac4[2] + ac4[3]);
            acc += __shfl_xor(acc, 1, 64);
            acc += __shfl_xor(acc, 2, 64);
            acc += __shfl_xor(acc, 4, 64);
            sw = acc;  // row a8's sum_j S_ij v_j, unscaled (L_i^-1 is applied with the coarse part in P2)
        }
        if constexpr (ADEF) {
            // A-DEF2: y = E^-1 Z~^T d, d = w - S~ w = -L_i^-1 sum_j S_ij v_j: the row's restriction of d, summed per
            // cluster run and added to atomic buffer `b0`, one grid barrier, then the coarse rows of y
            if (has_row) {
                const double dneg = lscale(sw);
                if (lane < D) dvec[rl][lane] = -dneg;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if (lane < MC) {
                    double d8[D], z8[D];
#pragma unroll
                    for (int a = 0; a < D; ++a) { d8[a] = dvec[rl][a]; z8[a] = Zrow[rl][a * MC + lane]; }
                    __builtin_amdgcn_sched_barrier(0);
                    double rr = 0.0;
#pragma unroll
                    for (int a = 0; a < D; ++a) rr += z8[a] * d8[a];
                    prt[rl][3 + lane] = rr;
                }
            }
            __syncthreads();
            // (DET: slots 3..11 of this iteration's parity records; their last readers, iteration it - 2's, passed
            // two grid barriers ago, and P1's readers of slots 0..2 of the same records do not touch them)
            if (has_row && (rl == 0 || pcl[rl - 1] != ci) && lane >= 3 && lane < 3 + MC) {
                double v = prt[rl][lane];
                for (int r2 = rl + 1; r2 < kCgpRows && pcl[r2] == ci; ++r2) v += prt[r2][lane];
                if constexpr (DET) st_sc1(runs + (size_t)(it & 1) * gridDim.x * kCgpRows * 12 + (size_t)pos * 12 + lane, v);
                else unsafeAtomicAdd(tl.Racc + (size_t)b0 * m + (size_t)ci * MC + (lane - 3), v);
            }
            if (!(alive = cgp_barrier(sync, ++epoch, &bflag))) break;
            if (use) {
                if (gw < m) {
#pragma unroll
                    for (int q = 0; q < LPL; ++q) ev[q] = erow[min(lane + 64 * q, m - 1)];
                }
                if constexpr (DET) {
                    det_cluster_sums<MC>(runs + (size_t)(it & 1) * gridDim.x * kCgpRows * 12, 3, clp, nc, rs);
                } else {
                    double rq0[RPT];
#pragma unroll
                    for (int q = 0; q < RPT; ++q) rq0[q] = ld_sc1(Rv + min(t + q * kCgpThreads, m - 1));
#pragma unroll
                    for (int q = 0; q < RPT; ++q)
                        if (t + q * kCgpThreads < m) rs[t + q * kCgpThreads] = rq0[q];
                }
                __syncthreads();
                if (gw < m) {
                    double rq[LPL];
#pragma unroll
                    for (int q = 0; q < LPL; ++q) rq[q] = rs[min(lane + 64 * q, m - 1)];
                    __builtin_amdgcn_sched_barrier(0);
                    double sy = 0.0;
#pragma unroll
                    for (int q = 0; q < LPL; ++q)
                        if (lane + 64 * q < m) sy += ev[q] * rq[q];
                    const double y = wave_sum(sy);
                    if (lane == 0) put_y(yg, gw, tag0 + (unsigned)it, y);
                }
                for (int g = gw + gridDim.x * kCgpWaves; g < m; g += gridDim.x * kCgpWaves) {
                    const double* er = Einv + (size_t)g * m;
                    double sy = 0.0;
                    for (int l = lane; l < m; l += 64) sy += er[l] * rs[l];
                    const double y = wave_sum(sy);
                    if (lane == 0) put_y(yg, g, tag0 + (unsigned)it, y);
                }
            }
        }
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[322 + 4 * it + 0] = (double)wall_clock64();
        // ======== P2 ========
        // y: every workgroup polls the tagged granules of all coarse rows until each carries this iteration's tag
        // (no grid barrier between the phases)
        if (use && !get_y(yg, ys, m, tag0 + (unsigned)it, sync)) {
            alive = false;
            break;
        }
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[322 + 4 * it + 1] = (double)wall_clock64();
        if (has_row) {
            const int la = lane & 7;
            const double w_ = V[VW + la];
            double mi = w_, ay = 0.0;
            if (use) {
                // (LDS operands read as a batch ahead of their products, here and below: under this kernel's register
                // pressure the compiler otherwise waits on each read before issuing the next)
                double z9[MC], y9[MC];
#pragma unroll
                for (int k = 0; k < MC; ++k) { z9[k] = Zrow[rl][la * MC + k]; y9[k] = ys[ci * MC + k]; }
                __builtin_amdgcn_sched_barrier(0);
                double sz = 0.0;
#pragma unroll
                for (int k = 0; k < MC; ++k) sz += z9[k] * y9[k];
                mi += sz;
                // lane (a, j) = (a8, b8): row a of B_ic y_c over the segments j, j + 8, ..., then summed over j -- the
                // layout of sw's row sums, so that L_i^-1 is applied once to both
                const int ns = min(nseg, kCgpSegMax);
                for (int sg = b8; sg < ns; sg += 8) {
                    const double* yc = ys + segc[rl][sg] * MC;
                    const double* A = &Aseg[rl][sg][a8 * MC];
                    double a9[MC], c9[MC];
#pragma unroll
                    for (int k = 0; k < MC; ++k) { a9[k] = A[k]; c9[k] = yc[k]; }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int k = 0; k < MC; ++k) ay += a9[k] * c9[k];
                }
                ay += __shfl_xor(ay, 1, 64);
                ay += __shfl_xor(ay, 2, 64);
                ay += __shfl_xor(ay, 4, 64);
            }
            // (S~ m)_i - m_i = L_i^-1 (sum_j S_ij v_j + sum_c B_ic y_c), entry la
            const double soff = lscale(sw + ay);
            const double vz = V[VZ + la], vq = V[VQ + la], vs = V[VS + la], vu = V[VU + la], vp = V[VP + la];
            const double vx = V[VX + la], vr = V[VR + la];
            __builtin_amdgcn_sched_barrier(0);
            const double prod = mi + soff;  // (the diagonal block of S~ is I)
            const double zn = prod + be * vz;
            const double qn = mi + be * vq;
            const double sn = w_ + be * vs;
            const double pn = vu + be * vp;
            const double xn = vx + alpha * pn;
            const double rn = vr - alpha * sn;
            const double un = vu - alpha * qn;
            const double wn = w_ - alpha * zn;
            // the row's new v = L_i^-T w for the neighbours first (w entry a8 from lane a8 by one permute, not
            // through LDS): its store overlaps the partials below
            const double vn = ltscale(__shfl(wn, a8, 64));
            if (lane < D) st_sc1(wx + (size_t)((it + 1) & 1) * C * D + (size_t)row * D + lane, vn);
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
            {
                const int lc = min(lane, MC - 1);
                double l8[D], r8[D], z8[D], w8[D];
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    l8[k] = Lrow[rl][la * D + k];
                    r8[k] = V[VR + k];
                    z8[k] = Zrow[rl][k * MC + lc];
                    w8[k] = V[VW + k];
                }
                __builtin_amdgcn_sched_barrier(0);
                if (lane < D) {
                    g0 = rn * un;
                    g1 = wn * un;
                    double lr = 0.0;
#pragma unroll
                    for (int k = 0; k < D; ++k)
                        if (k <= lane) lr += l8[k] * r8[k];
                    g2 = lr * lr;
                }
                if (!ADEF && lane < MC) {
#pragma unroll
                    for (int a = 0; a < D; ++a) rr += z8[a] * w8[a];
                }
            }
            wave_sum3(g0, g1, g2);
            if (lane == 0) { prt[rl][0] = g0; prt[rl][1] = g1; prt[rl][2] = g2; }
            if (!ADEF && lane < MC) prt[rl][3 + lane] = rr;
        }
        // DET: every wave's w stores complete before its run's partials are published (the consumers read w once they
        // hold every cluster's sums of the next iteration)
        if constexpr (DET) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the first row of each cluster run of the workgroup adds the run's partials (rows in order) to the cluster
        if (has_row && (rl == 0 || pcl[rl - 1] != ci) && lane < (ADEF ? 3 : 3 + MC)) {
            double v = prt[rl][lane];
            for (int r2 = rl + 1; r2 < kCgpRows && pcl[r2] == ci; ++r2) v += prt[r2][lane];
            if constexpr (DET) {
                // (at the run's head position, parity of iteration it + 1: every workgroup reads it after the barrier)
                st_sc1(runs + (size_t)((it + 1) & 1) * gridDim.x * kCgpRows * 12 + (size_t)pos * 12 + lane, v);
            } else {
                const int bsel = (it + 1) % 3;
                if (lane < 3) unsafeAtomicAdd(tl.Gacc + (size_t)bsel * 3 * nc + (size_t)lane * nc + ci, v);
                else unsafeAtomicAdd(tl.Racc + (size_t)bsel * m + (size_t)ci * MC + (lane - 3), v);
            }
        }
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[322 + 4 * it + 2] = (double)wall_clock64();
        if (trace && t == 0 && it == kCgpTraceIt && blockIdx.x < 256) trace[1028 + blockIdx.x] = (double)wall_clock64();
        if (!(alive = cgp_barrier(sync, ++epoch, &bflag))) break;
        if (trace && blockIdx.x == 0 && t == 0 && it < 64) trace[322 + 4 * it + 3] = (double)wall_clock64();
    }
    if (!alive && blockIdx.x == 0 && t == 0) {
        cg.status[1] = it;
        cg.status[0] = 4;
        if (cg.prog) {
            __hip_atomic_store(cg.prog + 2, it, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(cg.prog + 1, 4, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // the scaled solution for k_cg_finish, and the vectors as the launch path leaves them (not after an abort: the
    // host repeats the solve on the launch path from r0, which this kernel left untouched)
    if (has_row && alive) {
        double* dst = lane < 8 ? cg.r[0] : lane < 16 ? tl.u : lane < 24 ? cg.w[0] : lane < 32 ? cg.w[1]
                    : lane < 40 ? cg.r[1] : lane < 48 ? cg.s[0] : lane < 56 ? cg.p : cg.x;
        dst[own] = V[lane];
        // (round 5) the camera step dc_i = L_i^-T x~_i in k_cg_finish's order of additions, so that launch and its
        // gap are gone from the solve's tail
        if (dcout && lane < D) {
            double sdc = 0.0;
            for (int q = lane; q < D; ++q) sdc += Lirow[rl][q * D + lane] * V[VX + q];
            dcout[(size_t)row * D + lane] = sdc;
        }
    }
}

}  // namespace insfm
