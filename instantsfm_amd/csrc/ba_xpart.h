// Row-partitioned two-level CG across ranks (insfm_ba_cg_window / insfm_ba_cg_attach).
//
// The replicated multi-rank CG runs every iteration's S~ product on every rank.  Here rank r applies S~ to its own rows
// only -- the cluster-ordered positions [q_r, q_r+1) of the camera clusters, split at cluster boundaries -- and
// writes those rows' CG partials (w in cluster order, the three scalar partials, the restriction Z~_i^T w_i) straight
// into every rank's exchange window through peer mappings (IPC).  k_tl_pc stays replicated: it reads all rows'
// partials from its own window, so every rank computes the same recurrence scalars and coarse correction in the same
// order as the single-process deterministic path (bitwise the replicated CG's results).
//
// Ordering, per exchange (after each k_tl_pspmv): the rank's k_xsignal bumps its device exchange counter, makes its
// window writes visible system-wide (the kernel boundary behind k_tl_pspmv plus a system-scope release) and stores the
// counter into its flag word in every window; k_xwait then spins (bounded) until every rank's flag in its own window
// has reached its own counter.  Both skip once the CG status word is set, so all ranks perform the same exchanges.
// The window regions are double-buffered by iteration parity (k_tl_pspmv of iteration i writes region (i + 1) & 1,
// k_tl_pc of iteration i reads region i & 1): a rank one iteration ahead never overwrites what a peer still reads.
// The windows are uncached device memory (hipDeviceMallocUncached), so no cache holds a stale copy of a peer's write.
// After the CG, the solution rows are gathered the same way (slot 1) into the xg region.
#pragma once
#include "ba_common.h"

namespace insfm {

struct XPart {
    double* const* win = nullptr;   // [world] window bases (device array, own included); null: not partitioned
    int world = 0, q0 = 0;          // ranks; this rank's first cluster-ordered position
    long long off_vc = 0, off_gd = 0, off_rowR = 0;  // the region this launch writes (doubles from a window base)
};

// store v at offset `off` of every window (partitioned) or at `local` (not partitioned)
__device__ __forceinline__ void xstore(const XPart& xp, double* local, long long off, double v) {
    if (xp.win == nullptr) {
        *local = v;
        return;
    }
    for (int r = 0; r < xp.world; ++r) xp.win[r][off] = v;
}

constexpr int kXFlagStride = 32;          // unsigned words between flags (128 B)
constexpr unsigned kXSpinMax = 1u << 23;  // polls before k_xwait gives up

// flag of rank r, slot s (0 CG iterations, 1 solution gather) inside a window's flag block
__device__ __forceinline__ unsigned* xflag(unsigned* flags, int r, int s) { return flags + kXFlagStride * (2 * r + s); }

// pflags: [world] flag blocks of every window (device array); cnt: this rank's exchange counters [2]
__global__ __launch_bounds__(64) void k_xsignal(const int* __restrict__ status, unsigned* cnt, unsigned* const* pflags,
                                                int world, int rank, int slot) {
    if (threadIdx.x != 0) return;
    if (slot == 0 && status[0] != 0) return;
    const unsigned c = cnt[slot] + 1u;
    cnt[slot] = c;
    __threadfence_system();
    for (int r = 0; r < world; ++r)
        __hip_atomic_store(xflag(pflags[r], rank, slot), c, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// flags: this rank's own flag block; on timeout the CG status becomes 4 and the host-mapped progress word reports it
__global__ __launch_bounds__(64) void k_xwait(int* status, int* prog, const unsigned* cnt, unsigned* flags, int world,
                                              int slot) {
    if (threadIdx.x != 0) return;
    if (slot == 0 && status[0] != 0) return;
    const unsigned c = cnt[slot];
    for (int r = 0; r < world; ++r) {
        unsigned spins = 0;
        while (__hip_atomic_load(xflag(flags, r, slot), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < c) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins >= kXSpinMax) {
                status[1] = -1;
                status[0] = 4;
                if (prog) __hip_atomic_store(prog + 1, 4, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
        }
    }
    __threadfence_system();
}

// the solution rows of this rank (cluster-ordered positions [q0, q0 + n)) into the xg region of every window
__global__ __launch_bounds__(256) void k_xput_x(int n, int D, const int* __restrict__ cl_cams, const double* __restrict__ x,
                                                XPart xp, long long off_xg) {
    const int e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n * D) return;
    const int row = cl_cams[xp.q0 + e / D], a = e % D;
    const double v = x[(size_t)row * D + a];
    for (int r = 0; r < xp.world; ++r) xp.win[r][off_xg + (size_t)row * D + a] = v;
}

}  // namespace insfm
