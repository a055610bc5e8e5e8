// Schur complement for D <= 8 models with the camera-point blocks re-derived (as ba_schur_rc.h) and the D x D block
// sums accumulated in MFMA registers instead of LDS atomics.
//
// Why: a pair's block is rank 2 (W^_a W_q^T = J~c_a^T T_aq, T_aq = (A_a J~p_q^T) J~c_q, 2 x D), but adding it into an
// LDS row costs D^2 ds_add_f64 per pair: on config 3 that is 11M wave-instructions and kept the LDS pipe ~86 % busy
// (SQ_LDS_IDX_ACTIVE, profiles/r2_*), which bounded k_schur_rc at ~0.7 ms.  Here the pairs of a batch of own
// observations are staged in LDS GROUPED BY DESTINATION BLOCK (positions precomputed at create: the pattern is
// static), and each wave owns a quarter of the row's destination blocks as v_mfma_f64_4x4x4_4b_f64 accumulators:
// an 8 x 8 block is the 2 x 2 tiling of the instruction's four 4 x 4 blocks, and K = 4 = two pairs x two residual
// rows, so one MFMA adds two pairs' rank-2 updates with every lane holding one entry of the block.  LDS traffic per
// pair: 16 doubles written (T) and two operand reads per lane per MFMA, instead of 64 atomic adds.  The result is
// deterministic (fixed staging positions, fixed MFMA order, b summed in wave order).
//
// v_mfma_f64_4x4x4_4b_f64 layout (measured on gfx950, tools/mfma_layout_probe.hip): lane L, block g = (L >> 2) & 3,
// k = L >> 4:  A operand = A_g[L & 3][k],  B operand = B_g[k][L & 3],  C / D = C_g[L >> 4][L & 3].
// Tile g = (rt, ct) = (g >> 1, g & 1) of the 8 x 8 block: lane L accumulates entry (4 rt + (L >> 4), 4 ct + (L & 3)).
#pragma once
#include <hip/hip_runtime.h>

#include "ba_common.h"
#include "ba_device.h"
#include "ba_schur_rc.h"

#ifndef SCHUR_MF_PROBE
#define SCHUR_MF_PROBE 0  // timing-only variants (results wrong): 1 no consume phase, 2 no partner staging
#endif

namespace insfm {

constexpr int kMfOwn = 64;      // own observations per batch (16 per wave)
constexpr int kMfSlots = 64;    // destination blocks per work item (16 per wave)
constexpr int kMfSlotsW = 16;
constexpr int kMfOS = 17;       // LDS stride of an own observation's J~c (2 x 8 + 1 pad)
constexpr int kMfTS = 18;       // LDS stride of a staged pair's T (2 x 8 + 2 pad: 16-B stores land on distinct banks)
constexpr int kMfBR = kMfSlots + 3;  // per batch: slot offsets [0..64], first own descriptor, own count

// one work item: camera row i, upper blocks [kb, ke) (<= 64), batches [batch0, batch0 + nbatch) of rc_boff (each:
// kMfBR ints = its slot offsets, its first own descriptor in rc_sd and its own count <= 64)
struct MfWork {
    int i, kb, ke, nbatch, batch0, pad0, pad1, pad2;
};

template <int M>
inline size_t schur_mf_lds_bytes(int pcap, int C) {
    const size_t dbl = (size_t)pcap * kMfTS + (size_t)kMfOwn * kMfOS + (size_t)(kMfSlots + 1) * kCamTab<M> + 4 * 8;
    const size_t ints = (size_t)pcap + (kMfSlots + 1) + (size_t)C;
    return ((sizeof(double) * dbl + sizeof(int) * ints) + 15) & ~(size_t)15;
}

template <int M>
__global__ __launch_bounds__(256) void k_schur_mf(const MfWork* __restrict__ work, const int* __restrict__ row_ptr,
                                                  const int* __restrict__ col, int C, const int4* __restrict__ rc_sd,
                                                  const unsigned short* __restrict__ rc_ppos,
                                                  const int* __restrict__ rc_boff, int pcap,
                                                  const double2* __restrict__ obrec, const double* __restrict__ ptrec,
                                                  const double* __restrict__ cams, const double* __restrict__ U,
                                                  const double* __restrict__ gc, double f, double cmin, double cmax,
                                                  int add_diag, double* __restrict__ S, double* __restrict__ b) {
    constexpr int D = kD<M>, ST = kStride<M>, DD = D * D, CT = kCamTab<M>;
    static_assert(D <= 8, "the 2 x 2 tiling of 4 x 4 MFMA blocks covers D <= 8");
    extern __shared__ __attribute__((aligned(16))) double sh[];
    const MfWork wk = work[blockIdx.x];
    const int i = wk.i, kb = wk.kb, nb = wk.ke - wk.kb;
    double* tst = sh;                                   // [pcap][16] staged T, grouped by destination slot
    double* ost = tst + (size_t)pcap * kMfTS;           // [64][17] own J~c of the batch
    double* ctab = ost + kMfOwn * kMfOS;                // [(nb + 1)][CT]
    double* bpart = ctab + (size_t)(kMfSlots + 1) * CT; // [4 waves][D]  (D <= 8 -> 32 doubles)
    int* tidx = reinterpret_cast<int*>(bpart + 32);     // [pcap] own index (in the batch) of each staged pair
    int* boff = tidx + pcap;                            // [65] slot offsets of the current batch
    int* slot = boff + kMfSlots + 1;                    // [C]
    const int t = threadIdx.x, L = t & 63, w = t >> 6;
    for (int k = t; k < C; k += 256) slot[k] = -1;
    for (int e = t; e <= nb; e += 256) camtab_fill<M>(cams + (size_t)(e < nb ? col[kb + e] : i) * ST, ctab + (size_t)e * CT);
    __syncthreads();
    for (int e = kb + t; e < wk.ke; e += 256) slot[col[e]] = e - kb;
    const bool diag_chunk = (kb == row_ptr[i]);
    const double* own = ctab + (size_t)nb * CT;
    // this lane's own observation within a batch (16 per wave) and its share of the partners (u = sub, sub + 4, ...)
    const int oj = w * 16 + (L & 15), sub = L >> 4;
    // MFMA operand coordinates of this lane
    const int mp = L >> 5, mr = (L >> 4) & 1, mrt = (L >> 3) & 1, mct = (L >> 2) & 1, ml = L & 3;
    const int aofs = mr * 8 + 4 * mrt + ml, bofs = mr * 8 + 4 * mct + ml;
    double acc[kMfSlotsW + 1];  // [k] slot 1 + w + 4k, [kMfSlotsW] this wave's quarter of slot 0
#pragma unroll
    for (int k = 0; k <= kMfSlotsW; ++k) acc[k] = 0.0;
    double breg[D];
#pragma unroll
    for (int a = 0; a < D; ++a) breg[a] = 0.0;
    for (int bt = 0; bt < wk.nbatch; ++bt) {
        __syncthreads();  // the previous batch's stage has been consumed (and, first time, slot[] is ready)
        const int* brec = rc_boff + (size_t)(wk.batch0 + bt) * kMfBR;
        for (int s = t; s <= nb; s += 256) boff[s] = brec[s];
        const bool has = oj < brec[kMfSlots + 2];
        int4 sd = make_int4(0, 0, 0, 0);
        if (has) sd = rc_sd[brec[kMfSlots + 1] + oj];
        const int n = has ? (sd.z & 0xffff) : 0, ofs = sd.z >> 16;
        double X[3] = {0.0, 0.0, 1.0}, vi[6] = {1.0, 0.0, 0.0, 1.0, 0.0, 1.0}, yv[3] = {0.0, 0.0, 0.0}, sa = 0.0;
        if (has) {
            const double2* pr = reinterpret_cast<const double2*>(ptrec + 12 * (size_t)sd.x);
            const double2 p0 = pr[0], p1 = pr[1], p2 = pr[2], p3 = pr[3], p4 = pr[4], p5 = pr[5];
            vi[0] = p0.x; vi[1] = p0.y; vi[2] = p1.x; vi[3] = p1.y; vi[4] = p2.x; vi[5] = p2.y;
            yv[0] = p3.x; yv[1] = p3.y; yv[2] = p4.x;
            X[0] = p4.y; X[1] = p5.x; X[2] = p5.y;
            sa = obrec[sd.y + ofs].x;
        }
        // partner records of this lane's share, all in flight before the own Jacobian is evaluated
        constexpr int UPL = 3;  // partners per lane per batch (u = sub + 4 k); longer tracks loop below
        double psw[UPL];
        int pcam[UPL];
#pragma unroll
        for (int k = 0; k < UPL; ++k) {
            const int u = sub + 4 * k;
            pcam[k] = -1;
            psw[k] = 0.0;
            if (u < n) {
                const double2 r = obrec[sd.y + u];
                psw[k] = r.x;
                pcam[k] = (int)r.y;
            }
        }
        double Jc[2][D], Jp[2][3];
        eval_jac_tab<M>(own, X, sa, Jc, Jp);
        double A[2][3];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            A[r][0] = Jp[r][0] * vi[0] + Jp[r][1] * vi[1] + Jp[r][2] * vi[2];
            A[r][1] = Jp[r][0] * vi[1] + Jp[r][1] * vi[3] + Jp[r][2] * vi[4];
            A[r][2] = Jp[r][0] * vi[2] + Jp[r][1] * vi[4] + Jp[r][2] * vi[5];
        }
        if (sub == 0 && has) {
            if (diag_chunk) {  // b_i -= W_a y_p = J~c^T (J~p y)
                const double j0 = Jp[0][0] * yv[0] + Jp[0][1] * yv[1] + Jp[0][2] * yv[2];
                const double j1 = Jp[1][0] * yv[0] + Jp[1][1] * yv[1] + Jp[1][2] * yv[2];
#pragma unroll
                for (int a = 0; a < D; ++a) breg[a] -= Jc[0][a] * j0 + Jc[1][a] * j1;
            }
#pragma unroll
            for (int r = 0; r < 2; ++r) {
#pragma unroll
                for (int a = 0; a < 8; ++a) ost[oj * kMfOS + r * 8 + a] = a < D ? Jc[r][a] : 0.0;
            }
        }
        // stage T = (A J~p_q^T) J~c_q of every partner in this chunk at its precomputed (destination-sorted) position
        for (int k0 = 0; k0 < ((SCHUR_MF_PROBE & 2) ? 0 : n); k0 += 4 * UPL) {
#pragma unroll
            for (int k = 0; k < UPL; ++k) {
                const int u = k0 + sub + 4 * k;
                if (u >= n) continue;
                double swq;
                int cq;
                if (k0 == 0) {
                    swq = psw[k];
                    cq = pcam[k];
                } else {
                    const double2 r = obrec[sd.y + u];
                    swq = r.x;
                    cq = (int)r.y;
                }
                const int pos = rc_ppos[sd.w + u];
                if (pos == 0xffff) continue;  // partner camera outside this chunk
                const int sl = slot[cq];
                double Jcq[2][D], Jpq[2][3];
                eval_jac_tab<M>(ctab + (size_t)sl * CT, X, swq, Jcq, Jpq);
                double M2[2][2];
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
                        M2[r][s2] = A[r][0] * Jpq[s2][0] + A[r][1] * Jpq[s2][1] + A[r][2] * Jpq[s2][2];
                double2* dst = reinterpret_cast<double2*>(tst + (size_t)pos * kMfTS);
#pragma unroll
                for (int r = 0; r < 2; ++r)
#pragma unroll
                    for (int c2 = 0; c2 < 4; ++c2) {
                        const int c0 = 2 * c2, c1 = 2 * c2 + 1;
                        const double v0 = c0 < D ? M2[r][0] * Jcq[0][c0 < D ? c0 : 0] + M2[r][1] * Jcq[1][c0 < D ? c0 : 0] : 0.0;
                        const double v1 = c1 < D ? M2[r][0] * Jcq[0][c1 < D ? c1 : 0] + M2[r][1] * Jcq[1][c1 < D ? c1 : 0] : 0.0;
                        dst[r * 4 + c2] = make_double2(v0, v1);
                    }
                tidx[pos] = oj;
            }
        }
        __syncthreads();
        // consume, two staged pairs per MFMA.  Slot 0 (the diagonal block of a diagonal chunk: it also receives every
        // observation's pair with itself, ~10x the pairs of another block) is split into four quarters, one per wave,
        // each into its own accumulator (summed in wave order at the end); slots 1 + w + 4k belong to wave w.  Every
        // range is walked with wave-uniform bounds and branch-free loads (clamped addresses, masked operands); the
        // own index of the next step is loaded one step ahead.
        if (!(SCHUR_MF_PROBE & 1)) {
            const int b0 = __builtin_amdgcn_readfirstlane(boff[0]), e0 = __builtin_amdgcn_readfirstlane(boff[1]);
            const int q = ((e0 - b0 + 7) >> 3) << 1;  // quarter, rounded up to an even count
            const int lo0 = min(b0 + w * q, e0), hi0 = min(b0 + (w + 1) * q, e0);
            auto walk = [&](int lo, int hi, double& a) {
                if (lo >= hi) return;
                int pp = lo + mp;
                int oi = tidx[min(pp, hi - 1)];
                for (int p0 = lo; p0 < hi; p0 += 2) {
                    const bool ok = pp < hi;
                    const int ppc = ok ? pp : hi - 1;
                    const double av = ost[oi * kMfOS + aofs];
                    const double bv = tst[(size_t)ppc * kMfTS + bofs];
                    pp += 2;
                    oi = tidx[min(pp, hi - 1)];
                    a = __builtin_amdgcn_mfma_f64_4x4x4f64(ok ? av : 0.0, bv, a, 0, 0, 0);
                }
            };
            walk(lo0, hi0, acc[kMfSlotsW]);
#pragma unroll
            for (int k = 0; k < kMfSlotsW; ++k) {
                const int sidx = 1 + w + 4 * k;
                if (sidx < nb) walk(__builtin_amdgcn_readfirstlane(boff[sidx]), __builtin_amdgcn_readfirstlane(boff[sidx + 1]), acc[k]);
            }
        }
    }
    // b: fixed-order sums (butterfly per wave, then waves in order)
    if (diag_chunk) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const double s = wave_sum(breg[a]);
            if (L == 0) bpart[w * 8 + a] = s;
        }
    }
    __syncthreads();
    if (diag_chunk && t < D)
        b[(size_t)i * D + t] = (add_diag ? gc[(size_t)i * D + t] : 0.0) + ((bpart[t] + bpart[8 + t]) + bpart[16 + t]) + bpart[24 + t];
    // S blocks: lane L holds entry (4 rt + (L >> 4), 4 ct + (L & 3)) of tile g = (L >> 2) & 3 of each owned block
    const int g = (L >> 2) & 3;
    const int ea = 4 * (g >> 1) + (L >> 4), eb = 4 * (g & 1) + (L & 3);
    // slot 0: the four quarters in wave order (the staged T area is free now)
    tst[w * 64 + L] = acc[kMfSlotsW];
    __syncthreads();
    if (w == 0 && ea < D && eb < D) {
        double v = -(((tst[L] + tst[64 + L]) + tst[128 + L]) + tst[192 + L]);
        if (diag_chunk && add_diag) {
            double u = U[(size_t)i * DD + ea * D + eb];
            if (ea == eb) u = clampd(u, cmin, cmax) * f;
            v = u + v;
        }
        S[(size_t)kb * DD + ea * D + eb] = v;
    }
#pragma unroll
    for (int k = 0; k < kMfSlotsW; ++k) {
        const int s = 1 + w + 4 * k;
        if (s < nb && ea < D && eb < D) S[(size_t)(kb + s) * DD + ea * D + eb] = -acc[k];
    }
}

}  // namespace insfm
