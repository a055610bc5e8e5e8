// Shared definitions of the BA kernels (ba_kernels.hip, ba_twolevel.h, tools/bench_dense.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace insfm {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// three wave_sums with their butterfly steps interleaved: the same additions in the same order per value (bitwise
// wave_sum's results), one cross-lane latency per step instead of three
__device__ __forceinline__ void wave_sum3(double& a, double& b, double& c) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double ta = __shfl_xor(a, off, 64), tb = __shfl_xor(b, off, 64), tc = __shfl_xor(c, off, 64);
        a += ta;
        b += tb;
        c += tc;
    }
}


struct CgBufs {
    double* r[2];
    double* w[2];
    double* s[2];
    double* p;
    double* x;
    double* part[2];  // [nwg][3]: gamma, delta, rho
    double* hist;     // [maxit + 2][2]: alpha_i, gamma_i ; hist_bb at the end
    double* scal;     // [4]: alpha, beta, flag of the current recurrence step (written by k_cg_dots)
    int* status;      // [0] 0 running / 1 converged / 2 breakdown ; [1] iterations
    int* prog;        // host-mapped (two-level path): [0] iterations started, [1] status, [2] iterations, [3] coarse
                      // used, [4] sequence of the last k_cg_gate that saw its status (CG-stream path)
};


constexpr int kCgThreads = 512;
constexpr int kCgWaves = kCgThreads / 64;

template <int D>
struct CgGeom {
    static constexpr int DP = D + (D & 1);     // padded row length
    static constexpr int HP = DP / 2;          // 16-byte pieces per block row
    static constexpr int PPB = D * HP;         // pieces per block
    static constexpr int BPW = PPB <= 64 ? 64 / PPB : 1;          // blocks per wave per round
    static constexpr int PPL = PPB <= 64 ? 1 : (PPB + 63) / 64;   // pieces per lane
    static constexpr int BPR = BPW * kCgWaves;                    // blocks per round per workgroup
};

// INSFM_DIAG=stamps: tracer-free timestamps of selected main-queue kernels (wall_clock64, 100 MHz, one clock for the
// whole device).  p[0] = the entry of workgroup 0, p[1] = the latest end of the last kStampTail workgroups' thread 0
// (no-return atomic max; workgroups are dispatched in index order, so the last to finish is among the last
// dispatched; an atomic from every workgroup of a 16k-workgroup grid tripled its duration); p null: off (the default,
// no code path change).
constexpr unsigned kStampTail = 1024;
struct StampScope {
    unsigned long long* p;
    __device__ explicit StampScope(long long* q) : p(reinterpret_cast<unsigned long long*>(q)) {
        if (p && blockIdx.x == 0 && threadIdx.x == 0) p[0] = (unsigned long long)wall_clock64();
    }
    __device__ ~StampScope() {
        if (p && threadIdx.x == 0 && blockIdx.x + kStampTail >= gridDim.x)
            atomicMax(p + 1, (unsigned long long)wall_clock64());
    }
};
constexpr int kStampSteps = 1024;  // ring of LM steps
enum StampKind {
    kStLinPoints = 0, kStSchur = 1, kStCgp = 2, kStCgFinish = 3, kStPublish = 4,  // (round 5, first set)
    kStFactor = 5, kStBasis = 6, kStBacksub = 7, kStCost = 8, kStFinal = 9, kStKinds = 10
};

}  // namespace insfm
