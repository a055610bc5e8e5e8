// Dense coarse-factorization harness (k_tl_chol / k_tl_dinv / k_tl_trinv / k_tl_gram): random SPD E of size m,
// checks ||E E^-1 - I||_max and reports per-kernel device time plus the Cholesky's per-phase clocks.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bench_dense.hip -o tools/bench_dense && tools/bench_dense 279
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../instantsfm_amd/csrc/ba_twolevel.h"

using namespace insfm;

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } \
    } while (0)

int main(int argc, char** argv) {
    const int m = argc > 1 ? std::atoi(argv[1]) : 279;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
    const bool verify_all = argc > 3 && std::atoi(argv[3]) != 0;
    int nbad = 0;
    if (m < 1 || m > kCoarseMax) { std::printf("m out of range\n"); return 2; }
    std::mt19937_64 rng(1);
    std::normal_distribution<double> nd;
    // E = B B^T + m I scaled by a wide diagonal (condition ~1e8, like the coarse matrix)
    std::vector<double> B((size_t)m * m), E((size_t)m * m, 0.0), sc(m);
    for (auto& v : B) v = nd(rng);
    for (int i = 0; i < m; ++i) sc[i] = std::pow(10.0, 4.0 * i / std::max(1, m - 1));
    for (int i = 0; i < m; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = 0.0;
            for (int k = 0; k < m; ++k) s += B[(size_t)i * m + k] * B[(size_t)j * m + k];
            if (i == j) s += 1e-3 * m;
            E[(size_t)i * m + j] = E[(size_t)j * m + i] = s * sc[i] * sc[j];
        }
    const int nB = (m + kNB - 1) / kNB;
    double *dE, *dA, *dDinv, *dLinv, *dEinv;
    int* dok;
    long long* dprof;
    CK(hipMalloc(&dE, sizeof(double) * m * m));
    CK(hipMalloc(&dA, sizeof(double) * m * m));
    CK(hipMalloc(&dDinv, sizeof(double) * nB * kNB * kNB));
    CK(hipMalloc(&dLinv, sizeof(double) * m * m));
    CK(hipMalloc(&dEinv, sizeof(double) * m * m));
    CK(hipMalloc(&dok, sizeof(int) * 4));
    CK(hipMalloc(&dprof, sizeof(long long) * 64));
    CK(hipMemset(dLinv, 0, sizeof(double) * m * m));
    CK(hipMemset(dprof, 0, sizeof(long long) * 64));
    CK(hipMemcpy(dE, E.data(), sizeof(double) * m * m, hipMemcpyHostToDevice));
    const size_t chol_lds = sizeof(double) * (size_t)m * kCPS;
    const size_t trinv_lds = sizeof(double) * ((size_t)m * kPS + (size_t)kNB * (m + 1));
    CK(hipFuncSetAttribute((const void*)k_tl_chol, hipFuncAttributeMaxDynamicSharedMemorySize, (int)chol_lds));
    CK(hipFuncSetAttribute((const void*)k_tl_trinv, hipFuncAttributeMaxDynamicSharedMemorySize, (int)trinv_lds));
    hipStream_t st = nullptr;
    if (argc > 4 && std::atoi(argv[4]) != 0) CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t ev[5];
    for (auto& e : ev) CK(hipEventCreate(&e));
    float tms[4] = {0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        CK(hipMemcpyAsync(dA, dE, sizeof(double) * m * m, hipMemcpyDeviceToDevice, st));
        CK(hipEventRecord(ev[0], st));
        k_tl_chol<<<1, 1024, chol_lds, st>>>(m, dA, dok, r == reps - 1 ? dprof : nullptr);
        CK(hipEventRecord(ev[1], st));
        k_tl_dinv<<<nB, 64, 0, st>>>(m, dA, dDinv, dok);
        CK(hipEventRecord(ev[2], st));
        k_tl_trinv<<<nB, 256, trinv_lds, st>>>(m, dA, dDinv, dLinv, dok);
        CK(hipEventRecord(ev[3], st));
        k_tl_gram<<<nB * nB, 256, 0, st>>>(m, dLinv, dEinv, dok);
        CK(hipEventRecord(ev[4], st));
        CK(hipEventSynchronize(ev[4]));
        if (verify_all) {
            int okr = 0;
            CK(hipMemcpy(&okr, dok, sizeof(int), hipMemcpyDeviceToHost));
            std::vector<double> Er((size_t)m * m);
            CK(hipMemcpy(Er.data(), dEinv, sizeof(double) * m * m, hipMemcpyDeviceToHost));
            double e2 = 0.0;
            for (int j = 0; j < m; j += std::max(1, m / 16))
                for (int i = 0; i < m; ++i) {
                    double s = 0.0;
                    for (int k = 0; k < m; ++k) s += E[(size_t)i * m + k] * Er[(size_t)k * m + j];
                    s -= (i == j) ? 1.0 : 0.0;
                    e2 = std::max(e2, std::fabs(s) * sc[j] / sc[i]);
                }
            if (!okr || !(e2 < 1e-6)) { ++nbad; std::printf("rep %d: ok=%d err=%.3e\n", r, okr, e2); }
        }
        if (r >= 2)
            for (int k = 0; k < 4; ++k) {
                float ms;
                CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
                tms[k] += ms;
            }
    }
    int ok = 0;
    CK(hipMemcpy(&ok, dok, sizeof(int), hipMemcpyDeviceToHost));
    std::vector<double> Ei((size_t)m * m);
    CK(hipMemcpy(Ei.data(), dEinv, sizeof(double) * m * m, hipMemcpyDeviceToHost));
    // scaled residual: D^-1 (E Einv - I) D with D = diag(sc) removes the diagonal scaling
    double err = 0.0;
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < m; ++j) {
            double s = 0.0;
            for (int k = 0; k < m; ++k) s += E[(size_t)i * m + k] * Ei[(size_t)k * m + j];
            s -= (i == j) ? 1.0 : 0.0;
            err = std::max(err, std::fabs(s) * sc[j] / sc[i]);
        }
    std::vector<long long> pf(64);
    CK(hipMemcpy(pf.data(), dprof, sizeof(long long) * 64, hipMemcpyDeviceToHost));
    const int n = reps - 2;
    std::printf("m=%d ok=%d max|D^-1(E Einv - I)D|=%.3e  us: chol %.1f dinv %.1f trinv %.1f gram %.1f\n", m, ok, err,
                1e3 * tms[0] / n, 1e3 * tms[1] / n, 1e3 * tms[2] / n, 1e3 * tms[3] / n);
    long long prev = pf[63];
    long long tot[3] = {0, 0, 0};
    const int nsteps = std::min(20, (m + kCB - 1) / kCB);
    for (int b = 0; b < nsteps; ++b)
        for (int p = 0; p < 3; ++p) {
            tot[p] += pf[3 * b + p] - prev;
            prev = pf[3 * b + p];
        }
    std::printf("chol clocks (first %d block steps): diag %lld panel %lld trailing %lld\n", nsteps, tot[0], tot[1], tot[2]);
    if (verify_all) std::printf("verified %d reps: %d bad\n", reps, nbad);
    return (ok && err < 1e-6 && nbad == 0) ? 0 : 1;
}
