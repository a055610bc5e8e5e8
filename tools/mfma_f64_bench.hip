// Throughput of the f64 MFMA forms on gfx950: back-to-back, 8 independent accumulators per wave, one wave per SIMD
// (and 2 per SIMD); reports cycles per instruction per SIMD at 2.4 GHz and TFLOP/s for the chip.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k4(int iters, double* out) {
    double a = 1.0 + threadIdx.x * 1e-6, b = 1.0 - threadIdx.x * 1e-6;
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += c[k];
    if (s == 1234.5) out[0] = s;
}

__global__ __launch_bounds__(256) void k16(int iters, double* out) {
    double a = 1.0 + threadIdx.x * 1e-6, b = 1.0 - threadIdx.x * 1e-6;
    v4d c[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 4; ++k) c[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[k], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += c[k][0] + c[k][1] + c[k][2] + c[k][3];
    if (s == 1234.5) out[0] = s;
}

__global__ __launch_bounds__(256) void kfma(int iters, double* out) {
    double a = 1.0 + threadIdx.x * 1e-6, b = 1.0 - threadIdx.x * 1e-6;
    double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) c[k] = fma(a, b, c[k]);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += c[k];
    if (s == 1234.5) out[0] = s;
}

int main() {
    double* out;
    (void)hipMalloc(&out, 8);
    const int iters = 20000;
    for (int wps : {1, 2}) {
        const int blocks = 256 * wps;  // 256-thread WGs: 4 waves = one per SIMD per WG
        for (int kind = 0; kind < 3; ++kind) {
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            auto launch = [&](int it) {
                if (kind == 0) k4<<<blocks, 256>>>(it, out);
                else if (kind == 1) k16<<<blocks, 256>>>(it, out);
                else kfma<<<blocks, 256>>>(it, out);
            };
            launch(100);
            (void)hipEventRecord(e0);
            launch(iters);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const int per_it = kind == 1 ? 4 : 8;
            const double instr_per_simd = (double)wps * iters * per_it;  // per SIMD
            const double flops_per_instr = kind == 0 ? 512.0 : (kind == 1 ? 2048.0 : 128.0);
            const double total_flops = instr_per_simd * 1024 * flops_per_instr;
            printf("%s waves/SIMD %d: %.3f ms, %.1f cycles/instr/SIMD, %.1f TFLOP/s\n",
                   kind == 0 ? "mfma_f64_4x4x4_4b" : (kind == 1 ? "mfma_f64_16x16x4 " : "v_fma_f64        "), wps, ms,
                   ms * 1e-3 * 2.4e9 / instr_per_simd, total_flops / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
