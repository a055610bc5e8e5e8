// Probe the operand / result layout of v_mfma_f64_4x4x4_4b_f64 on gfx950: A[lane] = 2^lane, B one-hot (lane s0):
// C[lane] = sum over the A lanes paired with B lane s0 that land on this output lane.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__global__ void k(double* out) {
    const int l = threadIdx.x;
    for (int s0 = 0; s0 < 64; ++s0) {
        const double a = ldexp(1.0, l);
        const double b = (l == s0) ? 1.0 : 0.0;
        double c = 0.0;
        c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
        out[s0 * 64 + l] = c;
    }
}

int main() {
    double* d;
    (void)hipMalloc(&d, 64 * 64 * 8);
    k<<<1, 64>>>(d);
    static double h[64 * 64];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    // for each B lane s0: list (output lane <- A lane)
    for (int s0 = 0; s0 < 64; ++s0) {
        printf("B%02d:", s0);
        for (int l = 0; l < 64; ++l)
            if (h[s0 * 64 + l] != 0.0) printf(" %d<-A%d", l, (int)std::log2(h[s0 * 64 + l]));
        printf("\n");
    }
    return 0;
}
