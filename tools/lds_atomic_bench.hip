// Microbenchmark: LDS f64 accumulate / store patterns on gfx950 (CU-cycles per wave-instruction, 2.4 GHz assumed).
// Addresses are fixed per lane; the 16 operations of an iteration use immediate offsets (no address math).
//   mode 0: ds_add_f64, lane -> address lane (conflict-free, contiguous)
//   mode 1: ds_add_f64, 8 groups of 8 lanes, each group 8 contiguous doubles of its own block (stride 72)
//   mode 2: ds_add_f64, lane -> block (lane) of stride 65 (bank pair = lane mod 32: 2-way)
//   mode 3: ds_read_b64 + add + ds_write_b64 (non-atomic RMW), lane -> address lane
//   mode 4: ds_write_b64, lane -> address lane
//   mode 5: ds_write_b128 (two doubles per lane)
//   mode 6: ds_read_b64 only
//   mode 7: ds_add_f64, all lanes of a wave the same address
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k_bench(int iters, double* out) {
    __shared__ double acc[9216];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int k = t; k < 9216; k += 256) acc[k] = 0.0;
    __syncthreads();
    int a;
    if (MODE == 1) a = wv * 1152 + (lane >> 3) * 72 + (lane & 7);
    else if (MODE == 2) a = wv * 64 + lane * 65 % 4096;
    else if (MODE == 5) a = wv * 2048 + 2 * lane;
    else if (MODE == 7) a = wv * 8;
    else a = wv * 1024 + lane;
    double* p = acc + a;
    double v = 1.0 + t * 1e-3, fold = 0.0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            if (MODE == 3) { double x = p[r * 128 % 1024]; p[r * 128 % 1024] = x + v; }
            else if (MODE == 4) { p[r * 128 % 1024] = v; }
            else if (MODE == 5) { *reinterpret_cast<double2*>(p + (r * 128 % 1024)) = make_double2(v, v); }
            else if (MODE == 6) { fold += p[r * 128 % 1024]; }
            else atomicAdd(p + (MODE == 7 ? r : (r * 128 % 1024)) * (MODE == 1 ? 0 : 1) + (MODE == 1 ? r * 576 % 1152 * 0 : 0), v);
        }
        v += 1e-9;
    }
    __syncthreads();
    double sum = fold;
    for (int k = t; k < 9216; k += 256) sum += acc[k];
    if (sum == 12345.0) out[0] = sum;
}

template <int MODE>
void run(double* out, int wpc) {
    const int iters = 2000, blocks = 256 * wpc / 4;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    k_bench<MODE><<<blocks, 256>>>(10, out);
    (void)hipEventRecord(e0);
    k_bench<MODE><<<blocks, 256>>>(iters, out);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winstr = (double)blocks / 256 * 4 * iters * 16;  // LDS wave-instructions per CU
    printf("waves/CU %2d mode %d: %.3f ms, %.1f clk per wave-instr per CU\n", wpc, MODE, ms, ms * 1e6 / winstr * 2.4);
}

int main() {
    double* out;
    (void)hipMalloc(&out, 8);
    for (int wpc : {8, 16}) {
        run<0>(out, wpc); run<1>(out, wpc); run<2>(out, wpc); run<3>(out, wpc);
        run<4>(out, wpc); run<5>(out, wpc); run<6>(out, wpc); run<7>(out, wpc);
    }
    return 0;
}
