// Cross-stream event ordering check: main writes X (slow kernel), side waits on an event and copies X -> Y, main waits
// on a second event and verifies Y.  Counts violations over many rounds.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_write(double* x, int n, double v, int spin) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    double acc = v;
    for (int k = 0; k < spin; ++k) acc = acc * 1.0000001 - 1e-7 * acc;   // keep the kernel busy
    if (i < n) x[i] = v + (acc - acc);
}
__global__ void k_copy(const double* x, double* y, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = x[i];
}
__global__ void k_check(const double* y, int n, double v, int* bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && y[i] != v) atomicAdd(bad, 1);
}
int main(int argc, char** argv) {
    const int n = 1 << 16, rounds = 400;
    const bool nonblocking = argc > 1 && argv[1][0] == 'n';
    double *x, *y;
    int* bad;
    hipMalloc(&x, n * 8); hipMalloc(&y, n * 8); hipMalloc(&bad, 4); hipMemset(bad, 0, 4);
    hipStream_t main_s, side;
    hipStreamCreateWithFlags(&main_s, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&side, nonblocking ? hipStreamNonBlocking : hipStreamDefault);
    hipEvent_t e1, e2;
    hipEventCreateWithFlags(&e1, hipEventDisableTiming);
    hipEventCreateWithFlags(&e2, hipEventDisableTiming);
    for (int r = 0; r < rounds; ++r) {
        k_write<<<n / 256, 256, 0, main_s>>>(x, n, (double)r, 2000);
        hipEventRecord(e1, main_s);
        hipStreamWaitEvent(side, e1, 0);
        k_copy<<<n / 256, 256, 0, side>>>(x, y, n);
        hipEventRecord(e2, side);
        hipStreamWaitEvent(main_s, e2, 0);
        k_check<<<n / 256, 256, 0, main_s>>>(y, n, (double)r, bad);
    }
    hipStreamSynchronize(main_s);
    int h = 0;
    hipMemcpy(&h, bad, 4, hipMemcpyDeviceToHost);
    std::printf("side %s: %d bad elements over %d rounds\n", nonblocking ? "non-blocking" : "blocking", h, rounds);
    return h != 0;
}
