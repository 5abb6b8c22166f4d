// Microbenchmark: v_mfma_f64_16x16x4_f64 throughput (one kernel, all CUs, registers only).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k(double* out, int iters, double a0) {
    dbl4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = dbl4{0, 0, 0, 0};
    double a = a0 + threadIdx.x * 1e-9, b = a0 * 0.5;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void kfma(double* out, int iters, double a0) {
    double x0 = a0, x1 = a0 * 2, x2 = a0 * 3, x3 = a0 * 4, b = 1.0000001, c = 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) { x0 = fma(x0, b, c); x1 = fma(x1, b, c); x2 = fma(x2, b, c); x3 = fma(x3, b, c); }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3;
}
int main() {
    double* d; hipMalloc(&d, 1 << 26);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int iters = 4000;
    for (int blocks : {256, 512, 1024, 2048}) {
        k<8><<<blocks, 256>>>(d, 10, 1.0); hipDeviceSynchronize();
        hipEventRecord(e0); k<8><<<blocks, 256>>>(d, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double flops = (double)blocks * 4 /*waves*/ * iters * 8 * 2.0 * 16 * 16 * 4;
        printf("mfma_f64_16x16x4  blocks %5d: %.2f ms  %.1f TFLOP/s\n", blocks, ms, flops / ms / 1e9);
    }
    for (int blocks : {1024, 4096}) {
        kfma<<<blocks, 256>>>(d, 10, 1.0); hipDeviceSynchronize();
        hipEventRecord(e0); kfma<<<blocks, 256>>>(d, iters, 1.0); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        double flops = (double)blocks * 256 * iters * 32 * 2.0;
        printf("v_fma_f64 VALU    blocks %5d: %.2f ms  %.1f TFLOP/s\n", blocks, ms, flops / ms / 1e9);
    }
    return 0;
}
