// Calibration micro-benchmark (not part of the product): issue cost of v_fmac_f64 with and without
// a row_newbcast DPP source, and of the leaf's dependent pivot chain, in shader clocks, one wave.
//   hipcc --offload-arch=gfx950 -O3 dpp_rate.hip -o dpp_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k_rate(double* out, long long* clk, int iters) {
    double a[16];
    const double s = 1.0 + threadIdx.x * 1e-9, m = 1e-12;
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = i;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (MODE == 0) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(m));
            else if (MODE == 1) asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a[i]) : "v"(s), "v"(m));
            else if (MODE == 2) asm volatile("v_mov_b64_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "=v"(a[i]) : "v"(a[(i + 1) & 15]));
            else if (MODE == 3) asm volatile("v_rsq_f64_e32 %0, %1" : "=v"(a[i]) : "v"(a[i]));
            else asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(s), "v"(m));  // dependent chain per i
        }
    }
    long long t1 = clock64();
    double acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc += a[i];
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) *clk = t1 - t0;
}

// a dependent chain: each op uses the previous result
template <int MODE>
__global__ void k_chain(double* out, long long* clk, int iters) {
    double v = 1.0 + threadIdx.x * 1e-9;
    const double m = 1e-12;
    long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (MODE == 0) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(v) : "v"(m));
            else if (MODE == 1) asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(v));
            else asm volatile("v_rsq_f64_e32 %0, %0" : "+v"(v));
        }
    }
    long long t1 = clock64();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) *clk = t1 - t0;
}

int main() {
    double* out; long long* clk;
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&clk, sizeof(long long));
    const int iters = 1000;
    auto run = [&](auto kern, const char* name) {
        kern<<<1, 64>>>(out, clk, iters);
        kern<<<1, 64>>>(out, clk, iters);
        long long c = 0;
        (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("%-34s %.2f clocks per instruction\n", name, (double)c / (iters * 16.0));
    };
    run(k_rate<0>, "v_fmac_f64 independent");
    run(k_rate<1>, "v_fmac_f64_dpp independent");
    run(k_rate<2>, "v_mov_b64_dpp independent");
    run(k_rate<3>, "v_rsq_f64 independent");
    run(k_rate<4>, "v_fma_f64 16 chains");
    run(k_chain<0>, "v_fma_f64 dependent");
    run(k_chain<1>, "s_nop1 + v_mov_b64_dpp dependent");
    run(k_chain<2>, "v_rsq_f64 dependent");
    return 0;
}
