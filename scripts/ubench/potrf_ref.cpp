// Calibration only (not part of the product): rocSOLVER dpotrf time at the config-4 reduced size.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>
#include <cstdio>
#include <vector>
#include <random>
int main() {
    for (int n : {1280, 6144, 24576}) {
        std::vector<double> h((size_t)n * n);
        std::mt19937_64 g(1);
        std::uniform_real_distribution<double> u(-1, 1);
        for (auto& x : h) x = u(g) * 1e-3;
        for (int i = 0; i < n; ++i) h[(size_t)i * n + i] = n;
        double* d; int* info;
        if (hipMalloc(&d, h.size() * 8) || hipMalloc(&info, 4)) return 1;
        rocblas_handle hd; rocblas_create_handle(&hd);
        hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        float best = 1e30f;
        for (int rep = 0; rep < 4; ++rep) {
            (void)hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            rocsolver_dpotrf(hd, rocblas_fill_lower, n, d, n, info);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep) best = ms < best ? ms : best;
        }
        printf("rocsolver_dpotrf n=%d: %.3f ms  %.1f TFLOP/s\n", n, best, (double)n * n * n / 3 / best / 1e9);
        (void)hipFree(d); (void)hipFree(info); rocblas_destroy_handle(hd);
    }
}
