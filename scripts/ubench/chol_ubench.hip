// Calibration micro-benchmark of the Cholesky kernels (not part of the product):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 chol_ubench.hip -o chol_ubench
// k_potrf128 alone on one 128x128 SPD block (timed, checked against a host Cholesky) and its
// shader-clock breakdown (k_potrf128<true>: stamps of wave 0's critical path); k_trsm128 on a tall
// panel; k_syrk_multi with one target / one source (the latency floor of a trailing-update launch).
#include "../../fish-eye_bundle_adjustment_amd/csrc/fba_chol.hip"

#include <cmath>
#include <cstdio>
#include <vector>

namespace fba { void set_error(const std::string&) {} }
using namespace fba;

// the barrier-synchronised potrf (A/B against the dataflow one)
__global__ __launch_bounds__(POTRF_THREADS) void k_potrf128_sync(double* S, int64_t ld, const int32_t* cols, double* dinv,
                                                                 double* scal) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    potrf_body_sync<false>(S, ld, cols[blockIdx.x], dinv, scal, nullptr, nullptr, smem);
}

// |L L' - A| / |A| over the 128x128 block and max |D_s L_ss - I| over the eight leaf inverses
static void check(const std::vector<double>& M, const std::vector<double>& L, const std::vector<double>& D, int64_t ld,
                  const char* name, float us) {
    const int n = 128;
    double err = 0.0, nrm = 0.0, derr = 0.0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            double v = 0;
            for (int k = 0; k <= j; ++k) v += L[i * ld + k] * L[j * ld + k];
            err = std::max(err, std::fabs(v - M[i * ld + j]));
            nrm = std::max(nrm, std::fabs(M[i * ld + j]));
        }
    for (int s = 0; s < 8; ++s)
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double v = 0;
                for (int k = 0; k < 16; ++k) v += D[s * 256 + i * 16 + k] * (k >= j ? L[(16 * s + k) * ld + 16 * s + j] : 0.0);
                derr = std::max(derr, std::fabs(v - (i == j ? 1.0 : 0.0)));
            }
    printf("%-20s %8.2f us  |LL'-A|/|A| %.2e  max|D L - I| %.2e\n", name, us, err / nrm, derr);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

template <class F>
static float time_us(F&& f, int reps) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        (void)hipEventRecord(a);
        f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = std::min(best, ms);
    }
    return 1e3f * best;
}

int main() {
    const int n = 128;
    const int64_t ld = 8192;
    const int64_t rows = 7808 + 128;  // 61 block rows + RHS block row
    std::vector<double> M((size_t)rows * ld, 0.0);
    unsigned s = 12345;
    auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0 / 16777216.0) - 0.5; };
    std::vector<double> B((size_t)n * n);
    for (auto& b : B) b = rnd();
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = 0;
            for (int k = 0; k < n; ++k) v += B[i * n + k] * B[j * n + k];
            M[i * ld + j] = v + (i == j ? n : 0);
        }
    for (int64_t i = n; i < rows; ++i)
        for (int j = 0; j < n; ++j) M[i * ld + j] = rnd();
    double *dS, *dinv, *scal;
    unsigned long long* dts;
    int32_t* dl;
    CK(hipMalloc(&dS, M.size() * 8));
    CK(hipMalloc(&dinv, 64 * 256 * 8));
    CK(hipMalloc(&scal, 64 * 8));
    CK(hipMalloc(&dts, 64 * 8));
    CK(hipMalloc(&dl, 4096 * 4));
    CK(hipMemset(scal, 0, 64 * 8));
    std::vector<int32_t> lists(4096, 0);
    // [0] = potrf column 0; [2..] = trsm records (0, 2 r + h), r = 1..61; [400] = syrk task
    // (1, 0, quarter 0, sources [0, 1), in place), [410] = source list {0}
    for (int q = 0; q < 122; ++q) { lists[2 + 2 * q] = 0; lists[3 + 2 * q] = 2 * (1 + q / 2) + (q & 1); }
    const int32_t task[6] = {1, 0, 0, 0, 1, -1};
    for (int q = 0; q < 6; ++q) lists[400 + q] = task[q];
    lists[410] = 0;
    CK(hipMemcpy(dl, lists.data(), lists.size() * 4, hipMemcpyHostToDevice));
    CK(hipFuncSetAttribute((const void*)k_potrf128<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)POTRF_LDS));
    CK(hipFuncSetAttribute((const void*)k_potrf128<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)POTRF_LDS));
    CK(hipFuncSetAttribute((const void*)k_trsm128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TRSM_LDS));
    auto reset = [&]() { return hipMemcpy(dS, M.data(), M.size() * 8, hipMemcpyHostToDevice); };
    CK(hipFuncSetAttribute((const void*)k_potrf128_sync, hipFuncAttributeMaxDynamicSharedMemorySize, (int)POTRF_LDS));
    std::vector<double> L((size_t)n * ld), D(8 * 256);
    for (int variant = 0; variant < 2; ++variant) {
        auto run = [&] {
            if (variant) k_potrf128_sync<<<1, POTRF_THREADS, POTRF_LDS>>>(dS, ld, dl, dinv, scal);
            else k_potrf128<false><<<1, POTRF_THREADS, POTRF_LDS>>>(dS, ld, dl, dinv, scal, nullptr);
        };
        CK(reset());
        const float tp = time_us(run, 20);
        CK(reset());  // check: factor the original block once
        CK(hipMemset(dinv, 0, 8 * 256 * 8));
        run();
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(L.data(), dS, L.size() * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(D.data(), dinv, D.size() * 8, hipMemcpyDeviceToHost));
        check(M, L, D, ld, variant ? "k_potrf128 (sync)" : "k_potrf128 (dataflow)", tp);
    }
    CK(reset());
    k_potrf128<true><<<1, POTRF_THREADS, POTRF_LDS>>>(dS, ld, dl, dinv, scal, dts);
    CK(hipDeviceSynchronize());
    CK(reset());
    const float tq = time_us([&] { k_potrf128<true><<<1, POTRF_THREADS, POTRF_LDS>>>(dS, ld, dl, dinv, scal, dts); }, 1);
    unsigned long long q[64];
    CK(hipMemcpy(q, dts, sizeof q, hipMemcpyDeviceToHost));
    printf("k_potrf128<TS>       %8.2f us, %llu clocks (wave 0) = %.2f GHz\n", tq, q[40] - q[0], (q[40] - q[0]) / (1e3 * tq));
    printf("  start->leaf0 %llu  leaf0 %llu  ->barrier %llu\n", q[1] - q[0], q[2] - q[1], q[3] - q[2]);
    unsigned long long tl = q[2] - q[1], tw = 0, tpd = 0, tb = 0, prev = q[3];
    for (int t = 0; t < 7; ++t) {
        const unsigned long long w = q[4 + 4 * t] - prev, pd = q[5 + 4 * t] - q[4 + 4 * t],
                                 lf = q[6 + 4 * t] - q[5 + 4 * t], bb = q[7 + 4 * t] - q[6 + 4 * t];
        prev = q[7 + 4 * t];
        tw += w; tpd += pd; tl += lf; tb += bb;
        printf("  s%d: wait %5llu  panel+diag %5llu  leaf %5llu  publish %5llu\n", t, w, pd, lf, bb);
    }
    printf("  totals: leaves %llu  waits %llu  panel+diag %llu  publish %llu  end %llu\n", tl, tw, tpd, tb, q[40] - q[31]);
    for (int t = 0; t < 6; ++t)  // bulk wave 1 (owner of the row-(s+2) unit), relative to wave 0's step starts
        printf("  bulk s%d: leaf seen %6lld  step s-1 all done %6lld  row s+2 out %6lld   (wave 0 step s+1 ready %6lld)\n", t,
               (long long)(q[41 + 3 * t] - q[3]), (long long)(q[42 + 3 * t] - q[3]), (long long)(q[43 + 3 * t] - q[3]),
               (long long)((t + 1 < 7 ? q[4 + 4 * (t + 1)] : q[40]) - q[3]));
    // trsm: 61 panel blocks below the factored block (two workgroups each)
    CK(reset());
    k_potrf128<false><<<1, POTRF_THREADS, POTRF_LDS>>>(dS, ld, dl, dinv, scal, nullptr);
    for (int nt : {1, 8, 61}) {
        const float tt = time_us([&] { k_trsm128<<<(unsigned)(2 * nt), 256, TRSM_LDS>>>(dS, ld, dl + 2, dinv); }, 10);
        printf("k_trsm128 %2d blocks  %8.2f us\n", nt, tt);
    }
    const float ts1 = time_us([&] { k_syrk_multi<<<1, 256>>>(dS, ld, dl + 400, dl + 410, nullptr, nullptr, nullptr); }, 10);
    printf("k_syrk_multi 1 quarter %7.2f us (K = 128)\n", ts1);
    const float te = time_us([&] { k_neg_copy<<<1, 64>>>(dinv, dinv + 64, 1); }, 20);
    printf("empty-ish launch      %8.2f us\n", te);
    return 0;
}
