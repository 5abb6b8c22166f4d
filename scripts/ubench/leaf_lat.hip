// Calibration micro-benchmark (not part of the product): shader clocks of one 16x16 leaf factor
// (potrf_body's critical chain) in one wave, variants of what rides along with the pivot chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 leaf_lat.hip -o leaf_lat
#include "../../fish-eye_bundle_adjustment_amd/csrc/fba_chol.hip"
#include <cstdio>

namespace fba { void set_error(const std::string&) {} }
using namespace fba;

// the pivot chain alone: per column broadcast -> rsq -> correction -> next column's first update
__device__ __forceinline__ bool leaf_chain_only(double (&a)[IB]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < IB; ++j) {
        const double d = bcl(a[j], j);
        ok &= d > 0.0;
        const double r = __builtin_amdgcn_rsq(d);
        const double ar = a[j] * r;
        const double t = d * r;
        const double e = __builtin_fma(t, r, -1.0);
        const double p = __builtin_fma(e, 0.375, -0.5);
        a[j] = __builtin_fma(ar * e, p, ar);
        if (j + 1 < IB) fmac_bcn_first(a[j + 1], a[j], a[j], j + 1);
    }
    return ok;
}


// the factor without the inverse's substitution
__device__ __forceinline__ bool leaf_factor_noinv_ub(double (&a)[IB]) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < IB; ++j) {
        const double d = bcl(a[j], j);
        ok &= d > 0.0;
        const double r = __builtin_amdgcn_rsq(d);
        const double ar = a[j] * r;
        const double t = d * r;
        const double e = __builtin_fma(t, r, -1.0);
        const double p = __builtin_fma(e, 0.375, -0.5);
        a[j] = __builtin_fma(ar * e, p, ar);
#pragma unroll
        for (int l = j + 1; l < IB; ++l) {
            if (l == j + 1) fmac_bcn_first(a[l], a[j], a[j], l);
            else fmac_bcn(a[l], a[j], a[j], l);
        }
    }
    return ok;
}

template <int MODE>
__global__ void k_leaf(const double* __restrict__ A, double* __restrict__ out, long long* clk, int reps) {
    const int lane = threadIdx.x & 63, lr = lane & 15;
    __shared__ double Lw[16 * 17], Dw[16 * 17], tags[16], junk[64], hammer[4096];
    if (threadIdx.x >= 64) {  // MODE >= 5: other waves keep the LDS busy meanwhile
        double v = 0.0;
        for (int it = 0; it < reps * 200; ++it) v += hammer[(threadIdx.x * 17 + it * 64) & 4095];
        out[threadIdx.x] = v;
        return;
    }
    double a0[IB];
#pragma unroll
    for (int c = 0; c < IB; ++c) a0[c] = A[lr * IB + c];
    double acc = 0.0;
    long long t0 = clock64();
    for (int it = 0; it < reps; ++it) {
        double a[IB], x[IB];
#pragma unroll
        for (int c = 0; c < IB; ++c) a[c] = a0[c] + acc * 1e-300;  // (a dependence on the last rep)
        bool ok;
        if (MODE == 0) ok = leaf_factor(a, x, lr);
        else if (MODE == 1) ok = leaf_factor_noinv_ub(a);
        else if (MODE == 2) ok = leaf_chain_only(a);
        else if (MODE == 3) ok = leaf_factor_noinv(a, [&](int j, double inv) {  // + the potrf's column stores
                Lw[lr * 17 + j] = a[j];
                asm volatile("" ::: "memory");
                *(lane == 0 ? &tags[j] : &junk[lane]) = inv;  // (no branch: an exec-mask region would split the block)
            });
        else if (MODE == 4) ok = leaf_factor(a, x, lr, [&](int j) { Lw[lr * 17 + j] = a[j]; Dw[j * 17 + lr] = x[j]; });
        else if (MODE == 5) ok = leaf_factor_noinv(a, [&](int j, double) { Lw[lr * 17 + j] = a[j]; });
        else if (MODE == 6) ok = leaf_factor_noinv(a, [&](int j, double inv) { *(lane == 0 ? &tags[j] : &junk[lane]) = inv; });
        else if (MODE == 7) ok = leaf_factor_noinv(a, [&](int j, double) { *(lane < 16 ? &Lw[lr * 17 + j] : &junk[lane]) = a[j]; });
        else ok = leaf_factor_noinv(a, [&](int j, double inv) {  // one store: row 0 the column, lane 16 the tag
                *(lane < 16 ? &Lw[lr * 17 + j] : lane == 16 ? &tags[j] : &junk[lane]) = lane == 16 ? inv : a[j];
            });
        acc += a[IB - 1] + ((MODE == 0 || MODE == 4) ? x[IB - 1] : 0.0) + (ok ? 0.0 : 1.0) + Lw[lr] + tags[0] + Dw[lr] + junk[lane];
    }
    long long t1 = clock64();
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) *clk = t1 - t0;
}

int main() {
    double hA[256];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) hA[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    double *dA, *out; long long* clk;
    (void)hipMalloc(&dA, sizeof(hA));
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&clk, sizeof(long long));
    (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    const int reps = 200;
    auto run = [&](auto kern, const char* name) {
        kern<<<1, 64>>>(dA, out, clk, reps);
        kern<<<1, 64>>>(dA, out, clk, reps);
        long long c = 0;
        (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("%-40s %8.0f clocks per leaf (%.0f per column)\n", name, (double)c / reps, (double)c / reps / 16);
    };
    run(k_leaf<0>, "factor + inverse (leaf_factor)");
    run(k_leaf<1>, "factor only");
    run(k_leaf<2>, "pivot chain only");
    run(k_leaf<3>, "factor only + column stores and tags");
    run(k_leaf<4>, "factor + inverse + column stores");
    auto run8 = [&](auto kern, const char* name) {  // 512 threads: waves 1-7 read LDS meanwhile
        kern<<<1, 512>>>(dA, out, clk, reps);
        kern<<<1, 512>>>(dA, out, clk, reps);
        long long c = 0;
        (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("%-40s %8.0f clocks per leaf (%.0f per column)\n", name, (double)c / reps, (double)c / reps / 16);
    };
    run(k_leaf<5>, "factor only + column stores");
    run(k_leaf<6>, "factor only + tags");
    run(k_leaf<7>, "factor only + column stores, row 0 only");
    run(k_leaf<8>, "factor only + one store: column + tag");
    run8(k_leaf<3>, "  same, 7 waves reading LDS");
    run8(k_leaf<4>, "  same (inverse), 7 waves reading LDS");
    run8(k_leaf<1>, "  factor only, 7 waves reading LDS");
    return 0;
}
