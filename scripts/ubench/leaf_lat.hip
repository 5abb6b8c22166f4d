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

// the factor without the inverse, with a per-column hook put(j, inv) (inv = 1 / L[j][j])
template <class PUT>
__device__ __forceinline__ bool leaf_factor_noinv(double (&a)[IB], PUT&& put) {
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
        const double inv = __builtin_fma(r * e, p, r);
        a[j] = __builtin_fma(ar * e, p, ar);
#pragma unroll
        for (int l = j + 1; l < IB; ++l) {
            if (l == j + 1) fmac_bcn_first(a[l], a[j], a[j], l);
            else fmac_bcn(a[l], a[j], a[j], l);
        }
        put(j, inv);
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

// MODE 9: wave 0 factors without the inverse and stores each column of L once (lanes 0-15); wave 1
// (another SIMD) polls the columns (NaN sentinel, every lane of a column in the one ds_write_b64) and
// runs the substitutions beside it: row 0 of its lanes the inverse D_s (lane c = column c), row 1 a
// panel tile's rows X = A L^-T (lane i = row i).  Clocks: wave 0's leaf, wave 1 done (same start)
__global__ __launch_bounds__(128) void k_leaf_split(const double* __restrict__ A, double* __restrict__ out,
                                                      long long* clk, int reps) {
    const int lane = threadIdx.x & 63, lr = lane & 15, wave = threadIdx.x >> 6;
    __shared__ double Lw[16 * 17], junk[64];
    double a0[IB], y0[IB];
#pragma unroll
    for (int c = 0; c < IB; ++c) {
        a0[c] = A[lr * IB + c];
        y0[c] = (lane < 16) ? (c == lr ? 1.0 : 0.0) : A[((lr + 3) & 15) * IB + c] * 0.5;
    }
    long long s0 = 0, s1 = 0, s2 = 0;
    double acc = 0.0;
    const double SENT = __builtin_nan("");
    for (int it = 0; it < reps; ++it) {
        if (wave == 1 && lane < 16)
            for (int c = 0; c < IB; ++c) Lw[lane * 17 + c] = SENT;
        __syncthreads();
        const long long t0 = clock64();
        if (wave == 0) {
            double a[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = a0[c] + acc * 1e-300;
            bool ok = leaf_factor_noinv(a, [&](int j, double) { *(lane < 16 ? &Lw[lr * 17 + j] : &junk[lane]) = a[j]; });
            const long long t1 = clock64();
            s1 += t1 - t0;
            acc += a[IB - 1] + (ok ? 0.0 : 1.0);
        } else {
            double y[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) y[c] = y0[c];
#pragma unroll
            for (int j = 0; j < IB; ++j) {
                double lc;
                for (;;) {  // column j of L: lane l holds L[l][j] (lanes >= j meaningful)
                    lc = *(volatile double*)&Lw[lr * 17 + j];
                    const bool miss = (lr >= j) && (lc != lc);
                    if (!__builtin_amdgcn_ballot_w64(miss)) break;
                }
                const double dj = bcl(lc, j);
                double inv = __builtin_amdgcn_rcp(dj);
                const double e = __builtin_fma(-dj, inv, 1.0);
                inv = __builtin_fma(inv, e, inv);
                inv = __builtin_fma(inv, __builtin_fma(-dj, inv, 1.0), inv);
                y[j] *= inv;
#pragma unroll
                for (int l = j + 1; l < IB; ++l) {
                    if (l == j + 1) fmac_bcn_first(y[l], lc, y[j], l);
                    else fmac_bcn(y[l], lc, y[j], l);
                }
            }
            const long long t2 = clock64();
            s2 += t2 - t0;
            acc += y[IB - 1];
        }
        __syncthreads();
    }
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) clk[0] = s1;
    if (threadIdx.x == 64) clk[1] = s2;
}

// MODE 10: as MODE 9, with wave 1 prefetching column j+1 while it works on column j; WINV: wave 0's
// column store also carries 1 / L[j][j] (lane 16 -> invs[j], the same ds_write), else wave 1 forms it
template <bool WINV>
__global__ __launch_bounds__(128) void k_leaf_split2(const double* __restrict__ A, double* __restrict__ out,
                                                       long long* clk, int reps) {
    const int lane = threadIdx.x & 63, lr = lane & 15, wave = threadIdx.x >> 6;
    __shared__ double Lw[16 * 17], invs[16], junk[64];
    double a0[IB], y0[IB];
#pragma unroll
    for (int c = 0; c < IB; ++c) {
        a0[c] = A[lr * IB + c];
        y0[c] = (lane < 16) ? (c == lr ? 1.0 : 0.0) : A[((lr + 3) & 15) * IB + c] * 0.5;
    }
    long long s1 = 0, s2 = 0;
    double acc = 0.0;
    const double SENT = __builtin_nan("");
    for (int it = 0; it < reps; ++it) {
        if (wave == 1 && lane < 16) {
            for (int c = 0; c < IB; ++c) Lw[lane * 17 + c] = SENT;
            invs[lane] = SENT;
        }
        __syncthreads();
        const long long t0 = clock64();
        if (wave == 0) {
            double a[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = a0[c] + acc * 1e-300;
            bool ok;
            if (WINV)
                ok = leaf_factor_noinv(a, [&](int j, double inv) {
                    *(lane < 16 ? &Lw[lr * 17 + j] : lane == 16 ? &invs[j] : &junk[lane]) = lane == 16 ? inv : a[j];
                });
            else
                ok = leaf_factor_noinv(a, [&](int j, double) { *(lane < 16 ? &Lw[lr * 17 + j] : &junk[lane]) = a[j]; });
            const long long t1 = clock64();
            s1 += t1 - t0;
            acc += a[IB - 1] + (ok ? 0.0 : 1.0);
        } else {
            double y[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) y[c] = y0[c];
            double lcn = *(volatile double*)&Lw[lr * 17], ivn = WINV ? *(volatile double*)&invs[0] : 0.0;
#pragma unroll
            for (int j = 0; j < IB; ++j) {
                double lc = lcn, iv = ivn;
                for (;;) {
                    const bool miss = ((lr >= j) && (lc != lc)) || (WINV && iv != iv);
                    if (!__builtin_amdgcn_ballot_w64(miss)) break;
                    lc = *(volatile double*)&Lw[lr * 17 + j];
                    if (WINV) iv = *(volatile double*)&invs[j];
                }
                if (j + 1 < IB) {
                    lcn = *(volatile double*)&Lw[lr * 17 + j + 1];
                    if (WINV) ivn = *(volatile double*)&invs[j + 1];
                }
                double inv = iv;
                if (!WINV) {
                    const double dj = bcl(lc, j);
                    inv = __builtin_amdgcn_rcp(dj);
                    inv = __builtin_fma(inv, __builtin_fma(-dj, inv, 1.0), inv);
                    inv = __builtin_fma(inv, __builtin_fma(-dj, inv, 1.0), inv);
                }
                y[j] *= inv;
#pragma unroll
                for (int l = j + 1; l < IB; ++l) {
                    if (l == j + 1) fmac_bcn_first(y[l], lc, y[j], l);
                    else fmac_bcn(y[l], lc, y[j], l);
                }
            }
            const long long t2 = clock64();
            s2 += t2 - t0;
            acc += y[IB - 1];
        }
        __syncthreads();
    }
    out[threadIdx.x] = acc;
    if (threadIdx.x == 0) clk[0] = s1;
    if (threadIdx.x == 64) clk[1] = s2;
}

int main() {
    double hA[256];
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) hA[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    double *dA, *out; long long* clk;
    (void)hipMalloc(&dA, sizeof(hA));
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&clk, 2 * sizeof(long long));
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
    for (int r = 0; r < 2; ++r) {
        k_leaf_split<<<1, 128>>>(dA, out, clk, reps);
        long long c[2] = {0, 0};
        (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("split: wave 0 factor-only leaf %6.0f clocks, wave 1 inverse + panel rows done %6.0f clocks\n",
               (double)c[0] / reps, (double)c[1] / reps);
    }
    for (int r = 0; r < 2; ++r) {
        k_leaf_split2<false><<<1, 128>>>(dA, out, clk, reps);
        long long c[2] = {0, 0};
        (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("split, prefetch: wave 0 %6.0f, wave 1 done %6.0f clocks\n", (double)c[0] / reps, (double)c[1] / reps);
        k_leaf_split2<true><<<1, 128>>>(dA, out, clk, reps);
        (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
        printf("split, prefetch, inv from wave 0: wave 0 %6.0f, wave 1 done %6.0f clocks\n", (double)c[0] / reps, (double)c[1] / reps);
    }
    return 0;
}
