// Calibration micro-benchmark (not part of the product): shader clocks of one 16x16 leaf factor
// (potrf_body's critical chain) in one wave, variants of what rides along with the pivot chain.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 leaf_lat.hip -o leaf_lat
#include "../../fish-eye_bundle_adjustment_amd/csrc/fba_chol.hip"
#include <cstdio>
#include <cstring>

namespace fba { void set_error(const std::string&) {} }
using namespace fba;
template <class PUT>
__device__ __forceinline__ bool leaf_factor_ref(double (&a)[IB], double (&x)[IB], int lane16, PUT&& put) {
    return leaf_factor(a, x, lane16, put);
}

// The scheduled leaf.  Every instruction of the pivot chain is its own asm statement too, so program
// order is issue order (a wave issues in order; asm volatile statements keep their source order), and
// column C's bulk work -- x[C] *= 1/L[C][C], the a-updates of rows C+2..15 and the inverse's updates,
// 30 - 2C instructions that only need L's column C -- is spread over the dependent steps of column
// C+1's pivot chain (DPP broadcast -> rsq -> correction -> L[.][C+1] -> the first update of column C+2),
// filling their latencies instead of queueing in front of them.  Same instructions, same operands and
// the same order of updates per register as leaf_factor_ref: bit-identical results.
// Hazards the compiler cannot see inside asm: 2 wait states between a VALU write and a DPP read of the
// same VGPR (s_nop 1 in as_bcl and fmac_bcn_first), 1 after a transcendental (s_nop 0 after rsq).
__device__ __forceinline__ double as_mul(double a, double b) {
    double r;
    asm volatile("v_mul_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double as_fma(double a, double b, double c) {
    double r;
    asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ double as_rsq(double a) {
    double r;
    asm volatile("v_rsq_f64 %0, %1\n\ts_nop 0" : "=v"(r) : "v"(a));
    return r;
}
template <int J>
__device__ __forceinline__ double as_bcl(double v) {
    double r;
    asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf bound_ctrl:1"
                 : "=v"(r) : "v"(v), "i"(J));
    return r;
}
// column C's bulk: op 0 x[C] *= inv_C, ops 1..NA a[l] -= L[l][C] L[i][C] (l = C+2..15), then
// x[l] -= L[l][C] x[C] (l = C+1..15)
template <int C>
constexpr int leaf_nbulk() { return C < 0 ? 0 : 1 + (C < IB - 2 ? IB - 2 - C : 0) + (IB - 1 - C); }
template <int C, int K>
__device__ __forceinline__ void leaf_bulk_op(double (&a)[IB], double (&x)[IB], double inv) {
    constexpr int NA = C < IB - 2 ? IB - 2 - C : 0;
    if constexpr (K == 0) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[C]) : "v"(inv));
    else if constexpr (K <= NA) fmac_bcn(a[C + 1 + K], a[C], a[C], C + 1 + K);
    else fmac_bcn(x[C + K - NA], a[C], x[C], C + K - NA);
}
template <int C, int K0, int K1>
__device__ __forceinline__ void leaf_bulk(double (&a)[IB], double (&x)[IB], double inv) {
    if constexpr (K0 < K1) {
        leaf_bulk_op<C, K0>(a, x, inv);
        leaf_bulk<C, K0 + 1, K1>(a, x, inv);
    }
}
// cumulative shares (of 18) of the bulk placed in the gaps after each chain step: bcl, rsq, ar/t, e,
// p/re/are, inv/a[J], F
template <int SCHED>
struct LeafGaps;
template <> struct LeafGaps<0> { static constexpr int w[6] = {2, 7, 9, 11, 14, 16}; };
template <> struct LeafGaps<1> { static constexpr int w[6] = {0, 18, 18, 18, 18, 18}; };  // all behind the rsq
template <> struct LeafGaps<2> { static constexpr int w[6] = {0, 9, 9, 18, 18, 18}; };    // rsq / e
template <> struct LeafGaps<3> { static constexpr int w[6] = {0, 9, 9, 9, 9, 18}; };      // rsq / a[J]
template <> struct LeafGaps<4> { static constexpr int w[6] = {0, 6, 6, 12, 12, 18}; };    // rsq / e / a[J]
// window J: column J's pivot chain with column J-1's bulk between its steps (J = IB: the last bulk)
template <int J, int SCHED, class PUT>
__device__ __forceinline__ void leaf_window(double (&a)[IB], double (&x)[IB], double& inv, bool& ok,
                                            const double m1, const double c38, const double mh, PUT& put) {
    constexpr int C = J - 1, NB = leaf_nbulk<C>();
    const double invc = inv;  // 1 / L[C][C]
    if constexpr (J == IB) {
        leaf_bulk<C, 0, NB>(a, x, invc);
        put(C);
    } else {
        using G = LeafGaps<SCHED>;
        constexpr int b0 = NB * G::w[0] / 18, b1 = NB * G::w[1] / 18, b2 = NB * G::w[2] / 18,
                      b3 = NB * G::w[3] / 18, b4 = NB * G::w[4] / 18, b5 = NB * G::w[5] / 18;
        const double d = as_bcl<J>(a[J]);
        if constexpr (C >= 0) leaf_bulk<C, 0, b0>(a, x, invc);
        const double r = as_rsq(d);
        if constexpr (C >= 0) leaf_bulk<C, b0, b1>(a, x, invc);
        const double ar = as_mul(a[J], r);
        const double t = as_mul(d, r);
        if constexpr (C >= 0) leaf_bulk<C, b1, b2>(a, x, invc);
        const double e = as_fma(t, r, m1);
        if constexpr (C >= 0) leaf_bulk<C, b2, b3>(a, x, invc);
        const double p = as_fma(e, c38, mh);
        const double re = as_mul(r, e);
        const double are = as_mul(ar, e);
        if constexpr (C >= 0) leaf_bulk<C, b3, b4>(a, x, invc);
        inv = as_fma(re, p, r);
        a[J] = as_fma(are, p, ar);  // lane J: sqrt(d); lanes > J: L[i][J]
        if constexpr (C >= 0) leaf_bulk<C, b4, b5>(a, x, invc);
        if constexpr (J + 1 < IB) fmac_bcn_first(a[J + 1], a[J], a[J], J + 1);
        if constexpr (C >= 0) {
            leaf_bulk<C, b5, NB>(a, x, invc);
            put(C);
        }
        ok &= d > 0.0;
    }
}
template <int SCHED, class PUT>
__device__ __forceinline__ bool leaf_factor_s(double (&a)[IB], double (&x)[IB], int lane16, PUT&& put) {
    bool ok = true;
    double inv = 0.0;
#pragma unroll
    for (int r = 0; r < IB; ++r) x[r] = (r == lane16) ? 1.0 : 0.0;
    const double m1 = -1.0, c38 = 0.375, mh = -0.5;
    bulk_for(std::make_integer_sequence<int, IB + 1>{}, [&](auto jc) {
        leaf_window<decltype(jc)::value, SCHED>(a, x, inv, ok, m1, c38, mh, put);
    });
    return ok;
}



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

// the potrf's use: rows from LDS, factor + inverse, column stores (put); REF: leaf_factor_ref.  Writes
// L and D of the last rep to out2 (bit-identity check on the host)
template <int REF>
__global__ __launch_bounds__(64) void k_leaf_lds(const double* __restrict__ A, double* __restrict__ out2,
                                                 long long* clk, int reps) {
    const int lane = threadIdx.x & 63, lr = lane & 15;
    __shared__ double Ash[16 * 17], Lw[16 * 17], Dw[16 * 17];
    if (lane < 16)
        for (int c = 0; c < IB; ++c) Ash[lane * 17 + c] = A[lane * IB + c];
    __syncthreads();
    long long t = 0;
    for (int it = 0; it < reps; ++it) {
        double a[IB], x[IB];
#pragma unroll
        for (int c = 0; c < IB; ++c) a[c] = Ash[lr * 17 + c];
        const long long t0 = clock64();
        auto put = [&](int j) { Lw[lr * 17 + j] = a[j]; Dw[j * 17 + lr] = x[j]; };
        bool ok;
        if constexpr (REF < 0) ok = leaf_factor_ref(a, x, lr, put);
        else ok = leaf_factor_s<REF>(a, x, lr, put);
        __builtin_amdgcn_s_waitcnt(0xC07F);
        const long long t1 = clock64();
        t += t1 - t0;
        if (!ok) Ash[0] = 0.0;
        // feed back (a dependence on this rep, numerically nothing)
        if (lane == 0) Ash[17 * 15 + 15] += Lw[0] * 0.0;
        __syncthreads();
    }
    if (lane < 16)
        for (int c = 0; c < IB; ++c) {
            out2[lane * IB + c] = Lw[lane * 17 + c];
            out2[256 + lane * IB + c] = Dw[lane * 17 + c];
        }
    if (lane == 0) *clk = t;
}

// The row-shared leaf: the four 16-lane rows of the wave run ONE instruction stream on different data --
// row 0 the leaf's rows (the factor), row 1 the columns of its inverse (identity at the start), row 2 the
// leaf again, row 3 the rows of the panel tile below (X = A L^-T); one update instruction per (j, l) serves
// all four, its broadcast source being L's column j on every row (rows 1 / 3 get it from rows 0 / 2 with
// v_permlane16_swap).  The pivot d comes from lane j by v_readlane (uniform), so the pivot chain's values
// (r, e, p, 1/L_jj) are the same on every row and column j is scaled by one multiply on all four.
// put(j): after column j (row 0: L col j, row 1: row j of L^-1, row 3: column j of X)
template <class PUT>
__device__ __forceinline__ bool leaf_rows(double (&v)[IB], PUT&& put) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < IB; ++j) {
        const uint64_t bits = __builtin_bit_cast(uint64_t, v[j]);
        const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)bits, j);
        const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(bits >> 32), j);
        const double d = __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
        ok &= d > 0.0;
        const double r = __builtin_amdgcn_rsq(d);
        const double t = d * r;
        const double e = __builtin_fma(t, r, -1.0);
        const double p = __builtin_fma(e, 0.375, -0.5);
        const double inv = __builtin_fma(r * e, p, r);
        v[j] *= inv;  // row 0: L[.][j] (lane j: sqrt(d)); row 1: (L^-1)[j][c]; row 3: X[.][j]
        // src = L's column j on every row: rows 1, 3 take rows 0, 2's v[j]
        const uint64_t vb = __builtin_bit_cast(uint64_t, v[j]);
        const auto slo = __builtin_amdgcn_permlane16_swap((uint32_t)vb, (uint32_t)vb, false, false);
        const auto shi = __builtin_amdgcn_permlane16_swap((uint32_t)(vb >> 32), (uint32_t)(vb >> 32), false, false);
        // (the swap exchanges odd rows of its first operand with even rows of its second: element 0 is the
        // first operand after the swap -- odd rows now hold the even rows' values, even rows their own)
        const double src = __builtin_bit_cast(double, ((uint64_t)shi[0] << 32) | slo[0]);
#pragma unroll
        for (int l = j + 1; l < IB; ++l) {
            if (l == j + 1) fmac_bcn_first(v[l], src, v[j], l);
            else fmac_bcn(v[l], src, v[j], l);
        }
        put(j);
    }
    return ok;
}

template <int MODE>
__global__ __launch_bounds__(64) void k_leaf_rows(const double* __restrict__ A, const double* __restrict__ Pn,
                                                  double* __restrict__ out2, long long* clk, int reps) {
    const int lane = threadIdx.x & 63, lr = lane & 15, row = lane >> 4;
    __shared__ double Ash[16 * 17], Psh[16 * 17], Lw[16 * 17], Dw[16 * 17], Xw[16 * 17], junk[64];
    if (lane < 16)
        for (int c = 0; c < IB; ++c) {
            Ash[lane * 17 + c] = A[lane * IB + c];
            Psh[lane * 17 + c] = Pn[lane * IB + c];
        }
    __syncthreads();
    long long t = 0;
    for (int it = 0; it < reps; ++it) {
        double v[IB];
#pragma unroll
        for (int c = 0; c < IB; ++c)
            v[c] = row == 1 ? (c == lr ? 1.0 : 0.0) : (row == 3 ? Psh[lr * 17 + c] : Ash[lr * 17 + c]);
        const long long t0 = clock64();
        bool ok;
        if (MODE == 0) {
            ok = leaf_rows(v, [&](int j) {  // one store: row 0 L col j, row 1 D row j, row 3 X col j
                double* dst = row == 0 ? &Lw[lr * 17 + j] : row == 1 ? &Dw[j * 17 + lr] : row == 3 ? &Xw[lr * 17 + j] : &junk[lane];
                *dst = v[j];
            });
        } else {
            double x[IB];
            ok = leaf_factor(v, x, lr, [&](int j) { Lw[lr * 17 + j] = v[j]; Dw[j * 17 + lr] = x[j]; });
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        const long long t1 = clock64();
        t += t1 - t0;
        if (!ok) Ash[0] = 0.0;
        if (lane == 0) Ash[17 * 15 + 15] += Lw[0] * 0.0;
        __syncthreads();
    }
    if (lane < 16)
        for (int c = 0; c < IB; ++c) {
            out2[lane * IB + c] = Lw[lane * 17 + c];
            out2[256 + lane * IB + c] = Dw[lane * 17 + c];
            out2[512 + lane * IB + c] = Xw[lane * 17 + c];
        }
    if (lane == 0) *clk = t;
}

// raw issue / latency of f64 VALU ops on one wave (clocks per op, 64 ops a rep)
template <int MODE>
__global__ __launch_bounds__(64) void k_lat(const double* __restrict__ A, double* __restrict__ out, long long* clk, int reps) {
    const int lane = threadIdx.x;
    double c = A[lane & 15], d = c * 0.5, e = c * 0.25, v[8];
    for (int i = 0; i < 8; ++i) v[i] = A[(lane + i) & 15];
    const long long t0 = clock64();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            if constexpr (MODE == 0) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c) : "v"(d), "v"(e));
            else if constexpr (MODE == 1) fmac_bcn(v[k & 7], d, e, 1 + (k & 7));
            else if constexpr (MODE == 2) fmac_bcn(c, d, e, 1 + (k & 7));
            else if constexpr (MODE == 3) {
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c) : "v"(d), "v"(e));
                fmac_bcn(v[(2 * k) & 7], d, e, 1 + (k & 7));
                fmac_bcn(v[(2 * k + 1) & 7], d, e, 2 + (k & 7));
            } else if constexpr (MODE == 4) {
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c) : "v"(d), "v"(e));
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v[(2 * k) & 7]) : "v"(d), "v"(e));
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v[(2 * k + 1) & 7]) : "v"(d), "v"(e));
            } else if constexpr (MODE == 5) {  // dependent chain with 4 DPP fmacs between
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(c) : "v"(d), "v"(e));
#pragma unroll
                for (int q = 0; q < 4; ++q) fmac_bcn(v[(4 * k + q) & 7], d, e, 1 + q);
            } else if constexpr (MODE == 6) {  // 1 non-DPP fma independent, 1 DPP: mix
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v[k & 7]) : "v"(d), "v"(e));
                fmac_bcn(v[(k + 4) & 7], d, e, 1 + (k & 7));
            } else if constexpr (MODE == 7) {  // rsq chain
                asm volatile("v_rsq_f64 %0, %0\n\ts_nop 0" : "+v"(c));
            }
        }
    }
    const long long t1 = clock64();
    double acc = c;
    for (int i = 0; i < 8; ++i) acc += v[i];
    out[lane] = acc;
    if (lane == 0) *clk = t1 - t0;
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
    {
        auto lat = [&](auto kern, const char* name, int ops) {
            long long c = 0;
            kern<<<1, 64>>>(dA, out, clk, 50);
            kern<<<1, 64>>>(dA, out, clk, 50);
            (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
            printf("%-58s %6.2f clocks per step (%d instr)\n", name, (double)c / (50 * 64), ops);
        };
        lat(k_lat<0>, "dependent v_fma_f64 chain", 1);
        lat(k_lat<1>, "independent v_fmac_f64_dpp (8 accumulators)", 1);
        lat(k_lat<2>, "dependent v_fmac_f64_dpp chain", 1);
        lat(k_lat<3>, "dependent fma + 2 independent dpp fmacs", 3);
        lat(k_lat<4>, "dependent fma + 2 independent fmas", 3);
        lat(k_lat<5>, "dependent fma + 4 independent dpp fmacs", 5);
        lat(k_lat<6>, "independent fma + independent dpp fmac", 2);
        lat(k_lat<7>, "dependent v_rsq_f64 chain", 1);
    }
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
    {
        double *o1, *o2;
        (void)hipMalloc(&o1, 512 * sizeof(double));
        (void)hipMalloc(&o2, 512 * sizeof(double));
        auto one = [&](auto kern, double* o) {
            long long c = 0;
            kern<<<1, 64>>>(dA, o, clk, reps);
            (void)hipMemcpy(&c, clk, sizeof(c), hipMemcpyDeviceToHost);
            return (double)c / reps;
        };
        for (int r = 0; r < 3; ++r) {
            const double t_ref = one(k_leaf_lds<-1>, o1), t1 = one(k_leaf_lds<1>, o2), t2 = one(k_leaf_lds<2>, o2),
                         t3 = one(k_leaf_lds<3>, o2), t4 = one(k_leaf_lds<4>, o2), t0 = one(k_leaf_lds<0>, o2);
            printf("potrf-style leaf (LDS rows, column stores): reference order %6.0f, scheduled 0..4: %6.0f %6.0f %6.0f %6.0f %6.0f clocks\n",
                   t_ref, t0, t1, t2, t3, t4);
        }
        double h1[512], h2[512];
        (void)hipMemcpy(h1, o1, sizeof(h1), hipMemcpyDeviceToHost);
        (void)hipMemcpy(h2, o2, sizeof(h2), hipMemcpyDeviceToHost);
        int diff = 0;
        for (int i = 0; i < 512; ++i) {
            const int r = (i & 255) / 16, c = i & 15;
            const bool used = c <= r;  // lower triangles of L and of L^-1 (Dw[j][lane] = (L^-1)[j][lane])
            if (used && memcmp(&h1[i], &h2[i], 8) != 0) ++diff;
        }
        printf("scheduled vs reference leaf: %d differing entries of L and L^-1 (bitwise)\n", diff);
        // the row-shared leaf against the reference leaf (L, L^-1) and X = P L^-T from that L
        double hP[256];
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) hP[i * 16 + j] = 0.3 * std::sin(1.0 + i * 0.7 + j * 1.3);
        double* dP;
        (void)hipMalloc(&dP, sizeof(hP));
        (void)hipMemcpy(dP, hP, sizeof(hP), hipMemcpyHostToDevice);
        double *r1, *r2;
        (void)hipMalloc(&r1, 768 * sizeof(double));
        (void)hipMalloc(&r2, 768 * sizeof(double));
        for (int r = 0; r < 3; ++r) {
            long long c1 = 0, c2 = 0;
            k_leaf_rows<1><<<1, 64>>>(dA, dP, r1, clk, reps);
            (void)hipMemcpy(&c1, clk, sizeof(c1), hipMemcpyDeviceToHost);
            k_leaf_rows<0><<<1, 64>>>(dA, dP, r2, clk, reps);
            (void)hipMemcpy(&c2, clk, sizeof(c2), hipMemcpyDeviceToHost);
            printf("leaf, LDS rows + stores: reference %6.0f clocks; row-shared (factor + inverse + a panel tile) %6.0f clocks\n",
                   (double)c1 / reps, (double)c2 / reps);
        }
        double g1[768], g2[768];
        (void)hipMemcpy(g1, r1, sizeof(g1), hipMemcpyDeviceToHost);
        (void)hipMemcpy(g2, r2, sizeof(g2), hipMemcpyDeviceToHost);
        double eL = 0, eD = 0, eX = 0, mL = 0, mD = 0, mX = 0;
        for (int i = 0; i < 16; ++i)
            for (int c = 0; c <= i; ++c) {
                eL = std::max(eL, std::fabs(g1[i * 16 + c] - g2[i * 16 + c]));
                mL = std::max(mL, std::fabs(g1[i * 16 + c]));
                eD = std::max(eD, std::fabs(g1[256 + i * 16 + c] - g2[256 + i * 16 + c]));
                mD = std::max(mD, std::fabs(g1[256 + i * 16 + c]));
            }
        for (int i = 0; i < 16; ++i)  // X = P L^-T by substitution with the reference L
            for (int j = 0; j < 16; ++j) {
                double x = hP[((i + 3) & 15) * 0 + i * 16 + j];
                (void)x;
            }
        {
            double X[256];
            for (int i = 0; i < 16; ++i)
                for (int j = 0; j < 16; ++j) {
                    double s2 = hP[i * 16 + j];
                    for (int k = 0; k < j; ++k) s2 -= X[i * 16 + k] * g1[j * 16 + k];
                    X[i * 16 + j] = s2 / g1[j * 16 + j];
                }
            for (int q = 0; q < 256; ++q) {
                eX = std::max(eX, std::fabs(X[q] - g2[512 + q]));
                mX = std::max(mX, std::fabs(X[q]));
            }
        }
        printf("row-shared vs reference: L %.2e, L^-1 %.2e, X %.2e (max abs diff / max abs)\n", eL / mL, eD / mD, eX / mX);
    }
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
