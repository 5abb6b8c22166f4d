// Micro-benchmark of the 128x128 diagonal-block factorisation kernels (calibration only).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../fish-eye_bundle_adjustment_amd/csrc \
//         potrf_ubench.hip -o potrf_ubench
// Times k_potrf128 (library) and the instrumented/experimental variants on one SPD block, checks
// them against a host Cholesky, and prints a per-phase cycle breakdown of the instrumented copy.
#include "../../fish-eye_bundle_adjustment_amd/csrc/fba_chol.hip"

#include <cmath>
#include <cstdio>
#include <vector>

namespace fba { void set_error(const std::string&) {} }
using namespace fba;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

#define TS(i) do { if (tid == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)

// instrumented copy of k_potrf128 (same algorithm)
__global__ __launch_bounds__(256) void k_potrf_prof(double* __restrict__ S, int64_t ld, int64_t k0,
                                                    double* __restrict__ dinv, double* __restrict__ scal,
                                                    unsigned long long* ts) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem;
    double* Dl = smem + CB * LDA;
    double* rd = Dl + IB * 17;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    TS(0);
    for (int idx = tid; idx < CB * CB / 2; idx += 256) {
        const int r = idx >> 6, c = (idx & 63) * 2;
        const double2 v = *reinterpret_cast<const double2*>(S + (k0 + r) * ld + k0 + c);
        A[r * LDA + c] = v.x;
        A[r * LDA + c + 1] = v.y;
    }
    __syncthreads();
    TS(1);
    const int lr = lane & 15, lk = lane >> 4;
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        if (wave == 0) {
            double a[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = (lane < IB) ? A[(c0 + lane) * LDA + c0 + c] : 0.0;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < IB; ++j) {
                double d = readlane_d(a[j], j);
                if (!(d > 0.0)) { bad = true; d = 1.0; }
                const double inv = rsqrt_d(d), sd = d * inv;
                if (lane == 0) rd[j] = inv;
                a[j] = (lane == j) ? sd : (lane > j ? a[j] * inv : a[j]);
#pragma unroll
                for (int l = j + 1; l < IB; ++l) a[l] -= a[j] * readlane_d(a[j], l);
            }
            if (bad && lane == 0 && scal[1] == 0.0) scal[1] = (double)(k0 + c0 + 1);
            if (lane < IB) {
#pragma unroll
                for (int c = 0; c < IB; ++c)
                    if (c <= lane) A[(c0 + lane) * LDA + c0 + c] = a[c];
            }
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            TS(2 + 4 * s);
            double x[IB];
#pragma unroll
            for (int i = 0; i < IB; ++i) {
                double acc = (i == lane) ? 1.0 : 0.0;
#pragma unroll
                for (int m = 0; m < i; ++m) acc -= A[(c0 + i) * LDA + c0 + m] * x[m];
                x[i] = acc * rd[i];
            }
            if (lane < IB) {
#pragma unroll
                for (int i = 0; i < IB; ++i) {
                    const double v = (i >= lane) ? x[i] : 0.0;
                    Dl[i * 17 + lane] = v;
                    dinv[((k0 / CB) * (CB / IB) + s) * (IB * IB) + i * IB + lane] = v;
                }
            }
        }
        __syncthreads();
        TS(3 + 4 * s);
        for (int t = s + 1 + wave; t < CB / IB; t += 4) {
            const int r0 = t * IB;
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4) {
                const double av = A[(r0 + lr) * LDA + c0 + kk + lk];
                const double bv = Dl[lr * 17 + kk + lk];
                acc = mfma(av, bv, acc);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(r0 + lk + 4 * r) * LDA + c0 + lr] = acc[r];
        }
        __syncthreads();
        TS(4 + 4 * s);
        const int m = CB / IB - 1 - s;
        const int ntile = m * (m + 1) / 2;
        for (int q = wave; q < ntile; q += 4) {
            int ti = 0, rem = q;
            while (rem > ti) { rem -= ti + 1; ++ti; }
            const int tj = rem;
            const int R = (s + 1 + ti) * IB, C = (s + 1 + tj) * IB;
            dbl4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = A[(R + lk + 4 * r) * LDA + C + lr];
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4) {
                const double av = -A[(R + lr) * LDA + c0 + kk + lk];
                const double bv = A[(C + lr) * LDA + c0 + kk + lk];
                acc = mfma(av, bv, acc);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(R + lk + 4 * r) * LDA + C + lr] = acc[r];
        }
        __syncthreads();
        TS(5 + 4 * s);
    }
    for (int idx = tid; idx < CB * CB; idx += 256) {
        const int r = idx >> 7, c = idx & 127;
        if (c <= r) S[(k0 + r) * ld + k0 + c] = A[r * LDA + c];
    }
    __syncthreads();
    TS(40);
}


__global__ void k_rsq_acc(const double* d, double* r0, double* r1, double* r2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    double r = __builtin_amdgcn_rsq(x);
    r0[i] = r;
    r = r * (1.5 - 0.5 * x * r * r);
    r1[i] = r;
    r = r * (1.5 - 0.5 * x * r * r);
    r2[i] = r;
}

// instrumented copy of k_trsm128
__global__ __launch_bounds__(256) void k_trsm_prof(double* __restrict__ S, int64_t ld, int64_t k0, int64_t row0,
                                                 const double* __restrict__ dinv, unsigned long long* ts) {
#define TT(i) do { if (blockIdx.x == 5 && threadIdx.x == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)
    TT(0);
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* X = smem;                       // [4][IB][LDA]   panel rows of each wave
    double* T = X + 4 * IB * LDA;           // [4][IB][17]    per-wave 16x16 staging
    double* Lt = T + 4 * IB * 17;           // [28][IB][17]   L_st, p = s(s-1)/2 + t
    double* Dt = Lt + TRSM_NT * IB * 17;    // [8][IB][17]    D_s
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int64_t rbase = row0 + (int64_t)blockIdx.x * 64 + wave * IB;
    double* Xw = X + wave * IB * LDA;
    double* Tw = T + wave * IB * 17;
    const double* L = S + k0 * ld + k0;
    const double* Dk = dinv + (k0 / CB) * (CB / IB) * (IB * IB);
    {
        double2 v[16], lv[14], dv[4];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int idx = lane + 64 * q, r = idx >> 6, c = (idx & 63) * 2;
            v[q] = *reinterpret_cast<const double2*>(S + (rbase + r) * ld + k0 + c);
        }
        // off-diagonal tiles: item i -> tile p = i >> 7, row n = (i >> 3) & 15, columns 2*(i & 7)
#pragma unroll
        for (int q = 0; q < 14; ++q) {
            const int i = tid + 256 * q, p = i >> 7, n = (i >> 3) & 15, kc = (i & 7) * 2;
            int sr = 1, pp = p;
            while (pp >= sr) { pp -= sr; ++sr; }
            lv[q] = *reinterpret_cast<const double2*>(L + (int64_t)(sr * IB + n) * ld + pp * IB + kc);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) dv[q] = *reinterpret_cast<const double2*>(Dk + 2 * (tid + 256 * q));
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int idx = lane + 64 * q, r = idx >> 6, c = (idx & 63) * 2;
            Xw[r * LDA + c] = v[q].x;
            Xw[r * LDA + c + 1] = v[q].y;
        }
#pragma unroll
        for (int q = 0; q < 14; ++q) {
            const int i = tid + 256 * q, p = i >> 7, n = (i >> 3) & 15, kc = (i & 7) * 2;
            Lt[(p * IB + n) * 17 + kc] = lv[q].x;
            Lt[(p * IB + n) * 17 + kc + 1] = lv[q].y;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = 2 * (tid + 256 * q), sd = e >> 8, n = (e >> 4) & 15, kc = e & 15;
            Dt[(sd * IB + n) * 17 + kc] = dv[q].x;
            Dt[(sd * IB + n) * 17 + kc + 1] = dv[q].y;
        }
    }
    __syncthreads();
    TT(1);
#pragma unroll
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        // Z = A_s - sum_{t<s} X_t L_st^T : output 16x16, K = 16 s.  All operands of the step are read
        // from LDS in one batch, then two independent MFMA chains.
        double av[CB / 4], bv[CB / 4];
#pragma unroll
        for (int t = 0; t < s; ++t) {
            const double* Lst = Lt + (s * (s - 1) / 2 + t) * IB * 17;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) {  // B[k][n] = L[c0+n][t*16+k]
                av[4 * t + kk] = Xw[lr * LDA + t * IB + 4 * kk + lk];
                bv[4 * t + kk] = Lst[lr * 17 + 4 * kk + lk];
            }
        }
        dbl4 p0 = dbl4{0.0, 0.0, 0.0, 0.0}, p1 = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 4 * s; q += 2) {
            p0 = mfma(av[q], bv[q], p0);
            p1 = mfma(av[q + 1], bv[q + 1], p1);
        }
        dbl4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = Xw[(lk + 4 * r) * LDA + c0 + lr] - (p0[r] + p1[r]);
        // Z (D layout) -> LDS, then X_s = Z D_s^T
#pragma unroll
        for (int r = 0; r < 4; ++r) Tw[(lk + 4 * r) * 17 + lr] = acc[r];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        dbl4 out = dbl4{0.0, 0.0, 0.0, 0.0};
        const double* Ds = Dt + s * IB * 17;
#pragma unroll
        for (int kk = 0; kk < IB; kk += 4) out = mfma(Tw[lr * 17 + kk + lk], Ds[lr * 17 + kk + lk], out);
#pragma unroll
        for (int r = 0; r < 4; ++r) Xw[(lk + 4 * r) * LDA + c0 + lr] = out[r];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    TT(2);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int idx = lane + 64 * q, r = idx >> 6, c = (idx & 63) * 2;
        double2 v;
        v.x = Xw[r * LDA + c];
        v.y = Xw[r * LDA + c + 1];
        *reinterpret_cast<double2*>(S + (rbase + r) * ld + k0 + c) = v;
    }
    __builtin_amdgcn_s_waitcnt(0);
    TT(3);
#undef TT
}

// previous (full 128x130 LDS block) version, for the contention comparison
__global__ __launch_bounds__(256) void k_potrf_old(double* __restrict__ S, int64_t ld, int64_t k0,
                                                  double* __restrict__ dinv, double* __restrict__ scal) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem;                  // [128][LDA]
    double* Dl = smem + CB * LDA;      // [16][17] current inverse D_s
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    {
        // 128 x 128 block: thread -> row tid >> 1, 64 columns; 2 batches of 16 double2
        const int r = tid >> 1, cb = (tid & 1) * 64;
        const double* g = S + (k0 + r) * ld + k0 + cb;
        double2 v[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) v[q] = *reinterpret_cast<const double2*>(g + 2 * q);
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            A[r * LDA + cb + 2 * q] = v[q].x;
            A[r * LDA + cb + 2 * q + 1] = v[q].y;
        }
    }
    __syncthreads();
    const int64_t dbase = (k0 / CB) * (CB / IB) * (IB * IB);
    bool ok = true;
    // leaf 0 (wave 0)
    if (wave == 0) {
        double a[IB], x[IB];
#pragma unroll
        for (int c = 0; c < IB; ++c) a[c] = A[lr * LDA + c];
        ok = leaf_factor(a, x, lr);
        if (lane < IB) {
#pragma unroll
            for (int c = 0; c < IB; ++c) {
                if (c <= lane) A[lane * LDA + c] = a[c];
                const double v = (c >= lane) ? x[c] : 0.0;  // (L^-1)[c][lane]
                Dl[c * 17 + lane] = v;
                dinv[dbase + c * IB + lane] = v;
            }
        }
    }
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        __syncthreads();  // B1: L_ss, D_s in LDS; column s updated
        if (s == CB / IB - 1) break;
        // panel solve X_t = A_ts D_s^T: wave 0 tile s+1, waves 1..3 tiles s+2..7
        {
            const int t0 = (wave == 0) ? s + 1 : s + 1 + wave;
            const int step = (wave == 0) ? CB : 3;
            for (int t = t0; t < CB / IB; t += step) {
                const int r0 = t * IB;
                dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kk = 0; kk < IB; kk += 4)
                    acc = mfma(A[(r0 + lr) * LDA + c0 + kk + lk], Dl[lr * 17 + kk + lk], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) A[(r0 + lk + 4 * r) * LDA + c0 + lr] = acc[r];
            }
        }
        __syncthreads();  // B2: panel column s solved
        const int m = CB / IB - 1 - s;  // tiles (ti, tj), s < tj <= ti
        if (wave == 0) {
            // next diagonal tile, then its leaf factor
            const int R = c0 + IB;
            dbl4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = A[(R + lk + 4 * r) * LDA + R + lr];
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4)
                acc = mfma(-A[(R + lr) * LDA + c0 + kk + lk], A[(R + lr) * LDA + c0 + kk + lk], acc);
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(R + lk + 4 * r) * LDA + R + lr] = acc[r];
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            double a[IB], x[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = A[(R + lr) * LDA + R + c];
            ok &= leaf_factor(a, x, lr);
            if (lane < IB) {
#pragma unroll
                for (int c = 0; c < IB; ++c) {
                    if (c <= lane) A[(R + lane) * LDA + R + c] = a[c];
                    const double v = (c >= lane) ? x[c] : 0.0;  // (L^-1)[c][lane]
                    Dl[c * 17 + lane] = v;  // safe: every wave finished reading D_s before B2
                    dinv[dbase + (s + 1) * IB * IB + c * IB + lane] = v;
                }
            }
        } else {
            const int ntile = m * (m + 1) / 2;
            for (int q = 1 + (wave - 1); q < ntile; q += 3) {
                int ti = 0, rem = q;
                while (rem > ti) { rem -= ti + 1; ++ti; }
                const int tj = rem;
                const int R = (s + 1 + ti) * IB, C = (s + 1 + tj) * IB;
                dbl4 acc;
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[r] = A[(R + lk + 4 * r) * LDA + C + lr];
#pragma unroll
                for (int kk = 0; kk < IB; kk += 4)
                    acc = mfma(-A[(R + lr) * LDA + c0 + kk + lk], A[(C + lr) * LDA + c0 + kk + lk], acc);
#pragma unroll
                for (int r = 0; r < 4; ++r) A[(R + lk + 4 * r) * LDA + C + lr] = acc[r];
            }
        }
    }
    if (!ok && lane == 0 && scal[1] == 0.0) scal[1] = (double)(k0 + 1);
    {
        const int r = tid >> 1, cb = (tid & 1) * 64;
        double* g = S + (k0 + r) * ld + k0 + cb;
#pragma unroll
        for (int q = 0; q < 32; ++q) {
            const int c = cb + 2 * q;
            if (c + 1 <= r) {
                double2 v;
                v.x = A[r * LDA + c];
                v.y = A[r * LDA + c + 1];
                *reinterpret_cast<double2*>(g + 2 * q) = v;
            } else if (c == r) {
                g[2 * q] = A[r * LDA + c];
            }
        }
    }
}



__global__ void k_spin(long long cycles) {
    const long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < cycles) __builtin_amdgcn_s_sleep(2);
}

// instrumented copy of k_potrf128
__global__ __launch_bounds__(256) void k_potrf_ts(double* __restrict__ S, int64_t ld, int64_t k0,
                                                  double* __restrict__ dinv, double* __restrict__ scal, unsigned long long* ts) {
#define T0(i) do { if (threadIdx.x == 0) ts[i] = __builtin_amdgcn_s_memtime(); } while (0)
    T0(0);
    extern __shared__ __attribute__((aligned(16))) double smem[];
    // lower-triangle tiles only (80 KB, so the kernel fits beside a bulk-update workgroup on a CU):
    // element (r, c), r/16 >= c/16, at tile (r/16)(r/16+1)/2 + c/16, row r%16 (stride 17), col c%16
#define AT_(r, c) smem[(((r) >> 4) * (((r) >> 4) + 1) / 2 + ((c) >> 4)) * (IB * 17) + ((r) & 15) * 17 + ((c) & 15)]
    double* Dt = smem + POTRF_NT * IB * 17;  // [16][18] current inverse, transposed: Dt[c][i] = D_s[i][c]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int64_t dbase = (k0 / CB) * (CB / IB) * (IB * IB);
    bool ok = true;
    // store the final tiles (t, sc), t >= sc, of block column sc (diagonal tile: lower part only);
    // item i -> tile row t = sc + (i >> 7), row (i >> 3) & 15, columns 2 (i & 7)
    auto store_col = [&](int sc, int t0, int nthr) {
        for (int i = t0; i < (CB / IB - sc) * 128; i += nthr) {
            const int ti = sc + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
            double* g = S + (k0 + ti * IB + n) * ld + k0 + sc * IB + m;
            const double* t = smem + (ti * (ti + 1) / 2 + sc) * IB * 17 + n * 17 + m;
            if (ti > sc || m + 1 <= n) {
                double2 v;
                v.x = t[0];
                v.y = t[1];
                *reinterpret_cast<double2*>(g) = v;
            } else if (m == n) {
                g[0] = t[0];
            }
        }
    };
    {
        // wave 0 reads the rows of diagonal tile 0 straight into registers (issued first, so leaf 0
        // starts after one load latency); the other 35 lower tiles go through LDS: item i -> tile
        // p = 1 + (i >> 7), row (i >> 3) & 15, columns 2 (i & 7), all of a thread's loads in flight
        double a[IB], x[IB];
        if (wave == 0) {
#pragma unroll
            for (int h = 0; h < IB / 2; ++h) {
                const double2 v = *reinterpret_cast<const double2*>(S + (k0 + lr) * ld + k0 + 2 * h);
                a[2 * h] = v.x;
                a[2 * h + 1] = v.y;
            }
        }
        constexpr int NQ = ((POTRF_NT - 1) * 128 + 255) / 256;  // 18
        double2 v[NQ];
        int off[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int i = tid + 256 * q, p = 1 + (i >> 7), n = (i >> 3) & 15, m = (i & 7) * 2;
            int ti = 0, pp = p;
            while (pp > ti) { pp -= ti + 1; ++ti; }
            off[q] = -1;
            if (p < POTRF_NT) {
                v[q] = *reinterpret_cast<const double2*>(S + (k0 + ti * IB + n) * ld + k0 + pp * IB + m);
                off[q] = p * IB * 17 + n * 17 + m;
            }
        }
        if (wave == 0) {
            T0(1);
            ok = leaf_factor(a, x, lr);
            T0(2);
            if (lane < IB) put_leaf(smem, Dt, 0, lane, a, x);
        }
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (off[q] >= 0) {
                smem[off[q]] = v[q].x;
                smem[off[q] + 1] = v[q].y;
            }
        }
    }
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        __syncthreads();  // B1: L_ss, D_s in LDS; column s updated
        T0(3 + 4 * s);
        if (s == CB / IB - 1) break;
        if (wave > 0) copy_dinv(dinv + dbase + s * IB * IB, Dt, tid - 64, 192);  // D_s -> global
        // panel solve X_t = A_ts D_s^T: wave 0 tile s+1, waves 1..3 tiles s+2..7
        {
            const int t0 = (wave == 0) ? s + 1 : s + 1 + wave;
            const int step = (wave == 0) ? CB : 3;
            for (int t = t0; t < CB / IB; t += step) {
                const int r0 = t * IB;
                dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int kk = 0; kk < IB; kk += 4)
                    acc = mfma(AT_((r0 + lr), c0 + kk + lk), Dt[(kk + lk) * 18 + lr], acc);  // B[k][n] = D[n][k]
#pragma unroll
                for (int r = 0; r < 4; ++r) AT_((r0 + lk + 4 * r), c0 + lr) = acc[r];
            }
        }
        __syncthreads();  // B2: panel column s solved
        T0(4 + 4 * s);
        if (wave == 0) {
            // next diagonal tile, then its leaf factor
            const int R = c0 + IB;
            dbl4 acc;
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = AT_((R + lk + 4 * r), R + lr);
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4)
                acc = mfma(-AT_((R + lr), c0 + kk + lk), AT_((R + lr), c0 + kk + lk), acc);
#pragma unroll
            for (int r = 0; r < 4; ++r) AT_((R + lk + 4 * r), R + lr) = acc[r];
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            double a[IB], x[IB];
#pragma unroll
            for (int c = 0; c < IB; ++c) a[c] = AT_((R + lr), R + c);
            T0(5 + 4 * s);
            ok &= leaf_factor(a, x, lr);
            T0(6 + 4 * s);
            if (lane < IB) put_leaf(smem, Dt, s + 1, lane, a, x);  // D_s was last read before B2
        } else {
            // waves 1-3: the rest of the trailing update, by tile rows s+2 .. 7 dealt in snake order
            // (largest first) for balance; the tiles of a row go in pairs sharing the A operand,
            // two independent MFMA chains
            const int nrows = CB / IB - 2 - s;
            for (int i = 0; i < nrows; ++i) {
                const int w = ((i / 3) & 1) ? 3 - (i % 3) : 1 + (i % 3);
                if (w != wave) continue;
                const int R = (CB / IB - 1 - i) * IB;
                for (int C = c0 + IB; C <= R; C += 2 * IB) {
                    const bool two = C + IB <= R;
                    dbl4 acc1, acc2 = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc1[r] = AT_((R + lk + 4 * r), C + lr);
                    if (two)
#pragma unroll
                        for (int r = 0; r < 4; ++r) acc2[r] = AT_((R + lk + 4 * r), C + IB + lr);
#pragma unroll
                    for (int kk = 0; kk < IB; kk += 4) {
                        const double av = -AT_((R + lr), c0 + kk + lk);
                        acc1 = mfma(av, AT_((C + lr), c0 + kk + lk), acc1);
                        if (two) acc2 = mfma(av, AT_((C + IB + lr), c0 + kk + lk), acc2);
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r) AT_((R + lk + 4 * r), C + lr) = acc1[r];
                    if (two)
#pragma unroll
                        for (int r = 0; r < 4; ++r) AT_((R + lk + 4 * r), C + IB + lr) = acc2[r];
                }
            }
            store_col(s, tid - 64, 192);  // block column s is final: write it out behind the update
        }
    }
    if (!ok && lane == 0 && scal[1] == 0.0) scal[1] = (double)(k0 + 1);
    store_col(CB / IB - 1, tid, 256);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    T0(40);
    copy_dinv(dinv + dbase + (CB / IB - 1) * IB * IB, Dt, tid, 256);
#undef AT_
#undef T0
}



// end of instrumented copy
static double check(const std::vector<double>& L, const std::vector<double>& A0, int n, int ld) {
    // || L L' - A0 ||_max / ||A0||_max over the lower triangle
    double err = 0, mx = 0;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            double s = 0;
            for (int k = 0; k <= j; ++k) s += L[i * ld + k] * L[j * ld + k];
            err = fmax(err, fabs(s - A0[i * ld + j]));
            mx = fmax(mx, fabs(A0[i * ld + j]));
        }
    return err / mx;
}

template <typename F>
static float time_kernel(F launch, double* dS, const std::vector<double>& A0, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float tot = 0;
    for (int r = 0; r < reps; ++r) {
        (void)hipMemcpy(dS, A0.data(), A0.size() * 8, hipMemcpyHostToDevice);
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r > 0) tot += ms;
    }
    return 1e3f * tot / (reps - 1);
}

int main() {
    const int n = 128, ld = 256;
    std::vector<double> A0((size_t)n * ld, 0.0);
    unsigned s = 12345;
    std::vector<double> B((size_t)n * n);
    for (auto& b : B) { s = s * 1664525u + 1013904223u; b = (s >> 8) * (1.0 / 16777216.0) - 0.5; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double v = 0;
            for (int k = 0; k < n; ++k) v += B[i * n + k] * B[j * n + k];
            A0[i * ld + j] = v + (i == j ? n : 0);
        }
    double *dS, *dinv, *scal;
    unsigned long long* dts;
    CK(hipMalloc(&dS, A0.size() * 8));
    CK(hipMalloc(&dinv, 8 * 256 * 8));
    CK(hipMalloc(&scal, 16 * 8));
    CK(hipMalloc(&dts, 64 * 8));
    CK(hipMemset(scal, 0, 16 * 8));
    const size_t lds = sizeof(double) * (CB * LDA + IB * 17 + IB);
    CK(hipFuncSetAttribute((const void*)k_potrf128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)POTRF_LDS));
    CK(hipFuncSetAttribute((const void*)k_potrf_prof, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    std::vector<double> L(A0.size());
    float t = time_kernel([&] { k_potrf128<<<1, 256, POTRF_LDS>>>(dS, ld, 0, dinv, scal); }, dS, A0, 20);
    CK(hipMemcpy(L.data(), dS, L.size() * 8, hipMemcpyDeviceToHost));
    printf("k_potrf128        %8.2f us  err %.2e\n", t, check(L, A0, n, ld));
    t = time_kernel([&] { k_potrf_prof<<<1, 256, lds>>>(dS, ld, 0, dinv, scal, dts); }, dS, A0, 20);
    CK(hipMemcpy(L.data(), dS, L.size() * 8, hipMemcpyDeviceToHost));
    printf("k_potrf_prof      %8.2f us  err %.2e\n", t, check(L, A0, n, ld));
    unsigned long long ts[64];
    CK(hipMemcpy(ts, dts, sizeof ts, hipMemcpyDeviceToHost));
    printf("  load %llu cycles; alone: %llu cycles over %.2f us = %.2f GHz\n", ts[1] - ts[0], ts[40] - ts[0], t, (ts[40] - ts[0]) / (1e3 * t));
    unsigned long long fa = 0, fb = 0, fc = 0, fd = 0;
    for (int q = 0; q < 8; ++q) {
        unsigned long long a = ts[2 + 4 * q] - (q ? ts[1 + 4 * q] : ts[1]);
        unsigned long long b = ts[3 + 4 * q] - ts[2 + 4 * q];
        unsigned long long c = ts[4 + 4 * q] - ts[3 + 4 * q];
        unsigned long long d = ts[5 + 4 * q] - ts[4 + 4 * q];
        fa += a; fb += b; fc += c; fd += d;
        printf("  s=%d factor %6llu  inverse %6llu  panel %6llu  update %6llu\n", q, a, b, c, d);
    }
    printf("  totals factor %llu inverse %llu panel %llu update %llu store %llu  all %llu\n", fa, fb, fc, fd,
           ts[40] - ts[33], ts[40] - ts[0]);
    {
        CK(hipFuncSetAttribute((const void*)k_potrf_ts, hipFuncAttributeMaxDynamicSharedMemorySize, (int)POTRF_LDS));
        float tt = time_kernel([&] { k_potrf_ts<<<1, 256, POTRF_LDS>>>(dS, ld, 0, dinv, scal, dts); }, dS, A0, 5);
        unsigned long long q[64];
        CK(hipMemcpy(q, dts, sizeof q, hipMemcpyDeviceToHost));
        printf("potrf_ts %.2f us: load->leaf0 start %llu, leaf0 %llu, to B1 %llu\n", tt, q[1] - q[0], q[2] - q[1], q[3] - q[2]);
        for (int s = 0; s < 7; ++s)
            printf("  s%d: B1->B2 (panel) %llu | B2->leaf start (diag upd) %llu | leaf %llu | leaf end->B1 %llu\n", s,
                   q[4 + 4 * s] - q[3 + 4 * s], q[5 + 4 * s] - q[4 + 4 * s], q[6 + 4 * s] - q[5 + 4 * s],
                   q[7 + 4 * s] - q[6 + 4 * s]);
        printf("  end (store + drain) %llu, total %llu cycles\n", q[40] - q[31], q[40] - q[0]);
    }
    // k_trsm128 on a tall panel (config-4 size): rows 128 .. 6144 of a 6144-wide matrix
    {
        const int64_t N = 6144, nb = N / CB;
        std::vector<double> P((size_t)(N + CB) * N);
        for (auto& v : P) { s = s * 1664525u + 1013904223u; v = (s >> 8) * (1.0 / 16777216.0) - 0.5; }
        for (int i = 0; i < CB; ++i)
            for (int j = 0; j < CB; ++j) P[(size_t)i * N + j] = A0[i * ld + j];
        double* dP;
        CK(hipMalloc(&dP, P.size() * 8));
        CK(hipMemcpy(dP, P.data(), P.size() * 8, hipMemcpyHostToDevice));
        CK(hipFuncSetAttribute((const void*)k_trsm128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TRSM_LDS));
        k_potrf128<<<1, 256, POTRF_LDS>>>(dP, N, 0, dinv, scal);
        CK(hipDeviceSynchronize());
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        float best = 1e9f;
        for (int r = 0; r < 10; ++r) {
            CK(hipEventRecord(e0));
            k_trsm128<<<(unsigned)(nb * 2), 256, TRSM_LDS>>>(dP, N, 0, CB, dinv);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = fminf(best, ms);
        }
        CK(hipFuncSetAttribute((const void*)k_trsm_prof, hipFuncAttributeMaxDynamicSharedMemorySize, (int)TRSM_LDS));
        k_trsm_prof<<<(unsigned)(nb * 2), 256, TRSM_LDS>>>(dP, N, 0, CB, dinv, dts);
        CK(hipDeviceSynchronize());
        unsigned long long tt[64];
        CK(hipMemcpy(tt, dts, sizeof tt, hipMemcpyDeviceToHost));
        printf("  trsm wg5: load %llu compute %llu store %llu\n", tt[1] - tt[0], tt[2] - tt[1], tt[3] - tt[2]);
        printf("k_trsm128 (%lld rows)  %8.2f us (best of 10, repeated in place)\n", (long long)(nb * CB), 1e3f * best);
        CK(hipFree(dP));
    }
    // contention: a bulk k_syrk128 grid on a low-priority stream, potrf on a high-priority one
    {
        const int64_t N = 6144, nb = N / CB - 1;
        double* dM;
        CK(hipMalloc(&dM, (size_t)(N + CB) * N * 8));
        CK(hipMemset(dM, 0, (size_t)(N + CB) * N * 8));
        for (int i = 0; i < CB; ++i) CK(hipMemcpy(dM + (size_t)i * N, A0.data() + i * ld, CB * 8, hipMemcpyHostToDevice));
        int lo, hi;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t sA, sB;
        CK(hipStreamCreateWithPriority(&sA, hipStreamNonBlocking, hi));
        CK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, lo));
        CK(hipFuncSetAttribute((const void*)k_potrf_old, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(double) * (CB * LDA + IB * 17 + IB))));
        hipEvent_t a0, a1, b0, b1;
        CK(hipEventCreate(&a0)); CK(hipEventCreate(&a1)); CK(hipEventCreate(&b0)); CK(hipEventCreate(&b1));
        int64_t nt = 0;
        for (int64_t j = 2; j < nb; ++j) nt += nb - j + 1;
        CK(hipFuncSetAttribute((const void*)k_potrf_prof, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(sizeof(double) * (CB * LDA + IB * 17 + IB))));
        for (int variant = 0; variant < 3; ++variant) {
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(b0, sB));
                k_syrk128<<<(unsigned)nt, 256, 0, sB>>>(dM, N, 0, nb, 2, nt);
                CK(hipEventRecord(b1, sB));
                // give the bulk grid a head start, then the critical kernel
                k_spin<<<1, 64, 0, sA>>>(20000);
                CK(hipEventRecord(a0, sA));
                if (variant == 0) k_potrf_old<<<1, 256, sizeof(double) * (CB * LDA + IB * 17 + IB), sA>>>(dM, N, 0, dinv, scal);
                else if (variant == 1) k_potrf128<<<1, 256, POTRF_LDS, sA>>>(dM, N, 0, dinv, scal);
                else k_potrf_prof<<<1, 256, sizeof(double) * (CB * LDA + IB * 17 + IB), sA>>>(dM, N, 0, dinv, scal, dts);
                CK(hipEventRecord(a1, sA));
                CK(hipDeviceSynchronize());
                float ta, tb;
                CK(hipEventElapsedTime(&ta, a0, a1));
                CK(hipEventElapsedTime(&tb, b0, b1));
                unsigned long long tq[64];
                CK(hipMemcpy(tq, dts, sizeof tq, hipMemcpyDeviceToHost));
                printf("  contention %s: potrf %.1f us, bulk syrk (%lld tiles) %.1f us%s", variant == 0 ? "old(135KB)" : variant == 1 ? "new(80KB)" : "prof", 1e3f * ta, (long long)nt, 1e3f * tb, variant == 2 ? "" : "\n");
                if (variant == 2) printf("  -> %llu shader cycles = %.2f GHz over the kernel\n", tq[40] - tq[0], (tq[40] - tq[0]) / (1e3 * ta));
            }
        }
        CK(hipFree(dM));
    }
    {
        const int nn = 1 << 20;
        std::vector<double> h(nn), o0(nn), o1(nn), o2(nn);
        unsigned z = 777;
        for (auto& v : h) { z = z * 1664525u + 1013904223u; v = std::ldexp(1.0 + (z >> 8) / 16777216.0, (int)(z % 60) - 30); }
        double *dd, *d0, *d1, *d2;
        CK(hipMalloc(&dd, nn * 8)); CK(hipMalloc(&d0, nn * 8)); CK(hipMalloc(&d1, nn * 8)); CK(hipMalloc(&d2, nn * 8));
        CK(hipMemcpy(dd, h.data(), nn * 8, hipMemcpyHostToDevice));
        k_rsq_acc<<<nn / 256, 256>>>(dd, d0, d1, d2, nn);
        CK(hipMemcpy(o0.data(), d0, nn * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o1.data(), d1, nn * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o2.data(), d2, nn * 8, hipMemcpyDeviceToHost));
        double e0 = 0, e1 = 0, e2 = 0;
        for (int i = 0; i < nn; ++i) {
            long double ref = 1.0L / sqrtl((long double)h[i]);
            e0 = fmax(e0, (double)fabsl((o0[i] - ref) / ref));
            e1 = fmax(e1, (double)fabsl((o1[i] - ref) / ref));
            e2 = fmax(e2, (double)fabsl((o2[i] - ref) / ref));
        }
        printf("rsq rel err: raw %.3e  1 newton %.3e  2 newton %.3e (eps %.3e)\n", e0, e1, e2, 2.220446e-16);
    }
    return 0;
}
