// fba_chol.hip -- dense fp64 Cholesky of the reduced camera system on gfx950 (MI355X).
//
// The reference inverts the bordered normal matrix explicitly, Cx = [N G; G' 0]^-1
// (main.m:428-440).  Here the tie points have already been eliminated (Schur complement), the
// border is folded in as M = S + G W G' (SPD whenever the bordered matrix is nonsingular; W = one
// equilibrating weight per constraint column, fba_kernels.hip k_border_weights), and
//
//   M = L L'        right-looking blocked Cholesky, NB = 128, depth-1 lookahead on two streams:
//     k_potrf128    the 128x128 diagonal block, LDS-resident in one workgroup: 8 sub-panels of 16
//                   (16x16 factor in registers with v_readlane broadcasts, its 16x16 inverse, then
//                   the in-block panel solve and trailing update on v_mfma_f64_16x16x4_f64); writes
//                   L_kk and the eight 16x16 inverses D_s = L_ss^-1 used by the solves below
//     k_trsm128     the panel below, X = A L_kk^-T by blocked substitution
//                   X_s = (A_s - sum_{t<s} X_t L_st^T) D_s^T: all MFMA, 16 rows per wave
//     k_syrk128     trailing update C -= X_i X_j^T, 128x128 tiles (4 waves x 64x64), K = 128
//                   staged through LDS in 32-deep slices, v_mfma_f64_16x16x4_f64
//   forward solve   the right-hand sides [r | G W^1/2] are stored as extra ROWS below M (one extra
//                   block row), so the panel solves compute Y' = (L^-1 B)' as a by-product
//   border combine  H = Z'Z, h = Z'y, k = -H^-1 h, y <- y + Z k      (Z, y = forward-solved G W^1/2, r)
//   backward solve  L' x = y with the 128x128 diagonal-block inverses (k_trtri128, all blocks in
//                   parallel), then one short launch per block row (k_bwd_step: two 128x128 GEMVs
//                   on the critical workgroup)
// so delta_c = -x = -M^-1 (r + G W^1/2 k) satisfies [S G; G' 0][delta; W^1/2 k] = [-r; 0] as the
// reference's bordered system does.
#include "fba_internal.h"

namespace fba {

typedef double dbl4 __attribute__((ext_vector_type(4)));

constexpr int CB = 128;   // outer block
constexpr int IB = 16;    // inner block (MFMA tile)
constexpr int LDA = 130;  // LDS row stride in doubles for 128-wide tiles: bank = (4r + 2k) mod 64

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// 1/sqrt(d) from v_rsq_f64 refined by two Newton steps (full double precision), no IEEE divide
__device__ __forceinline__ double rsqrt_d(double d) {
    double r = __builtin_amdgcn_rsq(d);
    r = r * (1.5 - 0.5 * d * r * r);
    r = r * (1.5 - 0.5 * d * r * r);
    return r;
}

__device__ __forceinline__ dbl4 mfma(double a, double b, dbl4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------------------------
// k_potrf128: factor the 128x128 diagonal block at (k0, k0); 256 threads
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_potrf128(double* __restrict__ S, int64_t ld, int64_t k0,
                                                  double* __restrict__ dinv, double* __restrict__ scal) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* A = smem;                  // [128][LDA]
    double* Dl = smem + CB * LDA;      // [16][17] current inverse D_s
    double* rd = Dl + IB * 17;         // [16] reciprocal diagonal of the current L_ss
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int idx = tid; idx < CB * CB / 2; idx += 256) {
        const int r = idx >> 6, c = (idx & 63) * 2;
        const double2 v = *reinterpret_cast<const double2*>(S + (k0 + r) * ld + k0 + c);
        A[r * LDA + c] = v.x;
        A[r * LDA + c + 1] = v.y;
    }
    __syncthreads();
    const int lr = lane & 15, lk = lane >> 4;
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        if (wave == 0) {
            // (a) 16x16 factor: lane i (< 16) holds row c0+i of the sub-block in registers
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
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the block's L is in LDS
            __builtin_amdgcn_wave_barrier();
            // (b) D_s = L_ss^-1: lane c (< 16) computes column c by forward substitution
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
        // (c) in-block panel solve: rows below the sub-block, X = A_s D_s^T  (16-row tiles)
        for (int t = s + 1 + wave; t < CB / IB; t += 4) {
            const int r0 = t * IB;
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4) {
                const double av = A[(r0 + lr) * LDA + c0 + kk + lk];
                const double bv = Dl[lr * 17 + kk + lk];  // B[k][n] = D[n][k]
                acc = mfma(av, bv, acc);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(r0 + lk + 4 * r) * LDA + c0 + lr] = acc[r];
        }
        __syncthreads();
        // (d) in-block trailing update of the lower tiles (ti >= tj > s), K = 16
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
    }
    for (int idx = tid; idx < CB * CB; idx += 256) {
        const int r = idx >> 7, c = idx & 127;
        if (c <= r) S[(k0 + r) * ld + k0 + c] = A[r * LDA + c];
    }
}

// ------------------------------------------------------------------------------------------------
// k_trsm128: rows [row0, row0 + 64*gridDim.x) of the panel at columns [k0, k0+128):
//   X = A L^-T by blocked substitution, X_s = (A_s - sum_{t<s} X_t L_st^T) D_s^T.
// 256 threads = 4 waves x 16 rows; each wave works on its own rows (no barriers).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_trsm128(double* __restrict__ S, int64_t ld, int64_t k0, int64_t row0,
                                                 const double* __restrict__ dinv) {
    __shared__ __attribute__((aligned(16))) double X[4][IB][LDA];
    __shared__ __attribute__((aligned(16))) double T[4][IB][17];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int64_t rbase = row0 + (int64_t)blockIdx.x * 64 + wave * IB;
    double* Xw = &X[wave][0][0];
    double* Tw = &T[wave][0][0];
    // load the wave's 16 x 128 panel rows
    for (int idx = lane; idx < IB * CB / 2; idx += 64) {
        const int r = idx >> 6, c = (idx & 63) * 2;
        const double2 v = *reinterpret_cast<const double2*>(S + (rbase + r) * ld + k0 + c);
        Xw[r * LDA + c] = v.x;
        Xw[r * LDA + c + 1] = v.y;
    }
    const double* L = S + k0 * ld + k0;
    const double* Dk = dinv + (k0 / CB) * (CB / IB) * (IB * IB);
    for (int s = 0; s < CB / IB; ++s) {
        const int c0 = s * IB;
        // Z = A_s - sum_{t<s} X_t L_st^T : output 16x16, K = 16 s
        dbl4 acc;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = Xw[(lk + 4 * r) * LDA + c0 + lr];
        for (int kk = 0; kk < c0; kk += 4) {
            const double av = -Xw[lr * LDA + kk + lk];
            const double bv = L[(c0 + lr) * ld + kk + lk];  // B[k][n] = L[c0+n][k]
            acc = mfma(av, bv, acc);
        }
        // Z (D layout) -> LDS, then X_s = Z D_s^T
#pragma unroll
        for (int r = 0; r < 4; ++r) Tw[(lk + 4 * r) * 17 + lr] = acc[r];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
        dbl4 out = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < IB; kk += 4) {
            const double av = Tw[lr * 17 + kk + lk];
            const double bv = Dk[s * IB * IB + lr * IB + kk + lk];  // B[k][n] = D[n][k]
            out = mfma(av, bv, out);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Xw[(lk + 4 * r) * LDA + c0 + lr] = out[r];
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_wave_barrier();
    }
    for (int idx = lane; idx < IB * CB / 2; idx += 64) {
        const int r = idx >> 6, c = (idx & 63) * 2;
        double2 v;
        v.x = Xw[r * LDA + c];
        v.y = Xw[r * LDA + c + 1];
        *reinterpret_cast<double2*>(S + (rbase + r) * ld + k0 + c) = v;
    }
}

// ------------------------------------------------------------------------------------------------
// k_syrk128: trailing update C(bi,bj) -= X_bi X_bj^T, 128x128 tiles, K = 128 in 32-deep slices.
// Tiles: block columns bj in [jlo, jlo + ncol), block rows bi in [bj, nb] (bi == nb: RHS block row).
// 4 waves, each a 64x64 quadrant = 4x4 MFMA tiles.  The accumulators start from C (its loads overlap
// the first slice), each next slice is prefetched into registers while the MFMAs of the current one
// run, and the epilogue is a plain store.
// ------------------------------------------------------------------------------------------------
constexpr int KS = 32;
constexpr int LDK = 34;   // LDS stride of a 32-deep slice: bank = (4r + 2k) mod 64, conflict-free

__global__ __launch_bounds__(256) void k_syrk128(double* __restrict__ S, int64_t ld, int64_t kb, int64_t nb,
                                                 int64_t jlo) {
    int64_t q = blockIdx.x, bj = jlo, bi = 0;
    for (;;) {
        const int64_t cnt = nb - bj + 1;
        if (q < cnt) { bi = bj + q; break; }
        q -= cnt;
        ++bj;
    }
    __shared__ __attribute__((aligned(16))) double As[CB][LDK];
    __shared__ __attribute__((aligned(16))) double Bs[CB][LDK];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
    const int64_t k0 = kb * CB;
    double* Cp = S + (bi * CB + wr + lk) * ld + bj * CB + wc + lr;
    dbl4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[a][b][r] = Cp[(a * 16 + 4 * r) * ld + b * 16];
    // staging: thread -> (row rr, 16 columns at cc) of the 128 x 32 slice, for A and B
    const int rr = tid >> 1, cc = (tid & 1) * 16;
    const double* ga = S + (bi * CB + rr) * ld + k0 + cc;
    const double* gb = S + (bj * CB + rr) * ld + k0 + cc;
    double2 pa[8], pb[8];
#pragma unroll
    for (int h = 0; h < 8; ++h) {
        pa[h] = *reinterpret_cast<const double2*>(ga + 2 * h);
        pb[h] = *reinterpret_cast<const double2*>(gb + 2 * h);
    }
    for (int ks = 0; ks < CB; ks += KS) {
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 8; ++h) {
            As[rr][cc + 2 * h] = pa[h].x; As[rr][cc + 2 * h + 1] = pa[h].y;
            Bs[rr][cc + 2 * h] = pb[h].x; Bs[rr][cc + 2 * h + 1] = pb[h].y;
        }
        __syncthreads();
        if (ks + KS < CB) {
#pragma unroll
            for (int h = 0; h < 8; ++h) {
                pa[h] = *reinterpret_cast<const double2*>(ga + ks + KS + 2 * h);
                pb[h] = *reinterpret_cast<const double2*>(gb + ks + KS + 2 * h);
            }
        }
#pragma unroll
        for (int kk = 0; kk < KS; kk += 4) {
            double av[4], bv[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                av[t] = -As[wr + t * 16 + lr][kk + lk];
                bv[t] = Bs[wc + t * 16 + lr][kk + lk];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = mfma(av[a], bv[b], acc[a][b]);
        }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) Cp[(a * 16 + 4 * r) * ld + b * 16] = acc[a][b][r];
}

// k_syrk_col64: the critical-path update of block column kb+1 (rows (kb+1)*128 .. (nb+1)*128) with
// 64x64 tiles, K = 128: 4x the workgroups of k_syrk128, a quarter of the latency each.
// Tile q: sub-row q >> 1 (64 rows), sub-column q & 1 of the 128-wide block column.
__global__ __launch_bounds__(256) void k_syrk_col64(double* __restrict__ S, int64_t ld, int64_t kb) {
    const int64_t r0 = (kb + 1) * CB + (int64_t)(blockIdx.x >> 1) * 64;
    const int64_t c0 = (kb + 1) * CB + (int64_t)(blockIdx.x & 1) * 64;
    __shared__ __attribute__((aligned(16))) double As[64][LDK];
    __shared__ __attribute__((aligned(16))) double Bs[64][LDK];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    const int64_t k0 = kb * CB;
    double* Cp = S + (r0 + wr + lk) * ld + c0 + wc + lr;
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[a][b][r] = Cp[(a * 16 + 4 * r) * ld + b * 16];
    const int rr = tid >> 2, cc = (tid & 3) * 8;
    const double* ga = S + (r0 + rr) * ld + k0 + cc;
    const double* gb = S + (c0 + rr) * ld + k0 + cc;
    double2 pa[4], pb[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
        pa[h] = *reinterpret_cast<const double2*>(ga + 2 * h);
        pb[h] = *reinterpret_cast<const double2*>(gb + 2 * h);
    }
    for (int ks = 0; ks < CB; ks += KS) {
        __syncthreads();
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            As[rr][cc + 2 * h] = pa[h].x; As[rr][cc + 2 * h + 1] = pa[h].y;
            Bs[rr][cc + 2 * h] = pb[h].x; Bs[rr][cc + 2 * h + 1] = pb[h].y;
        }
        __syncthreads();
        if (ks + KS < CB) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                pa[h] = *reinterpret_cast<const double2*>(ga + ks + KS + 2 * h);
                pb[h] = *reinterpret_cast<const double2*>(gb + ks + KS + 2 * h);
            }
        }
#pragma unroll
        for (int kk = 0; kk < KS; kk += 4) {
            double av[2], bv[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                av[t] = -As[wr + t * 16 + lr][kk + lk];
                bv[t] = Bs[wc + t * 16 + lr][kk + lk];
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = mfma(av[a], bv[b], acc[a][b]);
        }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) Cp[(a * 16 + 4 * r) * ld + b * 16] = acc[a][b][r];
}

static inline int64_t syrk_tiles(int64_t nb, int64_t jlo, int64_t ncol) {
    int64_t t = 0;
    for (int64_t j = jlo; j < jlo + ncol; ++j) t += nb - j + 1;
    return t;
}

// ------------------------------------------------------------------------------------------------
// border combine (inner constraints): RHS rows n_pad + 0 (y) and n_pad + 1..7 (Z), length n
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_border_combine(double* __restrict__ S, int64_t ld, int64_t n_pad) {
    __shared__ double red[8][256];
    __shared__ double H[7][8];
    __shared__ double kk[7];
    const int tid = threadIdx.x;
    const double* y = S + n_pad * ld;
    for (int a = 0; a < 7; ++a) {
        const double* za = S + (n_pad + 1 + a) * ld;
        double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int64_t i = tid; i < n_pad; i += 256) {
            const double z = za[i];
            acc[0] += z * y[i];
            for (int b = a; b < 7; ++b) acc[1 + b] += z * S[(n_pad + 1 + b) * ld + i];
        }
        for (int b = 0; b < 8; ++b) red[b][tid] = acc[b];
        __syncthreads();
        for (int w = 128; w > 0; w >>= 1) {
            if (tid < w)
                for (int b = 0; b < 8; ++b) red[b][tid] += red[b][tid + w];
            __syncthreads();
        }
        if (tid == 0) {
            H[a][0] = red[0][0];
            for (int b = a; b < 7; ++b) { H[a][1 + b] = red[1 + b][0]; H[b][1 + a] = red[1 + b][0]; }
        }
        __syncthreads();
    }
    if (tid == 0) {
        // solve H[:,1..7] k = -H[:,0]  (SPD 7x7; Gaussian elimination with partial pivoting)
        double A[7][8];
        for (int a = 0; a < 7; ++a) {
            for (int b = 0; b < 7; ++b) A[a][b] = H[a][b + 1];
            A[a][7] = -H[a][0];
        }
        for (int col = 0; col < 7; ++col) {
            int piv = col;
            for (int r = col + 1; r < 7; ++r)
                if (fabs(A[r][col]) > fabs(A[piv][col])) piv = r;
            if (piv != col)
                for (int b = 0; b < 8; ++b) {
                    const double t = A[col][b];
                    A[col][b] = A[piv][b];
                    A[piv][b] = t;
                }
            for (int r = col + 1; r < 7; ++r) {
                const double f = A[r][col] / A[col][col];
                for (int b = col; b < 8; ++b) A[r][b] -= f * A[col][b];
            }
        }
        for (int r = 6; r >= 0; --r) {
            double s = A[r][7];
            for (int b = r + 1; b < 7; ++b) s -= A[r][b] * kk[b];
            kk[r] = s / A[r][r];
        }
    }
    __syncthreads();
    double* yw = S + n_pad * ld;
    for (int64_t i = tid; i < n_pad; i += 256) {
        double v = yw[i];
        for (int m = 0; m < 7; ++m) v += S[(n_pad + 1 + m) * ld + i] * kk[m];
        yw[i] = v;
    }
}

// ------------------------------------------------------------------------------------------------
// k_trtri128: inverse of every 128x128 diagonal block of L (one workgroup per block, all blocks in
// parallel after the factorisation): block forward substitution on the 8x8 grid of 16x16 tiles,
// X_ii = D_i, X_ij = -D_i sum_{k=j}^{i-1} L_ik X_kj, on v_mfma_f64_16x16x4_f64.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_trtri128(const double* __restrict__ S, int64_t ld,
                                                  const double* __restrict__ dinv, double* __restrict__ linv) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* X = smem;                   // [128][LDA]
    double* Y = smem + CB * LDA;        // [4 waves][16][17]
    const int kb = blockIdx.x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 15, lk = lane >> 4;
    const double* L = S + (int64_t)kb * CB * ld + (int64_t)kb * CB;
    const double* Dk = dinv + (int64_t)kb * (CB / IB) * (IB * IB);
    for (int idx = tid; idx < CB * CB; idx += 256) {
        const int r = idx >> 7, c = idx & 127;
        X[r * LDA + c] = ((r >> 4) == (c >> 4)) ? Dk[(r >> 4) * IB * IB + (r & 15) * IB + (c & 15)] : 0.0;
    }
    __syncthreads();
    double* Yw = Y + wave * IB * 17;
    for (int i = 1; i < CB / IB; ++i) {
        for (int j = wave; j < i; j += 4) {
            dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
            for (int k = j; k < i; ++k) {
#pragma unroll
                for (int kk = 0; kk < IB; kk += 4) {
                    const double av = L[(int64_t)(IB * i + lr) * ld + IB * k + kk + lk];
                    const double bv = X[(IB * k + kk + lk) * LDA + IB * j + lr];
                    acc = mfma(av, bv, acc);
                }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) Yw[(lk + 4 * r) * 17 + lr] = acc[r];
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
            dbl4 out = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int kk = 0; kk < IB; kk += 4) {
                const double av = -Dk[i * IB * IB + lr * IB + kk + lk];
                const double bv = Yw[(kk + lk) * 17 + lr];
                out = mfma(av, bv, out);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) X[(IB * i + lk + 4 * r) * LDA + IB * j + lr] = out[r];
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
    }
    double* out = linv + (int64_t)kb * CB * CB;
    for (int idx = tid; idx < CB * CB; idx += 256) out[idx] = X[(idx >> 7) * LDA + (idx & 127)];
}

// ------------------------------------------------------------------------------------------------
// backward solve L' x = y with the diagonal-block inverses:
//   k_bwd_first  x_{nb-1} = Linv_{nb-1}^T y_{nb-1}
//   k_bwd_step   (kb): workgroup 0 (the critical one) y_{kb-1} -= L_{kb,kb-1}^T x_kb and then
//                x_{kb-1} = Linv_{kb-1}^T y_{kb-1}; workgroup 1+j updates y_j -= L_{kb,j}^T x_kb
// 256 threads = 128 columns x 2 halves of the 128 rows, halves summed in a fixed order.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ double gemv_t128(const double* __restrict__ M, int64_t ldm, const double* __restrict__ v,
                                            int tid, double* red) {
    const int c = tid & 127, h = tid >> 7;
    double acc = 0.0;
#pragma unroll 8
    for (int r = h * 64; r < h * 64 + 64; ++r) acc += M[(int64_t)r * ldm + c] * v[r];
    red[tid] = acc;
    __syncthreads();
    const double s = red[c] + red[128 + c];
    __syncthreads();
    return s;  // valid for every thread (column c = tid & 127)
}

__global__ __launch_bounds__(256) void k_bwd_first(const double* __restrict__ S, int64_t ld, int64_t n_pad, int64_t kb,
                                                   const double* __restrict__ linv, double* __restrict__ X) {
    __shared__ double ys[CB];
    __shared__ double red[256];
    const int tid = threadIdx.x;
    if (tid < CB) ys[tid] = S[n_pad * ld + kb * CB + tid];
    __syncthreads();
    const double x = gemv_t128(linv + kb * CB * CB, CB, ys, tid, red);
    if (tid < CB) X[kb * CB + tid] = x;
}

__global__ __launch_bounds__(256) void k_bwd_step(double* __restrict__ S, int64_t ld, int64_t n_pad, int64_t kb,
                                                  const double* __restrict__ linv, double* __restrict__ X) {
    __shared__ double xs[CB];
    __shared__ double ys[CB];
    __shared__ double red[256];
    const int tid = threadIdx.x;
    const int64_t k0 = kb * CB;
    double* y = S + n_pad * ld;
    if (tid < CB) xs[tid] = X[k0 + tid];
    __syncthreads();
    const int64_t j = blockIdx.x == 0 ? kb - 1 : (int64_t)blockIdx.x - 1;
    const double u = gemv_t128(S + k0 * ld + j * CB, ld, xs, tid, red);
    if (blockIdx.x != 0) {
        if (tid < CB) y[j * CB + tid] -= u;
        return;
    }
    if (tid < CB) ys[tid] = y[j * CB + tid] - u;
    __syncthreads();
    const double x = gemv_t128(linv + j * CB * CB, CB, ys, tid, red);
    if (tid < CB) X[j * CB + tid] = x;
}

__global__ void k_neg_copy(const double* __restrict__ X, double* __restrict__ delta, int64_t u_c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < u_c) delta[i] = -X[i];
}

// ------------------------------------------------------------------------------------------------
// Right-looking with depth-1 lookahead on two streams:
//   stream A (critical path): potrf(k) -> trsm(k) -> [wait rest(k-1)] -> col(k) -> potrf(k+1) ...
//   stream B (bulk):          [wait trsm(k)] -> rest(k)
// col(k) updates block column k+1 (the next panel), rest(k) the columns >= k+2; so the bulk update
// rest(k-1) runs concurrently with potrf(k) and trsm(k).
int launch_cholesky(Ctx& c) {
    const int64_t ld = c.L.ld, nb = c.L.n_pad / CB;
    const size_t lds_potrf = sizeof(double) * (CB * LDA + IB * 17 + IB);
    hipStream_t A = c.stream, B = c.stream2;
    for (int64_t kb = 0; kb < nb; ++kb) {
        k_potrf128<<<1, 256, lds_potrf, A>>>(c.d_S, ld, kb * CB, c.d_dinv, c.d_scal);
        // panel rows below the diagonal block, RHS block row included: (nb - kb) * 128 rows
        k_trsm128<<<(unsigned)((nb - kb) * 2), 256, 0, A>>>(c.d_S, ld, kb * CB, (kb + 1) * CB, c.d_dinv);
        FBA_HIP(hipEventRecord(c.ev_trsm[kb], A));
        const int64_t m = nb - kb - 1;  // trailing block columns
        if (m > 1) {
            FBA_HIP(hipStreamWaitEvent(B, c.ev_trsm[kb], 0));
            k_syrk128<<<(unsigned)syrk_tiles(nb, kb + 2, m - 1), 256, 0, B>>>(c.d_S, ld, kb, nb, kb + 2);
            FBA_HIP(hipEventRecord(c.ev_rest[kb], B));
        }
        if (m > 0) {
            if (kb > 0 && nb - kb > 1) FBA_HIP(hipStreamWaitEvent(A, c.ev_rest[kb - 1], 0));
            // block column kb+1: (nb - kb) block rows of 128 (RHS row included) x 2 sub-columns of 64
            k_syrk_col64<<<(unsigned)((nb - kb) * 4), 256, 0, A>>>(c.d_S, ld, kb);
        }
    }
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_backward(Ctx& c) {
    const int64_t ld = c.L.ld, nb = c.L.n_pad / CB;
    const size_t lds_trtri = sizeof(double) * (CB * LDA + 4 * IB * 17);
    if (c.set.inner_constraints) k_border_combine<<<1, 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad);
    k_trtri128<<<(unsigned)nb, 256, lds_trtri, c.stream>>>(c.d_S, ld, c.d_dinv, c.d_linv);
    k_bwd_first<<<1, 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad, nb - 1, c.d_linv, c.d_X);
    for (int64_t kb = nb - 1; kb >= 1; --kb)
        k_bwd_step<<<(unsigned)kb, 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad, kb, c.d_linv, c.d_X);
    k_neg_copy<<<(unsigned)((c.L.u_c + 255) / 256), 256, 0, c.stream>>>(c.d_X, c.d_delta, c.L.u_c);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int chol_setup(Ctx& c) {
    const size_t lds_potrf = sizeof(double) * (CB * LDA + IB * 17 + IB);
    FBA_HIP(hipFuncSetAttribute((const void*)k_potrf128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_potrf));
    const size_t lds_trtri = sizeof(double) * (CB * LDA + 4 * IB * 17);
    FBA_HIP(hipFuncSetAttribute((const void*)k_trtri128, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_trtri));
    const int64_t nb = c.L.n_pad / CB;
    FBA_HIP(hipStreamCreateWithFlags(&c.stream2, hipStreamNonBlocking));
    c.ev_trsm.assign(nb, nullptr);
    c.ev_rest.assign(nb, nullptr);
    for (int64_t k = 0; k < nb; ++k) {
        FBA_HIP(hipEventCreateWithFlags(&c.ev_trsm[k], hipEventDisableTiming));
        FBA_HIP(hipEventCreateWithFlags(&c.ev_rest[k], hipEventDisableTiming));
    }
    return FBA_OK;
}

}  // namespace fba
