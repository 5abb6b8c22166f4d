// fba_chol.hip -- dense fp64 Cholesky of the reduced camera system on gfx950 (MI355X).
//
// The reference inverts the bordered normal matrix explicitly, Cx = [N G; G' 0]^-1
// (main.m:428-440).  Here the tie points have already been eliminated (Schur complement), the
// border is folded in as M = S + G W G' (SPD whenever the bordered matrix is nonsingular; W = one
// equilibrating weight per constraint column, fba_kernels.hip k_border_weights), and
//   M = L L'        right-looking blocked Cholesky, NB = 64:
//                     k_potrf_diag   64x64 diagonal block in LDS (one workgroup)
//                     k_trsm_panel   rows below the diagonal block, one thread per row
//                     k_syrk_update  trailing update C -= L_i L_j' on v_mfma_f64_16x16x4_f64
//   forward solve    the right-hand sides [r | G W^1/2] are stored as extra ROWS below M, so the
//                    factorisation's panel solves compute Y' = (L^-1 B)' as a by-product
//   border combine   H = Z'Z, h = Z'y, k = -H^-1 h, y <- y + Z k      (Z, y = forward-solved G W^1/2, r)
//   backward solve   L' x = y, one launch per block row (k_trsv_bwd)
// so delta_c = -x = -M^-1 (r + G W^1/2 k) satisfies [S G; G' 0][delta; W^1/2 k] = [-r; 0] as the
// reference's bordered system does.
#include "fba_internal.h"

namespace fba {

typedef double dbl4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_potrf_diag(double* __restrict__ S, int64_t ld, int64_t k0,
                                                    double* __restrict__ scal) {
    __shared__ double A[64][65];
    const int tid = threadIdx.x;
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int r = idx >> 6, c = idx & 63;
        A[r][c] = S[(k0 + r) * ld + k0 + c];
    }
    __syncthreads();
    for (int j = 0; j < 64; ++j) {
        if (tid == 0) {
            double d = A[j][j];
            if (!(d > 0.0)) {
                if (scal[1] == 0.0) scal[1] = (double)(k0 + j + 1);
                d = 1.0;
            }
            A[j][j] = sqrt(d);
        }
        __syncthreads();
        if (tid > j && tid < 64) A[tid][j] /= A[j][j];
        __syncthreads();
        for (int idx = tid; idx < 64 * 64; idx += 256) {
            const int i = idx >> 6, l = idx & 63;
            if (l > j && i >= l) A[i][l] -= A[i][j] * A[l][j];
        }
        __syncthreads();
    }
    for (int idx = tid; idx < 64 * 64; idx += 256) {
        const int r = idx >> 6, c = idx & 63;
        if (c <= r) S[(k0 + r) * ld + k0 + c] = A[r][c];
    }
}

// rows [row0, row0 + 64*gridDim.x): A_ik <- A_ik L_kk^-T  (one thread per row)
__global__ __launch_bounds__(64) void k_trsm_panel(double* __restrict__ S, int64_t ld, int64_t k0, int64_t row0) {
    __shared__ double Lk[64][65];
    __shared__ double inv[64];
    const int tid = threadIdx.x;
    for (int c = 0; c < 64; ++c) Lk[tid][c] = S[(k0 + tid) * ld + k0 + c];
    __syncthreads();
    inv[tid] = 1.0 / Lk[tid][tid];
    __syncthreads();
    const int64_t row = row0 + (int64_t)blockIdx.x * 64 + tid;
    double* a = S + row * ld + k0;
    double x[64];
#pragma unroll
    for (int j = 0; j < 64; ++j) x[j] = a[j];
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        double s = x[j];
#pragma unroll
        for (int m = 0; m < j; ++m) s -= x[m] * Lk[j][m];
        x[j] = s * inv[j];
    }
#pragma unroll
    for (int j = 0; j < 64; ++j) a[j] = x[j];
}

// trailing update of block (i, j), j <= i, both below panel kb; i == nb is the RHS block row.
// 256 threads = 4 waves, each wave a 32x32 quadrant = 2x2 tiles of 16x16 (v_mfma_f64_16x16x4_f64).
__global__ __launch_bounds__(256) void k_syrk_update(double* __restrict__ S, int64_t ld, int64_t kb, int64_t nb) {
    const int64_t bi = kb + 1 + blockIdx.y;
    const int64_t bj = kb + 1 + blockIdx.x;
    if (bi < nb && bj > bi) return;
    __shared__ double As[64][66];
    __shared__ double Bs[64][66];
    const int tid = threadIdx.x;
    const int64_t k0 = kb * 64;
    {
        const int r = tid >> 2, q = (tid & 3) * 16;
        const double* ga = S + (bi * 64 + r) * ld + k0 + q;
        const double* gb = S + (bj * 64 + r) * ld + k0 + q;
#pragma unroll
        for (int c = 0; c < 16; c += 2) {
            const double2 va = *reinterpret_cast<const double2*>(ga + c);
            const double2 vb = *reinterpret_cast<const double2*>(gb + c);
            As[r][q + c] = va.x; As[r][q + c + 1] = va.y;
            Bs[r][q + c] = vb.x; Bs[r][q + c + 1] = vb.y;
        }
    }
    __syncthreads();
    const int wave = tid >> 6, lane = tid & 63;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    const int lr = lane & 15, lk = lane >> 4;
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int kk = 0; kk < 64; kk += 4) {
        double av[2], bv[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            av[t] = As[wr + t * 16 + lr][kk + lk];
            bv[t] = Bs[wc + t * 16 + lr][kk + lk];
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    // D layout (f64 16x16x4): lane holds D[row = (lane>>4) + 4*r][col = lane & 15]
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = bi * 64 + wr + a * 16 + lk + 4 * r;
                const int64_t col = bj * 64 + wc + b * 16 + lr;
                S[row * ld + col] -= acc[a][b][r];
            }
}

// ------------------------------------------------------------------------------------------------
// border combine (inner constraints): RHS rows n_pad + 0 (y) and n_pad + 1..7 (Z), length n
__global__ __launch_bounds__(256) void k_border_combine(double* __restrict__ S, int64_t ld, int64_t n_pad) {
    __shared__ double red[256];
    __shared__ double H[7][8];
    __shared__ double kk[7];
    const int tid = threadIdx.x;
    const double* y = S + n_pad * ld;
    for (int a = 0; a < 7; ++a) {
        const double* za = S + (n_pad + 1 + a) * ld;
        for (int b = 0; b < 8; ++b) {
            if (b > 0 && b - 1 < a) continue;  // symmetric: H[a][b-1] = H[b-1][a]
            const double* zb = (b == 0) ? y : S + (n_pad + b) * ld;
            double acc = 0.0;
            for (int64_t i = tid; i < n_pad; i += 256) acc += za[i] * zb[i];
            red[tid] = acc;
            __syncthreads();
            for (int w = 128; w > 0; w >>= 1) {
                if (tid < w) red[tid] += red[tid + w];
                __syncthreads();
            }
            if (tid == 0) {
                H[a][b] = red[0];
                if (b > 0) H[b - 1][a + 1] = red[0];
            }
            __syncthreads();
        }
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

// backward solve step: x_kb = L_kbkb^-T y_kb (every block redundantly), then block jb < kb updates
// y_jb -= L_{kb,jb}^T x_kb; block jb == kb stores x_kb.  One wave per block.
__global__ __launch_bounds__(64) void k_trsv_bwd(double* __restrict__ S, int64_t ld, int64_t n_pad, int64_t kb,
                                                 double* __restrict__ X) {
    __shared__ double Lk[64][65];
    __shared__ double xs[64];
    const int lane = threadIdx.x;
    const int64_t k0 = kb * 64;
    for (int r = 0; r < 64; ++r) Lk[r][lane] = S[(k0 + r) * ld + k0 + lane];
    double* y = S + n_pad * ld;
    double yl = y[k0 + lane];
    __syncthreads();
    for (int i = 63; i >= 0; --i) {
        if (lane == i) xs[i] = yl / Lk[i][i];
        __syncthreads();
        if (lane < i) yl -= Lk[i][lane] * xs[i];
    }
    __syncthreads();
    const int64_t jb = blockIdx.x;
    if (jb == kb) {
        X[k0 + lane] = xs[lane];
        return;
    }
    // y_jb[c] -= sum_r L[k0 + r][jb*64 + c] * x[r]
    double acc = 0.0;
    const double* Lr = S + k0 * ld + jb * 64 + lane;
    for (int r = 0; r < 64; ++r) acc += Lr[r * ld] * xs[r];
    y[jb * 64 + lane] -= acc;
}

__global__ void k_neg_copy(const double* __restrict__ X, double* __restrict__ delta, int64_t u_c) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < u_c) delta[i] = -X[i];
}

// ------------------------------------------------------------------------------------------------
int launch_cholesky(Ctx& c) {
    const int64_t ld = c.L.ld, nb = c.L.n_pad / NB;
    for (int64_t kb = 0; kb < nb; ++kb) {
        k_potrf_diag<<<1, 256, 0, c.stream>>>(c.d_S, ld, kb * NB, c.d_scal);
        k_trsm_panel<<<(unsigned)(nb - kb), 64, 0, c.stream>>>(c.d_S, ld, kb * NB, (kb + 1) * NB);
        const int64_t m = nb - kb - 1;
        if (m > 0) k_syrk_update<<<dim3((unsigned)m, (unsigned)(m + 1)), 256, 0, c.stream>>>(c.d_S, ld, kb, nb);
    }
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_backward(Ctx& c) {
    const int64_t ld = c.L.ld, nb = c.L.n_pad / NB;
    if (c.set.inner_constraints) k_border_combine<<<1, 256, 0, c.stream>>>(c.d_S, ld, c.L.n_pad);
    for (int64_t kb = nb - 1; kb >= 0; --kb)
        k_trsv_bwd<<<(unsigned)(kb + 1), 64, 0, c.stream>>>(c.d_S, ld, c.L.n_pad, kb, c.d_X);
    k_neg_copy<<<(unsigned)((c.L.u_c + 255) / 256), 256, 0, c.stream>>>(c.d_X, c.d_delta, c.L.u_c);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

}  // namespace fba
