// fba_cov.hip -- post-fit covariance of the unknowns on the device (gfx950 / MI355X).
//
// The reference keeps Cx = the (bordered) inverse of the normal matrix of the last iteration
// (main.m:428-444), its correlation matrix (main.m:446-456, before the distortion de-scaling), the
// diagonal de-scaling of Cx for the distortion terms (main.m:460-482) and Cx *= sigma0^2 (main.m:602);
// the .out/.par writers read sqrt(diag Cx) and small correlation sub-blocks (main.m:711-880).  Dense,
// that is a u x u inverse (u = 156,010 at config 4).  Here only the entries those outputs read are
// formed, from the block Cholesky factor M = L L' the last iteration left in S (fba_chol.hip):
//
//   selected inversion  Q = M^-1 on the block pattern of L (Takahashi recurrence), top level first:
//                         Y_i  = L_ik L_kk^-1                       (i in R_k, the block rows of column k)
//                         Q_ik = -sum_{j in R_k} Q_ij Y_j            (Q_ij of higher levels, already formed)
//                         Q_kk = L_kk^-T L_kk^-1 - sum_i Y_i' Q_ik
//                       written over L in place (a level only reads columns of higher levels);
//   border (inner constraints)  the bordered inverse's camera block is C = Q - Z H^-1 Z' with
//                       Z = L^-T [A~ B~] (14 backward solves of the forward-solved border rows) and H the
//                       14x14 matrix k_border_combine solves with (derivation: u = (I - F H^-1 F') y);
//                       without inner constraints C = Q;
//   camera side         diag C, and per image the (6 + cw)^2 block over its EOPs and its camera's
//                       unknowns (the reference's EOP/IOP correlation sub-matrices);
//   tie points          Cx_pp = V^-1 + T' C T with T = W V^-1 of the point's observations and camera
//                       (the Schur identity for the eliminated points), diagonal only.
// All sums run in a fixed order (no atomics).  The factor in S is consumed; the next iteration
// re-accumulates S from scratch (k_zero_blocks), so nothing else is affected.
#include "fba_internal.h"

#include <algorithm>
#include <array>
#include <vector>

namespace fba {

constexpr int CB = NB;  // 128

// ------------------------------------------------------------------------------------------------
// k_blk_gemm: one workgroup per PART of a task, C(128x128) = sum_t sign_t op(A_t) op(B_t), terms in list
// order, on v_mfma_f64_16x16x4_f64.  Operand/output bases: 0 = S (leading dimension ld), 1 = linv, 2 = Y
// scratch (both 128).  Four waves, each a 64x64 quarter of C as 4x4 MFMA tiles (64 accumulators per
// lane); K in slices of 16 staged through LDS (rows padded to 17 doubles: the 16 lanes of an MFMA
// operand read hit distinct banks), the next slice's global loads in flight during the current
// slice's MFMAs.  A phase of the selected inversion has few tasks at the top levels (one per block row
// of a separator column), each with many terms, so a task's slices are split into parts (split K) that
// run on workgroups of their own: a part writes C directly (one part) or its partial to a scratch
// block, and k_blk_combine adds a task's partials in part order.  Fixed order throughout -- bitwise
// reproducible.
// task record (int64): out offset, out base, first term, end term
// term record (int64): A offset, B offset, flags = baseA | baseB << 2 | tA << 4 | tB << 5 | neg << 6
// part record (int64): task, first slice, end slice (slice = term * 8 + K block), scratch slot (-1: C)
// combine record (int64): task, first slot, slots
// ------------------------------------------------------------------------------------------------
constexpr int KS = 16;
constexpr int LK = KS + 1;
typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_blk_gemm(const int64_t* __restrict__ parts, const int64_t* __restrict__ tasks,
                                                  const int64_t* __restrict__ terms, double* __restrict__ S, int64_t ld,
                                                  const double* __restrict__ linv, double* __restrict__ Y,
                                                  double* __restrict__ P) {
    __shared__ double As[CB * LK];  // op(A)[i][k0 + kk] at i * LK + kk (sign applied)
    __shared__ double Bs[CB * LK];  // op(B)[k0 + kk][j] at j * LK + kk
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, lr = lane & 15, lk = lane >> 4;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
    const int64_t* pk = parts + 4 * (int64_t)blockIdx.x;
    const int64_t* tk = tasks + 4 * pk[0];
    dbl4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int64_t t0 = tk[2];
    const int sl0 = (int)pk[1], nsl = (int)(pk[2] - pk[1]);
    // slice sl0 + s = (term t0 + (sl0 + s) / 8, k0 = 16 ((sl0 + s) % 8)): 8 elements of each operand per
    // thread, loaded one slice ahead (plain code, no lambda: captured register arrays went to scratch)
    double va[8], vb[8];
    int tt = 0;
#define BLK_FETCH(SL)                                                                                              \
    do {                                                                                                           \
        const int sl_ = (SL) + sl0;                                                                                \
        const int64_t* tr = terms + 3 * (t0 + sl_ / (CB / KS));                                                    \
        const int k0 = (sl_ % (CB / KS)) * KS;                                                                     \
        const int fl = (int)tr[2];                                                                                 \
        const int ba = fl & 3, bb = (fl >> 2) & 3, ta = (fl >> 4) & 1, tb = (fl >> 5) & 1;                         \
        const double sg = (fl >> 6) & 1 ? -1.0 : 1.0;                                                              \
        const double* A = (ba == 0 ? S : ba == 1 ? linv : Y) + tr[0];                                              \
        const double* B = (bb == 0 ? S : bb == 1 ? linv : Y) + tr[1];                                              \
        const int64_t lda = ba == 0 ? ld : CB, ldb = bb == 0 ? ld : CB;                                            \
        _Pragma("unroll") for (int q = 0; q < 8; ++q) {                                                            \
            const int idx = tid + 256 * q;                                                                         \
            va[q] = sg * (!ta ? A[(int64_t)(idx >> 4) * lda + k0 + (idx & 15)] : A[(int64_t)(k0 + (idx >> 7)) * lda + (idx & 127)]); \
            vb[q] = !tb ? B[(int64_t)(k0 + (idx >> 7)) * ldb + (idx & 127)] : B[(int64_t)(idx >> 4) * ldb + k0 + (idx & 15)]; \
        }                                                                                                          \
        tt = (ta ? 1 : 0) | (tb ? 2 : 0);                                                                          \
    } while (0)
    if (nsl > 0) BLK_FETCH(0);
    for (int sl = 0; sl < nsl; ++sl) {
        __syncthreads();  // the previous slice's MFMA reads are done
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int idx = tid + 256 * q;
            if (!(tt & 1)) As[(idx >> 4) * LK + (idx & 15)] = va[q];
            else As[(idx & 127) * LK + (idx >> 7)] = va[q];
            if (!(tt & 2)) Bs[(idx & 127) * LK + (idx >> 7)] = vb[q];
            else Bs[(idx >> 4) * LK + (idx & 15)] = vb[q];
        }
        __syncthreads();
        if (sl + 1 < nsl) BLK_FETCH(sl + 1);
#pragma unroll
        for (int kk = 0; kk < KS; kk += 4) {
            double av[4], bv[4];
#pragma unroll
            for (int a = 0; a < 4; ++a) av[a] = As[(wr + 16 * a + lr) * LK + kk + lk];
#pragma unroll
            for (int b = 0; b < 4; ++b) bv[b] = Bs[(wc + 16 * b + lr) * LK + kk + lk];
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
    }
#undef BLK_FETCH
    double* C = pk[3] >= 0 ? P + pk[3] * CB * CB : (tk[1] == 0 ? S : Y) + tk[0];
    const int64_t ldc = pk[3] < 0 && tk[1] == 0 ? ld : CB;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) C[(int64_t)(wr + 16 * a + lk + 4 * r) * ldc + wc + 16 * b + lr] = acc[a][b][r];
}

// k_blk_combine: C = P[first] + P[first + 1] + ... (part order) for a split task; blockIdx.y = which
// eighth of the 128 x 128 tile (16 rows), so a task split into many parts is summed by 8 workgroups
constexpr int COMB_SEG = 8;
__global__ __launch_bounds__(256) void k_blk_combine(const int64_t* __restrict__ combs, const int64_t* __restrict__ tasks,
                                                     double* __restrict__ S, int64_t ld, double* __restrict__ Y,
                                                     const double* __restrict__ P) {
    const int64_t* cb = combs + 3 * (int64_t)blockIdx.x;
    const int64_t* tk = tasks + 4 * cb[0];
    double* C = (tk[1] == 0 ? S : Y) + tk[0];
    const int64_t ldc = tk[1] == 0 ? ld : CB;
    constexpr int SEG = CB * CB / COMB_SEG, NQ = SEG / 2 / 256;  // 2048 doubles, 4 per thread
    const int64_t e0 = (int64_t)blockIdx.y * SEG;
    const double2* Pp = reinterpret_cast<const double2*>(P + cb[1] * CB * CB + e0);
    double2 acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = Pp[threadIdx.x + 256 * q];
    for (int64_t p = 1; p < cb[2]; ++p) {
        const double2* Pq = Pp + p * CB * CB / 2;
        double2 v[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) v[q] = Pq[threadIdx.x + 256 * q];
#pragma unroll
        for (int q = 0; q < NQ; ++q) { acc[q].x += v[q].x; acc[q].y += v[q].y; }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int64_t e = e0 + 2 * (threadIdx.x + 256 * q);
        const int64_t r = e / CB, cc = e % CB;
        *reinterpret_cast<double2*>(C + r * ldc + cc) = acc[q];
    }
}

// H^-1 of the 14x14 border system (k_border_combine's H = [[A'A - I, A'B], [B'A, B'B]] from the Gram of
// the forward-solved rows 1..14), Gauss-Jordan with partial pivoting, one wave; gpart as k_border_gram,
// or (gblk != nullptr) the per-column-block 16 x 16 Gram partials k_chol_flow's RHS panel halves leave,
// summed in block order -- the subtree split's, all-reduced over the ranks (a rank's S holds the
// forward-solved rows of its own and the top columns only).  The split forward-solves the B rows
// unscaled; H and Z (k_border_wz) then both miss the same diagonal scaling D, and Z' H^-1 Z is
// unchanged by it: Z' D (D H D)^-1 D Z = Z' H^-1 Z.
__global__ __launch_bounds__(64) void k_border_hinv(const double* __restrict__ gpart, int nseg,
                                                    const double* __restrict__ gblk, int nblk,
                                                    double* __restrict__ hinv) {
    __shared__ double g[15][15];
    __shared__ double H[14][28];
    const int tid = threadIdx.x;
    for (int e = tid; e < 120; e += 64) {
        int a = 0, rem = e;
        while (rem >= 15 - a) { rem -= 15 - a; ++a; }
        const int b = a + rem;
        double v = 0.0;
        if (gblk)
            for (int q = 0; q < nblk; ++q) v += gblk[(int64_t)q * 256 + a * 16 + b];
        else
            for (int q = 0; q < nseg; ++q) v += gpart[q * 120 + e];
        g[a][b] = g[b][a] = v;
    }
    __syncthreads();
    for (int i = tid; i < 14 * 28; i += 64) {
        const int r = i / 28, q = i % 28;
        H[r][q] = q < 14 ? g[1 + r][1 + q] - ((r == q && r < 7) ? 1.0 : 0.0) : (q - 14 == r ? 1.0 : 0.0);
    }
    __syncthreads();
    for (int col = 0; col < 14; ++col) {
        if (tid == 0) {
            int p = col;
            for (int r = col + 1; r < 14; ++r)
                if (fabs(H[r][col]) > fabs(H[p][col])) p = r;
            if (p != col)
                for (int q = 0; q < 28; ++q) { const double t = H[col][q]; H[col][q] = H[p][q]; H[p][q] = t; }
        }
        __syncthreads();
        const double piv = H[col][col];
        __syncthreads();
        if (tid < 28) H[col][tid] /= piv;
        __syncthreads();
        for (int i = tid; i < 14 * 28; i += 64) {
            const int r = i / 28, q = i % 28;
            if (r != col && q != col) H[r][q] -= H[r][col] * H[col][q];
        }
        __syncthreads();
        if (tid < 14 && tid != col) H[tid][col] = 0.0;
        __syncthreads();
    }
    for (int i = tid; i < 196; i += 64) hinv[i] = H[i / 14][14 + i % 14];
}

// Wz[a][i] = sum_b Hinv[a][b] Z[b][i]
__global__ void k_border_wz(const double* __restrict__ Z, const double* __restrict__ hinv, double* __restrict__ Wz,
                            int64_t n_pad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    double z[14];
#pragma unroll
    for (int b = 0; b < 14; ++b) z[b] = Z[b * n_pad + i];
#pragma unroll
    for (int a = 0; a < 14; ++a) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b < 14; ++b) s += hinv[a * 14 + b] * z[b];
        Wz[a * n_pad + i] = s;
    }
}

// C(r, c) of the camera-side system: Q from the selected inverse in S (lower blocks; diagonal blocks
// full), minus the border's low-rank term when nz = 14
__device__ __forceinline__ double cget(const double* __restrict__ S, int64_t ld, const double* __restrict__ Z,
                                       const double* __restrict__ Wz, int nz, int64_t n_pad, int64_t r, int64_t c) {
    const int64_t rr = (r / CB >= c / CB) ? r : c, cc = (r / CB >= c / CB) ? c : r;
    double v = S[rr * ld + cc];
    for (int a = 0; a < nz; ++a) v -= Z[a * n_pad + r] * Wz[a * n_pad + c];
    return v;
}

// camera side: diag C (de-scaled as main.m:460-482) and the (6+cw)^2 block of every image slot
__global__ void k_cov_cam(const double* __restrict__ S, int64_t ld, const double* __restrict__ Z,
                          const double* __restrict__ Wz, int nz, int64_t n_pad, int64_t u_c, int n_img, int cw, int nk,
                          const double* __restrict__ cam_tab, int cam_stride, double* __restrict__ cdiag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= u_c) return;
    double v = cget(S, ld, Z, Wz, nz, n_pad, i, i);
    const int64_t cb = 6 * (int64_t)n_img;
    if (i >= cb) {
        const int64_t k = (i - cb) / cw;
        const int q = (int)((i - cb) % cw);
        const double* ct = cam_tab + k * cam_stride;
        if (q >= 3 && q < 3 + nk) { const double s = ct[CAM_TAB_HDR + nk + (q - 3)]; v /= s * s; }
        else if (q >= 3 + nk) { const double s = ct[6]; v /= s * s; }
    }
    cdiag[i] = v;
}

__global__ __launch_bounds__(256) void k_cov_img(const double* __restrict__ S, int64_t ld, const double* __restrict__ Z,
                                                 const double* __restrict__ Wz, int nz, int64_t n_pad,
                                                 const int32_t* __restrict__ slots, const int32_t* __restrict__ cams,
                                                 int n_img, int cw, double* __restrict__ blk) {
    const int e = blockIdx.x;
    const int m = 6 + cw;
    const int64_t s = slots[e], k = cams[e];
    for (int idx = threadIdx.x; idx < m * m; idx += blockDim.x) {
        const int a = idx / m, b = idx % m;
        const int64_t r = a < 6 ? 6 * s + a : 6 * (int64_t)n_img + k * cw + (a - 6);
        const int64_t c = b < 6 ? 6 * s + b : 6 * (int64_t)n_img + k * cw + (b - 6);
        blk[(int64_t)e * m * m + idx] = cget(S, ld, Z, Wz, nz, n_pad, r, c);
    }
}

// tie points: one wave per local point.  Row groups g = 0..m-1 (observation g: 6 rows of its image,
// T = WT[o]), g = m (the camera: cw rows, Tc).  The entries of the group pairs (g >= h) are dealt to
// the lanes, which add sum T_g' C_gh T_h (diagonal of the 3x3 only, twice for g > h); lanes a < nz add the border term (Z_a' T)(Wz_a' T).  Fixed-order
// wave reduction.
__global__ __launch_bounds__(256) void k_cov_pts(const double* __restrict__ S, int64_t ld, const double* __restrict__ Z,
                                                 const double* __restrict__ Wz, int nz, int64_t n_pad,
                                                 const double* __restrict__ WT, const double* __restrict__ PT, int ps,
                                                 const int32_t* __restrict__ lp_start, const int32_t* __restrict__ lp_tie,
                                                 const int32_t* __restrict__ lp_cam, const int32_t* __restrict__ img,
                                                 int64_t n_lp, int n_img, int cw, int64_t u_c, double* __restrict__ pdiag) {
    const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (p >= n_lp) return;
    const int o0 = lp_start[p], m = lp_start[p + 1] - o0;
    const double* P = PT + p * ps;
    const double* Tc = P + 12 + 3 * cw;
    const int64_t cam0 = 6 * (int64_t)n_img + (int64_t)lp_cam[p] * cw;
    auto grp_rows = [&](int g, int64_t& r0, int& n, const double*& T) {
        if (g < m) { r0 = 6 * (int64_t)img[o0 + g]; n = 6; T = WT + (int64_t)(o0 + g) * 18; }
        else { r0 = cam0; n = cw; T = Tc; }
    };
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    const int ng = m + 1;
    // pairs g >= h only (diag(T_g' C_gh T_h) = diag(T_h' C_hg T_g): an off-diagonal pair counts twice),
    // their entries flattened and dealt to the lanes so that every lane issues the same number of
    // independent loads: first the image pairs (36 entries each, pair index = triangular (g, h)), then
    // camera x image g (6 cw), then camera x camera (cw^2)
    const int n_ii = m * (m + 1) / 2 * 36, n_ci = m * 6 * cw, n_all = n_ii + n_ci + cw * cw;
#pragma unroll 4
    for (int e = lane; e < n_all; e += 64) {
        int g, h, a, b;
        if (e < n_ii) {
            const int pr = e / 36, en = e - 36 * pr;
            g = 0;
            h = pr;
            while (h > g) { h -= g + 1; ++g; }
            a = en / 6;
            b = en - 6 * a;
        } else if (e < n_ii + n_ci) {
            const int e2 = e - n_ii;
            g = m;
            h = e2 / (6 * cw);
            const int en = e2 - 6 * cw * h;
            a = en / 6;
            b = en - 6 * a;
        } else {
            const int e3 = e - n_ii - n_ci;
            g = h = m;
            a = e3 / cw;
            b = e3 - cw * a;
        }
        int64_t r0, c0;
        int nr, nc;
        const double *Tg, *Th;
        grp_rows(g, r0, nr, Tg);
        grp_rows(h, c0, nc, Th);
        const int64_t r = r0 + a, c = c0 + b;
        const int64_t rr = (r / CB >= c / CB) ? r : c, cc = (r / CB >= c / CB) ? c : r;
        const double q = S[rr * ld + cc] * (g == h ? 1.0 : 2.0);
        acc0 += Tg[3 * a] * q * Th[3 * b];
        acc1 += Tg[3 * a + 1] * q * Th[3 * b + 1];
        acc2 += Tg[3 * a + 2] * q * Th[3 * b + 2];
    }
    if (lane < nz) {
        double z0 = 0, z1 = 0, z2 = 0, w0 = 0, w1 = 0, w2 = 0;
        for (int g = 0; g < ng; ++g) {
            int64_t r0;
            int nr;
            const double* Tg;
            grp_rows(g, r0, nr, Tg);
            for (int a = 0; a < nr; ++a) {
                const double zv = Z[lane * n_pad + r0 + a], wv = Wz[lane * n_pad + r0 + a];
                z0 += zv * Tg[3 * a]; z1 += zv * Tg[3 * a + 1]; z2 += zv * Tg[3 * a + 2];
                w0 += wv * Tg[3 * a]; w1 += wv * Tg[3 * a + 1]; w2 += wv * Tg[3 * a + 2];
            }
        }
        acc0 -= z0 * w0; acc1 -= z1 * w1; acc2 -= z2 * w2;
    }
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) {
        acc0 += __shfl_xor(acc0, w, 64);
        acc1 += __shfl_xor(acc1, w, 64);
        acc2 += __shfl_xor(acc2, w, 64);
    }
    if (lane == 0) {
        double* out = pdiag + 3 * (int64_t)lp_tie[p];
        out[0] = P[0] + acc0;
        out[1] = P[3] + acc1;
        out[2] = P[5] + acc2;
    }
}

// backward solve of one right-hand-side row (fba_chol.hip)
int launch_backward_rows(Ctx& c, int row0, int nrows, double* X);
int launch_obs_T(Ctx& c, double* T);
int launch_trtri_last(Ctx& c);
int launch_border_gram(Ctx& c, double* gpart, int* nseg);

// ------------------------------------------------------------------------------------------------
// driver: rebuilds the last linearisation's point tables (k_lin_point), the 14 border columns, the
// selected inverse level by level (top down), then the requested diagonals / blocks.
// Outputs (device, internal order): cdiag [u_c] (de-scaled camera-side diag C), pdiag [3 n_tie]
// (tie points of this rank), iblk [n_img_ref][(6+cw)^2] (raw C blocks per reference image).
// ------------------------------------------------------------------------------------------------
static bool s_split(const Ctx& c) { return c.sched.split; }

// (subtree split) every quantity below for a column of this rank's subtrees or of the top reads only
// such columns -- the Takahashi recurrence of column k reads Q over k's ancestors, the backward solve of
// column j the solutions of j's ancestors -- so the selected inverse runs on the whole block pattern as
// it stands: the other ranks' columns, never factored here, come out as garbage no output reads
// (fba_covariance keeps the entries of this rank's rows only)
int launch_covariance(Ctx& c, double* d_cdiag, double* d_pdiag, double* d_iblk, const int32_t* d_islot,
                      const int32_t* d_icam, int n_iblk) {
    const Layout& L = c.L;
    const int64_t ld = L.ld, n_pad = L.n_pad, nb = n_pad / CB;
    const Sched& s = c.sched;
    int rc;
    // point tables of the last linearisation (V^-1, T, Tc), as fba_residuals does
    if ((rc = launch_params(c, c.d_xlin)) || (rc = launch_linearize(c, c.d_xlin)) || (rc = launch_gen_tables(c, c.d_xlin)))
        return rc;

    // the last level's diagonal-block inverses (the iteration's backward solve does without them)
    if ((rc = launch_trtri_last(c))) return rc;
    const int nz = L.nrhs > 1 ? 14 : 0;
    double *d_Z = nullptr, *d_Wz = nullptr, *d_h = nullptr, *d_g = nullptr;
    // scratch from the context's covariance workspace (kept across calls: no allocation per call)
    int next_slot = 0;
    auto alloc = [&](double** p, size_t n) -> int { return ws_get(c, next_slot++, sizeof(double) * std::max<size_t>(n, 1), (void**)p); };
    auto cleanup = [&]() {};
    if (nz) {
        if ((rc = alloc(&d_Z, 14 * (size_t)n_pad)) || (rc = alloc(&d_Wz, 14 * (size_t)n_pad)) ||
            (rc = alloc(&d_h, 196)) || (rc = alloc(&d_g, 64 * 120))) { cleanup(); return rc; }
        int nseg = 0;
        // (subtree split: the Gram from the all-reduced per-block partials; another rank's columns of this
        // rank's RHS rows were never forward-solved here)
        if ((!s_split(c) && (rc = launch_border_gram(c, d_g, &nseg))) || (rc = launch_backward_rows(c, 1, 14, d_Z))) {
            cleanup();
            return rc;
        }
        k_border_hinv<<<1, 64, 0, c.stream>>>(d_g, nseg, s_split(c) ? c.d_gblk : nullptr, (int)nb, d_h);
        k_border_wz<<<(unsigned)((n_pad + 255) / 256), 256, 0, c.stream>>>(d_Z, d_h, d_Wz, n_pad);
    }

    // block rows R_k of every column (from the panel-solve records, half 0), RHS block row excluded
    std::vector<std::vector<int32_t>> R(nb);
    for (int w = 0; w < s.n_waves; ++w) {
        const int32_t* tr = s.buf.data() + s.w[w].trsm;
        for (int t = 0; t < s.w[w].ntrsm; ++t) {
            const int32_t k = tr[2 * t], r2 = tr[2 * t + 1];
            if ((r2 & 1) == 0 && r2 / 2 < nb) R[k].push_back(r2 / 2);
        }
    }
    size_t ymax = 1;
    for (int w = 0; w < s.n_waves; ++w) {
        size_t n = 0;
        const int32_t* cols = s.buf.data() + s.w[w].cols;
        for (int q = 0; q < s.w[w].ncol; ++q) n += R[cols[q]].size();
        ymax = std::max(ymax, n);
    }
    double* d_Y = nullptr;
    int64_t *d_tasks = nullptr, *d_terms = nullptr;
    if ((rc = alloc(&d_Y, ymax * CB * CB))) { cleanup(); return rc; }
    // every phase's task / term lists built up front and uploaded once; the phases (three per level,
    // top level first) then run back to back on the stream, no host round trip in between
    auto blk = [&](int64_t i, int64_t j) { return i * CB * ld + j * CB; };
    std::vector<int64_t> tasks, terms;
    std::vector<std::pair<int64_t, int64_t>> phases;  // [first task, end task)
    auto task = [&](int64_t out, int base) {
        tasks.insert(tasks.end(), {out, (int64_t)base, (int64_t)terms.size() / 3, 0});
    };
    auto term = [&](int64_t a, int64_t b, int fl) { terms.insert(terms.end(), {a, b, (int64_t)fl}); };
    auto close_task = [&]() { tasks.back() = (int64_t)terms.size() / 3; };
    auto phase = [&](int64_t first) { if ((int64_t)tasks.size() / 4 > first) phases.emplace_back(first, (int64_t)tasks.size() / 4); };
    enum { BS = 0, BL = 1, BY = 2 };
    for (int w = s.n_waves - 1; w >= 0; --w) {
        const int32_t* cols = s.buf.data() + s.w[w].cols;
        const int ncol = s.w[w].ncol;
        std::vector<size_t> ybase(ncol);
        size_t ny = 0;
        for (int q = 0; q < ncol; ++q) { ybase[q] = ny; ny += R[cols[q]].size(); }
        // (1) Y_i = L_ik Linv_k
        int64_t first = (int64_t)tasks.size() / 4;
        for (int q = 0; q < ncol; ++q) {
            const int64_t k = cols[q];
            for (size_t a = 0; a < R[k].size(); ++a) {
                task((int64_t)(ybase[q] + a) * CB * CB, BY);
                term(blk(R[k][a], k), k * CB * CB, BS | BL << 2);
                close_task();
            }
        }
        phase(first);
        // (2) Q_ik = -sum_j Q_ij Y_j
        first = (int64_t)tasks.size() / 4;
        for (int q = 0; q < ncol; ++q) {
            const int64_t k = cols[q];
            for (size_t a = 0; a < R[k].size(); ++a) {
                const int64_t i = R[k][a];
                task(blk(i, k), BS);
                for (size_t b = 0; b < R[k].size(); ++b) {
                    const int64_t j = R[k][b];
                    const int64_t y = (int64_t)(ybase[q] + b) * CB * CB;
                    if (i >= j) term(blk(i, j), y, BS | BY << 2 | 1 << 6);
                    else term(blk(j, i), y, BS | BY << 2 | 1 << 4 | 1 << 6);
                }
                close_task();
            }
        }
        phase(first);
        // (3) Q_kk = Linv_k' Linv_k - sum_i Y_i' Q_ik
        first = (int64_t)tasks.size() / 4;
        for (int q = 0; q < ncol; ++q) {
            const int64_t k = cols[q];
            task(blk(k, k), BS);
            term(k * CB * CB, k * CB * CB, BL | BL << 2 | 1 << 4);
            for (size_t a = 0; a < R[k].size(); ++a)
                term((int64_t)(ybase[q] + a) * CB * CB, blk(R[k][a], k), BY | BS << 2 | 1 << 4 | 1 << 6);
            close_task();
        }
        phase(first);
    }
    // split K: a phase's tasks split into parts of >= 4 slices so that the phase fills the chip (about
    // one part per CU), the partials of a split task in scratch slots (reused by every phase)
    std::vector<int64_t> parts, combs;
    std::vector<std::array<int64_t, 4>> pph;  // per phase: first part, end part, first combine, end combine
    int64_t max_slots = 0;
    const int64_t target = (int64_t)std::max(c.n_cu, 1);
    for (auto& ph : phases) {
        const int64_t ntask = ph.second - ph.first;
        const int64_t p0 = (int64_t)parts.size() / 4, c0 = (int64_t)combs.size() / 3;
        int64_t slot = 0;
        for (int64_t t = ph.first; t < ph.second; ++t) {
            const int64_t nsl = (tasks[4 * t + 3] - tasks[4 * t + 2]) * (CB / KS);
            const int64_t np = std::max<int64_t>(1, std::min<int64_t>((target + ntask - 1) / ntask, nsl / 4));
            if (np == 1) {
                parts.insert(parts.end(), {t, 0, nsl, -1});
                continue;
            }
            combs.insert(combs.end(), {t, slot, np});
            for (int64_t q = 0; q < np; ++q) parts.insert(parts.end(), {t, nsl * q / np, nsl * (q + 1) / np, slot++});
        }
        max_slots = std::max(max_slots, slot);
        pph.push_back({p0, (int64_t)parts.size() / 4, c0, (int64_t)combs.size() / 3});
    }
    double* d_P = nullptr;
    int64_t *d_parts = nullptr, *d_combs = nullptr;
    if ((rc = alloc((double**)&d_tasks, std::max<size_t>(tasks.size(), 1))) ||
        (rc = alloc((double**)&d_terms, std::max<size_t>(terms.size(), 1))) ||
        (rc = alloc((double**)&d_parts, std::max<size_t>(parts.size(), 1))) ||
        (rc = alloc((double**)&d_combs, std::max<size_t>(combs.size(), 1))) ||
        (rc = alloc(&d_P, (size_t)std::max<int64_t>(max_slots, 1) * CB * CB))) { cleanup(); return rc; }
    if (!tasks.empty()) {
        FBA_HIP(hipMemcpyAsync(d_tasks, tasks.data(), sizeof(int64_t) * tasks.size(), hipMemcpyHostToDevice, c.stream));
        FBA_HIP(hipMemcpyAsync(d_terms, terms.data(), sizeof(int64_t) * terms.size(), hipMemcpyHostToDevice, c.stream));
        FBA_HIP(hipMemcpyAsync(d_parts, parts.data(), sizeof(int64_t) * parts.size(), hipMemcpyHostToDevice, c.stream));
        if (!combs.empty())
            FBA_HIP(hipMemcpyAsync(d_combs, combs.data(), sizeof(int64_t) * combs.size(), hipMemcpyHostToDevice, c.stream));
    }
    for (auto& ph : pph) {
        k_blk_gemm<<<(unsigned)(ph[1] - ph[0]), 256, 0, c.stream>>>(d_parts + 4 * ph[0], d_tasks, d_terms, c.d_S, ld,
                                                                   c.d_linv, d_Y, d_P);
        if (ph[3] > ph[2])
            k_blk_combine<<<dim3((unsigned)(ph[3] - ph[2]), COMB_SEG), 256, 0, c.stream>>>(d_combs + 3 * ph[2], d_tasks, c.d_S, ld, d_Y, d_P);
    }
    FBA_HIP(hipGetLastError());

    if (d_cdiag)
        k_cov_cam<<<(unsigned)((L.u_c + 255) / 256), 256, 0, c.stream>>>(c.d_S, ld, d_Z, d_Wz, nz, n_pad, L.u_c, L.n_img,
                                                                         L.cw, L.nk, c.d_cam_tab, c.cam_tab_stride, d_cdiag);
    if (d_iblk && n_iblk > 0)
        k_cov_img<<<(unsigned)n_iblk, 256, 0, c.stream>>>(c.d_S, ld, d_Z, d_Wz, nz, n_pad, d_islot, d_icam, L.n_img, L.cw,
                                                          d_iblk);
    double* d_T = nullptr;  // T = W Vinv per tie observation, rebuilt from the records (OBS_REC)
    if (d_pdiag && c.n_lp > 0 &&
        ((rc = alloc(&d_T, (size_t)18 * std::max<int64_t>(c.n_obs_tie, 1))) || (rc = launch_obs_T(c, d_T)))) {
        cleanup();
        return rc;
    }
    if (d_pdiag && c.n_lp > 0)
        k_cov_pts<<<(unsigned)((c.n_lp + 3) / 4), 256, 0, c.stream>>>(c.d_S, ld, d_Z, d_Wz, nz, n_pad, d_T, c.d_pt_tab,
                                                                      c.pt_comp, c.d_lp_start, c.d_lp_tie, c.d_lp_cam,
                                                                      c.d_img, c.n_lp, L.n_img, L.cw, L.u_c, d_pdiag);
    FBA_HIP(hipGetLastError());
    if (d_pdiag && (rc = launch_gen_cov(c, d_Z, d_Wz, nz, d_pdiag))) { cleanup(); return rc; }
    FBA_HIP(hipStreamSynchronize(c.stream));
    cleanup();
    c.have_factor = false;
    return FBA_OK;
}

}  // namespace fba
