// fba_general.hip -- the tie points the chunked fast path (k_lin_reduce) does not take.
//
// The reference accepts any PHO table: BuildAwG loops over every image point (BuildAwG.m:46), places
// each observation's IOP / distortion columns by that point's own camera (cam_num, :448-451), and its
// tie columns do not depend on the camera (:501-502); N = A'PA (main.m:424-425) then couples whatever
// the rows couple.  k_lin_reduce's chunks hold whole points of ONE camera, at most CHUNK_OBS
// observations each, at most one per image.  A "general" point -- seen through several cameras (a
// multi-camera rig sharing targets, main.m:323), by more images than a chunk holds, or measured twice
// in one image -- is reduced here instead, into the same fixed-order partial slots the k_red_*
// kernels sum (plus two block kinds only such points create), so the reduced system is the same
// Schur complement of the same normal equations:
//   k_lin_point     (fba_kernels.hip) the Jacobian rows of the general observations (J-only chunks)
//   k_gen_point     one wave per point: V = Jp'PJp, b = Jp'Pw over all its observations, V^-1, the
//                   factor R = L^-T, rb = R'b, vb = V^-1 b; per camera of the point ("gpc")
//                   Wc = Jc'PJp -> Uc = Wc R, Tc = Wc V^-1; per image of the point ("gimg")
//                   Ug = sum_o W_o R and sum_o W_o V^-1 (W_o = Je'PJp)
//   k_gen_keys      one thread per partial entry:
//                     pair (e1 > e2)        -Ug1 Ug2'                              -> ppart (k_red_pairs)
//                     image e               sum_o Je'PJe - Ug Ug', Je'Pw - Ug rb,
//                                           Jc'PJe - Uc Ug' (own camera)           -> ipart (k_red_images)
//                     image e x camera k'   -Uc_k' Ug'  (a camera other than e's)  -> xpart (k_red_gen)
//                     camera k              Jc'PJc - Uc Uc', Jc'Pw - Uc rb          -> cpart (k_red_cam)
//                     camera k1 x k2        -Uc_k1 Uc_k2'                           -> kpart (k_red_gen)
//   k_red_gen       the image x foreign-camera and camera x camera blocks, partials in slot order
//   k_gen_backsub   dp = -(vb + sum_gimg T_e' d_e + sum_gpc Tc' d_k)
// Every sum has a fixed association, so results stay bitwise reproducible.
#include "fba_internal.h"

namespace fba {

template <int NK>
struct GL {
    static constexpr int CW = 5 + NK, NJ = 9 + CW, JS = 2 * NJ + 2;
    static constexpr int NIMG = 27 + 6 * CW;           // image partial (LR<NK>::NIMG)
    static constexpr int NPK = CW * (CW + 1) / 2;
    static constexpr int NCAM = NPK + CW;              // camera partial (LR<NK>::NCAM)
    static constexpr int NX = 6 * CW, NKK = CW * CW;
    static constexpr int GC = 6 * CW;                  // gpc table: Uc 3CW | Tc 3CW
};
constexpr int GPT = 18;  // point table: Vinv 6 | R 6 | rb 3 | vb 3
constexpr int GUG = 36;  // gimg table: Ug 18 | T 18

// fixed xor-butterfly sum over the 64 lanes of a wave (every lane gets the sum)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) v += __shfl_xor(v, w, 64);
    return v;
}

// lower-triangle index q = a (a + 1) / 2 + b, a >= b
__device__ __forceinline__ void tri_ab(int q, int& a, int& b) {
    a = 0;
    while (q > a) { q -= a + 1; ++a; }
    b = q;
}

template <int NK>
__global__ __launch_bounds__(64) void k_gen_point(const double* __restrict__ J, const int32_t* __restrict__ A,
                                                  const GenPlan g, double* __restrict__ gpt, double* __restrict__ gcu,
                                                  double* __restrict__ gug, double px, double py) {
    using Q = GL<NK>;
    constexpr int CW = Q::CW, NJ = Q::NJ, JS = Q::JS, GC = Q::GC;
    const int q = blockIdx.x, l = threadIdx.x;
    const int o0 = A[g.g_obs + q], o1 = A[g.g_obs + q + 1];
    double V[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // V00 V01 V02 V11 V12 V22 b0 b1 b2
    for (int o = o0 + l; o < o1; o += 64) {
        const double* Jo = J + (int64_t)o * JS;
#pragma unroll
        for (int row = 0; row < 2; ++row) {
            const double pr = row ? py : px;
            const double j0 = Jo[row * NJ + 6 + CW], j1 = Jo[row * NJ + 7 + CW], j2 = Jo[row * NJ + 8 + CW];
            const double wv = Jo[2 * NJ + row];
            const double q0 = pr * j0, q1 = pr * j1, q2 = pr * j2;
            V[0] += q0 * j0; V[1] += q0 * j1; V[2] += q0 * j2;
            V[3] += q1 * j1; V[4] += q1 * j2; V[5] += q2 * j2;
            V[6] += q0 * wv; V[7] += q1 * wv; V[8] += q2 * wv;
        }
    }
#pragma unroll
    for (int m = 0; m < 9; ++m) V[m] = wave_sum(V[m]);
    const double V00 = V[0], V01 = V[1], V02 = V[2], V11 = V[3], V12 = V[4], V22 = V[5];
    const double b0 = V[6], b1 = V[7], b2 = V[8];
    // symmetric 3x3 inverse (adjugate) and R = L^-T of V = L L' (as k_lin_reduce)
    const double c00 = V11 * V22 - V12 * V12, c01 = V02 * V12 - V01 * V22, c02 = V01 * V12 - V02 * V11;
    const double id = 1.0 / (V00 * c00 + V01 * c01 + V02 * c02);
    const double I00 = c00 * id, I01 = c01 * id, I02 = c02 * id;
    const double I11 = (V00 * V22 - V02 * V02) * id, I12 = (V01 * V02 - V00 * V12) * id, I22 = (V00 * V11 - V01 * V01) * id;
    const double l00 = sqrt(V00), l10 = V01 / l00, l20 = V02 / l00;
    const double l11 = sqrt(V11 - l10 * l10), l21 = (V12 - l20 * l10) / l11;
    const double l22 = sqrt(V22 - l20 * l20 - l21 * l21);
    const double m00 = 1.0 / l00, m11 = 1.0 / l11, m22 = 1.0 / l22;
    const double m10 = -l10 * m00 * m11, m21 = -l21 * m11 * m22, m20 = -(l20 * m00 + l21 * m10) * m22;
    if (l == 0) {
        double* P = gpt + (int64_t)q * GPT;
        P[0] = I00; P[1] = I01; P[2] = I02; P[3] = I11; P[4] = I12; P[5] = I22;
        P[6] = m00; P[7] = m10; P[8] = m20; P[9] = m11; P[10] = m21; P[11] = m22;
        P[12] = m00 * b0;
        P[13] = m10 * b0 + m11 * b1;
        P[14] = m20 * b0 + m21 * b1 + m22 * b2;
        P[15] = I00 * b0 + I01 * b1 + I02 * b2;
        P[16] = I01 * b0 + I11 * b1 + I12 * b2;
        P[17] = I02 * b0 + I12 * b1 + I22 * b2;
    }
    // per camera of the point: Wc = Jc'PJp over its observations through that camera
    for (int gc = A[g.g_gc + q]; gc < A[g.g_gc + q + 1]; ++gc) {
        double Wc[CW][3];
#pragma unroll
        for (int c = 0; c < CW; ++c) Wc[c][0] = Wc[c][1] = Wc[c][2] = 0.0;
        for (int x = A[g.gc_o + gc] + l; x < A[g.gc_o + gc + 1]; x += 64) {
            const double* Jo = J + (int64_t)A[g.gc_list + x] * JS;
#pragma unroll
            for (int row = 0; row < 2; ++row) {
                const double pr = row ? py : px;
                const double q0 = pr * Jo[row * NJ + 6 + CW], q1 = pr * Jo[row * NJ + 7 + CW], q2 = pr * Jo[row * NJ + 8 + CW];
#pragma unroll
                for (int c = 0; c < CW; ++c) {
                    const double jc = Jo[row * NJ + 6 + c];
                    Wc[c][0] += jc * q0; Wc[c][1] += jc * q1; Wc[c][2] += jc * q2;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < CW; ++c)
#pragma unroll
            for (int m = 0; m < 3; ++m) Wc[c][m] = wave_sum(Wc[c][m]);
        if (l == 0) {
            double* T = gcu + (int64_t)gc * GC;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const double w0 = Wc[c][0], w1 = Wc[c][1], w2 = Wc[c][2];
                T[3 * c] = w0 * m00;
                T[3 * c + 1] = w0 * m10 + w1 * m11;
                T[3 * c + 2] = w0 * m20 + w1 * m21 + w2 * m22;
                T[3 * CW + 3 * c] = w0 * I00 + w1 * I01 + w2 * I02;
                T[3 * CW + 3 * c + 1] = w0 * I01 + w1 * I11 + w2 * I12;
                T[3 * CW + 3 * c + 2] = w0 * I02 + w1 * I12 + w2 * I22;
            }
        }
    }
    // per image of the point: Ug = sum_o W_o R, T = sum_o W_o V^-1 over its observations there
    for (int gi = A[g.g_gi + q] + l; gi < A[g.g_gi + q + 1]; gi += 64) {
        double u[18], t[18];
#pragma unroll
        for (int m = 0; m < 18; ++m) u[m] = t[m] = 0.0;
        for (int o = A[g.gi_obs + gi]; o < A[g.gi_obs + gi + 1]; ++o) {
            const double* Jo = J + (int64_t)o * JS;
            const double px0 = Jo[6 + CW], px1 = Jo[7 + CW], px2 = Jo[8 + CW];
            const double py0 = Jo[NJ + 6 + CW], py1 = Jo[NJ + 7 + CW], py2 = Jo[NJ + 8 + CW];
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double e0 = px * Jo[a], e1 = py * Jo[NJ + a];
                const double v0 = e0 * px0 + e1 * py0, v1 = e0 * px1 + e1 * py1, v2 = e0 * px2 + e1 * py2;
                t[3 * a] += v0 * I00 + v1 * I01 + v2 * I02;
                t[3 * a + 1] += v0 * I01 + v1 * I11 + v2 * I12;
                t[3 * a + 2] += v0 * I02 + v1 * I12 + v2 * I22;
                u[3 * a] += v0 * m00;
                u[3 * a + 1] += v0 * m10 + v1 * m11;
                u[3 * a + 2] += v0 * m20 + v1 * m21 + v2 * m22;
            }
        }
        double* out = gug + (int64_t)gi * GUG;
#pragma unroll
        for (int m = 0; m < 18; ++m) { out[m] = u[m]; out[18 + m] = t[m]; }
    }
}

// one thread per partial entry, five segments: pair keys | image keys | foreign-camera keys | camera
// partials | camera-pair keys
template <int NK>
__global__ __launch_bounds__(256) void k_gen_keys(const double* __restrict__ J, const int32_t* __restrict__ A,
                                                  const GenPlan g, const double* __restrict__ gpt,
                                                  const double* __restrict__ gcu, const double* __restrict__ gug,
                                                  double* __restrict__ ppart, double* __restrict__ ipart,
                                                  double* __restrict__ cpart, double* __restrict__ xpart,
                                                  double* __restrict__ kpart, double px, double py) {
    using Q = GL<NK>;
    constexpr int CW = Q::CW, NJ = Q::NJ, JS = Q::JS, GC = Q::GC, NIMG = Q::NIMG, NPK = Q::NPK, NCAM = Q::NCAM;
    constexpr int NX = Q::NX, NKK = Q::NKK;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    auto dot3 = [](const double* x, const double* y) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
    // pair keys: value 6 a + b = -Ug1[a] . Ug2[b] (a: row of the higher image, as k_lin_reduce)
    if (t < g.n_gpk * 36) {
        const int64_t k = t / 36;
        const int v = (int)(t % 36), a = v / 6, b = v % 6;
        const double* u1 = gug + (int64_t)A[g.gpk + 2 * k] * GUG;
        const double* u2 = gug + (int64_t)A[g.gpk + 2 * k + 1] * GUG;
        ppart[(int64_t)A[g.pk_slot + g.pk0 + k] * 36 + v] = -dot3(u1 + 3 * a, u2 + 3 * b);
        return;
    }
    t -= g.n_gpk * 36;
    if (t < g.n_gi * NIMG) {
        const int64_t gi = t / NIMG;
        const int v = (int)(t % NIMG);
        const double* ug = gug + gi * GUG;
        const int o0 = A[g.gi_obs + gi], o1 = A[g.gi_obs + gi + 1];
        double s = 0.0, r;
        if (v < 21) {  // lower diagonal block (a, b)
            int a, b;
            tri_ab(v, a, b);
            for (int o = o0; o < o1; ++o) {
                const double* Jo = J + (int64_t)o * JS;
                s += px * Jo[a] * Jo[b] + py * Jo[NJ + a] * Jo[NJ + b];
            }
            r = dot3(ug + 3 * a, ug + 3 * b);
        } else if (v < 27) {  // right-hand side
            const int a = v - 21;
            for (int o = o0; o < o1; ++o) {
                const double* Jo = J + (int64_t)o * JS;
                s += px * Jo[a] * Jo[2 * NJ] + py * Jo[NJ + a] * Jo[2 * NJ + 1];
            }
            r = dot3(ug + 3 * a, gpt + (int64_t)A[g.gi_gp + gi] * GPT + 12);
        } else {  // own camera: 27 + 6 b + a (camera column b, image row a)
            const int a = (v - 27) % 6, b = (v - 27) / 6;
            for (int o = o0; o < o1; ++o) {
                const double* Jo = J + (int64_t)o * JS;
                s += px * Jo[6 + b] * Jo[a] + py * Jo[NJ + 6 + b] * Jo[NJ + a];
            }
            r = dot3(ug + 3 * a, gcu + (int64_t)A[g.gi_gc + gi] * GC + 3 * b);
        }
        ipart[(int64_t)A[g.ik_slot + g.ik0 + gi] * NIMG + v] = s - r;
        return;
    }
    t -= g.n_gi * NIMG;
    if (t < g.n_gx * NX) {  // image x another camera: 6 b + a = -Ug[a] . Uc[b]
        const int64_t k = t / NX;
        const int v = (int)(t % NX), a = v % 6, b = v / 6;
        const double* ug = gug + (int64_t)A[g.gx + 2 * k] * GUG;
        const double* uc = gcu + (int64_t)A[g.gx + 2 * k + 1] * GC;
        xpart[k * NX + v] = -dot3(ug + 3 * a, uc + 3 * b);
        return;
    }
    t -= g.n_gx * NX;
    if (t < g.n_gc * NCAM) {  // camera block (lower, k_red_cam's entry order) and RHS
        const int64_t gc = t / NCAM;
        const int v = (int)(t % NCAM);
        const double* uc = gcu + gc * GC;
        const int x0 = A[g.gc_o + gc], x1 = A[g.gc_o + gc + 1];
        double s = 0.0, r;
        if (v < NPK) {
            int c1, c2;
            tri_ab(v, c1, c2);
            for (int x = x0; x < x1; ++x) {
                const double* Jo = J + (int64_t)A[g.gc_list + x] * JS;
                s += px * Jo[6 + c1] * Jo[6 + c2] + py * Jo[NJ + 6 + c1] * Jo[NJ + 6 + c2];
            }
            r = dot3(uc + 3 * c1, uc + 3 * c2);
        } else {
            const int c1 = v - NPK;
            for (int x = x0; x < x1; ++x) {
                const double* Jo = J + (int64_t)A[g.gc_list + x] * JS;
                s += px * Jo[6 + c1] * Jo[2 * NJ] + py * Jo[NJ + 6 + c1] * Jo[2 * NJ + 1];
            }
            r = dot3(uc + 3 * c1, gpt + (int64_t)A[g.gc_gp + gc] * GPT + 12);
        }
        cpart[(g.ck0 + gc) * NCAM + v] = s - r;
        return;
    }
    t -= g.n_gc * NCAM;
    if (t < g.n_gkk * NKK) {  // camera k1 x camera k2 (k1 > k2): a CW + b = -Uc1[a] . Uc2[b]
        const int64_t k = t / NKK;
        const int v = (int)(t % NKK), a = v / CW, b = v % CW;
        const double* u1 = gcu + (int64_t)A[g.gkk + 2 * k] * GC;
        const double* u2 = gcu + (int64_t)A[g.gkk + 2 * k + 1] * GC;
        kpart[k * NKK + v] = -dot3(u1 + 3 * a, u2 + 3 * b);
    }
}

// the blocks only general points touch, each the sum of its partials in slot order:
// image e x camera k (k not e's camera) and camera k1 x camera k2 (k1 > k2), lower part of S
template <int NK>
__global__ __launch_bounds__(256) void k_red_gen(const int32_t* __restrict__ A, const GenPlan g,
                                                 const double* __restrict__ xpart, const double* __restrict__ kpart,
                                                 double* __restrict__ S, int64_t ld, int n_img) {
    using Q = GL<NK>;
    constexpr int CW = Q::CW, NX = Q::NX, NKK = Q::NKK;
    int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t cam0 = 6 * (int64_t)n_img;
    if (t < g.n_xt * NX) {
        const int64_t x = t / NX;
        const int v = (int)(t % NX), a = v % 6, b = v / 6;
        double s = 0.0;
        for (int q = A[g.xt_start + x]; q < A[g.xt_start + x + 1]; ++q) s += xpart[(int64_t)A[g.xt_list + q] * NX + v];
        const int64_t e = A[g.xt_key + 2 * x], k = A[g.xt_key + 2 * x + 1];
        S[(cam0 + k * CW + b) * ld + 6 * e + a] = s;
        return;
    }
    t -= g.n_xt * NX;
    if (t < g.n_kt * NKK) {
        const int64_t x = t / NKK;
        const int v = (int)(t % NKK), a = v / CW, b = v % CW;
        double s = 0.0;
        for (int q = A[g.kt_start + x]; q < A[g.kt_start + x + 1]; ++q) s += kpart[(int64_t)A[g.kt_list + q] * NKK + v];
        const int64_t k1 = A[g.kt_key + 2 * x], k2 = A[g.kt_key + 2 * x + 1];
        S[(cam0 + k1 * CW + a) * ld + cam0 + k2 * CW + b] = s;
    }
}

// tie-point corrections of the general points: dp = -(vb + sum_gimg T' d_e + sum_gpc Tc' d_k)
template <int NK>
__global__ __launch_bounds__(256) void k_gen_backsub(const int32_t* __restrict__ A, const GenPlan g,
                                                     const double* __restrict__ gpt, const double* __restrict__ gcu,
                                                     const double* __restrict__ gug, const int32_t* __restrict__ lp_tie,
                                                     double* __restrict__ delta, int64_t u_c, int n_img) {
    constexpr int CW = GL<NK>::CW, GC = GL<NK>::GC;
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= g.n_gp) return;
    const double* P = gpt + q * GPT;
    double d0 = P[15], d1 = P[16], d2 = P[17];
    for (int gi = A[g.g_gi + q]; gi < A[g.g_gi + q + 1]; ++gi) {
        const double* T = gug + (int64_t)gi * GUG + 18;
        const double* de = delta + 6 * (int64_t)A[g.gi_img + gi];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double e = de[a];
            d0 += T[3 * a] * e; d1 += T[3 * a + 1] * e; d2 += T[3 * a + 2] * e;
        }
    }
    for (int gc = A[g.g_gc + q]; gc < A[g.g_gc + q + 1]; ++gc) {
        const double* Tc = gcu + (int64_t)gc * GC + 3 * CW;
        const double* dk = delta + 6 * (int64_t)n_img + (int64_t)A[g.gc_cam + gc] * CW;
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            d0 += Tc[3 * c] * dk[c]; d1 += Tc[3 * c + 1] * dk[c]; d2 += Tc[3 * c + 2] * dk[c];
        }
    }
    double* out = delta + u_c + 3 * (int64_t)lp_tie[g.lp0 + q];
    out[0] = -d0; out[1] = -d1; out[2] = -d2;
}

// tie-point variances of the general points (fba_covariance): diag(V^-1 + K' C K) with the row groups
// K = [T of each gimg (6 rows of its image); Tc of each gpc (CW rows of its camera)], C read from the
// selected inverse in S's lower blocks, minus the border term (Z' K)(Wz' K); one wave per point
template <int NK>
__global__ __launch_bounds__(256) void k_cov_gen(const double* __restrict__ S, int64_t ld, const double* __restrict__ Z,
                                                 const double* __restrict__ Wz, int nz, int64_t n_pad,
                                                 const int32_t* __restrict__ A, const GenPlan g,
                                                 const double* __restrict__ gpt, const double* __restrict__ gcu,
                                                 const double* __restrict__ gug, const int32_t* __restrict__ lp_tie,
                                                 int n_img, double* __restrict__ pdiag) {
    constexpr int CW = GL<NK>::CW, GC = GL<NK>::GC;
    const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (q >= g.n_gp) return;
    const int i0 = A[g.g_gi + q], ni = A[g.g_gi + q + 1] - i0;
    const int c0 = A[g.g_gc + q], nc = A[g.g_gc + q + 1] - c0;
    auto grp = [&](int x, int64_t& r0, int& n, const double*& T) {
        if (x < ni) { r0 = 6 * (int64_t)A[g.gi_img + i0 + x]; n = 6; T = gug + (int64_t)(i0 + x) * GUG + 18; }
        else { r0 = 6 * (int64_t)n_img + (int64_t)A[g.gc_cam + c0 + x - ni] * CW; n = CW; T = gcu + (int64_t)(c0 + x - ni) * GC + 3 * CW; }
    };
    const int ng = ni + nc;
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0;
    for (int pr = lane; pr < ng * ng; pr += 64) {
        const int x = pr / ng, y = pr % ng;
        int64_t r0, c0_;
        int nr, ncc;
        const double *Tg, *Th;
        grp(x, r0, nr, Tg);
        grp(y, c0_, ncc, Th);
        for (int a = 0; a < nr; ++a) {
            double s0 = 0.0, s1 = 0.0, s2 = 0.0;
            for (int b = 0; b < ncc; ++b) {
                const int64_t r = r0 + a, c = c0_ + b;
                const int64_t rr = (r / NB >= c / NB) ? r : c, cc = (r / NB >= c / NB) ? c : r;
                const double v = S[rr * ld + cc];
                s0 += v * Th[3 * b]; s1 += v * Th[3 * b + 1]; s2 += v * Th[3 * b + 2];
            }
            acc0 += Tg[3 * a] * s0; acc1 += Tg[3 * a + 1] * s1; acc2 += Tg[3 * a + 2] * s2;
        }
    }
    if (lane < nz) {
        double z0 = 0, z1 = 0, z2 = 0, w0 = 0, w1 = 0, w2 = 0;
        for (int x = 0; x < ng; ++x) {
            int64_t r0;
            int nr;
            const double* Tg;
            grp(x, r0, nr, Tg);
            for (int a = 0; a < nr; ++a) {
                const double zv = Z[lane * n_pad + r0 + a], wv = Wz[lane * n_pad + r0 + a];
                z0 += zv * Tg[3 * a]; z1 += zv * Tg[3 * a + 1]; z2 += zv * Tg[3 * a + 2];
                w0 += wv * Tg[3 * a]; w1 += wv * Tg[3 * a + 1]; w2 += wv * Tg[3 * a + 2];
            }
        }
        acc0 -= z0 * w0; acc1 -= z1 * w1; acc2 -= z2 * w2;
    }
    acc0 = wave_sum(acc0);
    acc1 = wave_sum(acc1);
    acc2 = wave_sum(acc2);
    if (lane == 0) {
        const double* P = gpt + q * GPT;
        double* out = pdiag + 3 * (int64_t)lp_tie[g.lp0 + q];
        out[0] = P[0] + acc0;
        out[1] = P[3] + acc1;
        out[2] = P[5] + acc2;
    }
}

// ================================================================================================
// launchers
// ================================================================================================
#define GEN_NK_DISPATCH(nk, F)        \
    switch (nk) {                     \
        case 1: F(1); break;          \
        case 2: F(2); break;          \
        case 3: F(3); break;          \
        case 4: F(4); break;          \
        case 5: F(5); break;          \
        case 6: F(6); break;          \
        case 7: F(7); break;          \
        case 8: F(8); break;          \
        default: set_error("num_radial out of range"); return FBA_ERR_UNSUPPORTED; \
    }

static inline unsigned grid_of(int64_t n, int per) { return (unsigned)std::max<int64_t>((n + per - 1) / per, 1); }

int launch_gen_tables(Ctx& c, const double* x) {
    const GenPlan& g = c.gen;
    if (g.n_gp == 0) return FBA_OK;
    int rc;
    if ((rc = launch_linearize_range(c, x, c.n_chunks_lr, c.n_chunks))) return rc;  // J of the general observations
    const double px = 1.0 / (c.set.meas_std_x * c.set.meas_std_x), py = 1.0 / (c.set.meas_std_y * c.set.meas_std_y);
#define GP(NKV) k_gen_point<NKV><<<(unsigned)g.n_gp, 64, 0, c.stream>>>(c.d_J, c.d_acc, g, c.d_gpt, c.d_gcu, c.d_gug, px, py)
    GEN_NK_DISPATCH(c.L.nk, GP);
#undef GP
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_gen_keys(Ctx& c) {
    const GenPlan& g = c.gen;
    if (g.n_gp == 0) return FBA_OK;
    const double px = 1.0 / (c.set.meas_std_x * c.set.meas_std_x), py = 1.0 / (c.set.meas_std_y * c.set.meas_std_y);
#define GK(NKV)                                                                                                       \
    {                                                                                                                 \
        using Q = GL<NKV>;                                                                                            \
        const int64_t n = g.n_gpk * 36 + g.n_gi * Q::NIMG + g.n_gx * Q::NX + g.n_gc * Q::NCAM + g.n_gkk * Q::NKK;     \
        k_gen_keys<NKV><<<grid_of(n, 256), 256, 0, c.stream>>>(c.d_J, c.d_acc, g, c.d_gpt, c.d_gcu, c.d_gug, c.d_ppart, \
                                                               c.d_ipart, c.d_cpart, c.d_xpart, c.d_kpart, px, py);  \
    }
    GEN_NK_DISPATCH(c.L.nk, GK);
#undef GK
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_gen_reduce(Ctx& c) {
    const GenPlan& g = c.gen;
    if (g.n_xt == 0 && g.n_kt == 0) return FBA_OK;
#define GR(NKV)                                                                                                 \
    {                                                                                                           \
        using Q = GL<NKV>;                                                                                      \
        const int64_t n = g.n_xt * Q::NX + g.n_kt * Q::NKK;                                                     \
        k_red_gen<NKV><<<grid_of(n, 256), 256, 0, c.stream>>>(c.d_acc, g, c.d_xpart, c.d_kpart, c.d_S, c.L.ld,    \
                                                              c.L.n_img);                                       \
    }
    GEN_NK_DISPATCH(c.L.nk, GR);
#undef GR
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_gen_backsub(Ctx& c) {
    const GenPlan& g = c.gen;
    if (g.n_gp == 0) return FBA_OK;
#define GB(NKV)                                                                                                     \
    k_gen_backsub<NKV><<<grid_of(g.n_gp, 256), 256, 0, c.stream>>>(c.d_acc, g, c.d_gpt, c.d_gcu, c.d_gug, c.d_lp_tie, \
                                                                   c.d_delta, c.L.u_c, c.L.n_img)
    GEN_NK_DISPATCH(c.L.nk, GB);
#undef GB
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_gen_cov(Ctx& c, const double* Z, const double* Wz, int nz, double* pdiag) {
    const GenPlan& g = c.gen;
    if (g.n_gp == 0) return FBA_OK;
#define GV(NKV)                                                                                                  \
    k_cov_gen<NKV><<<grid_of(g.n_gp, 4), 256, 0, c.stream>>>(c.d_S, c.L.ld, Z, Wz, nz, c.L.n_pad, c.d_acc, g, c.d_gpt, \
                                                             c.d_gcu, c.d_gug, c.d_lp_tie, c.L.n_img, pdiag)
    GEN_NK_DISPATCH(c.L.nk, GV);
#undef GV
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

}  // namespace fba
