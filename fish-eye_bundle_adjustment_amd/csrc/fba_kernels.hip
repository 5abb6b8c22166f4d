// fba_kernels.hip -- linearisation and normal-equation kernels for gfx950 (MI355X).
//
// One Gauss-Newton pass (the reference's main.m:413-488 with BuildAwG.m:46-527 inside) becomes:
//   k_params        per image: EOPs + rotation M and dM/d(omega,phi,kappa) (BuildAwG.m:163-165),
//                   inner-constraint block G (BuildAwG.m:516-523); per camera: IOPs, rmax^(2j)
//                   scales (BuildAwG.m:422-426)
//   k_linearize     one thread per image point: misclosure w (BuildAwG.m:505-512) and the 2 Jacobian
//                   rows over [6 EOP | xp yp c K1..Knk P1 P2 | X Y Z] (BuildAwG.m:216-503) by the
//                   chain rule of the forward model (BuildAwG.m:163-213)
//   k_point         one thread per tie point: V = Jp'PJp, Vinv, the coupling blocks W = Je'PJp and
//                   T = W Vinv per observation (Schur elimination of the tie points)
//   k_image         one workgroup per image: reduced diagonal block, image-camera block, RHS rows
//   k_pairs         one wave per co-visible image pair: off-diagonal reduced blocks
//   k_cam_*         two-stage deterministic reduction of the camera block
//   k_border        inner-constraint bordering M = S + G W G' (reference: NG = [N G; G' 0],
//                   main.m:428-432), unit diagonal for fixed parameters, RHS rows
//   k_backsub       tie-point corrections from the camera-side solution
//   k_update        de-scaling of distortion corrections (main.m:460-482), xhat += delta
//                   (main.m:484), deltasum = sumabs(delta) (main.m:487, sumabs.m:12-14)
//   k_residuals     v = A*delta + w (main.m:569), BuildRSD rows (BuildRSD.m:29-40), v'Pv
// Every reduction is a fixed-order sum (no float atomics), so results are bitwise reproducible.
#include "fba_internal.h"

namespace fba {

__device__ __forceinline__ int64_t jc_index(int r, int col, int nj) { return (int64_t)(r * nj + col); }

// ------------------------------------------------------------------------------------------------
// k_params: per-image and per-camera tables
// ------------------------------------------------------------------------------------------------
__global__ void k_params(const double* __restrict__ xfull, const double* __restrict__ caminfo,
                         double* __restrict__ img_tab, double* __restrict__ cam_tab, double* __restrict__ G,
                         int n_img, int n_cam, int nk, int cw, int cam_stride, int ic) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n_img) {
        const double* e = xfull + 6 * (int64_t)t;
        double Xc = e[0], Yc = e[1], Zc = e[2], w = e[3], p = e[4], k = e[5];
        double cw_, sw, cp, sp, ck, sk;
        sincos(w, &sw, &cw_);
        sincos(p, &sp, &cp);
        sincos(k, &sk, &ck);
        double* o = img_tab + (int64_t)t * IMG_TAB;
        o[0] = Xc; o[1] = Yc; o[2] = Zc; o[3] = w; o[4] = p; o[5] = k;
        double* M = o + 6;
        // rows of M: U,V,W = M (X - Xc) with the reference's sign conventions (BuildAwG.m:163-165)
        M[0] = ck * cp;  M[1] = cw_ * sk + ck * sp * sw;  M[2] = sk * sw - ck * cw_ * sp;
        M[3] = -cp * sk; M[4] = ck * cw_ - sk * sp * sw;  M[5] = ck * sw + cw_ * sk * sp;
        M[6] = sp;       M[7] = -cp * sw;                 M[8] = cp * cw_;
        double* Mw = o + 15;
        Mw[0] = 0.0; Mw[1] = -sw * sk + ck * sp * cw_; Mw[2] = sk * cw_ + ck * sw * sp;
        Mw[3] = 0.0; Mw[4] = -ck * sw - sk * sp * cw_; Mw[5] = ck * cw_ - sw * sk * sp;
        Mw[6] = 0.0; Mw[7] = -cp * cw_;                Mw[8] = -cp * sw;
        double* Mp = o + 24;
        Mp[0] = -ck * sp; Mp[1] = ck * cp * sw;  Mp[2] = -ck * cw_ * cp;
        Mp[3] = sp * sk;  Mp[4] = -sk * cp * sw; Mp[5] = cw_ * sk * cp;
        Mp[6] = cp;       Mp[7] = sp * sw;       Mp[8] = -sp * cw_;
        double* Mk = o + 33;
        Mk[0] = -sk * cp; Mk[1] = cw_ * ck - sk * sp * sw;  Mk[2] = ck * sw + sk * cw_ * sp;
        Mk[3] = -cp * ck; Mk[4] = -sk * cw_ - ck * sp * sw; Mk[5] = -sk * sw + cw_ * ck * sp;
        Mk[6] = 0.0;      Mk[7] = 0.0;                      Mk[8] = 0.0;
        if (ic) {  // BuildAwG.m:516-523, rows Xc Yc Zc w p k, 7 columns
            double* g = G + (int64_t)t * 42;
            double tp = tan(p), secp = 1.0 / cos(p);
            const double rows[42] = {
                1, 0, 0, 0, -Zc, Yc, Xc,
                0, 1, 0, Zc, 0, -Xc, Yc,
                0, 0, 1, -Yc, Xc, 0, Zc,
                0, 0, 0, -1, -sin(w) * tp, cos(w) * tp, 0,
                0, 0, 0, 0, -cos(w), -sin(w), 0,
                0, 0, 0, 0, sin(w) * secp, -cos(w) * secp, 0};
            for (int i = 0; i < 42; ++i) g[i] = rows[i];
        }
    } else if (t < n_img + n_cam) {
        int k = t - n_img;
        const double* q = xfull + 6 * (int64_t)n_img + (int64_t)k * cw;
        const double* ci = caminfo + 5 * k;
        double* o = cam_tab + (int64_t)k * cam_stride;
        o[0] = q[0];            // xp
        o[1] = q[1];            // yp
        o[2] = q[2];            // c
        o[3] = ci[0];           // y_dir
        o[4] = q[3 + nk];       // P1
        o[5] = q[4 + nk];       // P2
        double hx = (ci[3] - ci[1]) * 0.5, hy = (ci[4] - ci[2]) * 0.5;
        double rmax = sqrt(hx * hx + hy * hy);  // BuildAwG.m:422
        o[7] = rmax;
        for (int j = 1; j <= nk; ++j) {
            o[CAM_TAB_HDR + j - 1] = q[2 + j];                   // K_j
            o[CAM_TAB_HDR + nk + j - 1] = pow(rmax, 2.0 * j);    // rmax^(2j), BuildAwG.m:424-426
        }
        o[6] = o[CAM_TAB_HDR + nk];                              // rmax^2
    }
}

// ------------------------------------------------------------------------------------------------
// k_linearize: one thread per image point
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(256) void k_linearize(
    const double* __restrict__ xy, const int32_t* __restrict__ img, const int32_t* __restrict__ cam,
    const int32_t* __restrict__ pt, const int32_t* __restrict__ lp_tie, const double* __restrict__ ctl,
    const double* __restrict__ xfull, const double* __restrict__ img_tab, const double* __restrict__ cam_tab,
    double* __restrict__ J, int64_t n_obs, int64_t stride, int64_t u_c, int type, int cam_stride,
    unsigned eop_mask, unsigned cam_mask) {
    constexpr int CW = 5 + NK;
    constexpr int NJ = 9 + CW;
    int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_obs) return;
    const double x = xy[2 * o], y = xy[2 * o + 1];
    const int e = img[o], k = cam[o], p = pt[o];
    const double* it = img_tab + (int64_t)e * IMG_TAB;
    const double* ct = cam_tab + (int64_t)k * cam_stride;
    double X, Y, Z;
    if (p >= 0) {
        const double* q = xfull + u_c + 3 * (int64_t)lp_tie[p];
        X = q[0]; Y = q[1]; Z = q[2];
    } else {
        const double* q = ctl + 3 * (int64_t)(-1 - p);
        X = q[0]; Y = q[1]; Z = q[2];
    }
    const double d0 = X - it[0], d1 = Y - it[1], d2 = Z - it[2];
    const double* M = it + 6;
    const double U = M[0] * d0 + M[1] * d1 + M[2] * d2;
    const double V = M[3] * d0 + M[4] * d1 + M[5] * d2;
    const double W = M[6] * d0 + M[7] * d1 + M[8] * d2;
    const double R = sqrt(U * U + V * V);
    // radial factor s(R,W): f_proj = -c*(U, ydir*V)*s  (BuildAwG.m:184-208)
    double s, sR, sW;
    if (type == FBA_TYPE_PINHOLE) {
        s = 1.0 / W; sR = 0.0; sW = -1.0 / (W * W);
    } else {
        const double t = atan(R / W);
        const double q = R * R + W * W;
        const double tR = W / q, tW = -R / q;
        double g, gt;
        if (type == FBA_TYPE_FISHEYE) { g = t; gt = 1.0; }
        else if (type == FBA_TYPE_EQUISOLID) { double sh, ch; sincos(0.5 * t, &sh, &ch); g = 2.0 * sh; gt = ch; }
        else if (type == FBA_TYPE_ORTHOGRAPHIC) { double st, ctt; sincos(t, &st, &ctt); g = st; gt = ctt; }
        else { double th = tan(0.5 * t); double ch = cos(0.5 * t); g = 2.0 * th; gt = 1.0 / (ch * ch); }
        s = g / R;
        sR = gt * tR / R - g / (R * R);
        sW = gt * tW / R;
    }
    const double xp = ct[0], yp = ct[1], c = ct[2], ydir = ct[3], P1 = ct[4], P2 = ct[5];
    const double* K = ct + CAM_TAB_HDR;
    const double* sc = ct + CAM_TAB_HDR + NK;
    const double xb = x - xp, yb = y - yp;
    const double r2 = xb * xb + yb * yb;
    double r2j[NK + 1];
    r2j[0] = 1.0;
#pragma unroll
    for (int j = 1; j <= NK; ++j) r2j[j] = r2j[j - 1] * r2;
    double dr = 0.0, dxr = 0.0, dyr = 0.0, dxy = 0.0;
#pragma unroll
    for (int j = 1; j <= NK; ++j) {
        dr += K[j - 1] * r2j[j];
        const double tj = 2.0 * j * K[j - 1] * r2j[j - 1];
        dxr += tj * xb * xb;
        dyr += tj * yb * yb;
        dxy += tj * xb * yb;
    }
    const double decx = P1 * (yb * yb + 3.0 * xb * xb) + 2.0 * P2 * xb * yb;
    const double decy = P2 * (xb * xb + 3.0 * yb * yb) + 2.0 * P1 * xb * yb;
    const double cs = c * s;
    const double cys = c * ydir;
    const double fx = -cs * U + xp + dr * xb + decx;
    const double fy = -cys * V * s + yp + dr * yb + decy;

    auto put = [&](int r, int col, double v) { J[jc_index(r, col, NJ) * stride + o] = v; };
    // chain rule through (U,V,W) -> (fx,fy)
    auto chain = [&](double dU, double dV, double dW, double& gx, double& gy) {
        const double dR = (U * dU + V * dV) / R;
        const double ds = (type == FBA_TYPE_PINHOLE) ? sW * dW : sR * dR + sW * dW;
        gx = -c * (dU * s + U * ds);
        gy = -cys * (dV * s + V * ds);
    };
    double gx, gy;
    // EOP columns Xc Yc Zc: d(UVW)/dXc = -M[:,0] ...
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        chain(-M[q], -M[3 + q], -M[6 + q], gx, gy);
        const double en = (eop_mask >> q) & 1u ? 1.0 : 0.0;
        put(0, q, gx * en);
        put(1, q, gy * en);
        if (p >= 0) { put(0, 6 + CW + q, -gx); put(1, 6 + CW + q, -gy); }  // d/dX = -d/dXc
        else { put(0, 6 + CW + q, 0.0); put(1, 6 + CW + q, 0.0); }
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double* Md = it + 15 + 9 * a;
        const double dU = Md[0] * d0 + Md[1] * d1 + Md[2] * d2;
        const double dV = Md[3] * d0 + Md[4] * d1 + Md[5] * d2;
        const double dW = Md[6] * d0 + Md[7] * d1 + Md[8] * d2;
        chain(dU, dV, dW, gx, gy);
        const double en = (eop_mask >> (3 + a)) & 1u ? 1.0 : 0.0;
        put(0, 3 + a, gx * en);
        put(1, 3 + a, gy * en);
    }
    // camera columns: xp yp c K1..KNK P1 P2 (BuildAwG.m:373-445)
    auto cen = [&](int col) { return (cam_mask >> col) & 1u ? 1.0 : 0.0; };
    {
        double ax = 1.0 - dr - dxr - 6.0 * P1 * xb - 2.0 * P2 * yb;  // d fx / d xp
        double ay = -dxy - 2.0 * P1 * yb - 2.0 * P2 * xb;            // d fy / d xp
        put(0, 6, ax * cen(0)); put(1, 6, ay * cen(0));
        double bx = -dxy - 2.0 * P2 * xb - 2.0 * P1 * yb;            // d fx / d yp
        double by = 1.0 - dr - dyr - 6.0 * P2 * yb - 2.0 * P1 * xb;  // d fy / d yp
        put(0, 7, bx * cen(1)); put(1, 7, by * cen(1));
        put(0, 8, -U * s * cen(2)); put(1, 8, -ydir * V * s * cen(2));  // d/dc
    }
#pragma unroll
    for (int j = 1; j <= NK; ++j) {
        const double en = cen(2 + j);
        put(0, 8 + j, r2j[j] * xb / sc[j - 1] * en);
        put(1, 8 + j, r2j[j] * yb / sc[j - 1] * en);
    }
    {
        const double en1 = cen(3 + NK), en2 = cen(4 + NK);
        const double s1 = sc[0];
        put(0, 9 + NK, (yb * yb + 3.0 * xb * xb) / s1 * en1);
        put(1, 9 + NK, 2.0 * xb * yb / s1 * en1);
        put(0, 10 + NK, 2.0 * xb * yb / s1 * en2);
        put(1, 10 + NK, (xb * xb + 3.0 * yb * yb) / s1 * en2);
    }
    J[(int64_t)(2 * NJ) * stride + o] = fx - x;
    J[(int64_t)(2 * NJ + 1) * stride + o] = fy - y;
}

// ------------------------------------------------------------------------------------------------
// k_point: one thread per local tie point (Schur elimination of the 3 point unknowns)
// pt_tab components: [0..5] Vinv (00 01 02 11 12 22), [6..8] vb = Vinv b, [9..11] b,
//                    [12 .. 12+3CW) Wc[c][m], [12+3CW .. 12+6CW) Tc[c][m] = (Wc Vinv)[c][m]
// WT per obs: [0..17] W[a][m] = (Je' P Jp)[a][m], [18..35] T = W Vinv
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(64) void k_point(const double* __restrict__ J, const int32_t* __restrict__ lp_start,
                                              double* __restrict__ pt_tab, double* __restrict__ WT, int64_t n_lp,
                                              int64_t stride, int64_t pstride, double px, double py) {
    constexpr int CW = 5 + NK;
    constexpr int NJ = 9 + CW;
    int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_lp) return;
    const int o0 = lp_start[p], o1 = lp_start[p + 1];
    double V00 = 0, V01 = 0, V02 = 0, V11 = 0, V12 = 0, V22 = 0, b0 = 0, b1 = 0, b2 = 0;
    double Wc[CW][3];
#pragma unroll
    for (int c = 0; c < CW; ++c) Wc[c][0] = Wc[c][1] = Wc[c][2] = 0.0;
    for (int o = o0; o < o1; ++o) {
        double jp[2][3], w[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int m = 0; m < 3; ++m) jp[r][m] = J[jc_index(r, 6 + CW + m, NJ) * stride + o];
            w[r] = J[(int64_t)(2 * NJ + r) * stride + o];
        }
        const double pr[2] = {px, py};
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double a0 = pr[r] * jp[r][0], a1 = pr[r] * jp[r][1], a2 = pr[r] * jp[r][2];
            V00 += a0 * jp[r][0]; V01 += a0 * jp[r][1]; V02 += a0 * jp[r][2];
            V11 += a1 * jp[r][1]; V12 += a1 * jp[r][2]; V22 += a2 * jp[r][2];
            b0 += a0 * w[r]; b1 += a1 * w[r]; b2 += a2 * w[r];
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                const double jc = J[jc_index(r, 6 + c, NJ) * stride + o];
                Wc[c][0] += jc * a0; Wc[c][1] += jc * a1; Wc[c][2] += jc * a2;
            }
        }
    }
    // symmetric 3x3 inverse (adjugate)
    const double c00 = V11 * V22 - V12 * V12, c01 = V02 * V12 - V01 * V22, c02 = V01 * V12 - V02 * V11;
    const double det = V00 * c00 + V01 * c01 + V02 * c02;
    const double id = 1.0 / det;
    const double I00 = c00 * id, I01 = c01 * id, I02 = c02 * id;
    const double I11 = (V00 * V22 - V02 * V02) * id, I12 = (V01 * V02 - V00 * V12) * id,
                 I22 = (V00 * V11 - V01 * V01) * id;
    const double vb0 = I00 * b0 + I01 * b1 + I02 * b2;
    const double vb1 = I01 * b0 + I11 * b1 + I12 * b2;
    const double vb2 = I02 * b0 + I12 * b1 + I22 * b2;
    double* t = pt_tab + p;
    t[0 * pstride] = I00; t[1 * pstride] = I01; t[2 * pstride] = I02;
    t[3 * pstride] = I11; t[4 * pstride] = I12; t[5 * pstride] = I22;
    t[6 * pstride] = vb0; t[7 * pstride] = vb1; t[8 * pstride] = vb2;
    t[9 * pstride] = b0; t[10 * pstride] = b1; t[11 * pstride] = b2;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        t[(12 + 3 * c + 0) * pstride] = Wc[c][0];
        t[(12 + 3 * c + 1) * pstride] = Wc[c][1];
        t[(12 + 3 * c + 2) * pstride] = Wc[c][2];
        t[(12 + 3 * CW + 3 * c + 0) * pstride] = Wc[c][0] * I00 + Wc[c][1] * I01 + Wc[c][2] * I02;
        t[(12 + 3 * CW + 3 * c + 1) * pstride] = Wc[c][0] * I01 + Wc[c][1] * I11 + Wc[c][2] * I12;
        t[(12 + 3 * CW + 3 * c + 2) * pstride] = Wc[c][0] * I02 + Wc[c][1] * I12 + Wc[c][2] * I22;
    }
    for (int o = o0; o < o1; ++o) {
        double jp[2][3];
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int m = 0; m < 3; ++m) jp[r][m] = J[jc_index(r, 6 + CW + m, NJ) * stride + o];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double je0 = px * J[jc_index(0, a, NJ) * stride + o];
            const double je1 = py * J[jc_index(1, a, NJ) * stride + o];
            const double w0 = je0 * jp[0][0] + je1 * jp[1][0];
            const double w1 = je0 * jp[0][1] + je1 * jp[1][1];
            const double w2 = je0 * jp[0][2] + je1 * jp[1][2];
            WT[(int64_t)(3 * a + 0) * stride + o] = w0;
            WT[(int64_t)(3 * a + 1) * stride + o] = w1;
            WT[(int64_t)(3 * a + 2) * stride + o] = w2;
            WT[(int64_t)(18 + 3 * a + 0) * stride + o] = w0 * I00 + w1 * I01 + w2 * I02;
            WT[(int64_t)(18 + 3 * a + 1) * stride + o] = w0 * I01 + w1 * I11 + w2 * I12;
            WT[(int64_t)(18 + 3 * a + 2) * stride + o] = w0 * I02 + w1 * I12 + w2 * I22;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_image: one workgroup per image; thread q owns one output entry:
//   q < 21            reduced diagonal block U_e (lower, a >= b)
//   21 <= q < 27      reduced RHS r_e
//   27 <= q < 27+6CW  image-camera block (camera row c, image column a)
// ------------------------------------------------------------------------------------------------
__constant__ int c_tri_a[21] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5};
__constant__ int c_tri_b[21] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4, 0, 1, 2, 3, 4, 5};

template <int NK>
__global__ __launch_bounds__(128) void k_image(const double* __restrict__ J, const double* __restrict__ WT,
                                               const double* __restrict__ pt_tab, const int32_t* __restrict__ pt,
                                               const int32_t* __restrict__ cam, const int32_t* __restrict__ img_start,
                                               const int32_t* __restrict__ img_obs, double* __restrict__ S, int64_t ld,
                                               int64_t n_pad, int n_img, int64_t stride, int64_t pstride,
                                               double px, double py) {
    constexpr int CW = 5 + NK;
    constexpr int NJ = 9 + CW;
    const int e = blockIdx.x;
    const int q = threadIdx.x;
    const int i0 = img_start[e], i1 = img_start[e + 1];
    if (i0 == i1) return;
    if (q >= 27 + 6 * CW) return;
    int kind, a, b;
    if (q < 21) { kind = 0; a = c_tri_a[q]; b = c_tri_b[q]; }
    else if (q < 27) { kind = 1; a = q - 21; b = 0; }
    else { kind = 2; a = (q - 27) % 6; b = (q - 27) / 6; }  // b = camera column
    double acc = 0.0;
    for (int i = i0; i < i1; ++i) {
        const int o = img_obs[i];
        const int p = pt[o];
        const double ea0 = J[jc_index(0, a, NJ) * stride + o];
        const double ea1 = J[jc_index(1, a, NJ) * stride + o];
        double s0, s1;
        if (kind == 0) { s0 = J[jc_index(0, b, NJ) * stride + o]; s1 = J[jc_index(1, b, NJ) * stride + o]; }
        else if (kind == 1) { s0 = J[(int64_t)(2 * NJ) * stride + o]; s1 = J[(int64_t)(2 * NJ + 1) * stride + o]; }
        else { s0 = J[jc_index(0, 6 + b, NJ) * stride + o]; s1 = J[jc_index(1, 6 + b, NJ) * stride + o]; }
        acc += px * ea0 * s0 + py * ea1 * s1;
        if (p >= 0) {
            if (kind == 0) {
                const double* T = WT + (int64_t)(18 + 3 * a) * stride + o;
                const double* Wb = WT + (int64_t)(3 * b) * stride + o;
                acc -= T[0] * Wb[0] + T[stride] * Wb[stride] + T[2 * stride] * Wb[2 * stride];
            } else if (kind == 1) {
                const double* Wa = WT + (int64_t)(3 * a) * stride + o;
                const double* vb = pt_tab + 6 * pstride + p;
                acc -= Wa[0] * vb[0] + Wa[stride] * vb[pstride] + Wa[2 * stride] * vb[2 * pstride];
            } else {
                const double* T = WT + (int64_t)(18 + 3 * a) * stride + o;
                const double* Wc = pt_tab + (int64_t)(12 + 3 * b) * pstride + p;
                acc -= T[0] * Wc[0] + T[stride] * Wc[pstride] + T[2 * stride] * Wc[2 * pstride];
            }
        }
    }
    if (kind == 0) {
        S[(int64_t)(6 * e + a) * ld + 6 * e + b] = acc;
    } else if (kind == 1) {
        S[n_pad * ld + 6 * e + a] = acc;
    } else {
        const int k = cam[img_obs[i0]];
        S[(int64_t)(6 * (int64_t)n_img + (int64_t)k * CW + b) * ld + 6 * e + a] = acc;
    }
}

// ------------------------------------------------------------------------------------------------
// k_pairs: off-diagonal image-image blocks S(e1,e2) = -sum W_i Vinv W_j^T over shared tie points
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pairs(const double* __restrict__ WT, const int32_t* __restrict__ pair_e,
                                              const int32_t* __restrict__ pair_start, const int32_t* __restrict__ pair_ij,
                                              double* __restrict__ S, int64_t ld, int64_t stride) {
    const int64_t pr = blockIdx.x;
    const int q = threadIdx.x;
    if (q >= 36) return;
    const int a = q / 6, b = q % 6;
    const int e1 = pair_e[2 * pr], e2 = pair_e[2 * pr + 1];
    const int t0 = pair_start[pr], t1 = pair_start[pr + 1];
    double acc = 0.0;
    for (int t = t0; t < t1; ++t) {
        const int i = pair_ij[2 * t], j = pair_ij[2 * t + 1];
        const double* T = WT + (int64_t)(18 + 3 * a) * stride + i;
        const double* W = WT + (int64_t)(3 * b) * stride + j;
        acc -= T[0] * W[0] + T[stride] * W[stride] + T[2 * stride] * W[2 * stride];
    }
    S[(int64_t)(6 * e1 + a) * ld + 6 * e2 + b] = acc;
}

// ------------------------------------------------------------------------------------------------
// camera block: stage 1 (NSLAB x n_cam workgroups) -> slabs, stage 2 -> S
// entry q < CW(CW+1)/2: lower (c1 >= c2);  q >= that: RHS entry c
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(128) void k_cam_stage1(const double* __restrict__ J, const double* __restrict__ pt_tab,
                                                    const int32_t* __restrict__ lp_start,
                                                    const int32_t* __restrict__ cam_lp, const int32_t* __restrict__ cam_ctl,
                                                    double* __restrict__ slab, int64_t n_obs_tie, int64_t stride,
                                                    int64_t pstride, double px, double py) {
    constexpr int CW = 5 + NK;
    constexpr int NJ = 9 + CW;
    constexpr int NPK = CW * (CW + 1) / 2;
    const int s = blockIdx.x, k = blockIdx.y, q = threadIdx.x;
    if (q >= NPK + CW) return;
    int c1, c2 = -1;
    if (q < NPK) {
        c1 = 0;
        int rem = q;
        while (rem > c1) { rem -= c1 + 1; ++c1; }
        c2 = rem;
    } else {
        c1 = q - NPK;
    }
    double acc = 0.0;
    // tie points of camera k, slab s
    const int64_t p0 = cam_lp[k], p1 = cam_lp[k + 1];
    const int64_t np = p1 - p0;
    const int64_t a0 = p0 + np * s / NSLAB, a1 = p0 + np * (s + 1) / NSLAB;
    for (int64_t p = a0; p < a1; ++p) {
        const int o0 = lp_start[p], o1 = lp_start[p + 1];
        for (int o = o0; o < o1; ++o) {
            const double j10 = J[jc_index(0, 6 + c1, NJ) * stride + o];
            const double j11 = J[jc_index(1, 6 + c1, NJ) * stride + o];
            double s0, s1;
            if (c2 >= 0) { s0 = J[jc_index(0, 6 + c2, NJ) * stride + o]; s1 = J[jc_index(1, 6 + c2, NJ) * stride + o]; }
            else { s0 = J[(int64_t)(2 * NJ) * stride + o]; s1 = J[(int64_t)(2 * NJ + 1) * stride + o]; }
            acc += px * j10 * s0 + py * j11 * s1;
        }
        if (c2 >= 0) {
            const double* T = pt_tab + (int64_t)(12 + 3 * CW + 3 * c1) * pstride + p;
            const double* W = pt_tab + (int64_t)(12 + 3 * c2) * pstride + p;
            acc -= T[0] * W[0] + T[pstride] * W[pstride] + T[2 * pstride] * W[2 * pstride];
        } else {
            const double* W = pt_tab + (int64_t)(12 + 3 * c1) * pstride + p;
            const double* vb = pt_tab + 6 * pstride + p;
            acc -= W[0] * vb[0] + W[pstride] * vb[pstride] + W[2 * pstride] * vb[2 * pstride];
        }
    }
    // control observations of camera k, slab s
    const int64_t q0 = cam_ctl[k], q1 = cam_ctl[k + 1];
    const int64_t nq = q1 - q0;
    const int64_t b0 = q0 + nq * s / NSLAB, b1 = q0 + nq * (s + 1) / NSLAB;
    for (int64_t oo = b0; oo < b1; ++oo) {
        const int64_t o = n_obs_tie + oo;
        const double j10 = J[jc_index(0, 6 + c1, NJ) * stride + o];
        const double j11 = J[jc_index(1, 6 + c1, NJ) * stride + o];
        double s0, s1;
        if (c2 >= 0) { s0 = J[jc_index(0, 6 + c2, NJ) * stride + o]; s1 = J[jc_index(1, 6 + c2, NJ) * stride + o]; }
        else { s0 = J[(int64_t)(2 * NJ) * stride + o]; s1 = J[(int64_t)(2 * NJ + 1) * stride + o]; }
        acc += px * j10 * s0 + py * j11 * s1;
    }
    slab[((int64_t)k * NSLAB + s) * (NPK + CW) + q] = acc;
}

template <int NK>
__global__ void k_cam_stage2(const double* __restrict__ slab, double* __restrict__ S, int64_t ld, int64_t n_pad,
                             int n_img) {
    constexpr int CW = 5 + NK;
    constexpr int NPK = CW * (CW + 1) / 2;
    const int k = blockIdx.x, q = threadIdx.x;
    if (q >= NPK + CW) return;
    double acc = 0.0;
    for (int s = 0; s < NSLAB; ++s) acc += slab[((int64_t)k * NSLAB + s) * (NPK + CW) + q];
    const int64_t base = 6 * (int64_t)n_img + (int64_t)k * CW;
    if (q < NPK) {
        int c1 = 0, rem = q;
        while (rem > c1) { rem -= c1 + 1; ++c1; }
        S[(base + c1) * ld + base + rem] = acc;
    } else {
        S[n_pad * ld + base + (q - NPK)] = acc;
    }
}

// ------------------------------------------------------------------------------------------------
// border: M = S + G W G^T with one weight per constraint column, w_m = 1 / sum_i G_im^2 / S_ii
// (EOP rows).  The constraints G^T delta = 0 are invariant to the column weights; this choice
// equilibrates the added curvature against S row by row, so the Cholesky of M keeps S's precision
// (a single trace-based weight put 1e7 x S_ii on the translation rows of cam0 and lost 7 digits).
// scal layout: [1] Cholesky failure flag, [2] sumabs, [8..14] w_m
// ------------------------------------------------------------------------------------------------
__global__ void k_border_weights(const double* __restrict__ S, const double* __restrict__ G,
                                 double* __restrict__ scal, int64_t ld, int n_img, int ic) {
    __shared__ double red[7][256];
    double a[7] = {0, 0, 0, 0, 0, 0, 0};
    if (ic) {
        for (int64_t i = threadIdx.x; i < 6 * (int64_t)n_img; i += blockDim.x) {
            const double sii = S[i * ld + i];
            if (!(sii > 0.0)) continue;
            const double* g = G + (i / 6) * 42 + (i % 6) * 7;
            for (int m = 0; m < 7; ++m) a[m] += g[m] * g[m] / sii;
        }
    }
    for (int m = 0; m < 7; ++m) red[m][threadIdx.x] = a[m];
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int m = 0; m < 7; ++m) red[m][threadIdx.x] += red[m][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x < 7) scal[8 + threadIdx.x] = red[threadIdx.x][0] > 0.0 ? 1.0 / red[threadIdx.x][0] : 1.0;
    if (threadIdx.x == 0) scal[1] = 0.0;  // Cholesky failure flag
}

__global__ void k_border(double* __restrict__ S, const double* __restrict__ G, const double* __restrict__ scal,
                         int64_t ld, int n_img, int ic) {
    // 2D grid of 64x64 tiles over the EOP rows; lower tiles only
    const int64_t i = (int64_t)blockIdx.y * 64 + threadIdx.y;
    const int64_t jb = (int64_t)blockIdx.x * 64;
    if (blockIdx.x > blockIdx.y) return;
    const int64_t n = 6 * (int64_t)n_img;
    if (!ic || i >= n) return;
    const double* gi = G + (i / 6) * 42 + (i % 6) * 7;
    double g[7];
    for (int m = 0; m < 7; ++m) g[m] = gi[m] * scal[8 + m];
    for (int jj = threadIdx.x; jj < 64; jj += blockDim.x) {
        const int64_t j = jb + jj;
        if (j > i || j >= n) continue;
        const double* gj = G + (j / 6) * 42 + (j % 6) * 7;
        double acc = 0.0;
        for (int m = 0; m < 7; ++m) acc += g[m] * gj[m];
        S[i * ld + j] += acc;
    }
}

__global__ void k_finish_rhs(double* __restrict__ S, const double* __restrict__ G, const double* __restrict__ scal,
                             const uint8_t* __restrict__ active, int64_t ld, int64_t n_pad, int64_t u_c, int n_img,
                             int ic) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    if (i >= u_c || !active[i]) {
        // fixed parameter or padding: decoupled unit row, zero RHS
        S[i * ld + i] = 1.0;
        S[n_pad * ld + i] = 0.0;
    }
    if (ic) {
        for (int m = 0; m < 7; ++m)
            S[(n_pad + 1 + m) * ld + i] =
                (i < 6 * (int64_t)n_img) ? sqrt(scal[8 + m]) * G[(i / 6) * 42 + (i % 6) * 7 + m] : 0.0;
    }
}

// ------------------------------------------------------------------------------------------------
// back-substitution of tie points: dp = -(vb + sum_o T_o^T d_e(o) + Tc^T d_cam)
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ void k_backsub(const double* __restrict__ WT, const double* __restrict__ pt_tab,
                          const int32_t* __restrict__ lp_start, const int32_t* __restrict__ lp_tie,
                          const int32_t* __restrict__ lp_cam, const int32_t* __restrict__ img,
                          double* __restrict__ delta, int64_t n_lp, int64_t stride, int64_t pstride, int64_t u_c,
                          int n_img) {
    constexpr int CW = 5 + NK;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_lp) return;
    double d0 = pt_tab[6 * pstride + p], d1 = pt_tab[7 * pstride + p], d2 = pt_tab[8 * pstride + p];
    for (int o = lp_start[p]; o < lp_start[p + 1]; ++o) {
        const double* de = delta + 6 * (int64_t)img[o];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double* T = WT + (int64_t)(18 + 3 * a) * stride + o;
            d0 += T[0] * de[a]; d1 += T[stride] * de[a]; d2 += T[2 * stride] * de[a];
        }
    }
    const double* dk = delta + 6 * (int64_t)n_img + (int64_t)lp_cam[p] * CW;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        const double* T = pt_tab + (int64_t)(12 + 3 * CW + 3 * c) * pstride + p;
        d0 += T[0] * dk[c]; d1 += T[pstride] * dk[c]; d2 += T[2 * pstride] * dk[c];
    }
    double* out = delta + u_c + 3 * (int64_t)lp_tie[p];
    out[0] = -d0; out[1] = -d1; out[2] = -d2;
}

// ------------------------------------------------------------------------------------------------
// update: de-scale (main.m:460-482), xhat += delta, partial sumabs (fixed-order block sums)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_update(double* __restrict__ xfull, double* __restrict__ delta,
                                                const double* __restrict__ cam_tab, const uint8_t* __restrict__ counted,
                                                double* __restrict__ part, int64_t u_full, int n_img, int n_cam, int nk,
                                                int cw, int cam_stride) {
    __shared__ double red[256];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double a = 0.0;
    if (i < u_full) {
        double d = delta[i];
        const int64_t cb = 6 * (int64_t)n_img;
        if (i >= cb && i < cb + (int64_t)n_cam * cw) {
            const int64_t k = (i - cb) / cw;
            const int c = (int)((i - cb) % cw);
            const double* ct = cam_tab + k * cam_stride;
            if (c >= 3 && c < 3 + nk) d = d / ct[CAM_TAB_HDR + nk + (c - 3)];  // K_j / rmax^(2j)
            else if (c >= 3 + nk) d = d / ct[6];                               // P / rmax^2
        }
        delta[i] = d;
        xfull[i] += d;
        if (counted[i]) a = fabs(d);
        if (!isfinite(d)) a = __builtin_nan("");
    }
    red[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void k_sum_parts(const double* __restrict__ part, int n, double* __restrict__ out) {
    __shared__ double red[256];
    double a = 0.0;
    // each thread sums a contiguous range (fixed order), then a fixed tree
    const int per = (n + 255) / 256;
    for (int i = threadIdx.x * per; i < min(n, (threadIdx.x + 1) * per); ++i) a += part[i];
    red[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = red[0];
}

// ------------------------------------------------------------------------------------------------
// residuals: v = J delta + w (main.m:569; delta = de-scaled last correction, as the reference),
// RSD (BuildRSD.m:29-40) with xp,yp of the updated parameters; block partials of vx^2, vy^2, v'Pv
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(256) void k_residuals(const double* __restrict__ J, const double* __restrict__ xy,
                                                   const int32_t* __restrict__ img, const int32_t* __restrict__ cam,
                                                   const int32_t* __restrict__ pt, const int32_t* __restrict__ lp_tie,
                                                   const double* __restrict__ delta, const double* __restrict__ xfull,
                                                   double* __restrict__ v, double* __restrict__ rsd,
                                                   double* __restrict__ part, int64_t n_obs, int64_t stride,
                                                   int64_t u_c, int n_img, double px, double py) {
    constexpr int CW = 5 + NK;
    constexpr int NJ = 9 + CW;
    __shared__ double red[3][256];
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double sx = 0.0, sy = 0.0, sp = 0.0;
    if (o < n_obs) {
        const int e = img[o], k = cam[o], p = pt[o];
        const double* de = delta + 6 * (int64_t)e;
        const double* dk = delta + 6 * (int64_t)n_img + (int64_t)k * CW;
        double vv[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            double acc = J[(int64_t)(2 * NJ + r) * stride + o];
#pragma unroll
            for (int a = 0; a < 6; ++a) acc += J[jc_index(r, a, NJ) * stride + o] * de[a];
#pragma unroll
            for (int c = 0; c < CW; ++c) acc += J[jc_index(r, 6 + c, NJ) * stride + o] * dk[c];
            if (p >= 0) {
                const double* dp = delta + u_c + 3 * (int64_t)lp_tie[p];
#pragma unroll
                for (int m = 0; m < 3; ++m) acc += J[jc_index(r, 6 + CW + m, NJ) * stride + o] * dp[m];
            }
            vv[r] = acc;
        }
        v[2 * o] = vv[0];
        v[2 * o + 1] = vv[1];
        const double* kp = xfull + 6 * (int64_t)n_img + (int64_t)k * CW;
        const double xb = xy[2 * o] - kp[0], yb = xy[2 * o + 1] - kp[1];
        const double theta = atan2(yb, xb), phi = atan2(vv[1], vv[0]);
        const double vd = sqrt(vv[0] * vv[0] + vv[1] * vv[1]);
        double* rr = rsd + 5 * o;
        rr[0] = sqrt(xb * xb + yb * yb);
        rr[1] = vv[0];
        rr[2] = vv[1];
        rr[3] = vd * cos(theta - phi);
        rr[4] = vd * sin(theta - phi);
        sx = vv[0] * vv[0];
        sy = vv[1] * vv[1];
        sp = px * sx + py * sy;
    }
    red[0][threadIdx.x] = sx; red[1][threadIdx.x] = sy; red[2][threadIdx.x] = sp;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            for (int m = 0; m < 3; ++m) red[m][threadIdx.x] += red[m][threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int m = 0; m < 3; ++m) part[3 * blockIdx.x + m] = red[m][0];
}

// ------------------------------------------------------------------------------------------------
// dense debug A (BuildAwG's A, column-major n x u_ref, PHO row order)
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ void k_dense_awg(const double* __restrict__ J, const int32_t* __restrict__ img,
                            const int32_t* __restrict__ cam, const int32_t* __restrict__ pt,
                            const int32_t* __restrict__ lp_tie, const int64_t* __restrict__ obs_pho,
                            const int64_t* __restrict__ map, double* __restrict__ A, double* __restrict__ w,
                            int64_t n_obs, int64_t stride, int64_t n_rows, int64_t u_c, int n_img) {
    constexpr int CW = 5 + NK;
    constexpr int NJ = 9 + CW;
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_obs) return;
    const int e = img[o], k = cam[o], p = pt[o];
    const int64_t row0 = 2 * obs_pho[o];
    for (int r = 0; r < 2; ++r) {
        const int64_t row = row0 + r;
        w[row] = J[(int64_t)(2 * NJ + r) * stride + o];
        for (int a = 0; a < 6; ++a) {
            const int64_t col = map[6 * (int64_t)e + a];
            if (col >= 0) A[col * n_rows + row] = J[jc_index(r, a, NJ) * stride + o];
        }
        for (int c = 0; c < CW; ++c) {
            const int64_t col = map[6 * (int64_t)n_img + (int64_t)k * CW + c];
            if (col >= 0) A[col * n_rows + row] = J[jc_index(r, 6 + c, NJ) * stride + o];
        }
        if (p >= 0) {
            for (int m = 0; m < 3; ++m) {
                const int64_t col = map[u_c + 3 * (int64_t)lp_tie[p] + m];
                if (col >= 0) A[col * n_rows + row] = J[jc_index(r, 6 + CW + m, NJ) * stride + o];
            }
        }
    }
}

// ================================================================================================
// launchers
// ================================================================================================
#define FBA_NK_DISPATCH(nk, F)        \
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

static inline unsigned eop_mask(const fba_settings& s) {
    return (s.est_Xc ? 1u : 0u) | (s.est_Yc ? 2u : 0u) | (s.est_Zc ? 4u : 0u) | (s.est_omega ? 8u : 0u) |
           (s.est_phi ? 16u : 0u) | (s.est_kappa ? 32u : 0u);
}
static inline unsigned cam_mask(const fba_settings& s, int nk) {
    unsigned m = (s.est_xp ? 1u : 0u) | (s.est_yp ? 2u : 0u) | (s.est_c ? 4u : 0u);
    if (s.est_radial)
        for (int j = 0; j < nk; ++j) m |= 1u << (3 + j);
    if (s.est_decent) m |= (1u << (3 + nk)) | (1u << (4 + nk));
    return m;
}
static inline double px_of(const Ctx& c) { return 1.0 / (c.set.meas_std_x * c.set.meas_std_x); }
static inline double py_of(const Ctx& c) { return 1.0 / (c.set.meas_std_y * c.set.meas_std_y); }


int launch_params(Ctx& c) {
    const int n = c.L.n_img + c.L.n_cam;
    k_params<<<(n + 63) / 64, 64, 0, c.stream>>>(c.d_xfull, c.d_caminfo, c.d_img_tab, c.d_cam_tab, c.d_G,
                                                   c.L.n_img, c.L.n_cam, c.L.nk, c.L.cw, c.cam_tab_stride,
                                                   c.set.inner_constraints);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_linearize(Ctx& c) {
    if (c.n_obs == 0) return FBA_OK;
    const unsigned em = eop_mask(c.set), cm = cam_mask(c.set, c.L.nk);
    const int blocks = (int)((c.n_obs + 255) / 256);
#define LIN(NKV)                                                                                               \
    k_linearize<NKV><<<blocks, 256, 0, c.stream>>>(c.d_xy, c.d_img, c.d_cam, c.d_pt, c.d_lp_tie, c.d_ctl,      \
                                                   c.d_xfull, c.d_img_tab, c.d_cam_tab, c.d_J, c.n_obs,        \
                                                   c.n_obs_pad, c.L.u_c, c.set.type, c.cam_tab_stride, em, cm)
    FBA_NK_DISPATCH(c.L.nk, LIN);
#undef LIN
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_point(Ctx& c) {
    if (c.n_lp == 0) return FBA_OK;
    const int blocks = (int)((c.n_lp + 63) / 64);
#define PT(NKV)                                                                                            \
    k_point<NKV><<<blocks, 64, 0, c.stream>>>(c.d_J, c.d_lp_start, c.d_pt_tab, c.d_WT, c.n_lp, c.n_obs_pad, \
                                              c.n_lp_pad, px_of(c), py_of(c))
    FBA_NK_DISPATCH(c.L.nk, PT);
#undef PT
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_accumulate(Ctx& c) {
    const Layout& L = c.L;
    FBA_HIP(hipMemsetAsync(c.d_S, 0, sizeof(double) * (size_t)(L.n_pad + NB) * L.ld, c.stream));
    const double px = px_of(c), py = py_of(c);
#define IMG(NKV)                                                                                          \
    k_image<NKV><<<L.n_img, 128, 0, c.stream>>>(c.d_J, c.d_WT, c.d_pt_tab, c.d_pt, c.d_cam, c.d_img_start, \
                                                c.d_img_obs, c.d_S, L.ld, L.n_pad, L.n_img, c.n_obs_pad,   \
                                                c.n_lp_pad, px, py)
    FBA_NK_DISPATCH(L.nk, IMG);
#undef IMG
    FBA_HIP(hipGetLastError());
    if (c.n_pairs > 0) {
        k_pairs<<<(unsigned)c.n_pairs, 64, 0, c.stream>>>(c.d_WT, c.d_pair_e, c.d_pair_start, c.d_pair_ij, c.d_S,
                                                           L.ld, c.n_obs_pad);
        FBA_HIP(hipGetLastError());
    }
    dim3 g1(NSLAB, L.n_cam);
#define CAM(NKV)                                                                                               \
    k_cam_stage1<NKV><<<g1, 128, 0, c.stream>>>(c.d_J, c.d_pt_tab, c.d_lp_start, c.d_cam_lp, c.d_cam_ctl,     \
                                                c.d_slab, c.n_obs_tie, c.n_obs_pad, c.n_lp_pad, px, py);      \
    k_cam_stage2<NKV><<<L.n_cam, 128, 0, c.stream>>>(c.d_slab, c.d_S, L.ld, L.n_pad, L.n_img)
    FBA_NK_DISPATCH(L.nk, CAM);
#undef CAM
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_border(Ctx& c) {
    const Layout& L = c.L;
    const int ic = c.set.inner_constraints;
    k_border_weights<<<1, 256, 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, L.ld, L.n_img, ic);
    FBA_HIP(hipGetLastError());
    if (ic) {
        const int nb = (int)((6 * (int64_t)L.n_img + 63) / 64);
        k_border<<<dim3(nb, nb), dim3(16, 64), 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, L.ld, L.n_img, ic);
        FBA_HIP(hipGetLastError());
    }
    k_finish_rhs<<<(unsigned)((L.n_pad + 255) / 256), 256, 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, c.d_active,
                                                                           L.ld, L.n_pad, L.u_c, L.n_img, ic);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_backsub_update(Ctx& c) {
    const Layout& L = c.L;
    if (c.n_lp > 0) {
        const int blocks = (int)((c.n_lp + 255) / 256);
#define BS(NKV)                                                                                               \
    k_backsub<NKV><<<blocks, 256, 0, c.stream>>>(c.d_WT, c.d_pt_tab, c.d_lp_start, c.d_lp_tie, c.d_lp_cam,    \
                                                 c.d_img, c.d_delta, c.n_lp, c.n_obs_pad, c.n_lp_pad, L.u_c, \
                                                 L.n_img)
        FBA_NK_DISPATCH(L.nk, BS);
#undef BS
        FBA_HIP(hipGetLastError());
    }
    const int nblk = (int)((L.u_full + 255) / 256);
    k_update<<<nblk, 256, 0, c.stream>>>(c.d_xfull, c.d_delta, c.d_cam_tab, c.d_counted, c.d_part, L.u_full,
                                         L.n_img, L.n_cam, L.nk, L.cw, c.cam_tab_stride);
    FBA_HIP(hipGetLastError());
    k_sum_parts<<<1, 256, 0, c.stream>>>(c.d_part, nblk, c.d_scal + 2);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_residuals(Ctx& c) {
    const Layout& L = c.L;
    if (c.n_obs == 0) return FBA_OK;
    const int blocks = (int)((c.n_obs + 255) / 256);
#define RS(NKV)                                                                                                \
    k_residuals<NKV><<<blocks, 256, 0, c.stream>>>(c.d_J, c.d_xy, c.d_img, c.d_cam, c.d_pt, c.d_lp_tie,        \
                                                   c.d_delta, c.d_xfull, c.d_res, c.d_res + 2 * c.n_obs,       \
                                                   c.d_part, c.n_obs, c.n_obs_pad, L.u_c, L.n_img, px_of(c),   \
                                                   py_of(c))
    FBA_NK_DISPATCH(L.nk, RS);
#undef RS
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_dense_awg(Ctx& c, double* dA, double* dW, const int64_t* d_map, int64_t n_rows, int64_t u_ref) {
    (void)u_ref;
    if (c.n_obs == 0) return FBA_OK;
    const int blocks = (int)((c.n_obs + 255) / 256);
#define DA(NKV)                                                                                               \
    k_dense_awg<NKV><<<blocks, 256, 0, c.stream>>>(c.d_J, c.d_img, c.d_cam, c.d_pt, c.d_lp_tie,               \
                                                   c.d_obs_pho, d_map, dA, dW, c.n_obs, c.n_obs_pad,      \
                                                   n_rows, c.L.u_c, c.L.n_img)
    FBA_NK_DISPATCH(c.L.nk, DA);
#undef DA
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

}  // namespace fba
