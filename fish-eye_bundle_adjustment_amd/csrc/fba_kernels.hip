// fba_kernels.hip -- linearisation and normal-equation kernels for gfx950 (MI355X).
//
// One Gauss-Newton pass (the reference's main.m:413-488 with BuildAwG.m:46-527 inside) becomes:
//   k_params        per image: EOPs + rotation M and dM/d(omega,phi,kappa) (BuildAwG.m:163-165),
//                   inner-constraint block G (BuildAwG.m:516-523); per camera: IOPs, rmax^(2j)
//                   scales (BuildAwG.m:422-426)
//   k_lin_point     one thread per image point: misclosure w (BuildAwG.m:505-512) and the 2 Jacobian
//                   rows over [6 EOP | xp yp c K1..Knk P1 P2 | X Y Z] (BuildAwG.m:216-503) by the
//                   chain rule of the forward model (BuildAwG.m:163-213); then, per chunk of whole
//                   tie points in LDS, V = Jp'PJp, Vinv and the couplings W = Je'PJp, T = W Vinv
//                   (Schur elimination of the tie points)
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


// ------------------------------------------------------------------------------------------------
// k_params: per-image and per-camera tables
// ------------------------------------------------------------------------------------------------
__global__ void k_params(const double* __restrict__ xfull, const double* __restrict__ caminfo,
                         double* __restrict__ img_tab, double* __restrict__ cam_tab, double* __restrict__ G,
                         const uint8_t* __restrict__ active, int n_img, int n_cam, int nk, int cw, int cam_stride,
                         int ic) {
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
            const bool slot = active[6 * (int64_t)t];  // padding slots (fba_order.cpp) carry no constraint
            for (int i = 0; i < 42; ++i) g[i] = slot ? rows[i] : 0.0;
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
// Device layouts (observation-major so a thread / wave touches contiguous bytes):
//   J   [o][JS], JS = 2*NJ + 2: Jacobian row x (NJ columns: 6 EOP | CW camera | 3 XYZ), row y, w
//   WT  [o][36]: W[a][m] = (Je' P Jp)[a][m] at 3a+m, T = W Vinv at 18+3a+m
//   PT  [p][PS], PS = 12 + 6*CW: Vinv (00 01 02 11 12 22), vb = Vinv b, b, Wc[c][m], Tc = Wc Vinv
// ------------------------------------------------------------------------------------------------
template <int NK>
struct Lay {
    static constexpr int CW = 5 + NK;
    static constexpr int NJ = 9 + CW;
    static constexpr int JS = 2 * NJ + 2;
    static constexpr int PS = 12 + 6 * CW;
};

// Forward model and Jacobian of one image point (BuildAwG.m:163-503 by the chain rule).
template <int NK>
__device__ __forceinline__ void obs_model(double x, double y, const double* __restrict__ it,
                                          const double* __restrict__ ct, double X, double Y, double Z, bool tie,
                                          int type, unsigned eop_mask, unsigned cam_mask,
                                          double (&jr)[2][Lay<NK>::NJ], double& w0, double& w1) {
    constexpr int CW = Lay<NK>::CW;
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
    const double cys = c * ydir;
    const double fx = -c * s * U + xp + dr * xb + decx;
    const double fy = -cys * V * s + yp + dr * yb + decy;
    auto chain = [&](double dU, double dV, double dW, double& gx, double& gy) {
        const double dR = (U * dU + V * dV) / R;
        const double ds = (type == FBA_TYPE_PINHOLE) ? sW * dW : sR * dR + sW * dW;
        gx = -c * (dU * s + U * ds);
        gy = -cys * (dV * s + V * ds);
    };
    double gx, gy;
#pragma unroll
    for (int q = 0; q < 3; ++q) {  // Xc Yc Zc: d(UVW)/dXc = -M[:,q]; tie XYZ = -(that)
        chain(-M[q], -M[3 + q], -M[6 + q], gx, gy);
        const double en = (eop_mask >> q) & 1u ? 1.0 : 0.0;
        jr[0][q] = gx * en;
        jr[1][q] = gy * en;
        jr[0][6 + CW + q] = tie ? -gx : 0.0;
        jr[1][6 + CW + q] = tie ? -gy : 0.0;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {  // omega phi kappa
        const double* Md = it + 15 + 9 * a;
        const double dU = Md[0] * d0 + Md[1] * d1 + Md[2] * d2;
        const double dV = Md[3] * d0 + Md[4] * d1 + Md[5] * d2;
        const double dW = Md[6] * d0 + Md[7] * d1 + Md[8] * d2;
        chain(dU, dV, dW, gx, gy);
        const double en = (eop_mask >> (3 + a)) & 1u ? 1.0 : 0.0;
        jr[0][3 + a] = gx * en;
        jr[1][3 + a] = gy * en;
    }
    auto cen = [&](int col) { return (cam_mask >> col) & 1u ? 1.0 : 0.0; };
    // camera columns xp yp c K1..KNK P1 P2 (BuildAwG.m:373-445)
    jr[0][6] = (1.0 - dr - dxr - 6.0 * P1 * xb - 2.0 * P2 * yb) * cen(0);
    jr[1][6] = (-dxy - 2.0 * P1 * yb - 2.0 * P2 * xb) * cen(0);
    jr[0][7] = (-dxy - 2.0 * P2 * xb - 2.0 * P1 * yb) * cen(1);
    jr[1][7] = (1.0 - dr - dyr - 6.0 * P2 * yb - 2.0 * P1 * xb) * cen(1);
    jr[0][8] = -U * s * cen(2);
    jr[1][8] = -ydir * V * s * cen(2);
#pragma unroll
    for (int j = 1; j <= NK; ++j) {
        const double en = cen(2 + j);
        jr[0][8 + j] = r2j[j] * xb / sc[j - 1] * en;
        jr[1][8 + j] = r2j[j] * yb / sc[j - 1] * en;
    }
    const double s1 = sc[0], en1 = cen(3 + NK), en2 = cen(4 + NK);
    jr[0][9 + NK] = (yb * yb + 3.0 * xb * xb) / s1 * en1;
    jr[1][9 + NK] = 2.0 * xb * yb / s1 * en1;
    jr[0][10 + NK] = 2.0 * xb * yb / s1 * en2;
    jr[1][10 + NK] = (xb * xb + 3.0 * yb * yb) / s1 * en2;
    w0 = fx - x;
    w1 = fy - y;
}

// ------------------------------------------------------------------------------------------------
// k_lin_point: one workgroup per chunk of whole tie points (<= 256 observations), one thread per
// image point.  (1) linearise and store J; (2) one thread per point reduces its observations
// (staged in LDS): V = Jp'PJp, b = Jp'Pw, Wc = Jc'PJp, Vinv, vb, Tc; (3) one thread per observation
// forms W = Je'PJp and T = W Vinv.  Chunks of control observations run step (1) only.
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(256) void k_lin_point(
    const double* __restrict__ xy, const int32_t* __restrict__ img, const int32_t* __restrict__ cam,
    const int32_t* __restrict__ pt, const int32_t* __restrict__ lp_tie, const double* __restrict__ ctl,
    const double* __restrict__ xfull, const double* __restrict__ img_tab, const double* __restrict__ cam_tab,
    const int32_t* __restrict__ chunk_obs, const int32_t* __restrict__ chunk_pt, const int32_t* __restrict__ lp_start,
    double* __restrict__ J, double* __restrict__ WT, double* __restrict__ PT, int64_t u_c, int type, int cam_stride,
    unsigned eop_mask, unsigned cam_mask, double px, double py) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, NJ = LY::NJ, JS = LY::JS, PS = LY::PS;
    constexpr int SH = 8 + 2 * CW;  // Jp (2x3), w (2), Jc (2xCW)
    __shared__ double sh[256][SH + 1];
    __shared__ double vinv[256][6];
    const int t = threadIdx.x;
    const int c = blockIdx.x;
    const int o0 = chunk_obs[c], o1 = chunk_obs[c + 1];
    const int p0 = chunk_pt[c], p1 = chunk_pt[c + 1];
    const int o = o0 + t;
    const bool active = o < o1;
    double jr[2][NJ];
    double w0 = 0.0, w1 = 0.0;
    int p = -1;
    if (active) {
        const double x = xy[2 * (int64_t)o], y = xy[2 * (int64_t)o + 1];
        const int e = img[o], k = cam[o];
        p = pt[o];
        double X, Y, Z;
        if (p >= 0) {
            const double* q = xfull + u_c + 3 * (int64_t)lp_tie[p];
            X = q[0]; Y = q[1]; Z = q[2];
        } else {
            const double* q = ctl + 3 * (int64_t)(-1 - p);
            X = q[0]; Y = q[1]; Z = q[2];
        }
        obs_model<NK>(x, y, img_tab + (int64_t)e * IMG_TAB, cam_tab + (int64_t)k * cam_stride, X, Y, Z, p >= 0, type,
                      eop_mask, cam_mask, jr, w0, w1);
        double* Jo = J + (int64_t)o * JS;
#pragma unroll
        for (int q = 0; q < NJ; q += 1) { Jo[q] = jr[0][q]; Jo[NJ + q] = jr[1][q]; }
        Jo[2 * NJ] = w0;
        Jo[2 * NJ + 1] = w1;
        if (p >= 0) {
#pragma unroll
            for (int m = 0; m < 3; ++m) { sh[t][m] = jr[0][6 + CW + m]; sh[t][3 + m] = jr[1][6 + CW + m]; }
            sh[t][6] = w0;
            sh[t][7] = w1;
#pragma unroll
            for (int q = 0; q < CW; ++q) { sh[t][8 + q] = jr[0][6 + q]; sh[t][8 + CW + q] = jr[1][6 + q]; }
        }
    }
    if (p1 == p0) return;  // control chunk (uniform across the workgroup)
    __syncthreads();
    if (t < p1 - p0) {
        const int lp = p0 + t;
        const int a0 = lp_start[lp] - o0, a1 = lp_start[lp + 1] - o0;
        double V00 = 0, V01 = 0, V02 = 0, V11 = 0, V12 = 0, V22 = 0, b0 = 0, b1 = 0, b2 = 0;
        double Wc[CW][3];
#pragma unroll
        for (int q = 0; q < CW; ++q) Wc[q][0] = Wc[q][1] = Wc[q][2] = 0.0;
        for (int i = a0; i < a1; ++i) {
            const double* r = sh[i];
#pragma unroll
            for (int row = 0; row < 2; ++row) {
                const double pr = row ? py : px;
                const double j0 = r[3 * row], j1 = r[3 * row + 1], j2 = r[3 * row + 2], wv = r[6 + row];
                const double q0 = pr * j0, q1 = pr * j1, q2 = pr * j2;
                V00 += q0 * j0; V01 += q0 * j1; V02 += q0 * j2;
                V11 += q1 * j1; V12 += q1 * j2; V22 += q2 * j2;
                b0 += q0 * wv; b1 += q1 * wv; b2 += q2 * wv;
#pragma unroll
                for (int q = 0; q < CW; ++q) {
                    const double jc = r[8 + row * CW + q];
                    Wc[q][0] += jc * q0; Wc[q][1] += jc * q1; Wc[q][2] += jc * q2;
                }
            }
        }
        // symmetric 3x3 inverse (adjugate)
        const double c00 = V11 * V22 - V12 * V12, c01 = V02 * V12 - V01 * V22, c02 = V01 * V12 - V02 * V11;
        const double id = 1.0 / (V00 * c00 + V01 * c01 + V02 * c02);
        const double I00 = c00 * id, I01 = c01 * id, I02 = c02 * id;
        const double I11 = (V00 * V22 - V02 * V02) * id, I12 = (V01 * V02 - V00 * V12) * id,
                     I22 = (V00 * V11 - V01 * V01) * id;
        double* P = PT + (int64_t)lp * PS;
        P[0] = I00; P[1] = I01; P[2] = I02; P[3] = I11; P[4] = I12; P[5] = I22;
        P[6] = I00 * b0 + I01 * b1 + I02 * b2;
        P[7] = I01 * b0 + I11 * b1 + I12 * b2;
        P[8] = I02 * b0 + I12 * b1 + I22 * b2;
        P[9] = b0; P[10] = b1; P[11] = b2;
#pragma unroll
        for (int q = 0; q < CW; ++q) {
            P[12 + 3 * q] = Wc[q][0];
            P[13 + 3 * q] = Wc[q][1];
            P[14 + 3 * q] = Wc[q][2];
            P[12 + 3 * CW + 3 * q] = Wc[q][0] * I00 + Wc[q][1] * I01 + Wc[q][2] * I02;
            P[13 + 3 * CW + 3 * q] = Wc[q][0] * I01 + Wc[q][1] * I11 + Wc[q][2] * I12;
            P[14 + 3 * CW + 3 * q] = Wc[q][0] * I02 + Wc[q][1] * I12 + Wc[q][2] * I22;
        }
        vinv[t][0] = I00; vinv[t][1] = I01; vinv[t][2] = I02;
        vinv[t][3] = I11; vinv[t][4] = I12; vinv[t][5] = I22;
    }
    __syncthreads();
    if (active && p >= 0) {
        const double* vi = vinv[p - p0];
        const double I00 = vi[0], I01 = vi[1], I02 = vi[2], I11 = vi[3], I12 = vi[4], I22 = vi[5];
        double* Wo = WT + (int64_t)o * 36;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double e0 = px * jr[0][a], e1 = py * jr[1][a];
            const double v0 = e0 * jr[0][6 + CW + 0] + e1 * jr[1][6 + CW + 0];
            const double v1 = e0 * jr[0][6 + CW + 1] + e1 * jr[1][6 + CW + 1];
            const double v2 = e0 * jr[0][6 + CW + 2] + e1 * jr[1][6 + CW + 2];
            Wo[3 * a] = v0; Wo[3 * a + 1] = v1; Wo[3 * a + 2] = v2;
            Wo[18 + 3 * a] = v0 * I00 + v1 * I01 + v2 * I02;
            Wo[19 + 3 * a] = v0 * I01 + v1 * I11 + v2 * I12;
            Wo[20 + 3 * a] = v0 * I02 + v1 * I12 + v2 * I22;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_image: one workgroup per image; 32 observations at a time staged in LDS (J row, W/T, the
// point's vb and Wc); thread q owns one output entry:
//   q < 21            reduced diagonal block U_e (lower, a >= b)
//   21 <= q < 27      reduced RHS r_e
//   27 <= q < 27+6CW  image-camera block (camera row c, image column a)
// Two thread groups split the staged observations; their sums are added in a fixed order.
// The gathers are software-pipelined: the observation/point indices of chunk c+1 are fetched before
// chunk c is published to LDS, and its rows are loaded into registers (all loads of a thread in
// flight together) while chunk c is reduced.
// ------------------------------------------------------------------------------------------------
__constant__ int c_tri_a[21] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5};
__constant__ int c_tri_b[21] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4, 0, 1, 2, 3, 4, 5};

template <int NK>
__global__ __launch_bounds__(256) void k_image(const double* __restrict__ J, const double* __restrict__ WT,
                                               const double* __restrict__ PT, const int32_t* __restrict__ pt,
                                               const int32_t* __restrict__ cam, const int32_t* __restrict__ img_start,
                                               const int32_t* __restrict__ img_obs, double* __restrict__ S, int64_t ld,
                                               int64_t n_pad, int n_img, double px, double py) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, NJ = LY::NJ, JS = LY::JS, PS = LY::PS;
    constexpr int NP = 3 + 3 * CW;           // vb | Wc
    constexpr int F = JS + 36 + NP;          // J row | W,T | vb | Wc
    constexpr int CH = 32;
    constexpr int NOUT = 27 + 6 * CW;
    constexpr int NJ2 = JS / 2, NW2 = 18;
    constexpr int RJ = (CH * NJ2 + 255) / 256, RW = (CH * NW2 + 255) / 256, RP = (CH * NP + 255) / 256;
    static_assert(JS % 2 == 0, "J rows are read as double2");
    __shared__ double st[CH][F + 1];
    __shared__ double part[128];
    __shared__ int so[2][CH], sp[2][CH];
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int g = tid >> 7, q = tid & 127;
    const int i0 = img_start[e], i1 = img_start[e + 1];
    if (i0 == i1) return;
    int kind = 0, a = 0, b = 0;
    if (q < 21) { kind = 0; a = c_tri_a[q]; b = c_tri_b[q]; }
    else if (q < 27) { kind = 1; a = q - 21; }
    else if (q < NOUT) { kind = 2; a = (q - 27) % 6; b = (q - 27) / 6; }
    const double2* J2 = reinterpret_cast<const double2*>(J);
    const double2* W2 = reinterpret_cast<const double2*>(WT);
    double2 rj[RJ], rw[RW];
    double rp[RP];
    auto fetch_idx = [&](int base, int buf) {
        if (tid < CH) {
            const int o = (base + tid < i1) ? img_obs[base + tid] : 0;
            so[buf][tid] = o;
            sp[buf][tid] = (base + tid < i1) ? pt[o] : -1;
        }
    };
    auto fetch_rows = [&](int buf, int n) {
#pragma unroll
        for (int r = 0; r < RJ; ++r) {
            const int idx = tid + 256 * r, k = idx / NJ2, f = idx - k * NJ2;
            if (idx < n * NJ2) rj[r] = J2[(int64_t)so[buf][k] * NJ2 + f];
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int idx = tid + 256 * r, k = idx / NW2, f = idx - k * NW2;
            if (idx < n * NW2) rw[r] = W2[(int64_t)so[buf][k] * NW2 + f];
        }
#pragma unroll
        for (int r = 0; r < RP; ++r) {
            const int idx = tid + 256 * r, k = idx / NP, f = idx - k * NP;
            if (idx < n * NP) {
                const int p = sp[buf][k];
                rp[r] = (p < 0) ? 0.0 : PT[(int64_t)p * PS + (f < 3 ? 6 + f : 12 + f - 3)];
            }
        }
    };
    auto publish = [&](int n) {
#pragma unroll
        for (int r = 0; r < RJ; ++r) {
            const int idx = tid + 256 * r, k = idx / NJ2, f = idx - k * NJ2;
            if (idx < n * NJ2) { st[k][2 * f] = rj[r].x; st[k][2 * f + 1] = rj[r].y; }
        }
#pragma unroll
        for (int r = 0; r < RW; ++r) {
            const int idx = tid + 256 * r, k = idx / NW2, f = idx - k * NW2;
            if (idx < n * NW2) { st[k][JS + 2 * f] = rw[r].x; st[k][JS + 2 * f + 1] = rw[r].y; }
        }
#pragma unroll
        for (int r = 0; r < RP; ++r) {
            const int idx = tid + 256 * r, k = idx / NP, f = idx - k * NP;
            if (idx < n * NP) st[k][JS + 36 + f] = rp[r];
        }
    };
    fetch_idx(i0, 0);
    __syncthreads();
    fetch_rows(0, min(CH, i1 - i0));
    double acc = 0.0;
    int buf = 0;
    for (int base = i0; base < i1; base += CH, buf ^= 1) {
        const int n = min(CH, i1 - base);
        const bool more = base + CH < i1;
        if (more) fetch_idx(base + CH, buf ^ 1);
        publish(n);
        __syncthreads();
        if (more) fetch_rows(buf ^ 1, min(CH, i1 - base - CH));
        if (q < NOUT) {
            for (int k = g; k < n; k += 2) {
                const double* r = st[k];
                const double ea0 = r[a], ea1 = r[NJ + a];
                const bool tie = sp[buf][k] >= 0;
                if (kind == 0) {
                    acc += px * ea0 * r[b] + py * ea1 * r[NJ + b];
                    if (tie) {
                        const double* T = r + JS + 18 + 3 * a;
                        const double* W = r + JS + 3 * b;
                        acc -= T[0] * W[0] + T[1] * W[1] + T[2] * W[2];
                    }
                } else if (kind == 1) {
                    acc += px * ea0 * r[2 * NJ] + py * ea1 * r[2 * NJ + 1];
                    if (tie) {
                        const double* W = r + JS + 3 * a;
                        const double* vb = r + JS + 36;
                        acc -= W[0] * vb[0] + W[1] * vb[1] + W[2] * vb[2];
                    }
                } else {
                    acc += px * ea0 * r[6 + b] + py * ea1 * r[NJ + 6 + b];
                    if (tie) {
                        const double* T = r + JS + 18 + 3 * a;
                        const double* Wc = r + JS + 39 + 3 * b;
                        acc -= T[0] * Wc[0] + T[1] * Wc[1] + T[2] * Wc[2];
                    }
                }
            }
        }
        __syncthreads();
    }
    if (g == 1) part[q] = acc;
    __syncthreads();
    if (g == 0 && q < NOUT) {
        acc += part[q];
        if (kind == 0) {
            S[(int64_t)(6 * e + a) * ld + 6 * e + b] = acc;
        } else if (kind == 1) {
            S[n_pad * ld + 6 * e + a] = acc;
        } else {
            const int k = cam[img_obs[i0]];
            S[(int64_t)(6 * (int64_t)n_img + (int64_t)k * CW + b) * ld + 6 * e + a] = acc;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_pairs: off-diagonal image-image blocks S(e1,e2) = -sum W_i Vinv W_j^T = -sum T_i W_j^T over the tie
// points the two images share; one wave per co-visible pair.  The (T_i, W_j) rows of 32 terms at a
// time are gathered with 16-byte loads into LDS (9 per lane per chunk -- narrow per-entry loads made
// this kernel bound by vector-memory instruction issue), the next chunk's rows and indices are in
// flight while the current chunk is reduced; lanes 0..35 own the 6x6 entries, 4 partial sums each.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_pairs(const double* __restrict__ WT, const int32_t* __restrict__ pair_e,
                                              const int32_t* __restrict__ pair_start, const int32_t* __restrict__ pair_ij,
                                              double* __restrict__ S, int64_t ld, int64_t n_pairs) {
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs, so block b works on pair
    // (b % 8) * per + b / 8 -- each XCD walks a contiguous run of the (e1, e2)-sorted pair list and
    // the W/T rows of an image's observations are re-read from that XCD's L2
    const int64_t per = (n_pairs + 7) / 8;
    const int64_t pr = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    if (pr >= n_pairs) return;
    constexpr int CH = 32, RS = 18;  // terms per chunk, doubles per staged row
    __shared__ __attribute__((aligned(16))) double rows[CH][2][RS];
    __shared__ int2 idx[2][CH];
    const int q = threadIdx.x;
    const int a = q / 6, b = q % 6;
    const int e1 = pair_e[2 * pr], e2 = pair_e[2 * pr + 1];
    const int t0 = pair_start[pr], t1 = pair_start[pr + 1];
    const int nch = (t1 - t0 + CH - 1) / CH;
    const int2* ij2 = reinterpret_cast<const int2*>(pair_ij);
    const double2* WT2 = reinterpret_cast<const double2*>(WT);
    // item it (< 2*9*CH): term it / 18, row (it / 9) & 1 (0: T_i = WT[i][18..36), 1: W_j = WT[j][0..18)),
    // 16-byte part it % 9
    constexpr int NR = (2 * 9 * CH + 63) / 64;  // 9 loads per lane
    double2 rv[NR];
    int2 iv = make_int2(0, 0);
    auto fetch_rows = [&](int c, int buf) {
        const int n = min(CH, t1 - t0 - c * CH);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int it = q + 64 * r, k = it / 18, row = (it / 9) & 1, part = it % 9;
            if (k < n) {
                const int2 t = idx[buf][k];
                rv[r] = WT2[(int64_t)(row ? t.y : t.x) * 18 + (row ? 0 : 9) + part];
            }
        }
    };
    auto fetch_idx = [&](int c) {
        if (q < CH && t0 + c * CH + q < t1) iv = ij2[t0 + c * CH + q];
    };
    fetch_idx(0);
    if (q < CH) idx[0][q] = iv;
    __syncthreads();
    if (nch > 0) fetch_rows(0, 0);
    if (nch > 1) fetch_idx(1);
    double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
    for (int c = 0; c < nch; ++c) {
        const int n = min(CH, t1 - t0 - c * CH);
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int it = q + 64 * r, k = it / 18, row = (it / 9) & 1, part = it % 9;
            if (k < n) *reinterpret_cast<double2*>(&rows[k][row][2 * part]) = rv[r];
        }
        if (c + 1 < nch && q < CH) idx[(c + 1) & 1][q] = iv;
        __syncthreads();
        if (c + 1 < nch) fetch_rows(c + 1, (c + 1) & 1);
        if (c + 2 < nch) fetch_idx(c + 2);
        if (q < 36) {
            int k = 0;
            for (; k + 4 <= n; k += 4) {
                const double* T0 = rows[k][0] + 3 * a; const double* W0 = rows[k][1] + 3 * b;
                const double* T1 = rows[k + 1][0] + 3 * a; const double* W1 = rows[k + 1][1] + 3 * b;
                const double* T2 = rows[k + 2][0] + 3 * a; const double* W2 = rows[k + 2][1] + 3 * b;
                const double* T3 = rows[k + 3][0] + 3 * a; const double* W3 = rows[k + 3][1] + 3 * b;
                acc0 -= T0[0] * W0[0] + T0[1] * W0[1] + T0[2] * W0[2];
                acc1 -= T1[0] * W1[0] + T1[1] * W1[1] + T1[2] * W1[2];
                acc2 -= T2[0] * W2[0] + T2[1] * W2[1] + T2[2] * W2[2];
                acc3 -= T3[0] * W3[0] + T3[1] * W3[1] + T3[2] * W3[2];
            }
            for (; k < n; ++k) {
                const double* T = rows[k][0] + 3 * a;
                const double* W = rows[k][1] + 3 * b;
                acc0 -= T[0] * W[0] + T[1] * W[1] + T[2] * W[2];
            }
        }
        __syncthreads();
    }
    if (q < 36) S[(int64_t)(6 * e1 + a) * ld + 6 * e2 + b] = (acc0 + acc1) + (acc2 + acc3);
}

// ------------------------------------------------------------------------------------------------
// camera block: stage 1 (NSLAB x n_cam workgroups) -> slabs, stage 2 -> S.  Each slab covers a
// contiguous range of the camera's tie points (their observations are contiguous) and of its
// control observations; observations and point rows are staged through LDS 32 at a time.
// entry q < CW(CW+1)/2: lower (c1 >= c2);  q >= that: RHS entry c
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(128) void k_cam_stage1(const double* __restrict__ J, const double* __restrict__ PT,
                                                    const int32_t* __restrict__ lp_start,
                                                    const int32_t* __restrict__ cam_lp, const int32_t* __restrict__ cam_ctl,
                                                    double* __restrict__ slab, int64_t n_obs_tie, double px, double py) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, NJ = LY::NJ, JS = LY::JS, PS = LY::PS;
    constexpr int NPK = CW * (CW + 1) / 2;
    constexpr int CH = 32;
    constexpr int FP = 3 + 6 * CW;  // vb, Wc, Tc of a point
    __shared__ double so[CH][2 * CW + 3];
    __shared__ double sp[CH][FP + 1];
    const int s = blockIdx.x, k = blockIdx.y, q = threadIdx.x;
    int c1 = 0, c2 = -1;
    if (q < NPK) {
        int rem = q;
        while (rem > c1) { rem -= c1 + 1; ++c1; }
        c2 = rem;
    } else {
        c1 = q - NPK;
    }
    const bool act = q < NPK + CW;
    double acc = 0.0;
    const int64_t p0 = cam_lp[k], p1 = cam_lp[k + 1];
    const int64_t np = p1 - p0;
    const int64_t a0 = p0 + np * s / NSLAB, a1 = p0 + np * (s + 1) / NSLAB;
    const int64_t q0 = cam_ctl[k], q1 = cam_ctl[k + 1];
    const int64_t nq = q1 - q0;
    const int64_t b0 = q0 + nq * s / NSLAB, b1 = q0 + nq * (s + 1) / NSLAB;
    // direct terms over the observations: tie observations of points [a0,a1), then control ones.
    // Chunks of 32 observations; the rows of chunk c+1 are loaded into registers while chunk c is
    // reduced from LDS.
    const int64_t oa0 = (a0 < a1) ? lp_start[a0] : 0, oa1 = (a0 < a1) ? lp_start[a1] : 0;
    const int64_t ob0 = n_obs_tie + b0, ob1 = n_obs_tie + b1;
    const int nc0 = (int)((oa1 - oa0 + CH - 1) / CH), nc1 = (int)((ob1 - ob0 + CH - 1) / CH);
    constexpr int FO = 2 * CW + 2;
    constexpr int RO = (CH * FO + 127) / 128, RPT = (CH * FP + 127) / 128;
    auto chunk = [&](int c, int64_t& base) -> int {
        if (c < nc0) { base = oa0 + (int64_t)c * CH; return (int)min((int64_t)CH, oa1 - base); }
        base = ob0 + (int64_t)(c - nc0) * CH;
        return (int)min((int64_t)CH, ob1 - base);
    };
    double ro[RO];
    auto fetch_o = [&](int c) {
        int64_t base;
        const int n = chunk(c, base);
#pragma unroll
        for (int r = 0; r < RO; ++r) {
            const int idx = q + 128 * r, kk = idx / FO, f = idx - kk * FO;
            if (idx < n * FO) {
                const double* row = J + (base + kk) * JS;
                ro[r] = (f < CW) ? row[6 + f] : (f < 2 * CW ? row[NJ + 6 + f - CW] : row[2 * NJ + f - 2 * CW]);
            }
        }
        return n;
    };
    const int nco = nc0 + nc1;
    int n_cur = nco > 0 ? fetch_o(0) : 0;
    for (int c = 0; c < nco; ++c) {
        const int n = n_cur;
#pragma unroll
        for (int r = 0; r < RO; ++r) {
            const int idx = q + 128 * r, kk = idx / FO, f = idx - kk * FO;
            if (idx < n * FO) so[kk][f] = ro[r];
        }
        __syncthreads();
        if (c + 1 < nco) n_cur = fetch_o(c + 1);
        if (act)
            for (int kk = 0; kk < n; ++kk) {
                const double* r = so[kk];
                const double s0 = (c2 >= 0) ? r[c2] : r[2 * CW];
                const double s1 = (c2 >= 0) ? r[CW + c2] : r[2 * CW + 1];
                acc += px * r[c1] * s0 + py * r[CW + c1] * s1;
            }
        __syncthreads();
    }
    // Schur terms of the points [a0, a1), pipelined the same way
    double rpt[RPT];
    auto fetch_p = [&](int64_t base) {
        const int n = (int)min((int64_t)CH, a1 - base);
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const int idx = q + 128 * r, kk = idx / FP, f = idx - kk * FP;
            if (idx < n * FP) rpt[r] = PT[(base + kk) * PS + 6 + (f < 3 ? f : f + 3)];
        }
        return n;
    };
    n_cur = a0 < a1 ? fetch_p(a0) : 0;
    for (int64_t base = a0; base < a1; base += CH) {
        const int n = n_cur;
#pragma unroll
        for (int r = 0; r < RPT; ++r) {
            const int idx = q + 128 * r, kk = idx / FP, f = idx - kk * FP;
            if (idx < n * FP) sp[kk][f] = rpt[r];
        }
        __syncthreads();
        if (base + CH < a1) n_cur = fetch_p(base + CH);
        if (act)
            for (int kk = 0; kk < n; ++kk) {
                const double* r = sp[kk];  // vb 0..2, Wc 3.., Tc 3+3CW..
                if (c2 >= 0) {
                    const double* T = r + 3 + 3 * CW + 3 * c1;
                    const double* W = r + 3 + 3 * c2;
                    acc -= T[0] * W[0] + T[1] * W[1] + T[2] * W[2];
                } else {
                    const double* W = r + 3 + 3 * c1;
                    acc -= W[0] * r[0] + W[1] * r[1] + W[2] * r[2];
                }
            }
        __syncthreads();
    }
    if (act) slab[((int64_t)k * NSLAB + s) * (NPK + CW) + q] = acc;
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
// border (inner constraints, main.m:428-436).  The reference solves [S G; G' 0].  Here
//   M = S + G_l W_l G_l'   with G_l = the rows of G of the first n_loc images only (local border:
//                           M stays banded), w_m = 1 / sum_{i in loc} G_im^2 / S_ii (equilibrated)
// and the exact bordered solution follows from the forward-solved right-hand sides
//   r | A = G_l W_l^1/2 | B = G D   (D = the same equilibration over all images; B'x = 0 <=> G'x = 0)
// in k_border_combine.  scal: [1] Cholesky failure flag, [2] sumabs, [8..14] W_l, [16..22] D^2.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_border_weights(const double* __restrict__ S, const double* __restrict__ G,
                                                         double* __restrict__ scal, int64_t ld, int n_img, int n_loc,
                                                         int ic) {
    __shared__ double red[16][14];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    double a[14];
#pragma unroll
    for (int m = 0; m < 14; ++m) a[m] = 0.0;
    if (ic) {
        for (int64_t i = tid; i < 6 * (int64_t)n_img; i += 1024) {
            const double sii = S[i * ld + i];
            const double* g = G + (i / 6) * 42 + (i % 6) * 7;
            const bool ok = sii > 0.0, loc = i < 6 * (int64_t)n_loc;
            const double inv = ok ? 1.0 / sii : 0.0;
#pragma unroll
            for (int m = 0; m < 7; ++m) {
                const double v = g[m] * g[m] * inv;
                a[7 + m] += v;
                if (loc) a[m] += v;
            }
        }
    }
#pragma unroll
    for (int m = 0; m < 14; ++m) {
        double v = a[m];
#pragma unroll
        for (int w = 32; w > 0; w >>= 1) v += __shfl_xor(v, w, 64);
        if (lane == 0) red[wave][m] = v;
    }
    __syncthreads();
    if (tid < 14) {
        double v = 0.0;
        for (int w = 0; w < 16; ++w) v += red[w][tid];
        const int m = tid % 7;
        if (tid < 7) scal[8 + m] = v > 0.0 ? 1.0 / v : 1.0;
        else scal[16 + m] = v > 0.0 ? 1.0 / v : 1.0;
    }
    if (tid == 0) scal[1] = 0.0;  // Cholesky failure flag
}

// M += G_l W_l G_l' on the 6 n_loc x 6 n_loc block (lower part)
__global__ void k_border(double* __restrict__ S, const double* __restrict__ G, const double* __restrict__ scal,
                         int64_t ld, int n_loc) {
    const int64_t n = 6 * (int64_t)n_loc;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n * n; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = q / n, j = q % n;
        if (j > i) continue;
        const double* gi = G + (i / 6) * 42 + (i % 6) * 7;
        const double* gj = G + (j / 6) * 42 + (j % 6) * 7;
        double acc = 0.0;
        for (int m = 0; m < 7; ++m) acc += gi[m] * scal[8 + m] * gj[m];
        S[i * ld + j] += acc;
    }
}

__global__ void k_finish_rhs(double* __restrict__ S, const double* __restrict__ G, const double* __restrict__ scal,
                             const uint8_t* __restrict__ active, int64_t ld, int64_t n_pad, int64_t u_c, int n_img,
                             int n_loc, int ic) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    if (i >= u_c || !active[i]) {
        // fixed parameter or padding: decoupled unit row, zero RHS
        S[i * ld + i] = 1.0;
        S[n_pad * ld + i] = 0.0;
    }
    if (ic) {
        const double* g = G + (i / 6) * 42 + (i % 6) * 7;
        for (int m = 0; m < 7; ++m) {
            S[(n_pad + 1 + m) * ld + i] = (i < 6 * (int64_t)n_loc) ? sqrt(scal[8 + m]) * g[m] : 0.0;   // A
            S[(n_pad + 8 + m) * ld + i] = (i < 6 * (int64_t)n_img) ? sqrt(scal[16 + m]) * g[m] : 0.0;  // B
        }
    }
}


// ------------------------------------------------------------------------------------------------
// back-substitution of tie points: dp = -(vb + sum_o T_o^T d_e(o) + Tc^T d_cam)
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ void k_backsub(const double* __restrict__ WT, const double* __restrict__ PT,
                          const int32_t* __restrict__ lp_start, const int32_t* __restrict__ lp_tie,
                          const int32_t* __restrict__ lp_cam, const int32_t* __restrict__ img,
                          double* __restrict__ delta, int64_t n_lp, int64_t u_c, int n_img) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, PS = LY::PS;
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_lp) return;
    const double* P = PT + p * PS;
    double d0 = P[6], d1 = P[7], d2 = P[8];
    for (int o = lp_start[p]; o < lp_start[p + 1]; ++o) {
        const double* de = delta + 6 * (int64_t)img[o];
        const double* T = WT + (int64_t)o * 36 + 18;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            d0 += T[3 * a] * de[a]; d1 += T[3 * a + 1] * de[a]; d2 += T[3 * a + 2] * de[a];
        }
    }
    const double* dk = delta + 6 * (int64_t)n_img + (int64_t)lp_cam[p] * CW;
    const double* Tc = P + 12 + 3 * CW;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        d0 += Tc[3 * c] * dk[c]; d1 += Tc[3 * c + 1] * dk[c]; d2 += Tc[3 * c + 2] * dk[c];
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
                                                   double* __restrict__ part, int64_t n_obs, int64_t u_c, int n_img,
                                                   double px, double py) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, NJ = LY::NJ, JS = LY::JS;
    __shared__ double red[3][256];
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double sx = 0.0, sy = 0.0, sp = 0.0;
    if (o < n_obs) {
        const int e = img[o], k = cam[o], p = pt[o];
        const double* de = delta + 6 * (int64_t)e;
        const double* dk = delta + 6 * (int64_t)n_img + (int64_t)k * CW;
        const double* Jo = J + o * JS;
        double vv[2];
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const double* jr = Jo + r * NJ;
            double acc = Jo[2 * NJ + r];
#pragma unroll
            for (int a = 0; a < 6; ++a) acc += jr[a] * de[a];
#pragma unroll
            for (int c = 0; c < CW; ++c) acc += jr[6 + c] * dk[c];
            if (p >= 0) {
                const double* dp = delta + u_c + 3 * (int64_t)lp_tie[p];
#pragma unroll
                for (int m = 0; m < 3; ++m) acc += jr[6 + CW + m] * dp[m];
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
                            int64_t n_obs, int64_t n_rows, int64_t u_c, int n_img) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, NJ = LY::NJ, JS = LY::JS;
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_obs) return;
    const int e = img[o], k = cam[o], p = pt[o];
    const int64_t row0 = 2 * obs_pho[o];
    const double* Jo = J + o * JS;
    for (int r = 0; r < 2; ++r) {
        const int64_t row = row0 + r;
        const double* jr = Jo + r * NJ;
        w[row] = Jo[2 * NJ + r];
        for (int a = 0; a < 6; ++a) {
            const int64_t col = map[6 * (int64_t)e + a];
            if (col >= 0) A[col * n_rows + row] = jr[a];
        }
        for (int c = 0; c < CW; ++c) {
            const int64_t col = map[6 * (int64_t)n_img + (int64_t)k * CW + c];
            if (col >= 0) A[col * n_rows + row] = jr[6 + c];
        }
        if (p >= 0) {
            for (int m = 0; m < 3; ++m) {
                const int64_t col = map[u_c + 3 * (int64_t)lp_tie[p] + m];
                if (col >= 0) A[col * n_rows + row] = jr[6 + CW + m];
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
    k_params<<<(n + 63) / 64, 64, 0, c.stream>>>(c.d_xfull, c.d_caminfo, c.d_img_tab, c.d_cam_tab, c.d_G, c.d_active,
                                                   c.L.n_img, c.L.n_cam, c.L.nk, c.L.cw, c.cam_tab_stride,
                                                   c.set.inner_constraints);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

// linearisation fused with the tie-point reduction (the dense debug path uses the same kernel)
int launch_linearize(Ctx& c) {
    if (c.n_chunks == 0) return FBA_OK;
    const unsigned em = eop_mask(c.set), cm = cam_mask(c.set, c.L.nk);
#define LIN(NKV)                                                                                               \
    k_lin_point<NKV><<<(unsigned)c.n_chunks, 256, 0, c.stream>>>(                                              \
        c.d_xy, c.d_img, c.d_cam, c.d_pt, c.d_lp_tie, c.d_ctl, c.d_xfull, c.d_img_tab, c.d_cam_tab,             \
        c.d_chunk_obs, c.d_chunk_pt, c.d_lp_start, c.d_J, c.d_WT, c.d_pt_tab, c.L.u_c, c.set.type,              \
        c.cam_tab_stride, em, cm, px_of(c), py_of(c))
    FBA_NK_DISPATCH(c.L.nk, LIN);
#undef LIN
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_point(Ctx& c) {
    (void)c;  // fused into k_lin_point
    return FBA_OK;
}

int launch_accumulate(Ctx& c) {
    const Layout& L = c.L;
    FBA_HIP(hipMemsetAsync(c.d_S, 0, sizeof(double) * (size_t)(L.n_pad + NB) * L.ld, c.stream));
    const double px = px_of(c), py = py_of(c);
#define IMG(NKV)                                                                                          \
    k_image<NKV><<<L.n_img, 256, 0, c.stream>>>(c.d_J, c.d_WT, c.d_pt_tab, c.d_pt, c.d_cam, c.d_img_start, \
                                                c.d_img_obs, c.d_S, L.ld, L.n_pad, L.n_img, px, py)
    FBA_NK_DISPATCH(L.nk, IMG);
#undef IMG
    FBA_HIP(hipGetLastError());
    if (c.n_pairs > 0) {
        k_pairs<<<(unsigned)(8 * ((c.n_pairs + 7) / 8)), 64, 0, c.stream>>>(c.d_WT, c.d_pair_e, c.d_pair_start,
                                                                       c.d_pair_ij, c.d_S, L.ld, c.n_pairs);
        FBA_HIP(hipGetLastError());
    }
    dim3 g1(NSLAB, L.n_cam);
#define CAM(NKV)                                                                                               \
    k_cam_stage1<NKV><<<g1, 128, 0, c.stream>>>(c.d_J, c.d_pt_tab, c.d_lp_start, c.d_cam_lp, c.d_cam_ctl,     \
                                                c.d_slab, c.n_obs_tie, px, py);                               \
    k_cam_stage2<NKV><<<L.n_cam, 128, 0, c.stream>>>(c.d_slab, c.d_S, L.ld, L.n_pad, L.n_img)
    FBA_NK_DISPATCH(L.nk, CAM);
#undef CAM
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_border(Ctx& c) {
    const Layout& L = c.L;
    const int ic = c.set.inner_constraints;
    k_border_weights<<<1, 1024, 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, L.ld, L.n_img, c.n_loc, ic);
    FBA_HIP(hipGetLastError());
    if (ic && c.n_loc > 0) {
        const int64_t n = 6 * (int64_t)c.n_loc;
        k_border<<<(unsigned)((n * n + 255) / 256), 256, 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, L.ld, c.n_loc);
        FBA_HIP(hipGetLastError());
    }
    k_finish_rhs<<<(unsigned)((L.n_pad + 255) / 256), 256, 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, c.d_active,
                                                                           L.ld, L.n_pad, L.u_c, L.n_img, c.n_loc, ic);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_backsub_update(Ctx& c) {
    const Layout& L = c.L;
    if (c.n_lp > 0) {
        const int blocks = (int)((c.n_lp + 255) / 256);
#define BS(NKV)                                                                                               \
    k_backsub<NKV><<<blocks, 256, 0, c.stream>>>(c.d_WT, c.d_pt_tab, c.d_lp_start, c.d_lp_tie, c.d_lp_cam,    \
                                                 c.d_img, c.d_delta, c.n_lp, L.u_c, L.n_img)
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
                                                   c.d_part, c.n_obs, L.u_c, L.n_img, px_of(c), py_of(c))
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
                                                   c.d_obs_pho, d_map, dA, dW, c.n_obs, n_rows, c.L.u_c,      \
                                                   c.L.n_img)
    FBA_NK_DISPATCH(c.L.nk, DA);
#undef DA
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}


// ------------------------------------------------------------------------------------------------
// multi-rank compact reduce buffer: [global pair blocks 6x6 | diagonal blocks 6x6 | camera rows | RHS row]
// dir 0: red <- S (after the accumulation), dir 1: S <- red (after the all-reduce)
// ------------------------------------------------------------------------------------------------
__global__ void k_pack(double* __restrict__ S, int64_t ld, double* __restrict__ red, const int32_t* __restrict__ gp,
                       int64_t n_gp, int n_img, int64_t n_camrows, int64_t n_pad, int dir) {
    const int64_t n_blk = 36 * (n_gp + n_img), n_cam = n_camrows * n_pad;
    const int64_t total = n_blk + n_cam + n_pad;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (int64_t)gridDim.x * blockDim.x) {
        int64_t pos;
        if (q < n_blk) {
            const int64_t b = q / 36;
            const int a = (int)(q % 36) / 6, c = (int)(q % 6);
            const int64_t e1 = b < n_gp ? gp[2 * b] : b - n_gp, e2 = b < n_gp ? gp[2 * b + 1] : b - n_gp;
            pos = (6 * e1 + a) * ld + 6 * e2 + c;
        } else if (q < n_blk + n_cam) {
            const int64_t r = (q - n_blk) / n_pad, col = (q - n_blk) % n_pad;
            pos = (6 * (int64_t)n_img + r) * ld + col;
        } else {
            pos = n_pad * ld + (q - n_blk - n_cam);
        }
        if (dir == 0) red[q] = S[pos];
        else S[pos] = red[q];
    }
}

int launch_pack(Ctx& c, int dir) {
    const int64_t ncr = (int64_t)c.L.cw * c.L.n_cam;
    const int64_t total = c.n_red;
    const unsigned grid = (unsigned)std::min<int64_t>((total + 255) / 256, 8192);
    k_pack<<<grid, 256, 0, c.stream>>>(c.d_S, c.L.ld, c.d_red, c.d_gpairs, c.n_gpairs, c.L.n_img, ncr, c.L.n_pad, dir);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

}  // namespace fba
