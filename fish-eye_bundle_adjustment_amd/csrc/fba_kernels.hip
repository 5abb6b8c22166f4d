// fba_kernels.hip -- linearisation and normal-equation kernels for gfx950 (MI355X).
//
// One Gauss-Newton pass (the reference's main.m:413-488 with BuildAwG.m:46-527 inside) becomes:
//   k_params        per image: EOPs + rotation M and dM/d(omega,phi,kappa) (BuildAwG.m:163-165),
//                   inner-constraint block G (BuildAwG.m:516-523); per camera: IOPs, rmax^(2j)
//                   scales (BuildAwG.m:422-426)
//   k_lin_reduce    per chunk of whole tie points (one camera): the misclosure w (BuildAwG.m:505-512)
//                   and the 2 Jacobian rows over [6 EOP | xp yp c K1..Knk P1 P2 | X Y Z]
//                   (BuildAwG.m:216-503) by the chain rule of the forward model (BuildAwG.m:163-213),
//                   the tie-point elimination (V = Jp'PJp, its factor, couplings) and the chunk's
//                   partial sums of every reduced block it touches, all in registers and LDS
//   k_red_*         the partials of each reduced block added in chunk order: image-pair blocks,
//                   image diagonal blocks + RHS + image-camera blocks, camera blocks
//   k_lin_point     the same linearisation writing the Jacobian rows out (residuals, dense AwG)
//   k_border_rhs    inner-constraint bordering M = S + G W G' (reference: NG = [N G; G' 0],
//                   main.m:428-432), unit diagonal for fixed parameters, RHS rows
//   k_backsub       tie-point corrections from the camera-side solution
//   k_update        de-scaling of distortion corrections (main.m:460-482), xhat += delta
//                   (main.m:484), deltasum = sumabs(delta) (main.m:487, sumabs.m:12-14)
//   k_residuals     v = A*delta + w (main.m:569), BuildRSD rows (BuildRSD.m:29-40), v'Pv
// Every reduction is a fixed-order sum (no float atomics), so results are bitwise reproducible.
#include "fba_internal.h"

namespace fba {

// lane-permuted copy of a double within rows of the wave (DPP control CTRL: quad_perm, row_half_mirror)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}


// ------------------------------------------------------------------------------------------------
// k_params: per-image and per-camera tables
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void params_body(int t, int nthreads, const double* __restrict__ xfull,
                                            const double* __restrict__ caminfo, double* __restrict__ img_tab,
                                            double* __restrict__ cam_tab, double* __restrict__ G,
                                            const uint8_t* __restrict__ active, int n_img, int n_cam, int nk, int cw,
                                            int cam_stride, int ic, double* __restrict__ xcopy, int64_t n_copy) {
    if (xcopy)  // the linearisation point (main.m:569 uses it for v), copied by the whole grid
        for (int64_t i = t; i < n_copy; i += nthreads) xcopy[i] = xfull[i];
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
            // tan(phi), sec(phi) from the sincos above (equal to tan() / 1 / cos() to rounding)
            const double secp = 1.0 / cp, tp = sp * secp;
            const double rows[42] = {
                1, 0, 0, 0, -Zc, Yc, Xc,
                0, 1, 0, Zc, 0, -Xc, Yc,
                0, 0, 1, -Yc, Xc, 0, Zc,
                0, 0, 0, -1, -sw * tp, cw_ * tp, 0,
                0, 0, 0, 0, -cw_, -sw, 0,
                0, 0, 0, 0, sw * secp, -cw_ * secp, 0};
            const bool slot = active[6 * (int64_t)t];  // padding slots (fba_order.cpp) carry no constraint
#pragma unroll
            for (int i = 0; i < 42; ++i) g[i] = slot ? rows[i] : 0.0;
        }
    }
}

// the camera table of camera k, one workgroup: thread 0 the header, thread j in 1..nk the distortion term j
// (its rmax^(2j) and reciprocal) -- the nk pow calls in parallel instead of one thread's chain
__device__ __forceinline__ void cam_params_body(int k, int j, const double* __restrict__ xfull,
                                                const double* __restrict__ caminfo, double* __restrict__ cam_tab, int n_img,
                                                int nk, int cw, int cam_stride) {
    const double* q = xfull + 6 * (int64_t)n_img + (int64_t)k * cw;
    const double* ci = caminfo + 5 * k;
    double* o = cam_tab + (int64_t)k * cam_stride;
    const double hx = (ci[3] - ci[1]) * 0.5, hy = (ci[4] - ci[2]) * 0.5;
    const double rmax = sqrt(hx * hx + hy * hy);  // BuildAwG.m:422
    if (j == 0) {
        o[0] = q[0];            // xp
        o[1] = q[1];            // yp
        o[2] = q[2];            // c
        o[3] = ci[0];           // y_dir
        o[4] = q[3 + nk];       // P1
        o[5] = q[4 + nk];       // P2
        o[6] = pow(rmax, 2.0);  // rmax^2 (= the j = 1 term below)
        o[7] = rmax;
    } else if (j <= nk) {
        o[CAM_TAB_HDR + j - 1] = q[2 + j];                     // K_j
        const double r2j = pow(rmax, 2.0 * j);                  // rmax^(2j), BuildAwG.m:424-426
        o[CAM_TAB_HDR + nk + j - 1] = r2j;
        o[CAM_TAB_HDR + 2 * nk + j - 1] = 1.0 / r2j;            // its reciprocal (obs_model)
    }
}

// 64-thread workgroups: [0, nbi) the image tables, [nbi, nb) one camera each, [nb, grid) the copy of
// the linearisation point with four independent loads in flight per thread, so the table waves do not
// first wait out serial copy iterations (kernel time = max of the three instead of their sum)
constexpr int PARAMS_WG = 64;
__global__ __launch_bounds__(PARAMS_WG) void k_params(const double* __restrict__ xfull, const double* __restrict__ caminfo,
                                                      double* __restrict__ img_tab, double* __restrict__ cam_tab,
                                                      double* __restrict__ G, const uint8_t* __restrict__ active, int n_img,
                                                      int n_cam, int nk, int cw, int cam_stride, int ic,
                                                      double* __restrict__ xcopy, int64_t n_copy) {
    const int nbi = (n_img + PARAMS_WG - 1) / PARAMS_WG, nb = nbi + n_cam;
    if ((int)blockIdx.x < nbi) {
        params_body(blockIdx.x * PARAMS_WG + threadIdx.x, nbi * PARAMS_WG, xfull, caminfo, img_tab, cam_tab, G, active,
                    n_img, n_cam, nk, cw, cam_stride, ic, nullptr, 0);
        return;
    }
    if ((int)blockIdx.x < nb) {
        cam_params_body(blockIdx.x - nbi, threadIdx.x, xfull, caminfo, cam_tab, n_img, nk, cw, cam_stride);
        return;
    }
    if (!xcopy) return;
    const int64_t t = (int64_t)(blockIdx.x - nb) * PARAMS_WG + threadIdx.x, st = (int64_t)(gridDim.x - nb) * PARAMS_WG;
    double v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = t + j * st < n_copy ? xfull[t + j * st] : 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (t + j * st < n_copy) xcopy[t + j * st] = v[j];
    for (int64_t i = t + 4 * st; i < n_copy; i += st) xcopy[i] = xfull[i];
}


// ------------------------------------------------------------------------------------------------
// Device layouts (observation-major so a thread / wave touches contiguous bytes):
//   J   [o][JS], JS = 2*NJ + 2: Jacobian row x (NJ columns: 6 EOP | CW camera | 3 XYZ), row y, w
//   WT  [o][18]: T = W Vinv at 3a+m, W = Je' P Jp (the back-substitution's only per-observation input)
//   PT  [p][PS], PS = 12 + 6*CW: Vinv (00 01 02 11 12 22), vb = Vinv b, b, Wc[c][m], Tc = Wc Vinv
// ------------------------------------------------------------------------------------------------
template <int NK>
struct Lay {
    static constexpr int CW = 5 + NK;
    static constexpr int NJ = 9 + CW;
    static constexpr int JS = 2 * NJ + 2;
    static constexpr int PS = 12 + 6 * CW;
};

// The per-observation record of the back-substitution, WT[o] (OBS_REC = 12 doubles, 96 B): the raw
// tie-point Jacobian rows Jp (x: 0..2, y: 3..5) and the rotation columns of the EOP rows (x: 6..8, y:
// 9..11).  The position columns of the EOP rows are -Jp (obs_model: d(UVW)/dXc = -d(UVW)/dX exactly),
// masked by the EOP mask; so W = Je'PJp and T = W Vinv follow from the record and the point's Vinv.
constexpr int OBS_REC = 12;
__device__ __forceinline__ void obs_rec_rows(const double* __restrict__ r, unsigned eop_mask, double (&j0)[6],
                                             double (&j1)[6]) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double en = (eop_mask >> q) & 1u ? 1.0 : 0.0;
        j0[q] = -r[q] * en;
        j1[q] = -r[3 + q] * en;
        j0[3 + q] = r[6 + q];
        j1[3 + q] = r[9 + q];
    }
}
// T = W Vinv (6 x 3, row a at 3 a) of one observation from its record and the point's Vinv (00 01 02 11 12 22)
__device__ __forceinline__ void obs_rec_T(const double* __restrict__ r, const double* __restrict__ vi, unsigned eop_mask,
                                          double px, double py, double* __restrict__ To) {
    double j0[6], j1[6];
    obs_rec_rows(r, eop_mask, j0, j1);
    const double I00 = vi[0], I01 = vi[1], I02 = vi[2], I11 = vi[3], I12 = vi[4], I22 = vi[5];
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        const double e0 = px * j0[a], e1 = py * j1[a];
        const double v0 = e0 * r[0] + e1 * r[3];
        const double v1 = e0 * r[1] + e1 * r[4];
        const double v2 = e0 * r[2] + e1 * r[5];
        To[3 * a] = v0 * I00 + v1 * I01 + v2 * I02;
        To[3 * a + 1] = v0 * I01 + v1 * I11 + v2 * I12;
        To[3 * a + 2] = v0 * I02 + v1 * I12 + v2 * I22;
    }
}

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
    // (divisions by R, q and the distortion scalings as products with reciprocals: one f64 division
    // is ~10 instructions, the model had ~25 of them per observation)
    const double iR = 1.0 / R;
    // radial factor s(R,W): f_proj = -c*(U, ydir*V)*s  (BuildAwG.m:184-208)
    double s, sR, sW;
    if (type == FBA_TYPE_PINHOLE) {
        s = 1.0 / W; sR = 0.0; sW = -1.0 / (W * W);
    } else {
        const double t = atan(R / W);
        const double iq = 1.0 / (R * R + W * W);
        const double tR = W * iq, tW = -R * iq;
        double g, gt;
        if (type == FBA_TYPE_FISHEYE) { g = t; gt = 1.0; }
        else if (type == FBA_TYPE_EQUISOLID) { double sh, ch; sincos(0.5 * t, &sh, &ch); g = 2.0 * sh; gt = ch; }
        else if (type == FBA_TYPE_ORTHOGRAPHIC) { double st, ctt; sincos(t, &st, &ctt); g = st; gt = ctt; }
        else { double th = tan(0.5 * t); double ch = cos(0.5 * t); g = 2.0 * th; gt = 1.0 / (ch * ch); }
        s = g * iR;
        sR = (gt * tR - s) * iR;
        sW = gt * tW * iR;
    }
    const double xp = ct[0], yp = ct[1], c = ct[2], ydir = ct[3], P1 = ct[4], P2 = ct[5];
    const double* K = ct + CAM_TAB_HDR;
    const double* isc = ct + CAM_TAB_HDR + 2 * NK;  // 1 / rmax^(2j)
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
        const double dR = (U * dU + V * dV) * iR;
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
        jr[0][8 + j] = r2j[j] * xb * isc[j - 1] * en;
        jr[1][8 + j] = r2j[j] * yb * isc[j - 1] * en;
    }
    const double is1 = isc[0], en1 = cen(3 + NK), en2 = cen(4 + NK);
    jr[0][9 + NK] = (yb * yb + 3.0 * xb * xb) * is1 * en1;
    jr[1][9 + NK] = 2.0 * xb * yb * is1 * en1;
    jr[0][10 + NK] = 2.0 * xb * yb * is1 * en2;
    jr[1][10 + NK] = (xb * xb + 3.0 * yb * yb) * is1 * en2;
    w0 = fx - x;
    w1 = fy - y;
}

// ------------------------------------------------------------------------------------------------
// k_lin_point: one workgroup per chunk of whole tie points (<= 256 observations), one thread per
// image point.  (1) linearise and store J; (2) one thread per point reduces its observations
// (staged in LDS): V = Jp'PJp, b = Jp'Pw, Wc = Jc'PJp, Vinv, vb, Tc; (3) one thread per observation
// stores its record (OBS_REC).  Chunks of control observations run step (1) only.
// ------------------------------------------------------------------------------------------------
template <int NK>
__global__ __launch_bounds__(256) void k_lin_point(
    const double* __restrict__ xy, const int32_t* __restrict__ img, const int32_t* __restrict__ cam,
    const int32_t* __restrict__ pt, const int32_t* __restrict__ lp_tie, const double* __restrict__ ctl,
    const double* __restrict__ xfull, const double* __restrict__ img_tab, const double* __restrict__ cam_tab,
    const int32_t* __restrict__ chunk_obs, const int32_t* __restrict__ chunk_pt, const int32_t* __restrict__ lp_start,
    double* __restrict__ J, double* __restrict__ WT, double* __restrict__ PT, int64_t u_c, int type, int cam_stride,
    unsigned eop_mask, unsigned cam_mask, double px, double py, int c_off) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, NJ = LY::NJ, JS = LY::JS, PS = LY::PS;
    constexpr int SH = 8 + 2 * CW;  // Jp (2x3), w (2), Jc (2xCW)
    __shared__ double sh[256][SH + 1];
    __shared__ double vinv[256][6];
    const int t = threadIdx.x;
    const int c = blockIdx.x + c_off;
    const int o0 = chunk_obs[c], o1 = chunk_obs[c + 1];
    const int p0 = chunk_pt[c], p1 = chunk_pt[c + 1];
    const int o = o0 + t;
    const bool active = t < CHUNK_OBS && o < o1;
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
    if (active && p >= 0) {  // the observation's record (OBS_REC)
        double2* r = reinterpret_cast<double2*>(WT + (int64_t)o * OBS_REC);
        r[0] = double2{jr[0][6 + CW], jr[0][7 + CW]};
        r[1] = double2{jr[0][8 + CW], jr[1][6 + CW]};
        r[2] = double2{jr[1][7 + CW], jr[1][8 + CW]};
        r[3] = double2{jr[0][3], jr[0][4]};
        r[4] = double2{jr[0][5], jr[1][3]};
        r[5] = double2{jr[1][4], jr[1][5]};
    }
}

// ------------------------------------------------------------------------------------------------
// k_lin_reduce: the Gauss-Newton linearisation and the point-reduced normal equations of one chunk
// (<= 256 observations of <= 64 whole tie points of one camera, or control observations), from
// registers and LDS only -- no Jacobian round trip through HBM, no gathers:
//   (A) one thread per observation: forward model and Jacobian (obs_model, BuildAwG.m:163-503);
//   (B) one thread per point: V = Jp'PJp, b = Jp'Pw, Wc = Jc'PJp, V^-1, vb = V^-1 b, Tc = Wc V^-1
//       (V^-1, vb, Tc to HBM for the back-substitution), and the factor R = L^-T of V = L L' (so
//       V^-1 = R R'), rb = R'b, Uc = Wc R;
//   (C) one thread per observation: W = Je'PJp, U = W R; its record (OBS_REC, 96 B: Jp and the
//       rotation columns of Je) to HBM for the back-substitution;
//       the observation's P^1/2-scaled Jacobian rows and misclosures into LDS;
//   (D) every (key, entry) of the chunk's partial sums (keys from the host plan, AccPlan):
//         camera     Jc'PJc - Uc Uc',  Jc'Pw - Uc rb                         (summed over the chunk)
//         image e    Je'PJe - U U' (lower), Je'Pw - U rb, Jc'PJe - Uc U'     (its observations)
//         pair e1>e2 -sum U_i U_j'  over the chunk's points seen by both     (= -T_i W_j')
//       each summed in a fixed order and stored as one partial; k_red_* add the partials of a
//       block in chunk order, so the result is deterministic.  A U-row chunk (AccPlan::ck_tm: its
//       pair keys hold few terms each, a dense network's) registers no pair keys and writes its
//       observations' U rows instead (Ug, 144 B each); k_red_blocks sums those terms per pair.
// The Schur complement identities: W V^-1 W' = U U', W V^-1 b = U rb, Wc V^-1 W' = Uc U'.
// ------------------------------------------------------------------------------------------------
__constant__ int c_tri_a[21] = {0, 1, 1, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 5, 5};
__constant__ int c_tri_b[21] = {0, 0, 1, 0, 1, 2, 0, 1, 2, 3, 0, 1, 2, 3, 4, 0, 1, 2, 3, 4, 5};

template <int NK>
struct LR {
    static constexpr int CW = 5 + NK;
    // row strides of the per-observation LDS rows: even (16-B aligned rows, ds_read_b128) and = 2 mod 4
    // doubles, so a row starts 4 x (odd) dwords apart from the next: 16 distinct bank quadruples over 16
    // rows (the (D) loops read the rows of random observations; a stride = 0 mod 4 doubles gives 8)
    static constexpr int ES = 14 + 2 * CW + ((14 + 2 * CW) % 4 == 0 ? 2 : 0);  // staging: Je | w | Jc (+ 2 for even nK)
    static constexpr int US = 18;                   // U row (exactly)
    static_assert(ES % 4 == 2 && US % 4 == 2, "LDS row strides of 2 mod 4 doubles");
    static constexpr int PPS = 15 + 3 * CW;         // per-point: Vinv 6 | R 6 | rb 3 | Uc 3CW
    static constexpr int NIMG = 27 + 6 * CW;        // image partial: 21 lower + 6 RHS + 6CW image-camera
    static constexpr int NCAM = CW * (CW + 1) / 2 + CW;
    // + ints: point of each observation, the chunk's plan (pair-key term offsets, terms, image-key
    // observation offsets, observations)
    static constexpr int CP = chunk_pts(NK), CT = chunk_terms(NK);
    static constexpr int NI = CHUNK_OBS + (CT + 1) + CT + (CHUNK_OBS + 1) + CHUNK_OBS + CT + CHUNK_OBS;
    // camera entries: CAM_SPLIT - 1 observation sub-ranges and the points' Schur terms in parallel
    static constexpr int CAM_SPLIT = 512 / NCAM;
    static_assert(CAM_SPLIT >= 2, "camera entries: at least one observation part and the points' part");
    static constexpr size_t LDS = sizeof(double) * (CHUNK_OBS * ES + CHUNK_OBS * US + CP * PPS + 512) +
                                  sizeof(int) * NI;
    static_assert(LDS <= 160 * 1024, "k_lin_reduce LDS over the 160 KiB of a CU");
};

constexpr int LR_THREADS = 512;  // observation phases use the first CHUNK_OBS threads, (D) all of them

template <int NK, int IKL>
__global__ __launch_bounds__(LR_THREADS) void k_lin_reduce(
    const double* __restrict__ xy, const int32_t* __restrict__ img, const int32_t* __restrict__ cam,
    const int32_t* __restrict__ pt, const int32_t* __restrict__ lp_tie, const double* __restrict__ ctl,
    const double* __restrict__ xfull, const double* __restrict__ img_tab, const double* __restrict__ cam_tab,
    const int32_t* __restrict__ chunk_obs, const int32_t* __restrict__ chunk_pt, const int32_t* __restrict__ lp_start,
    const int32_t* __restrict__ A, const AccPlan plan, double* __restrict__ WT, double* __restrict__ PT,
    double* __restrict__ ppart, double* __restrict__ ipart, double* __restrict__ cpart, int64_t u_c, int type,
    int cam_stride, unsigned eop_mask, unsigned cam_mask, double px, double py, uint64_t* __restrict__ tprof,
    int n_chunks, double* __restrict__ S, int64_t ld, const int32_t* __restrict__ zblk,
    const int32_t* __restrict__ xoff, double* __restrict__ Ug) {
    using LY = Lay<NK>;
    using R_ = LR<NK>;
    if ((int)blockIdx.x >= n_chunks) {  // tail workgroups: zero one 128x128 block of the factor's pattern
        // (Sched::zero) each; they run on the CUs the last round of chunks leaves idle.  They are
        // launched with the chunk workgroups' dynamic LDS (LR<NK>::LDS) and thread count, so each takes
        // a chunk-sized LDS allocation: a larger chunk footprint serialises them too.
        static_assert(NB == 128 && (NB * NB / 2) % LR_THREADS == 0, "tail zeroing assumes 128x128 blocks");
        const int b = blockIdx.x - n_chunks;
        const int64_t r0 = (int64_t)zblk[2 * b] * NB, c0 = (int64_t)zblk[2 * b + 1] * NB;
        const double2 z = {0.0, 0.0};
#pragma unroll
        for (int q = 0; q < NB * NB / 2 / LR_THREADS; ++q) {
            const int i = threadIdx.x + LR_THREADS * q, r = i >> 6, cc = (i & 63) * 2;
            *reinterpret_cast<double2*>(S + (r0 + r) * ld + c0 + cc) = z;
        }
        return;
    }
    // optional phase timestamps (FBA_LR_PROFILE): 100 MHz wall clock at the phase boundaries
    auto stamp = [&](int i) {
        if (tprof && threadIdx.x == 0) tprof[(int64_t)blockIdx.x * 8 + i] = wall_clock64();
    };
    stamp(0);
    constexpr int CW = LY::CW, NJ = LY::NJ, PS = LY::PS;
    constexpr int ES = R_::ES, US = R_::US, PPS = R_::PPS, NIMG = R_::NIMG, NCAM = R_::NCAM;
    constexpr int CAM_SPLIT = R_::CAM_SPLIT;
    static_assert(LR_THREADS >= 512 && LR_THREADS >= CHUNK_OBS, "thread roles");
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* QE = lds;                                  // [CHUNK_OBS][ES]
    double* Us = QE + CHUNK_OBS * ES;                  // [CHUNK_OBS][US]
    double* PP = Us + CHUNK_OBS * US;                  // [CP][PPS]
    double* camp = PP + R_::CP * PPS;                        // [CAM_SPLIT][NCAM] camera sub-range sums
    int* pl = reinterpret_cast<int*>(camp + 512);            // [CHUNK_OBS] chunk-local point or -1
    int* s_pkt = pl + CHUNK_OBS;                             // [<= CT + 1] term offsets of the pair keys
    int* s_term = s_pkt + R_::CT + 1;                        // [<= CT]
    int* s_iko = s_term + R_::CT;                            // [<= CHUNK_OBS + 1] observation offsets of image keys
    int* s_ikobs = s_iko + CHUNK_OBS + 1;                    // [<= CHUNK_OBS]
    int* s_pks = s_ikobs + CHUNK_OBS;                        // [<= CT] the pair keys' partial rows (pk_slot)
    int* s_iks = s_pks + R_::CT;                             // [<= CHUNK_OBS] the image keys' rows (ik_slot)
    const int t = threadIdx.x;
    const int c = blockIdx.x;
    const int o0 = chunk_obs[c], o1 = chunk_obs[c + 1];
    const int p0 = chunk_pt[c], p1 = chunk_pt[c + 1];
    const int o = o0 + t;
    const bool active = t < CHUNK_OBS && o < o1;
    // the chunk's plan lists, staged in LDS for (D) (every inner loop then runs out of LDS; the terms
    // of a chunk holding one point with more than CT of them stay in HBM) by the threads
    // (A) leaves idle, while (A) runs
    const int kp0 = A[plan.ck_pk + c], kp1 = A[plan.ck_pk + c + 1];
    const int ki0 = A[plan.ck_ik + c], ki1 = A[plan.ck_ik + c + 1];
    const int tb0 = A[plan.pk_t + kp0], ntm = A[plan.pk_t + kp1] - tb0;
    const int ob0 = A[plan.ik_o + ki0], nio = A[plan.ik_o + ki1] - ob0;
    const bool stage_terms = ntm <= R_::CT;
    if (t >= CHUNK_OBS) {  // the threads the linearisation leaves idle, 8 loads each in flight
        constexpr int NS = LR_THREADS - CHUNK_OBS;
        const int u = t - CHUNK_OBS;
        auto stage = [&](int n, const int32_t* __restrict__ src, int sub, int* __restrict__ dst) {
            for (int i0 = 0; i0 < n; i0 += 8 * NS) {
                int v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + u + NS * q;
                    v[q] = i < n ? src[i] : 0;
                }
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int i = i0 + u + NS * q;
                    if (i < n) dst[i] = v[q] - sub;
                }
            }
        };
        if (stage_terms) {
            stage(kp1 - kp0 + 1, A + plan.pk_t + kp0, tb0, s_pkt);
            stage(ntm, A + plan.pk_term + tb0, 0, s_term);
            stage(kp1 - kp0, A + plan.pk_slot + kp0, 0, s_pks);
        }
        stage(ki1 - ki0, A + plan.ik_slot + ki0, 0, s_iks);
        stage(ki1 - ki0 + 1, A + plan.ik_o + ki0, ob0, s_iko);
        stage(nio, A + plan.ik_obs + ob0, 0, s_ikobs);
    }
    double jr[2][NJ];
    double w0 = 0.0, w1 = 0.0;
    int p = -1;
    // (A)
    if (active) {
        // (the point's coordinates at xfull[xoff[o]]: one gather level fewer than pt -> lp_tie -> xfull)
        const double2 xyv = *reinterpret_cast<const double2*>(xy + 2 * (int64_t)o);
        const int e = img[o], k = cam[o], xo = xoff[o];
        p = pt[o];
        const double* q = p >= 0 ? xfull + xo : ctl + 3 * (int64_t)(-1 - p);
        const double X = q[0], Y = q[1], Z = q[2];
        obs_model<NK>(xyv.x, xyv.y, img_tab + (int64_t)e * IMG_TAB, cam_tab + (int64_t)k * cam_stride, X, Y, Z, p >= 0,
                      type, eop_mask, cam_mask, jr, w0, w1);
        if (p >= 0) {
            double* q = QE + t * ES;  // Jp (2x3) | w (2) | Jc (2xCW), raw
#pragma unroll
            for (int m = 0; m < 3; ++m) { q[m] = jr[0][6 + CW + m]; q[3 + m] = jr[1][6 + CW + m]; }
            q[6] = w0;
            q[7] = w1;
#pragma unroll
            for (int m = 0; m < CW; ++m) { q[8 + m] = jr[0][6 + m]; q[8 + CW + m] = jr[1][6 + m]; }
        }
    }
    if (t < CHUNK_OBS) pl[t] = (active && p >= 0) ? p - p0 : -1;
    __syncthreads();
    stamp(1);
    // (B) four lanes per point (g = t & 3): lane g accumulates the point's observations g, g + 4, ..;
    // V and b are all-reduced over the four lanes, the camera couplings Wc reduce-scattered (lane g
    // keeps camera columns [CWQ g', CWQ g' + CWQ)), each by two DPP exchange steps in a fixed order;
    // every lane then forms V^-1 and the factor R, and the outputs of its own Wc columns
    if (t < 4 * (p1 - p0)) {
        constexpr int CWQ = (CW + 3) / 4, CWP = 4 * CWQ;  // columns per lane, padded count
        const int g = t & 3, tp = t >> 2;
        const int lp = p0 + tp;
        const int a0 = lp_start[lp] - o0, a1 = lp_start[lp + 1] - o0;
        double V[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // V00 V01 V02 V11 V12 V22 b0 b1 b2
        double Wc[CWP][3];
#pragma unroll
        for (int q = 0; q < CWP; ++q) Wc[q][0] = Wc[q][1] = Wc[q][2] = 0.0;
        for (int i = a0 + g; i < a1; i += 4) {
            const double* r = QE + i * ES;
#pragma unroll
            for (int row = 0; row < 2; ++row) {
                const double pr = row ? py : px;
                const double j0 = r[3 * row], j1 = r[3 * row + 1], j2 = r[3 * row + 2], wv = r[6 + row];
                const double q0 = pr * j0, q1 = pr * j1, q2 = pr * j2;
                V[0] += q0 * j0; V[1] += q0 * j1; V[2] += q0 * j2;
                V[3] += q1 * j1; V[4] += q1 * j2; V[5] += q2 * j2;
                V[6] += q0 * wv; V[7] += q1 * wv; V[8] += q2 * wv;
#pragma unroll
                for (int q = 0; q < CW; ++q) {
                    const double jc = r[8 + row * CW + q];
                    Wc[q][0] += jc * q0; Wc[q][1] += jc * q1; Wc[q][2] += jc * q2;
                }
            }
        }
#pragma unroll
        for (int m = 0; m < 9; ++m) {
            V[m] += dpp_d<0x4E>(V[m]);  // quad_perm [2,3,0,1]
            V[m] += dpp_d<0xB1>(V[m]);  // quad_perm [1,0,3,2]
        }
        const bool hA = (g & 2) != 0, hB = (g & 1) != 0;
        double W2[2 * CWQ][3], W1[CWQ][3];
#pragma unroll
        for (int q = 0; q < 2 * CWQ; ++q)
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const double keep = hA ? Wc[2 * CWQ + q][m] : Wc[q][m], give = hA ? Wc[q][m] : Wc[2 * CWQ + q][m];
                W2[q][m] = keep + dpp_d<0x4E>(give);
            }
#pragma unroll
        for (int q = 0; q < CWQ; ++q)
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const double keep = hB ? W2[CWQ + q][m] : W2[q][m], give = hB ? W2[q][m] : W2[CWQ + q][m];
                W1[q][m] = keep + dpp_d<0xB1>(give);
            }
        const int qb = (hA ? 2 * CWQ : 0) + (hB ? CWQ : 0);  // this lane's first camera column
        const double V00 = V[0], V01 = V[1], V02 = V[2], V11 = V[3], V12 = V[4], V22 = V[5];
        const double b0 = V[6], b1 = V[7], b2 = V[8];
        // symmetric 3x3 inverse (adjugate)
        const double c00 = V11 * V22 - V12 * V12, c01 = V02 * V12 - V01 * V22, c02 = V01 * V12 - V02 * V11;
        const double id = 1.0 / (V00 * c00 + V01 * c01 + V02 * c02);
        const double I00 = c00 * id, I01 = c01 * id, I02 = c02 * id;
        const double I11 = (V00 * V22 - V02 * V02) * id, I12 = (V01 * V02 - V00 * V12) * id,
                     I22 = (V00 * V11 - V01 * V01) * id;
        // V = L L', R = L^-T (upper): r00 = m00, r01 = m10, r02 = m20, r11 = m11, r12 = m21, r22 = m22
        const double l00 = sqrt(V00), l10 = V01 / l00, l20 = V02 / l00;
        const double l11 = sqrt(V11 - l10 * l10), l21 = (V12 - l20 * l10) / l11;
        const double l22 = sqrt(V22 - l20 * l20 - l21 * l21);
        const double m00 = 1.0 / l00, m11 = 1.0 / l11, m22 = 1.0 / l22;
        const double m10 = -l10 * m00 * m11, m21 = -l21 * m11 * m22, m20 = -(l20 * m00 + l21 * m10) * m22;
        double* P = PT + (int64_t)lp * PS;
        double* pp = PP + tp * PPS;
        if (g == 0) {
            P[0] = I00; P[1] = I01; P[2] = I02; P[3] = I11; P[4] = I12; P[5] = I22;
            P[6] = I00 * b0 + I01 * b1 + I02 * b2;
            P[7] = I01 * b0 + I11 * b1 + I12 * b2;
            P[8] = I02 * b0 + I12 * b1 + I22 * b2;
            pp[0] = I00; pp[1] = I01; pp[2] = I02; pp[3] = I11; pp[4] = I12; pp[5] = I22;
            pp[6] = m00; pp[7] = m10; pp[8] = m20; pp[9] = m11; pp[10] = m21; pp[11] = m22;
            pp[12] = m00 * b0;
            pp[13] = m10 * b0 + m11 * b1;
            pp[14] = m20 * b0 + m21 * b1 + m22 * b2;
        }
#pragma unroll
        for (int u = 0; u < CWQ; ++u) {
            const int q = qb + u;
            if (q < CW) {
                const double w0_ = W1[u][0], w1_ = W1[u][1], w2_ = W1[u][2];
                P[12 + 3 * CW + 3 * q] = w0_ * I00 + w1_ * I01 + w2_ * I02;
                P[13 + 3 * CW + 3 * q] = w0_ * I01 + w1_ * I11 + w2_ * I12;
                P[14 + 3 * CW + 3 * q] = w0_ * I02 + w1_ * I12 + w2_ * I22;
                pp[15 + 3 * q] = w0_ * m00;
                pp[16 + 3 * q] = w0_ * m10 + w1_ * m11;
                pp[17 + 3 * q] = w0_ * m20 + w1_ * m21 + w2_ * m22;
            }
        }
    }
    __syncthreads();
    stamp(2);
    // (C)
    const bool urow = A[plan.ck_tm + c] != 0;  // U-row chunk: its pair terms are reduced by k_red_blocks
    if (active) {
        double* u = Us + t * US;
        if (p >= 0) {
            const double* pp = PP + (p - p0) * PPS;
            const double r00 = pp[6], r01 = pp[7], r02 = pp[8], r11 = pp[9], r12 = pp[10], r22 = pp[11];
            {  // the observation's record (OBS_REC): the back-substitution forms T from it and Vinv
                double2* r = reinterpret_cast<double2*>(WT + (int64_t)o * OBS_REC);
                r[0] = double2{jr[0][6 + CW], jr[0][7 + CW]};
                r[1] = double2{jr[0][8 + CW], jr[1][6 + CW]};
                r[2] = double2{jr[1][7 + CW], jr[1][8 + CW]};
                r[3] = double2{jr[0][3], jr[0][4]};
                r[4] = double2{jr[0][5], jr[1][3]};
                r[5] = double2{jr[1][4], jr[1][5]};
            }
#pragma unroll
            for (int a = 0; a < 6; ++a) {
                const double e0 = px * jr[0][a], e1 = py * jr[1][a];
                const double v0 = e0 * jr[0][6 + CW + 0] + e1 * jr[1][6 + CW + 0];
                const double v1 = e0 * jr[0][6 + CW + 1] + e1 * jr[1][6 + CW + 1];
                const double v2 = e0 * jr[0][6 + CW + 2] + e1 * jr[1][6 + CW + 2];
                u[3 * a] = v0 * r00;
                u[3 * a + 1] = v0 * r01 + v1 * r11;
                u[3 * a + 2] = v0 * r02 + v1 * r12 + v2 * r22;
            }
            if (urow) {
                double2* ug = reinterpret_cast<double2*>(Ug + (int64_t)o * 18);
#pragma unroll
                for (int m = 0; m < 9; ++m) ug[m] = double2{u[2 * m], u[2 * m + 1]};
            }
        } else {
#pragma unroll
            for (int m = 0; m < 18; ++m) u[m] = 0.0;
        }
        const double sx = sqrt(px), sy = sqrt(py);
        double* E = QE + t * ES;  // own row: the point phase has finished reading it
#pragma unroll
        for (int a = 0; a < 6; ++a) { E[a] = sx * jr[0][a]; E[6 + a] = sy * jr[1][a]; }
        E[12] = sx * w0;
        E[13] = sy * w1;
#pragma unroll
        for (int q = 0; q < CW; ++q) { E[14 + q] = sx * jr[0][6 + q]; E[14 + CW + q] = sy * jr[1][6 + q]; }
    }
    __syncthreads();
    stamp(3);
    // (D) camera entries first (the longest items), then image keys, then pair keys (the plan lists
    // were staged in LDS before (A)).
    const int nob = o1 - o0, np = p1 - p0;
    // camera entries: parts 0 .. CAM_SPLIT - 2 sum observation sub-ranges, part CAM_SPLIT - 1 the points'
    // Schur terms (so no thread runs both loops)
    if (t < CAM_SPLIT * NCAM) {
        constexpr int NPK = CW * (CW + 1) / 2;
        const int it = t % NCAM, part = t / NCAM;
        int c1 = 0, c2 = -1;
        if (it < NPK) {
            int rem = it;
            while (rem > c1) { rem -= c1 + 1; ++c1; }
            c2 = rem;
        } else {
            c1 = it - NPK;
        }
        constexpr int NO = CAM_SPLIT - 1;
        const int l0 = part < NO ? nob * part / NO : 0, l1 = part < NO ? nob * (part + 1) / NO : 0;
        double s = 0.0;
#pragma unroll 4
        for (int l = l0; l < l1; ++l) {
            const double* r = QE + l * ES;
            const double s0 = (c2 >= 0) ? r[14 + c2] : r[12];
            const double s1 = (c2 >= 0) ? r[14 + CW + c2] : r[13];
            s += r[14 + c1] * s0 + r[14 + CW + c1] * s1;
        }
        if (part == CAM_SPLIT - 1)  // the points' Schur terms
#pragma unroll 4
            for (int q = 0; q < np; ++q) {
                const double* pp = PP + q * PPS;
                const double* u1 = pp + 15 + 3 * c1;
                const double* u2 = (c2 >= 0) ? pp + 15 + 3 * c2 : pp + 12;
                s -= u1[0] * u2[0] + u1[1] * u2[1] + u1[2] * u2[2];
            }
        camp[part * NCAM + it] = s;
    }
    __syncthreads();
    if (t < NCAM) {
        double s = 0.0;
        for (int part = 0; part < CAM_SPLIT; ++part) s += camp[part * NCAM + t];
        cpart[(int64_t)c * NCAM + t] = s;
    }
    stamp(4);
    // image keys: one 8-lane group per (key, part) -- part 0 the lower diagonal block and RHS (27
    // values), parts 1 and 2 the two halves of the image-camera block -- each lane accumulating
    // every 8th observation of the key from its own LDS rows (no broadcast reads), then a fixed
    // xor-butterfly over the 8 lanes; part-major unit order keeps the rows of a wave on one path
    constexpr int HALF = (CW + 1) / 2;
    constexpr int IV = 27 > 6 * HALF ? 27 : 6 * HALF;  // values per unit
    // lanes per unit, per launch (IKL, Ctx::ik_lanes): 8, or 4 when the scene's image keys hold <= 2
    // observations on average (a dense network's chunks: ~1.1 -- on eight lanes seven would mostly idle and
    // the units take twice the rounds: convergent k_lin_reduce 331.9 -> 313.4 us).  A grid's keys (~7
    // observations) on 4 lanes measured slower (image keys 6.54 -> 8.82 us per chunk); both lane counts in
    // one kernel slowed the eight-lane path (config 4 206.1 -> 210.2 us), hence two instantiations
    constexpr int GL = IKL;
    static_assert(GL == 8 || GL == 4, "image-key lanes per unit");
    constexpr int NV = (IV + GL - 1) / GL * GL, M = NV / GL;  // padded to the GL-lane reduce-scatter
    {
        const int nk = ki1 - ki0, nu = 3 * nk, g8 = t & (GL - 1);
        for (int ub = t / GL; ub < nu; ub += LR_THREADS / GL) {
            const int part = ub / nk, K = ki0 + ub % nk;
            const int x0 = s_iko[K - ki0], x1 = s_iko[K - ki0 + 1];
            double v[NV];
#pragma unroll
            for (int q = 0; q < NV; ++q) v[q] = 0.0;
            for (int x = x0 + g8; x < x1; x += GL) {
                const int l = s_ikobs[x];
                const double* E = QE + l * ES;
                const double* u = Us + l * US;
                const int pq = pl[l];
                double uu[18];
#pragma unroll
                for (int q = 0; q < 18; ++q) uu[q] = u[q];
                if (part == 0) {
                    double e[14];
#pragma unroll
                    for (int q = 0; q < 14; ++q) e[q] = E[q];
#pragma unroll
                    for (int aa = 0; aa < 6; ++aa)
#pragma unroll
                        for (int bb = 0; bb <= aa; ++bb)
                            v[aa * (aa + 1) / 2 + bb] += e[aa] * e[bb] + e[6 + aa] * e[6 + bb] -
                                                         (uu[3 * aa] * uu[3 * bb] + uu[3 * aa + 1] * uu[3 * bb + 1] +
                                                          uu[3 * aa + 2] * uu[3 * bb + 2]);
                    double rb0 = 0.0, rb1 = 0.0, rb2 = 0.0;
                    if (pq >= 0) { const double* pp = PP + pq * PPS; rb0 = pp[12]; rb1 = pp[13]; rb2 = pp[14]; }
#pragma unroll
                    for (int aa = 0; aa < 6; ++aa)
                        v[21 + aa] += e[aa] * e[12] + e[6 + aa] * e[13] - (uu[3 * aa] * rb0 + uu[3 * aa + 1] * rb1 + uu[3 * aa + 2] * rb2);
                } else {
                    const int q0 = (part - 1) * HALF;
                    double e[12];
#pragma unroll
                    for (int q = 0; q < 12; ++q) e[q] = E[q];
#pragma unroll
                    for (int q = 0; q < HALF; ++q) {
                        if (q0 + q >= CW) continue;
                        const double fx = E[14 + q0 + q], fy = E[14 + CW + q0 + q];
                        double c0 = 0.0, c1 = 0.0, c2 = 0.0;
                        if (pq >= 0) {
                            const double* pp = PP + pq * PPS + 15 + 3 * (q0 + q);
                            c0 = pp[0]; c1 = pp[1]; c2 = pp[2];
                        }
#pragma unroll
                        for (int aa = 0; aa < 6; ++aa)
                            v[6 * q + aa] += fx * e[aa] + fy * e[6 + aa] - (uu[3 * aa] * c0 + uu[3 * aa + 1] * c1 + uu[3 * aa + 2] * c2);
                    }
                }
            }
            // reduce-scatter over the group's GL lanes in log2(GL) DPP exchange steps (partners 7 - i
            // (GL = 8 only), i ^ 2, i ^ 1): each step a lane keeps half of its values, adds the partner's
            // copy of that half and hands over the other half, so lane g8 ends with the M fully summed
            // values q = 4M b2 + 2M b1 + M b0 + j (b = bits of g8), in a fixed order
            double h4[4 * M], h2[2 * M], h1[M];
            const bool bA = (g8 & 4) != 0, bB = (g8 & 2) != 0, bC = (g8 & 1) != 0;
            if constexpr (GL == 8) {
#pragma unroll
                for (int j = 0; j < 4 * M; ++j) {
                    const double keep = bA ? v[4 * M + j] : v[j], give = bA ? v[j] : v[4 * M + j];
                    h4[j] = keep + dpp_d<0x141>(give);  // row_half_mirror
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4 * M; ++j) h4[j] = v[j];
            }
#pragma unroll
            for (int j = 0; j < 2 * M; ++j) {
                const double keep = bB ? h4[2 * M + j] : h4[j], give = bB ? h4[j] : h4[2 * M + j];
                h2[j] = keep + dpp_d<0x4E>(give);  // quad_perm [2,3,0,1]
            }
#pragma unroll
            for (int j = 0; j < M; ++j) {
                const double keep = bC ? h2[M + j] : h2[j], give = bC ? h2[j] : h2[M + j];
                h1[j] = keep + dpp_d<0xB1>(give);  // quad_perm [1,0,3,2]
            }
            const int q0 = (GL == 8 && bA ? 4 * M : 0) + (bB ? 2 * M : 0) + (bC ? M : 0);
            // part 0: the 27 values at out[0 ..]; parts 1, 2: the 6 nq values of cameras columns
            // (part - 1) HALF .. at out[27 + 6 (part - 1) HALF ..]
            const int nval = part == 0 ? 27 : 6 * min(HALF, CW - (part - 1) * HALF);
            double* out = ipart + (int64_t)s_iks[K - ki0] * NIMG + (part == 0 ? 0 : 27 + 6 * (part - 1) * HALF);
#pragma unroll
            for (int j = 0; j < M; ++j)
                if (q0 + j < nval) out[q0 + j] = h1[j];
        }
    }
    if (tprof) {  // FBA_LR_PROFILE: image keys and pair keys timed apart (a barrier the real run does not have)
        __syncthreads();
        stamp(6);
    }
    // pair keys: one thread per (key, rows 2h, 2h+1) of the pair block, outputs in registers; the term
    // lists from LDS (staged above) or, for a chunk of one very large point, from HBM
    auto pair_items = [&](const int* __restrict__ pk, const int* __restrict__ tr, int toff_) {
        const int n3 = 3 * (kp1 - kp0);
        for (int it = t; it < n3; it += LR_THREADS) {
            const int K = kp0 + it / 3, a0 = 2 * (it % 3);
            double acc[12];
#pragma unroll
            for (int q = 0; q < 12; ++q) acc[q] = 0.0;
            for (int q = pk[K - kp0] - toff_; q < pk[K - kp0 + 1] - toff_; ++q) {
                const int tm = tr[q];
                const double* ui = Us + (tm & 0xffff) * US + 3 * a0;
                const double* uj = Us + (tm >> 16) * US;
                double vi[6], vj[18];
#pragma unroll
                for (int m = 0; m < 6; ++m) vi[m] = ui[m];
#pragma unroll
                for (int m = 0; m < 18; ++m) vj[m] = uj[m];
#pragma unroll
                for (int h = 0; h < 2; ++h)
#pragma unroll
                    for (int b = 0; b < 6; ++b)
                        acc[6 * h + b] += vi[3 * h] * vj[3 * b] + vi[3 * h + 1] * vj[3 * b + 1] + vi[3 * h + 2] * vj[3 * b + 2];
            }
            // (the key's row: pair-major slot, staged with the plan lists; 16-B aligned, as 6 double2 stores)
            double2* out = reinterpret_cast<double2*>(
                ppart + (int64_t)(stage_terms ? s_pks[K - kp0] : A[plan.pk_slot + K]) * 36 + 6 * a0);
#pragma unroll
            for (int q = 0; q < 6; ++q) out[q] = double2{-acc[2 * q], -acc[2 * q + 1]};
        }
    };
    if (stage_terms) pair_items(s_pkt, s_term, 0);
    else pair_items(A + plan.pk_t + kp0, A + plan.pk_term + tb0, tb0);
    __syncthreads();
    stamp(5);
}

// k_red_pairs: S(e1, e2) = the sum of the pair's partials in chunk order; seven pairs per wave, 9 lanes
// each holding a 2 x 2 sub-block (rows er, er + 1, columns ec, ec + 1; 16-B loads and stores) of the pair's
// 6 x 6 block
constexpr int RP_PER_WAVE = 7, RP_PER_WG = 4 * RP_PER_WAVE;
__device__ __forceinline__ void red_pairs_body(int blk, const double* __restrict__ ppart, const double* __restrict__ Ug,
                                               const int32_t* __restrict__ A, const AccPlan& plan, double* __restrict__ S,
                                               int64_t ld, int64_t n_pairs) {
    const int lane = threadIdx.x & 63, sub = lane / 9, l = lane - 9 * sub;
    const int64_t pr = ((int64_t)blk * 4 + (threadIdx.x >> 6)) * RP_PER_WAVE + sub;
    if (sub >= RP_PER_WAVE || pr >= n_pairs) return;
    const int er = 2 * (l / 3), ec = 2 * (l % 3);
    // the partials in chunk order, one contiguous range (pair-major slots), 4 x 2 loads in flight
    // (fixed association per entry: ((s + p0) + p1) + ...)
    const int q0 = A[plan.rp_start + pr], q1 = A[plan.rp_start + pr + 1];
    const int t0 = A[plan.tp_start + pr], t1 = A[plan.tp_start + pr + 1];
    const int64_t e1 = A[plan.rp_e + 2 * pr], e2 = A[plan.rp_e + 2 * pr + 1];
    const double2* pp = reinterpret_cast<const double2*>(ppart) + (6 * er + ec) / 2;  // row er; row er + 1 at + 3
    double2 s0 = {0.0, 0.0}, s1 = {0.0, 0.0};
    auto add = [&](double2& a, const double2 b) { a.x += b.x; a.y += b.y; };
    int q = q0;
    while (q + 4 <= q1) {
        double2 p[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) { p[j][0] = pp[(int64_t)(q + j) * 18]; p[j][1] = pp[(int64_t)(q + j) * 18 + 3]; }
#pragma unroll
        for (int j = 0; j < 4; ++j) { add(s0, p[j][0]); add(s1, p[j][1]); }
        q += 4;
    }
    for (; q < q1; ++q) {
        add(s0, pp[(int64_t)q * 18]);
        add(s1, pp[(int64_t)q * 18 + 3]);
    }
    // then the U-row terms (AccPlan::ck_tm chunks), in chunk order, TB in flight:
    // S(e1, e2)[r][c] -= U_a[r] . U_b[c], U rows of 6 x 3 (row r at 3 r: rows er, er + 1 of U_a and ec,
    // ec + 1 of U_b as three 16-B loads each)
    constexpr int TB = 1;
    int oa[TB], ob[TB];  // the batch's observations, loaded one batch ahead (the next batch's indices are
                         // in flight with this batch's U rows): convergent k_red_blocks 362.6 -> 337.0 us
#pragma unroll
    for (int u = 0; u < TB; ++u) {
        oa[u] = t0 + u < t1 ? A[plan.tp_ab + 2 * (t0 + u)] : 0;
        ob[u] = t0 + u < t1 ? A[plan.tp_ab + 2 * (t0 + u) + 1] : 0;
    }
    for (int t = t0; t < t1; t += TB) {
        const int nt = min(TB, t1 - t);
        double ua[TB][6], ub[TB][6];
#pragma unroll
        for (int u = 0; u < TB; ++u)
            if (u < nt) {
                const double2* a = reinterpret_cast<const double2*>(Ug + (int64_t)oa[u] * 18 + 3 * er);
                const double2* b = reinterpret_cast<const double2*>(Ug + (int64_t)ob[u] * 18 + 3 * ec);
#pragma unroll
                for (int m = 0; m < 3; ++m) {
                    const double2 va = a[m], vb = b[m];
                    ua[u][2 * m] = va.x; ua[u][2 * m + 1] = va.y;
                    ub[u][2 * m] = vb.x; ub[u][2 * m + 1] = vb.y;
                }
            }
        const int tn = t + TB;
#pragma unroll
        for (int u = 0; u < TB; ++u) {
            oa[u] = tn + u < t1 ? A[plan.tp_ab + 2 * (tn + u)] : 0;
            ob[u] = tn + u < t1 ? A[plan.tp_ab + 2 * (tn + u) + 1] : 0;
        }
#pragma unroll
        for (int u = 0; u < TB; ++u)
            if (u < nt) {
                const double* x = ua[u];
                const double* y = ub[u];
                s0.x -= x[0] * y[0] + x[1] * y[1] + x[2] * y[2];
                s0.y -= x[0] * y[3] + x[1] * y[4] + x[2] * y[5];
                s1.x -= x[3] * y[0] + x[4] * y[1] + x[5] * y[2];
                s1.y -= x[3] * y[3] + x[4] * y[4] + x[5] * y[5];
            }
    }
    *reinterpret_cast<double2*>(S + (6 * e1 + er) * ld + 6 * e2 + ec) = s0;
    *reinterpret_cast<double2*>(S + (6 * e1 + er + 1) * ld + 6 * e2 + ec) = s1;
}

// k_red_images: the diagonal block, RHS and image-camera block of image e from its partials; one image per
// workgroup, the two 128-thread halves summing the first and the second half of its partial rows (a dense
// network's image has ~440 of them: the chain of load round trips is the time), then half 1's sums are
// added to half 0's in LDS -- ((p0 + p1) + ...) + ((pm + pm+1) + ...), a fixed order
template <int NK>
__device__ __forceinline__ void red_images_body(int e, const double* __restrict__ ipart, const int32_t* __restrict__ A,
                                                const AccPlan& plan, double* __restrict__ S, int64_t ld, int64_t n_pad,
                                                int n_img) {
    constexpr int CW = 5 + NK, NIMG = LR<NK>::NIMG;
    __shared__ double half1[128];
    const int q = threadIdx.x & 127, h = threadIdx.x >> 7;
    const int r0 = A[plan.ri_start + e], r1 = A[plan.ri_start + e + 1];  // (uniform per workgroup)
    if (r0 == r1) return;
    const int rm = r0 + (r1 - r0) / 2;
    const int xa = h ? rm : r0, xb = h ? r1 : rm;
    // (8 loads in flight; 32 measured: convergent k_red_blocks 329 -> 323 us, at 64 more VGPRs for the launch)
    const double* ip = ipart + (q < NIMG ? q : 0);
    double s = 0.0;
    int x = xa;
    for (; x + 8 <= xb; x += 8) {
        double p[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) p[j] = ip[(int64_t)(x + j) * NIMG];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += p[j];
    }
    for (; x < xb; ++x) s += ip[(int64_t)x * NIMG];
    if (h) half1[q] = s;
    __syncthreads();
    if (h || q >= NIMG) return;
    s += half1[q];
    if (q < 21) {
        S[(6 * (int64_t)e + c_tri_a[q]) * ld + 6 * e + c_tri_b[q]] = s;
    } else if (q < 27) {
        S[n_pad * ld + 6 * e + (q - 21)] = s;
    } else {
        const int k = A[plan.img_cam + e], a = (q - 27) % 6, b = (q - 27) / 6;
        S[(6 * (int64_t)n_img + (int64_t)k * CW + b) * ld + 6 * e + a] = s;
    }
}

constexpr int BW_SEG = 32;
__device__ __forceinline__ void border_weights_body(int seg, const double* __restrict__ S, const double* __restrict__ G,
                                                    double* __restrict__ scal, double* __restrict__ part, int64_t ld,
                                                    int n_img, int n_loc, int ic, const int8_t* __restrict__ rown);

// camera block (lower) and camera RHS from the chunk partials of the camera, in two fixed-order
// stages: k_red_cam_seg sums CAM_SEG contiguous segments of the camera's chunk list in parallel
// (one workgroup each, 4 loads in flight per thread), k_red_cam adds the segment sums in order
constexpr int CAM_SEG = 64;

template <int NK>
__device__ __forceinline__ void red_cam_seg_body(int sg, int q, int n_cam, const double* __restrict__ cpart,
                                                 const int32_t* __restrict__ A, const AccPlan& plan,
                                                 double* __restrict__ cseg) {
    constexpr int NCAM = LR<NK>::NCAM;
    static_assert(NCAM <= 128, "one thread per camera entry");
    const int k = sg / CAM_SEG, g = sg % CAM_SEG;
    if (q >= NCAM || k >= n_cam) return;
    const int x0 = A[plan.rc_start + k], n = A[plan.rc_start + k + 1] - x0;
    const int y0 = x0 + (int)((int64_t)n * g / CAM_SEG), y1 = x0 + (int)((int64_t)n * (g + 1) / CAM_SEG);
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int x = y0;
    for (; x + 4 <= y1; x += 4) {
        s0 += cpart[(int64_t)A[plan.rc_list + x] * NCAM + q];
        s1 += cpart[(int64_t)A[plan.rc_list + x + 1] * NCAM + q];
        s2 += cpart[(int64_t)A[plan.rc_list + x + 2] * NCAM + q];
        s3 += cpart[(int64_t)A[plan.rc_list + x + 3] * NCAM + q];
    }
    for (; x < y1; ++x) s0 += cpart[(int64_t)A[plan.rc_list + x] * NCAM + q];
    cseg[((int64_t)k * CAM_SEG + g) * NCAM + q] = (s0 + s1) + (s2 + s3);
}

// the three independent reductions in one launch: workgroups [0, npb) the image pairs (RP_PER_WG per
// workgroup), then one image per workgroup, then two camera segments per workgroup
template <int NK>
__global__ __launch_bounds__(256) void k_red_blocks(const double* __restrict__ ppart, const double* __restrict__ ipart,
                                                    const double* __restrict__ cpart, const int32_t* __restrict__ A,
                                                    const AccPlan plan, double* __restrict__ S, int64_t ld,
                                                    int64_t n_pairs, int64_t n_pad, int n_img, int n_cam, int npb,
                                                    int nib, double* __restrict__ cseg, const double* __restrict__ Ug) {
    const int b = blockIdx.x;
    if (b < npb) {
        // XCD-aware: workgroup b runs on XCD b % 8 (round-robin dispatch); give each XCD a contiguous range
        // of the pairs, sorted by (e1, e2), so the U rows of an image's observations, gathered by all its
        // pairs (U-row terms), stay in that XCD's L2
        const int q = npb / 8, r = npb % 8, x = b % 8, i = b / 8;
        const int bx = x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
        red_pairs_body(bx, ppart, Ug, A, plan, S, ld, n_pairs);
    } else if (b < npb + nib) {
        red_images_body<NK>(b - npb, ipart, A, plan, S, ld, n_pad, n_img);
    } else {
        red_cam_seg_body<NK>(2 * (b - npb - nib) + (threadIdx.x >> 7), threadIdx.x & 127, n_cam, cpart, A, plan, cseg);
    }
}

// workgroups [0, n_cam): one camera each; [n_cam, n_cam + BW_SEG) when bw: the border weights' segments
// (k_border_weights' work, which needs only the image rows' diagonal: no launch of its own ahead of the
// solve when nothing adds to S between the two, border_weights_in_accumulate)
struct BorderW {
    const double* G;
    double* scal;
    double* part;
    int n_loc, ic;
};

template <int NK>
__global__ __launch_bounds__(256) void k_red_cam(const double* __restrict__ cseg, double* __restrict__ S, int64_t ld,
                                                 int64_t n_pad, int n_img, int n_cam, BorderW bw) {
    constexpr int CW = 5 + NK, NCAM = LR<NK>::NCAM, NPK = CW * (CW + 1) / 2;
    const int k = blockIdx.x, q = threadIdx.x;
    if (k >= n_cam) {
        border_weights_body(k - n_cam, S, bw.G, bw.scal, bw.part, ld, n_img, bw.n_loc, bw.ic, nullptr);
        return;
    }
    if (q >= NCAM) return;
    const double* p = cseg + (int64_t)k * CAM_SEG * NCAM + q;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll 4
    for (int g = 0; g < CAM_SEG; g += 4) {
        s0 += p[g * NCAM];
        s1 += p[(g + 1) * NCAM];
        s2 += p[(g + 2) * NCAM];
        s3 += p[(g + 3) * NCAM];
    }
    const double s = (s0 + s1) + (s2 + s3);
    const int64_t base = 6 * (int64_t)n_img + (int64_t)k * CW;
    if (q < NPK) {
        int c1 = 0, rem = q;
        while (rem > c1) { rem -= c1 + 1; ++c1; }
        S[(base + c1) * ld + base + rem] = s;
    } else {
        S[n_pad * ld + base + (q - NPK)] = s;
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
// k_border_weights: BW_SEG workgroups, each the 14 weight sums over a contiguous range of the 6 n_img
// EOP rows -> part[seg][14]; the consumer (k_border_rhs) adds the segments in order (BW_SEG above)

// rown (subtree split, per row): the weight sums over all images (7..13) take only this rank's images'
// rows -- a wholly-top image's diagonal is complete only after the ranks' sum (k_split_weights adds them)
__device__ __forceinline__ void border_weights_body(int seg, const double* __restrict__ S, const double* __restrict__ G,
                                                    double* __restrict__ scal, double* __restrict__ part, int64_t ld,
                                                    int n_img, int n_loc, int ic, const int8_t* __restrict__ rown) {
    __shared__ double red[4][14];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int64_t n = 6 * (int64_t)n_img;
    const int64_t i0 = n * seg / BW_SEG, i1 = n * (seg + 1) / BW_SEG;
    double a[14];
#pragma unroll
    for (int m = 0; m < 14; ++m) a[m] = 0.0;
    if (ic) {
        for (int64_t i = i0 + tid; i < i1; i += 256) {
            const double sii = S[i * ld + i];
            const double* g = G + (i / 6) * 42 + (i % 6) * 7;
            const bool ok = sii > 0.0, loc = i < 6 * (int64_t)n_loc, all = !rown || rown[i] == 1;
            const double inv = ok ? 1.0 / sii : 0.0;
#pragma unroll
            for (int m = 0; m < 7; ++m) {
                const double v = g[m] * g[m] * inv;
                if (all) a[7 + m] += v;
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
    if (tid < 14) part[seg * 14 + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
    if (seg == 0 && tid == 0) scal[1] = 0.0;  // Cholesky failure flag
}

__global__ __launch_bounds__(256) void k_border_weights(const double* __restrict__ S, const double* __restrict__ G,
                                                        double* __restrict__ scal, double* __restrict__ part, int64_t ld,
                                                        int n_img, int n_loc, int ic, const int8_t* __restrict__ rown) {
    border_weights_body(blockIdx.x, S, G, scal, part, ld, n_img, n_loc, ic, rown);
}

// the 14 weights (W_l: 0..6, D^2: 7..13) from the segment sums, into LDS w[14]; every thread calls it
__device__ __forceinline__ void border_weights_lds(const double* __restrict__ part, double* w) {
    const int t = threadIdx.x;
    if (t < 14) {
        double x[BW_SEG];
#pragma unroll
        for (int g = 0; g < BW_SEG; ++g) x[g] = part[g * 14 + t];
        double v = 0.0;
#pragma unroll
        for (int g = 0; g < BW_SEG; ++g) v += x[g];
        w[t] = v > 0.0 ? 1.0 / v : 1.0;
    }
    __syncthreads();
}

// One launch, two roles by workgroup (both need the 14 weights first):
//   workgroups [0, nbr): row i = blockIdx of the local border, M(i, j) += G_i W_l G_j' for j <= i (lower
//                        part); padding slots have zero G rows and are left alone (their unit diagonal
//                        is written by the other role, so the two never touch the same entry)
//   workgroups [nbr, ..): one thread per row i of S: unit row for fixed parameters and padding, the
//                        border's RHS rows A = G_l W_l^1/2 and B = G D; the hand-off flags and counters
//                        of the factorisation / backward solve zeroed
// rown (subtree split): the B rows unscaled (k_split_weights' scales enter the border combine), and the
// unit diagonal and B entries of a wholly-top image's row written by rank 0 only, of an image of a rank's
// subtree by that rank (the ranks' top blocks are summed)
__global__ __launch_bounds__(256) void k_border_rhs(double* __restrict__ S, const double* __restrict__ G,
                                                    double* __restrict__ scal, const double* __restrict__ part,
                                                    const uint8_t* __restrict__ active, int64_t ld, int64_t n_pad,
                                                    int64_t u_c, int n_img, int n_loc, int ic, int nbr,
                                                    unsigned* __restrict__ sync, int64_t n_sync, double* __restrict__ X,
                                                    const int8_t* __restrict__ rown, int rank) {
    __shared__ double w[14];
    if (ic) border_weights_lds(part, w);
    if ((int)blockIdx.x < nbr) {
        const int64_t i = blockIdx.x;
        const double* gi = G + (i / 6) * 42 + (i % 6) * 7;
        double gw[7];
#pragma unroll
        for (int m = 0; m < 7; ++m) gw[m] = gi[m] * w[m];
        for (int64_t j = threadIdx.x; j <= i; j += 256) {
            const double* gj = G + (j / 6) * 42 + (j % 6) * 7;
            double acc = 0.0;
#pragma unroll
            for (int m = 0; m < 7; ++m) acc += gw[m] * gj[m];
            // an inactive row's diagonal is the unit written by the other role (inner constraints need all
            // six EOPs, so such rows have zero G rows today; the guard keeps the two roles disjoint)
            if (acc != 0.0 && (j != i || active[i])) S[i * ld + j] += acc;
        }
        return;
    }
    const int64_t nthr = ((int64_t)gridDim.x - nbr) * blockDim.x;
    const int64_t i = ((int64_t)blockIdx.x - nbr) * blockDim.x + threadIdx.x;
    for (int64_t q = i; q < n_sync; q += nthr) sync[q] = 0u;
    if (ic && blockIdx.x == nbr && threadIdx.x < 14) scal[8 + (threadIdx.x / 7) * 8 + threadIdx.x % 7] = w[threadIdx.x];
    if (i >= n_pad) return;
    X[i] = __builtin_bit_cast(double, X_SENTINEL);  // k_bwd_flow's solution blocks: not yet published
    // (split: a wholly-top row's once-only entries on rank 0; another rank's rows are never read here)
    const bool once = !rown || rown[i] == 1 || (rown[i] == 2 && rank == 0);
    if (i >= u_c || !active[i]) {
        // fixed parameter or padding: decoupled unit row, zero RHS
        S[i * ld + i] = once ? 1.0 : 0.0;
        S[n_pad * ld + i] = 0.0;
    }
    if (ic) {
        const double* g = G + (i / 6) * 42 + (i % 6) * 7;
        for (int m = 0; m < 7; ++m) {
            S[(n_pad + 1 + m) * ld + i] = (i < 6 * (int64_t)n_loc) ? sqrt(w[m]) * g[m] : 0.0;  // A
            S[(n_pad + 8 + m) * ld + i] = (i < 6 * (int64_t)n_img && once) ? (rown ? g[m] : sqrt(w[7 + m]) * g[m]) : 0.0;  // B
        }
    }
}


// ------------------------------------------------------------------------------------------------
// back-substitution of tie points: dp = -(vb + Vinv sum_o W_o^T d_e(o) + Tc^T d_cam)
// ------------------------------------------------------------------------------------------------
// one workgroup per chunk (<= 256 observations of <= 64 whole tie points): thread per observation
// w_o = W_o' d_e(o) = Jp' P (Je d_e) into LDS (its 96-byte record, OBS_REC, coalesced across the wave),
// then thread per point d_p = -(vb + Vinv sum_o w_o + Tc' d_cam), its observations summed in order
template <int NK>
__global__ __launch_bounds__(256) void k_backsub(const double* __restrict__ WT, const double* __restrict__ PT,
                                                 const int32_t* __restrict__ chunk_obs, const int32_t* __restrict__ chunk_pt,
                                                 const int32_t* __restrict__ lp_start, const int32_t* __restrict__ lp_tie,
                                                 const int32_t* __restrict__ lp_cam, const int32_t* __restrict__ img,
                                                 double* __restrict__ delta, int64_t u_c, int n_img, unsigned eop_mask,
                                                 double px, double py) {
    using LY = Lay<NK>;
    constexpr int CW = LY::CW, PS = LY::PS;
    __shared__ double u[CHUNK_OBS][3];
    const int c = blockIdx.x, t = threadIdx.x;
    const int p0 = chunk_pt[c], p1 = chunk_pt[c + 1];
    if (p1 == p0) return;  // control chunk (uniform)
    const int o0 = chunk_obs[c], o = o0 + t;
    if (o < chunk_obs[c + 1]) {
        const double2* R = reinterpret_cast<const double2*>(WT + (int64_t)o * OBS_REC);
        double2 rv[OBS_REC / 2];
#pragma unroll
        for (int k = 0; k < OBS_REC / 2; ++k) rv[k] = R[k];
        const double* r = reinterpret_cast<const double*>(rv);
        const double* de = delta + 6 * (int64_t)img[o];
        double j0[6], j1[6];
        obs_rec_rows(r, eop_mask, j0, j1);
        double e0 = 0.0, e1 = 0.0;
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            const double e = de[a];
            e0 += j0[a] * e;
            e1 += j1[a] * e;
        }
        e0 *= px;
        e1 *= py;
        u[t][0] = r[0] * e0 + r[3] * e1;
        u[t][1] = r[1] * e0 + r[4] * e1;
        u[t][2] = r[2] * e0 + r[5] * e1;
    }
    __syncthreads();
    const int p = p0 + t;
    if (p < p1) {
        const double* P = PT + (int64_t)p * PS;
        double w0 = 0.0, w1 = 0.0, w2 = 0.0;
        for (int q = lp_start[p] - o0; q < lp_start[p + 1] - o0; ++q) { w0 += u[q][0]; w1 += u[q][1]; w2 += u[q][2]; }
        double d0 = P[6] + (P[0] * w0 + P[1] * w1 + P[2] * w2);
        double d1 = P[7] + (P[1] * w0 + P[3] * w1 + P[4] * w2);
        double d2 = P[8] + (P[2] * w0 + P[4] * w1 + P[5] * w2);
        const double* dk = delta + 6 * (int64_t)n_img + (int64_t)lp_cam[p] * CW;
        const double* Tc = P + 12 + 3 * CW;
#pragma unroll
        for (int k = 0; k < CW; ++k) {
            d0 += Tc[3 * k] * dk[k]; d1 += Tc[3 * k + 1] * dk[k]; d2 += Tc[3 * k + 2] * dk[k];
        }
        double* out = delta + u_c + 3 * (int64_t)lp_tie[p];
        out[0] = -d0; out[1] = -d1; out[2] = -d2;
    }
}

// T = W Vinv of every observation of the regular chunks (the covariance's k_cov_pts reads T rows)
__global__ __launch_bounds__(256) void k_obs_T(const double* __restrict__ WT, const double* __restrict__ PT, int ps,
                                               const int32_t* __restrict__ pt, int64_t n_obs, unsigned eop_mask, double px,
                                               double py, double* __restrict__ T) {
    const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (o >= n_obs) return;
    const int p = pt[o];
    if (p < 0) return;
    obs_rec_T(WT + o * OBS_REC, PT + (int64_t)p * ps, eop_mask, px, py, T + o * 18);
}


// ------------------------------------------------------------------------------------------------
// update: de-scale (main.m:460-482), xhat += delta, partial sumabs (fixed-order block sums)
// ------------------------------------------------------------------------------------------------
// (scal[1] < 0: a hand-off of the factorisation or backward solve timed out, fba_chol.hip -- delta is not
// a solution, xhat stays as it was and the host reports FBA_ERR_HIP)
// a workgroup's 256 values summed in a fixed order (xor butterfly per wave, then the four wave sums in
// order); every thread calls it, thread 0 returns the sum
__device__ __forceinline__ double block_sum256(double a, double* red) {
#pragma unroll
    for (int w = 32; w > 0; w >>= 1) a += __shfl_xor(a, w, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void k_update(double* __restrict__ xfull, double* __restrict__ delta,
                                                const double* __restrict__ cam_tab, const uint8_t* __restrict__ counted,
                                                double* __restrict__ part, int64_t u_full, int n_img, int n_cam, int nk,
                                                int cw, int cam_stride, const double* __restrict__ scal) {
    __shared__ double red[4];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool apply = !(scal[1] < 0.0);
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
        if (apply) xfull[i] += d;
        if (counted[i]) a = fabs(d);
        if (!isfinite(d)) a = __builtin_nan("");
    }
    const double s = block_sum256(a, red);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// deltasum into scal[2]; scal[0..3] also to the host-mapped scratch `host` (read after the stream sync)
__global__ void k_sum_parts(const double* __restrict__ part, int n, double* __restrict__ scal, double* __restrict__ host) {
    __shared__ double red[4];
    double a = 0.0;
    // thread t sums parts t, t + 256, ... in order (coalesced, 16 loads in flight), then block_sum256's
    // fixed order
    for (int i0 = threadIdx.x; i0 < n; i0 += 16 * 256) {
        double x[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) x[k] = i0 + 256 * k < n ? part[i0 + 256 * k] : 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (i0 + 256 * k < n) a += x[k];
    }
    const double sum = block_sum256(a, red);
    if (threadIdx.x == 0) {
        scal[2] = sum;
        if (host) {
            host[0] = scal[0];
            host[1] = scal[1];
            host[2] = sum;
            host[3] = scal[3];
            // the solve's sequence number last, behind the values (the host polls it instead of waiting
            // for the stream: this kernel ends every solve)
            __threadfence_system();
            const double seq = scal[5] + 1.0;
            scal[5] = seq;
            host[4] = seq;
        }
    }
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

// BuildRSD.m:29-40 for a given v (PHO order): one thread per local observation, xp / yp of its camera
// from `xpyp` (BuildRSD.m:12-26 gathered on the host), rows written at the observation's PHO row
__global__ __launch_bounds__(256) void k_build_rsd(const double* __restrict__ xy, const int32_t* __restrict__ cam,
                                                   const int64_t* __restrict__ obs_pho, const double* __restrict__ v,
                                                   const double* __restrict__ xpyp, double* __restrict__ rsd,
                                                   int64_t n_obs) {
    const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_obs) return;
    const int64_t i = obs_pho[o];
    const double vx = v[2 * i], vy = v[2 * i + 1];
    const double xb = xy[2 * o] - xpyp[2 * cam[o]], yb = xy[2 * o + 1] - xpyp[2 * cam[o] + 1];
    const double theta = atan2(yb, xb), phi = atan2(vy, vx);
    const double vd = sqrt(vx * vx + vy * vy);
    double* r = rsd + 5 * i;
    r[0] = sqrt(xb * xb + yb * yb);
    r[1] = vx;
    r[2] = vy;
    r[3] = vd * cos(theta - phi);
    r[4] = vd * sin(theta - phi);
}

int launch_build_rsd(Ctx& c, const double* d_v, const double* d_xpyp, double* d_rsd) {
    if (c.n_obs == 0) return FBA_OK;
    k_build_rsd<<<(unsigned)((c.n_obs + 255) / 256), 256, 0, c.stream>>>(c.d_xy, c.d_cam, c.d_obs_pho, d_v, d_xpyp, d_rsd,
                                                                      c.n_obs);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
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

// T = W Vinv of the tie observations (the first n_obs_tie) into T [n_obs_tie][18], for k_cov_pts
int launch_obs_T(Ctx& c, double* T) {
    const int64_t n = c.n_obs_tie;
    if (n <= 0) return FBA_OK;
    k_obs_T<<<(unsigned)((n + 255) / 256), 256, 0, c.stream>>>(c.d_WT, c.d_pt_tab, c.pt_comp, c.d_pt, n, eop_mask(c.set),
                                                               px_of(c), py_of(c), T);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_params(Ctx& c, const double* x, double* copy_to) {
    const int64_t nb = (c.L.n_img + PARAMS_WG - 1) / PARAMS_WG + c.L.n_cam;
    const int64_t blocks = copy_to ? nb + std::min<int64_t>(2048, (c.L.u_full + 4 * PARAMS_WG - 1) / (4 * PARAMS_WG)) : nb;
    k_params<<<(unsigned)blocks, PARAMS_WG, 0, c.stream>>>(x ? x : c.d_xfull, c.d_caminfo, c.d_img_tab, c.d_cam_tab, c.d_G,
                                                    c.d_active, c.L.n_img, c.L.n_cam, c.L.nk, c.L.cw, c.cam_tab_stride,
                                                    c.set.inner_constraints, copy_to, c.L.u_full);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

// Jacobian rows of every observation (+ the regular points' tables): residuals, dense AwG, covariance
int launch_linearize(Ctx& c, const double* x) { return launch_linearize_range(c, x, 0, c.n_chunks); }

int launch_linearize_range(Ctx& c, const double* x, int64_t c0, int64_t c1) {
    if (c1 <= c0) return FBA_OK;
    const unsigned em = eop_mask(c.set), cm = cam_mask(c.set, c.L.nk);
#define LIN(NKV)                                                                                               \
    k_lin_point<NKV><<<(unsigned)(c1 - c0), 256, 0, c.stream>>>(                                               \
        c.d_xy, c.d_img, c.d_cam, c.d_pt, c.d_lp_tie, c.d_ctl, x ? x : c.d_xfull, c.d_img_tab, c.d_cam_tab,     \
        c.d_chunk_obs, c.d_chunk_pt, c.d_lp_start, c.d_J, c.d_WT, c.d_pt_tab, c.L.u_c, c.set.type,              \
        c.cam_tab_stride, em, cm, px_of(c), py_of(c), (int)c0)
    FBA_NK_DISPATCH(c.L.nk, LIN);
#undef LIN
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

// zero the blocks of the factor's pattern (Sched::zero); 8 workgroups of 16 rows per 128x128 block
__global__ __launch_bounds__(256) void k_zero_blocks(double* __restrict__ S, int64_t ld, const int32_t* __restrict__ blk) {
    const int b = blockIdx.x >> 3;
    const int64_t r0 = (int64_t)blk[2 * b] * NB + (blockIdx.x & 7) * 16, c0 = (int64_t)blk[2 * b + 1] * NB;
    const double2 z = {0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = threadIdx.x + 256 * q, r = i >> 6, c = (i & 63) * 2;
        *reinterpret_cast<double2*>(S + (r0 + r) * ld + c0 + c) = z;
    }
}

// the border weights read the image rows' diagonal of S: final at the end of the accumulation when no
// general tie points (launch_gen_reduce) and no other rank (launch_pack / the split) add to S after it
bool border_weights_in_accumulate(const Ctx& c) {
    return c.n_chunks_lr > 0 && c.gen.n_gp == 0 && c.opt.world <= 1 && !c.sched.split;
}

int launch_accumulate(Ctx& c, bool zeroed) {
    const Layout& L = c.L;
    // the pattern is zeroed by tail workgroups of k_lin_reduce (it does not touch S), unless done already
    const int64_t nlr = c.n_chunks_lr;
    const int ztail = (zeroed || nlr == 0) ? 0 : c.sched.nzero;
    if (c.sched.nzero > 0 && !zeroed && nlr == 0)
        k_zero_blocks<<<(unsigned)(8 * c.sched.nzero), 256, 0, c.stream>>>(c.d_S, L.ld, c.d_sched + c.sched.zero);
    if (nlr == 0 && c.gen.n_gp == 0) return FBA_OK;
    const unsigned em = eop_mask(c.set), cm = cam_mask(c.set, c.L.nk);
    const double px = px_of(c), py = py_of(c);
#define LR_ARGS                                                                                                   \
    c.d_xy, c.d_img, c.d_cam, c.d_pt, c.d_lp_tie, c.d_ctl, c.d_xfull, c.d_img_tab, c.d_cam_tab, c.d_chunk_obs,    \
        c.d_chunk_pt, c.d_lp_start, c.d_acc, c.acc, c.d_WT, c.d_pt_tab, c.d_ppart, c.d_ipart, c.d_cpart, c.L.u_c, \
        c.set.type, c.cam_tab_stride, em, cm, px, py, c.d_lrprof, (int)nlr, c.d_S, L.ld, c.d_sched + c.sched.zero, \
        c.d_xoff, c.d_U
#define ACC(NKV)                                                                                                  \
    if (nlr > 0 && c.ik_lanes == 4)                                                                               \
        k_lin_reduce<NKV, 4><<<(unsigned)(nlr + ztail), LR_THREADS, LR<NKV>::LDS, c.stream>>>(LR_ARGS);           \
    else if (nlr > 0)                                                                                             \
        k_lin_reduce<NKV, 8><<<(unsigned)(nlr + ztail), LR_THREADS, LR<NKV>::LDS, c.stream>>>(LR_ARGS);           \
    {                                                                                                             \
        const int npb = (int)((c.n_pairs + RP_PER_WG - 1) / RP_PER_WG), nib = L.n_img, ncb = (L.n_cam * CAM_SEG + 1) / 2;   \
        k_red_blocks<NKV><<<(unsigned)(npb + nib + ncb), 256, 0, c.stream>>>(                                     \
            c.d_ppart, c.d_ipart, c.d_cpart, c.d_acc, c.acc, c.d_S, L.ld, c.n_pairs, L.n_pad, L.n_img, L.n_cam, npb, \
            nib, c.d_cseg, c.d_U);                                                                                \
    }                                                                                                             \
    k_red_cam<NKV><<<(unsigned)(L.n_cam + (bwa ? BW_SEG : 0)), 256, 0, c.stream>>>(c.d_cseg, c.d_S, L.ld, L.n_pad,   \
                                                                               L.n_img, L.n_cam, bw)
    const bool bwa = border_weights_in_accumulate(c);
    const BorderW bw{c.d_G, c.d_scal, c.d_bscr, c.n_loc, c.set.inner_constraints};
    FBA_NK_DISPATCH(L.nk, ACC);
#undef ACC
#undef LR_ARGS
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int acc_setup(Ctx& c) {
#define SET(NKV)                                                                                                     \
    FBA_HIP(hipFuncSetAttribute((const void*)k_lin_reduce<NKV, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                (int)LR<NKV>::LDS));                                                                  \
    FBA_HIP(hipFuncSetAttribute((const void*)k_lin_reduce<NKV, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                (int)LR<NKV>::LDS))
    FBA_NK_DISPATCH(c.L.nk, SET);
#undef SET
    return FBA_OK;
}

int launch_border(Ctx& c) {
    const Layout& L = c.L;
    const int ic = c.set.inner_constraints;
    const int8_t* rown = c.sched.split ? c.d_rown : nullptr;
    if (!border_weights_in_accumulate(c)) {
        k_border_weights<<<BW_SEG, 256, 0, c.stream>>>(c.d_S, c.d_G, c.d_scal, c.d_bscr, L.ld, L.n_img, c.n_loc, ic, rown);
        FBA_HIP(hipGetLastError());
    }
    const int nbr = (ic && c.n_loc > 0) ? 6 * c.n_loc : 0;
    k_border_rhs<<<(unsigned)(nbr + (L.n_pad + 255) / 256), 256, 0, c.stream>>>(
        c.d_S, c.d_G, c.d_scal, c.d_bscr, c.d_active, L.ld, L.n_pad, L.u_c, L.n_img, c.n_loc, ic, nbr, c.d_flags,
        c.n_sync, c.d_X, rown, c.opt.rank);
    FBA_HIP(hipGetLastError());
    return FBA_OK;
}

int launch_backsub_update(Ctx& c) {
    const Layout& L = c.L;
    int rc;
    if ((rc = launch_gen_backsub(c))) return rc;
    if (c.n_lp > 0) {
#define BS(NKV)                                                                                                    \
    k_backsub<NKV><<<(unsigned)c.n_chunks_lr, 256, 0, c.stream>>>(c.d_WT, c.d_pt_tab, c.d_chunk_obs, c.d_chunk_pt,    \
                                                              c.d_lp_start, c.d_lp_tie, c.d_lp_cam, c.d_img, c.d_delta, \
                                                              L.u_c, L.n_img, eop_mask(c.set), px_of(c), py_of(c))
        FBA_NK_DISPATCH(L.nk, BS);
#undef BS
        FBA_HIP(hipGetLastError());
    }
    const int nblk = (int)((L.u_full + 255) / 256);
    // (forming deltasum in k_update's last-arriving workgroup measured slower: 612 agent-scope atomics)
    k_update<<<nblk, 256, 0, c.stream>>>(c.d_xfull, c.d_delta, c.d_cam_tab, c.d_counted, c.d_part, L.u_full,
                                         L.n_img, L.n_cam, L.nk, L.cw, c.cam_tab_stride, c.d_scal);
    FBA_HIP(hipGetLastError());
    k_sum_parts<<<1, 256, 0, c.stream>>>(c.d_part, nblk, c.d_scal, c.d_hpinned);
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

// Subtree split: the reduce buffer (fba_reduce_buffer) is
//   [top blocks: 128 x 128 each, row-major, an RHS block row's its nrhs rows only]
//   [the accumulated diagonal of the top rows carrying image unknowns, packed before the subtree flow]
//   [Gram partials (16 x 16) of every non-top block column: this rank's own, zeros for the others']
//   [this rank's 7 inner-constraint weight sums over its subtree rows (k_border_weights' segments)]
//   [1: this rank's flow A aborted (a hand-off timed out, scal[1] < 0): its top-block contributions are
//    incomplete; after the sum every rank sees it, raises the abort ahead of flow B and fails the step]
//   [1: this rank's flow A met a non-positive pivot (scal[1] = row + 1 > 0): after the sum every rank reports
//    it, so the ranks agree that the step failed]
// dir 0: S (+ gblk, weight segments) -> buffer; dir 1: buffer -> S top blocks, gblk.  (The diagonal part
// is written by k_pack_topdiag ahead of the subtree flow.)
__global__ __launch_bounds__(256) void k_pack_split(double* __restrict__ S, int64_t ld, double* __restrict__ red,
                                                    const int32_t* __restrict__ tb, int ntb, int64_t n_pad, int nrhs,
                                                    double* __restrict__ gblk, const int8_t* __restrict__ bown, int nb,
                                                    int64_t red_gblk, int64_t red_w, const double* __restrict__ wseg,
                                                    double* __restrict__ scal, int dir) {
    const int q = blockIdx.x;
    if (q < ntb) {  // one top block per workgroup
        const int64_t a = tb[2 * q], b = tb[2 * q + 1];
        const int rows = a * 128 == n_pad ? nrhs : 128;
        int64_t off = 0;  // blocks before q: 128 rows each except RHS blocks
        for (int x = 0; x < q; ++x) off += (int64_t)(tb[2 * x] * 128 == n_pad ? nrhs : 128) * 128;
        double2* R = reinterpret_cast<double2*>(red + off);
        for (int e = threadIdx.x; e < rows * 64; e += 256) {
            const int r = e >> 6, c2 = (e & 63) * 2;
            double2* Sp = reinterpret_cast<double2*>(S + (a * 128 + r) * ld + b * 128 + c2);
            if (dir == 0) R[e] = *Sp;
            else *Sp = R[e];
        }
        return;
    }
    if (q == ntb) {  // the Gram partials of the non-top columns, and the weight sums
        int g = 0;
        for (int k = 0; k < nb; ++k) {
            if (bown[k] == 2) continue;
            for (int e = threadIdx.x; e < 256; e += 256) {
                if (dir == 0) red[red_gblk + 256 * (int64_t)g + e] = bown[k] == 1 ? gblk[256 * (int64_t)k + e] : 0.0;
                else gblk[256 * (int64_t)k + e] = red[red_gblk + 256 * (int64_t)g + e];
            }
            ++g;
        }
        if (dir == 0 && threadIdx.x < 7) {
            double v = 0.0;
            for (int sg = 0; sg < 32; ++sg) v += wseg[sg * 14 + 7 + threadIdx.x];  // (BW_SEG segments)
            red[red_w + threadIdx.x] = v;
        }
        if (threadIdx.x == 7) {
            // (flow A has finished: k_pack_split follows it on the stream, so scal[1] is final here)
            const double f = scal[1];
            if (dir == 0) {
                red[red_w + 7] = f < 0.0 ? 1.0 : 0.0;  // a hand-off timed out
                red[red_w + 8] = f > 0.0 ? f : 0.0;    // a non-positive pivot at row f - 1 of this rank's subtree
            } else if (red[red_w + 7] != 0.0) {
                scal[1] = -1.0;  // some rank's flow A aborted: skip flow B, k_update
            } else if (red[red_w + 8] != 0.0 && f == 0.0) {
                // some rank's flow A hit a non-positive pivot: every rank reports it (FBA_ERR_NOT_SPD), as the
                // failing rank does, instead of solving on top blocks that hold its bad Schur updates
                // (the row is the failing rank's, or the sum of the rows when several ranks failed)
                scal[1] = red[red_w + 8];
            }
        }
    }
}

// the accumulated diagonal of the top image rows (before the subtree flow updates them) -> buffer
__global__ void k_pack_topdiag(const double* __restrict__ S, int64_t ld, const int32_t* __restrict__ rows, int64_t n,
                               double* __restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) out[q] = S[(int64_t)rows[q] * ld + rows[q]];
}

// after the ranks' sum: the 7 weights of the B rows, W_d = 1 / (sum over every image row of g^2 / s_ii)
// = 1 / (the ranks' subtree sums + the top rows' part from the summed diagonal), as k_border_weights
// forms them on one GPU; the border combine scales the B rows' Gram by sqrt(W_d) (bsc) and the
// coefficients it hands the backward solve by the same factors
__global__ __launch_bounds__(256) void k_split_weights(const double* __restrict__ red, int64_t red_diag, int64_t red_w,
                                                       const int32_t* __restrict__ rows, int64_t n, const double* __restrict__ G,
                                                       double* __restrict__ bsc, double* __restrict__ scal) {
    __shared__ double part[256][7];
    double a[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int64_t q = threadIdx.x; q < n; q += 256) {
        const int64_t i = rows[q];
        const double sii = red[red_diag + q];
        const double inv = sii > 0.0 ? 1.0 / sii : 0.0;
        const double* g = G + (i / 6) * 42 + (i % 6) * 7;
#pragma unroll
        for (int m = 0; m < 7; ++m) a[m] += g[m] * g[m] * inv;
    }
#pragma unroll
    for (int m = 0; m < 7; ++m) part[threadIdx.x][m] = a[m];
    __syncthreads();
    if (threadIdx.x < 7) {
        double v = red[red_w + threadIdx.x];
        for (int t = 0; t < 256; ++t) v += part[t][threadIdx.x];
        const double w = v > 0.0 ? 1.0 / v : 1.0;
        bsc[threadIdx.x] = sqrt(w);
        scal[16 + threadIdx.x] = w;
    }
}

int launch_pack_split(Ctx& c, int dir) {
    const Sched& s = c.sched;
    if (dir == 2) {  // the top rows' accumulated diagonal
        if (c.n_topdiag > 0)
            k_pack_topdiag<<<(unsigned)((c.n_topdiag + 255) / 256), 256, 0, c.stream>>>(c.d_S, c.L.ld, c.d_topdiag, c.n_topdiag,
                                                                                     c.d_red + c.red_diag);
        FBA_HIP(hipGetLastError());
        return FBA_OK;
    }
    k_pack_split<<<(unsigned)(s.n_top_blocks + 1), 256, 0, c.stream>>>(
        c.d_S, c.L.ld, c.d_red, c.d_sched + s.top_blocks, s.n_top_blocks, c.L.n_pad, c.L.nrhs, c.d_gblk, c.d_bown,
        (int)(c.L.n_pad / 128), c.red_gblk, c.red_w, c.d_bscr, c.d_scal, dir);
    FBA_HIP(hipGetLastError());
    if (dir == 1 && c.set.inner_constraints) {
        k_split_weights<<<1, 256, 0, c.stream>>>(c.d_red, c.red_diag, c.red_w, c.d_topdiag, c.n_topdiag, c.d_G,
                                                 c.d_bscr + BSC_OFF, c.d_scal);
        FBA_HIP(hipGetLastError());
    }
    return FBA_OK;
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
