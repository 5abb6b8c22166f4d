/*
 * fba_mex.c -- MATLAB MEX gateway to libfba.so (source only: MATLAB and mex.h are not in this image).
 *
 * Build (where MATLAB exists):  mex -R2018a fba_mex.c -I../include -L<dir of libfba.so> -lfba
 *
 * Replaces, in the reference's main.m, the body from Buildxhat to the end of the statistics
 * (main.m:386-494 Buildxhat + the Gauss-Newton loop, main.m:567-602 v / BuildRSD / RMS / sigma0^2)
 * and the explicit inverse's by-products the writers read (main.m:446-482 Correlation and the
 * de-scaled Cx, main.m:602 Cx = sigma02 * Cx):
 *
 *   [xhat, count, deltasum, v, rsd, stats, cx_diag, corr] = fba_mex(xy, img, cam, tie, xyz_fixed, eop0,
 *                                                                  iop0, cam_info, tie0, flags, cfg)
 *     xy         2 x n_pts double (x; y per PHO row)
 *     img, cam   1 x n_pts int32, 0-based EXT row / INT pair ([P.ext_index] - 1, [P.cam_num] - 1)
 *     tie        1 x n_pts int32, 0-based TIE index, -1 for a fixed (control) point
 *     xyz_fixed  3 x n_pts double (CNT coordinates of each point)
 *     eop0       6 x numImg double (Xc Yc Zc omega phi kappa, radians)
 *     iop0       (5+nK) x numCam double (xp yp c K1..KnK P1 P2)
 *     cam_info   5 x numCam double (y_dir xmin ymin xmax ymax)
 *     tie0       3 x numtie double (CNT coordinates of the TIE list)
 *     flags      1 x 15 int32: Estimate_Xc Yc Zc w p k xp yp c radial decent, nK, Type (0 fisheye,
 *                1 pinhole, 2 equisolid, 3 orthographic, 4 stereographic), Inner_Constraints, Iteration_Cap
 *     cfg        1 x 3 double: Threshold_Value, Meas_std, Meas_std_y
 *   outputs: xhat (u x 1), count, deltasum (1 x count), v (2 n_pts x 1), rsd (5 x n_pts: r vx vy vr vt),
 *            stats (6 x 1: RMSx RMSy RMS sigma02 vTPv n-u), cx_diag (u x 1: diag of the final Cx),
 *            corr (mu x mu x numImg: per image the Correlation sub-block over its EOPs and its camera's
 *            IOPs, mu = u_img + u_cam)
 * Errors raise MATLAB errors with fba_last_error()'s message (the reference sets main_error = 1).
 */
#include <stdint.h>

#include "fba.h"
#include "mex.h"

static void fail(fba_ctx* ctx, const char* id) {
    if (ctx) fba_destroy(ctx);
    mexErrMsgIdAndTxt(id, "%s", fba_last_error());
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    if (nrhs != 11) mexErrMsgIdAndTxt("fba:args", "fba_mex expects 11 inputs");
    if (!mxIsInt32(prhs[1]) || !mxIsInt32(prhs[2]) || !mxIsInt32(prhs[3]) || !mxIsInt32(prhs[9]))
        mexErrMsgIdAndTxt("fba:args", "img, cam, tie and flags must be int32");
    fba_problem p = {0};
    p.n_pts = (int64_t)mxGetN(prhs[0]);
    p.xy = mxGetDoubles(prhs[0]);
    p.img = (const int32_t*)mxGetInt32s(prhs[1]);
    p.cam = (const int32_t*)mxGetInt32s(prhs[2]);
    p.tie = (const int32_t*)mxGetInt32s(prhs[3]);
    p.xyz_fixed = mxGetDoubles(prhs[4]);
    p.eop0 = mxGetDoubles(prhs[5]);
    p.n_img = (int32_t)mxGetN(prhs[5]);
    p.iop0 = mxGetDoubles(prhs[6]);
    p.n_cam = (int32_t)mxGetN(prhs[6]);
    p.cam_info = mxGetDoubles(prhs[7]);
    p.tie0 = mxGetDoubles(prhs[8]);
    p.n_tie = (int32_t)mxGetN(prhs[8]);
    const int32_t* f = (const int32_t*)mxGetInt32s(prhs[9]);
    const double* cfg = mxGetDoubles(prhs[10]);
    fba_settings s = {f[0], f[1], f[2], f[3], f[4], f[5], f[6], f[7], f[8], f[9], f[10], f[11], f[12], f[13], f[14],
                      0, cfg[0], cfg[1], cfg[2]};
    fba_options o = {0, 0, 1, 0, NULL};
    fba_ctx* ctx = NULL;
    if (fba_create(&p, &s, &o, &ctx)) fail(NULL, "fba:create");

    int64_t u = 0;
    fba_buildxhat(ctx, NULL, &u);
    const int cap = s.iteration_cap > 0 ? s.iteration_cap : 1;
    double* hist = (double*)mxMalloc(sizeof(double) * cap);
    int32_t it = 0;
    if (fba_adjust(ctx, &it, hist)) { mxFree(hist); fail(ctx, "fba:adjust"); }

    plhs[0] = mxCreateDoubleMatrix((mwSize)u, 1, mxREAL);
    if (fba_get_xhat(ctx, mxGetDoubles(plhs[0]), 0)) { mxFree(hist); fail(ctx, "fba:xhat"); }
    if (nlhs > 1) plhs[1] = mxCreateDoubleScalar(it);
    if (nlhs > 2) {
        plhs[2] = mxCreateDoubleMatrix(1, (mwSize)it, mxREAL);
        for (int i = 0; i < it; ++i) mxGetDoubles(plhs[2])[i] = hist[i];
    }
    mxFree(hist);

    mxArray* v = mxCreateDoubleMatrix((mwSize)(2 * p.n_pts), 1, mxREAL);   /* main.m:569 */
    mxArray* rsd = mxCreateDoubleMatrix(5, (mwSize)p.n_pts, mxREAL);       /* BuildRSD.m:29-40 */
    mxArray* st = mxCreateDoubleMatrix(6, 1, mxREAL);                      /* main.m:594-601 */
    if (fba_residuals(ctx, mxGetDoubles(v), mxGetDoubles(rsd), mxGetDoubles(st))) fail(ctx, "fba:residuals");
    if (nlhs > 3) plhs[3] = v; else mxDestroyArray(v);
    if (nlhs > 4) plhs[4] = rsd; else mxDestroyArray(rsd);
    const double sigma02 = mxGetDoubles(st)[3];
    if (nlhs > 5) plhs[5] = st; else mxDestroyArray(st);

    if (nlhs > 6) {  /* main.m:428-482, :602 -- from the factor of the last solve */
        const int u_img = f[0] + f[1] + f[2] + f[3] + f[4] + f[5];
        const int u_cam = f[8] + f[6] + f[7] + f[9] * f[11] + 2 * f[10];
        const mwSize mu = (mwSize)(u_img + u_cam);
        const mwSize dims[3] = {mu, mu, (mwSize)p.n_img};
        plhs[6] = mxCreateDoubleMatrix((mwSize)u, 1, mxREAL);
        double* corr = NULL;
        if (nlhs > 7) {
            plhs[7] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
            corr = mxGetDoubles(plhs[7]);  /* row-major mu x mu per image = MATLAB's transpose: symmetric */
        }
        if (fba_covariance(ctx, sigma02, mxGetDoubles(plhs[6]), corr)) fail(ctx, "fba:covariance");
    }
    fba_destroy(ctx);
}
