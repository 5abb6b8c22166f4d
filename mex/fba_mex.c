/*
 * fba_mex.c -- whole-loop MEX gateway to libfba.so (source; build where MATLAB exists:
 *   mex -R2018a fba_mex.c -I../include -L<dir of libfba.so> -lfba).
 *
 *   [error, xhat, count, deltasum, v, RSD, stats, cx_diag, corr] = fba_mex(data, EXT, INT, TIE, CNT)
 *
 * Replaces, in the reference's main.m, everything from Buildxhat to the statistics -- main.m:386-494
 * (Buildxhat, then the Gauss-Newton loop: BuildAwG, u = A'Pw, N = A'PA, the bordered inverse,
 * de-scaling, xhat += delta, deltasum = sumabs(delta), the stop rule) and main.m:567-602 (v = A*delta + w,
 * RSD = BuildRSD(v, data, xhat), RMSx / RMSy / RMS, sigma02 = v'Pv/(n-u), Cx = sigma02*Cx) -- plus the
 * by-products of the explicit inverse the report writers read (main.m:446-482 Correlation, the de-scaled
 * diag(Cx)).  It takes exactly what main.m holds at line 386: the `data` struct (main.m:112-177
 * data.settings, main.m:280-383 data.points, numImg, numCam, numtie) and the EXT / INT / TIE / CNT cell
 * arrays after main.m:196-264 (EXT angles in radians), read as Buildxhat.m and BuildAwG.m read them
 * (fba_mex_common.h), so main.m calls it in place of lines 386-602:
 *
 *   [main_error, xhat, count, deltasum, v, RSD, st, Cxd, Corr] = fba_mex(data, EXT, INT, TIE, CNT);
 *   RMSx = st(1); RMSy = st(2); RMS = st(3); sigma02 = st(4);
 *
 * outputs
 *   error     0, or 1 where the reference sets main_error = 1 (message printed, like main.m:389-393,
 *             :417-421); the other outputs are then empty
 *   xhat      u x 1, the reference's layout (Buildxhat.m:22-134), after the last update (main.m:484)
 *   count     iterations run (main.m:413, stop rule main.m:412 and :490-493)
 *   deltasum  1 x count, sumabs(delta) of every iteration (main.m:487, functions/sumabs.m)
 *   v         data.n x 1, A*delta + w of the last linearisation (main.m:569)
 *   RSD       (data.n/2) x 9 cell {targetID, imageID, x, y, r, vx, vy, vr, vt} (BuildRSD.m:6, :29-40)
 *   stats     [RMSx; RMSy; RMS; sigma02; v'Pv; n-u] (main.m:594-601)
 *   cx_diag   u x 1, diag of the final Cx = sigma02 * Cx with the distortion entries de-scaled
 *             (main.m:460-482 diagonal only, :602)
 *   corr      mu x mu x numImg, per EXT image the Correlation matrix (main.m:446-456) over the image's
 *             estimated EOPs and its camera's estimated IOP / distortion unknowns (main.m:831-840),
 *             mu = u_perimage + u_percam
 * Num_Radial_Distortions = 0 with Estimate_Radial_Distortions = 1 is rejected (error = 1): there
 * Buildxhat.m:13 lays out no K while BuildAwG.m:18-20 builds one K column, so the reference's
 * xhat + delta does not conform.
 */
#include "fba_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char msg[512] = "";
    mex_problem m;
    memset(&m, 0, sizeof m);
    int error = 0, nk_ref = 1;
    mxArray* tie_cells = NULL;
    const mxArray* TIE = NULL;
    fba_ctx* ctx = NULL;
    mxArray* out[9] = {NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL};
    if (nrhs != 5 || !mxIsStruct(prhs[0]) || !mxIsCell(prhs[1]) || !mxIsCell(prhs[2]) || !mxIsCell(prhs[4])) {
        snprintf(msg, sizeof msg, "fba_mex: expects (data, EXT, INT, TIE, CNT) with cell arrays EXT, INT, CNT");
        error = 1;
    }
    if (!error && fm_settings(prhs[0], &m.s, 0, msg, sizeof msg, &nk_ref)) error = 1;  /* (invalid Type: BuildAwG.m:209-213) */
    if (!error && nk_ref < 1 && (int)fm_num(mxGetField(prhs[0], 0, "settings"), 0, "Estimate_radial", 0, NULL)) {
        snprintf(msg, sizeof msg, "fba_mex: Num_Radial_Distortions = 0 with Estimate_Radial_Distortions = 1: "
                 "Buildxhat.m:13 and BuildAwG.m:18-20 disagree on the number of unknowns");
        error = 1;
    }
    if (!error && fm_problem(prhs[0], &m, msg, sizeof msg)) error = 1;
    if (!error && fm_start_values(&m, prhs[1], prhs[2], prhs[3], prhs[4], nk_ref, &TIE, &tie_cells, msg, sizeof msg))
        error = 1;
    (void)TIE;
    fba_options o;
    memset(&o, 0, sizeof o);
    o.world = 1;
    if (!error && fba_create(&m.p, &m.s, &o, &ctx) != 0) {
        snprintf(msg, sizeof msg, "fba_mex: %s", fba_last_error());
        ctx = NULL;
        error = 1;
    }
    int64_t u = 0;
    int32_t count = 0;
    double* hist = NULL;
    double st[6] = {0, 0, 0, 0, 0, 0};
    const int64_t n = m.p.n_pts;
    if (!error) {  /* main.m:386-494 */
        fba_buildxhat(ctx, NULL, &u);
        const int cap = m.s.iteration_cap > 0 ? m.s.iteration_cap : 1;
        hist = (double*)mxCalloc((size_t)cap + 1, sizeof(double));
        if (fba_adjust(ctx, &count, hist) != 0) {
            snprintf(msg, sizeof msg, "fba_mex: iteration %d: %s", (int)count, fba_last_error());
            error = 1;
        }
    }
    if (!error) {
        out[1] = mxCreateDoubleMatrix((mwSize)u, 1, mxREAL);
        out[2] = mxCreateDoubleScalar((double)count);
        out[3] = mxCreateDoubleMatrix(1, (mwSize)count, mxREAL);
        for (int i = 0; i < count; ++i) mxGetDoubles(out[3])[i] = hist[i];
        out[4] = mxCreateDoubleMatrix((mwSize)(2 * n), 1, mxREAL);
        double* rsd = (double*)mxCalloc((size_t)(5 * n + 1), sizeof(double));
        if (fba_get_xhat(ctx, mxGetDoubles(out[1]), 0) != 0 ||
            fba_residuals(ctx, mxGetDoubles(out[4]), rsd, st) != 0) {  /* main.m:567-601 */
            snprintf(msg, sizeof msg, "fba_mex: %s", fba_last_error());
            error = 1;
        }
        if (!error) {  /* BuildRSD.m:6, :40: {targetID, imageID, x, y, r, vx, vy, vr, vt} per PHO row */
            const mxArray* pts = mxGetField(prhs[0], 0, "points");
            static const char* idf[2] = {"targetID", "imageID"};
            out[5] = mxCreateCellMatrix((mwSize)n, 9);
            for (int64_t i = 0; i < n; ++i) {
                for (int c = 0; c < 2; ++c) {
                    const mxArray* id = mxGetField(pts, (mwIndex)i, idf[c]);
                    mxSetCell(out[5], (mwIndex)(c * n + i), id ? mxDuplicateArray(id) : mxCreateString(""));
                }
                mxSetCell(out[5], (mwIndex)(2 * n + i), mxCreateDoubleScalar(m.xy[2 * i]));
                mxSetCell(out[5], (mwIndex)(3 * n + i), mxCreateDoubleScalar(m.xy[2 * i + 1]));
                for (int c = 0; c < 5; ++c)
                    mxSetCell(out[5], (mwIndex)((4 + c) * n + i), mxCreateDoubleScalar(rsd[5 * i + c]));
            }
            out[6] = mxCreateDoubleMatrix(6, 1, mxREAL);
            for (int i = 0; i < 6; ++i) mxGetDoubles(out[6])[i] = st[i];
        }
        mxFree(rsd);
    }
    if (!error && nlhs > 7) {  /* main.m:428-482, :602 -- from the factor of the last solve */
        const fba_settings* s = &m.s;
        const int u_img = s->est_Xc + s->est_Yc + s->est_Zc + s->est_omega + s->est_phi + s->est_kappa;
        const int u_cam = s->est_xp + s->est_yp + s->est_c + s->est_radial * s->num_radial + 2 * s->est_decent;
        const mwSize mu = (mwSize)(u_img + u_cam);
        const mwSize dims[3] = {mu, mu, (mwSize)m.p.n_img};
        out[7] = mxCreateDoubleMatrix((mwSize)u, 1, mxREAL);
        out[8] = mxCreateNumericArray(3, dims, mxDOUBLE_CLASS, mxREAL);
        /* row-major mu x mu per image = MATLAB's column-major transpose; the blocks are symmetric */
        if (fba_covariance(ctx, st[3], mxGetDoubles(out[7]), nlhs > 8 ? mxGetDoubles(out[8]) : NULL) != 0) {
            snprintf(msg, sizeof msg, "fba_mex: %s", fba_last_error());
            error = 1;
        }
    }
    if (ctx) fba_destroy(ctx);
    if (hist) mxFree(hist);
    if (tie_cells) mxDestroyArray(tie_cells);
    fm_free(&m);
    if (error) {
        mexPrintf("%s\n", msg);
        for (int i = 1; i < 9; ++i) {
            if (out[i]) mxDestroyArray(out[i]);
            out[i] = i == 5 ? mxCreateCellMatrix(0, 0) : mxCreateDoubleMatrix(0, 0, mxREAL);
        }
    }
    out[0] = mxCreateDoubleScalar((double)error);
    for (int i = 0; i < 9; ++i) {
        if (!out[i]) out[i] = mxCreateDoubleMatrix(0, 0, mxREAL);
        if (i < (nlhs > 0 ? nlhs : 1)) plhs[i] = out[i];
        else mxDestroyArray(out[i]);
    }
}
