/*
 * BuildRSD.c -- MEX drop-in for functions/BuildRSD.m:1 (source; build where MATLAB exists:
 *   mex -R2018a BuildRSD.c -I../include -L<dir of libfba.so> -lfba).
 *
 *   RSD = BuildRSD(v, data, xhat)
 *
 * Same arguments and output as the reference: v the 2n x 1 residuals (main.m:569), RSD an
 * (n/2) x 9 cell {targetID, imageID, x, y, r, vx, vy, vr, vt} per PHO row (BuildRSD.m:6, :29-40),
 * xp / yp from xhat where estimated, else the INT values (BuildRSD.m:12-26).  The per-point
 * arithmetic runs on the GPU (fba_build_rsd, libfba.so).  The reference has no error output; a
 * failure raises a MATLAB error here.
 */
#include "fba_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    (void)nlhs;
    char msg[256] = "";
    mex_problem m;
    memset(&m, 0, sizeof m);
    if (nrhs != 3 || !mxIsDouble(prhs[0]) || !mxIsStruct(prhs[1]) || !mxIsDouble(prhs[2]))
        mexErrMsgIdAndTxt("BuildRSD:args", "BuildRSD: expects (v, data, xhat)");
    int r = fm_settings(prhs[1], &m.s, 0, msg, sizeof msg, NULL);
    if (r == 2) m.s.type = FBA_TYPE_FISHEYE;  /* BuildRSD does not read the model type */
    else if (r) mexErrMsgIdAndTxt("BuildRSD:data", "%s", msg);
    if (fm_problem(prhs[1], &m, msg, sizeof msg)) {
        fm_free(&m);
        mexErrMsgIdAndTxt("BuildRSD:data", "%s", msg);
    }
    const int64_t n = m.p.n_pts;
    if ((int64_t)mxGetNumberOfElements(prhs[0]) != 2 * n) {
        fm_free(&m);
        mexErrMsgIdAndTxt("BuildRSD:args", "BuildRSD: v must have data.n entries");
    }
    fba_ctx* ctx = fm_context(&m);
    int64_t u = 0;
    if (ctx) fba_buildxhat(ctx, NULL, &u);
    if (!ctx || (int64_t)mxGetNumberOfElements(prhs[2]) != u) {
        fm_free(&m);
        mexErrMsgIdAndTxt("BuildRSD:args", "BuildRSD: %s", ctx ? "xhat length does not match the settings" : fba_last_error());
    }
    double* rsd = (double*)mxCalloc((size_t)(5 * n + 1), sizeof(double));
    if (fba_build_rsd(ctx, mxGetDoubles(prhs[0]), mxGetDoubles(prhs[2]), rsd) != 0) {
        mxFree(rsd);
        fm_free(&m);
        mexErrMsgIdAndTxt("BuildRSD:gpu", "BuildRSD: %s", fba_last_error());
    }
    const mxArray* pts = mxGetField(prhs[1], 0, "points");
    mxArray* out = mxCreateCellMatrix((mwSize)n, 9);
    static const char* idf[2] = {"targetID", "imageID"};
    for (int64_t i = 0; i < n; ++i) {
        for (int c = 0; c < 2; ++c) {
            const mxArray* id = mxGetField(pts, (mwIndex)i, idf[c]);
            mxSetCell(out, (mwIndex)(c * n + i), id ? mxDuplicateArray(id) : mxCreateString(""));
        }
        mxSetCell(out, (mwIndex)(2 * n + i), mxCreateDoubleScalar(m.xy[2 * i]));
        mxSetCell(out, (mwIndex)(3 * n + i), mxCreateDoubleScalar(m.xy[2 * i + 1]));
        for (int c = 0; c < 5; ++c) mxSetCell(out, (mwIndex)((4 + c) * n + i), mxCreateDoubleScalar(rsd[5 * i + c]));
    }
    mxFree(rsd);
    fm_free(&m);
    plhs[0] = out;
}
