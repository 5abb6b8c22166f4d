/*
 * BuildAwG.c -- MEX drop-in for functions/BuildAwG.m:14 (source; build where MATLAB exists:
 *   mex -R2018a BuildAwG.c -I../include -L<dir of libfba.so> -lfba
 * and put the resulting BuildAwG.mex* ahead of functions/ on the MATLAB path).
 *
 *   [error, A, misclosure, G, dist_scaling] = BuildAwG(data, xhat)
 *
 * Same arguments, outputs and error behaviour as the reference: `data` is main.m's struct
 * (main.m:280-383), xhat the u x 1 unknowns in Buildxhat.m's layout; A is n x u dense (n = data.n),
 * misclosure n x 1, G u x 7 with inner constraints else the scalar 0 (BuildAwG.m:33-38),
 * dist_scaling numCam x (2 + nK) (BuildAwG.m:30, :138, :150, :424-426).  error = 1 (outputs empty)
 * for an invalid data.settings.type (BuildAwG.m:209-213) or any failure, the message printed; the
 * caller aborts as main.m:417-421.  The arithmetic runs on the GPU (fba_build_awg, libfba.so); the
 * context is created once per distinct `data` and reused every iteration.
 */
#include "fba_mex_common.h"

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char msg[256] = "";
    mex_problem m;
    memset(&m, 0, sizeof m);
    int error = 0;
    if (nrhs != 2 || !mxIsStruct(prhs[0]) || !mxIsDouble(prhs[1])) {
        snprintf(msg, sizeof msg, "BuildAwG: expects (data, xhat)");
        error = 1;
    }
    if (!error && fm_settings(prhs[0], &m.s, 1, msg, sizeof msg, NULL)) error = 1;
    if (!error && fm_problem(prhs[0], &m, msg, sizeof msg)) error = 1;
    fba_ctx* ctx = error ? NULL : fm_context(&m);
    if (!error && !ctx) {
        snprintf(msg, sizeof msg, "BuildAwG: %s", fba_last_error());
        error = 1;
    }
    int64_t u = 0;
    if (!error) {
        fba_buildxhat(ctx, NULL, &u);
        if ((int64_t)mxGetNumberOfElements(prhs[1]) != u) {
            snprintf(msg, sizeof msg, "BuildAwG: xhat has %ld entries, the settings give u = %ld",
                     (long)mxGetNumberOfElements(prhs[1]), (long)u);
            error = 1;
        }
    }
    const int64_t n = 2 * m.p.n_pts;
    const int nc = m.p.n_cam, ncol = 2 + m.s.num_radial;
    mxArray *A = NULL, *w = NULL, *G = NULL, *ds = NULL;
    if (!error) {
        A = mxCreateDoubleMatrix((mwSize)n, (mwSize)u, mxREAL);
        w = mxCreateDoubleMatrix((mwSize)n, 1, mxREAL);
        G = m.s.inner_constraints ? mxCreateDoubleMatrix((mwSize)u, 7, mxREAL) : mxCreateDoubleScalar(0.0);
        ds = mxCreateDoubleMatrix((mwSize)nc, (mwSize)ncol, mxREAL);
        /* column-major n x u, u x 7, numCam x (2 + nK): MATLAB's own layouts */
        if (fba_build_awg(ctx, mxGetDoubles(prhs[1]), mxGetDoubles(A), mxGetDoubles(w),
                          m.s.inner_constraints ? mxGetDoubles(G) : NULL, mxGetDoubles(ds)) != 0) {
            snprintf(msg, sizeof msg, "BuildAwG: %s", fba_last_error());
            error = 1;
        }
    }
    fm_free(&m);
    if (error) {
        mexPrintf("%s\n", msg);
        mxArray* out[4] = {A, w, G, ds};
        for (int i = 0; i < 4; ++i)
            if (out[i]) mxDestroyArray(out[i]);
        A = mxCreateDoubleMatrix(0, 0, mxREAL);
        w = mxCreateDoubleMatrix(0, 0, mxREAL);
        G = mxCreateDoubleScalar(0.0);
        ds = mxCreateDoubleMatrix(0, 0, mxREAL);
    }
    mxArray* out[5] = {mxCreateDoubleScalar((double)error), A, w, G, ds};
    for (int i = 0; i < 5; ++i) {
        if (i < (nlhs > 0 ? nlhs : 1)) plhs[i] = out[i];
        else mxDestroyArray(out[i]);
    }
}
