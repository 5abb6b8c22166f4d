/*
 * Buildxhat.c -- MEX drop-in for functions/Buildxhat.m:2 (source; build where MATLAB exists:
 *   mex -R2018a Buildxhat.c -I../include -L<dir of libfba.so> -lfba).
 *
 *   [error, xhat, xhatnames] = Buildxhat(data, EXT, INT, TIE, CNT)
 *
 * Same arguments and outputs as the reference: EXT / INT / CNT are main.m's cell arrays after its
 * string -> number conversion (main.m:196-258; EXT angles in radians), TIE the tie-point ID list
 * (a cellstr, or the string array ReadFiles returns).  xhat is u x 1 in the reference's layout --
 * [per EXT row: Xc Yc Zc w p k][per camera: xp yp c K1..KnK P1 P2][per TIE: X Y Z], each part only
 * when estimated (Buildxhat.m:22-134) -- from libfba.so's fba_buildxhat on the packed problem, and
 * xhatnames the reference's names ('Xc_<image>_<camera>', 'xp_<camera>', 'k<j>_<camera>',
 * 'X_<target>', Buildxhat.m:35-131).  error = 1 (message printed) when a TIE target is not in CNT
 * (Buildxhat.m:124-128) or on any failure.
 */
#include <stdlib.h>

#include "fba_mex_common.h"

static mxArray* make_name(const char* a, const char* b, const char* c) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s%s%s", a, b ? b : "", c ? c : "");
    return mxCreateString(buf);
}

void mexFunction(int nlhs, mxArray* plhs[], int nrhs, const mxArray* prhs[]) {
    char msg[256] = "";
    mex_problem m;
    memset(&m, 0, sizeof m);
    int error = 0;
    mxArray* tie_cells = NULL;
    if (nrhs != 5 || !mxIsStruct(prhs[0]) || !mxIsCell(prhs[1]) || !mxIsCell(prhs[2]) || !mxIsCell(prhs[4])) {
        snprintf(msg, sizeof msg, "Buildxhat: expects (data, EXT, INT, TIE, CNT) with cell arrays EXT, INT, CNT");
        error = 1;
    }
    /* Buildxhat does not read data.settings.type (an invalid one is BuildAwG's error) */
    int nk_ref = 1;  /* Num_Radial_Distortions as given: 0 means no K columns in INT (Buildxhat.m:71-72) */
    if (!error) {
        const int r = fm_settings(prhs[0], &m.s, 0, msg, sizeof msg, &nk_ref);
        if (r == 2) m.s.type = FBA_TYPE_FISHEYE;
        else if (r) error = 1;
    }
    if (!error && nk_ref < 0) {
        snprintf(msg, sizeof msg, "Buildxhat: Num_Radial_Distortions must be >= 0");
        error = 1;
    }
    if (!error && fm_problem(prhs[0], &m, msg, sizeof msg)) error = 1;
    const mxArray *EXT = prhs[1], *INT = prhs[2], *TIE = NULL;
    /* start values from EXT / INT / CNT as Buildxhat.m:22-131 (not from data.points) */
    if (!error && fm_start_values(&m, EXT, INT, prhs[3], prhs[4], nk_ref, &TIE, &tie_cells, msg, sizeof msg)) error = 1;
    const int nimg = m.p.n_img, ncam = m.p.n_cam;
    const int ntie = TIE ? (int)mxGetNumberOfElements(TIE) : 0;
    fba_ctx* ctx = error ? NULL : fm_context(&m);
    if (!error && !ctx) {
        snprintf(msg, sizeof msg, "Buildxhat: %s", fba_last_error());
        error = 1;
    }
    int64_t u = 0;
    mxArray *xhat = NULL, *names = NULL;
    if (!error) {
        fba_buildxhat(ctx, NULL, &u);
        xhat = mxCreateDoubleMatrix((mwSize)u, 1, mxREAL);
        if (fba_buildxhat(ctx, mxGetDoubles(xhat), &u) != 0) {
            snprintf(msg, sizeof msg, "Buildxhat: %s", fba_last_error());
            error = 1;
        }
    }
    if (!error) {  /* names, Buildxhat.m:35-131 */
        names = mxCreateCellMatrix((mwSize)u, 1);
        mwIndex q = 0;
        const fba_settings* s = &m.s;
        const int ee[6] = {s->est_Xc, s->est_Yc, s->est_Zc, s->est_omega, s->est_phi, s->est_kappa};
        static const char* en[6] = {"Xc_", "Yc_", "Zc_", "w_", "p_", "k_"};
        for (int i = 1; i <= nimg; ++i) {
            char *img = fm_cell_str(EXT, i, 1), *cam = fm_cell_str(EXT, i, 2);
            char suffix[256];
            snprintf(suffix, sizeof suffix, "%s_%s", img ? img : "", cam ? cam : "");
            for (int a = 0; a < 6; ++a)
                if (ee[a]) mxSetCell(names, q++, make_name(en[a], suffix, NULL));
            if (img) mxFree(img);
            if (cam) mxFree(cam);
        }
        for (int k = 1; k <= ncam; ++k) {
            char* cam = fm_cell_str(INT, 2 * k - 1, 1);
            if (s->est_xp) mxSetCell(names, q++, make_name("xp_", cam, NULL));
            if (s->est_yp) mxSetCell(names, q++, make_name("yp_", cam, NULL));
            if (s->est_c) mxSetCell(names, q++, make_name("c_", cam, NULL));
            char head[32];
            for (int j = 1; s->est_radial && j <= nk_ref; ++j) {
                snprintf(head, sizeof head, "k%d_", j);
                mxSetCell(names, q++, make_name(head, cam, NULL));
            }
            for (int j = 1; s->est_decent && j <= 2; ++j) {
                snprintf(head, sizeof head, "p%d_", j);
                mxSetCell(names, q++, make_name(head, cam, NULL));
            }
            if (cam) mxFree(cam);
        }
        for (int t = 0; t < ntie; ++t) {
            char* id = mxArrayToString(mxGetCell(TIE, t));
            mxSetCell(names, q++, make_name("X_", id, NULL));
            mxSetCell(names, q++, make_name("Y_", id, NULL));
            mxSetCell(names, q++, make_name("Z_", id, NULL));
            mxFree(id);
        }
    }
    fm_free(&m);
    if (tie_cells) mxDestroyArray(tie_cells);
    if (error) {
        mexPrintf("%s\n", msg);
        if (xhat) mxDestroyArray(xhat);
        if (names) mxDestroyArray(names);
        xhat = mxCreateDoubleMatrix(0, 0, mxREAL);
        names = mxCreateCellMatrix(0, 0);
    }
    mxArray* out[3] = {mxCreateDoubleScalar((double)error), xhat, names};
    for (int i = 0; i < 3; ++i) {
        if (i < (nlhs > 0 ? nlhs : 1)) plhs[i] = out[i];
        else mxDestroyArray(out[i]);
    }
}
