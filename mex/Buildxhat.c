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

/* cell (r, c) of an M x N cell array (1-based as in MATLAB) */
static const mxArray* cell_at(const mxArray* C, mwIndex r, mwIndex c) {
    const mwSize M = mxGetM(C);
    return mxGetCell(C, (c - 1) * M + (r - 1));
}
static double cell_num(const mxArray* C, mwIndex r, mwIndex c) {
    const mxArray* v = cell_at(C, r, c);
    return (v && mxGetNumberOfElements(v) > 0) ? mxGetScalar(v) : 0.0;
}
static char* cell_str(const mxArray* C, mwIndex r, mwIndex c) {
    const mxArray* v = cell_at(C, r, c);
    return (v && mxIsChar(v)) ? mxArrayToString(v) : NULL;
}

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
    if (!error) {
        const int r = fm_settings(prhs[0], &m.s, 0, msg, sizeof msg);
        if (r == 2) m.s.type = FBA_TYPE_FISHEYE;
        else if (r) error = 1;
    }
    if (!error && m.s.num_radial < 1) {
        snprintf(msg, sizeof msg, "Buildxhat: Num_Radial_Distortions must be >= 1");
        error = 1;
    }
    if (!error && fm_problem(prhs[0], &m, msg, sizeof msg)) error = 1;
    const mxArray *EXT = prhs[1], *INT = prhs[2], *CNT = prhs[4];
    const mxArray* TIE = nrhs > 3 ? prhs[3] : NULL;
    if (!error && TIE && mxIsClass(TIE, "string")) {  /* ReadFiles' string array -> cellstr */
        mxArray* in[1] = {(mxArray*)TIE};
        if (mexCallMATLAB(1, &tie_cells, 1, in, "cellstr") == 0) TIE = tie_cells;
    }
    const int nimg = m.p.n_img, ncam = m.p.n_cam, nk = m.s.num_radial, cw = 5 + nk;
    const int ntie = (TIE && mxIsCell(TIE)) ? (int)mxGetNumberOfElements(TIE) : 0;
    if (!error && ntie != m.p.n_tie) {
        snprintf(msg, sizeof msg, "Buildxhat: TIE has %d entries, data.numtie = %d", ntie, m.p.n_tie);
        error = 1;
    }
    /* start values from EXT / INT / CNT as Buildxhat.m:22-131 (not from data.points) */
    for (int i = 1; !error && i <= nimg; ++i)
        for (int a = 0; a < 6; ++a) m.eop0[6 * (i - 1) + a] = cell_num(EXT, i, 3 + a);
    for (int k = 1; !error && k <= ncam; ++k)
        for (int a = 0; a < cw; ++a) m.iop0[cw * (k - 1) + a] = cell_num(INT, 2 * k, 1 + a);
    for (int t = 0; !error && t < ntie; ++t) {
        char* id = mxIsChar(mxGetCell(TIE, t)) ? mxArrayToString(mxGetCell(TIE, t)) : NULL;
        int found = 0;
        for (mwIndex j = 1; id && j <= mxGetM(CNT) && !found; ++j) {
            char* cid = cell_str(CNT, j, 1);
            if (cid && strcmp(cid, id) == 0) {
                for (int a = 0; a < 3; ++a) m.tie0[3 * t + a] = cell_num(CNT, j, 2 + a);
                found = 1;
            }
            if (cid) mxFree(cid);
        }
        if (!found) {
            snprintf(msg, sizeof msg, "Error Buildxhat(): can't find %s from .tie in .cnt", id ? id : "?");
            error = 1;
        }
        if (id) mxFree(id);
    }
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
            char *img = cell_str(EXT, i, 1), *cam = cell_str(EXT, i, 2);
            char suffix[256];
            snprintf(suffix, sizeof suffix, "%s_%s", img ? img : "", cam ? cam : "");
            for (int a = 0; a < 6; ++a)
                if (ee[a]) mxSetCell(names, q++, make_name(en[a], suffix, NULL));
            if (img) mxFree(img);
            if (cam) mxFree(cam);
        }
        for (int k = 1; k <= ncam; ++k) {
            char* cam = cell_str(INT, 2 * k - 1, 1);
            if (s->est_xp) mxSetCell(names, q++, make_name("xp_", cam, NULL));
            if (s->est_yp) mxSetCell(names, q++, make_name("yp_", cam, NULL));
            if (s->est_c) mxSetCell(names, q++, make_name("c_", cam, NULL));
            char head[32];
            for (int j = 1; s->est_radial && j <= nk; ++j) {
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
