/*
 * fba_mex_common.h -- shared by the MEX drop-ins BuildAwG.c, Buildxhat.c and BuildRSD.c.
 *
 * Reads the reference's `data` struct (main.m:112-177 data.settings, main.m:280-383 data.points,
 * numImg, numCam, numtie) into the packed fba_problem / fba_settings of include/fba.h, and keeps one
 * libfba.so context per distinct problem across calls (BuildAwG is called every Gauss-Newton
 * iteration with the same `data`, main.m:416), released by mexAtExit.
 *
 * data.points(i) fields read: x y ext_index cam_num tieIndex X Y Z Xc Yc Zc w p k xp yp c K P y_dir
 * xmin ymin xmax ymax (the reference's names; indices 1-based, -1 = not a tie point).
 */
#ifndef FBA_MEX_COMMON_H_
#define FBA_MEX_COMMON_H_

#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "fba.h"
#include "mex.h"

typedef struct mex_problem {
    fba_problem p;
    fba_settings s;
    double *xy, *xyz, *eop0, *iop0, *caminfo, *tie0;
    int32_t *img, *cam, *tie;
} mex_problem;

/* a field of struct element i as a double (absent or empty: `dflt`, *found = 0) */
static double fm_num(const mxArray* st, mwIndex i, const char* name, double dflt, int* found) {
    const mxArray* f = mxGetField(st, i, name);
    if (found) *found = f != NULL && mxGetNumberOfElements(f) > 0;
    if (!f || mxGetNumberOfElements(f) == 0) return dflt;
    return mxGetScalar(f);
}

/* data.settings.type as the FBA_TYPE_* enum (BuildAwG.m:188-213), -1 when invalid */
static int fm_type(const mxArray* settings) {
    static const char* names[5] = {"fisheye", "pinhole", "equisolid", "orthographic", "stereographic"};
    const mxArray* f = mxGetField(settings, 0, "type");
    mxArray* tmp = NULL;
    if (f && mxIsClass(f, "string")) {  /* a string scalar: char() it */
        mxArray* in[1] = {(mxArray*)f};
        if (mexCallMATLAB(1, &tmp, 1, in, "char") == 0) f = tmp;
    }
    int t = -1;
    if (f && mxIsChar(f)) {
        char* str = mxArrayToString(f);
        for (int k = 0; k < 5 && str; ++k)
            if (strcmp(str, names[k]) == 0) t = k;
        mxFree(str);
    }
    if (tmp) mxDestroyArray(tmp);
    return t;
}

/* data.settings -> fba_settings (main.m:112-177); returns 0, 1 (settings missing) or 2 (invalid
 * type, BuildAwG.m:209-213) with a message.
 * Num_Radial_Distortions = 0 (nk_ref, when not NULL, receives the value as given):
 *   clamp_nk = 1  BuildAwG.m:18-20 -- a local copy clamped to 1, Estimate_radial kept;
 *   clamp_nk = 0  Buildxhat.m:13 / BuildRSD.m:3 -- no radial unknowns at all (the reference's K list is
 *                 empty): the library's layout with one radial slot that is not estimated, which has the
 *                 same unknowns in the same order. */
static int fm_settings(const mxArray* data, fba_settings* s, int clamp_nk, char* msg, size_t nmsg, int* nk_ref) {
    const mxArray* st = mxIsStruct(data) ? mxGetField(data, 0, "settings") : NULL;
    if (!st || !mxIsStruct(st)) { snprintf(msg, nmsg, "data.settings is missing"); return 1; }
    memset(s, 0, sizeof *s);
    s->est_Xc = (int32_t)fm_num(st, 0, "Estimate_Xc", 0, NULL);
    s->est_Yc = (int32_t)fm_num(st, 0, "Estimate_Yc", 0, NULL);
    s->est_Zc = (int32_t)fm_num(st, 0, "Estimate_Zc", 0, NULL);
    s->est_omega = (int32_t)fm_num(st, 0, "Estimate_w", 0, NULL);
    s->est_phi = (int32_t)fm_num(st, 0, "Estimate_p", 0, NULL);
    s->est_kappa = (int32_t)fm_num(st, 0, "Estimate_k", 0, NULL);
    s->est_xp = (int32_t)fm_num(st, 0, "Estimate_xp", 0, NULL);
    s->est_yp = (int32_t)fm_num(st, 0, "Estimate_yp", 0, NULL);
    s->est_c = (int32_t)fm_num(st, 0, "Estimate_c", 0, NULL);
    s->est_radial = (int32_t)fm_num(st, 0, "Estimate_radial", 0, NULL);
    s->est_decent = (int32_t)fm_num(st, 0, "Estimate_decent", 0, NULL);
    s->num_radial = (int32_t)fm_num(st, 0, "Num_Radial_Distortions", 1, NULL);
    if (nk_ref) *nk_ref = s->num_radial;
    if (s->num_radial < 1) {
        if (!clamp_nk) s->est_radial = 0; /* Buildxhat.m:88-93: an empty K, nothing estimated */
        s->num_radial = 1;                /* BuildAwG.m:18-20 (a local copy) */
    }
    s->type = fm_type(st);
    s->inner_constraints = (int32_t)fm_num(st, 0, "Inner_Constraints", 0, NULL);
    s->iteration_cap = (int32_t)fm_num(st, 0, "Iteration_Cap", 100, NULL);
    s->threshold = fm_num(st, 0, "threshold", 1e-6, NULL);
    /* weights do not enter BuildAwG / Buildxhat / BuildRSD; main.m:123-127 defaults them to 1 */
    s->meas_std_x = fm_num(st, 0, "Meas_std", 1.0, NULL);
    int has_y = 0;
    s->meas_std_y = fm_num(st, 0, "Meas_std_y", s->meas_std_x, &has_y);
    if (s->type < 0) { snprintf(msg, nmsg, "BuildAwG, invalid type in data.settings.type"); return 2; }
    return 0;
}

static void fm_free(mex_problem* m) {
    void* q[9] = {m->xy, m->xyz, m->eop0, m->iop0, m->caminfo, m->tie0, m->img, m->cam, m->tie};
    for (int i = 0; i < 9; ++i)
        if (q[i]) mxFree(q[i]);
    memset(m, 0, sizeof *m);
}

/* data.points + counts -> fba_problem (main.m:280-383 after the joins); fixed EOP / IOP / camera
 * bounds per image / camera from the points that reference them, tie start values from the points'
 * CNT coordinates.  Returns 0, or 1 with a message. */
static int fm_problem(const mxArray* data, mex_problem* m, char* msg, size_t nmsg) {
    const mxArray* pts = mxGetField(data, 0, "points");
    if (!pts || !mxIsStruct(pts)) { snprintf(msg, nmsg, "data.points is missing"); return 1; }
    const int64_t n = (int64_t)mxGetNumberOfElements(pts);
    const int nimg = (int)fm_num(data, 0, "numImg", 0, NULL), ncam = (int)fm_num(data, 0, "numCam", 0, NULL);
    const int ntie = (int)fm_num(data, 0, "numtie", 0, NULL);
    const int nk = m->s.num_radial < 1 ? 1 : m->s.num_radial, cw = 5 + nk;
    m->xy = (double*)mxCalloc((size_t)(2 * n + 1), sizeof(double));
    m->xyz = (double*)mxCalloc((size_t)(3 * n + 1), sizeof(double));
    m->img = (int32_t*)mxCalloc((size_t)(n + 1), sizeof(int32_t));
    m->cam = (int32_t*)mxCalloc((size_t)(n + 1), sizeof(int32_t));
    m->tie = (int32_t*)mxCalloc((size_t)(n + 1), sizeof(int32_t));
    m->eop0 = (double*)mxCalloc((size_t)(6 * nimg + 1), sizeof(double));
    m->iop0 = (double*)mxCalloc((size_t)(cw * ncam + 1), sizeof(double));
    m->caminfo = (double*)mxCalloc((size_t)(5 * ncam + 1), sizeof(double));
    m->tie0 = (double*)mxCalloc((size_t)(3 * ntie + 1), sizeof(double));
    for (int k = 0; k < ncam; ++k) m->caminfo[5 * k] = 1.0;
    static const char* eopf[6] = {"Xc", "Yc", "Zc", "w", "p", "k"};
    static const char* camf[5] = {"y_dir", "xmin", "ymin", "xmax", "ymax"};
    for (int64_t i = 0; i < n; ++i) {
        const mwIndex q = (mwIndex)i;
        const int e = (int)fm_num(pts, q, "ext_index", 0, NULL) - 1;
        const int k = (int)fm_num(pts, q, "cam_num", 0, NULL) - 1;
        const int t = (int)fm_num(pts, q, "tieIndex", -1, NULL);
        if (e < 0 || e >= nimg || k < 0 || k >= ncam || t == 0 || t > ntie) {
            snprintf(msg, nmsg, "data.points(%ld): ext_index / cam_num / tieIndex out of range", (long)i + 1);
            return 1;
        }
        m->xy[2 * i] = fm_num(pts, q, "x", 0, NULL);
        m->xy[2 * i + 1] = fm_num(pts, q, "y", 0, NULL);
        m->img[i] = e;
        m->cam[i] = k;
        m->tie[i] = t > 0 ? t - 1 : -1;
        m->xyz[3 * i] = fm_num(pts, q, "X", 0, NULL);
        m->xyz[3 * i + 1] = fm_num(pts, q, "Y", 0, NULL);
        m->xyz[3 * i + 2] = fm_num(pts, q, "Z", 0, NULL);
        for (int a = 0; a < 6; ++a) m->eop0[6 * e + a] = fm_num(pts, q, eopf[a], 0, NULL);
        double* io = m->iop0 + (int64_t)cw * k;
        io[0] = fm_num(pts, q, "xp", 0, NULL);
        io[1] = fm_num(pts, q, "yp", 0, NULL);
        io[2] = fm_num(pts, q, "c", 0, NULL);
        const mxArray* K = mxGetField(pts, q, "K");
        const mxArray* P = mxGetField(pts, q, "P");
        const size_t nK = K ? mxGetNumberOfElements(K) : 0, nP = P ? mxGetNumberOfElements(P) : 0;
        for (int j = 0; j < nk; ++j) io[3 + j] = (j < (int)nK && mxIsDouble(K)) ? mxGetDoubles(K)[j] : 0.0;
        for (int j = 0; j < 2; ++j) io[3 + nk + j] = (j < (int)nP && mxIsDouble(P)) ? mxGetDoubles(P)[j] : 0.0;
        for (int a = 0; a < 5; ++a) m->caminfo[5 * k + a] = fm_num(pts, q, camf[a], a == 0 ? 1.0 : 0.0, NULL);
        if (t > 0)
            for (int a = 0; a < 3; ++a) m->tie0[3 * (t - 1) + a] = m->xyz[3 * i + a];
    }
    fba_problem* p = &m->p;
    memset(p, 0, sizeof *p);
    p->n_pts = n;
    p->n_img = nimg;
    p->n_cam = ncam;
    p->n_tie = ntie;
    p->xy = m->xy;
    p->img = m->img;
    p->cam = m->cam;
    p->tie = m->tie;
    p->xyz_fixed = m->xyz;
    p->eop0 = m->eop0;
    p->iop0 = m->iop0;
    p->cam_info = m->caminfo;
    p->tie0 = m->tie0;
    return 0;
}

/* cell (r, c) of an M x N cell array (1-based as in MATLAB) */
static inline const mxArray* fm_cell_at(const mxArray* C, mwIndex r, mwIndex c) {
    const mwSize M = mxGetM(C);
    if (r < 1 || c < 1 || r > M || c > mxGetN(C)) return NULL;
    return mxGetCell(C, (c - 1) * M + (r - 1));
}
static inline double fm_cell_num(const mxArray* C, mwIndex r, mwIndex c) {
    const mxArray* v = fm_cell_at(C, r, c);
    return (v && mxGetNumberOfElements(v) > 0) ? mxGetScalar(v) : 0.0;
}
static inline char* fm_cell_str(const mxArray* C, mwIndex r, mwIndex c) {
    const mxArray* v = fm_cell_at(C, r, c);
    return (v && mxIsChar(v)) ? mxArrayToString(v) : NULL;
}

/* Buildxhat.m:22-131's start values from main.m's EXT / INT / TIE / CNT (EXT angles in radians,
 * main.m:215-217) over the packed problem's eop0 / iop0 / tie0.  TIE may be a cellstr or ReadFiles'
 * string array (*tie_cells receives the converted copy, to destroy); *tie_out the cellstr used.
 * nk_ref: Num_Radial_Distortions as given (0: INT row 2 is xp yp c P1 P2, Buildxhat.m:71-72).
 * Returns 0, or 1 with the reference's message (a TIE target not in CNT, Buildxhat.m:124-128). */
static inline int fm_start_values(mex_problem* m, const mxArray* EXT, const mxArray* INT, const mxArray* TIE,
                           const mxArray* CNT, int nk_ref, const mxArray** tie_out, mxArray** tie_cells,
                           char* msg, size_t nmsg) {
    *tie_cells = NULL;
    if (TIE && mxIsClass(TIE, "string")) {  /* ReadFiles' string array -> cellstr */
        mxArray* in[1] = {(mxArray*)TIE};
        if (mexCallMATLAB(1, tie_cells, 1, in, "cellstr") == 0) TIE = *tie_cells;
    }
    *tie_out = TIE;
    const int nimg = m->p.n_img, ncam = m->p.n_cam, nk = m->s.num_radial, cw = 5 + nk;
    const int ntie = (TIE && mxIsCell(TIE)) ? (int)mxGetNumberOfElements(TIE) : 0;
    if (ntie != m->p.n_tie || (TIE && !mxIsCell(TIE))) {
        snprintf(msg, nmsg, "TIE has %d entries, data.numtie = %d", ntie, m->p.n_tie);
        return 1;
    }
    for (int i = 1; i <= nimg; ++i)
        for (int a = 0; a < 6; ++a) m->eop0[6 * (i - 1) + a] = fm_cell_num(EXT, i, 3 + a);
    for (int k = 1; k <= ncam; ++k)  /* INT row 2: xp yp c K1..K_nk_ref P1 P2 */
        for (int a = 0; a < cw; ++a) {
            const int col = (a < 3 + nk_ref) ? a : (a < 3 + nk ? -1 : a - nk + nk_ref);
            m->iop0[cw * (k - 1) + a] = col < 0 ? 0.0 : fm_cell_num(INT, 2 * k, 1 + col);
        }
    for (int t = 0; t < ntie; ++t) {
        char* id = mxIsChar(mxGetCell(TIE, t)) ? mxArrayToString(mxGetCell(TIE, t)) : NULL;
        int found = 0;
        for (mwIndex j = 1; id && j <= mxGetM(CNT) && !found; ++j) {
            char* cid = fm_cell_str(CNT, j, 1);
            if (cid && strcmp(cid, id) == 0) {
                for (int a = 0; a < 3; ++a) m->tie0[3 * t + a] = fm_cell_num(CNT, j, 2 + a);
                found = 1;
            }
            if (cid) mxFree(cid);
        }
        if (!found) snprintf(msg, nmsg, "Error Buildxhat(): can't find %s from .tie in .cnt", id ? id : "?");
        if (id) mxFree(id);
        if (!found) return 1;
    }
    return 0;
}

/* ---- one cached context (the problem and settings hashed) ---- */
static fba_ctx* g_fm_ctx = NULL;
static uint64_t g_fm_key = 0;

static inline void fm_release(void) {
    if (g_fm_ctx) fba_destroy(g_fm_ctx);
    g_fm_ctx = NULL;
    g_fm_key = 0;
}

static inline uint64_t fm_hash(uint64_t h, const void* d, size_t n) {
    const unsigned char* b = (const unsigned char*)d;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

static inline uint64_t fm_key(const mex_problem* m) {
    const fba_problem* p = &m->p;
    const int cw = 5 + (m->s.num_radial < 1 ? 1 : m->s.num_radial);
    uint64_t h = 1469598103934665603ull;
    h = fm_hash(h, &m->s, sizeof m->s);
    h = fm_hash(h, &p->n_pts, sizeof p->n_pts);
    h = fm_hash(h, &p->n_img, 3 * sizeof(int32_t));
    h = fm_hash(h, m->xy, sizeof(double) * 2 * (size_t)p->n_pts);
    h = fm_hash(h, m->img, sizeof(int32_t) * (size_t)p->n_pts);
    h = fm_hash(h, m->cam, sizeof(int32_t) * (size_t)p->n_pts);
    h = fm_hash(h, m->tie, sizeof(int32_t) * (size_t)p->n_pts);
    h = fm_hash(h, m->xyz, sizeof(double) * 3 * (size_t)p->n_pts);
    h = fm_hash(h, m->eop0, sizeof(double) * 6 * (size_t)p->n_img);
    h = fm_hash(h, m->iop0, sizeof(double) * (size_t)cw * p->n_cam);
    h = fm_hash(h, m->caminfo, sizeof(double) * 5 * (size_t)p->n_cam);
    h = fm_hash(h, m->tie0, sizeof(double) * 3 * (size_t)p->n_tie);
    return h | 1ull;
}

/* the cached context for this problem (created on first use); NULL with fba_last_error() set */
static inline fba_ctx* fm_context(const mex_problem* m) {
    const uint64_t key = fm_key(m);
    if (g_fm_ctx && key == g_fm_key) return g_fm_ctx;
    fm_release();
    fba_options o;
    memset(&o, 0, sizeof o);
    o.world = 1;
    if (fba_create(&m->p, &m->s, &o, &g_fm_ctx) != 0) {
        g_fm_ctx = NULL;
        return NULL;
    }
    g_fm_key = key;
    mexAtExit(fm_release);
    return g_fm_ctx;
}

#endif /* FBA_MEX_COMMON_H_ */
