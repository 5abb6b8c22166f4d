/*
 * fba_cpu.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A C/OpenMP restatement of the reference's Gauss-Newton inner loop at scene sizes the dense
 * NumPy oracle (oracle/fba_oracle.py) cannot reach.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it (through oracle/fba_cpu.py); the product never does.
 *
 * What it restates (reference = wynandtredoux/Fish-Eye_Bundle_Adjustment, read as text):
 *   functions/BuildAwG.m:50-158   parameter gather from xhat (estimated) or the fixed tables
 *   functions/BuildAwG.m:160-503  forward model and Jacobian rows (chain rule of the same model;
 *                                 pinned against the reference's expression text by
 *                                 tests/golden/jac_golden.json via the NumPy oracle)
 *   functions/BuildAwG.m:419-451  radial / decentering columns scaled by rmax^(2j), rmax^2
 *   functions/BuildAwG.m:505-527  misclosure w = f - obs, inner-constraint G
 *   main.m:424-444                u = A'Pw, N = A'PA and the (bordered) solve -- here in its
 *                                 block-sparse form: the 3x3 tie-point blocks of N are eliminated
 *                                 per point (reduced camera system S, right-hand side r), the
 *                                 dense solve of S (with the border) is left to the caller
 *   main.m:460-488                de-scaling, xhat += delta, deltasum = sumabs(delta)
 *   main.m:569, :601              v = A*delta + w (last linearisation, de-scaled delta), v'Pv
 *
 * Layout: the reference's xhat (Buildxhat.m): [u_img per image] [u_cam per camera] [3 per tie].
 * The reduced system covers the first u_c = u_img*n_img + u_cam*n_cam unknowns, row-major dense.
 * Indices are 0-based (the reference's are 1-based).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NKMAX 8
#define CWMAX (5 + NKMAX)
#define NF (6 + CWMAX + 3)

typedef struct fbo_input {
    int64_t n_pts;
    int32_t n_img, n_cam, n_tie, nk; /* nk = Num_Radial_Distortions (>= 1)               */
    int32_t type;                   /* 0 fisheye 1 pinhole 2 equisolid 3 ortho 4 stereo  */
    int32_t est[11];                /* Xc Yc Zc omega phi kappa xp yp c radial decent    */
    int32_t ic;                     /* Inner_Constraints                                 */
    int32_t reserved;
    double sx, sy;                  /* Meas_std, Meas_std_y                              */
    const double* x;                /* [n_pts]                                           */
    const double* y;                /* [n_pts]                                           */
    const int64_t* img;             /* [n_pts] ext_index                                 */
    const int64_t* cam;             /* [n_pts] cam_num                                   */
    const int64_t* tie;             /* [n_pts] tie index or -1                           */
    const double* eop;              /* [n_pts*6] fixed EOP per point (main.m:285-300)    */
    const double* iop;              /* [n_pts*(5+nk)] fixed IOP per point                */
    const double* bounds;           /* [n_pts*5] y_dir xmin ymin xmax ymax               */
    const double* xyz;              /* [n_pts*3] CNT coordinates                         */
} fbo_input;

typedef struct fbo_ctx {
    fbo_input in;
    int u_img, u_cam, cw;           /* cw = full camera width 5+nk                         */
    int emap[6], cmap[CWMAX];       /* full -> compressed index (or -1)                    */
    int64_t u_c, u;
    double px, py;
    /* CSR of observations per image and per tie point */
    int64_t *img_ptr, *img_obs, *tie_ptr, *tie_obs;
    double* rmax;                   /* [n_cam]                                             */
    /* last linearisation */
    double* J;                      /* [n_pts][2][NF] full-width rows                      */
    double* w;                      /* [n_pts][2]                                          */
    double* Wc;                     /* [n_pts][6][3]   Je' P Jp (compressed image rows)    */
    double* Qc;                     /* [n_pts][CWMAX][3] Jc' P Jp (compressed camera rows) */
    double* Vinv;                   /* [n_tie][9]                                          */
    double* bp;                     /* [n_tie][3]                                          */
    double* delta;                  /* [u] last de-scaled correction                       */
    uint8_t* owned;                 /* [n_pts] observation shard mask (NULL = all)         */
    int count_cam;                  /* this shard's deltasum includes the camera unknowns  */
    int nthreads;
    struct fbo_sparse* sparse;      /* block-sparse form of the reduced system (fbo_sparse_setup) or NULL */
    int sparse_on;                  /* fbo_reduce writes into it instead of the dense S                */
} fbo_ctx;
static void sparse_free(struct fbo_sparse* sp);

#define SB 128                /* block size (the GPU's NB)               */
#define SBB (SB * SB)
#define NRHS 15               /* -r | A (7) | B (7)                      */

typedef struct fbo_sparse {
    int64_t n_pad;            /* padded order (multiple of SB)           */
    int nb, n_loc, n_slots;
    int64_t* pos;             /* [u_c] compressed index -> position      */
    int32_t* slot_of;         /* [n_img] EXT row -> slot                 */
    int32_t* boff;            /* [nb * nb] block (i, j), i >= j -> index in pool, -1 outside the pattern */
    int nblk;
    double* pool;             /* nblk blocks, column-major SB x SB       */
    int32_t *cptr, *crow;     /* rows(k) > k of L's pattern, ascending   */
    int nlev;
    int32_t *lptr, *lcol;     /* columns per level                       */
    int32_t *pptr, *pblk;     /* per level: panel blocks (i, k) as pairs */
    int32_t *tptr, *tgt;      /* per level: update targets (i, j) pairs  */
    int32_t *sptr, *src;      /* per target: its source columns k, ascending */
    double* rhs;              /* n_pad x NRHS column-major               */
    double* Sc;               /* camera block partials (thread-private)  */
} fbo_sparse;

static inline double* sblk(const fbo_sparse* sp, int64_t pi, int64_t pj) {  /* entry (pi, pj), pi >= pj */
    const int32_t b = sp->boff[(pi / SB) * sp->nb + pj / SB];
    return b < 0 ? NULL : sp->pool + (int64_t)b * SBB + (pj % SB) * SB + pi % SB;
}


/* ---------------------------------------------------------------------------------------------
 * forward model, BuildAwG.m:160-212
 * ------------------------------------------------------------------------------------------- */
static void rot(double w, double p, double k, double M[9], double Mw[9], double Mp[9], double Mk[9]) {
    double cw = cos(w), sw = sin(w), cp = cos(p), sp = sin(p), ck = cos(k), sk = sin(k);
    double m[9] = {ck * cp, cw * sk + ck * sp * sw, sk * sw - ck * cw * sp,
                   -cp * sk, ck * cw - sk * sp * sw, ck * sw + cw * sk * sp,
                   sp, -cp * sw, cp * cw};
    double mw[9] = {0, -sw * sk + ck * sp * cw, sk * cw + ck * sw * sp,
                    0, -ck * sw - sk * sp * cw, ck * cw - sw * sk * sp,
                    0, -cp * cw, -cp * sw};
    double mp[9] = {-ck * sp, ck * cp * sw, -ck * cw * cp,
                    sp * sk, -sk * cp * sw, cw * sk * cp,
                    cp, sp * sw, -sp * cw};
    double mk[9] = {-sk * cp, cw * ck - sk * sp * sw, ck * sw + sk * cw * sp,
                    -cp * ck, -sk * cw - ck * sp * sw, -sk * sw + cw * ck * sp,
                    0, 0, 0};
    memcpy(M, m, sizeof m);
    memcpy(Mw, mw, sizeof mw);
    memcpy(Mp, mp, sizeof mp);
    memcpy(Mk, mk, sizeof mk);
}

/* s(R,W) with f = -c*(U, ydir*V)*s, BuildAwG.m:184-208 */
static void radial(int type, double R, double W, double* s, double* sR, double* sW) {
    if (type == 1) {
        *s = 1.0 / W;
        *sR = 0.0;
        *sW = -1.0 / (W * W);
        return;
    }
    double t = atan(R / W), q = R * R + W * W, tR = W / q, tW = -R / q, g, gt;
    switch (type) {
    case 0: g = t; gt = 1.0; break;
    case 2: g = 2.0 * sin(0.5 * t); gt = cos(0.5 * t); break;
    case 3: g = sin(t); gt = cos(t); break;
    default: { double c = cos(0.5 * t); g = 2.0 * tan(0.5 * t); gt = 1.0 / (c * c); } break;
    }
    *s = g / R;
    *sR = gt * tR / R - g / (R * R);
    *sW = gt * tW / R;
}

/* One image point: full-width Jacobian rows J[2][NF] and misclosure w[2] at xhat. */
static void linearize(const fbo_ctx* c, const double* xhat, int64_t o, double* J, double* w) {
    const fbo_input* in = &c->in;
    const int nk = in->nk, cw = c->cw;
    const int64_t e = in->img[o], k = in->cam[o], t = in->tie[o];
    double eop[6], iop[CWMAX], X[3];
    for (int j = 0; j < 6; ++j)
        eop[j] = c->emap[j] >= 0 ? xhat[e * c->u_img + c->emap[j]] : in->eop[o * 6 + j];
    const int64_t cb = (int64_t)c->u_img * in->n_img + k * c->u_cam;
    for (int j = 0; j < cw; ++j)
        iop[j] = c->cmap[j] >= 0 ? xhat[cb + c->cmap[j]] : in->iop[o * (5 + nk) + j];
    for (int j = 0; j < 3; ++j)
        X[j] = t >= 0 ? xhat[c->u_c + 3 * t + j] : in->xyz[o * 3 + j];
    const double xp = iop[0], yp = iop[1], cc = iop[2], P1 = iop[3 + nk], P2 = iop[4 + nk];
    const double ydir = in->bounds[o * 5];
    double M[9], Mw[9], Mp[9], Mk[9];
    rot(eop[3], eop[4], eop[5], M, Mw, Mp, Mk);
    const double d[3] = {X[0] - eop[0], X[1] - eop[1], X[2] - eop[2]};
    const double U = M[0] * d[0] + M[1] * d[1] + M[2] * d[2];
    const double V = M[3] * d[0] + M[4] * d[1] + M[5] * d[2];
    const double W = M[6] * d[0] + M[7] * d[1] + M[8] * d[2];
    const double R = sqrt(U * U + V * V);
    double s, sR, sW;
    radial(in->type, R, W, &s, &sR, &sW);
    const double x = in->x[o], y = in->y[o];
    const double xb = x - xp, yb = y - yp, r = sqrt(xb * xb + yb * yb);
    double dr = 0.0;
    for (int j = 1; j <= nk; ++j) dr += iop[2 + j] * pow(r, 2.0 * j);
    const double decx = P1 * (yb * yb + 3 * xb * xb) + 2 * P2 * xb * yb;
    const double decy = P2 * (xb * xb + 3 * yb * yb) + 2 * P1 * xb * yb;
    w[0] = (-cc * U * s + xp + dr * xb + decx) - x;
    w[1] = (-cc * ydir * V * s + yp + dr * yb + decy) - y;

    memset(J, 0, sizeof(double) * 2 * NF);
    double* Jx = J;
    double* Jy = J + NF;
    /* chain rule through (U,V,W): d(fx,fy)/dq for dq = d(U,V,W)/dq */
#define CHAIN(dU, dV, dW, ox, oy)                                       \
    do {                                                                \
        double dR_ = (U * (dU) + V * (dV)) / R;                         \
        double ds_ = (in->type == 1 ? 0.0 : sR * dR_) + sW * (dW);      \
        ox = -cc * ((dU) * s + U * ds_);                                \
        oy = -cc * ydir * ((dV) * s + V * ds_);                         \
    } while (0)
    for (int j = 0; j < 3; ++j) CHAIN(-M[j], -M[3 + j], -M[6 + j], Jx[j], Jy[j]);
    const double* Ms[3] = {Mw, Mp, Mk};
    for (int a = 0; a < 3; ++a) {
        const double* m = Ms[a];
        double dU = m[0] * d[0] + m[1] * d[1] + m[2] * d[2];
        double dV = m[3] * d[0] + m[4] * d[1] + m[5] * d[2];
        double dW = m[6] * d[0] + m[7] * d[1] + m[8] * d[2];
        CHAIN(dU, dV, dW, Jx[3 + a], Jy[3 + a]);
    }
    for (int j = 0; j < 3; ++j) CHAIN(M[j], M[3 + j], M[6 + j], Jx[6 + cw + j], Jy[6 + cw + j]);
#undef CHAIN
    /* xp, yp (BuildAwG.m:373-398), c (:400-414) */
    double dxp = 0, dyp = 0, dxp2 = 0, dyp2 = 0;
    for (int j = 1; j <= nk; ++j) {
        double Kj = iop[2 + j], r2j = pow(r, 2.0 * j), r2jm2 = pow(r, 2.0 * (j - 1));
        dxp += -Kj * r2j - 2 * j * Kj * xb * xb * r2jm2;
        dyp += -2 * j * Kj * xb * yb * r2jm2;
        dxp2 += -2 * j * Kj * xb * yb * r2jm2;
        dyp2 += -Kj * r2j - 2 * j * Kj * yb * yb * r2jm2;
    }
    Jx[6] = 1 + dxp - 6 * P1 * xb - 2 * P2 * yb;
    Jy[6] = dyp - 2 * P1 * yb - 2 * P2 * xb;
    Jx[7] = dxp2 - 2 * P2 * xb - 2 * P1 * yb;
    Jy[7] = 1 + dyp2 - 6 * P2 * yb - 2 * P1 * xb;
    Jx[8] = -U * s;
    Jy[8] = -ydir * V * s;
    /* scaled distortion columns (BuildAwG.m:419-451) */
    const double rm = c->rmax[k];
    for (int j = 1; j <= nk; ++j) {
        double sc = pow(rm, 2.0 * j), r2j = pow(r, 2.0 * j);
        Jx[8 + j] = r2j * xb / sc;
        Jy[8 + j] = r2j * yb / sc;
    }
    const double sc2 = pow(rm, 2.0);
    Jx[9 + nk] = (yb * yb + 3 * xb * xb) / sc2;
    Jx[10 + nk] = (2 * xb * yb) / sc2;
    Jy[9 + nk] = (2 * xb * yb) / sc2;
    Jy[10 + nk] = (xb * xb + 3 * yb * yb) / sc2;
}

static void inv3(const double A[9], double B[9]) {
    double c0 = A[4] * A[8] - A[5] * A[7], c1 = A[5] * A[6] - A[3] * A[8], c2 = A[3] * A[7] - A[4] * A[6];
    double det = A[0] * c0 + A[1] * c1 + A[2] * c2, id = 1.0 / det;
    B[0] = c0 * id;
    B[1] = (A[2] * A[7] - A[1] * A[8]) * id;
    B[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    B[3] = c1 * id;
    B[4] = (A[0] * A[8] - A[2] * A[6]) * id;
    B[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    B[6] = c2 * id;
    B[7] = (A[1] * A[6] - A[0] * A[7]) * id;
    B[8] = (A[0] * A[4] - A[1] * A[3]) * id;
}

/* ---------------------------------------------------------------------------------------------
 * context
 * ------------------------------------------------------------------------------------------- */
static int64_t* csr(int64_t n_keys, int64_t n, const int64_t* key, int64_t** items) {
    int64_t* ptr = calloc(n_keys + 1, sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i)
        if (key[i] >= 0) ptr[key[i] + 1]++;
    for (int64_t k = 0; k < n_keys; ++k) ptr[k + 1] += ptr[k];
    int64_t* fill = malloc((n_keys + 1) * sizeof(int64_t));
    memcpy(fill, ptr, (n_keys + 1) * sizeof(int64_t));
    *items = malloc((ptr[n_keys] + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < n; ++i)
        if (key[i] >= 0) (*items)[fill[key[i]]++] = i;
    free(fill);
    return ptr;
}

int fbo_abi(void) { return 1; }

/* returns NULL on invalid input (nk out of range, IC without all six EOPs) */
fbo_ctx* fbo_create(const fbo_input* in, int nthreads) {
    if (in->nk < 1 || in->nk > NKMAX || in->type < 0 || in->type > 4) return NULL;
    fbo_ctx* c = calloc(1, sizeof(fbo_ctx));
    c->in = *in;
    c->cw = 5 + in->nk;
    c->nthreads = nthreads > 0 ? nthreads : 1;
    int n = 0;
    for (int j = 0; j < 6; ++j) c->emap[j] = in->est[j] ? n++ : -1;
    c->u_img = n;
    if (in->ic && n != 6) { free(c); return NULL; }
    n = 0;
    for (int j = 0; j < 3; ++j) c->cmap[j] = in->est[6 + j] ? n++ : -1;
    for (int j = 0; j < in->nk; ++j) c->cmap[3 + j] = in->est[9] ? n++ : -1;
    for (int j = 0; j < 2; ++j) c->cmap[3 + in->nk + j] = in->est[10] ? n++ : -1;
    c->u_cam = n;
    c->u_c = (int64_t)c->u_img * in->n_img + (int64_t)c->u_cam * in->n_cam;
    c->u = c->u_c + 3 * (int64_t)in->n_tie;
    c->px = 1.0 / (in->sx * in->sx);
    c->py = 1.0 / (in->sy * in->sy);
    c->img_ptr = csr(in->n_img, in->n_pts, in->img, &c->img_obs);
    c->tie_ptr = csr(in->n_tie, in->n_pts, in->tie, &c->tie_obs);
    c->rmax = calloc(in->n_cam, sizeof(double));
    for (int64_t o = 0; o < in->n_pts; ++o) {
        const double* b = in->bounds + 5 * o;
        double hx = (b[3] - b[1]) * 0.5, hy = (b[4] - b[2]) * 0.5;
        c->rmax[in->cam[o]] = sqrt(hx * hx + hy * hy);
    }
    c->J = malloc(sizeof(double) * 2 * NF * in->n_pts);
    c->w = malloc(sizeof(double) * 2 * in->n_pts);
    c->Wc = calloc((size_t)18 * in->n_pts, sizeof(double));
    c->Qc = calloc((size_t)3 * CWMAX * in->n_pts, sizeof(double));
    c->Vinv = calloc((size_t)9 * (in->n_tie + 1), sizeof(double));
    c->bp = calloc((size_t)3 * (in->n_tie + 1), sizeof(double));
    c->delta = calloc(c->u + 1, sizeof(double));
    c->count_cam = 1;
    return c;
}

/*
 * Restrict the context to one rank's observation shard (main.m has no multi-rank form; this mirrors
 * fba_partition's split so the rank-summed reduced systems can be checked against the full one).
 * owned[o] != 0 for this rank's observations (whole tie points + its share of control points).
 * count_cam: whether fbo_update's deltasum includes the replicated camera-side unknowns.
 */
void fbo_set_shard(fbo_ctx* c, const uint8_t* owned, int count_cam) {
    free(c->owned);
    c->owned = NULL;
    if (owned) {
        c->owned = malloc(c->in.n_pts);
        memcpy(c->owned, owned, c->in.n_pts);
    }
    c->count_cam = count_cam;
}
#define OWNED(c, o) (!(c)->owned || (c)->owned[o])

void fbo_destroy(fbo_ctx* c) {
    if (!c) return;
    free(c->img_ptr); free(c->img_obs); free(c->tie_ptr); free(c->tie_obs); free(c->rmax);
    free(c->J); free(c->w); free(c->Wc); free(c->Qc); free(c->Vinv); free(c->bp); free(c->delta);
    free(c->owned);
    sparse_free(c->sparse);
    free(c);
}

void fbo_sizes(const fbo_ctx* c, int64_t* out /*[4]: u, u_c, u_img, u_cam*/) {
    out[0] = c->u;
    out[1] = c->u_c;
    out[2] = c->u_img;
    out[3] = c->u_cam;
}

/* compressed image / camera parts of one Jacobian row */
static inline void split_row(const fbo_ctx* c, const double* Jr, double* je, double* jc, double* jp) {
    for (int j = 0; j < 6; ++j)
        if (c->emap[j] >= 0) je[c->emap[j]] = Jr[j];
    for (int j = 0; j < c->cw; ++j)
        if (c->cmap[j] >= 0) jc[c->cmap[j]] = Jr[6 + j];
    for (int j = 0; j < 3; ++j) jp[j] = Jr[6 + c->cw + j];
}

/*
 * Linearise at xhat and form the point-reduced normal equations (main.m:424-425 + Schur):
 *   S = N_cc - N_cp V^-1 N_pc   (u_c x u_c, row-major, both triangles)
 *   r = u_c  - N_cp V^-1 u_p
 * so that S * delta_c = -r; G (u_c x 7, row-major, BuildAwG.m:514-527) when inner constraints are on.
 * Returns 0, or 1 if a tie point's 3x3 block is singular / non-finite.
 */
int fbo_reduce(fbo_ctx* c, const double* xhat, double* S, double* r, double* G) {
    const fbo_input* in = &c->in;
    const int ui = c->u_img, uc = c->u_cam;
    const int64_t n = in->n_pts, u_c = c->u_c, cam0 = (int64_t)ui * in->n_img;
    const double px = c->px, py = c->py;
    int bad = 0;
#pragma omp parallel for schedule(static) num_threads(c->nthreads)
    for (int64_t o = 0; o < n; ++o) linearize(c, xhat, o, c->J + 2 * NF * o, c->w + 2 * o);

    /* per tie point: V, b, V^-1 and per observation W_i = Je' P Jp, Q_i = Jc' P Jp */
#pragma omp parallel for schedule(dynamic, 64) num_threads(c->nthreads) reduction(| : bad)
    for (int64_t p = 0; p < in->n_tie; ++p) {
        double V[9] = {0}, b[3] = {0};
        if (c->tie_ptr[p] == c->tie_ptr[p + 1] || !OWNED(c, c->tie_obs[c->tie_ptr[p]])) {
            memset(c->Vinv + 9 * p, 0, 9 * sizeof(double));
            memset(c->bp + 3 * p, 0, 3 * sizeof(double));
            continue;
        }
        for (int64_t q = c->tie_ptr[p]; q < c->tie_ptr[p + 1]; ++q) {
            int64_t o = c->tie_obs[q];
            double je[2][6] = {{0}}, jc[2][CWMAX] = {{0}}, jp[2][3];
            split_row(c, c->J + 2 * NF * o, je[0], jc[0], jp[0]);
            split_row(c, c->J + 2 * NF * o + NF, je[1], jc[1], jp[1]);
            const double* wo = c->w + 2 * o;
            for (int a = 0; a < 3; ++a) {
                for (int bb = 0; bb < 3; ++bb) V[a * 3 + bb] += px * jp[0][a] * jp[0][bb] + py * jp[1][a] * jp[1][bb];
                b[a] += px * jp[0][a] * wo[0] + py * jp[1][a] * wo[1];
            }
            double* Wi = c->Wc + 18 * o;
            double* Qi = c->Qc + 3 * CWMAX * o;
            for (int a = 0; a < ui; ++a)
                for (int k = 0; k < 3; ++k) Wi[a * 3 + k] = px * je[0][a] * jp[0][k] + py * je[1][a] * jp[1][k];
            for (int a = 0; a < uc; ++a)
                for (int k = 0; k < 3; ++k) Qi[a * 3 + k] = px * jc[0][a] * jp[0][k] + py * jc[1][a] * jp[1][k];
        }
        inv3(V, c->Vinv + 9 * p);
        for (int a = 0; a < 9; ++a)
            if (!isfinite(c->Vinv[9 * p + a])) bad |= 1;
        memcpy(c->bp + 3 * p, b, sizeof b);
    }
    if (bad) return 1;

    /* sparse (fbo_sparse_solve's form): S's lower pattern blocks in the permuted order, no dense array;
     * image-image entries written by the row that is lower in that order, image-camera entries
     * (camera rows come last) into the camera rows by the image's thread */
    fbo_sparse* sp = c->sparse_on ? c->sparse : NULL;
#define SADD_L(i, j, v)                                                             \
    do {                                                                            \
        if (!sp) S[(i) * u_c + (j)] += (v);                                         \
        else {                                                                      \
            const int64_t pi_ = sp->pos[i], pj_ = sp->pos[j];                       \
            if (pi_ >= pj_) *sblk(sp, pi_, pj_) += (v);                             \
        }                                                                           \
    } while (0)
#define SADD_T(i, j, v)                                                             \
    do {                                                                            \
        if (!sp) S[(i) * u_c + (j)] += (v);                                         \
        else *sblk(sp, sp->pos[j], sp->pos[i]) += (v);                              \
    } while (0)
    if (sp) memset(sp->pool, 0, sizeof(double) * SBB * (size_t)sp->nblk);
    else memset(S, 0, sizeof(double) * u_c * u_c);
    memset(r, 0, sizeof(double) * u_c);
    /* image row blocks: direct terms + Schur terms of every point the image sees */
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads)
    for (int64_t e = 0; e < in->n_img; ++e) {
        const int64_t re = e * ui;
        for (int64_t q = c->img_ptr[e]; q < c->img_ptr[e + 1]; ++q) {
            const int64_t o = c->img_obs[q], kc = cam0 + in->cam[o] * uc, t = in->tie[o];
            if (!OWNED(c, o)) continue;
            double je[2][6] = {{0}}, jc[2][CWMAX] = {{0}}, jp[2][3];
            split_row(c, c->J + 2 * NF * o, je[0], jc[0], jp[0]);
            split_row(c, c->J + 2 * NF * o + NF, je[1], jc[1], jp[1]);
            const double* wo = c->w + 2 * o;
            for (int a = 0; a < ui; ++a) {
                for (int bb = 0; bb < ui; ++bb) SADD_L(re + a, re + bb, px * je[0][a] * je[0][bb] + py * je[1][a] * je[1][bb]);
                for (int bb = 0; bb < uc; ++bb) SADD_T(re + a, kc + bb, px * je[0][a] * jc[0][bb] + py * je[1][a] * jc[1][bb]);
                r[re + a] += px * je[0][a] * wo[0] + py * je[1][a] * wo[1];
            }
            if (t < 0) continue;
            const double* Vi = c->Vinv + 9 * t;
            const double* Wi = c->Wc + 18 * o;
            double Y[6][3];
            for (int a = 0; a < ui; ++a)
                for (int k = 0; k < 3; ++k)
                    Y[a][k] = Wi[a * 3] * Vi[k] + Wi[a * 3 + 1] * Vi[3 + k] + Wi[a * 3 + 2] * Vi[6 + k];
            const double* bt = c->bp + 3 * t;
            for (int a = 0; a < ui; ++a) r[re + a] -= Y[a][0] * bt[0] + Y[a][1] * bt[1] + Y[a][2] * bt[2];
            for (int64_t q2 = c->tie_ptr[t]; q2 < c->tie_ptr[t + 1]; ++q2) {
                const int64_t o2 = c->tie_obs[q2], e2 = in->img[o2] * ui, k2 = cam0 + in->cam[o2] * uc;
                const double* W2 = c->Wc + 18 * o2;
                const double* Q2 = c->Qc + 3 * CWMAX * o2;
                if (sp && ui > 0) {
                    /* sparse fast path: the image pair's entries are all lower or all upper; when neither
                     * image's positions straddle a block boundary they sit in one block, and so do the
                     * camera columns of this row image */
                    const int64_t pr = sp->pos[re], pc = sp->pos[e2], pk = sp->pos[k2];
                    const int fit_r = pr % SB + ui <= SB, fit_c = pc % SB + ui <= SB, fit_k = uc == 0 || pk % SB + uc <= SB;
                    if (fit_r && fit_c && fit_k && e2 != re) {
                        if (pr > pc) {
                            double* base = sblk(sp, pr, pc);
                            for (int bb = 0; bb < ui; ++bb)
                                for (int a = 0; a < ui; ++a)
                                    base[bb * SB + a] -= Y[a][0] * W2[bb * 3] + Y[a][1] * W2[bb * 3 + 1] + Y[a][2] * W2[bb * 3 + 2];
                        }
                        if (uc > 0) {
                            double* kb = sblk(sp, pk, pr);  /* (camera row, image column), column-major */
                            for (int a = 0; a < ui; ++a)
                                for (int bb = 0; bb < uc; ++bb)
                                    kb[a * SB + bb] -= Y[a][0] * Q2[bb * 3] + Y[a][1] * Q2[bb * 3 + 1] + Y[a][2] * Q2[bb * 3 + 2];
                        }
                        continue;
                    }
                }
                for (int a = 0; a < ui; ++a) {
                    for (int bb = 0; bb < ui; ++bb)
                        SADD_L(re + a, e2 + bb, -(Y[a][0] * W2[bb * 3] + Y[a][1] * W2[bb * 3 + 1] + Y[a][2] * W2[bb * 3 + 2]));
                    for (int bb = 0; bb < uc; ++bb)
                        SADD_T(re + a, k2 + bb, -(Y[a][0] * Q2[bb * 3] + Y[a][1] * Q2[bb * 3 + 1] + Y[a][2] * Q2[bb * 3 + 2]));
                }
            }
        }
    }

    /* camera row blocks: thread-private accumulation, reduced in thread order */
    const int64_t nc = (int64_t)uc * in->n_cam;
    if (nc > 0) {
        const int nt = c->nthreads;
        double* part = calloc((size_t)nt * (nc * nc + nc), sizeof(double));
#pragma omp parallel num_threads(nt)
        {
            int tid = 0;
#ifdef _OPENMP
            tid = omp_get_thread_num();
#endif
            double* Sc = part + (size_t)tid * (nc * nc + nc);
            double* rc = Sc + nc * nc;
#pragma omp for schedule(static)
            for (int64_t o = 0; o < n; ++o) {
                if (!OWNED(c, o)) continue;
                double je[2][6] = {{0}}, jc[2][CWMAX] = {{0}}, jp[2][3];
                split_row(c, c->J + 2 * NF * o, je[0], jc[0], jp[0]);
                split_row(c, c->J + 2 * NF * o + NF, je[1], jc[1], jp[1]);
                const double* wo = c->w + 2 * o;
                const int64_t kb = in->cam[o] * uc;
                for (int a = 0; a < uc; ++a) {
                    for (int bb = 0; bb < uc; ++bb)
                        Sc[(kb + a) * nc + kb + bb] += px * jc[0][a] * jc[0][bb] + py * jc[1][a] * jc[1][bb];
                    rc[kb + a] += px * jc[0][a] * wo[0] + py * jc[1][a] * wo[1];
                }
            }
#pragma omp for schedule(static)
            for (int64_t p = 0; p < in->n_tie; ++p) {
                if (c->tie_ptr[p] == c->tie_ptr[p + 1] || !OWNED(c, c->tie_obs[c->tie_ptr[p]])) continue;
                /* per camera sum of Q_i over this point's observations */
                int64_t cams[16];
                double Qs[16][CWMAX * 3];
                int ncams = 0;
                for (int64_t q = c->tie_ptr[p]; q < c->tie_ptr[p + 1]; ++q) {
                    int64_t o = c->tie_obs[q], k = in->cam[o];
                    int s_ = 0;
                    while (s_ < ncams && cams[s_] != k) ++s_;
                    if (s_ == ncams) {
                        if (ncams == 16) continue; /* > 16 cameras on one point: not exercised */
                        cams[ncams++] = k;
                        memset(Qs[s_], 0, sizeof Qs[s_]);
                    }
                    for (int a = 0; a < uc * 3; ++a) Qs[s_][a] += c->Qc[3 * CWMAX * o + a];
                }
                const double* Vi = c->Vinv + 9 * p;
                const double* bt = c->bp + 3 * p;
                for (int s1 = 0; s1 < ncams; ++s1) {
                    double Y[CWMAX][3];
                    for (int a = 0; a < uc; ++a)
                        for (int k = 0; k < 3; ++k)
                            Y[a][k] = Qs[s1][a * 3] * Vi[k] + Qs[s1][a * 3 + 1] * Vi[3 + k] + Qs[s1][a * 3 + 2] * Vi[6 + k];
                    const int64_t k1 = cams[s1] * uc;
                    for (int a = 0; a < uc; ++a) rc[k1 + a] -= Y[a][0] * bt[0] + Y[a][1] * bt[1] + Y[a][2] * bt[2];
                    for (int s2 = 0; s2 < ncams; ++s2) {
                        const int64_t k2 = cams[s2] * uc;
                        for (int a = 0; a < uc; ++a)
                            for (int bb = 0; bb < uc; ++bb)
                                Sc[(k1 + a) * nc + k2 + bb] -= Y[a][0] * Qs[s2][bb * 3] + Y[a][1] * Qs[s2][bb * 3 + 1] +
                                                               Y[a][2] * Qs[s2][bb * 3 + 2];
                    }
                }
            }
        }
        for (int t = 0; t < nt; ++t) {
            const double* Sc = part + (size_t)t * (nc * nc + nc);
            for (int64_t a = 0; a < nc; ++a) {
                for (int64_t bb = 0; bb < nc; ++bb) SADD_L(cam0 + a, cam0 + bb, Sc[a * nc + bb]);
                r[cam0 + a] += Sc[nc * nc + a];
            }
        }
        free(part);
        /* camera-image blocks are the transpose of the image-camera blocks (the sparse form has them) */
        if (!sp) {
#pragma omp parallel for schedule(static) num_threads(c->nthreads)
            for (int64_t a = 0; a < nc; ++a)
                for (int64_t bb = 0; bb < cam0; ++bb) S[(cam0 + a) * u_c + bb] = S[bb * u_c + cam0 + a];
        }
    }
#undef SADD_L
#undef SADD_T

    if (G) {
        memset(G, 0, sizeof(double) * u_c * 7);
        if (in->ic) {
            for (int64_t e = 0; e < in->n_img; ++e) {
                const double* x = xhat + e * 6;
                double Xc = x[0], Yc = x[1], Zc = x[2], w = x[3], p = x[4];
                double g[6][7] = {
                    {1, 0, 0, 0, -Zc, Yc, Xc},
                    {0, 1, 0, Zc, 0, -Xc, Yc},
                    {0, 0, 1, -Yc, Xc, 0, Zc},
                    {0, 0, 0, -1, -sin(w) * tan(p), cos(w) * tan(p), 0},
                    {0, 0, 0, 0, -cos(w), -sin(w), 0},
                    {0, 0, 0, 0, sin(w) / cos(p), -cos(w) / cos(p), 0}};
                memcpy(G + e * 6 * 7, g, sizeof g);
            }
        }
    }
    return 0;
}

/*
 * Back-substitute the tie points, de-scale, update (main.m:460-488).
 * dc: solution of S*dc = -r (u_c).  xhat updated in place; returns deltasum = sumabs(delta).
 */
double fbo_update(fbo_ctx* c, const double* dc, double* xhat) {
    const fbo_input* in = &c->in;
    const int ui = c->u_img, uc = c->u_cam, nk = in->nk;
    const int64_t u_c = c->u_c, cam0 = (int64_t)ui * in->n_img;
    double* d = c->delta;
    memcpy(d, dc, sizeof(double) * u_c);
#pragma omp parallel for schedule(dynamic, 64) num_threads(c->nthreads)
    for (int64_t p = 0; p < in->n_tie; ++p) {
        double t[3];
        if (c->tie_ptr[p] == c->tie_ptr[p + 1] || !OWNED(c, c->tie_obs[c->tie_ptr[p]])) {
            for (int j = 0; j < 3; ++j) d[u_c + 3 * p + j] = 0.0;
            continue;
        }
        memcpy(t, c->bp + 3 * p, sizeof t);
        for (int64_t q = c->tie_ptr[p]; q < c->tie_ptr[p + 1]; ++q) {
            const int64_t o = c->tie_obs[q], e = in->img[o] * ui, k = cam0 + in->cam[o] * uc;
            const double* Wi = c->Wc + 18 * o;
            const double* Qi = c->Qc + 3 * CWMAX * o;
            for (int a = 0; a < ui; ++a)
                for (int j = 0; j < 3; ++j) t[j] += Wi[a * 3 + j] * dc[e + a];
            for (int a = 0; a < uc; ++a)
                for (int j = 0; j < 3; ++j) t[j] += Qi[a * 3 + j] * dc[k + a];
        }
        const double* Vi = c->Vinv + 9 * p;
        for (int j = 0; j < 3; ++j) d[u_c + 3 * p + j] = -(Vi[3 * j] * t[0] + Vi[3 * j + 1] * t[1] + Vi[3 * j + 2] * t[2]);
    }
    /* de-scaling (main.m:460-482) */
    for (int64_t k = 0; k < in->n_cam; ++k) {
        const double rm = c->rmax[k];
        const int64_t kb = cam0 + k * uc;
        if (in->est[9])
            for (int j = 0; j < nk; ++j) d[kb + c->cmap[3 + j]] /= pow(rm, 2.0 * (j + 1));
        if (in->est[10])
            for (int j = 0; j < 2; ++j) d[kb + c->cmap[3 + nk + j]] /= pow(rm, 2.0);
    }
    double s = 0.0;
    for (int64_t i = 0; i < c->u; ++i) {
        xhat[i] += d[i];
        if (i >= u_c || c->count_cam) s += fabs(d[i]);
    }
    return s;
}

/* main.m:569 v = A*delta + w with the last A, w and de-scaled delta; returns v'Pv. v may be NULL. */
double fbo_residuals(const fbo_ctx* c, double* v) {
    const fbo_input* in = &c->in;
    const int ui = c->u_img, uc = c->u_cam;
    const int64_t cam0 = (int64_t)ui * in->n_img;
    double vtpv = 0.0;
#pragma omp parallel for schedule(static) num_threads(c->nthreads) reduction(+ : vtpv)
    for (int64_t o = 0; o < in->n_pts; ++o) {
        const int64_t e = in->img[o] * ui, k = cam0 + in->cam[o] * uc, t = in->tie[o];
        double vv[2];
        if (!OWNED(c, o)) {
            if (v) v[2 * o] = v[2 * o + 1] = 0.0;
            continue;
        }
        for (int rr = 0; rr < 2; ++rr) {
            double je[6] = {0}, jc[CWMAX] = {0}, jp[3];
            split_row(c, c->J + 2 * NF * o + rr * NF, je, jc, jp);
            double s = c->w[2 * o + rr];
            for (int a = 0; a < ui; ++a) s += je[a] * c->delta[e + a];
            for (int a = 0; a < uc; ++a) s += jc[a] * c->delta[k + a];
            if (t >= 0)
                for (int a = 0; a < 3; ++a) s += jp[a] * c->delta[c->u_c + 3 * t + a];
            vv[rr] = s;
        }
        if (v) {
            v[2 * o] = vv[0];
            v[2 * o + 1] = vv[1];
        }
        vtpv += c->px * vv[0] * vv[0] + c->py * vv[1] * vv[1];
    }
    return vtpv;
}

/* =============================================================================================
 * Block-sparse Cholesky of the reduced camera system (bench.py's cpu_baseline; also a third solver
 * the parity tests cross-check).  The reference inverts the dense bordered matrix (main.m:428-440);
 * here -- as on the GPU, on the SAME block pattern -- the reduced system's unknowns are permuted into
 * the device factorisation's camera-side order (fba_image_order: nested dissection of the image
 * co-visibility graph, padding slots, camera unknowns last), S is accumulated straight into its
 * 128 x 128 lower pattern blocks (no dense u_c x u_c array), the inner-constraint border is folded in
 * locally (M = S + A A', A = G_l W_l^1/2 on the first n_loc slots, B = G D; the 14 x 14 combine below
 * restores the exact bordered solution), and M is factored right-looking, one elimination-tree level
 * at a time: the level's diagonal blocks (dpotrf), its panel blocks (dtrsm), then every target block
 * of the level's updates (dsyrk / dgemm, a target's sources in order), each step an OpenMP loop over
 * independent blocks with single-threaded BLAS calls (the caller's OpenBLAS through scipy's function
 * pointers, fbo_set_blas).
 * ============================================================================================= */
typedef void (*dgemm_fn)(const char*, const char*, const int*, const int*, const int*, const double*, const double*,
                         const int*, const double*, const int*, const double*, double*, const int*);
typedef void (*dsyrk_fn)(const char*, const char*, const int*, const int*, const double*, const double*, const int*,
                         const double*, double*, const int*);
typedef void (*dtrsm_fn)(const char*, const char*, const char*, const char*, const int*, const int*, const double*,
                         const double*, const int*, double*, const int*);
typedef void (*dpotrf_fn)(const char*, const int*, double*, const int*, int*);
static dgemm_fn g_dgemm;
static dsyrk_fn g_dsyrk;
static dtrsm_fn g_dtrsm;
static dpotrf_fn g_dpotrf;

void fbo_set_blas(void* dgemm, void* dsyrk, void* dtrsm, void* dpotrf) {
    g_dgemm = (dgemm_fn)dgemm;
    g_dsyrk = (dsyrk_fn)dsyrk;
    g_dtrsm = (dtrsm_fn)dtrsm;
    g_dpotrf = (dpotrf_fn)dpotrf;
}

/* symbolic factorisation on the permuted block pattern; slots[n_slots]: EXT row per slot (-1 padding) */
int fbo_sparse_setup(fbo_ctx* c, const int32_t* slots, int n_slots) {
    const fbo_input* in = &c->in;
    fbo_sparse* sp = calloc(1, sizeof(fbo_sparse));
    const int ui = c->u_img, uc = c->u_cam;
    sp->n_slots = n_slots;
    const int64_t cam0p = 6 * (int64_t)n_slots;
    sp->n_pad = ((cam0p + (int64_t)uc * in->n_cam + SB - 1) / SB) * SB;
    if (sp->n_pad == 0) sp->n_pad = SB;
    const int nb = sp->nb = (int)(sp->n_pad / SB);
    sp->n_loc = in->ic ? (n_slots < SB / 6 ? n_slots : SB / 6) : 0;
    sp->slot_of = malloc(sizeof(int32_t) * (in->n_img + 1));
    for (int e = 0; e < in->n_img; ++e) sp->slot_of[e] = -1;
    for (int s = 0; s < n_slots; ++s)
        if (slots[s] >= 0 && slots[s] < in->n_img) sp->slot_of[slots[s]] = s;
    for (int e = 0; e < in->n_img; ++e)
        if (sp->slot_of[e] < 0) { free(sp->slot_of); free(sp); return 1; }
    sp->pos = malloc(sizeof(int64_t) * (c->u_c + 1));
    for (int64_t e = 0; e < in->n_img; ++e)
        for (int a = 0; a < ui; ++a) sp->pos[e * ui + a] = 6 * (int64_t)sp->slot_of[e] + a;
    for (int64_t k = 0; k < in->n_cam; ++k)
        for (int a = 0; a < uc; ++a) sp->pos[(int64_t)ui * in->n_img + k * uc + a] = cam0p + k * uc + a;
    /* the initial block pattern (lower): diagonal, co-visible image pairs, camera rows, local border */
    uint8_t* pat = calloc((size_t)nb * nb, 1);
    for (int b = 0; b < nb; ++b) pat[b * nb + b] = 1;
#define MARK(pi, pj) do { int64_t a_ = (pi) / SB, b_ = (pj) / SB; if (a_ < b_) { int64_t t_ = a_; a_ = b_; b_ = t_; } pat[a_ * nb + b_] = 1; } while (0)
    for (int64_t p = 0; p < in->n_tie; ++p)
        for (int64_t q1 = c->tie_ptr[p]; q1 < c->tie_ptr[p + 1]; ++q1)
            for (int64_t q2 = c->tie_ptr[p]; q2 < c->tie_ptr[p + 1]; ++q2) {
                const int64_t s1 = 6 * (int64_t)sp->slot_of[in->img[c->tie_obs[q1]]], s2 = 6 * (int64_t)sp->slot_of[in->img[c->tie_obs[q2]]];
                MARK(s1, s2); MARK(s1 + 5, s2); MARK(s1, s2 + 5); MARK(s1 + 5, s2 + 5);
            }
    for (int64_t e = 0; e < in->n_img; ++e) MARK(6 * (int64_t)sp->slot_of[e] + 5, 6 * (int64_t)sp->slot_of[e]);  /* own 6 x 6 */
    for (int64_t r = cam0p; r < cam0p + (int64_t)uc * in->n_cam; ++r)
        for (int b = 0; b <= r / SB; ++b) pat[(r / SB) * nb + b] = 1;  /* camera rows couple to every image */
    /* (the local border, positions < 6 n_loc <= 126, lies inside diagonal block 0) */
#undef MARK
    /* fill: for k ascending, every pair of rows below k's diagonal */
    int32_t* rows = malloc(sizeof(int32_t) * nb);
    for (int k = 0; k < nb; ++k) {
        int n = 0;
        for (int i = k + 1; i < nb; ++i)
            if (pat[i * nb + k]) rows[n++] = i;
        for (int x = 0; x < n; ++x)
            for (int y = 0; y <= x; ++y) pat[rows[x] * nb + rows[y]] = 1;
    }
    sp->boff = malloc(sizeof(int32_t) * nb * nb);
    sp->cptr = calloc(nb + 1, sizeof(int32_t));
    int nblk = 0, nrow = 0;
    for (int i = 0; i < nb; ++i)
        for (int j = 0; j < nb; ++j) sp->boff[i * nb + j] = (j <= i && pat[i * nb + j]) ? nblk++ : -1;
    for (int k = 0; k < nb; ++k)
        for (int i = k + 1; i < nb; ++i) nrow += pat[i * nb + k];
    sp->nblk = nblk;
    sp->crow = malloc(sizeof(int32_t) * (nrow + 1));
    for (int k = 0, q = 0; k < nb; ++k) {
        for (int i = k + 1; i < nb; ++i)
            if (pat[i * nb + k]) sp->crow[q++] = i;
        sp->cptr[k + 1] = q;
    }
    /* elimination-tree levels: a column's level is one above its children's highest */
    int32_t* lev = calloc(nb, sizeof(int32_t));
    int nlev = 0;
    for (int k = 0; k < nb; ++k) {
        if (sp->cptr[k + 1] > sp->cptr[k]) {
            const int par = sp->crow[sp->cptr[k]];
            if (lev[par] < lev[k] + 1) lev[par] = lev[k] + 1;
        }
        if (lev[k] + 1 > nlev) nlev = lev[k] + 1;
    }
    sp->nlev = nlev;
    sp->lptr = calloc(nlev + 1, sizeof(int32_t));
    sp->lcol = malloc(sizeof(int32_t) * nb);
    for (int k = 0; k < nb; ++k) sp->lptr[lev[k] + 1]++;
    for (int l = 0; l < nlev; ++l) sp->lptr[l + 1] += sp->lptr[l];
    {
        int32_t* fill = malloc(sizeof(int32_t) * (nlev + 1));
        memcpy(fill, sp->lptr, sizeof(int32_t) * (nlev + 1));
        for (int k = 0; k < nb; ++k) sp->lcol[fill[lev[k]]++] = k;
        free(fill);
    }
    /* per level: panel blocks (i, k) and update targets (i, j) with their sources */
    sp->pptr = calloc(nlev + 1, sizeof(int32_t));
    sp->pblk = malloc(sizeof(int32_t) * 2 * (nrow + 1));
    int np = 0;
    int64_t cap_t = 1024, nt = 0, cap_s = 4096, ns = 0;
    sp->tptr = calloc(nlev + 1, sizeof(int32_t));
    sp->tgt = malloc(sizeof(int32_t) * 2 * cap_t);
    sp->sptr = malloc(sizeof(int32_t) * (cap_t + 1));
    sp->src = malloc(sizeof(int32_t) * cap_s);
    sp->sptr[0] = 0;
    int32_t* tmark = malloc(sizeof(int32_t) * nb * nb);
    int64_t* tkeys = malloc(sizeof(int64_t) * ((int64_t)nb * nb + 1));
    for (int64_t q = 0; q < (int64_t)nb * nb; ++q) tmark[q] = -1;
    for (int l = 0; l < nlev; ++l) {
        int64_t nk = 0;
        for (int x = sp->lptr[l]; x < sp->lptr[l + 1]; ++x) {
            const int k = sp->lcol[x];
            for (int q = sp->cptr[k]; q < sp->cptr[k + 1]; ++q) {
                sp->pblk[2 * np] = sp->crow[q];
                sp->pblk[2 * np + 1] = k;
                ++np;
                for (int q2 = sp->cptr[k]; q2 <= q; ++q2) {
                    const int64_t key = (int64_t)sp->crow[q] * nb + sp->crow[q2];
                    if (tmark[key] != l) { tmark[key] = l; tkeys[nk++] = key; }
                }
            }
        }
        sp->pptr[l + 1] = np;
        /* targets in ascending (i, j) order (shell sort of the keys); each target's sources: the level's
         * columns k with both i and j in rows(k), ascending */
        if (nk > 1) {
            int64_t* ks = tkeys;
            for (int64_t gap = nk / 2; gap > 0; gap /= 2)
                for (int64_t a = gap; a < nk; ++a) {
                    int64_t v = ks[a], b = a;
                    while (b >= gap && ks[b - gap] > v) { ks[b] = ks[b - gap]; b -= gap; }
                    ks[b] = v;
                }
        }
        for (int64_t t = 0; t < nk; ++t) {
            const int i = (int)(tkeys[t] / nb), j = (int)(tkeys[t] % nb);
            if (nt >= cap_t) {
                cap_t *= 2;
                sp->tgt = realloc(sp->tgt, sizeof(int32_t) * 2 * cap_t);
                sp->sptr = realloc(sp->sptr, sizeof(int32_t) * (cap_t + 1));
            }
            sp->tgt[2 * nt] = i;
            sp->tgt[2 * nt + 1] = j;
            for (int x = sp->lptr[l]; x < sp->lptr[l + 1]; ++x) {
                const int k = sp->lcol[x];
                if (sp->boff[i * nb + k] >= 0 && sp->boff[j * nb + k] >= 0 && i > k && j > k) {
                    if (ns >= cap_s) { cap_s *= 2; sp->src = realloc(sp->src, sizeof(int32_t) * cap_s); }
                    sp->src[ns++] = k;
                }
            }
            sp->sptr[++nt] = (int32_t)ns;
        }
        sp->tptr[l + 1] = (int32_t)nt;
    }
    free(tmark);
    free(tkeys);
    free(rows);
    free(lev);
    free(pat);
    sp->pool = malloc(sizeof(double) * SBB * (size_t)(nblk > 0 ? nblk : 1));
    sp->rhs = malloc(sizeof(double) * sp->n_pad * NRHS);
    const int64_t ncam = (int64_t)uc * in->n_cam;
    sp->Sc = malloc(sizeof(double) * ((size_t)c->nthreads * (ncam * ncam + ncam) + 1));
    c->sparse = sp;
    return 0;
}

void fbo_sparse_info(const fbo_ctx* c, int64_t* out /*[6]: n_pad, blocks, levels, panel blocks, targets, sources*/) {
    const fbo_sparse* sp = c->sparse;
    out[0] = sp->n_pad;
    out[1] = sp->nblk;
    out[2] = sp->nlev;
    out[3] = sp->pptr[sp->nlev];
    out[4] = sp->tptr[sp->nlev];
    out[5] = sp->sptr[sp->tptr[sp->nlev]];
}

static void sparse_free(fbo_sparse* sp) {
    if (!sp) return;
    free(sp->pos); free(sp->slot_of); free(sp->boff); free(sp->pool); free(sp->cptr); free(sp->crow);
    free(sp->lptr); free(sp->lcol); free(sp->pptr); free(sp->pblk); free(sp->tptr); free(sp->tgt); free(sp->sptr);
    free(sp->src); free(sp->rhs); free(sp->Sc);
    free(sp);
}

/* 14 x 14 (or smaller) dense solve with partial pivoting, in place: returns 0, or 1 if singular */
static int small_solve(int n, double* H /* n x n row-major */, double* b) {
    for (int col = 0; col < n; ++col) {
        int piv = col;
        for (int i = col + 1; i < n; ++i)
            if (fabs(H[i * n + col]) > fabs(H[piv * n + col])) piv = i;
        if (!(fabs(H[piv * n + col]) > 0.0)) return 1;
        if (piv != col) {
            for (int j = 0; j < n; ++j) { double t = H[col * n + j]; H[col * n + j] = H[piv * n + j]; H[piv * n + j] = t; }
            double t = b[col]; b[col] = b[piv]; b[piv] = t;
        }
        for (int i = col + 1; i < n; ++i) {
            const double f = H[i * n + col] / H[col * n + col];
            for (int j = col; j < n; ++j) H[i * n + j] -= f * H[col * n + j];
            b[i] -= f * b[col];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = b[i];
        for (int j = i + 1; j < n; ++j) v -= H[i * n + j] * b[j];
        b[i] = v / H[i * n + i];
    }
    return 0;
}

/*
 * Solve the reduced system accumulated by fbo_reduce in sparse form (fbo_set_sparse(c, 1)):
 * S dc = -r, bordered by G (u_c x 7 row-major, inner constraints) as [S G; G' 0][dc; l] = [-r; 0]
 * (main.m:428-440).  dc: u_c, compressed order.  times (may be NULL): [border + RHS, factor, solves] s.
 * Returns 0, 1 (a non-positive pivot), 2 (singular border combine), 3 (no BLAS / setup).
 */
int fbo_sparse_solve(fbo_ctx* c, const double* r, const double* G, double* dc, double* times) {
    fbo_sparse* sp = c->sparse;
    if (!sp || !g_dgemm || !g_dsyrk || !g_dtrsm || !g_dpotrf) return 3;
    const fbo_input* in = &c->in;
    const int64_t n = sp->n_pad, u_c = c->u_c;
    const int nb = sp->nb, ui = c->u_img;
    const int ic = in->ic && G;
    const int nr = ic ? NRHS : 1;
    const int sb = SB, ldy = (int)n;
    const double one = 1.0, mone = -1.0;
    double t0 = 0, t1 = 0, t2 = 0, t3 = 0;
#ifdef _OPENMP
    t0 = omp_get_wtime();
#endif
    double* Y = sp->rhs;
    double* AB = NULL;  /* the border's A | B columns (n x 14), kept for the combine */
    memset(Y, 0, sizeof(double) * n * nr);
    /* unit diagonal (zero RHS) for the positions that hold no unknown: padding slots, EOPs not estimated,
     * the padding after the camera unknowns */
    {
        uint8_t* used = calloc(n, 1);
        for (int64_t i = 0; i < u_c; ++i) used[sp->pos[i]] = 1;
        for (int64_t q = 0; q < n; ++q)
            if (!used[q]) *sblk(sp, q, q) = 1.0;
        free(used);
    }
    for (int64_t i = 0; i < u_c; ++i) Y[sp->pos[i]] = -r[i];
    if (ic) {
        /* equilibrating weights from diag(S) (the GPU's k_border_weights): W_l over the first n_loc slots,
         * D over all images; A = G_l W_l^1/2, B = G D as RHS columns 1..7, 8..14; M = S + A A' */
        double sa[7] = {0}, sb7[7] = {0};
        const int64_t nimg_u = (int64_t)ui * in->n_img;
        for (int64_t i = 0; i < nimg_u; ++i) {
            const int64_t p = sp->pos[i];
            const double d = *sblk(sp, p, p);
            const double inv = d > 0.0 ? 1.0 / d : 0.0;
            for (int m = 0; m < 7; ++m) {
                const double v = G[i * 7 + m] * G[i * 7 + m] * inv;
                sb7[m] += v;
                if (p < 6 * (int64_t)sp->n_loc) sa[m] += v;
            }
        }
        double wa[7], wb[7];
        for (int m = 0; m < 7; ++m) {
            wa[m] = sqrt(sa[m] > 0.0 ? 1.0 / sa[m] : 1.0);
            wb[m] = sqrt(sb7[m] > 0.0 ? 1.0 / sb7[m] : 1.0);
        }
        for (int64_t i = 0; i < nimg_u; ++i) {
            const int64_t p = sp->pos[i];
            for (int m = 0; m < 7; ++m) {
                if (p < 6 * (int64_t)sp->n_loc) Y[(1 + m) * n + p] = wa[m] * G[i * 7 + m];
                Y[(8 + m) * n + p] = wb[m] * G[i * 7 + m];
            }
        }
        AB = malloc(sizeof(double) * (size_t)n * 14);
        memcpy(AB, Y + n, sizeof(double) * (size_t)n * 14);
        for (int64_t pi = 0; pi < 6 * (int64_t)sp->n_loc; ++pi)
            for (int64_t pj = 0; pj <= pi; ++pj) {
                double acc = 0.0;
                for (int m = 0; m < 7; ++m) acc += Y[(1 + m) * n + pi] * Y[(1 + m) * n + pj];
                if (acc != 0.0) *sblk(sp, pi, pj) += acc;
            }
    }
#define BLK(i, j) (sp->pool + (int64_t)sp->boff[(i) * nb + (j)] * SBB)
#ifdef _OPENMP
    t1 = omp_get_wtime();
#endif
    int bad = 0;
    for (int l = 0; l < sp->nlev; ++l) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads) reduction(| : bad)
        for (int x = sp->lptr[l]; x < sp->lptr[l + 1]; ++x) {
            const int k = sp->lcol[x];
            int info = 0;
            g_dpotrf("L", &sb, BLK(k, k), &sb, &info);
            if (info != 0) bad |= 1;
        }
        if (bad) break;
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads)
        for (int q = sp->pptr[l]; q < sp->pptr[l + 1]; ++q) {
            const int i = sp->pblk[2 * q], k = sp->pblk[2 * q + 1];
            g_dtrsm("R", "L", "T", "N", &sb, &sb, &one, BLK(k, k), &sb, BLK(i, k), &sb);
        }
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads)
        for (int t = sp->tptr[l]; t < sp->tptr[l + 1]; ++t) {
            const int i = sp->tgt[2 * t], j = sp->tgt[2 * t + 1];
            for (int e = sp->sptr[t]; e < sp->sptr[t + 1]; ++e) {
                const int k = sp->src[e];
                if (i == j) g_dsyrk("L", "N", &sb, &sb, &mone, BLK(i, k), &sb, &one, BLK(i, i), &sb);
                else g_dgemm("N", "T", &sb, &sb, &sb, &mone, BLK(i, k), &sb, BLK(j, k), &sb, &one, BLK(i, j), &sb);
            }
        }
    }
#ifdef _OPENMP
    t2 = omp_get_wtime();
#endif
    if (bad) { free(AB); return 1; }
    /* forward Y = L^-1 Y, level by level: the level's columns, then each row block's updates from them
     * (the level's diagonal targets (i, i) list exactly those sources); backward Y = L^-T Y top down */
    for (int l = 0; l < sp->nlev; ++l) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads)
        for (int x = sp->lptr[l]; x < sp->lptr[l + 1]; ++x) {
            const int k = sp->lcol[x];
            g_dtrsm("L", "L", "N", "N", &sb, &nr, &one, BLK(k, k), &sb, Y + (int64_t)k * SB, &ldy);
        }
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads)
        for (int t = sp->tptr[l]; t < sp->tptr[l + 1]; ++t) {
            const int i = sp->tgt[2 * t];
            if (sp->tgt[2 * t + 1] != i) continue;
            for (int e = sp->sptr[t]; e < sp->sptr[t + 1]; ++e) {
                const int k = sp->src[e];
                g_dgemm("N", "N", &sb, &nr, &sb, &mone, BLK(i, k), &sb, Y + (int64_t)k * SB, &ldy, &one,
                        Y + (int64_t)i * SB, &ldy);
            }
        }
    }
    for (int l = sp->nlev - 1; l >= 0; --l) {
#pragma omp parallel for schedule(dynamic, 1) num_threads(c->nthreads)
        for (int x = sp->lptr[l]; x < sp->lptr[l + 1]; ++x) {
            const int k = sp->lcol[x];
            for (int q = sp->cptr[k]; q < sp->cptr[k + 1]; ++q) {
                const int i = sp->crow[q];
                g_dgemm("T", "N", &sb, &nr, &sb, &mone, BLK(i, k), &sb, Y + (int64_t)i * SB, &ldy, &one,
                        Y + (int64_t)k * SB, &ldy);
            }
            g_dtrsm("L", "L", "T", "N", &sb, &nr, &one, BLK(k, k), &sb, Y + (int64_t)k * SB, &ldy);
        }
    }
#undef BLK
    if (ic) {
        /* the exact bordered solution (the GPU's border combine): d = y0 + YA z + YB k with
         * [A'YA - I, A'YB; B'YA, B'YB] [z; k] = -[A'y0; B'y0], A and B the RHS columns kept in AB */
        double H[14 * 14], b[14];
        for (int a = 0; a < 14; ++a) {
            const double* va = AB + (int64_t)a * n;
            double s0 = 0.0;
            for (int64_t q = 0; q < n; ++q) s0 += va[q] * Y[q];
            b[a] = -s0;
            for (int m = 0; m < 14; ++m) {
                const double* ym = Y + (int64_t)(1 + m) * n;
                double s1 = 0.0;
                for (int64_t q = 0; q < n; ++q) s1 += va[q] * ym[q];
                H[a * 14 + m] = s1 - ((a < 7 && m == a) ? 1.0 : 0.0);
            }
        }
        free(AB);
        AB = NULL;
        if (small_solve(14, H, b)) return 2;
        for (int64_t q = 0; q < n; ++q) {
            double v = Y[q];
            for (int m = 0; m < 14; ++m) v += Y[(int64_t)(1 + m) * n + q] * b[m];
            Y[q] = v;
        }
    }
    for (int64_t i = 0; i < u_c; ++i) dc[i] = Y[sp->pos[i]];
#ifdef _OPENMP
    t3 = omp_get_wtime();
#endif
    if (times) { times[0] = t1 - t0; times[1] = t2 - t1; times[2] = t3 - t2; }
    return 0;
}

void fbo_set_sparse(fbo_ctx* c, int on) { c->sparse_on = on && c->sparse; }
