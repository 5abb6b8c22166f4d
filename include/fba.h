/*
 * fba.h -- C-ABI of libfba.so, the MI355X-native Gauss-Newton bundle-adjustment inner loop.
 *
 * Drop-in boundary for the reference's MATLAB hot path (wynandtredoux/Fish-Eye_Bundle_Adjustment):
 *
 *   fba_buildxhat     replaces  [error, xhat, xhatnames] = Buildxhat(data, EXT, INT, TIE, CNT)
 *                               functions/Buildxhat.m:2 (called at main.m:388)
 *   fba_build_awg     replaces  [error, A, misclosure, G, dist_scaling] = BuildAwG(data, xhat)
 *                               functions/BuildAwG.m:14 (called at main.m:416); dense debug form
 *   fba_accumulate +
 *   fba_solve_update  replace   one pass of the inline loop body main.m:413-488
 *                               (BuildAwG -> u = A'Pw, N = A'PA -> bordered solve -> de-scale ->
 *                               xhat += delta -> deltasum = sumabs(delta)), split at the point where a
 *                               multi-GPU caller all-reduces the normal equations
 *   fba_step          = fba_accumulate + fba_solve_update (single GPU)
 *   fba_adjust        replaces  the whole loop main.m:407-494 (while deltasum > threshold, cap)
 *   fba_build_rsd     replaces  RSD = BuildRSD(v, data, xhat) (functions/BuildRSD.m:1) for a given v
 *   fba_residuals     replaces  v = A*delta + w (main.m:569), RSD = BuildRSD(v, data, xhat)
 *                               (functions/BuildRSD.m:1, main.m:571), RMSx/RMSy/RMS (main.m:594-598),
 *                               sigma02 = v'Pv/(n-u) (main.m:601)
 *
 * Conventions (mirroring the reference's): every function returns 0 on success and a nonzero
 * FBA_ERR_* code where the reference would set error = 1 (BuildAwG.m:16, Buildxhat.m:3); the message
 * is available from fba_last_error().  No exceptions cross the ABI.  All arrays are caller-owned
 * host buffers; indices are 0-based (the reference's are 1-based); reals are IEEE fp64.
 * A context owns its device memory and is bound to one GPU; it is not re-entrant.
 */
#ifndef FBA_H_
#define FBA_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FBA_ABI_VERSION 2

/* projection models, BuildAwG.m:184-213 (the reference's `typeint`) */
enum {
    FBA_TYPE_FISHEYE = 0,       /* equidistant:  -c*U/R*atan(R/W)           */
    FBA_TYPE_PINHOLE = 1,       /* collinearity: -c*U/W                     */
    FBA_TYPE_EQUISOLID = 2,     /* -2c*U/R*sin(atan(R/W)/2)                 */
    FBA_TYPE_ORTHOGRAPHIC = 3,  /* -c*U/R*sin(atan(R/W))                    */
    FBA_TYPE_STEREOGRAPHIC = 4  /* -2c*U/R*tan(atan(R/W)/2)                 */
};

/* error codes */
enum {
    FBA_OK = 0,
    FBA_ERR_ARG = 1,         /* invalid argument / inconsistent problem                  */
    FBA_ERR_TYPE = 2,        /* invalid Type (BuildAwG.m:209-213)                        */
    FBA_ERR_HIP = 3,         /* HIP runtime failure                                      */
    FBA_ERR_NOT_SPD = 4,     /* reduced normal matrix not positive definite              */
    FBA_ERR_UNSUPPORTED = 5, /* input outside what this build implements (message says) */
    FBA_ERR_NONFINITE = 6    /* non-finite correction (divergence guard)                 */
};

#define FBA_NK_MAX 8 /* maximum Num_Radial_Distortions */

/* The .cfg flags that parameterise the hot path (main.m:150-171, findSetting.m). */
typedef struct fba_settings {
    int32_t est_Xc, est_Yc, est_Zc, est_omega, est_phi, est_kappa; /* Estimate_Xc..Estimate_Kappa */
    int32_t est_xp, est_yp, est_c;                                  /* Estimate_xp/_yp/_c          */
    int32_t est_radial;                                             /* Estimate_Radial_Distortions */
    int32_t est_decent;                                             /* Estimate_Decentering_...    */
    int32_t num_radial;        /* Num_Radial_Distortions (clamped >= 1, BuildAwG.m:18-20)   */
    int32_t type;              /* FBA_TYPE_*                                                */
    int32_t inner_constraints; /* Inner_Constraints                                         */
    int32_t iteration_cap;     /* Iteration_Cap                                             */
    int32_t reserved;
    double threshold;          /* Threshold_Value                                           */
    double meas_std_x;         /* Meas_std                                                  */
    double meas_std_y;         /* Meas_std_y (= Meas_std when absent, main.m:397-402)       */
} fba_settings;

/*
 * Packed problem (structure-of-arrays).  This is the reference's `data` struct (main.m:280-383)
 * after its joins: one entry per PHO row, in PHO order.
 */
typedef struct fba_problem {
    int64_t n_pts;            /* image points = PHO rows (n = 2*n_pts observations)         */
    int32_t n_img;            /* numImg: images = EXT rows 0..n_img-1 (Buildxhat.m:22)      */
    int32_t n_cam;            /* numCam: cameras = INT pairs 0..n_cam-1 (Buildxhat.m:65)    */
    int32_t n_tie;            /* numtie: estimated object points (TIE order)                */
    int32_t reserved;
    const double* xy;         /* [2*n_pts]  x0 y0 x1 y1 ... (pixels)                        */
    const int32_t* img;       /* [n_pts]    ext_index (EXT row)                              */
    const int32_t* cam;       /* [n_pts]    cam_num (INT pair), must equal EXT's camera     */
    const int32_t* tie;       /* [n_pts]    tieIndex, or -1 for a fixed (control) point      */
    const double* xyz_fixed;  /* [3*n_pts]  CNT coordinates (used where tie < 0)            */
    const double* eop0;       /* [6*n_img]  EXT Xc Yc Zc omega phi kappa (radians)          */
    const double* iop0;       /* [n_cam*(5+num_radial)] INT xp yp c K1..Knk P1 P2           */
    const double* cam_info;   /* [5*n_cam]  y_dir xmin ymin xmax ymax                        */
    const double* tie0;       /* [3*n_tie]  CNT coordinates of the TIE list                  */
} fba_problem;

typedef struct fba_options {
    int32_t device;      /* HIP device ordinal                                              */
    int32_t rank;        /* this process's rank (observation shard), 0 for single GPU      */
    int32_t world;       /* number of ranks, 1 for single GPU                               */
    int32_t verbose;
    void* stream;        /* hipStream_t to run on, or NULL for a context-owned stream       */
    int32_t split;       /* world > 1: 0 = replicated solve (every rank factors the summed reduced
                          * system), 1 = subtree split: the elimination tree is cut into top
                          * columns and subtrees dealt to the ranks; tie points follow their
                          * images' subtree, each rank factors its subtrees in fba_accumulate and
                          * the reduce buffer carries only the top blocks (no reference
                          * counterpart: main.m:432 inverts the dense matrix on one CPU)          */
} fba_options;

typedef struct fba_ctx fba_ctx;

/* Thread-local message of the last failure. */
const char* fba_last_error(void);
int fba_abi_version(void);

/* Number of unknowns u of the reference's xhat (Buildxhat.m:6-15); host only. */
int fba_count_unknowns(const fba_problem* p, const fba_settings* s, int64_t* u_out);

/* Deterministic observation shard: owner rank of every tie point (contiguous ranges balanced by
 * observation count) and of every control observation; host only, no GPU needed. */
int fba_partition(const fba_problem* p, int32_t world, int32_t* tie_owner /*[n_tie]*/,
                  int32_t* ctl_owner /*[n_pts], -1 for tie observations*/);

/* Camera-side elimination order of the reduced system the device factorisation uses (host only, no
 * GPU): nested dissection of the images' co-visibility graph (fba_order.cpp).  Slot k of the reduced
 * system's image part (unknowns 6k..6k+5) holds EXT row order[k], or -1 for a padding slot (padding
 * keeps independent subtrees in separate 128-row blocks); the camera unknowns follow the last slot, and
 * inner constraints are bordered on the first min(n_slots, 21) slots.  order may be NULL to query
 * *n_slots.  No reference counterpart (main.m:432 inverts the dense bordered matrix): for callers that
 * factor the reduced system themselves on the same block pattern (oracle/fba_cpu.c's cpu_baseline). */
int fba_image_order(const fba_problem* p, int32_t* order /*[n_slots]*/, int32_t* n_slots);

int fba_create(const fba_problem* p, const fba_settings* s, const fba_options* o, fba_ctx** out);
void fba_destroy(fba_ctx* ctx);

/* The solve the context actually runs: *split = 1 when fba_options.split was honoured (subtree split:
 * reduce-buffer layout, ownership and the one-solve-per-accumulation rule of the split), 0 for the
 * replicated / single-GPU solve -- a split request falls back to the replicated solve when the block
 * pattern cannot be cut (no reference counterpart). */
int fba_solve_mode(fba_ctx* ctx, int32_t* split);

/* Buildxhat.m: initial xhat in the reference's layout.  xhat may be NULL to query u only. */
int fba_buildxhat(fba_ctx* ctx, double* xhat /*[u]*/, int64_t* u_out);

/* Set / get the device-resident xhat (reference layout).  With owned_only != 0 the entries this
 * rank does not own are returned as 0 (tie points of other ranks; camera entries on rank > 0), so
 * that a sum over ranks reassembles the full vector. */
int fba_set_xhat(fba_ctx* ctx, const double* xhat);
int fba_get_xhat(fba_ctx* ctx, double* xhat, int32_t owned_only);

/* BuildAwG.m (dense debug/parity form): A is n x u column-major (n = 2*n_pts, PHO row order),
 * w is n, G is u x 7 column-major (only when inner constraints are on; may be NULL),
 * dist_scaling is n_cam x (2+num_radial) column-major; columns 0-1 hold the reference's 1-based xhat
 * index of the first radial / decentering unknown (0 when not estimated, BuildAwG.m:138, :150),
 * columns 2.. rmax^(2j) (BuildAwG.m:424-426).
 * Any output pointer may be NULL. */
int fba_build_awg(fba_ctx* ctx, const double* xhat, double* A, double* w, double* G,
                  double* dist_scaling);

/* One Gauss-Newton iteration, split for multi-GPU callers:
 *   fba_accumulate      linearise this rank's observations at the device xhat and accumulate the
 *                       (point-reduced) normal equations into the reduce buffer;
 *   fba_reduce_buffer   device pointer + length (doubles) of that buffer: ranks sum it elementwise
 *                       (e.g. an RCCL all-reduce) between the two calls.  With world == 1 there is
 *                       nothing to sum and the buffer IS the context's reduced system; the solve
 *                       reads weights fba_accumulate already derived from it, so the caller must not
 *                       modify it between fba_accumulate and fba_solve_update (reading is fine);
 *   fba_solve_update    bordered solve, point back-substitution, de-scaling, xhat update.
 *                       *deltasum_part receives this rank's share of sumabs(delta) (sum over ranks
 *                       = the reference's deltasum).
 * fba_step does both halves on one GPU and returns the full deltasum. */
int fba_accumulate(fba_ctx* ctx);
int fba_reduce_buffer(fba_ctx* ctx, void** dev_ptr, int64_t* n_doubles);
/* Block until every operation queued on the context's stream has completed (needed before a
 * caller touches the reduce buffer from another stream or the host). */
int fba_synchronize(fba_ctx* ctx);
int fba_solve_update(fba_ctx* ctx, double* deltasum_part);
/* The same split without the host round trip in the middle (multi-GPU): fba_solve_update_async only
 * enqueues the solve on the context's stream; fba_deltasum_device gives the device address of this
 * rank's deltasum share (one double), which the caller may all-reduce in place on that stream;
 * fba_solve_finish synchronises, checks the solve and returns that (reduced) value. */
int fba_solve_update_async(fba_ctx* ctx);
int fba_deltasum_device(fba_ctx* ctx, void** dev_ptr);
int fba_solve_finish(fba_ctx* ctx, double* deltasum);
int fba_step(fba_ctx* ctx, double* deltasum);

/* main.m:407-494: iterate while deltasum > threshold, at most iteration_cap times.
 * deltasum_hist (may be NULL) receives one entry per iteration (capacity iteration_cap). */
int fba_adjust(fba_ctx* ctx, int32_t* iterations, double* deltasum_hist);

/* main.m:567-602 + BuildRSD.m: from the last iteration's linearisation and de-scaled delta.
 * v [2*n_pts] (PHO order), rsd [5*n_pts] row-major per point: r, vx, vy, vr, vt,
 * stats [6]: RMSx, RMSy, RMS, sigma02, vTPv, n-u.  Pointers may be NULL.  With world > 1 each rank
 * fills only its observations (others 0) and stats hold this rank's partial sums
 * (sum vx^2, sum vy^2, 0, 0, vTPv, n-u); fba_finish_stats turns reduced sums into RMS / sigma02. */
int fba_residuals(fba_ctx* ctx, double* v, double* rsd, double* stats);

/* BuildRSD.m:1 for a caller-given v (e.g. the reference's v = A*delta + w, main.m:569-571): per PHO
 * row [r, vx, vy, vr, vt] (BuildRSD.m:29-40) with xp, yp from xhat where estimated, else the INT
 * values (BuildRSD.m:12-26).  v [2*n_pts] x y interleaved (PHO order), xhat [u] the reference layout,
 * rsd [5*n_pts] row-major.  With world > 1 only this rank's rows are written (others 0). */
int fba_build_rsd(fba_ctx* ctx, const double* v, const double* xhat, double* rsd);
int fba_finish_stats(const fba_problem* p, const fba_settings* s, const double* sums /*[2]: sum vx^2, sum vy^2*/,
                     double vtpv, double* stats /*[6]*/);

/* Post-fit covariance of the unknowns (main.m:428-456, :460-482, :602): from the factor of the LAST
 * solve (call right after the iterations, before any further fba_accumulate / fba_step; the factor is
 * consumed).  sigma02 is the a-posteriori variance factor (fba_residuals stats[3] or fba_finish_stats).
 *   cx_diag [u] (may be NULL): diag(Cx) of the reference's final Cx = sigma02 * (bordered) inverse of
 *           the last normal matrix, distortion entries de-scaled by dist_scaling^2 (main.m:460-482,
 *           diagonal only, as the reference); xhat order.  With world > 1 the tie entries of other
 *           ranks are 0 (camera entries are replicated); with the subtree split (fba_options.split)
 *           the camera-side entries too are this rank's rows only (its subtrees' images, and the top's
 *           images and the camera unknowns on rank 0), so the ranks' outputs sum to the whole vector.
 *   corr [n_img][(u_img+u_cam)^2] (may be NULL): per EXT image, the reference's Correlation matrix
 *           (main.m:446-456) restricted to [the image's estimated EOPs, its camera's estimated
 *           IOP/distortion unknowns] in xhat order, full symmetric, row-major (main.m:831-840); with
 *           the subtree split only this rank's images (the rank owning the image's first row; wholly
 *           top images on rank 0), zeros for the others. */
int fba_covariance(fba_ctx* ctx, double sigma02, double* cx_diag, double* corr);

/* Per-phase device timings of the last fba_step / fba_accumulate+fba_solve_update, in ms:
 * [0] params+linearize, [1] point-side, [2] image/pair/camera accumulation, [3] border,
 * [4] Cholesky+forward, [5] backward+border solve, [6] back-substitution+update, [7] total. */
int fba_last_timings(fba_ctx* ctx, double* ms /*[8]*/);
int fba_set_timing(fba_ctx* ctx, int32_t enabled);

/* Kernel probe (measurement only; no reference counterpart): while enabled, every launch of one
 * Cholesky kernel is bracketed by HIP events on the stream it runs on -- enabled = 1: k_syrk_multi (the
 * bulk trailing update of a tree level), 2: k_panel (the level's diagonal-block factorisations and
 * panel solves, the critical path); 0 turns the probe off.  fba_probe_stats synchronises and returns,
 * over the launches since the probe was enabled: out[0] launches, out[1] summed kernel ms, out[2]
 * algorithmic flops, out[3] reserved.  The probe records at most one step's worth of launches. */
int fba_set_probe(fba_ctx* ctx, int32_t enabled);
int fba_probe_stats(fba_ctx* ctx, double* out /*[4]*/);

/* (tests) The bound of every device hand-off poll of this context, in sleeps (0: the default
 * 1 << 22, ~0.3 s; negative: FBA_ERR_ARG; values above 2^32 - 1 are clamped to it; FBA_FLAG_SPINS in
 * the environment sets it at fba_create, where <= 0 is the default): a low bound forces the timeout path -- the abort
 * reaches every wait, the step returns FBA_ERR_HIP and xhat stays as before it. */
int fba_set_spin_bound(fba_ctx* ctx, int64_t spins);

/* Test hook (no reference counterpart): the 14x14 bordered solve of the inner-constraint combine
 * (k_border_combine, one workgroup on `device`) for a given symmetric 15x15 Gram matrix of the
 * forward-solved rows [y | A (7) | B (7)] (row-major): coef = [z; k] solving
 * [[A'A - I, A'B], [B'A, B'B]] [z; k] = -[A'y; B'y]. */
int fba_test_border_solve(int32_t device, const double* gram /*[225]*/, double* coef /*[14]*/);

#ifdef __cplusplus
}
#endif
#endif /* FBA_H_ */
