// fba_internal.h -- device layout and context of libfba.so (not part of the ABI).
//
// Unknowns live on the device in a FULL parameter space: every image carries all 6 EOPs
// (Xc Yc Zc omega phi kappa) and every camera all CW = 5 + nK IOPs (xp yp c K1..KnK P1 P2),
// followed by 3 coordinates per tie point.  Parameters the .cfg does not estimate get zero
// Jacobian columns, a unit diagonal in the reduced system and a zero correction, so the kernels
// need no per-flag variants; the reference's compressed xhat (Buildxhat.m:6-134) is produced only
// at the ABI boundary through the index maps below.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fba.h"

namespace fba {

constexpr int NB = 128;       // Cholesky block size (rows/cols of one panel block, fba_chol.hip)
constexpr int PTRACE_WG = 2048;  // FBA_PANEL_TRACE: workgroup slots per level
constexpr int FTRACE = 56;       // FBA_PANEL_TRACE: stamps per k_chol_flow record ([48]: its workgroup's start)
// k_chol_flow: a fused diagonal update's tiles of tile columns >= FLOW_CSPLIT go to a helper record,
// added into the potrf's LDS block during its bulk step FLOW_CSPLIT - 2 (fba_order.cpp build_flow)
constexpr int FLOW_CSPLIT = 3;
// k_bwd_flow's "not yet published" value of the solution blocks X (a signalling NaN with a payload no
// arithmetic produces): the consumers poll the data itself, k_border_rhs resets it every solve
constexpr uint64_t X_SENTINEL = 0x7FF4DEADBEEF5A5Aull;
constexpr int SCAL_SPINS = 6;  // d_scal slot: this context's hand-off poll bound (fba_chol.hip spin_expired)
// the value stored there for a requested bound: <= 0 means the default 1 << 22 (~0.3 s), and a bound is
// clamped to 2^32 - 1 (spin_expired compares it with a 32-bit counter)
inline double spin_bound_value(long long spins) {
    return spins <= 0 ? (double)(1u << 22) : (double)(spins < 0xffffffffLL ? spins : 0xffffffffLL);
}
constexpr int CHUNK_OBS = 256;  // observations per k_lin_reduce / k_lin_point workgroup (chunk)
// tie points per chunk and co-visibility terms per chunk staged in LDS (a single larger point's are
// read from HBM instead): smaller for nK >= 6, whose wider Jacobian rows leave less of the 160 KiB LDS
// (k_lin_reduce's LR<NK>::LDS, static_assert there); the host chunking uses the same numbers
constexpr int chunk_pts(int nk) { return nk <= 5 ? 64 : 32; }
constexpr int chunk_terms(int nk) { return nk <= 5 ? 2048 : 1024; }

// per-image device table (k_params): eop[6], M[9], dM/domega[9], dM/dphi[9], dM/dkappa[9], pad
constexpr int IMG_TAB = 48;
// per-camera device table: xp yp c ydir P1 P2 rmax2 pad, K[nK], scale[nK] (rmax^(2j))
constexpr int CAM_TAB_HDR = 8;
// d_bscr: [32][14] k_border_weights segments | [16][120] Gram segments | [16] combine coefficients |
// [16] the subtree split's B-row scales sqrt(W_d)
constexpr int BSC_OFF = 32 * 14 + 16 * 120 + 16;

struct Layout {
    int n_img = 0, n_cam = 0, n_tie = 0, nk = 1, cw = 6;  // n_img: internal image slots (padding included)
    int n_img_ref = 0;    // the reference's images (EXT rows)
    int64_t u_c = 0;      // 6*n_img + cw*n_cam (camera-side full unknowns)
    int64_t u_full = 0;   // u_c + 3*n_tie
    int64_t n_pad = 0;    // u_c rounded up to NB
    int64_t ld = 0;       // leading dimension of the normal matrix (row-major)
    int nrhs = 1;         // 1 (+14 with inner constraints: local border + constraint columns)
    int64_t u_ref = 0;    // the reference's u
    int u_img = 0, u_cam = 0;
};

// Block schedule of the reduced-system Cholesky (fba_order.cpp): one batched step per level of the
// elimination tree.  All offsets index the int32 device buffer Ctx::d_sched.
//   trsm records  (k, 2 r + h): panel block (r, k), row half h (halves of padding rows are skipped)
//   task records  SYRK_REC ints: (i, j, quarter 2 qr + qc, s0, s1, slot, comb, fidx): C(i,j) quarter -= sum
//                 of X_ik X_jk' over the sources src[s0..s1) (ascending); slot >= 0: the sum goes to the
//                 scratch quarter `slot` instead (split targets), and the last group to arrive (counter
//                 cbase + comb) applies the COMB_REC record `comb` of the level
//                 (i, j, quarter, first slot, slots): C -= P_first - ... in slot order; fidx: the target
//                 quarter's completion flag when the update runs inside the next level's k_panel
struct Sched {
    static constexpr int SYRK_REC = 8, COMB_REC = 5;
    struct Wave {
        int64_t cols = 0, trsm = 0, tasks = 0, src = 0, comb = 0;  // offsets
        int ncol = 0, ntrsm = 0, ntask = 0, ncomb = 0;
        int cbase = 0;            // first arrival counter of the level's split targets (k_syrk_multi)
        int ndiag = 0;            // the level's first ndiag tasks update next-level diagonal blocks,
        int npanel = 0;           // the next npanel next-level panel blocks, the rest later levels' blocks
        int64_t wstart = 0, wlist = 0;  // merged launch: wait lists (flags of the previous level's
                                        // updates) of this level's potrf columns then panel halves
        double flops = 0.0;       // trailing-update flops of the level (kernel probe)
        double pflops = 0.0;      // diagonal factorisations + panel solves of the level (kernel probe)
    };
    struct BWave {
        int64_t srcs = 0, tgts = 0, src_start = 0, src = 0;
        int nsrc = 0, ntgt = 0;
    };
    int n_waves = 0;
    int64_t n_tiles = 0;
    int64_t bf_start = 0, bf_src = 0;  // backward dataflow (k_bwd_flow): per block column j, the block
                                       // rows i > j of its panel, descending (offsets)
    int64_t zero = 0;             // (block row, block column) of every block of the factor's pattern
    int nzero = 0;                // (diagonal, panel and RHS blocks): zeroed before each accumulation
    int n_scratch = 0;            // 64x64 scratch quarters of the split targets (max over levels)
    int n_counters = 0;           // split-target arrival counters, all levels
    int n_tflags = 0;             // completion flags of the update targets (quarters), all levels
    std::vector<Wave> w;          // factorisation, level 0 up
    std::vector<BWave> b;         // backward solve, indexed by level (run top down)
    std::vector<int32_t> buf;     // host image of the lists (uploaded to Ctx::d_sched)

    // persistent dataflow factorisation (k_chol_flow, fba_order.cpp build_flow): the whole factorisation
    // in ONE launch, one FLOW_REC record per workgroup in dispatch order; every wait points to an earlier
    // record.  Roles: 0 = diagonal block j (its fused source's panel solve and diagonal update, then the
    // potrf), 1 = a panel half solve, 2 = an update task, 3 = a diagonal-block inverse.  Flags live in
    // the tflags region: progress flags [0, flow_nprog) (column blocks of a panel half solved), then the
    // update-completion flags
    static constexpr int FLOW_REC = 16;
    int64_t flow_rec = 0;
    int flow_n = 0, flow_nprog = 0, flow_nuflag = 0, flow_ncounter = 0, flow_nscratch = 0;
    int flow_cnt[5] = {0, 0, 0, 0, 0};  // records per role
    bool flow_ok = false;
    double flow_flops = 0.0;
    double flow_bytes = 0.0;      // operand bytes the records load and store (build_flow)

    // subtree split (fba_options.split, world > 1): the elimination tree is cut into a TOP part (the
    // columns above the cut: separators, camera rows) and subtrees dealt to the ranks.  A rank's points
    // touch only its own subtrees' blocks and the top, so its subtree columns are factored from its own
    // accumulation alone -- flow A, the flow_* fields above -- Schur-updating its partial copy of the top
    // blocks; the ranks sum the top blocks (the reduce buffer), then every rank factors the top columns:
    // flow B (`top`), whose flag, counter and scratch ids follow flow A's (offsets below).
    struct FlowPart {
        int64_t rec = 0;
        int n = 0, nprog = 0, nuflag = 0, ncounter = 0, nscratch = 0;
        int cnt[5] = {0, 0, 0, 0, 0};
        bool ok = false;
        double flops = 0.0;
    };
    bool split = false;
    FlowPart top;
    std::vector<int32_t> blk_rank;   // per block column: owner rank of its subtree, -1 top
    int64_t top_blocks = 0;          // offset of the (block row, block column) list of the top blocks
    int n_top_blocks = 0;            // (lower blocks (a, b) with a, b top, the RHS block row's included)
};

// Accumulation plan (fba_capi.cpp create, run by k_lin_reduce and the k_red_* kernels): offsets
// into the int32 device buffer Ctx::d_acc.
struct AccPlan {
    int64_t ck_cam = 0;    // [n_chunks] camera of each chunk
    int64_t ck_pk = 0;     // [n_chunks+1] pair-key range of each chunk
    int64_t pk_t = 0;      // [n_pk+1] term range of each pair key
    int64_t pk_term = 0;   // [n_terms] (i | j << 16): chunk-local observations in image e1 / e2
    int64_t ck_ik = 0;     // [n_chunks+1] image-key range of each chunk
    int64_t ik_o = 0;      // [n_ik+1] observation range of each image key
    int64_t ik_obs = 0;    // chunk-local observations of each image key
    int64_t rp_start = 0;  // [n_pairs+1] partial slots (pair keys) of each local pair, chunk order
    int64_t rp_e = 0;      // [2 n_pairs] (e1, e2)
    int64_t rp_list = 0;
    int64_t ri_start = 0;  // [n_img+1] image keys of each image
    int64_t ri_list = 0;
    // partial slots: the partials are stored pair-major / image-major (ppart row pk_slot[K] for pair key
    // K, ipart row ik_slot[K] for image key K), so k_red_blocks reads each pair's / image's partials as
    // one contiguous range [rp_start, rp_start+1) / [ri_start, ..) in the same (chunk) order as rp_list
    int64_t pk_slot = 0;   // [n_pk] = the inverse of rp_list
    int64_t ik_slot = 0;   // [n_ik] = the inverse of ri_list
    int64_t img_cam = 0;   // [n_img] camera of each image (-1: no local observation)
    int64_t rc_start = 0;  // [n_cam+1] chunks of each camera
    int64_t rc_list = 0;
    // pair terms reduced from U rows (a chunk whose pair keys hold few terms each -- a dense network's
    // -- registers no pair keys: its pair-block contributions -U_a U_b' are summed by k_red_blocks from
    // the observations' U rows, Ctx::d_U, instead of 288-B partial rows written and read back)
    int64_t ck_tm = 0;     // [n_chunks] 1: the chunk's pair terms go to the U-row path
    int64_t tp_start = 0;  // [n_pairs+1] U-row terms of each local pair, chunk order
    int64_t tp_ab = 0;     // [2 n_tt] (a, b): global observations in image e1 / e2
    int64_t n_pk = 0, n_ik = 0, n_tt = 0;
};

// General tie points (fba_general.hip): the points the chunked fast path does not take -- seen by
// several cameras, by more than CHUNK_OBS images, or measured more than once in one image.  The
// reference accepts all of them (it loops over every PHO row, BuildAwG.m:46; camera columns by the
// point's own cam_num, :448-451; tie columns camera-independent, :501-502).  Each general point q
// owns a contiguous range of the local observations, sorted by image; "gimg" = the observations of
// one point in one image (their eliminated image coupling Ug = sum U_o), "gpc" = the observations of
// one point through one camera (its camera coupling Uc).  Offsets into Ctx::d_acc.
struct GenPlan {
    int64_t n_gp = 0, n_gi = 0, n_gc = 0, n_gpk = 0, n_gx = 0, n_gkk = 0, n_xt = 0, n_kt = 0;
    int64_t lp0 = 0;      // local point index of general point 0
    int64_t g_obs = 0;    // [n_gp+1] observation range of each point
    int64_t g_gi = 0;     // [n_gp+1] its gimg range
    int64_t g_gc = 0;     // [n_gp+1] its gpc range
    int64_t gi_obs = 0;   // [n_gi+1] observation range of each gimg
    int64_t gi_img = 0;   // [n_gi] image slot
    int64_t gi_gp = 0;    // [n_gi] point
    int64_t gi_gc = 0;    // [n_gi] the gpc of the image's own camera
    int64_t gc_cam = 0;   // [n_gc] camera
    int64_t gc_gp = 0;    // [n_gc] point
    int64_t gc_o = 0;     // [n_gc+1] range in gc_list
    int64_t gc_list = 0;  // observations of each gpc (ascending)
    int64_t gpk = 0;      // [2 n_gpk] pair keys (gimg of the higher image, gimg of the lower image)
    int64_t gx = 0;       // [2 n_gx] foreign-camera keys (gimg, gpc of another camera)
    int64_t gkk = 0;      // [2 n_gkk] camera-pair keys (gpc of the higher camera, gpc of the lower camera)
    int64_t xt_start = 0, xt_list = 0, xt_key = 0;  // image x foreign camera blocks: [n_xt+1], slots, [2 n_xt] (e, k)
    int64_t kt_start = 0, kt_list = 0, kt_key = 0;  // camera x camera blocks: [n_kt+1], slots, [2 n_kt] (k1 > k2)
    int64_t pk0 = 0, ik0 = 0, ck0 = 0;  // first partial slot of the general keys in ppart / ipart / cpart
    int64_t pk_slot = 0, ik_slot = 0;   // AccPlan::pk_slot / ik_slot (the keys' rows in ppart / ipart)
};

struct Ctx {
    fba_problem prob{};   // shallow copy (pointers valid only during fba_create)
    fba_settings set{};
    fba_options opt{};
    Layout L;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // the two halves of an iteration captured once as HIP graphs (a capturable stream, no timing /
    // probe / profile events; FBA_NO_GRAPH=1 disables): [0] linearise + accumulate, [1] solve + update
    hipGraphExec_t graph[2] = {nullptr, nullptr};
    bool graphs_ok = true;
    int device = 0;

    // host copies of the problem (kept for residual output, xhat mapping)
    int64_t n_pts = 0;
    std::vector<int64_t> full_to_ref;   // [u_full] -> reference xhat index or -1
    std::vector<double> xfull0;         // initial full-space parameters
    std::vector<int32_t> tie_owner;     // [n_tie]
    std::vector<uint8_t> full_owned;    // [u_full] entries this rank owns (for owned_only output)

    // local (this rank) observation order
    int64_t n_obs = 0;       // local image points
    int64_t n_obs_tie = 0;   // of which tie observations (first), then control
    int64_t n_obs_pad = 0;
    int64_t n_lp = 0;        // local tie points
    std::vector<int64_t> obs_pho;  // local obs -> PHO row

    // ---- device buffers ----
    double* d_xy = nullptr;      // [2*n_obs] x,y interleaved
    int32_t* d_img = nullptr;    // [n_obs]
    int32_t* d_cam = nullptr;    // [n_obs]
    int32_t* d_pt = nullptr;     // [n_obs] local point (>=0) or -1-ctl
    double* d_ctl = nullptr;     // [3*n_ctl] fixed XYZ of control observations
    int32_t* d_lp_tie = nullptr; // [n_lp] global tie index of local point
    int32_t* d_xoff = nullptr;   // [n_obs] offset of the observation's tie point in xfull (u_c + 3 tie; 0: control)
    unsigned* d_lrt = nullptr;   // k_lin_reduce's work tickets [2]: next item, workgroups out (reset by the last out)
    int32_t* d_lp_start = nullptr;   // [n_lp+1] obs range of each local point
    int32_t* d_lp_cam = nullptr;     // [n_lp] camera of each local point
    int64_t n_chunks = 0;            // chunks: [k_lin_reduce's: whole regular tie points of one camera,
                                     // then control observations][the general points' observations,
                                     // linearised by k_lin_point only]
    int64_t n_chunks_lr = 0;         // k_lin_reduce workgroups (regular + control chunks)
    GenPlan gen;                     // general tie points (fba_general.hip)
    double* d_gpt = nullptr;         // [n_gp][18] Vinv 6 | R 6 | rb 3 | vb 3
    double* d_gcu = nullptr;         // [n_gc][6 cw] Uc 3cw | Tc 3cw
    double* d_gug = nullptr;         // [n_gi][36] Ug 18 | sum of T_o 18
    double* d_xpart = nullptr;       // [n_gx][6 cw] foreign-camera partials
    double* d_kpart = nullptr;       // [n_gkk][cw cw] camera-pair partials
    AccPlan acc;                     // accumulation plan (offsets into d_acc)
    int32_t* d_acc = nullptr;
    double* d_ppart = nullptr;       // [acc.n_pk][36] pair-block partials
    double* d_U = nullptr;           // [n_obs_pad][18] U = W R of the observations of U-row chunks (acc.ck_tm)
    int ik_lanes = 8;                // k_lin_reduce's lanes per image-key unit (4: keys of <= 2 observations)
    double* d_ipart = nullptr;       // [acc.n_ik][27 + 6 cw] image partials: diagonal block, RHS, image-camera
    uint64_t* d_lrprof = nullptr;    // FBA_LR_PROFILE: k_lin_reduce phase timestamps [n_chunks][8]
    uint64_t* d_ptrace = nullptr;    // FBA_PANEL_TRACE: k_panel workgroup timestamps [level][PTRACE_WG][8]
    double* d_cpart = nullptr;       // [n_chunks][cw(cw+1)/2 + cw] camera-block partials
    int32_t* d_chunk_obs = nullptr;  // [n_chunks+1] observation range of each chunk
    int32_t* d_chunk_pt = nullptr;   // [n_chunks+1] local point range of each chunk
    int64_t n_pairs = 0, n_pair_terms = 0;
    // multi-rank compact reduce buffer: the entries of S that any rank can write (global co-visible
    // image pairs, diagonal blocks, camera rows, RHS row), packed after fba_accumulate
    int64_t n_gpairs = 0, n_red = 0;
    // subtree split (Sched::split): the reduce buffer holds [top blocks | the raw diagonal of the top rows
    // | Gram partials of the subtree columns | this rank's 7 inner-constraint weight sums]; offsets
    int64_t red_diag = 0, red_gblk = 0, red_w = 0;
    int8_t* d_bown = nullptr;        // [nb] 1: this rank's subtree block, 2: top, 0: another rank's
    // [n_pad] per camera-side row, by its IMAGE: 1 an image of this rank's subtrees (its rows in a top block
    // included -- an image straddling a subtree block and a top block has its other EOPs, which its G rows
    // read, current on its subtree's rank only), 2 an image wholly in the top (and top camera / padding
    // rows), 0 another rank's; the once-only border entries, the weight sums and the top diagonal follow it
    int8_t* d_rown = nullptr;
    int32_t* d_topdiag = nullptr;    // [n_topdiag] rows of the top blocks carrying image unknowns
    int64_t n_topdiag = 0;
    // camera-side image order (nested dissection, fba_order.cpp) and the factorisation schedule
    std::vector<int32_t> img_ord, img_new;  // internal slot -> EXT row (-1: padding), EXT row -> slot
    int n_loc = 0;                          // image slots carrying the (local) inner-constraint border
    Sched sched;
    int32_t* d_sched = nullptr;             // device image of the schedule lists (offsets in sched)
    int32_t* d_gpairs = nullptr;     // [2*n_gpairs] (e1,e2), e1 > e2, over ALL tie points
    double* d_red = nullptr;         // [n_red]

    double* d_xfull = nullptr;   // [u_full]
    double* d_xlin = nullptr;    // [u_full] the last linearisation point (residuals after the loop)
    double* d_delta = nullptr;   // [u_full] last de-scaled correction
    double* d_img_tab = nullptr; // [n_img*IMG_TAB]
    double* d_cam_tab = nullptr; // [n_cam*cam_tab_stride]
    int cam_tab_stride = 0;
    double* d_G = nullptr;       // [n_img*42] inner-constraint blocks (6x7 per image, row-major)
    double* d_J = nullptr;       // [n_obs_pad][ncomp] per-obs Jacobian rows + misclosure (obs-major)
    int ncomp = 0;
    double* d_cseg = nullptr;    // [n_cam][64][NCAM] camera segment sums (k_red_cam_seg)
    double* d_bscr = nullptr;    // border scratch: [32][14] weight segment sums | [16][120] Gram segments
    double* d_gblk = nullptr;    // [n_pad / NB][16][16] per-column-block Gram partials of the forward-solved
                                 // RHS rows (k_chol_flow; inner constraints)
    double* d_WT = nullptr;      // [n_obs_pad][12] per-obs record: Jp and the EOP rotation columns (OBS_REC)
    double* d_pt_tab = nullptr;  // [n_lp_pad][pt_comp] Vinv(6) vb(3) b(3) Wc(3cw) Tc(3cw)
    int pt_comp = 0;
    int64_t n_lp_pad = 0;
    double* d_P = nullptr;       // [Sched::n_scratch][64*64] partial sums of split update targets
    unsigned* d_flags = nullptr; // [nb] k_panel hand-off flags (zeroed before each factorisation)
    unsigned* d_bflags = nullptr; // [nb] k_bwd_flow hand-off flags (zeroed before each backward solve)
    unsigned* d_counters = nullptr; // [Sched::n_counters] split-target arrival counters
    unsigned* d_tflags = nullptr;   // [Sched::n_tflags] update-target completion flags (merged k_panel)
    unsigned* d_tickets = nullptr;  // [2] start-order tickets of k_chol_flow / k_bwd_flow records
    int64_t n_sync = 0;           // unsigned words of flags + bflags + counters (one allocation at d_flags,
                                  // zeroed by k_border_rhs ahead of every factorisation)
    bool bwd_flow = true;
    bool merge_updates = true;      // a level's trailing updates inside the next level's k_panel
                                    // (FBA_MERGE_UPDATES=0: their own k_syrk_multi launch)
    bool chol_flow = true;          // the factorisation as one persistent k_chol_flow launch (FBA_CHOL_FLOW=0:
                                    // one k_panel launch per elimination-tree level)
    bool panel_progressive = true;  // k_panel: panel solves step with the potrf's published column blocks
                                    // (FBA_PANEL_PROGRESSIVE=0: wait for the whole factor)         // one-launch backward solve (FBA_BWD_LEVELS=1: one launch per level)
    size_t flags_bytes = 0;
    int n_cu = 0;                // compute units (k_panel needs its whole grid resident)
    double* d_S = nullptr;       // [(n_pad+NB)*ld] normal matrix (lower) + RHS rows
    double* d_X = nullptr;       // [n_pad] solution of the bordered solve
    double* d_dinv = nullptr;    // [(n_pad/NB)*8*256] inverses of the 16x16 diagonal blocks of L
    double* d_linv = nullptr;    // [(n_pad/NB)*128*128] inverses of the 128x128 diagonal blocks of L
    double* d_scal = nullptr;    // scalars: [1] Cholesky failure flag, [2] sumabs, [8..14] border weights
    double* d_part = nullptr;    // block partial sums
    int n_part = 0;
    double* d_res = nullptr;     // [7*n_obs] v (2) + rsd (5)
    double* d_caminfo = nullptr; // [5*n_cam]
    uint8_t* d_active = nullptr; // [n_pad] 1 = estimated camera-side parameter
    uint8_t* d_counted = nullptr;// [u_full] 1 = counted in this rank's sumabs share
    int64_t* d_obs_pho = nullptr;// [n_obs] PHO row of each local observation
    double* h_pinned = nullptr;  // pinned host scratch (coherent, mapped: k_sum_parts writes scal[0..3] here,
                                 // then [4] = its running count of solves, scal[5])
    double solve_seq = 0.0;      // solves the host has seen completed (h_pinned[4])
    int64_t solves_enqueued = 0; // solves enqueued on the stream (k_sum_parts' count once they are done)
    double* d_hpinned = nullptr; // its device address

    // state
    bool have_lin = false;       // d_J holds a linearisation
    bool solved = false;         // this accumulation's solve enqueued (S holds its factor now)
    bool force_sync = false;     // FBA_SYNC=1 at creation: wait for a solve by hipStreamSynchronize
    bool have_delta = false;
    bool have_factor = false;    // d_S holds the factor of the last solve (fba_covariance consumes it)
    bool pending = false;        // fba_solve_update_async enqueued, fba_solve_finish not yet called
    std::vector<int32_t> ref_img_cam;  // [n_img_ref] camera of each EXT image (-1: no observation)
    int iterations = 0;
    bool timing = false;
    // kernel probe (fba_set_probe): HIP events around every launch of one Cholesky kernel
    // (1: k_syrk_multi, the bulk trailing update; 2: k_panel, the diagonal factorisations + panel solves)
    int probe = 0;
    std::vector<hipEvent_t> probe_ev;  // [2*nb]
    int probe_n = 0;
    double probe_flops = 0.0;
    hipEvent_t ev[9] = {};
    double last_ms[8] = {0};
    std::vector<std::pair<void*, size_t>> ws;  // reusable device scratch (fba_covariance), by slot
};


// error helpers
void set_error(const std::string& msg);
#define FBA_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            fba::set_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + \
                           __FILE__ + ":" + std::to_string(__LINE__) + " (" #call ")"); \
            return FBA_ERR_HIP;                                                        \
        }                                                                              \
    } while (0)

// device scratch slot `slot` of at least `bytes` (grown when needed, kept until fba_destroy)
inline int ws_get(Ctx& c, int slot, size_t bytes, void** p) {
    if ((int)c.ws.size() <= slot) c.ws.resize(slot + 1, {nullptr, 0});
    auto& e = c.ws[slot];
    if (e.second < bytes) {
        if (e.first) (void)hipFree(e.first);
        e = {nullptr, 0};
        if (hipMalloc(&e.first, bytes) != hipSuccess) { set_error("hipMalloc failed (workspace)"); return FBA_ERR_HIP; }
        e.second = bytes;
    }
    *p = e.first;
    return FBA_OK;
}

// kernel launchers (fba_kernels.hip / fba_chol.hip)
std::vector<int32_t> camera_order(const fba_problem* p);  // internal image slot -> EXT row or -1 (fba_order.cpp)
void build_schedule(Ctx& c, const std::vector<std::pair<int32_t, int32_t>>& pairs);  // pairs: (e1, e2) slots, e1 > e2
int launch_params(Ctx& c, const double* x = nullptr, double* copy_to = nullptr);  // x: parameters (default d_xfull),
                                                                                   // also copied to copy_to
int launch_linearize(Ctx& c, const double* x = nullptr);  // Jacobian rows to d_J (residuals, dense AwG)
int launch_linearize_range(Ctx& c, const double* x, int64_t c0, int64_t c1);  // chunks [c0, c1) only
// general tie points (fba_general.hip): Jacobian rows of their observations + point tables
// (gen_tables), their partials (gen_keys), the blocks only they touch (gen_reduce, after
// launch_accumulate), back-substitution (gen_backsub), tie variances (gen_cov, fba_cov.hip)
int launch_gen_tables(Ctx& c, const double* x);
int launch_gen_keys(Ctx& c);
int launch_gen_reduce(Ctx& c);
int launch_gen_backsub(Ctx& c);
int launch_gen_cov(Ctx& c, const double* Z, const double* Wz, int nz, double* pdiag);
int launch_accumulate(Ctx& c, bool zeroed = false);  // zero S (unless zeroed), image, pair, camera blocks
int launch_border(Ctx& c);       // alpha, G G^T border, RHS rows
int chol_setup(Ctx& c);
int acc_setup(Ctx& c);            // kernel attributes of the accumulation kernels          // one-time kernel attributes, streams, events
int launch_pack(Ctx& c, int dir);  // multi-rank compact reduce buffer: 0 = S -> buffer, 1 = buffer -> S
int launch_cholesky(Ctx& c, int part = 0);  // factor + forward solve of RHS rows (split: 0 subtrees, 1 top)
int launch_pack_split(Ctx& c, int dir);      // subtree split's reduce buffer: 0 pack, 1 unpack + weights,
                                             // 2 the top rows' accumulated diagonal
int launch_backward(Ctx& c);     // border combine + backward solve -> delta_c
int launch_backsub_update(Ctx& c);
int launch_residuals(Ctx& c);    // v per obs, partial sums
int launch_build_rsd(Ctx& c, const double* d_v, const double* d_xpyp, double* d_rsd);  // BuildRSD for a given v
int launch_covariance(Ctx& c, double* d_cdiag, double* d_pdiag, double* d_iblk, const int32_t* d_islot,
                      const int32_t* d_icam, int n_iblk);  // post-fit covariance (fba_cov.hip)
int launch_dense_awg(Ctx& c, double* dA, double* dG, const int64_t* d_map, int64_t n_rows, int64_t u_ref);
int border_solve_selftest(int device, const double* gram, double* coef);  // fba_test_border_solve

}  // namespace fba
