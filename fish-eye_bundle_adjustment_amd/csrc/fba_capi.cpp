// fba_capi.cpp -- the extern "C" boundary of libfba.so (include/fba.h).
//
// Host side of the device-resident Gauss-Newton loop: validates the packed problem, builds the
// observation orderings (tie observations grouped by point, CSR lists per image, co-visible image
// pairs), allocates device memory once, and drives the kernels of fba_kernels.hip / fba_chol.hip.
// The loop semantics are the reference's main.m:407-494; the unknown layout is Buildxhat.m:6-134.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <map>
#include <numeric>
#include <tuple>

#include "fba_internal.h"

namespace fba {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

template <typename T>
static int dalloc(T** p, size_t n) {
    if (n == 0) n = 1;
    FBA_HIP(hipMalloc((void**)p, n * sizeof(T)));
    return FBA_OK;
}
template <typename T>
static int upload(T** p, const std::vector<T>& v) {
    int rc = dalloc(p, v.size());
    if (rc) return rc;
    if (!v.empty()) FBA_HIP(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return FBA_OK;
}

static int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

static int check_settings(const fba_settings* s) {
    if (!s) { set_error("settings is NULL"); return FBA_ERR_ARG; }
    if (s->type < 0 || s->type > 4) { set_error("BuildAwG, invalid type in data.settings.type"); return FBA_ERR_TYPE; }
    if (s->num_radial < 1) {
        // BuildAwG.m:18-20 clamps a local copy to 1 but Buildxhat.m:13 does not: with 0 the reference
        // indexes an empty K (radial not estimated) or misaligns columns (estimated).
        set_error("Num_Radial_Distortions must be >= 1");
        return FBA_ERR_UNSUPPORTED;
    }
    if (s->num_radial > FBA_NK_MAX) { set_error("Num_Radial_Distortions > FBA_NK_MAX"); return FBA_ERR_UNSUPPORTED; }
    if (!(s->meas_std_x > 0) || !(s->meas_std_y > 0)) { set_error("Meas_std must be > 0"); return FBA_ERR_ARG; }
    if (s->inner_constraints &&
        !(s->est_Xc && s->est_Yc && s->est_Zc && s->est_omega && s->est_phi && s->est_kappa)) {
        // BuildAwG.m:525 writes 6 rows per image: the reference assumes all EOPs are estimated
        set_error("Inner_Constraints requires all six EOPs to be estimated (BuildAwG.m:525)");
        return FBA_ERR_UNSUPPORTED;
    }
    return FBA_OK;
}

// n_slots: internal image slots (the EXT images in camera order plus padding slots, fba_order.cpp)
static void compute_layout(const fba_problem* p, const fba_settings* s, Layout& L, int n_slots) {
    L.n_img = n_slots;
    L.n_img_ref = p->n_img;
    L.n_cam = p->n_cam;
    L.n_tie = p->n_tie;
    L.nk = s->num_radial;
    L.cw = 5 + L.nk;
    L.u_c = 6 * (int64_t)L.n_img + (int64_t)L.cw * L.n_cam;
    L.u_full = L.u_c + 3 * (int64_t)L.n_tie;
    L.n_pad = round_up(std::max<int64_t>(L.u_c, 1), NB);
    L.ld = L.n_pad;
    L.nrhs = s->inner_constraints ? 15 : 1;
    L.u_img = s->est_Xc + s->est_Yc + s->est_Zc + s->est_omega + s->est_phi + s->est_kappa;
    L.u_cam = s->est_c + s->est_xp + s->est_yp + s->est_radial * s->num_radial + s->est_decent * 2;
    L.u_ref = (int64_t)L.u_img * L.n_img_ref + (int64_t)L.u_cam * L.n_cam + 3 * (int64_t)L.n_tie;
}

// full (internal) index -> the reference's xhat index.  Internal image slot e is EXT row img_ord[e]
// (-1: a padding slot, no reference unknowns).
static void full_to_ref_map(const fba_settings* s, const Layout& L, const std::vector<int32_t>& img_ord,
                            std::vector<int64_t>& map) {
    map.assign(L.u_full, -1);
    const int ee[6] = {s->est_Xc, s->est_Yc, s->est_Zc, s->est_omega, s->est_phi, s->est_kappa};
    for (int e = 0; e < L.n_img; ++e) {
        if (img_ord[e] < 0) continue;
        int cnt = 0;
        for (int a = 0; a < 6; ++a)
            if (ee[a]) map[6 * (int64_t)e + a] = (int64_t)img_ord[e] * L.u_img + cnt++;
    }
    std::vector<int> ce(L.cw, 0);
    ce[0] = s->est_xp;
    ce[1] = s->est_yp;
    ce[2] = s->est_c;
    for (int j = 0; j < L.nk; ++j) ce[3 + j] = s->est_radial;
    ce[3 + L.nk] = ce[4 + L.nk] = s->est_decent;
    for (int k = 0; k < L.n_cam; ++k) {
        int cnt = 0;
        for (int c = 0; c < L.cw; ++c)
            if (ce[c]) map[6 * (int64_t)L.n_img + (int64_t)k * L.cw + c] = (int64_t)L.u_img * L.n_img_ref + (int64_t)k * L.u_cam + cnt++;
    }
    const int64_t tb = (int64_t)L.u_img * L.n_img_ref + (int64_t)L.u_cam * L.n_cam;
    for (int64_t t = 0; t < 3 * (int64_t)L.n_tie; ++t) map[L.u_c + t] = tb + t;
}

static int check_problem(const fba_problem* p, const fba_settings* s) {
    if (!p) { set_error("problem is NULL"); return FBA_ERR_ARG; }
    if (p->n_pts < 0 || p->n_img < 0 || p->n_cam < 0 || p->n_tie < 0) { set_error("negative size"); return FBA_ERR_ARG; }
    if (p->n_pts > 0 && (!p->xy || !p->img || !p->cam || !p->tie || !p->xyz_fixed)) {
        set_error("NULL observation array");
        return FBA_ERR_ARG;
    }
    if ((p->n_img > 0 && !p->eop0) || (p->n_cam > 0 && (!p->iop0 || !p->cam_info)) || (p->n_tie > 0 && !p->tie0)) {
        set_error("NULL parameter array");
        return FBA_ERR_ARG;
    }
    for (int k = 0; k < p->n_cam; ++k) {
        const double yd = p->cam_info[5 * k];
        if (yd != 1.0 && yd != -1.0) { set_error("y_dir should be +-1 only (main.m:334-337)"); return FBA_ERR_ARG; }
    }
    std::vector<int32_t> img_cam(p->n_img, -1);
    for (int64_t i = 0; i < p->n_pts; ++i) {
        const int e = p->img[i], k = p->cam[i], t = p->tie[i];
        if (e < 0 || e >= p->n_img) { set_error("image index out of range (EXT must list the images of .pho in order)"); return FBA_ERR_ARG; }
        if (k < 0 || k >= p->n_cam) { set_error("camera index out of range"); return FBA_ERR_ARG; }
        if (t < -1 || t >= p->n_tie) { set_error("tie index out of range"); return FBA_ERR_ARG; }
        // an image's camera is its EXT row's (main.m:323): every observation of it goes through that camera
        if (img_cam[e] < 0) img_cam[e] = k;
        else if (img_cam[e] != k) { set_error("observations of one image with different cameras"); return FBA_ERR_ARG; }
    }
    (void)s;
    return FBA_OK;
}

// contiguous tie ranges balanced by observation count; control observations by contiguous ranges
static void partition(const fba_problem* p, int world, std::vector<int32_t>& tie_owner, std::vector<int32_t>& ctl_owner) {
    tie_owner.assign(p->n_tie, 0);
    ctl_owner.assign(p->n_pts, -1);
    std::vector<int64_t> cnt(p->n_tie, 0);
    int64_t n_ctl = 0;
    for (int64_t i = 0; i < p->n_pts; ++i) {
        if (p->tie[i] >= 0) cnt[p->tie[i]]++;
        else n_ctl++;
    }
    const int64_t n_tie_obs = p->n_pts - n_ctl;
    int64_t acc = 0;
    for (int t = 0; t < p->n_tie; ++t) {
        // owner = floor(world * (obs before the middle of this point) / total)
        const int64_t mid2 = 2 * acc + cnt[t];
        int r = n_tie_obs > 0 ? (int)((mid2 * world) / (2 * n_tie_obs)) : 0;
        tie_owner[t] = std::min(std::max(r, 0), world - 1);
        acc += cnt[t];
    }
    int64_t q = 0;
    for (int64_t i = 0; i < p->n_pts; ++i) {
        if (p->tie[i] >= 0) continue;
        ctl_owner[i] = n_ctl > 0 ? (int32_t)std::min<int64_t>((q * world) / n_ctl, world - 1) : 0;
        ++q;
    }
}

static void destroy(Ctx* c) {
    if (!c) return;
    void* ptrs[] = {c->d_chunk_obs, c->d_chunk_pt, c->d_xy, c->d_img, c->d_cam, c->d_pt, c->d_ctl, c->d_lp_tie, c->d_xoff, c->d_lrt, c->d_lp_start, c->d_lp_cam,
                    c->d_acc, c->d_ppart, c->d_U, c->d_ipart, c->d_cpart, c->d_cseg, c->d_bscr, c->d_gblk, c->d_lrprof, c->d_ptrace, c->d_gpairs, c->d_red, c->d_xfull, c->d_xlin, c->d_delta, c->d_img_tab, c->d_cam_tab, c->d_G, c->d_J, c->d_WT,
                    c->d_pt_tab, c->d_P, c->d_flags, c->d_S, c->d_X, c->d_dinv, c->d_linv, c->d_scal, c->d_part, c->d_res, c->d_caminfo,
                    c->d_active, c->d_counted, c->d_obs_pho, c->d_sched, c->d_gpt, c->d_gcu, c->d_gug, c->d_xpart,
                    c->d_kpart, c->d_bown, c->d_rown, c->d_topdiag};
    for (void* q : ptrs)
        if (q) (void)hipFree(q);
    for (auto& w : c->ws)
        if (w.first) (void)hipFree(w.first);
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : c->probe_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto g : c->graph)
        if (g) (void)hipGraphExecDestroy(g);

    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

static int create(const fba_problem* p, const fba_settings* s, const fba_options* o, Ctx** out) {
    int rc = check_settings(s);
    if (rc) return rc;
    rc = check_problem(p, s);
    if (rc) return rc;
    fba_options opt{};
    opt.world = 1;
    if (o) opt = *o;
    if (opt.world < 1 || opt.rank < 0 || opt.rank >= opt.world) { set_error("bad rank/world"); return FBA_ERR_ARG; }

    Ctx* c = new Ctx();
    c->prob = *p;
    c->set = *s;
    c->opt = opt;
    c->force_sync = getenv("FBA_SYNC") && atoi(getenv("FBA_SYNC")) != 0;  // (read per context)
    c->n_pts = p->n_pts;
    Layout& L = c->L;
    // camera-side order of the images: nested dissection with padding slots (fba_order.cpp)
    c->img_ord = camera_order(p);
    compute_layout(p, s, L, (int)c->img_ord.size());
    c->img_new.assign(L.n_img_ref, 0);
    for (int e = 0; e < L.n_img; ++e)
        if (c->img_ord[e] >= 0) c->img_new[c->img_ord[e]] = e;
    full_to_ref_map(s, L, c->img_ord, c->full_to_ref);
    c->ref_img_cam.assign(L.n_img_ref, -1);
    for (int64_t i = 0; i < p->n_pts; ++i) c->ref_img_cam[p->img[i]] = p->cam[i];

    FBA_HIP(hipSetDevice(opt.device));
    c->device = opt.device;
    if (opt.stream) {
        c->stream = (hipStream_t)opt.stream;
    } else {
        FBA_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }

    // initial full-space parameters
    c->xfull0.assign(L.u_full, 0.0);
    for (int e = 0; e < L.n_img; ++e)
        if (c->img_ord[e] >= 0)
            for (int a = 0; a < 6; ++a) c->xfull0[6 * (int64_t)e + a] = p->eop0[6 * (int64_t)c->img_ord[e] + a];
    for (int64_t i = 0; i < (int64_t)L.cw * L.n_cam; ++i) c->xfull0[6 * (int64_t)L.n_img + i] = p->iop0[i];
    for (int64_t i = 0; i < 3 * (int64_t)L.n_tie; ++i) c->xfull0[L.u_c + i] = p->tie0[i];

    // the co-visible image pairs of ALL tie points (identical on every rank): the compact reduce
    // buffer of ranks > 1 and the block envelope of the reduced system
    std::vector<std::pair<int32_t, int32_t>> gp;
    {
        std::vector<std::pair<int32_t, int32_t>> pi;  // (tie, internal image)
        for (int64_t i = 0; i < p->n_pts; ++i)
            if (p->tie[i] >= 0) pi.emplace_back(p->tie[i], c->img_new[p->img[i]]);
        std::sort(pi.begin(), pi.end());
        for (size_t a = 0; a < pi.size();) {
            size_t b = a;
            while (b < pi.size() && pi[b].first == pi[a].first) ++b;
            for (size_t x = a; x < b; ++x)
                for (size_t y = a; y < b; ++y)
                    if (pi[x].second > pi[y].second) gp.emplace_back(pi[x].second, pi[y].second);
            a = b;
        }
        std::sort(gp.begin(), gp.end());
        gp.erase(std::unique(gp.begin(), gp.end()), gp.end());
        // inner constraints: the border is applied on the first n_loc image slots only (local
        // border), so M keeps the sparsity of S
        c->n_loc = s->inner_constraints ? std::min<int>(L.n_img, (int)(NB / 6)) : 0;
        build_schedule(*c, gp);
    }
    const bool split = c->sched.split;

    // shard
    std::vector<int32_t> ctl_owner;
    if (!split) {
        partition(p, opt.world, c->tie_owner, ctl_owner);
    } else {
        // subtree split: a point's images lie on one root path of the elimination tree (every two of them
        // share a block of S), so at most one rank's subtree: the point goes to that rank; points of top
        // images only (and control observations of top images) go to the least loaded rank
        const std::vector<int32_t>& br = c->sched.blk_rank;
        auto img_rank = [&](int64_t e) {  // EXT image -> rank of its rows' subtree, or -1
            const int64_t slot = c->img_new[e];
            int r = -1;
            for (int64_t blk = 6 * slot / NB; blk <= (6 * slot + 5) / NB; ++blk) r = std::max(r, (int)br[blk]);
            return r;
        };
        std::vector<int64_t> load(opt.world, 0);
        std::vector<int32_t> tr(L.n_tie, -1);
        std::vector<int64_t> tcnt(L.n_tie, 0);
        for (int64_t i = 0; i < p->n_pts; ++i)
            if (p->tie[i] >= 0) {
                tr[p->tie[i]] = std::max(tr[p->tie[i]], img_rank(p->img[i]));
                tcnt[p->tie[i]]++;
            }
        c->tie_owner.assign(L.n_tie, 0);
        for (int t = 0; t < L.n_tie; ++t)
            if (tr[t] >= 0) { c->tie_owner[t] = tr[t]; load[tr[t]] += tcnt[t]; }
        for (int t = 0; t < L.n_tie; ++t)
            if (tr[t] < 0) {
                const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                c->tie_owner[t] = r;
                load[r] += tcnt[t];
            }
        ctl_owner.assign(p->n_pts, -1);
        for (int64_t i = 0; i < p->n_pts; ++i)
            if (p->tie[i] < 0) {
                int r = img_rank(p->img[i]);
                if (r < 0) r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                ctl_owner[i] = r;
                load[r]++;
            }
    }

    // local tie points sorted by camera; their observations in PHO order
    std::vector<std::vector<int64_t>> tie_obs(L.n_tie);
    std::vector<int32_t> tie_cam(L.n_tie, 0);
    for (int64_t i = 0; i < p->n_pts; ++i)
        if (p->tie[i] >= 0) {
            tie_obs[p->tie[i]].push_back(i);
            tie_cam[p->tie[i]] = p->cam[i];
        }
    // regular tie points (k_lin_reduce's chunks): one camera, <= CHUNK_OBS observations, at most one per
    // image; the others are "general" points (fba_general.hip) -- the reference accepts all of them
    auto is_general = [&](int t) {
        const std::vector<int64_t>& ob = tie_obs[t];
        if ((int64_t)ob.size() > CHUNK_OBS) return true;
        std::vector<int32_t> im;
        for (int64_t i : ob) {
            if (p->cam[i] != p->cam[ob[0]]) return true;
            im.push_back(p->img[i]);
        }
        std::sort(im.begin(), im.end());
        return std::adjacent_find(im.begin(), im.end()) != im.end();
    };
    std::vector<int32_t> lps, gps;
    for (int t = 0; t < L.n_tie; ++t)
        if (c->tie_owner[t] == opt.rank && !tie_obs[t].empty()) (is_general(t) ? gps : lps).push_back(t);
    // within a camera, points in Morton (Z-curve) order of their initial coordinates: the points two
    // co-visible images share -- and so the W/T and Jacobian rows a pair or an image gathers -- sit
    // close together in memory
    std::vector<uint64_t> zkey(L.n_tie, 0);
    {
        double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
        for (int32_t t : lps)
            for (int d = 0; d < 3; ++d) {
                lo[d] = std::min(lo[d], p->tie0[3 * (int64_t)t + d]);
                hi[d] = std::max(hi[d], p->tie0[3 * (int64_t)t + d]);
            }
        auto spread = [](uint64_t v) {  // 21 bits -> every third bit
            v &= 0x1fffff;
            v = (v | v << 32) & 0x1f00000000ffffULL;
            v = (v | v << 16) & 0x1f0000ff0000ffULL;
            v = (v | v << 8) & 0x100f00f00f00f00fULL;
            v = (v | v << 4) & 0x10c30c30c30c30c3ULL;
            v = (v | v << 2) & 0x1249249249249249ULL;
            return v;
        };
        for (int32_t t : lps) {
            uint64_t k = 0;
            for (int d = 0; d < 3; ++d) {
                const double span = hi[d] > lo[d] ? hi[d] - lo[d] : 1.0;
                double f = (p->tie0[3 * (int64_t)t + d] - lo[d]) / span;
                f = std::isfinite(f) ? std::min(std::max(f, 0.0), 1.0) : 0.0;
                k |= spread((uint64_t)(f * 2097151.0)) << d;
            }
            zkey[t] = k;
        }
    }
    // default: lexicographic order of the points' (sorted) image sets -- consecutive points share most
    // of their co-visible pairs, so the rows k_pairs gathers for one pair sit close together
    {
        std::vector<std::vector<int32_t>> iset(L.n_tie);
        for (int32_t t : lps) {
            for (int64_t i : tie_obs[t]) iset[t].push_back(c->img_new[p->img[i]]);
            std::sort(iset[t].begin(), iset[t].end());
        }
        std::stable_sort(lps.begin(), lps.end(), [&](int32_t a, int32_t b) {
            if (tie_cam[a] != tie_cam[b]) return tie_cam[a] < tie_cam[b];
            if (iset[a] != iset[b]) return iset[a] < iset[b];
            return zkey[a] < zkey[b];
        });
    }
    c->n_lp = (int64_t)lps.size();

    std::vector<double> xy;
    std::vector<int32_t> img, cam, pt, lp_start, lp_cam;
    std::vector<double> ctl;
    std::vector<int64_t>& pho = c->obs_pho;
    lp_start.push_back(0);
    for (int64_t lp = 0; lp < c->n_lp; ++lp) {
        const int t = lps[lp];
        for (int64_t i : tie_obs[t]) {
            pho.push_back(i);
            xy.push_back(p->xy[2 * i]);
            xy.push_back(p->xy[2 * i + 1]);
            img.push_back(c->img_new[p->img[i]]);
            cam.push_back(p->cam[i]);
            pt.push_back((int32_t)lp);
        }
        lp_start.push_back((int32_t)pho.size());
        lp_cam.push_back(tie_cam[t]);
    }
    c->n_obs_tie = (int64_t)pho.size();
    // control observations of this rank, sorted by camera (stable in PHO order)
    std::vector<int64_t> ctls;
    for (int64_t i = 0; i < p->n_pts; ++i)
        if (p->tie[i] < 0 && ctl_owner[i] == opt.rank) ctls.push_back(i);
    std::stable_sort(ctls.begin(), ctls.end(), [&](int64_t a, int64_t b) { return p->cam[a] < p->cam[b]; });
    for (size_t q = 0; q < ctls.size(); ++q) {
        const int64_t i = ctls[q];
        pho.push_back(i);
        xy.push_back(p->xy[2 * i]);
        xy.push_back(p->xy[2 * i + 1]);
        img.push_back(c->img_new[p->img[i]]);
        cam.push_back(p->cam[i]);
        pt.push_back(-1 - (int32_t)q);
        for (int m = 0; m < 3; ++m) ctl.push_back(p->xyz_fixed[3 * i + m]);
    }
    // the general points' observations, after the control observations: each point's contiguous,
    // sorted by image slot (then PHO row)
    const int64_t o_gen0 = (int64_t)pho.size();
    std::vector<int32_t> g_obs{(int32_t)o_gen0};
    for (size_t q = 0; q < gps.size(); ++q) {
        std::vector<int64_t> ob = tie_obs[gps[q]];
        std::stable_sort(ob.begin(), ob.end(), [&](int64_t a, int64_t b) { return c->img_new[p->img[a]] < c->img_new[p->img[b]]; });
        for (int64_t i : ob) {
            pho.push_back(i);
            xy.push_back(p->xy[2 * i]);
            xy.push_back(p->xy[2 * i + 1]);
            img.push_back(c->img_new[p->img[i]]);
            cam.push_back(p->cam[i]);
            pt.push_back((int32_t)(c->n_lp + (int64_t)q));
        }
        g_obs.push_back((int32_t)pho.size());
    }
    c->n_obs = (int64_t)pho.size();
    if (c->n_obs >= (int64_t)1 << 31) { set_error("too many observations per rank"); destroy(c); return FBA_ERR_UNSUPPORTED; }
    c->n_obs_pad = round_up(std::max<int64_t>(c->n_obs, 1), 64);
    c->n_lp_pad = round_up(std::max<int64_t>(c->n_lp, 1), 64);

    // chunks (one k_lin_reduce / k_lin_point workgroup each): consecutive whole tie points of one
    // camera, <= CHUNK_OBS observations and <= chunk_pts(nK) points, then control observations of one
    // camera, <= CHUNK_OBS at a time
    std::vector<int32_t> chunk_obs{0}, chunk_pt{0};
    int64_t cur_terms = 0;
    for (int64_t lp = 0; lp < c->n_lp; ++lp) {
        const int64_t n_lp_obs = lp_start[lp + 1] - lp_start[lp];
        const int64_t lp_terms = n_lp_obs * (n_lp_obs - 1) / 2;
        const bool split = lp > chunk_pt.back() &&
                           (lp_start[lp + 1] - chunk_obs.back() > CHUNK_OBS || lp - chunk_pt.back() >= chunk_pts(L.nk) ||
                            lp_cam[lp] != lp_cam[lp - 1] || cur_terms + lp_terms > chunk_terms(L.nk));
        if (split) {
            chunk_obs.push_back(lp_start[lp]);
            chunk_pt.push_back((int32_t)lp);
            cur_terms = 0;
        }
        cur_terms += lp_terms;
    }
    if (c->n_lp > 0) {
        chunk_obs.push_back(lp_start[c->n_lp]);
        chunk_pt.push_back((int32_t)c->n_lp);
    }
    for (int64_t o = c->n_obs_tie; o < o_gen0;) {
        int64_t e = o + 1;
        while (e < o_gen0 && e - o < CHUNK_OBS && cam[e] == cam[o]) ++e;
        chunk_obs.push_back((int32_t)e);
        chunk_pt.push_back((int32_t)c->n_lp);
        o = e;
    }
    c->n_chunks_lr = (int64_t)chunk_obs.size() - 1;
    // the general observations: linearised by k_lin_point only (empty point range), CHUNK_OBS at a time
    for (int64_t o = o_gen0; o < c->n_obs;) {
        const int64_t e = std::min<int64_t>(o + CHUNK_OBS, c->n_obs);
        chunk_obs.push_back((int32_t)e);
        chunk_pt.push_back((int32_t)c->n_lp);
        o = e;
    }
    c->n_chunks = (int64_t)chunk_obs.size() - 1;

    // accumulation plan (k_lin_reduce): per chunk its co-visible pair keys with their (i, j)
    // observation terms and its image keys with their observations; per pair / image / camera the
    // partial slots the reduce kernels add up, in chunk order
    AccPlan& A = c->acc;
    std::vector<int32_t> ck_cam, ck_pk{0}, pk_t{0}, pk_term, ck_ik{0}, ik_o{0}, ik_obs, ck_tm;
    std::vector<std::pair<int32_t, int32_t>> pk_key;
    std::vector<int32_t> ik_img;
    // a chunk's pair terms take the U-row path (AccPlan::ck_tm) when its pair keys hold at most tm_ratio
    // terms each on average: a partial row costs 288 B written and read back per key, the U-row path
    // one 144-B U row per observation plus two cached U-row reads per term (FBA_PAIR_TERMS: the ratio;
    // 0 = never, tested both ways in tests/test_gpu_parity.py)
    const double tm_ratio = getenv("FBA_PAIR_TERMS") ? atof(getenv("FBA_PAIR_TERMS")) : 2.0;
    std::vector<std::array<int32_t, 4>> tterm;  // (e1, e2, a, b) of the U-row chunks' terms, chunk order
    for (int64_t ch = 0; ch < c->n_chunks_lr; ++ch) {
        const int o0 = chunk_obs[ch], o1 = chunk_obs[ch + 1];
        ck_cam.push_back(cam[o0]);
        std::vector<std::tuple<int32_t, int32_t, int32_t>> tk;  // (e1, e2, term), e1 > e2, point order
        for (int32_t lp = chunk_pt[ch]; lp < chunk_pt[ch + 1]; ++lp)
            for (int i = lp_start[lp]; i < lp_start[lp + 1]; ++i)
                for (int j = lp_start[lp]; j < lp_start[lp + 1]; ++j) {
                    if (img[i] == img[j]) {
                        if (i != j) {
                            set_error("a tie point is measured twice in one image: not implemented in this build");
                            destroy(c);
                            return FBA_ERR_UNSUPPORTED;
                        }
                        continue;
                    }
                    if (img[i] > img[j]) tk.emplace_back(img[i], img[j], (i - o0) | ((j - o0) << 16));
                }
        std::stable_sort(tk.begin(), tk.end(), [](const auto& x, const auto& y) {
            return std::get<0>(x) != std::get<0>(y) ? std::get<0>(x) < std::get<0>(y) : std::get<1>(x) < std::get<1>(y);
        });
        // the chunk's pair keys, most terms first: the threads of a wave then run similar trip counts
        std::vector<std::pair<size_t, size_t>> kr;  // [begin, end) in tk
        for (size_t q = 0; q < tk.size(); ++q)
            if (q == 0 || std::get<0>(tk[q]) != std::get<0>(tk[q - 1]) || std::get<1>(tk[q]) != std::get<1>(tk[q - 1]))
                kr.emplace_back(q, q + 1);
            else
                kr.back().second = q + 1;
        std::stable_sort(kr.begin(), kr.end(), [](const auto& x, const auto& y) { return x.second - x.first > y.second - y.first; });
        const bool tmode = !kr.empty() && (double)tk.size() <= tm_ratio * (double)kr.size();
        ck_tm.push_back(tmode ? 1 : 0);
        if (tmode) {
            for (size_t q = 0; q < tk.size(); ++q) {  // (e1, e2) ascending, point order within a key
                const int32_t tm = std::get<2>(tk[q]);
                tterm.push_back({std::get<0>(tk[q]), std::get<1>(tk[q]), o0 + (tm & 0xffff), o0 + (tm >> 16)});
            }
        } else {
            for (auto& r : kr) {
                pk_key.emplace_back(std::get<0>(tk[r.first]), std::get<1>(tk[r.first]));
                for (size_t q = r.first; q < r.second; ++q) pk_term.push_back(std::get<2>(tk[q]));
                pk_t.push_back((int32_t)pk_term.size());
            }
        }
        ck_pk.push_back((int32_t)pk_key.size());
        std::vector<std::pair<int32_t, int32_t>> io;  // (image, local obs)
        for (int o = o0; o < o1; ++o) io.emplace_back(img[o], o - o0);
        std::sort(io.begin(), io.end());
        for (size_t q = 0; q < io.size(); ++q) {
            if (q == 0 || io[q].first != io[q - 1].first) {
                if (q > 0) ik_o.push_back((int32_t)ik_obs.size());
                ik_img.push_back(io[q].first);
            }
            ik_obs.push_back(io[q].second);
        }
        if (!io.empty()) ik_o.push_back((int32_t)ik_obs.size());
        ck_ik.push_back((int32_t)ik_img.size());
    }
    // image-key lanes of k_lin_reduce: 4 when the chunks' image keys hold <= 2 observations on average
    c->ik_lanes = (ck_ik.back() > 0 && ik_obs.size() <= 2 * (size_t)ck_ik.back()) ? 4 : 8;
    // general points: gimg / gpc groups and their keys, appended after the chunks' keys
    GenPlan& G = c->gen;
    G.n_gp = (int64_t)gps.size();
    G.lp0 = c->n_lp;
    G.pk0 = (int64_t)pk_key.size();
    G.ik0 = (int64_t)ik_img.size();
    G.ck0 = c->n_chunks_lr;
    std::vector<int32_t> g_gi{0}, g_gc{0}, gi_obs, gi_img, gi_gp, gi_gc, gc_cam, gc_gp, gc_o{0}, gc_list, gpk, gx, gkk;
    std::map<std::pair<int32_t, int32_t>, std::vector<int32_t>> xt, kt;  // target block -> slots, ascending
    for (int64_t q = 0; q < G.n_gp; ++q) {
        const int a = g_obs[q], b = g_obs[q + 1];
        const int gi0 = (int)gi_img.size(), gc0 = (int)gc_cam.size();
        for (int o = a; o < b; ++o)
            if (o == a || img[o] != img[o - 1]) {
                gi_obs.push_back(o);
                gi_img.push_back(img[o]);
                gi_gp.push_back((int32_t)q);
            }
        std::vector<int32_t> cams;
        for (int o = a; o < b; ++o) cams.push_back(cam[o]);
        std::sort(cams.begin(), cams.end());
        cams.erase(std::unique(cams.begin(), cams.end()), cams.end());
        for (int32_t k : cams) {
            gc_cam.push_back(k);
            gc_gp.push_back((int32_t)q);
            for (int o = a; o < b; ++o)
                if (cam[o] == k) gc_list.push_back(o);
            gc_o.push_back((int32_t)gc_list.size());
        }
        const int gi1 = (int)gi_img.size(), gc1 = (int)gc_cam.size();
        for (int i = gi0; i < gi1; ++i) {
            const int32_t own = cam[gi_obs[i]];
            for (int k = gc0; k < gc1; ++k) {
                if (gc_cam[k] == own) gi_gc.push_back(k);
                else {  // image i x another camera of the point
                    xt[{gi_img[i], gc_cam[k]}].push_back((int32_t)(gx.size() / 2));
                    gx.push_back(i);
                    gx.push_back(k);
                }
            }
            for (int j = gi0; j < i; ++j) {  // images ascending: gimg i is the higher image
                gpk.push_back(i);
                gpk.push_back(j);
                pk_key.emplace_back(gi_img[i], gi_img[j]);
            }
            ik_img.push_back(gi_img[i]);
        }
        for (int k1 = gc0; k1 < gc1; ++k1) {
            ck_cam.push_back(gc_cam[k1]);  // camera partial slot ck0 + gpc
            for (int k2 = gc0; k2 < k1; ++k2) {  // cameras ascending: k1 the higher camera
                kt[{gc_cam[k1], gc_cam[k2]}].push_back((int32_t)(gkk.size() / 2));
                gkk.push_back(k1);
                gkk.push_back(k2);
            }
        }
        g_gi.push_back(gi1);
        g_gc.push_back(gc1);
    }
    gi_obs.push_back(c->n_obs);
    G.n_gi = (int64_t)gi_img.size();
    G.n_gc = (int64_t)gc_cam.size();
    G.n_gpk = (int64_t)gpk.size() / 2;
    G.n_gx = (int64_t)gx.size() / 2;
    G.n_gkk = (int64_t)gkk.size() / 2;
    std::vector<int32_t> xt_start{0}, xt_list, xt_key, kt_start{0}, kt_list, kt_key;
    for (auto& e : xt) {
        xt_key.push_back(e.first.first);
        xt_key.push_back(e.first.second);
        xt_list.insert(xt_list.end(), e.second.begin(), e.second.end());
        xt_start.push_back((int32_t)xt_list.size());
    }
    for (auto& e : kt) {
        kt_key.push_back(e.first.first);
        kt_key.push_back(e.first.second);
        kt_list.insert(kt_list.end(), e.second.begin(), e.second.end());
        kt_start.push_back((int32_t)kt_list.size());
    }
    G.n_xt = (int64_t)xt.size();
    G.n_kt = (int64_t)kt.size();
    // the local co-visible pairs and, per pair, its partial slots
    std::vector<std::pair<int32_t, int32_t>> lpairs(pk_key);
    for (auto& t : tterm) lpairs.emplace_back(t[0], t[1]);
    std::sort(lpairs.begin(), lpairs.end());
    lpairs.erase(std::unique(lpairs.begin(), lpairs.end()), lpairs.end());
    c->n_pairs = (int64_t)lpairs.size();
    c->n_pair_terms = (int64_t)(pk_term.size() + tterm.size());
    // the U-row terms per pair (counting sort by pair: chunk order kept)
    std::vector<int32_t> tp_start(c->n_pairs + 1, 0), tp_ab(2 * tterm.size());
    {
        std::vector<int32_t> pid(tterm.size());
        for (size_t q = 0; q < tterm.size(); ++q) {
            pid[q] = (int32_t)(std::lower_bound(lpairs.begin(), lpairs.end(), std::make_pair(tterm[q][0], tterm[q][1])) -
                               lpairs.begin());
            tp_start[pid[q] + 1]++;
        }
        for (int64_t q = 0; q < c->n_pairs; ++q) tp_start[q + 1] += tp_start[q];
        std::vector<int32_t> fill(tp_start.begin(), tp_start.end() - 1);
        for (size_t q = 0; q < tterm.size(); ++q) {
            const int32_t x = fill[pid[q]]++;
            tp_ab[2 * x] = tterm[q][2];
            tp_ab[2 * x + 1] = tterm[q][3];
        }
    }
    std::vector<int32_t> rp_start(c->n_pairs + 1, 0), rp_list(pk_key.size()), rp_e;
    {
        std::vector<int32_t> pid(pk_key.size());
        for (size_t q = 0; q < pk_key.size(); ++q) {
            pid[q] = (int32_t)(std::lower_bound(lpairs.begin(), lpairs.end(), pk_key[q]) - lpairs.begin());
            rp_start[pid[q] + 1]++;
        }
        for (int64_t q = 0; q < c->n_pairs; ++q) rp_start[q + 1] += rp_start[q];
        std::vector<int32_t> fill(rp_start.begin(), rp_start.end() - 1);
        for (size_t q = 0; q < pk_key.size(); ++q) rp_list[fill[pid[q]]++] = (int32_t)q;
        for (auto& q : lpairs) { rp_e.push_back(q.first); rp_e.push_back(q.second); }
    }
    std::vector<int32_t> ri_start(L.n_img + 1, 0), ri_list(ik_img.size()), img_cam(L.n_img, -1);
    {
        for (int32_t e : ik_img) ri_start[e + 1]++;
        for (int e = 0; e < L.n_img; ++e) ri_start[e + 1] += ri_start[e];
        std::vector<int32_t> fill(ri_start.begin(), ri_start.end() - 1);
        for (size_t q = 0; q < ik_img.size(); ++q) ri_list[fill[ik_img[q]]++] = (int32_t)q;
        for (int64_t o = 0; o < c->n_obs; ++o) img_cam[img[o]] = cam[o];
    }
    // camera partial slots: the chunks', then one per general point-camera group (ck_cam covers both)
    std::vector<int32_t> rc_start(L.n_cam + 1, 0), rc_list(ck_cam.size());
    {
        for (int32_t k : ck_cam) rc_start[k + 1]++;
        for (int k = 0; k < L.n_cam; ++k) rc_start[k + 1] += rc_start[k];
        std::vector<int32_t> fill(rc_start.begin(), rc_start.end() - 1);
        for (size_t ch = 0; ch < ck_cam.size(); ++ch) rc_list[fill[ck_cam[ch]]++] = (int32_t)ch;
    }
    A.n_pk = (int64_t)pk_key.size();
    A.n_ik = (int64_t)ik_img.size();
    A.n_tt = (int64_t)tterm.size();
    std::vector<int32_t> abuf;
    auto put = [&](const std::vector<int32_t>& v) {
        const int64_t off = (int64_t)abuf.size();
        abuf.insert(abuf.end(), v.begin(), v.end());
        return off;
    };
    A.ck_cam = put(ck_cam);
    A.ck_pk = put(ck_pk);
    A.pk_t = put(pk_t);
    A.pk_term = put(pk_term);
    A.ck_ik = put(ck_ik);
    A.ik_o = put(ik_o);
    A.ik_obs = put(ik_obs);
    A.rp_start = put(rp_start);
    A.rp_e = put(rp_e);
    A.rp_list = put(rp_list);
    A.ri_start = put(ri_start);
    A.ri_list = put(ri_list);
    {
        std::vector<int32_t> pk_slot(rp_list.size()), ik_slot(ri_list.size());
        for (size_t x = 0; x < rp_list.size(); ++x) pk_slot[rp_list[x]] = (int32_t)x;
        for (size_t x = 0; x < ri_list.size(); ++x) ik_slot[ri_list[x]] = (int32_t)x;
        A.pk_slot = put(pk_slot);
        A.ik_slot = put(ik_slot);
        G.pk_slot = A.pk_slot;
        G.ik_slot = A.ik_slot;
    }
    A.img_cam = put(img_cam);
    A.rc_start = put(rc_start);
    A.rc_list = put(rc_list);
    A.ck_tm = put(ck_tm);
    A.tp_start = put(tp_start);
    A.tp_ab = put(tp_ab);
    G.g_obs = put(g_obs);
    G.g_gi = put(g_gi);
    G.g_gc = put(g_gc);
    G.gi_obs = put(gi_obs);
    G.gi_img = put(gi_img);
    G.gi_gp = put(gi_gp);
    G.gi_gc = put(gi_gc);
    G.gc_cam = put(gc_cam);
    G.gc_gp = put(gc_gp);
    G.gc_o = put(gc_o);
    G.gc_list = put(gc_list);
    G.gpk = put(gpk);
    G.gx = put(gx);
    G.gkk = put(gkk);
    G.xt_start = put(xt_start);
    G.xt_list = put(xt_list);
    G.xt_key = put(xt_key);
    G.kt_start = put(kt_start);
    G.kt_list = put(kt_list);
    G.kt_key = put(kt_key);
    std::vector<int32_t> gpairs;
    if (opt.world > 1 && !split) {
        for (auto& q : gp) { gpairs.push_back(q.first); gpairs.push_back(q.second); }
        c->n_gpairs = (int64_t)gp.size();
        c->n_red = 36 * (c->n_gpairs + L.n_img) + (int64_t)L.cw * L.n_cam * L.n_pad + L.n_pad;
    }
    // subtree split: the reduce buffer's layout (k_pack_split) and the per-block roles
    std::vector<int8_t> bown, rown;
    std::vector<int32_t> topdiag;
    if (split) {
        const Sched& sc = c->sched;
        const int64_t nb = L.n_pad / NB;
        bown.assign(nb, 0);
        for (int64_t k = 0; k < nb; ++k) bown[k] = sc.blk_rank[k] < 0 ? 2 : (sc.blk_rank[k] == opt.rank ? 1 : 0);
        rown.assign(L.n_pad, 0);
        for (int64_t i = 0; i < L.n_pad; ++i) {
            rown[i] = bown[i / NB];
            if (i < 6 * (int64_t)L.n_img && c->img_ord[i / 6] >= 0) {
                int r = -1;  // the rank of the image's subtree (any of its rows in one), -1 wholly top
                for (int64_t blk = 6 * (i / 6) / NB; blk <= (6 * (i / 6) + 5) / NB; ++blk) r = std::max(r, (int)sc.blk_rank[blk]);
                rown[i] = r < 0 ? 2 : (r == opt.rank ? 1 : 0);
            }
        }
        int64_t n = 0, ng = 0;
        for (int q = 0; q < sc.n_top_blocks; ++q) n += (int64_t)(sc.buf[sc.top_blocks + 2 * q] == nb ? L.nrhs : NB) * NB;
        for (int64_t i = 0; i < 6 * (int64_t)L.n_img; ++i)
            if (rown[i] == 2) topdiag.push_back((int32_t)i);
        for (int64_t k = 0; k < nb; ++k) ng += bown[k] != 2;
        c->n_topdiag = (int64_t)topdiag.size();
        c->red_diag = n;
        c->red_gblk = c->red_diag + c->n_topdiag;
        c->red_w = c->red_gblk + 256 * ng;
        c->n_red = c->red_w + 9;  // 7 weight sums, the abort flag, the pivot-failure row
    }
    // which full-space entries are estimated / owned / counted
    std::vector<uint8_t> active(L.n_pad, 0), counted(L.u_full, 0);
    c->full_owned.assign(L.u_full, 0);
    for (int64_t i = 0; i < L.u_c; ++i) {
        active[i] = c->full_to_ref[i] >= 0 ? 1 : 0;
        // (split: this rank's subtree rows, and the top rows on rank 0)
        const bool mine = split ? (bown[i / NB] == 1 || (bown[i / NB] == 2 && opt.rank == 0)) : opt.rank == 0;
        counted[i] = (mine && active[i]) ? 1 : 0;
        c->full_owned[i] = mine ? 1 : 0;
    }
    for (int t = 0; t < L.n_tie; ++t)
        for (int m = 0; m < 3; ++m) {
            const int64_t i = L.u_c + 3 * (int64_t)t + m;
            counted[i] = c->tie_owner[t] == opt.rank ? 1 : 0;
            c->full_owned[i] = counted[i];
        }

    // device allocations
    std::vector<int32_t> lp_tie(lps.begin(), lps.end());
    lp_tie.insert(lp_tie.end(), gps.begin(), gps.end());
    std::vector<double> caminfo(p->cam_info, p->cam_info + 5 * (size_t)L.n_cam);
    // k_lin_reduce reads the observation's point coordinates at xfull[xoff] (one gather level fewer than
    // pt -> lp_tie -> xfull, so the next chunk's inputs can be in flight behind the current chunk)
    std::vector<int32_t> xoff(pt.size(), 0);
    for (size_t o = 0; o < pt.size(); ++o)
        if (pt[o] >= 0) xoff[o] = (int32_t)(L.u_c + 3 * (int64_t)lp_tie[pt[o]]);
    if ((rc = upload(&c->d_xoff, xoff)) || (rc = dalloc(&c->d_lrt, 2)) ||
        hipMemset(c->d_lrt, 0, 2 * sizeof(unsigned)) != hipSuccess) {
        destroy(c);
        return rc ? rc : FBA_ERR_HIP;
    }
    if ((rc = upload(&c->d_xy, xy)) || (rc = upload(&c->d_img, img)) || (rc = upload(&c->d_cam, cam)) ||
        (rc = upload(&c->d_pt, pt)) || (rc = upload(&c->d_ctl, ctl)) || (rc = upload(&c->d_lp_tie, lp_tie)) ||
        (rc = upload(&c->d_lp_start, lp_start)) || (rc = upload(&c->d_lp_cam, lp_cam)) ||
        (rc = upload(&c->d_acc, abuf)) || (rc = upload(&c->d_xfull, c->xfull0)) ||
        (rc = upload(&c->d_caminfo, caminfo)) || (rc = upload(&c->d_active, active)) ||
        (rc = upload(&c->d_counted, counted)) || (rc = upload(&c->d_obs_pho, pho)) ||
        (rc = upload(&c->d_chunk_obs, chunk_obs)) || (rc = upload(&c->d_chunk_pt, chunk_pt)) ||
        (rc = upload(&c->d_sched, c->sched.buf)) ||
        (opt.world > 1 && !split && ((rc = upload(&c->d_gpairs, gpairs)) || (rc = dalloc(&c->d_red, (size_t)c->n_red)))) ||
        (split && ((rc = upload(&c->d_bown, bown)) || (rc = upload(&c->d_rown, rown)) || (rc = upload(&c->d_topdiag, topdiag)) ||
                   (rc = dalloc(&c->d_red, (size_t)c->n_red))))) {
        destroy(c);
        return rc;
    }
    const int nj = 9 + L.cw;
    c->ncomp = 2 * nj + 2;
    c->cam_tab_stride = CAM_TAB_HDR + 3 * L.nk;  // header | K_j | rmax^(2j) | rmax^-(2j)
    c->pt_comp = 12 + 6 * L.cw;
    const int npk = L.cw * (L.cw + 1) / 2 + L.cw;
    c->n_part = (int)std::max<int64_t>((L.u_full + 255) / 256, (c->n_obs + 255) / 256 * 3) + 8;
    if ((rc = dalloc(&c->d_delta, L.u_full)) || (rc = dalloc(&c->d_xlin, L.u_full)) || (rc = dalloc(&c->d_img_tab, (size_t)L.n_img * IMG_TAB)) ||
        (rc = dalloc(&c->d_cam_tab, (size_t)L.n_cam * c->cam_tab_stride)) ||
        (rc = dalloc(&c->d_G, (size_t)std::max(L.n_img, 1) * 42)) ||
        (rc = dalloc(&c->d_J, (size_t)c->ncomp * c->n_obs_pad)) || (rc = dalloc(&c->d_WT, (size_t)12 * c->n_obs_pad)) ||
        (rc = dalloc(&c->d_pt_tab, (size_t)c->pt_comp * c->n_lp_pad)) ||
        (rc = dalloc(&c->d_ppart, (size_t)A.n_pk * 36)) ||
        (rc = dalloc(&c->d_U, A.n_tt > 0 ? (size_t)18 * c->n_obs_pad : 1)) ||
        (rc = dalloc(&c->d_ipart, (size_t)A.n_ik * (27 + 6 * L.cw))) ||
        (rc = dalloc(&c->d_cpart, (size_t)(c->n_chunks_lr + G.n_gc) * npk)) ||
        (rc = dalloc(&c->d_gpt, (size_t)G.n_gp * 18)) || (rc = dalloc(&c->d_gcu, (size_t)G.n_gc * 6 * L.cw)) ||
        (rc = dalloc(&c->d_gug, (size_t)G.n_gi * 36)) || (rc = dalloc(&c->d_xpart, (size_t)G.n_gx * 6 * L.cw)) ||
        (rc = dalloc(&c->d_kpart, (size_t)G.n_gkk * L.cw * L.cw)) ||
        (rc = dalloc(&c->d_cseg, (size_t)std::max(L.n_cam, 1) * 64 * npk)) ||
        (rc = dalloc(&c->d_bscr, (size_t)(BSC_OFF + 16))) ||  // k_border_weights / k_border_gram segments, combine coefficients, split scales
        (rc = dalloc(&c->d_gblk, (size_t)(L.n_pad / NB) * 256)) ||
        (rc = dalloc(&c->d_S, (size_t)(L.n_pad + NB) * L.ld)) ||
        (rc = dalloc(&c->d_P, (size_t)std::max(c->sched.n_scratch, 1) * 4096)) || (rc = dalloc(&c->d_X, (size_t)L.n_pad)) ||
        (rc = dalloc(&c->d_dinv, (size_t)(L.n_pad / NB) * 8 * 256)) ||
        (rc = dalloc(&c->d_linv, (size_t)(L.n_pad / NB) * NB * NB)) ||
        (rc = dalloc(&c->d_scal, 32 + 256)) || (rc = dalloc(&c->d_part, (size_t)c->n_part)) ||
        (rc = dalloc(&c->d_res, (size_t)7 * std::max<int64_t>(c->n_obs, 1)))) {
        destroy(c);
        return rc;
    }
    FBA_HIP(hipMemset(c->d_scal, 0, sizeof(double) * 16));  // (chol_setup then sets scal[SCAL_SPINS])
    if ((rc = chol_setup(*c)) || (rc = acc_setup(*c))) { destroy(c); return rc; }
    if (getenv("FBA_LR_PROFILE") && c->n_chunks_lr > 0) FBA_HIP(hipMalloc((void**)&c->d_lrprof, sizeof(uint64_t) * 8 * c->n_chunks_lr));
    if (getenv("FBA_PANEL_TRACE") && c->sched.n_waves > 0)
    {
        const size_t nt = std::max<size_t>((size_t)PTRACE_WG * c->sched.n_waves, (size_t)c->sched.flow_n * FTRACE / 8);
        FBA_HIP(hipMalloc((void**)&c->d_ptrace, sizeof(uint64_t) * 8 * nt));
        FBA_HIP(hipMemset(c->d_ptrace, 0, sizeof(uint64_t) * 8 * nt));
    }
    FBA_HIP(hipMemset(c->d_delta, 0, sizeof(double) * L.u_full));
    // outside the factor's block pattern S stays zero; the pattern itself is zeroed per accumulation
    FBA_HIP(hipMemsetAsync(c->d_S, 0, sizeof(double) * (size_t)(L.n_pad + NB) * L.ld, c->stream));
    FBA_HIP(hipStreamSynchronize(c->stream));
    FBA_HIP(hipHostMalloc((void**)&c->h_pinned, sizeof(double) * 64, hipHostMallocMapped | hipHostMallocCoherent));
    FBA_HIP(hipHostGetDevicePointer((void**)&c->d_hpinned, c->h_pinned, 0));
    std::fill(c->h_pinned, c->h_pinned + 64, 0.0);
    for (auto& e : c->ev) FBA_HIP(hipEventCreate(&e));
    if (opt.verbose)
        fprintf(stderr, "[fba] rank %d/%d: n_obs %ld (tie %ld), points %ld, pairs %ld (%ld terms), u_c %ld, n_pad %ld; "
                "chunks %ld, pair keys %ld, U-row pair terms %ld, image keys %ld (%d lanes each); general points %ld\n",
                opt.rank, opt.world, (long)c->n_obs, (long)c->n_obs_tie, (long)c->n_lp, (long)c->n_pairs,
                (long)c->n_pair_terms, (long)L.u_c, (long)L.n_pad, (long)c->n_chunks_lr, (long)c->acc.n_pk, (long)c->acc.n_tt, (long)c->acc.n_ik, c->ik_lanes, (long)G.n_gp);
    *out = c;
    return FBA_OK;
}

static int set_xhat_ref(Ctx* c, const double* xhat) {
    std::vector<double> xf = c->xfull0;
    for (int64_t i = 0; i < c->L.u_full; ++i)
        if (c->full_to_ref[i] >= 0) xf[i] = xhat[c->full_to_ref[i]];
    FBA_HIP(hipMemcpyAsync(c->d_xfull, xf.data(), sizeof(double) * xf.size(), hipMemcpyHostToDevice, c->stream));
    FBA_HIP(hipStreamSynchronize(c->stream));
    c->have_lin = false;
    c->have_delta = false;
    return FBA_OK;
}

static inline void mark(Ctx* c, int i) {
    if (c->timing) (void)hipEventRecord(c->ev[i], c->stream);
}

static bool graph_eligible(const Ctx* c) {
    return c->graphs_ok && c->stream && !c->timing && !c->probe && !c->d_lrprof && !c->d_ptrace;
}

// run body() on the context's stream, through a graph captured from its first run when eligible
template <class F>
static int run_graph(Ctx* c, int which, F&& body) {
    if (!graph_eligible(c)) return body();
    if (!c->graph[which]) {
        if (hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) {
            (void)hipGetLastError();  // e.g. a stream that cannot be captured: launch eagerly from now on
            c->graphs_ok = false;
            return body();
        }
        const int rc = body();
        hipGraph_t g = nullptr;
        const hipError_t e = hipStreamEndCapture(c->stream, &g);
        if (rc != FBA_OK || e != hipSuccess || !g) {
            if (g) (void)hipGraphDestroy(g);
            (void)hipGetLastError();  // do not leave the capture's error to the next call's checks
            if (rc != FBA_OK) return rc;
            c->graphs_ok = false;  // capture unsupported here: run eagerly from now on
            return body();
        }
        const hipError_t ei = hipGraphInstantiate(&c->graph[which], g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (ei != hipSuccess) {
            c->graph[which] = nullptr;
            c->graphs_ok = false;
            return body();
        }
    }
    FBA_HIP(hipGraphLaunch(c->graph[which], c->stream));
    return FBA_OK;
}

static int accumulate_body(Ctx* c) {
    int rc;
    mark(c, 0);
    // tables + the linearisation point; S's pattern is zeroed by k_lin_reduce's tail workgroups
    if ((rc = launch_params(*c, nullptr, c->d_xlin))) return rc;
    mark(c, 1);
    // general tie points: their Jacobian rows, point tables and partials (ahead of the reductions)
    if ((rc = launch_gen_tables(*c, nullptr)) || (rc = launch_gen_keys(*c))) return rc;
    mark(c, 2);
    if ((rc = launch_accumulate(*c)) || (rc = launch_gen_reduce(*c))) return rc;
    if (c->d_lrprof) {  // FBA_LR_PROFILE: per-phase averages of k_lin_reduce (us)
        std::vector<uint64_t> tp(8 * c->n_chunks_lr);
        FBA_HIP(hipMemcpyAsync(tp.data(), c->d_lrprof, sizeof(uint64_t) * tp.size(), hipMemcpyDeviceToHost, c->stream));
        FBA_HIP(hipStreamSynchronize(c->stream));
        double ph[6] = {0, 0, 0, 0, 0, 0};
        uint64_t lo = UINT64_MAX, hi = 0;
        const double nch = (double)c->n_chunks_lr;
        for (int64_t ch = 0; ch < c->n_chunks_lr; ++ch) {
            const uint64_t* q = &tp[8 * ch];
            for (int i = 0; i < 4; ++i) ph[i] += (double)(q[i + 1] - q[i]) * 0.01 / nch;
            ph[4] += (double)(q[6] - q[4]) * 0.01 / nch;  // image keys
            ph[5] += (double)(q[5] - q[6]) * 0.01 / nch;  // pair keys
            lo = std::min(lo, q[0]);
            hi = std::max(hi, q[5]);
        }
        fprintf(stderr, "[fba] k_lin_reduce per chunk (us): model %.2f points %.2f couplings %.2f stage+camera %.2f "
                "image keys %.2f pair keys %.2f; span %.1f\n", ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], (double)(hi - lo) * 0.01);
    }
    if (c->sched.split) {
        // subtree split: the top rows' accumulated diagonal (before k_border_rhs writes unit rows), the
        // border rows, this rank's subtree columns (flow A: their factor, forward solve and Schur updates of
        // the top blocks), then the buffer
        if ((rc = launch_pack_split(*c, 2)) || (rc = launch_border(*c)) || (rc = launch_cholesky(*c, 0)) ||
            (rc = launch_pack_split(*c, 0)))
            return rc;
    } else if (c->opt.world > 1 && (rc = launch_pack(*c, 0))) {
        return rc;
    }
    mark(c, 3);
    return FBA_OK;
}

static int accumulate(Ctx* c) {
    c->have_factor = false;
    const int rc = run_graph(c, 0, [&] { return accumulate_body(c); });
    if (rc == FBA_OK) {
        c->have_lin = true;
        c->solved = false;
    }
    return rc;
}

static int solve_body(Ctx* c) {
    int rc;
    const Layout& L = c->L;
    if (c->sched.split) {  // the summed top blocks (+ the B rows' weights), then the top columns (flow B)
        if ((rc = launch_pack_split(*c, 1))) return rc;
        mark(c, 4);
        if ((rc = launch_cholesky(*c, 1))) return rc;
    } else {
        if (c->opt.world > 1 && (rc = launch_pack(*c, 1))) return rc;
        if ((rc = launch_border(*c))) return rc;
        mark(c, 4);
        if ((rc = launch_cholesky(*c))) return rc;
    }
    mark(c, 5);
    // tie-point corrections of other ranks' points stay zero (a single rank writes every one of them in
    // k_backsub; a zero-byte memset is not a valid graph node)
    if (L.u_full > L.u_c && c->opt.world > 1)
        FBA_HIP(hipMemsetAsync(c->d_delta + L.u_c, 0, sizeof(double) * (L.u_full - L.u_c), c->stream));
    if ((rc = launch_backward(*c))) return rc;
    mark(c, 6);
    if ((rc = launch_backsub_update(*c))) return rc;
    mark(c, 7);
    // scal[0..3] reach h_pinned from k_sum_parts itself (host-mapped stores, no copy node)
    return FBA_OK;
}

static int solve_enqueue(Ctx* c) {
    if (!c->have_lin) { set_error("fba_solve_update before fba_accumulate"); return FBA_ERR_ARG; }
    // the solve factors S in place (and with the subtree split, flow A's sync words are not re-zeroed by
    // the solve: flow B's tickets would be past its grid), so a second solve of one accumulation would
    // factor a factor -- refused; accumulate again
    if (c->solved) {
        set_error("one fba_solve_update per fba_accumulate (the solve factors the accumulated system in place)");
        return FBA_ERR_ARG;
    }
    // marked before the launches: a solve that fails part way may already have factored S in place, so a
    // retry must accumulate again too (accumulate() clears the mark)
    c->solved = true;
    const int rc = run_graph(c, 1, [&] { return solve_body(c); });
    if (rc == FBA_OK) ++c->solves_enqueued;  // k_sum_parts' count once this solve is done
    return rc;
}

// wait for the solve, read scal (again from the device when `recopy`: a caller may have all-reduced
// the deltasum share in place after the graph's own copy), check the failure flags
// FBA_PANEL_TRACE: one line per elimination-tree level, times in us from the first k_panel's start:
// launch span, the gap after the previous launch, and per workgroup role the last end (diagonal-block
// updates, potrf start / after its waits / end, panel solves, inverses, other updates)
// k_chol_flow (FBA_PANEL_TRACE=1): per diagonal-block record, times in us from the launch's first start:
// start, waits done, fused panel solve + diagonal update done, late partials added, end (potrf done);
// then per role the record count and the last end
static void print_flow_trace(Ctx* c) {
    const Sched& s = c->sched;
    std::vector<uint64_t> t((size_t)FTRACE * s.flow_n);
    if (hipMemcpy(t.data(), c->d_ptrace, t.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t t0 = UINT64_MAX;
    for (int b = 0; b < s.flow_n; ++b)
        if (t[FTRACE * (size_t)b]) t0 = std::min(t0, t[FTRACE * (size_t)b]);
    const uint64_t M = (1ull << 63) - 1;
    auto us = [&](uint64_t v) { return (v & M) ? (double)((v & M) - t0) * 0.01 : -1.0; };
    uint64_t rend[5] = {0, 0, 0, 0, 0};
    int rn[5] = {0, 0, 0, 0, 0};
    const int32_t* recs = s.buf.data() + s.flow_rec;
    const bool detail = getenv("FBA_PANEL_TRACE")[0] == '2';
    if (getenv("FBA_PANEL_TRACE")[0] == '3')  // every record in dispatch order: role, ids, start, waits done, end
        for (int b = 0; b < s.flow_n; ++b) {
            const uint64_t* r = &t[FTRACE * (size_t)b];
            const int32_t* rec = recs + (size_t)Sched::FLOW_REC * b;
            fprintf(stderr, "[fba] rec %d %d %d %d %d %.2f %.2f %.2f %.2f %.2f\n", b, rec[0], rec[1], rec[2], rec[3], us(r[0]),
                    us(r[1]), us(r[2]), us(r[48]), us(r[49]));
        }
    for (int b = 0; b < s.flow_n; ++b) {
        const uint64_t* r = &t[FTRACE * (size_t)b];
        const int32_t* rec = recs + (size_t)Sched::FLOW_REC * b;
        const int role = rec[0];
        rend[role] = std::max(rend[role], r[2]);
        rn[role]++;
        if (role != 0) continue;
        fprintf(stderr, "[fba]   diag wg %5d block %3d (fused %3d%s): start %7.1f  waits %7.1f  fused %7.1f  late %7.1f  end %7.1f\n",
                b, rec[1], rec[2], rec[6] > 0 ? ", late" : "", us(r[0]), us(r[1]), rec[2] >= 0 ? us(r[4]) : -1.0,
                rec[2] >= 0 ? us(r[5]) : -1.0, us(r[2]));
        if (!detail) continue;
        fprintf(stderr, "[fba]       potrf leaf 0 %.1f, barrier %.1f, panel tile (2, 0) %.1f; column solved / published:",
                us(r[3]), us(r[6]), us(r[7]));
        for (int q = 0; q < 8; ++q) fprintf(stderr, " %.1f/%.1f", us(r[24 + q]), us(r[32 + q]));
        fprintf(stderr, "\n");
        if (rec[2] < 0) continue;
        fprintf(stderr, "[fba]       block in LDS / applied:");
        for (int q = 0; q < 8; ++q) fprintf(stderr, " %.1f/%.1f%s", us(r[8 + q]), us(r[16 + q]), (r[16 + q] >> 63) ? "p" : "");
        fprintf(stderr, "\n");
        fprintf(stderr, "[fba]       loading group's share stored:");
        for (int q = 0; q < 8; ++q) fprintf(stderr, " %.1f", us(r[40 + q]));
        fprintf(stderr, "\n");
        for (int x = 0; x < s.flow_n; ++x) {  // the panel halves of its fused rows
            const int32_t* rx = recs + (size_t)Sched::FLOW_REC * x;
            const uint64_t* q = &t[FTRACE * (size_t)x];
            if (!(rx[0] == 1 && rx[1] == rec[2] && (rx[2] >> 1) == rec[1])) continue;
            fprintf(stderr, "[fba]       half %d wg %5d: start %.1f waits %.1f column in / published:", rx[2] & 1, x, us(q[0]),
                    us(q[1]));
            for (int u = 0; u < 8; ++u) fprintf(stderr, " %.1f/%.1f", us(q[8 + u]), us(q[16 + u]));
            fprintf(stderr, "  end %.1f\n", us(q[2]));
        }
        for (int x = 0; x < s.flow_n && rec[9] >= 0; ++x) {  // its split helper
            const int32_t* rx = recs + (size_t)Sched::FLOW_REC * x;
            const uint64_t* q = &t[FTRACE * (size_t)x];
            if (!(rx[0] == 4 && rx[1] == rec[1])) continue;
            fprintf(stderr, "[fba]       split helper wg %5d: start %.1f block in LDS / applied:", x, us(q[0]));
            for (int u = 0; u < 8; ++u) fprintf(stderr, " %.1f/%.1f", us(q[8 + u]), us(q[16 + u]));
            fprintf(stderr, "  end %.1f\n", us(q[2]));
        }
    }
    fprintf(stderr, "[fba] flow: diag %d (last end %.1f), panel halves %d (%.1f), updates %d (%.1f), inverses %d (%.1f), "
            "split helpers %d (%.1f)\n", rn[0], us(rend[0]), rn[1], us(rend[1]), rn[2], us(rend[2]), rn[3], us(rend[3]),
            rn[4], us(rend[4]));
    (void)hipMemset(c->d_ptrace, 0, t.size() * sizeof(uint64_t));
}

static void print_panel_trace(Ctx* c) {
    if (c->chol_flow && c->sched.flow_ok && c->sched.flow_n > 0) { print_flow_trace(c); return; }
    const int nw = c->sched.n_waves;
    std::vector<uint64_t> t((size_t)8 * PTRACE_WG * nw);
    if (hipMemcpy(t.data(), c->d_ptrace, t.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return;
    uint64_t t0 = UINT64_MAX, prev_end = 0;
    for (int w = 0; w < nw; ++w)
        for (int b = 0; b < PTRACE_WG; ++b)
            if (t[(size_t)8 * (w * PTRACE_WG + b)] != 0) t0 = std::min(t0, t[(size_t)8 * (w * PTRACE_WG + b)]);
    auto us = [&](uint64_t v) { return v ? (double)(v - t0) * 0.01 : -1.0; };
    auto hi_trsm_end = [&](int w) {
        uint64_t m = 0;
        for (int b = 0; b < PTRACE_WG; ++b) {
            const uint64_t* r = &t[(size_t)8 * (w * PTRACE_WG + b)];
            if (r[0] != 0 && r[3] == 3) m = std::max(m, r[2]);
        }
        return m;
    };
    for (int w = 0; w < nw; ++w) {
        uint64_t lo = UINT64_MAX, hi = 0, rend[6] = {0, 0, 0, 0, 0, 0}, pst = 0, prd = 0, tfirst = UINT64_MAX, tseen = 0;
        int n = 0;
        for (int b = 0; b < PTRACE_WG; ++b) {
            const uint64_t* r = &t[(size_t)8 * (w * PTRACE_WG + b)];
            if (r[0] == 0) continue;
            ++n;
            lo = std::min(lo, r[0]);
            hi = std::max(hi, r[2]);
            const int role = (int)r[3];
            if (role >= 0 && role < 6) rend[role] = std::max(rend[role], r[2]);
            if (role == 1) { pst = std::max(pst, r[0]); prd = std::max(prd, r[1]); }
            if (role == 3) { tfirst = std::min(tfirst, r[0]); tseen = std::max(tseen, r[1]); }
            if (role == 3 && getenv("FBA_PANEL_TRACE")[0] == '3' && r[2] == hi_trsm_end(w))
                fprintf(stderr, "[fba]   level %2d last panel solve wg %4d: start %6.1f  step 6 done %6.1f  factor seen %6.1f  "
                        "step 7 done %6.1f  end %6.1f  batches %llx\n", w, b, us(r[0]), us(r[5]), us(r[1]), us(r[6]), us(r[2]),
                        (unsigned long long)r[4]);
            if (role == 0 && getenv("FBA_PANEL_TRACE")[0] == '2')
                fprintf(stderr, "[fba]   level %2d diag-update wg %3d: %2d sources%s  %6.1f .. %6.1f (%4.1f us)\n", w, b,
                        (int)(r[1] & 0xff), (r[1] & 0x100) ? " (split group)" : "", us(r[0]), us(r[2]), (double)(r[2] - r[0]) * 0.01);
            if (role == 0 && getenv("FBA_PANEL_TRACE")[0] == '2')
                fprintf(stderr, "[fba]       loaded +%.1f  products +%.1f  published +%.1f\n", (double)(r[4] - r[0]) * 0.01,
                        (double)(r[5] - r[0]) * 0.01, (double)(r[2] - r[0]) * 0.01);
        }
        if (n == 0) { fprintf(stderr, "[fba] level %2d: own k_potrf128/k_trsm128 launches (no trace)\n", w); continue; }
        fprintf(stderr, "[fba] level %2d: %4d wg  span %7.1f .. %7.1f (%5.1f)  gap %5.1f | diag-upd end %7.1f | potrf %7.1f wait-end %7.1f "
                "end %7.1f | panel-upd end %7.1f | trsm %7.1f .. (factor seen %7.1f) %7.1f | trtri end %7.1f | other-upd end %7.1f\n",
                w, n, us(lo), us(hi), (double)(hi - lo) * 0.01, prev_end ? (double)(lo - prev_end) * 0.01 : 0.0, us(rend[0]),
                us(pst), us(prd), us(rend[1]), us(rend[2]), tfirst == UINT64_MAX ? -1.0 : us(tfirst), us(tseen), us(rend[3]),
                us(rend[4]), us(rend[5]));
        prev_end = hi;
    }
    (void)hipMemset(c->d_ptrace, 0, t.size() * sizeof(uint64_t));
}

// Completion of a solve: k_sum_parts, the last kernel of every solve, writes its results to host-mapped
// memory and then the device's count of finished solves; fba_step polls that count until it reaches the
// number of solves enqueued on the context (a spin on coherent host memory returns a few us after the
// GPU's write, where hipStreamSynchronize's wake-up is slower) -- later work on the stream is ordered after
// the solve anyway.  The poll spins briefly, then yields the core between reads; once the count is there,
// hipStreamQuery surfaces an asynchronous error of the stream at once.  The stream is synchronised instead
// when a caller re-copies scal (the multi-GPU path), with tracing or timing on, with FBA_SYNC=1, and after
// ~5 s without the count (a faulted launch: the synchronisation reports it).
static bool wait_solve_seq(Ctx* c) {
    if (c->force_sync || c->timing || c->d_ptrace || c->d_lrprof) return false;
    const double want = (double)c->solves_enqueued;
    volatile const double* seq = c->h_pinned + 4;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0; *seq < want; ++it) {
        if (it < 4096) continue;  // ~the first 10-20 us: spin
        std::this_thread::yield();
        if ((it & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) return false;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return true;
}

static int solve_finish(Ctx* c, double* dsum, bool recopy) {
    if (recopy) FBA_HIP(hipMemcpyAsync(c->h_pinned, c->d_scal, sizeof(double) * 4, hipMemcpyDeviceToHost, c->stream));
    if (recopy || !wait_solve_seq(c)) {
        FBA_HIP(hipStreamSynchronize(c->stream));
    } else {
        const hipError_t q = hipStreamQuery(c->stream);  // (hipErrorNotReady: later work queued, no error)
        if (q != hipSuccess && q != hipErrorNotReady) FBA_HIP(q);
    }
    c->solve_seq = c->h_pinned[4];
    if (c->d_ptrace && !c->sched.split) print_panel_trace(c);
    if (c->timing) {
        float ms;
        for (int i = 0; i < 7; ++i) {
            (void)hipEventElapsedTime(&ms, c->ev[i], c->ev[i + 1]);
            c->last_ms[i] = ms;
        }
        (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[7]);
        c->last_ms[7] = ms;
    }
    c->iterations++;
    const double info = c->h_pinned[1];
    *dsum = c->h_pinned[2];
    if (info < 0.0) {
        // k_update left xhat as it was (fba_chol.hip, bounded polls): the context stays usable
        set_error("device hand-off timeout in the block Cholesky / backward solve (a workgroup of k_chol_flow, "
                  "k_panel or k_bwd_flow was not resident); xhat left unchanged");
        c->have_delta = false;
        c->have_factor = false;
        return FBA_ERR_HIP;
    }
    c->have_delta = true;
    c->have_factor = true;
    if (info != 0.0) {
        char buf[160];
        snprintf(buf, sizeof buf, "reduced normal matrix not positive definite (pivot %ld): singular / unconstrained network",
                 (long)info);
        set_error(buf);
        return FBA_ERR_NOT_SPD;
    }
    if (!std::isfinite(*dsum)) { set_error("non-finite correction vector"); return FBA_ERR_NONFINITE; }
    return FBA_OK;
}

static int solve_update(Ctx* c, double* dsum) {
    int rc;
    if ((rc = solve_enqueue(c))) return rc;
    return solve_finish(c, dsum, false);
}

}  // namespace fba

using namespace fba;

extern "C" {

const char* fba_last_error(void) { return g_err.c_str(); }
int fba_abi_version(void) { return FBA_ABI_VERSION; }

int fba_set_spin_bound(fba_ctx* ctx, int64_t spins) {
    if (!ctx || spins < 0) { set_error("fba_set_spin_bound: bad argument"); return FBA_ERR_ARG; }
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    const double v = spin_bound_value(spins);
    FBA_HIP(hipStreamSynchronize(c->stream));
    FBA_HIP(hipMemcpy(c->d_scal + SCAL_SPINS, &v, sizeof v, hipMemcpyHostToDevice));
    return FBA_OK;
}

int fba_solve_mode(fba_ctx* ctx, int32_t* split) {
    if (!ctx || !split) { set_error("fba_solve_mode: null argument"); return FBA_ERR_ARG; }
    *split = reinterpret_cast<Ctx*>(ctx)->sched.split ? 1 : 0;
    return FBA_OK;
}

int fba_count_unknowns(const fba_problem* p, const fba_settings* s, int64_t* u_out) {
    if (!p || !s || !u_out) { set_error("NULL argument"); return FBA_ERR_ARG; }
    *u_out = (int64_t)(s->est_Xc + s->est_Yc + s->est_Zc + s->est_omega + s->est_phi + s->est_kappa) * p->n_img +
             (int64_t)(s->est_c + s->est_xp + s->est_yp + s->est_radial * s->num_radial + s->est_decent * 2) * p->n_cam +
             3 * (int64_t)p->n_tie;
    return FBA_OK;
}

int fba_partition(const fba_problem* p, int32_t world, int32_t* tie_owner, int32_t* ctl_owner) {
    if (!p || world < 1) { set_error("bad argument"); return FBA_ERR_ARG; }
    std::vector<int32_t> t, q;
    partition(p, world, t, q);
    if (tie_owner) std::copy(t.begin(), t.end(), tie_owner);
    if (ctl_owner) std::copy(q.begin(), q.end(), ctl_owner);
    return FBA_OK;
}

int fba_image_order(const fba_problem* p, int32_t* order, int32_t* n_slots) {
    if (!p || !n_slots) { set_error("NULL argument"); return FBA_ERR_ARG; }
    if (p->n_img < 0 || (p->n_pts > 0 && (!p->img || !p->tie))) { set_error("bad problem"); return FBA_ERR_ARG; }
    for (int64_t i = 0; i < p->n_pts; ++i)
        if (p->img[i] < 0 || p->img[i] >= p->n_img || p->tie[i] < -1 || p->tie[i] >= p->n_tie) {
            set_error("image / tie index out of range");
            return FBA_ERR_ARG;
        }
    const std::vector<int32_t> ord = camera_order(p);
    *n_slots = (int32_t)ord.size();
    if (order) std::copy(ord.begin(), ord.end(), order);
    return FBA_OK;
}

int fba_create(const fba_problem* p, const fba_settings* s, const fba_options* o, fba_ctx** out) {
    if (!out) { set_error("out is NULL"); return FBA_ERR_ARG; }
    *out = nullptr;
    Ctx* c = nullptr;
    int rc = create(p, s, o, &c);
    if (rc) return rc;
    *out = reinterpret_cast<fba_ctx*>(c);
    return FBA_OK;
}

void fba_destroy(fba_ctx* ctx) { destroy(reinterpret_cast<Ctx*>(ctx)); }

int fba_buildxhat(fba_ctx* ctx, double* xhat, int64_t* u_out) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    if (u_out) *u_out = c->L.u_ref;
    if (xhat)
        for (int64_t i = 0; i < c->L.u_full; ++i)
            if (c->full_to_ref[i] >= 0) xhat[c->full_to_ref[i]] = c->xfull0[i];
    return FBA_OK;
}

int fba_set_xhat(fba_ctx* ctx, const double* xhat) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !xhat) { set_error("NULL argument"); return FBA_ERR_ARG; }
    return set_xhat_ref(c, xhat);
}

int fba_get_xhat(fba_ctx* ctx, double* xhat, int32_t owned_only) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !xhat) { set_error("NULL argument"); return FBA_ERR_ARG; }
    std::vector<double> xf(c->L.u_full);
    FBA_HIP(hipMemcpyAsync(xf.data(), c->d_xfull, sizeof(double) * xf.size(), hipMemcpyDeviceToHost, c->stream));
    FBA_HIP(hipStreamSynchronize(c->stream));
    for (int64_t i = 0; i < c->L.u_full; ++i)
        if (c->full_to_ref[i] >= 0) xhat[c->full_to_ref[i]] = (owned_only && !c->full_owned[i]) ? 0.0 : xf[i];
    return FBA_OK;
}

int fba_build_awg(fba_ctx* ctx, const double* xhat, double* A, double* w, double* G, double* dist_scaling) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    int rc;
    if (xhat && (rc = set_xhat_ref(c, xhat))) return rc;
    if ((rc = launch_params(*c)) || (rc = launch_linearize(*c))) return rc;
    const Layout& L = c->L;
    const int64_t n = 2 * c->n_pts, u = L.u_ref;
    double *dA = nullptr, *dW = nullptr;
    int64_t* dmap = nullptr;
    if ((rc = dalloc(&dA, (size_t)n * u)) || (rc = dalloc(&dW, (size_t)n)) || (rc = upload(&dmap, c->full_to_ref)))
        return rc;
    FBA_HIP(hipMemsetAsync(dA, 0, sizeof(double) * n * u, c->stream));
    FBA_HIP(hipMemsetAsync(dW, 0, sizeof(double) * n, c->stream));
    if ((rc = launch_dense_awg(*c, dA, dW, dmap, n, u))) return rc;
    if (A) FBA_HIP(hipMemcpyAsync(A, dA, sizeof(double) * n * u, hipMemcpyDeviceToHost, c->stream));
    if (w) FBA_HIP(hipMemcpyAsync(w, dW, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    std::vector<double> g((size_t)std::max(L.n_img, 1) * 42), ct((size_t)L.n_cam * c->cam_tab_stride);
    FBA_HIP(hipMemcpyAsync(g.data(), c->d_G, sizeof(double) * g.size(), hipMemcpyDeviceToHost, c->stream));
    FBA_HIP(hipMemcpyAsync(ct.data(), c->d_cam_tab, sizeof(double) * ct.size(), hipMemcpyDeviceToHost, c->stream));
    FBA_HIP(hipStreamSynchronize(c->stream));
    (void)hipFree(dA);
    (void)hipFree(dW);
    (void)hipFree(dmap);
    if (G && c->set.inner_constraints) {
        std::fill(G, G + u * 7, 0.0);
        for (int e = 0; e < L.n_img; ++e)
            for (int a = 0; a < 6; ++a) {
                const int64_t r = c->full_to_ref[6 * (int64_t)e + a];
                if (r < 0) continue;  // padding slot
                for (int m = 0; m < 7; ++m) G[r + m * u] = g[(size_t)e * 42 + a * 7 + m];
            }
    }
    if (dist_scaling) {
        const int nc = L.n_cam, ncol = 2 + L.nk;
        std::fill(dist_scaling, dist_scaling + (size_t)nc * ncol, 0.0);
        for (int k = 0; k < nc; ++k) {
            // the reference stores 1-based xhat indices (BuildAwG.m:138, :150)
            const int64_t base = 6 * (int64_t)L.n_img + (int64_t)k * L.cw;
            if (c->set.est_radial) dist_scaling[k + 0 * nc] = (double)(c->full_to_ref[base + 3] + 1);
            if (c->set.est_decent) dist_scaling[k + 1 * nc] = (double)(c->full_to_ref[base + 3 + L.nk] + 1);
            for (int j = 0; j < L.nk; ++j)
                dist_scaling[k + (2 + j) * nc] = ct[(size_t)k * c->cam_tab_stride + CAM_TAB_HDR + L.nk + j];
        }
    }
    c->have_lin = false;
    return FBA_OK;
}

int fba_accumulate(fba_ctx* ctx) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    return accumulate(c);
}

int fba_reduce_buffer(fba_ctx* ctx, void** dev_ptr, int64_t* n_doubles) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !dev_ptr || !n_doubles) { set_error("NULL argument"); return FBA_ERR_ARG; }
    if (c->opt.world > 1) {  // compact: only the entries any rank writes (~6 MB at config 4)
        *dev_ptr = c->d_red;
        *n_doubles = c->n_red;
    } else {
        *dev_ptr = c->d_S;
        *n_doubles = (c->L.n_pad + 1) * c->L.ld;  // lower normal matrix + RHS row 0
    }
    return FBA_OK;
}

int fba_synchronize(fba_ctx* ctx) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    FBA_HIP(hipStreamSynchronize(c->stream));
    return FBA_OK;
}

int fba_solve_update(fba_ctx* ctx, double* deltasum_part) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    double d = 0.0;
    int rc = solve_update(c, &d);
    if (deltasum_part) *deltasum_part = d;
    return rc;
}

int fba_solve_update_async(fba_ctx* ctx) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    const int rc = solve_enqueue(c);
    if (rc == FBA_OK) c->pending = true;
    return rc;
}

int fba_deltasum_device(fba_ctx* ctx, void** dev_ptr) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !dev_ptr) { set_error("NULL argument"); return FBA_ERR_ARG; }
    *dev_ptr = c->d_scal + 2;
    return FBA_OK;
}

int fba_solve_finish(fba_ctx* ctx, double* deltasum) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    if (!c->pending) { set_error("fba_solve_finish without fba_solve_update_async"); return FBA_ERR_ARG; }
    c->pending = false;
    double d = 0.0;
    const int rc = solve_finish(c, &d, true);
    if (deltasum) *deltasum = d;
    return rc;
}

int fba_step(fba_ctx* ctx, double* deltasum) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    if (c->opt.world != 1) { set_error("fba_step is single-GPU; use fba_accumulate/fba_solve_update"); return FBA_ERR_ARG; }
    int rc = accumulate(c);
    if (rc) return rc;
    double d = 0.0;
    rc = solve_update(c, &d);
    if (deltasum) *deltasum = d;
    return rc;
}

int fba_adjust(fba_ctx* ctx, int32_t* iterations, double* deltasum_hist) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    double deltasum = 100.0;  // main.m:407
    int count = 0;
    while (deltasum > c->set.threshold) {  // main.m:412
        ++count;
        int rc = fba_step(ctx, &deltasum);
        if (deltasum_hist) deltasum_hist[count - 1] = deltasum;
        if (iterations) *iterations = count;
        if (rc) return rc;
        if (count >= c->set.iteration_cap) break;  // main.m:490-493
    }
    if (iterations) *iterations = count;
    return FBA_OK;
}

int fba_residuals(fba_ctx* ctx, double* v, double* rsd, double* stats) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    if (!c->have_lin || !c->have_delta) { set_error("fba_residuals needs at least one iteration"); return FBA_ERR_ARG; }
    // v = A delta + w with A, w of the last linearisation (main.m:569): its Jacobian rows again, at
    // the parameters it was taken at
    int rc;
    if ((rc = launch_params(*c, c->d_xlin)) || (rc = launch_linearize(*c, c->d_xlin)) || (rc = launch_residuals(*c)))
        return rc;
    const int64_t n = c->n_obs;
    const int nblk = (int)((n + 255) / 256);
    std::vector<double> res(7 * (size_t)n), part(3 * (size_t)nblk);
    if (n > 0) {
        FBA_HIP(hipMemcpyAsync(res.data(), c->d_res, sizeof(double) * res.size(), hipMemcpyDeviceToHost, c->stream));
        FBA_HIP(hipMemcpyAsync(part.data(), c->d_part, sizeof(double) * part.size(), hipMemcpyDeviceToHost, c->stream));
    }
    FBA_HIP(hipStreamSynchronize(c->stream));
    if (v) std::fill(v, v + 2 * c->n_pts, 0.0);
    if (rsd) std::fill(rsd, rsd + 5 * c->n_pts, 0.0);
    for (int64_t o = 0; o < n; ++o) {
        const int64_t i = c->obs_pho[o];
        if (v) { v[2 * i] = res[2 * o]; v[2 * i + 1] = res[2 * o + 1]; }
        if (rsd)
            for (int m = 0; m < 5; ++m) rsd[5 * i + m] = res[2 * n + 5 * o + m];
    }
    double sx = 0, sy = 0, sp = 0;
    for (int b = 0; b < nblk; ++b) { sx += part[3 * b]; sy += part[3 * b + 1]; sp += part[3 * b + 2]; }
    if (stats) {
        const double nu = (double)(2 * c->n_pts - c->L.u_ref);
        if (c->opt.world == 1) {
            const double rx = std::sqrt(sx / (double)c->n_pts), ry = std::sqrt(sy / (double)c->n_pts);
            stats[0] = rx; stats[1] = ry; stats[2] = std::sqrt(rx * rx + ry * ry);
            stats[3] = sp / nu;  // main.m:601: v'Pv / (n - u)
        } else {
            stats[0] = sx; stats[1] = sy; stats[2] = 0; stats[3] = 0;
        }
        stats[4] = sp;
        stats[5] = nu;
    }
    return FBA_OK;
}

int fba_build_rsd(fba_ctx* ctx, const double* v, const double* xhat, double* rsd) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !v || !xhat || !rsd) { set_error("NULL argument"); return FBA_ERR_ARG; }
    const Layout& L = c->L;
    // xp, yp per camera: from xhat when estimated, else the INT values (BuildRSD.m:12-26)
    std::vector<double> xpyp(2 * (size_t)std::max(L.n_cam, 1));
    for (int k = 0; k < L.n_cam; ++k)
        for (int a = 0; a < 2; ++a) {
            const int64_t f = 6 * (int64_t)L.n_img + (int64_t)k * L.cw + a;
            xpyp[2 * k + a] = c->full_to_ref[f] >= 0 ? xhat[c->full_to_ref[f]] : c->xfull0[f];
        }
    const int64_t n = c->n_pts;
    double *dv = nullptr, *dx = nullptr, *dr = nullptr;
    int rc;
    auto release = [&]() { for (void* q : {(void*)dv, (void*)dx, (void*)dr}) if (q) (void)hipFree(q); };
    if ((rc = dalloc(&dv, 2 * (size_t)n)) || (rc = upload(&dx, xpyp)) || (rc = dalloc(&dr, 5 * (size_t)n))) { release(); return rc; }
    hipError_t e = hipMemcpyAsync(dv, v, sizeof(double) * 2 * n, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipMemsetAsync(dr, 0, sizeof(double) * 5 * n, c->stream);
    if (e == hipSuccess && (rc = launch_build_rsd(*c, dv, dx, dr))) { release(); return rc; }
    if (e == hipSuccess) e = hipMemcpyAsync(rsd, dr, sizeof(double) * 5 * n, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    release();
    if (e != hipSuccess) { set_error(std::string("HIP error in fba_build_rsd: ") + hipGetErrorString(e)); return FBA_ERR_HIP; }
    return FBA_OK;
}

int fba_covariance(fba_ctx* ctx, double sigma02, double* cx_diag, double* corr) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    if (!c->have_factor || !c->have_delta) {
        set_error("fba_covariance needs the factor of the last solve (call it once, right after the iterations)");
        return FBA_ERR_ARG;
    }
    const Layout& L = c->L;
    const bool split = c->sched.split;
    const int m = 6 + L.cw;
    double *d_cdiag = nullptr, *d_pdiag = nullptr, *d_iblk = nullptr;
    int32_t *d_islot = nullptr, *d_icam = nullptr;
    std::vector<int32_t> islot(std::max(L.n_img_ref, 1), 0), icam(std::max(L.n_img_ref, 1), 0);
    for (int e = 0; e < L.n_img_ref; ++e) {
        islot[e] = c->img_new[e];
        icam[e] = std::max(c->ref_img_cam[e], 0);
    }
    auto release = [&]() {};  // (the context's workspace slots 64..68, kept for the next call)
    int rc;
    if ((rc = ws_get(*c, 64, sizeof(double) * std::max<int64_t>(L.u_c, 1), (void**)&d_cdiag)) ||
        (rc = ws_get(*c, 65, sizeof(double) * 3 * (size_t)std::max(L.n_tie, 1), (void**)&d_pdiag)) ||
        (corr && (rc = ws_get(*c, 66, sizeof(double) * (size_t)std::max(L.n_img_ref, 1) * m * m, (void**)&d_iblk))) ||
        (rc = ws_get(*c, 67, sizeof(int32_t) * islot.size(), (void**)&d_islot)) ||
        (rc = ws_get(*c, 68, sizeof(int32_t) * icam.size(), (void**)&d_icam))) {
        return rc;
    }
    if (hipMemcpyAsync(d_islot, islot.data(), sizeof(int32_t) * islot.size(), hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        hipMemcpyAsync(d_icam, icam.data(), sizeof(int32_t) * icam.size(), hipMemcpyHostToDevice, c->stream) != hipSuccess) {
        set_error("hipMemcpyAsync failed");
        return FBA_ERR_HIP;
    }
    if (hipMemsetAsync(d_pdiag, 0, sizeof(double) * 3 * std::max(L.n_tie, 1), c->stream) != hipSuccess) {
        release();
        set_error("hipMemsetAsync failed");
        return FBA_ERR_HIP;
    }
    if ((rc = launch_covariance(*c, d_cdiag, d_pdiag, d_iblk, d_islot, d_icam, corr ? L.n_img_ref : 0))) {
        release();
        return rc;
    }
    std::vector<double> cd(L.u_c), pd(3 * (size_t)L.n_tie), ib(corr ? (size_t)L.n_img_ref * m * m : 0);
    const hipError_t e1 = hipMemcpy(cd.data(), d_cdiag, sizeof(double) * cd.size(), hipMemcpyDeviceToHost);
    const hipError_t e2 = pd.empty() ? hipSuccess : hipMemcpy(pd.data(), d_pdiag, sizeof(double) * pd.size(), hipMemcpyDeviceToHost);
    const hipError_t e3 = ib.empty() ? hipSuccess : hipMemcpy(ib.data(), d_iblk, sizeof(double) * ib.size(), hipMemcpyDeviceToHost);
    release();
    if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess) {
        set_error("HIP error copying the covariance back");
        return FBA_ERR_HIP;
    }
    if (cx_diag) {
        std::fill(cx_diag, cx_diag + L.u_ref, 0.0);
        for (int64_t i = 0; i < L.u_full; ++i) {
            const int64_t r = c->full_to_ref[i];
            // (tie entries: this rank's points; camera-side entries: every rank, or with the subtree split
            // this rank's rows -- its subtrees', and the top's on rank 0 -- so that the ranks' outputs sum)
            if (r < 0 || ((i >= L.u_c || split) && !c->full_owned[i])) continue;
            cx_diag[r] = sigma02 * (i < L.u_c ? cd[i] : pd[i - L.u_c]);  // main.m:602: Cx = sigma02 .* Cx
        }
    }
    if (corr) {
        // the reference's Correlation (main.m:446-456, before the distortion de-scaling) over
        // [the image's estimated EOPs, its camera's estimated IOPs] (main.m:831-840), in xhat order
        const int mu = L.u_img + L.u_cam;
        std::vector<int> sel;
        const int ee[6] = {c->set.est_Xc, c->set.est_Yc, c->set.est_Zc, c->set.est_omega, c->set.est_phi, c->set.est_kappa};
        for (int a = 0; a < 6; ++a)
            if (ee[a]) sel.push_back(a);
        const int64_t cb = 6 * (int64_t)L.n_img;
        for (int q = 0; q < L.cw; ++q)
            if (L.n_cam > 0 && c->full_to_ref[cb + q] >= 0) sel.push_back(6 + q);
        for (int e = 0; e < L.n_img_ref; ++e) {
            const double* b = ib.data() + (size_t)e * m * m;
            double* out = corr + (size_t)e * mu * mu;
            // (subtree split: an image's block on the rank that owns its first row -- its subtree's rank, even
            // when the image straddles into a top block; a wholly-top image on rank 0 -- zeros elsewhere)
            if (split && !c->full_owned[6 * (int64_t)c->img_new[e]]) {
                std::fill(out, out + (size_t)mu * mu, 0.0);
                continue;
            }
            for (int a = 0; a < (int)sel.size(); ++a)
                for (int q = 0; q < (int)sel.size(); ++q) {
                    const int ra = sel[a], rq = sel[q];
                    out[a * mu + q] = c->ref_img_cam[e] < 0
                                          ? 0.0
                                          : b[ra * m + rq] / (std::sqrt(b[ra * m + ra]) * std::sqrt(b[rq * m + rq]));
                }
        }
    }
    return FBA_OK;
}

int fba_finish_stats(const fba_problem* p, const fba_settings* s, const double* sums, double vtpv, double* stats) {
    if (!p || !s || !sums || !stats) { set_error("NULL argument"); return FBA_ERR_ARG; }
    int64_t u = 0;
    fba_count_unknowns(p, s, &u);
    const double n = (double)p->n_pts;
    const double rx = std::sqrt(sums[0] / n), ry = std::sqrt(sums[1] / n);
    const double nu = (double)(2 * p->n_pts - u);
    stats[0] = rx; stats[1] = ry; stats[2] = std::sqrt(rx * rx + ry * ry);
    stats[3] = vtpv / nu; stats[4] = vtpv; stats[5] = nu;
    return FBA_OK;
}

int fba_last_timings(fba_ctx* ctx, double* ms) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !ms) { set_error("NULL argument"); return FBA_ERR_ARG; }
    for (int i = 0; i < 8; ++i) ms[i] = c->last_ms[i];
    return FBA_OK;
}

int fba_set_probe(fba_ctx* ctx, int32_t enabled) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    if (enabled < 0 || enabled > 2) { set_error("fba_set_probe: 0 (off), 1 (k_syrk_multi) or 2 (k_panel)"); return FBA_ERR_ARG; }
    c->probe = enabled;
    c->probe_n = 0;
    c->probe_flops = 0.0;
    return FBA_OK;
}

int fba_probe_stats(fba_ctx* ctx, double* out) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c || !out) { set_error("NULL argument"); return FBA_ERR_ARG; }
    FBA_HIP(hipStreamSynchronize(c->stream));
    double ms = 0.0;
    for (int i = 0; i < c->probe_n; ++i) {
        float t = 0.f;
        FBA_HIP(hipEventElapsedTime(&t, c->probe_ev[2 * i], c->probe_ev[2 * i + 1]));
        ms += t;
    }
    out[0] = c->probe_n;
    out[1] = ms;
    out[2] = c->probe_flops;
    out[3] = 0.0;
    return FBA_OK;
}

int fba_test_border_solve(int32_t device, const double* gram, double* coef) {
    if (!gram || !coef) { set_error("NULL argument"); return FBA_ERR_ARG; }
    return border_solve_selftest(device, gram, coef);
}

int fba_set_timing(fba_ctx* ctx, int32_t enabled) {
    Ctx* c = reinterpret_cast<Ctx*>(ctx);
    if (!c) { set_error("NULL context"); return FBA_ERR_ARG; }
    c->timing = enabled != 0;
    return FBA_OK;
}

}  // extern "C"
