// sched_check.cpp -- host-only check of the camera-side ordering and the level schedule of the
// block Cholesky (fish-eye_bundle_adjustment_amd/csrc/fba_order.cpp), built and run by
// tests/test_schedule.py (no GPU needed).
//
// A synthetic aerial block (images on a grid, tie points seen by the images within a radius) is
// ordered by camera_order(); build_schedule() makes the per-level task lists.  Then a random SPD
// matrix with exactly the block pattern of the reduced camera system (co-visible image pairs, the
// local border block, dense camera rows) plus 15 RHS rows is factored by EMULATING the kernels'
// schedule on the CPU (potrf per level column, panel solves per (k, r) task, trailing updates per
// target with its source list, backward solve per level), and compared with a plain dense
// Cholesky / solve of the same matrix.  It also checks that the task lists stay inside the
// matrix, that no two independent subtrees share a block, and that every padding slot is unused.
//
//   sched_check <n_img> <seed>     prints "ok levels=<L> blocks=<B> err=<e>" or "FAIL ..."
//   sched_check <n_img> 0 <file>   ordering statistics only, for the observations in <file>
//                                  (int64 n_pts, int32 img[n_pts], int32 tie[n_pts], f64 eop[6 n_img])
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <map>
#include <set>
#include <functional>

#include "../fish-eye_bundle_adjustment_amd/csrc/fba_internal.h"

using namespace fba;

static int fail(const char* m) {
    printf("FAIL %s\n", m);
    return 1;
}

int main(int argc, char** argv) {
    const int n_img = argc > 1 ? atoi(argv[1]) : 300;
    const int seed = argc > 2 ? atoi(argv[2]) : 1;
    std::mt19937_64 rng(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    // images on a grid (strips), tie points at random positions seen by images within a radius
    const int gw = std::max(1, (int)std::sqrt(n_img * 0.6));
    std::vector<double> ix(n_img), iy(n_img);
    for (int e = 0; e < n_img; ++e) { ix[e] = e % gw; iy[e] = e / gw; }
    std::vector<int32_t> img, tie, cam;
    std::vector<double> eop;
    int n_tie = 20 * n_img;
    const bool stats_only = argc > 3;
    if (stats_only) {
        FILE* f = fopen(argv[3], "rb");
        int64_t np = 0;
        if (!f || fread(&np, 8, 1, f) != 1) return fail("cannot read observation file");
        img.resize(np);
        tie.resize(np);
        cam.assign(np, 0);
        if (fread(img.data(), 4, np, f) != (size_t)np || fread(tie.data(), 4, np, f) != (size_t)np) return fail("short file");
        eop.assign(6 * (size_t)n_img, 0.0);
        if (fread(eop.data(), 8, eop.size(), f) != eop.size()) eop.clear();
        fclose(f);
        n_tie = 0;
        for (int32_t t : tie) n_tie = std::max(n_tie, t + 1);
    }
    for (int t = 0; t < n_tie && !stats_only; ++t) {
        const double px = U(rng) * gw, py = U(rng) * ((n_img + gw - 1) / gw);
        for (int e = 0; e < n_img; ++e)
            if (std::hypot(ix[e] - px, iy[e] - py) < 1.6) { img.push_back(e); tie.push_back(t); cam.push_back(0); }
    }
    fba_problem p{};
    p.n_pts = (int64_t)img.size();
    p.n_img = n_img;
    p.n_cam = 1;
    p.n_tie = n_tie;
    p.img = img.data();
    p.tie = tie.data();
    p.cam = cam.data();
    if (!stats_only) {  // image centres on the grid (spacing 1000), for the coordinate bisection
        eop.assign(6 * (size_t)n_img, 0.0);
        for (int e = 0; e < n_img; ++e) { eop[6 * e] = 1000.0 * ix[e]; eop[6 * e + 1] = 1000.0 * iy[e]; eop[6 * e + 2] = 800.0; }
    }
    p.eop0 = eop.empty() ? nullptr : eop.data();
    const std::vector<int32_t> ord = camera_order(&p);
    // every image exactly once, the rest padding
    {
        std::vector<int> seen(n_img, 0);
        for (int32_t v : ord)
            if (v >= 0) seen[v]++;
        for (int e = 0; e < n_img; ++e)
            if (seen[e] != 1) return fail("camera_order is not a permutation");
    }
    Ctx c;
    c.img_ord = ord;
    Layout& L = c.L;
    L.n_img = (int)ord.size();
    L.n_img_ref = n_img;
    L.n_cam = 1;
    L.cw = 10;
    L.u_c = 6 * (int64_t)L.n_img + L.cw;
    L.n_pad = (L.u_c + NB - 1) / NB * NB;
    L.ld = L.n_pad;
    L.nrhs = 15;
    c.n_loc = std::min(L.n_img, NB / 6);
    c.opt.verbose = stats_only ? 1 : 0;
    std::vector<int32_t> slot(n_img);
    for (int e = 0; e < L.n_img; ++e)
        if (ord[e] >= 0) slot[ord[e]] = e;
    std::set<std::pair<int32_t, int32_t>> ps;
    std::vector<size_t> by_tie(img.size());
    for (size_t q = 0; q < img.size(); ++q) by_tie[q] = q;
    std::stable_sort(by_tie.begin(), by_tie.end(), [&](size_t a, size_t b) { return tie[a] < tie[b]; });
    for (size_t a = 0; a < img.size();) {
        size_t b = a;
        while (b < img.size() && tie[by_tie[b]] == tie[by_tie[a]]) ++b;
        for (size_t x = a; x < b; ++x)
            for (size_t y = a; y < b; ++y)
                if (slot[img[by_tie[x]]] > slot[img[by_tie[y]]]) ps.insert({slot[img[by_tie[x]]], slot[img[by_tie[y]]]});
        a = b;
    }
    std::vector<std::pair<int32_t, int32_t>> pairs(ps.begin(), ps.end());
    build_schedule(c, pairs);
    const Sched& s = c.sched;
    // (SCHED_EMULATE=1 with an observation file: the emulation below on that network instead of the stats)
    if (stats_only && !getenv("SCHED_EMULATE")) {
        std::vector<int> per(s.n_waves);
        for (int w = 0; w < s.n_waves; ++w) per[w] = s.w[w].ncol;
        printf("ok levels=%d blocks=%ld slots=%d tiles=%ld cols/level:", s.n_waves, (long)(L.n_pad / NB), L.n_img,
               (long)s.n_tiles);
        for (int v : per) printf(" %d", v);
        printf("\n");
        for (int w = 0; w < s.n_waves; ++w) {  // per level: columns, panel halves, quarter tasks, GFLOP
            const int32_t* tk = s.buf.data() + s.w[w].tasks;
            int mx = 0;
            std::map<int, int> hist;
            for (int t = 0; t < s.w[w].ntask; ++t) {
                const int ns = tk[Sched::SYRK_REC * t + 4] - tk[Sched::SYRK_REC * t + 3];
                mx = std::max(mx, ns);
                hist[ns]++;
            }
            printf("level %2d: cols %3d trsm %4d tasks %5d comb %3d gflop %.3f max-src %d  src-hist:", w, s.w[w].ncol,
                   s.w[w].ntrsm, s.w[w].ntask, s.w[w].ncomb, s.w[w].flops * 1e-9, mx);
            for (auto& h : hist) printf(" %d:%d", h.first, h.second);
            printf("\n");
        }
        printf("scratch quarters %d\n", s.n_scratch);
        // work of the covariance's selected inversion (fba_cov.hip): per column k, |R_k| + |R_k|^2 + |R_k| + 1
        // 128^3 block products (R_k = the block rows below k, RHS row excluded)
        std::vector<int64_t> nr(L.n_pad / NB, 0);
        for (int w = 0; w < s.n_waves; ++w) {
            const int32_t* tr = s.buf.data() + s.w[w].trsm;
            for (int t = 0; t < s.w[w].ntrsm; ++t)
                if ((tr[2 * t + 1] & 1) == 0 && tr[2 * t + 1] / 2 < L.n_pad / NB) nr[tr[2 * t]]++;
        }
        double prods = 0.0;
        for (int64_t r : nr) prods += (double)(2 * r + r * r + 1);
        printf("selected inversion: %.0f block products, %.1f GFLOP\n", prods, prods * 2.0 * NB * NB * NB * 1e-9);
        for (int w : {2, 4, 8}) {  // the subtree split's cut (fba_options.split)
            Ctx cr;
            cr.img_ord = c.img_ord;
            cr.L = c.L;
            cr.n_loc = c.n_loc;
            cr.opt.verbose = 1;
            cr.opt.world = w;
            cr.opt.split = 1;
            build_schedule(cr, pairs);
        }
        return 0;
    }
    const int64_t n = L.n_pad, nb = n / NB, nr = n + NB;  // rows: matrix + RHS block row
    const int32_t* B = s.buf.data();
    const int64_t nbuf = (int64_t)s.buf.size();
    // matrix with the pattern of the reduced system; padding slots and padding rows decoupled
    std::vector<double> M((size_t)nr * n, 0.0);
    auto at = [&](int64_t r, int64_t q) -> double& { return M[(size_t)r * n + q]; };
    std::vector<char> used(n, 0);
    for (int e = 0; e < L.n_img; ++e)
        if (ord[e] >= 0)
            for (int a = 0; a < 6; ++a) used[6 * e + a] = 1;
    for (int64_t i = 6 * (int64_t)L.n_img; i < L.u_c; ++i) used[i] = 1;
    auto blk = [&](int64_t r0, int64_t c0) {  // random 6x6 coupling (lower part only)
        for (int a = 0; a < 6; ++a)
            for (int b = 0; b < 6; ++b)
                if (r0 + a > c0 + b) at(r0 + a, c0 + b) = (U(rng) - 0.5) * 0.05;
    };
    for (auto& q : pairs) blk(6 * (int64_t)q.first, 6 * (int64_t)q.second);
    for (int e = 0; e < L.n_img; ++e)
        if (ord[e] >= 0) blk(6 * (int64_t)e, 6 * (int64_t)e);
    for (int64_t i = 0; i < 6 * (int64_t)c.n_loc; ++i)  // local border block (dense)
        for (int64_t j = 0; j < i; ++j)
            if (used[i] && used[j]) at(i, j) += (U(rng) - 0.5) * 0.01;
    for (int64_t i = 6 * (int64_t)L.n_img; i < L.u_c; ++i)  // camera rows (dense)
        for (int64_t j = 0; j < i; ++j)
            if (used[j]) at(i, j) = (U(rng) - 0.5) * 0.01;
    for (int64_t i = 0; i < n; ++i) {  // diagonal dominance
        double r = 0.0;
        for (int64_t j = 0; j < n; ++j) r += std::fabs(j < i ? at(i, j) : at(j, i));
        at(i, i) = used[i] ? r + 1.0 + U(rng) : 1.0;
    }
    for (int64_t q = 0; q < 15; ++q)
        for (int64_t j = 0; j < n; ++j) at(n + q, j) = used[j] ? U(rng) - 0.5 : 0.0;
    std::vector<double> M0 = M;
    // -- the emulated schedule --
    auto Bk = [&](int64_t i, int64_t j) { return &M[(size_t)(i * NB) * n + j * NB]; };
    std::vector<int> done(nb, 0);
    for (int w = 0; w < s.n_waves; ++w) {
        const Sched::Wave& W = s.w[w];
        if (W.cols + W.ncol > nbuf || W.trsm + 2 * W.ntrsm > nbuf || W.tasks + Sched::SYRK_REC * W.ntask > nbuf ||
            W.comb + Sched::COMB_REC * W.ncomb > nbuf)
            return fail("list bounds");
        for (int q = 0; q < W.ncol; ++q) {  // potrf
            const int64_t k = B[W.cols + q];
            if (k < 0 || k >= nb || done[k]) return fail("potrf column");
            done[k] = 1;
            double* A = Bk(k, k);
            for (int j = 0; j < NB; ++j) {
                double d = A[(size_t)j * n + j];
                for (int t = 0; t < j; ++t) d -= A[(size_t)j * n + t] * A[(size_t)j * n + t];
                if (!(d > 0)) return fail("not SPD in emulation");
                d = std::sqrt(d);
                A[(size_t)j * n + j] = d;
                for (int i = j + 1; i < NB; ++i) {
                    double v = A[(size_t)i * n + j];
                    for (int t = 0; t < j; ++t) v -= A[(size_t)i * n + t] * A[(size_t)j * n + t];
                    A[(size_t)i * n + j] = v / d;
                }
            }
        }
        for (int q = 0; q < W.ntrsm; ++q) {  // X = A L^-T on one 64-row half
            const int64_t k = B[W.trsm + 2 * q], r = B[W.trsm + 2 * q + 1] >> 1, h = B[W.trsm + 2 * q + 1] & 1;
            if (k < 0 || k >= nb || !done[k] || r <= k || r > nb) return fail("trsm task");
            const double* Lk = Bk(k, k);
            double* X = Bk(r, k);
            for (int i = 64 * h; i < 64 * h + 64; ++i)
                for (int j = 0; j < NB; ++j) {
                    double v = X[(size_t)i * n + j];
                    for (int t = 0; t < j; ++t) v -= X[(size_t)i * n + t] * Lk[(size_t)j * n + t];
                    X[(size_t)i * n + j] = v / Lk[(size_t)j * n + j];
                }
        }
        std::vector<double> P((size_t)std::max(s.n_scratch, 1) * 4096, 0.0);
        std::vector<int> slot_used(std::max(s.n_scratch, 1), 0);
        for (int q = 0; q < W.ntask; ++q) {  // C quarter -= sum_k X_ik X_jk', or the group's partial
            const int32_t* tk = B + W.tasks + Sched::SYRK_REC * q;
            const int64_t i = tk[0], j = tk[1];
            const int qr = tk[2] >> 1, qc = tk[2] & 1, slot = tk[5];
            if (j < 0 || j >= nb || i < j || i > nb || done[j]) return fail("update target");
            if (i == j && qr == 0 && qc == 1) return fail("upper quarter of a diagonal block");
            if (slot >= s.n_scratch || (slot >= 0 && slot_used[slot]++)) return fail("scratch slot");
            int64_t prev = -1;
            for (int32_t u = tk[3]; u < tk[4]; ++u) {
                const int64_t k = B[W.src + u];
                if (k <= prev || !done[k]) return fail("update sources");
                prev = k;
                const double* Xi = Bk(i, k);
                const double* Xj = Bk(j, k);
                double* C = Bk(i, j);
                for (int a = 64 * qr; a < 64 * qr + 64; ++a)
                    for (int b = 64 * qc; b < 64 * qc + 64; ++b) {
                        if (i == j && b > a) continue;
                        double v = 0.0;
                        for (int t = 0; t < NB; ++t) v += Xi[(size_t)a * n + t] * Xj[(size_t)b * n + t];
                        if (slot < 0) C[(size_t)a * n + b] -= v;
                        else P[(size_t)slot * 4096 + (a - 64 * qr) * 64 + (b - 64 * qc)] -= v;
                    }
            }
        }
        for (int q = 0; q < W.ncomb; ++q) {  // split targets: C += the group partials in slot order
            const int32_t* cb = B + W.comb + Sched::COMB_REC * q;
            double* C = Bk(cb[0], cb[1]);
            const int qr = cb[2] >> 1, qc = cb[2] & 1;
            for (int g = 0; g < cb[4]; ++g) {
                if (cb[3] + g >= s.n_scratch || slot_used[cb[3] + g] != 1) return fail("combine slot");
                for (int a = 0; a < 64; ++a)
                    for (int b = 0; b < 64; ++b)
                        C[(size_t)(64 * qr + a) * n + 64 * qc + b] += P[(size_t)(cb[3] + g) * 4096 + a * 64 + b];
            }
        }
    }
    for (int64_t k = 0; k < nb; ++k)
        if (!done[k]) return fail("column never factored");
    // -- reference: dense right-looking Cholesky of the same matrix (RHS rows as extra rows) --
    std::vector<double> R = M0;
    auto rat = [&](int64_t r, int64_t q) -> double& { return R[(size_t)r * n + q]; };
    for (int64_t j = 0; j < n; ++j) {
        const double d = std::sqrt(rat(j, j));
        rat(j, j) = d;
        for (int64_t i = j + 1; i < nr; ++i) rat(i, j) /= d;
        for (int64_t q = j + 1; q < n; ++q) {
            const double f = rat(q, j);
            if (f == 0.0) continue;
            for (int64_t i = q; i < nr; ++i) rat(i, q) -= rat(i, j) * f;
        }
    }
    double err = 0.0, scale = 0.0;
    for (int64_t i = 0; i < nr; ++i)
        for (int64_t j = 0; j < std::min(i + 1, n); ++j) {
            // structurally-zero blocks of the emulation were never touched: compare every entry
            err = std::max(err, std::fabs(at(i, j) - rat(i, j)));
            scale = std::max(scale, std::fabs(rat(i, j)));
        }
    // -- backward solve by levels (k_bwd_wave) vs dense back substitution --
    std::vector<double> y(M.begin() + (size_t)n * n, M.begin() + (size_t)n * n + n), x(n, 0.0);
    for (int w = s.n_waves - 1; w >= 0; --w) {
        const Sched::BWave& Bw = s.b[w];
        auto solve_diag = [&](int64_t i, double* out) {  // out = L_ii^-T y_i
            const double* Lk = Bk(i, i);
            for (int a = NB - 1; a >= 0; --a) {
                double v = y[i * NB + a];
                for (int t = a + 1; t < NB; ++t) v -= Lk[(size_t)t * n + a] * out[t];
                out[a] = v / Lk[(size_t)a * n + a];
            }
        };
        std::vector<double> xs(NB);
        std::vector<std::vector<double>> upd;
        for (int q = 0; q < Bw.ntgt; ++q) {  // targets first read the level's y (as the kernel does)
            const int64_t j = B[Bw.tgts + q];
            std::vector<double> acc(NB, 0.0);
            for (int32_t u = B[Bw.src_start + q]; u < B[Bw.src_start + q + 1]; ++u) {
                const int64_t i = B[Bw.src + u];
                solve_diag(i, xs.data());
                const double* Lij = Bk(i, j);
                for (int b = 0; b < NB; ++b)
                    for (int a = 0; a < NB; ++a) acc[b] += Lij[(size_t)a * n + b] * xs[a];
            }
            upd.push_back(acc);
        }
        for (int q = 0; q < Bw.nsrc; ++q) {
            const int64_t i = B[Bw.srcs + q];
            solve_diag(i, &x[i * NB]);
        }
        for (int q = 0; q < Bw.ntgt; ++q) {
            const int64_t j = B[Bw.tgts + q];
            for (int b = 0; b < NB; ++b) y[j * NB + b] -= upd[q][b];
        }
    }
    std::vector<double> xr(n);
    for (int64_t a = n - 1; a >= 0; --a) {
        double v = rat(n, a);
        for (int64_t t = a + 1; t < n; ++t) v -= rat(t, a) * xr[t];
        xr[a] = v / rat(a, a);
    }
    double xerr = 0.0, xs_ = 0.0;
    for (int64_t a = 0; a < n; ++a) {
        xerr = std::max(xerr, std::fabs(x[a] - xr[a]));
        xs_ = std::max(xs_, std::fabs(xr[a]));
    }
    // independence: no block mixes the rows of two sibling subtrees (checked via the level count
    // being below the block count when a dissection happened)
    const double rel = err / scale, xrel = xerr / xs_;
    if (!(rel < 1e-12) || !(xrel < 1e-12)) {
        printf("FAIL factor err %.3e solve err %.3e\n", rel, xrel);
        return 1;
    }
    // -- the persistent dataflow schedule (k_chol_flow): records run to completion in an order the
    // dispatch can produce; every flag a record waits for must already be raised --
    std::vector<double> F = M0;
    auto Fk = [&](int64_t i, int64_t j) { return &F[(size_t)(i * NB) * n + j * NB]; };
    std::vector<unsigned> colf(nb, 0);
    auto solve_rows = [&](int64_t k, int64_t r, int i0, int i1) {  // rows i0..i1 of block (r, k): X = A L_kk^-T
        const double* Lk = Fk(k, k);
        double* X = Fk(r, k);
        for (int i = i0; i < i1; ++i)
            for (int j = 0; j < NB; ++j) {
                double v = X[(size_t)i * n + j];
                for (int t = 0; t < j; ++t) v -= X[(size_t)i * n + t] * Lk[(size_t)j * n + t];
                X[(size_t)i * n + j] = v / Lk[(size_t)j * n + j];
            }
    };
    // one flow: its records (at rec_off, n_rec), flag / counter / scratch spaces of its own; cols_ok(k):
    // the columns the flow may factor, tgt_ok(a, b): the blocks it may write (subtree split checks)
    struct FlowView { const int32_t* B; int64_t rec; int n, nfl, ncnt, nscr; int64_t nbuf; };
    auto emulate = [&](const FlowView& v, const std::function<bool(int64_t)>& cols_ok,
                       const std::function<bool(int64_t, int64_t)>& tgt_ok) -> int {
    const int32_t* B = v.B;
    std::vector<unsigned> fl((size_t)std::max(v.nfl, 1), 0), cntr(std::max(v.ncnt, 1), 0);
    std::vector<double> Pf((size_t)std::max(v.nscr, 1) * 4096, 0.0);
    std::vector<int> slot_set(std::max(v.nscr, 1), 0);
    auto flag_ok = [&](int32_t x, unsigned q) { return x >= 0 && x < (int32_t)fl.size() && fl[x] >= q; };
    if (v.rec + (int64_t)Sched::FLOW_REC * v.n > v.nbuf) return fail("flow record bounds");
    // records in the static ticket order (k_chol_flow: every wait points to an earlier record)
    std::vector<int> order;
    for (int b = 0; b < v.n; ++b) order.push_back(b);
    std::vector<char> ran(v.n, 0);
    // a split helper (role 4): tiles (ta, tb), tb >= FLOW_CSPLIT, of C_jj -= X X', X = L(j, f)
    auto run_helper = [&](const int32_t* rec) -> int {
        const int64_t j = rec[1], f = rec[2];
        if (colf[f] != 8 || f >= j) return fail("flow: split helper before its source");
        if (!flag_ok(rec[7], 8) || (rec[8] >= 0 && !flag_ok(rec[8], 8))) return fail("flow: split helper rows not solved");
        if (rec[10] < 0 || rec[10] >= v.nscr || slot_set[rec[10]]++) return fail("flow: split helper slot");
        const double* X = Fk(j, f);
        int h = 0;
        for (int ta = 0; ta < NB / 16; ++ta)
            for (int tb = FLOW_CSPLIT; tb <= ta; ++tb, ++h)
                for (int r = 0; r < 16; ++r)
                    for (int c2 = 0; c2 < 16; ++c2) {
                        double v = 0.0;
                        for (int t = 0; t < NB; ++t) v += X[(size_t)(16 * ta + r) * n + t] * X[(size_t)(16 * tb + c2) * n + t];
                        Pf[(size_t)rec[10] * 4096 + h * 256 + r * 16 + c2] = -v;
                    }
        fl[rec[9]] = 1;
        return 0;
    };
    for (int b : order) {
        const int32_t* rec = B + v.rec + (int64_t)Sched::FLOW_REC * b;
        if (ran[b]) continue;
        ran[b] = 1;
        if (rec[0] == 0) {
            const int64_t j = rec[1], f = rec[2];
            if (!cols_ok(j)) return fail("flow: diagonal block of a column outside the flow");
            for (int x = 0; x < rec[4]; ++x)
                if (!flag_ok(B[rec[3] + x], 1)) return fail("flow: diagonal block waits for an unset flag");
            double* C = Fk(j, j);
            if (f >= 0) {
                if (colf[f] != 8 || f >= j) return fail("flow: fused source not factored");
                if (!flag_ok(rec[7], 8) || (rec[8] >= 0 && !flag_ok(rec[8], 8))) return fail("flow: fused rows not solved");
                const double* X = Fk(j, f);
                // every column block; with a split helper (rec[9] >= 0) only the tile columns < FLOW_CSPLIT
                const int cmax = rec[9] >= 0 ? 16 * FLOW_CSPLIT : NB;
                for (int a = 0; a < NB; ++a)
                    for (int c2 = 0; c2 <= a && c2 < cmax; ++c2) {
                        double v = 0.0;
                        for (int t = 0; t < NB; ++t) v += X[(size_t)a * n + t] * X[(size_t)c2 * n + t];
                        C[(size_t)a * n + c2] -= v;
                    }
            }
            for (int e = 0; e < rec[6]; ++e) {
                const int32_t* l3 = B + rec[5] + 3 * e;
                if (!flag_ok(l3[2], 1) || !slot_set[l3[1]]) return fail("flow: late partial not ready");
                const int qr = l3[0] >> 1, qc = l3[0] & 1;
                for (int a = 0; a < 64; ++a)
                    for (int c2 = 0; c2 < 64; ++c2)
                        if (64 * qr + a >= 64 * qc + c2) C[(size_t)(64 * qr + a) * n + 64 * qc + c2] += Pf[(size_t)l3[1] * 4096 + a * 64 + c2];
            }
            if (rec[9] >= 0) {  // the split helper's partial (the potrf's bulk waves add it)
                if (!flag_ok(rec[9], 1) || rec[10] < 0 || rec[10] >= v.nscr || !slot_set[rec[10]])
                    return fail("flow: split helper partial not ready");
                int h = 0;
                for (int ta = 0; ta < NB / 16; ++ta)
                    for (int tb = FLOW_CSPLIT; tb <= ta; ++tb, ++h)
                        for (int r = 0; r < 16; ++r)
                            for (int c2 = 0; c2 < 16; ++c2)
                                if (16 * ta + r >= 16 * tb + c2)
                                    C[(size_t)(16 * ta + r) * n + 16 * tb + c2] += Pf[(size_t)rec[10] * 4096 + h * 256 + r * 16 + c2];
            }
            for (int jj = 0; jj < NB; ++jj) {  // potrf
                double d = C[(size_t)jj * n + jj];
                for (int t = 0; t < jj; ++t) d -= C[(size_t)jj * n + t] * C[(size_t)jj * n + t];
                if (!(d > 0)) return fail("flow: not SPD in emulation");
                d = std::sqrt(d);
                C[(size_t)jj * n + jj] = d;
                for (int i = jj + 1; i < NB; ++i) {
                    double v = C[(size_t)i * n + jj];
                    for (int t = 0; t < jj; ++t) v -= C[(size_t)i * n + t] * C[(size_t)jj * n + t];
                    C[(size_t)i * n + jj] = v / d;
                }
            }
            colf[j] = 8;
        } else if (rec[0] == 1) {
            const int64_t k = rec[1], r = rec[2] >> 1, h = rec[2] & 1;
            if (colf[k] != 8 || r <= k || r > nb) return fail("flow: panel half before its column");
            if (!cols_ok(k)) return fail("flow: panel half of a column outside the flow");
            for (int x = 0; x < rec[4]; ++x)
                if (!flag_ok(B[rec[3] + x], 1)) return fail("flow: panel half waits for an unset flag");
            solve_rows(k, r, 64 * (int)h, 64 * (int)h + 64);
            fl[rec[5]] = 8;
        } else if (rec[0] == 2 && rec[3] == 4) {  // a whole off-diagonal block (syrk_block_body)
            const int64_t a = rec[1], bb = rec[2];
            const int mode = rec[7];
            if (bb >= nb || a <= bb || a > nb) return fail("flow: block update target");
            if (!tgt_ok(a, bb)) return fail("flow: update target outside the flow's blocks");
            std::vector<double> acc(NB * NB, 0.0);
            for (int u = 0; u < rec[5]; ++u) {
                const int32_t* e = B + rec[4] + 5 * u;
                for (int x = 1; x <= 4; ++x)
                    if (!flag_ok(e[x], 8)) return fail("flow: block update source not published");
                const double* Xa = Fk(a, e[0]);
                const double* Xb = Fk(bb, e[0]);
                for (int x = 0; x < NB; ++x)
                    for (int y = 0; y < NB; ++y) {
                        double v = 0.0;
                        for (int t = 16 * rec[13]; t < 16 * rec[14]; ++t) v += Xa[(size_t)x * n + t] * Xb[(size_t)y * n + t];
                        acc[x * NB + y] -= v;
                    }
            }
            double* C = Fk(a, bb);
            auto add_c = [&](const double* src) {
                for (int x = 0; x < NB; ++x)
                    for (int y = 0; y < NB; ++y) C[(size_t)x * n + y] += src[x * NB + y];
            };
            if (mode == 0) {
                if (rec[9] >= 0 && !flag_ok(rec[9], 1)) return fail("flow: previous writer not done");
                add_c(acc.data());
                fl[rec[8]] = 1;
            } else {
                if (rec[6] < 0 || rec[6] + 4 > v.nscr) return fail("flow: block scratch slot");
                for (int g = 0; g < 4; ++g)
                    if (slot_set[rec[6] + g]++) return fail("flow: block scratch slot reused");
                std::copy(acc.begin(), acc.end(), Pf.begin() + (size_t)rec[6] * 4096);
                if (++cntr[rec[10]] == (unsigned)rec[12]) {
                    if (rec[9] >= 0 && !flag_ok(rec[9], 1)) return fail("flow: previous writer not done (combine)");
                    for (int g = 0; g < rec[12]; ++g) add_c(&Pf[(size_t)(rec[11] + 4 * g) * 4096]);
                    fl[rec[8]] = 1;
                }
            }
        } else if (rec[0] == 2) {
            const int64_t a = rec[1], bb = rec[2];
            const int qr = rec[3] >> 1, qc = rec[3] & 1, mode = rec[7];
            if (bb >= nb || a < bb || a > nb) return fail("flow: update target");
            if (!tgt_ok(a, bb)) return fail("flow: update target outside the flow's blocks");
            std::vector<double> acc(4096, 0.0);
            for (int u = 0; u < rec[5]; ++u) {
                const int32_t* tri = B + rec[4] + 3 * u;
                if (!flag_ok(tri[1], 8) || !flag_ok(tri[2], 8)) return fail("flow: update source not published");
                const double* Xa = Fk(a, tri[0]);
                const double* Xb = Fk(bb, tri[0]);
                if (rec[13] < 0 || rec[14] > 8 || rec[13] >= rec[14]) return fail("flow: update column-block range");
                for (int x = 0; x < 64; ++x)
                    for (int y = 0; y < 64; ++y) {
                        double v = 0.0;
                        for (int t = 16 * rec[13]; t < 16 * rec[14]; ++t)
                            v += Xa[(size_t)(64 * qr + x) * n + t] * Xb[(size_t)(64 * qc + y) * n + t];
                        acc[x * 64 + y] -= v;
                    }
            }
            double* C = Fk(a, bb);
            auto add_c = [&](const double* src) {
                for (int x = 0; x < 64; ++x)
                    for (int y = 0; y < 64; ++y) C[(size_t)(64 * qr + x) * n + 64 * qc + y] += src[x * 64 + y];
            };
            if (mode == 0) {
                if (rec[9] >= 0 && !flag_ok(rec[9], 1)) return fail("flow: previous writer not done");
                add_c(acc.data());
                fl[rec[8]] = 1;
            } else {
                if (rec[6] < 0 || rec[6] >= v.nscr || slot_set[rec[6]]++) return fail("flow: scratch slot");
                std::copy(acc.begin(), acc.end(), Pf.begin() + (size_t)rec[6] * 4096);
                if (mode == 2) {
                    fl[rec[8]] = 1;
                } else if (++cntr[rec[10]] == (unsigned)rec[12]) {
                    if (rec[9] >= 0 && !flag_ok(rec[9], 1)) return fail("flow: previous writer not done (combine)");
                    for (int g = 0; g < rec[12]; ++g) add_c(&Pf[(size_t)(rec[11] + g) * 4096]);
                    fl[rec[8]] = 1;
                }
            }
        } else if (rec[0] == 3) {
            if (colf[rec[1]] != 8) return fail("flow: inverse before its factor");
        } else if (rec[0] == 4) {
            if (run_helper(rec)) return 1;
        } else {
            return fail("flow: record role");
        }
    }
    return 0;
    };
    if (!s.flow_ok) return fail("flow schedule order check");
    const char* sw = getenv("SCHED_SPLIT_WORLD");
    const int split_world = sw ? atoi(sw) : 0;
    if (split_world > 1) {
        // subtree split: every rank's flow A on the same matrix (their updates of the top blocks add up
        // in place, as the all-reduce sums them), then the top flow B; each rank's flow may only factor
        // its own columns and write its own or top blocks
        std::vector<int> seen(nb, 0);
        std::vector<Sched> per(split_world);
        for (int r = 0; r < split_world; ++r) {
            Ctx cr;
            cr.img_ord = c.img_ord;
            cr.L = c.L;
            cr.n_loc = c.n_loc;
            cr.opt.verbose = 0;
            cr.opt.rank = r;
            cr.opt.world = split_world;
            cr.opt.split = 1;
            build_schedule(cr, pairs);
            per[r] = cr.sched;
            if (!per[r].split) return fail("split: no subtree split");
            if (per[r].blk_rank != per[0].blk_rank) return fail("split: ranks disagree on the cut");
            if (!per[r].flow_ok || !per[r].top.ok) return fail("split: flow order check");
        }
        const std::vector<int32_t>& br = per[0].blk_rank;
        for (int64_t k = 0; k < nb; ++k) seen[k] = br[k];
        for (int r = 0; r < split_world; ++r) {
            const Sched& q = per[r];
            FlowView v{q.buf.data(), q.flow_rec, q.flow_n, q.flow_nprog + q.flow_nuflag, q.flow_ncounter, q.flow_nscratch,
                       (int64_t)q.buf.size()};
            auto own = [&](int64_t k) { return k < nb && br[k] == r; };
            auto topb = [&](int64_t k) { return k == nb || br[k] < 0; };
            if (emulate(v, own, [&](int64_t a, int64_t bb) { return (own(a) || topb(a)) && (own(bb) || topb(bb)); })) return 1;
            for (int64_t k = 0; k < nb; ++k)
                if (own(k) && colf[k] != 8) return fail("split: a subtree column left unfactored");
        }
        const Sched& q = per[0];
        FlowView vt{q.buf.data(), q.top.rec, q.top.n, q.top.nprog + q.top.nuflag, q.top.ncounter, q.top.nscratch,
                    (int64_t)q.buf.size()};
        auto topc = [&](int64_t k) { return k < nb && br[k] < 0; };
        if (emulate(vt, topc, [&](int64_t a, int64_t bb) { return (a == nb || br[a] < 0) && br[bb] < 0; })) return 1;
        int ntop = 0;
        for (int64_t k = 0; k < nb; ++k) {
            if (colf[k] != 8) return fail("split: a column left unfactored");
            ntop += br[k] < 0;
        }
        printf("split world=%d top_columns=%d top_blocks=%d ", split_world, ntop, per[0].n_top_blocks);
    } else {
        FlowView v{s.buf.data(), s.flow_rec, s.flow_n, s.flow_nprog + s.flow_nuflag, s.flow_ncounter, s.flow_nscratch, nbuf};
        if (emulate(v, [](int64_t) { return true; }, [](int64_t, int64_t) { return true; })) return 1;
    }
    double ferr = 0.0;
    for (int64_t i = 0; i < nr; ++i)
        for (int64_t j = 0; j < std::min(i + 1, n); ++j) ferr = std::max(ferr, std::fabs(F[(size_t)i * n + j] - rat(i, j)));
    const double frel = ferr / scale;
    if (!(frel < 1e-12)) {
        printf("FAIL flow factor err %.3e\n", frel);
        return 1;
    }
    int ncomb = 0;
    for (int w = 0; w < s.n_waves; ++w) ncomb += s.w[w].ncomb;
    printf("ok levels=%d blocks=%ld slots=%d split=%d err=%.3e xerr=%.3e flow_err=%.3e flow_records=%d\n", s.n_waves, (long)nb,
           L.n_img, ncomb, rel, xrel, frel, s.flow_n);
    return 0;
}
