// fba_order.cpp -- camera-side ordering and the block schedule of the reduced-system Cholesky.
//
// The reference inverts the whole normal matrix (main.m:438-440); here the tie points are eliminated
// first and the reduced camera system S (images, then cameras) is factored by 128x128 blocks.  Its
// image-image part is sparse: images are coupled only when they share a tie point.  This file
//   1. orders the images by nested dissection of their co-visibility graph (level-structure
//      bisection, reverse Cuthill-McKee inside the leaves and the separators), padding with unused
//      image slots so that two independent subtrees never share a 128-row block;
//   2. runs the block-level symbolic factorisation (fill of the lower block pattern), and
//   3. groups the block columns by their level in the elimination tree.  Columns of one level are
//      independent, so each level is ONE batched step (potrf | panel solves | trailing updates) and
//      the factorisation's critical path is the tree height, not the block count: at config 4
//      (1,000 images) 21 steps instead of 47, at config 5 (4,000 images) 38 instead of 188.
// Trailing-update targets that several columns of a level update are summed in one workgroup in
// ascending column order, so results do not depend on the schedule (no floating-point atomics).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <map>
#include <queue>
#include <tuple>

#include "fba_internal.h"

namespace fba {

namespace {

struct Graph {
    int n = 0;
    std::vector<int32_t> start, adj;  // CSR, no self loops, neighbours ascending
};

Graph covis_graph(const fba_problem* p) {
    Graph g;
    g.n = p->n_img;
    std::vector<std::pair<int32_t, int32_t>> ti;  // (tie, image)
    for (int64_t i = 0; i < p->n_pts; ++i)
        if (p->tie[i] >= 0) ti.emplace_back(p->tie[i], p->img[i]);
    std::sort(ti.begin(), ti.end());
    std::vector<std::pair<int32_t, int32_t>> edges;
    for (size_t a = 0; a < ti.size();) {
        size_t b = a;
        while (b < ti.size() && ti[b].first == ti[a].first) ++b;
        for (size_t x = a; x < b; ++x)
            for (size_t y = a; y < b; ++y)
                if (ti[x].second != ti[y].second) edges.emplace_back(ti[x].second, ti[y].second);
        a = b;
    }
    std::sort(edges.begin(), edges.end());
    edges.erase(std::unique(edges.begin(), edges.end()), edges.end());
    g.start.assign(g.n + 1, 0);
    g.adj.resize(edges.size());
    for (auto& e : edges) g.start[e.first + 1]++;
    for (int v = 0; v < g.n; ++v) g.start[v + 1] += g.start[v];
    for (size_t q = 0; q < edges.size(); ++q) g.adj[q] = edges[q].second;
    return g;
}

class Dissection {
  public:
    // pos: image centres (3 per image) for coordinate bisection, or empty (level-structure bisection)
    Dissection(const Graph& g, int leaf, std::vector<double> pos)
        : g_(g), leaf_(leaf), pos_(std::move(pos)), tag_(g.n, -1), lev_(g.n, -1), deg_(g.n, 0) {}

    // order the vertices (all of one tag), appending to out; -1 entries are padding slots
    void nd(std::vector<int32_t> verts, std::vector<int32_t>& out) {
        if ((int)verts.size() <= leaf_) return rcm(verts, out);
        std::vector<int32_t> A, B, S;
        if (!(pos_.empty() ? bisect(verts, A, B, S) : bisect_geo(verts, A, B, S))) return rcm(verts, out);
        verts.clear();
        verts.shrink_to_fit();
        nd(std::move(A), out);
        // B starts in a fresh 128-row block: A and B then share no block and factor independently
        const int64_t e = (int64_t)out.size();
        const int64_t m = (6 * e + NB - 1) / NB;
        const int64_t e1 = (NB * m + 5) / 6;
        out.insert(out.end(), (size_t)(e1 - e), -1);
        nd(std::move(B), out);
        rcm(S, out);
    }

  private:
    const Graph& g_;
    int leaf_;
    std::vector<double> pos_;
    int next_ = 0;
    int frac_lo_ = 45, frac_hi_ = 55, frac_step_ = 1;
    std::vector<int> tag_, lev_, deg_;

    int mark(const std::vector<int32_t>& verts) {
        const int t = next_++;
        for (int32_t v : verts) tag_[v] = t;
        for (int32_t v : verts) {
            int d = 0;
            for (int32_t q = g_.start[v]; q < g_.start[v + 1]; ++q) d += tag_[g_.adj[q]] == t;
            deg_[v] = d;
        }
        return t;
    }

    // BFS from root inside tag t; returns the vertices reached in BFS order, lev_ set
    std::vector<int32_t> bfs(int root, int t) {
        std::vector<int32_t> order{root};
        lev_[root] = 0;
        for (size_t h = 0; h < order.size(); ++h) {
            const int v = order[h];
            for (int32_t q = g_.start[v]; q < g_.start[v + 1]; ++q) {
                const int w = g_.adj[q];
                if (tag_[w] == t && lev_[w] < 0) {
                    lev_[w] = lev_[v] + 1;
                    order.push_back(w);
                }
            }
        }
        return order;
    }
    void clear_lev(const std::vector<int32_t>& vs) {
        for (int32_t v : vs) lev_[v] = -1;
    }

    void rcm(const std::vector<int32_t>& verts, std::vector<int32_t>& out) {
        const int t = mark(verts);
        std::vector<int32_t> roots(verts);
        std::stable_sort(roots.begin(), roots.end(), [&](int32_t a, int32_t b) { return deg_[a] < deg_[b]; });
        std::vector<int32_t> order;
        order.reserve(verts.size());
        for (int32_t r : roots) {
            if (lev_[r] >= 0) continue;
            size_t h = order.size();
            order.push_back(r);
            lev_[r] = 0;
            while (h < order.size()) {
                const int v = order[h++];
                std::vector<int32_t> nb;
                for (int32_t q = g_.start[v]; q < g_.start[v + 1]; ++q) {
                    const int w = g_.adj[q];
                    if (tag_[w] == t && lev_[w] < 0) nb.push_back(w);
                }
                std::stable_sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) { return deg_[a] < deg_[b]; });
                for (int32_t w : nb) {
                    lev_[w] = 0;
                    order.push_back(w);
                }
            }
        }
        clear_lev(verts);
        out.insert(out.end(), order.rbegin(), order.rend());
    }

    // coordinate bisection: cut the images across the principal axis of their centres (a flight
    // block's long side), the cut placed where the one-sided vertex separator (the images of one
    // side that share a tie point with the other side) is smallest within 40-60 % of the images
    bool bisect_geo(const std::vector<int32_t>& verts, std::vector<int32_t>& A, std::vector<int32_t>& B,
                    std::vector<int32_t>& S) {
        const int t = mark(verts);
        const size_t n = verts.size();
        double mu[3] = {0, 0, 0}, C[3][3] = {};
        for (int32_t v : verts)
            for (int d = 0; d < 3; ++d) mu[d] += pos_[3 * v + d] / (double)n;
        for (int32_t v : verts)
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) C[a][b] += (pos_[3 * v + a] - mu[a]) * (pos_[3 * v + b] - mu[b]);
        double ax[3] = {1.0, 0.7, 0.3};
        for (int it = 0; it < 100; ++it) {  // power iteration: principal axis
            double y[3] = {0, 0, 0}, nn = 0.0;
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) y[a] += C[a][b] * ax[b];
            for (int a = 0; a < 3; ++a) nn += y[a] * y[a];
            if (!(nn > 0.0)) return false;
            nn = std::sqrt(nn);
            for (int a = 0; a < 3; ++a) ax[a] = y[a] / nn;
        }
        // candidate cut directions: the principal axis, the coordinate axes of the plane and the two
        // diagonals (a near-square block has no meaningful principal axis; a diagonal cut is ~1.4x longer)
        std::vector<std::array<double, 3>> axes{{ax[0], ax[1], ax[2]}, {1, 0, 0}, {0, 1, 0},
                                                {0.7071067811865476, 0.7071067811865476, 0},
                                                {0.7071067811865476, -0.7071067811865476, 0}};
        // separator of a cut (vertices of rank < cut on the left): a minimum vertex cover of the cut
        // edges (Koenig, from a maximum matching of the bipartite graph left- x right-boundary), never
        // larger than either side's boundary; returns the cover as a flag per vertex of `sep`
        std::vector<int> slot(g_.n, -1);
        auto cover = [&](const std::vector<std::pair<double, int32_t>>& ord, size_t cut, std::vector<int32_t>& sep) {
            std::vector<int32_t> lb, rb;
            for (size_t q = 0; q < n; ++q) {
                const int32_t v = ord[q].second;
                const bool left = q < cut;
                bool cross = false;
                for (int32_t e = g_.start[v]; e < g_.start[v + 1] && !cross; ++e) {
                    const int w = g_.adj[e];
                    cross = tag_[w] == t && (((size_t)lev_[w] < cut) != left);
                }
                if (cross) (left ? lb : rb).push_back(v);
            }
            for (size_t a = 0; a < lb.size(); ++a) slot[lb[a]] = (int)a;
            for (size_t b = 0; b < rb.size(); ++b) slot[rb[b]] = (int)b;
            std::vector<std::vector<int>> nbr(lb.size());
            for (size_t a = 0; a < lb.size(); ++a)
                for (int32_t e = g_.start[lb[a]]; e < g_.start[lb[a] + 1]; ++e) {
                    const int w = g_.adj[e];
                    if (tag_[w] == t && (size_t)lev_[w] >= cut) nbr[a].push_back(slot[w]);
                }
            std::vector<int> ml(lb.size(), -1), mr(rb.size(), -1), seen(rb.size(), -1);
            std::function<bool(int, int)> augment = [&](int a, int stamp) -> bool {
                for (int b : nbr[a]) {
                    if (seen[b] == stamp) continue;
                    seen[b] = stamp;
                    if (mr[b] < 0 || augment(mr[b], stamp)) { ml[a] = b; mr[b] = a; return true; }
                }
                return false;
            };
            for (size_t a = 0; a < lb.size(); ++a) augment((int)a, (int)a);
            // Z = reachable from unmatched left vertices by alternating paths; cover = (L \ Z) + (R & Z)
            std::vector<char> zl(lb.size(), 0), zr(rb.size(), 0);
            std::vector<int> stack;
            for (size_t a = 0; a < lb.size(); ++a)
                if (ml[a] < 0) { zl[a] = 1; stack.push_back((int)a); }
            while (!stack.empty()) {
                const int a = stack.back();
                stack.pop_back();
                for (int b : nbr[a]) {
                    if (zr[b]) continue;
                    zr[b] = 1;
                    if (mr[b] >= 0 && !zl[mr[b]]) { zl[mr[b]] = 1; stack.push_back(mr[b]); }
                }
            }
            sep.clear();
            for (size_t a = 0; a < lb.size(); ++a)
                if (!zl[a]) sep.push_back(lb[a]);
            for (size_t b = 0; b < rb.size(); ++b)
                if (zr[b]) sep.push_back(rb[b]);
            for (int32_t v : lb) slot[v] = -1;
            for (int32_t v : rb) slot[v] = -1;
        };
        std::vector<std::pair<double, int32_t>> pr(n), best_pr;
        std::vector<int32_t> best_sep_v;
        size_t best_cut = n / 2, best_sep = n + 1;
        for (const auto& a3 : axes) {
            for (size_t q = 0; q < n; ++q) {
                const int32_t v = verts[q];
                double x = 0.0;
                for (int d = 0; d < 3; ++d) x += (pos_[3 * v + d] - mu[d]) * a3[d];
                pr[q] = {x, v};
            }
            std::sort(pr.begin(), pr.end());
            for (size_t q = 0; q < n; ++q) lev_[pr[q].second] = (int)q;  // rank along the axis
            // the cut is chosen by the smaller one-sided boundary (choosing by the cover size measured
            // worse: it favours unbalanced cuts and deeper trees); its separator is then the cover
            for (int f = frac_lo_; f <= frac_hi_; f += frac_step_) {
                const size_t cut = n * f / 100;
                if (cut == 0 || cut >= n) continue;
                size_t sl = 0, sr = 0;  // left vertices with a right neighbour, and vice versa
                for (size_t q = 0; q < n; ++q) {
                    const int32_t v = pr[q].second;
                    const bool left = q < cut;
                    for (int32_t e = g_.start[v]; e < g_.start[v + 1]; ++e) {
                        const int w = g_.adj[e];
                        if (tag_[w] != t) continue;
                        if (((size_t)lev_[w] < cut) != left) { (left ? sl : sr)++; break; }
                    }
                }
                if (std::min(sl, sr) < best_sep) {
                    best_sep = std::min(sl, sr);
                    best_cut = cut;
                    best_pr = pr;
                }
            }
        }
        if (best_pr.empty()) return false;
        for (size_t q = 0; q < n; ++q) lev_[best_pr[q].second] = (int)q;
        cover(best_pr, best_cut, best_sep_v);
        std::vector<char> insep(g_.n, 0);
        for (int32_t v : best_sep_v) insep[v] = 1;
        for (size_t q = 0; q < n; ++q) {
            const int32_t v = best_pr[q].second;
            if (insep[v]) S.push_back(v);
            else (q < best_cut ? A : B).push_back(v);
        }
        clear_lev(verts);
        std::sort(A.begin(), A.end());
        std::sort(B.begin(), B.end());
        return !A.empty() && !B.empty();
    }

    // level-structure bisection: A | separator S (one BFS level) | B, no edge between A and B
    bool bisect(const std::vector<int32_t>& verts, std::vector<int32_t>& A, std::vector<int32_t>& B,
                std::vector<int32_t>& S) {
        const int t = mark(verts);
        int root = verts[0];
        for (int32_t v : verts)
            if (deg_[v] < deg_[root] || (deg_[v] == deg_[root] && v < root)) root = v;
        std::vector<int32_t> reach;
        int ecc = -1;
        for (int it = 0; it < 4; ++it) {  // pseudo-peripheral root
            reach = bfs(root, t);
            const int e = lev_[reach.back()];
            int far = root;
            for (int32_t v : reach)
                if (lev_[v] == e && (far == root || deg_[v] < deg_[far] || (deg_[v] == deg_[far] && v < far))) far = v;
            if (e <= ecc) break;
            ecc = e;
            clear_lev(reach);
            root = far;
        }
        clear_lev(reach);
        reach = bfs(root, t);
        const int maxl = lev_[reach.back()];
        if (maxl < 2) { clear_lev(reach); return false; }
        std::vector<int64_t> cnt(maxl + 1, 0);
        for (int32_t v : reach) cnt[lev_[v]]++;
        const double half = 0.5 * (double)verts.size();
        int best = 1;
        double bscore = 1e300;
        int64_t cum = 0;
        for (int l = 0; l <= maxl; ++l) {
            if (l >= 1 && l <= maxl - 1) {
                const double score = std::fabs((double)cum + 0.5 * (double)cnt[l] - half);
                if (score < bscore || (score == bscore && cnt[l] < cnt[best])) { bscore = score; best = l; }
            }
            cum += cnt[l];
        }
        // sides: 0 = A, 1 = S, 2 = B (unreached components go to B)
        std::vector<int32_t> sepv;
        for (int32_t v : verts) {
            const int l = lev_[v];
            if (l >= 0 && l < best) A.push_back(v);
            else if (l == best) sepv.push_back(v);
            else B.push_back(v);
        }
        clear_lev(reach);
        for (int32_t v : A) lev_[v] = 0;
        for (int32_t v : sepv) lev_[v] = 1;
        for (int32_t v : B) lev_[v] = 2;
        for (int32_t v : sepv) {  // a separator vertex without a neighbour on one side joins the other
            bool inA = false, inB = false;
            for (int32_t q = g_.start[v]; q < g_.start[v + 1]; ++q) {
                const int w = g_.adj[q];
                if (tag_[w] != t) continue;
                inA |= lev_[w] == 0;
                inB |= lev_[w] == 2;
            }
            if (!inB) { lev_[v] = 0; A.push_back(v); }
            else if (!inA) { lev_[v] = 2; B.push_back(v); }
            else S.push_back(v);
        }
        clear_lev(verts);
        std::sort(A.begin(), A.end());
        std::sort(B.begin(), B.end());
        return !A.empty() && !B.empty();
    }
};

}  // namespace

std::vector<int32_t> camera_order(const fba_problem* p) {
    const char* le = getenv("FBA_ND_LEAF");
    // levels at configs 3 / 4 / 5 (cuts along the best of five directions, minimum-vertex-cover
    // separators): leaf 100 -> 7 / 16 / 31, 150 -> 7 / 17 / 31; config 4 measured 808-812 iter/s at 100,
    // 804 at 120, 776-778 at 150 (round 1).  Round 5, same box: config 4 1,266-1,272 at 100, 1,270-1,277
    // at 130, 1,251-1,270 at 120; config 5 282.8 at 100, 288.9 / 289.1 at 160, 284.9 at 200, 281-282 at
    // 250 / 320; config 3 flat -- larger scenes take larger leaves: 100 (n / 1000)^(1/3), at least 100
    int leaf = le ? atoi(le) : std::max(100, (int)std::lround(100.0 * std::cbrt(p->n_img / 1000.0)));
    if (leaf <= 0) leaf = p->n_img;  // 0: reverse Cuthill-McKee only
    Graph g = covis_graph(p);
    std::vector<int32_t> all(p->n_img), out;
    for (int v = 0; v < p->n_img; ++v) all[v] = v;
    out.reserve(p->n_img + p->n_img / 8);
    // coordinate bisection on the approximate image centres when they span the block (otherwise a
    // level-structure bisection of the graph alone)
    std::vector<double> pos;
    if (p->eop0) {
        pos.resize(3 * (size_t)p->n_img);
        double lo = 1e300, hi = -1e300;
        for (int v = 0; v < p->n_img; ++v)
            for (int d = 0; d < 3; ++d) {
                pos[3 * v + d] = p->eop0[6 * (int64_t)v + d];
                lo = std::min(lo, pos[3 * v + d]);
                hi = std::max(hi, pos[3 * v + d]);
            }
        if (!(hi > lo) || !std::isfinite(hi - lo)) pos.clear();
    }
    Dissection(g, std::max(leaf, 1), std::move(pos)).nd(std::move(all), out);
    return out;
}

// Persistent dataflow schedule of the whole block factorisation (k_chol_flow).  Records (one
// workgroup each):
//   diagonal block j   waits for the final in-place writers of its diagonal quarters, loads C_jj into
//                      LDS, then applies its FUSED source f_j (the source of the highest elimination-
//                      tree level, then the highest index) itself: C_jj -= X X' column block by column
//                      block as the two panel-half records of (f_j, j) publish X = L(j, f_j) -- so the
//                      last hand-off before its potrf is panel solve -> diagonal workgroup, with no
//                      update task and no write-back of C_jj in between; adds the late partials (other
//                      sources of f_j's level); then the potrf, publishing its column blocks
//   panel half (k,r,h) solves as k's column blocks are published, publishes each solved column block
//                      (progress flag = column blocks done)
//   update task        C(a,b) quarter += -sum X_ak X_bk' over the sources of ONE level (<= SPLIT per
//                      task), consuming the sources' column blocks as they are published; in place
//                      after the previous level's writer of the quarter, or via scratch partials
//                      combined by the last group; diagonal contributions of the fused source's own
//                      level other than the fused source ("late") go to scratch partials
//   inverse            of every diagonal block below the top level (k_bwd_flow, covariance)
// Dispatch order: a topological order of the record dependencies picking, among the ready records,
// the smallest (level of need, role rank): diagonal blocks first (each placed right after the last
// record it waits for), then panel halves, the updates feeding the next level, the others, inverses.
// Every wait points to an earlier record, so in-order dispatch always progresses (checked here).
// inc (subtree split): the block columns whose records this flow holds -- their diagonal blocks,
// panel halves and inverses, and the updates they source, whatever the target; nullptr: every column
static void build_flow(Sched& s, std::vector<int32_t>& buf, const std::vector<std::vector<int32_t>>& R,
                       const std::vector<int32_t>& level, int64_t nb, const std::function<int64_t(int64_t)>& real_rows,
                       bool verbose, const std::vector<char>* inc = nullptr) {
    auto in = [&](int64_t k) { return !inc || (*inc)[k] != 0; };
    constexpr int REC = Sched::FLOW_REC, CB_BLOCKS = NB / 16;
    // sources per update task (FBA_FLOW_SPLIT; a target quarter's sources of one level are split into
    // groups of at most SPLIT, summed through scratch partials when there are several groups); config 4
    // (iter/s, two runs each): 1: 1050, 2: 1120 / 1137, 3: 1153 / 1143, 4: 1152 / 1147, all in one: 1087
    // -- fewer update records hold fewer CUs while waiting for their sources' columns
    const int SPLIT = getenv("FBA_FLOW_SPLIT") ? std::max(1, atoi(getenv("FBA_FLOW_SPLIT"))) : 4;
    const int nw = nb > 0 ? 1 + *std::max_element(level.begin(), level.end()) : 0;
    std::vector<std::vector<int32_t>> srcs(nb);
    for (int64_t k = 0; k < nb; ++k)
        for (int32_t i : R[k])
            if (i < nb && in(k)) srcs[i].push_back((int32_t)k);
    // (dispatch keys by as-late-as-possible levels measured slower: config 4 1197-1202 vs 1238-1244
    // iter/s -- a shallow subtree's records dispatched late then hold the CUs when the chain's arrive)
    auto kl = [&](int64_t x) { return level[x]; };
    std::vector<int32_t> fsrc(nb, -1);
    for (int64_t j = 0; j < nb; ++j)
        for (int32_t k : srcs[j])
            if (in(j))
            if (fsrc[j] < 0 || level[k] > level[fsrc[j]] || (level[k] == level[fsrc[j]] && k > fsrc[j])) fsrc[j] = k;
    auto halves = [&](int64_t r) { return real_rows(r) > NB / 2 ? 2 : 1; };
    // the fused source's panel rows of block j are solved by two panel-half records and handed to j's
    // diagonal workgroup (that workgroup solving them itself measured slower: config 4 1133-1139 vs
    // 1222-1228 iter/s -- one CU's f64 MFMA rate then paces the panel solve plus the fused update)
    // progress flags of every panel half (k, r, h), r in R[k] (the RHS block row included)
    std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t> prog;
    int np = 0;
    for (int64_t k = 0; k < nb; ++k)
        for (int32_t r : R[k]) {
            if (!in(k)) break;
            for (int h = 0; h < halves(r); ++h) prog[std::make_tuple((int32_t)k, r, h)] = np++;
        }
    struct Task {
        std::array<int32_t, REC> rec;
        std::array<int, 3> key;  // level of need, role rank, tie-break
        std::vector<int> deps;   // producer records (flags resolved below)
    };
    std::vector<Task> T;
    std::vector<int> col_task(nb, -1), prog_task(np, -1);
    std::vector<std::vector<int>> uflag_tasks;  // update flag -> the records that may raise it
    std::vector<std::vector<int32_t>> flag_deps;  // per record: flags it waits for (resolved to records)
    auto new_uflag = [&]() { uflag_tasks.emplace_back(); return (int32_t)(np + uflag_tasks.size() - 1); };
    auto add = [&](std::initializer_list<int32_t> r, std::array<int, 3> key) {
        Task t;
        t.rec.fill(0);
        int q = 0;
        for (int32_t v : r) t.rec[q++] = v;
        t.key = key;
        T.push_back(std::move(t));
        flag_deps.emplace_back();
        return (int)T.size() - 1;
    };
    // the tile-column split of the fused updates (helper records, role 4): the
    // diagonal workgroup applies the tiles of tile columns < FLOW_CSPLIT, a helper workgroup the others
    // (consuming the same published rows) into a scratch partial that the potrf's bulk waves add at
    // their step FLOW_CSPLIT - 2, well after the potrf has started -- so the update's arithmetic no
    // longer trails the panel solves (the diagonal workgroup alone is MFMA-bound at ~1.5 us per
    // column block, behind panel halves that publish one every ~1-2 us).  (Measured and not kept: the
    // fused update's first column blocks on helper update tasks, 1076-1096 vs 1129 iter/s; panel halves
    // promoted a level, 1102-1126 vs 1125-1130; update tasks deferred towards their need, 724-1035 --
    // an update deferred lands on the critical path.)
    // FBA_FLOW_MERGE = G: writer groups over consecutive source levels when the target is read >= G levels later
    // (config 4, k_chol_flow per launch: G = 0 / 1 / 2 / 3: 465 / 458 / 453 / 454 us; convergent config 4:
    // 3.80 / 3.18 / 3.22 ms); FBA_FLOW_MSPLIT: the sources a merged group may hold (default SPLIT)
    // (default: 2 for a quarter-record schedule, 1 for a whole-block one, decided below -- same-box A/B, three
    // runs each, G = 2 / 1: convergent config 4 270.0 / 273.8 iter/s, config 5 280.4 / 282.2, config 4 1,266 / 1,258)
    int merge_gap = getenv("FBA_FLOW_MERGE") ? atoi(getenv("FBA_FLOW_MERGE")) : -1;
    const int msplit = getenv("FBA_FLOW_MSPLIT") ? std::max(1, atoi(getenv("FBA_FLOW_MSPLIT"))) : SPLIT;
    int nslot = 0, ncnt = 0, n_whole_t = 0;
    // diagonal blocks
    for (int64_t j = 0; j < nb; ++j) {
        if (!in(j)) continue;
        const int32_t f = fsrc[j];
        int need = kl(j) - 1;
        const int32_t p0 = f >= 0 ? prog[std::make_tuple(f, (int32_t)j, 0)] : -1;
        const int32_t p1 = (f >= 0 && halves(j) > 1) ? prog[std::make_tuple(f, (int32_t)j, 1)] : -1;
        const bool split = f >= 0 && halves(j) > 1;
        const int32_t hflag = split ? new_uflag() : -1, hslot = split ? nslot++ : -1;
        col_task[j] = add({0, (int32_t)j, f, 0, 0, 0, 0, p0, p1, hflag, hslot}, {need, 0, (int)j});
        if (f >= 0) {
            flag_deps[col_task[j]].push_back(p0);
            if (p1 >= 0) flag_deps[col_task[j]].push_back(p1);
        }
        if (split) {
            const int hid = add({4, (int32_t)j, f, 0, 0, 0, 0, p0, p1, hflag, hslot}, {need, 0, (int)j});
            flag_deps[hid] = {p0};
            if (p1 >= 0) flag_deps[hid].push_back(p1);
            uflag_tasks[hflag - np].push_back(hid);
            flag_deps[col_task[j]].push_back(hflag);
        }
        s.flow_flops += (double)NB * NB * NB / 3.0 + (f >= 0 ? (double)NB * NB * NB : 0.0);
    }
    // panel-half solves
    for (int64_t k = 0; k < nb; ++k)
        for (int32_t r : R[k])
            if (in(k))
            for (int h = 0; h < halves(r); ++h) {
                const int32_t p = prog[std::make_tuple((int32_t)k, r, h)];
                // rec[7]: the RHS block row's half 0 accumulates its rows' Gram into partial k
                const int id = add({1, (int32_t)k, 2 * r + h, 0, 0, p, 0, (r == nb && h == 0) ? (int32_t)k : -1},
                                   {kl(k), 1, (int)(k * (nb + 1) + r) * 2 + h});
                T[id].deps.push_back(col_task[k]);
                prog_task[p] = id;
                s.flow_flops += 64.0 * NB * NB;
            }
    // update tasks, target quarter by target quarter, a chain of writers over the source levels
    std::map<std::pair<int32_t, int32_t>, std::vector<int32_t>> tg;  // (a, b) -> sources, ascending
    for (int64_t k = 0; k < nb; ++k)
        for (size_t bi = 0; bi < R[k].size() && in(k); ++bi) {
            const int32_t b = R[k][bi];
            if (b == nb) continue;
            for (size_t ai = bi; ai < R[k].size(); ++ai) {
                const int32_t a = R[k][ai];
                if (a == b && fsrc[b] == (int32_t)k) continue;  // the fused diagonal update
                tg[{a, b}].push_back((int32_t)k);
            }
        }
    std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t> writer;  // final in-place writer flag per quarter
    std::vector<std::vector<std::array<int32_t, 3>>> late(nb);          // (quarter, slot, flag) per diagonal block
    // whole-block update tasks (syrk_block_body, FBA_FLOW_BLOCK): an off-diagonal target with both row
    // halves real in one record instead of four quarter records -- the sources' rows are loaded once for
    // the four quarters (config 4 operand bytes 1047 -> 814 MB) but the record runs ~4x a quarter's
    // latency on one CU (MFMA-bound, ~14 us per 128-deep source).  Measured (iter/s | k_chol_flow us):
    //   config 4:    quarters 1224-1239 | 446-449, all whole 881-889 | 763-776, whole but the urgent last
    //                group 909-913 | 739-744, whole while the sources fit the levels left (mode 3, R = 1)
    //                971 | 670 -- a latency-bound factorisation: the writer chains' latency delays the
    //                panel halves (mean wait 4.7 -> 33 us) and every diagonal block after them
    //   config 5:    quarters 276.1 | 2390-2398, all whole 276.7-277.3 | 2367-2374
    //                mode 3 272.0-272.3 | 2445-2446 (vs 276.0 | 2394-2399 and 276.4-276.7 | 2362-2383, same box)
    //   convergent:  quarters 234-236 | 3076-3134, all whole 252-254 | 2781-2828, mode 3 258-258.5 | 2717-2739
    // so the default (FBA_FLOW_BLOCK unset) makes every group whole (mode 1, the one setting that gains on
    // both) for a throughput-bound factorisation -- update work per elimination-tree level >= 1.5 GFLOP
    // (config 4: 0.39, config 5: 1.92, convergent: 1.6) -- and keeps quarters otherwise.  0: quarters,
    // 1: every group whole, 2: all but the urgent last group, 3: the leading groups whose sources fit the
    // levels left.  Counted over the columns this flow holds and the levels they span: the subtree split's
    // flows each hold a fraction of the work per level (config 5, 4 ranks: flow A 1.05, flow B 0.32
    // GFLOP per level; per iteration flow A + flow B 1.036 + 0.788 ms with quarters vs 1.251 + 0.927 ms
    // with whole blocks, profiles/r05_v3_split_scaling_config5*.log)
    double upd_flops = 0.0;
    std::vector<char> lev_used(nb + 1, 0);
    int nw_in = 0;
    for (int64_t k = 0; k < nb; ++k) {
        if (!in(k)) continue;
        if (!lev_used[level[k]]) { lev_used[level[k]] = 1; ++nw_in; }
        for (size_t bi = 0; bi < R[k].size(); ++bi)
            if (R[k][bi] < nb)
                for (size_t ai = bi; ai < R[k].size(); ++ai) upd_flops += (R[k][ai] == R[k][bi] ? 3 : 4) * 2.0 * 64 * 64 * NB;
    }
    const int blockm = getenv("FBA_FLOW_BLOCK") ? atoi(getenv("FBA_FLOW_BLOCK")) : (nw_in > 0 && upd_flops / nw_in >= 1.5e9 ? 1 : 0);
    if (merge_gap < 0) merge_gap = blockm > 0 ? 1 : 2;
    if (verbose)
        fprintf(stderr, "[fba] flow schedule: update work %.2f GFLOP over %d levels, update records mode %d\n", upd_flops * 1e-9,
                nw_in, blockm);
    for (auto& t : tg) {
        const int32_t a = t.first.first, b = t.first.second;
        std::map<int, std::vector<int32_t>> bylev;
        for (int32_t k : t.second) bylev[level[k]].push_back(k);
        // the writer groups of the target: one per source level, except that consecutive levels are
        // merged into one task (sources ascending, so the in-place sums are bitwise those of separate
        // tasks) while they hold at most msplit sources together, none is the fused source's ("late")
        // level, and the target is read at least merge_gap levels after the group's last source level
        // (a dense network's chain of one-source writers per target otherwise becomes one record per
        // source: 70k update records at convergent config 4)
        const int need_t = a == b ? level[b] - 1 : level[b];
        std::vector<std::pair<int, std::vector<int32_t>>> groups;  // (last source level, sources)
        std::vector<char> glate;
        for (auto& lv : bylev) {
            const bool late_w = a == b && fsrc[b] >= 0 && lv.first == level[fsrc[b]];
            if (merge_gap > 0 && !late_w && !groups.empty() && !glate.back() &&
                groups.back().second.size() + lv.second.size() <= (size_t)msplit && need_t - lv.first >= merge_gap) {
                groups.back().first = lv.first;
                groups.back().second.insert(groups.back().second.end(), lv.second.begin(), lv.second.end());
            } else {
                groups.emplace_back(lv.first, lv.second);
                glate.push_back(late_w);
            }
        }
        const bool whole = blockm > 0 && a != b && halves(a) == 2 && halves(b) == 2;
        size_t gq = 0;        // the first group by quarter tasks
        int32_t wprev = -1;   // the whole-block chain's last writer flag
        if (whole) {
            gq = groups.size();
            if (blockm == 2 && level[b] == groups.back().first + 1) gq = groups.size() - 1;
            // 3: a group is whole while its sources fit the levels left before the target is read (one
            // level per source)
            if (blockm == 3)
                for (gq = 0; gq < groups.size(); ++gq)
                    if (std::min<double>((double)groups[gq].second.size(), SPLIT) > level[b] - groups[gq].first - 1)
                        break;
            int32_t prev = -1;
            if (gq > 0) ++n_whole_t;
            for (size_t gi = 0; gi < gq; ++gi) {
                const int w = groups[gi].first;
                const std::vector<int32_t>& S = groups[gi].second;
                const int ng = (int)((S.size() + SPLIT - 1) / SPLIT);
                const int rank = level[b] == w + 1 ? 3 : 4;
                const int32_t wflag = new_uflag();
                const int32_t cidx = ng > 1 ? ncnt++ : -1;
                const int first = nslot;
                for (int g = 0; g < ng; ++g) {
                    const int32_t soff = (int32_t)buf.size();
                    std::vector<int32_t> fd;
                    const int g0 = g * SPLIT, g1 = std::min((int)S.size(), g0 + SPLIT);
                    for (int x = g0; x < g1; ++x) {
                        const int32_t k = S[x];
                        const int32_t f4[4] = {prog.at(std::make_tuple(k, a, 0)), prog.at(std::make_tuple(k, a, 1)),
                                               prog.at(std::make_tuple(k, b, 0)), prog.at(std::make_tuple(k, b, 1))};
                        buf.insert(buf.end(), {k, f4[0], f4[1], f4[2], f4[3]});
                        fd.insert(fd.end(), f4, f4 + 4);
                        s.flow_flops += 4 * 2.0 * 64 * 64 * NB;
                    }
                    int32_t mode = 0, slot = -1;
                    if (ng > 1) {
                        mode = 1;
                        slot = nslot;
                        nslot += 4;
                    }
                    int lev = w;  // dispatched among the records of its sources' level
                    for (int32_t k : S) lev = std::max(lev, kl(k));
                    const int id = add({2, a, b, 4, soff, g1 - g0, slot, mode, wflag, prev, cidx, first, ng, 0, CB_BLOCKS},
                                       {lev, rank, (int)(b * (nb + 1) + a) * 4});
                    flag_deps[id] = fd;
                    if (prev >= 0) flag_deps[id].push_back(prev);
                    uflag_tasks[wflag - np].push_back(id);
                }
                prev = wflag;
            }
            wprev = prev;
            if (gq == groups.size()) {
                for (int q = 0; q < 4; ++q) writer[std::make_tuple(a, b, q)] = prev;
                continue;
            }
        }
        for (int q = 0; q < 4; ++q) {
            const int qr = q >> 1, qc = q & 1;
            if (a == b && qr == 0 && qc == 1) continue;
            if ((qr == 1 && halves(a) < 2) || (qc == 1 && halves(b) < 2)) continue;
            int32_t prev = wprev;
            for (size_t gi = gq; gi < groups.size(); ++gi) {
                const int w = groups[gi].first;
                const std::vector<int32_t>& S = groups[gi].second;
                const bool is_late = glate[gi] != 0;
                const int ng = (int)((S.size() + SPLIT - 1) / SPLIT);
                // urgency: the target is read at level level[b] (its column's potrf / panel solves)
                const int rank = level[b] == w + 1 ? (a == b ? 2 : 3) : 4;
                const int32_t wflag = is_late ? -1 : new_uflag();
                const int32_t cidx = (!is_late && ng > 1) ? ncnt++ : -1;
                const int first = nslot;
                for (int g = 0; g < ng; ++g) {
                    const int32_t soff = (int32_t)buf.size();
                    std::vector<int32_t> fd;
                    const int g0 = g * SPLIT, g1 = std::min((int)S.size(), g0 + SPLIT);
                    for (int x = g0; x < g1; ++x) {
                        const int32_t k = S[x];
                        const int32_t pa = prog.at(std::make_tuple(k, a, qr)), pb = prog.at(std::make_tuple(k, b, qc));
                        buf.insert(buf.end(), {k, pa, pb});
                        fd.push_back(pa);
                        fd.push_back(pb);
                        s.flow_flops += 2.0 * 64 * 64 * NB;
                    }
                    int32_t mode, flag, slot = -1;
                    if (is_late) {
                        mode = 2;
                        slot = nslot++;
                        flag = new_uflag();
                        late[b].push_back({q, slot, flag});
                    } else if (ng > 1) {
                        mode = 1;
                        slot = nslot++;
                        flag = wflag;
                    } else {
                        mode = 0;
                        flag = wflag;
                    }
                    int lev = w;  // dispatched among the records of its sources' level
                    for (int32_t k : S) lev = std::max(lev, kl(k));
                    const int id = add({2, a, b, q, soff, g1 - g0, slot, mode, flag, is_late ? -1 : prev, cidx, first, ng, 0,
                                        CB_BLOCKS},
                                       {lev, is_late ? 2 : rank, (int)(b * (nb + 1) + a) * 4 + q});
                    flag_deps[id] = fd;
                    if (!is_late && prev >= 0) flag_deps[id].push_back(prev);
                    uflag_tasks[flag - np].push_back(id);
                }
                if (!is_late) prev = wflag;
            }
            writer[std::make_tuple(a, b, q)] = prev;
        }
    }
    // panel halves wait for the final writers of their quarters; diagonal blocks for those of their
    // diagonal quarters and for their late partials
    for (int id = 0; id < (int)T.size(); ++id) {
        Task& X = T[id];
        if (X.rec[0] == 1) {
            const int32_t k = X.rec[1], r = X.rec[2] >> 1, h = X.rec[2] & 1;
            const int32_t woff = (int32_t)buf.size();
            for (int qc = 0; qc < halves(k); ++qc) {
                auto it = writer.find(std::make_tuple(r, k, 2 * h + qc));
                if (it != writer.end() && it->second >= 0) buf.push_back(it->second);
            }
            X.rec[3] = woff;
            X.rec[4] = (int32_t)buf.size() - woff;
            for (int32_t x = woff; x < (int32_t)buf.size(); ++x) flag_deps[id].push_back(buf[x]);
        } else if (X.rec[0] == 0) {
            const int32_t j = X.rec[1];
            const int32_t woff = (int32_t)buf.size();
            for (int q : {0, 2, 3}) {
                if (q > 0 && halves(j) < 2) continue;
                auto it = writer.find(std::make_tuple(j, j, q));
                if (it != writer.end() && it->second >= 0) buf.push_back(it->second);
            }
            X.rec[3] = woff;
            X.rec[4] = (int32_t)buf.size() - woff;
            for (int32_t x = woff; x < (int32_t)buf.size(); ++x) flag_deps[id].push_back(buf[x]);
            const int32_t loff = (int32_t)buf.size();
            for (auto& l : late[j]) {
                buf.insert(buf.end(), l.begin(), l.end());
                flag_deps[id].push_back(l[2]);
            }
            X.rec[5] = loff;
            X.rec[6] = (int32_t)late[j].size();
        }
    }
    // inverses of the diagonal blocks below the top level
    for (int64_t j = 0; j < nb; ++j)
        if (level[j] < nw - 1 && in(j)) {
            const int id = add({3, (int32_t)j}, {kl(j) + 1, 5, (int)j});
            T[id].deps.push_back(col_task[j]);
            s.flow_flops += (double)NB * NB * NB / 3.0;
        }
    // flags -> producer records
    for (size_t i = 0; i < T.size(); ++i)
        for (int32_t fg : flag_deps[i]) {
            if (fg < np) T[i].deps.push_back(prog_task[fg]);
            else for (int p : uflag_tasks[fg - np]) T[i].deps.push_back(p);
        }
    // dispatch order: Kahn's algorithm, the smallest key among the ready records first
    const int n = (int)T.size();
    std::vector<int> indeg(n, 0), ord;
    std::vector<std::vector<int>> succ(n);
    bool ok = true;
    for (int i = 0; i < n; ++i) {
        std::sort(T[i].deps.begin(), T[i].deps.end());
        T[i].deps.erase(std::unique(T[i].deps.begin(), T[i].deps.end()), T[i].deps.end());
        for (int d : T[i].deps) {
            if (d < 0 || d >= n || d == i) { ok = false; continue; }
            succ[d].push_back(i);
            indeg[i]++;
        }
    }
    {
        auto cmp = [&](int x, int y) { return T[x].key != T[y].key ? T[x].key > T[y].key : x > y; };
        std::priority_queue<int, std::vector<int>, decltype(cmp)> ready(cmp);
        for (int i = 0; i < n; ++i)
            if (indeg[i] == 0) ready.push(i);
        std::vector<char> placed(n, 0);
        while (!ready.empty()) {
            const int i = ready.top();
            ready.pop();
            if (placed[i]) continue;
            placed[i] = 1;
            ord.push_back(i);
            for (int x : succ[i])
                if (--indeg[x] == 0 && !placed[x]) ready.push(x);
        }
    }
    if ((int)ord.size() != n) ok = false;  // a dependency cycle
    std::vector<int> pos(n, -1);
    for (size_t i = 0; i < ord.size(); ++i) pos[ord[i]] = (int)i;
    for (int i = 0; i < n && ok; ++i)
        for (int d : T[i].deps)
            if (pos[d] < 0 || pos[d] >= pos[i]) ok = false;
    s.flow_ok = ok;
    s.flow_nprog = np;
    s.flow_nuflag = (int)uflag_tasks.size();
    s.flow_ncounter = ncnt;
    s.flow_nscratch = nslot;
    s.flow_rec = (int64_t)buf.size();
    s.flow_n = ok ? n : 0;
    for (int r = 0; r < 5; ++r) s.flow_cnt[r] = 0;
    if (ok)
        for (int i : ord) {
            buf.insert(buf.end(), T[i].rec.begin(), T[i].rec.end());
            s.flow_cnt[T[i].rec[0]]++;
        }
    // operand bytes the records move (each record's global loads and stores as the kernels issue them:
    // a diagonal block its 128x128 block, the fused source's 128 panel rows, late / helper partials, the
    // published factor and leaf inverses; a panel half its 64 rows in and out, the column's factor and
    // leaf inverses; an update 2 x 64 x 128 per source plus its target quarter or scratch partial in and
    // out; an inverse the factor in, the inverse out) -- the HBM-side traffic of the decomposition, to set
    // against the PMC bytes of a launch
    s.flow_bytes = 0.0;
    double rb[5] = {0, 0, 0, 0, 0};
    if (ok)
        for (int i : ord) {
            const auto& r = T[i].rec;
            const double blk = 8.0 * NB * NB, q = 8.0 * 64 * 64, dv = 8.0 * 8 * 16 * 16;
            double b = 0.0;
            switch (r[0]) {
                case 0: b = blk + (r[2] >= 0 ? blk : 0.0) + r[6] * q + (r[9] >= 0 ? 21 * 8.0 * 256 : 0.0) + blk + dv; break;
                case 1: b = 2 * 8.0 * 64 * NB + blk + dv; break;
                case 2: b = r[3] == 4 ? r[5] * 2 * blk + 8 * q : r[5] * 2 * 8.0 * 64 * NB + 2 * q; break;
                case 3: b = 2 * blk; break;
                case 4: b = blk + 21 * 8.0 * 256; break;
                default: break;
            }
            rb[r[0]] += b;
            s.flow_bytes += b;
        }
    if (verbose)
        fprintf(stderr, "[fba] flow schedule: operand bytes %.1f MB (diagonal %.1f, panel halves %.1f, updates %.1f, inverses %.1f, "
                "split helpers %.1f), %.2f GFLOP\n", s.flow_bytes * 1e-6, rb[0] * 1e-6, rb[1] * 1e-6, rb[2] * 1e-6,
                rb[3] * 1e-6, rb[4] * 1e-6, s.flow_flops * 1e-9);
    if (verbose)
        fprintf(stderr, "[fba] flow schedule: %d records (%d diagonal, %d panel halves, %d updates, %d inverses, "
                "%d split helpers), %d progress + %d update flags, %d scratch quarters, %d of %d targets by whole-block "
                "tasks, %d levels%s\n", n, s.flow_cnt[0], s.flow_cnt[1], s.flow_cnt[2], s.flow_cnt[3], s.flow_cnt[4], np,
                s.flow_nuflag, nslot, n_whole_t, (int)tg.size(), nw, ok ? "" : " -- ORDER CHECK FAILED, not used");
}

void build_schedule(Ctx& c, const std::vector<std::pair<int32_t, int32_t>>& pairs) {
    const Layout& L = c.L;
    const int64_t nb = L.n_pad / NB;
    Sched& s = c.sched;
    // lower block pattern, P[j][i] = block (i, j) nonzero, i >= j; row nb = the RHS block row
    std::vector<std::vector<uint8_t>> P(nb, std::vector<uint8_t>(nb + 1, 0));
    auto touch = [&](int64_t e1, int64_t e2) {  // rows of image e1 x columns of image e2 (6 each)
        for (int64_t bi = 6 * e1 / NB; bi <= (6 * e1 + 5) / NB; ++bi)
            for (int64_t bj = 6 * e2 / NB; bj <= (6 * e2 + 5) / NB; ++bj)
                if (bi >= bj) P[bj][bi] = 1;
    };
    for (int64_t e = 0; e < L.n_img; ++e)  // (a padding slot is decoupled: it must not join two blocks)
        if (c.img_ord[e] >= 0) touch(e, e);
    for (auto& q : pairs) touch(q.first, q.second);
    if (c.n_loc > 0) {  // the local inner-constraint border: dense on its block rows
        const int64_t bl = (6 * (int64_t)c.n_loc - 1) / NB;
        for (int64_t i = 0; i <= bl; ++i)
            for (int64_t j = 0; j <= i; ++j) P[j][i] = 1;
    }
    const int64_t T = std::min<int64_t>(6 * (int64_t)L.n_img / NB, nb);  // camera rows: dense
    for (int64_t j = 0; j < nb; ++j) {
        for (int64_t i = std::max(T, j); i < nb; ++i) P[j][i] = 1;
        P[j][nb] = 1;
    }
    // symbolic factorisation (fill) and elimination-tree levels
    std::vector<std::vector<int32_t>> R(nb);
    std::vector<int32_t> level(nb, 0);
    for (int64_t k = 0; k < nb; ++k) {
        for (int64_t i = k + 1; i <= nb; ++i)
            if (P[k][i]) R[k].push_back((int32_t)i);
        for (size_t a = 0; a < R[k].size(); ++a) {
            const int32_t ia = R[k][a];
            if (ia == nb) continue;
            level[ia] = std::max(level[ia], level[k] + 1);
            for (size_t b = a; b < R[k].size(); ++b) P[ia][R[k][b]] = 1;
        }
    }
    const int nw = nb > 0 ? 1 + *std::max_element(level.begin(), level.end()) : 0;
    s = Sched();
    s.n_waves = nw;
    std::vector<std::vector<int32_t>> wave(nw);
    for (int64_t k = 0; k < nb; ++k) wave[level[k]].push_back((int32_t)k);
    // rows of block row i that carry unknowns (the rest is padding: zero rows that stay zero, so the
    // second 64-row half of a block row with <= 64 of them is skipped by the panel solves and updates)
    auto real_rows = [&](int64_t i) -> int64_t {
        if (i == nb) return L.nrhs;
        return std::max<int64_t>(0, std::min<int64_t>(NB, L.u_c - i * NB));
    };
    std::vector<int32_t> buf;  // device image
    auto at = [&]() { return (int64_t)buf.size(); };
    s.w.resize(nw);
    std::vector<std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t>> tflag(nw);  // (i, j, quarter) -> flag
    int64_t ntile_total = 0;
    for (int w = 0; w < nw; ++w) {
        Sched::Wave& W = s.w[w];
        W.cols = at();
        W.ncol = (int)wave[w].size();
        buf.insert(buf.end(), wave[w].begin(), wave[w].end());
        W.trsm = at();
        for (int32_t k : wave[w])
            for (int32_t r : R[k])
                for (int h = 0; h < 2; ++h)
                    if (h == 0 || real_rows(r) > NB / 2) { buf.push_back(k); buf.push_back(2 * r + h); }
        W.ntrsm = (int)((at() - W.trsm) / 2);
        // potrf of each 128 block (NB^3/3) + the triangular solve of each 64-row half panel (64 NB^2)
        W.pflops = (double)W.ncol * NB * NB * NB / 3.0 + (double)W.ntrsm * 64.0 * NB * NB;
        // trailing-update targets (i, j), j < nb, with their source columns in ascending order
        std::map<std::pair<int32_t, int32_t>, std::vector<int32_t>> tg;
        for (int32_t k : wave[w])
            for (size_t b = 0; b < R[k].size(); ++b) {
                if (R[k][b] == nb) continue;
                for (size_t a = b; a < R[k].size(); ++a) tg[{R[k][a], R[k][b]}].push_back(k);
            }
        // quarter tasks; a target with more than SPLIT sources is split into groups of <= SPLIT
        // consecutive sources summed into scratch quarters and combined in group order afterwards,
        // so no workgroup runs more than SPLIT * 128 deep (the long poles of a level)
        constexpr int SPLIT = 2;
        struct Task { int32_t i, j, q, s0, s1, slot, comb, fidx, rank; };
        std::vector<Task> tasks;
        std::vector<int32_t> src, comb;
        int slots = 0, ncomb = 0;
        W.flops = 0.0;
        // completion flag of every target quarter (the in-launch hand-off to the next level's k_panel);
        // rank: 0 a diagonal block of a next-level column, 1 a panel block of one, 2 the rest
        std::map<std::tuple<int32_t, int32_t, int32_t>, int32_t>& fmap = tflag[w];
        auto rank_of = [&](int32_t i, int32_t j) {
            if (w + 1 >= nw || level[j] != w + 1) return 2;
            return i == j ? 0 : 1;
        };
        for (auto& t : tg) {
            const int32_t i = t.first.first, j = t.first.second;
            const int32_t s0 = (int32_t)src.size();
            src.insert(src.end(), t.second.begin(), t.second.end());
            const int32_t ns = (int32_t)t.second.size();
            const bool split = ns > SPLIT;
            for (int q = 0; q < 4; ++q) {
                const int qr = q >> 1, qc = q & 1;
                if (i == j && qr == 0 && qc == 1) continue;  // strictly upper quarter of a diagonal block
                if ((qr == 1 && real_rows(i) <= NB / 2) || (qc == 1 && real_rows(j) <= NB / 2)) continue;
                const int32_t fidx = s.n_tflags++;
                fmap[std::make_tuple(i, j, q)] = fidx;
                const int32_t rk = rank_of(i, j);
                if (!split) {
                    tasks.push_back({i, j, q, s0, s0 + ns, -1, -1, fidx, rk});
                } else {
                    const int first = slots;
                    for (int32_t g = 0; g < ns; g += SPLIT)
                        tasks.push_back({i, j, q, s0 + g, s0 + std::min(ns, g + SPLIT), slots++, ncomb, fidx, rk});
                    comb.insert(comb.end(), {i, j, q, first, slots - first});
                    ++ncomb;
                }
                W.flops += (double)ns * 2.0 * 64 * 64 * NB;
            }
        }
        // the next level's diagonal blocks first, then its panel blocks (their consumers wait in the merged
        // launch), then the rest; within a rank longest (most sources) first, then by block column
        std::stable_sort(tasks.begin(), tasks.end(), [](const Task& a, const Task& b) {
            if (a.rank != b.rank) return a.rank < b.rank;
            if (a.s1 - a.s0 != b.s1 - b.s0) return a.s1 - a.s0 > b.s1 - b.s0;
            return a.j != b.j ? a.j < b.j : a.i < b.i;
        });
        W.ndiag = W.npanel = 0;
        for (auto& t : tasks) {
            W.ndiag += t.rank == 0 ? 1 : 0;
            W.npanel += t.rank == 1 ? 1 : 0;
        }
        W.src = at();
        buf.insert(buf.end(), src.begin(), src.end());
        W.tasks = at();
        W.ntask = (int)tasks.size();
        for (auto& t : tasks) buf.insert(buf.end(), {t.i, t.j, t.q, t.s0, t.s1, t.slot, t.comb, t.fidx});
        W.comb = at();
        W.ncomb = ncomb;
        W.cbase = s.n_counters;
        s.n_counters += ncomb;
        buf.insert(buf.end(), comb.begin(), comb.end());
        s.n_scratch = std::max(s.n_scratch, slots);
        ntile_total += (int64_t)tg.size();
    }
    // wait lists of the merged launches: level v's potrf workgroups wait for the flags of level v-1's
    // updates of their diagonal block, its panel-solve halves (k, 2 r + h) for those of quarters
    // (r, k, 2 h + 0/1)
    for (int v = 1; v < nw; ++v) {
        Sched::Wave& W = s.w[v];
        const auto& fm = tflag[v - 1];
        std::vector<int32_t> start, list;
        auto add = [&](int32_t i, int32_t j, int32_t q) {
            auto it = fm.find(std::make_tuple(i, j, q));
            if (it != fm.end()) list.push_back(it->second);
        };
        for (int32_t k : wave[v]) {
            start.push_back((int32_t)list.size());
            for (int q : {0, 2, 3}) add(k, k, q);
        }
        const int32_t* tr = buf.data() + W.trsm;
        std::vector<std::pair<int32_t, int32_t>> recs;
        for (int t = 0; t < W.ntrsm; ++t) recs.push_back({tr[2 * t], tr[2 * t + 1]});
        for (auto& rc : recs) {
            start.push_back((int32_t)list.size());
            const int32_t k = rc.first, r = rc.second >> 1, h = rc.second & 1;
            add(r, k, 2 * h);  // (r = nb: the RHS block row, updated like any other)
            add(r, k, 2 * h + 1);
        }
        start.push_back((int32_t)list.size());
        W.wstart = at();
        buf.insert(buf.end(), start.begin(), start.end());
        W.wlist = at();
        buf.insert(buf.end(), list.begin(), list.end());
    }
    // backward solve L' x = y by levels, top down: the columns of level w get x = Linv' y; every
    // column j whose panel holds one of them gets y_j -= sum_i L(i,j)' x_i (i ascending)
    std::vector<std::vector<int32_t>> rev(nb);  // rev[i] = columns j < i with i in R[j]
    for (int64_t j = 0; j < nb; ++j)
        for (int32_t i : R[j])
            if (i < nb) rev[i].push_back((int32_t)j);
    s.b.resize(nw);
    for (int w = nw - 1; w >= 0; --w) {
        Sched::BWave& B = s.b[w];
        B.srcs = s.w[w].cols;
        B.nsrc = s.w[w].ncol;
        std::map<int32_t, std::vector<int32_t>> tg;
        for (int32_t i : wave[w])
            for (int32_t j : rev[i]) tg[j].push_back(i);
        B.ntgt = (int)tg.size();
        B.tgts = at();
        for (auto& t : tg) buf.push_back(t.first);
        B.src_start = at();
        int32_t acc = 0;
        for (auto& t : tg) { buf.push_back(acc); acc += (int32_t)t.second.size(); }
        buf.push_back(acc);
        B.src = at();
        for (auto& t : tg) buf.insert(buf.end(), t.second.begin(), t.second.end());
    }
    // backward dataflow lists: the sources of every block column, descending
    s.bf_start = at();
    {
        int32_t acc = 0;
        for (int64_t j = 0; j < nb; ++j) {
            buf.push_back(acc);
            for (int32_t i : R[j]) acc += i < nb ? 1 : 0;
        }
        buf.push_back(acc);
    }
    s.bf_src = at();
    for (int64_t j = 0; j < nb; ++j)
        for (auto it = R[j].rbegin(); it != R[j].rend(); ++it)
            if (*it < nb) buf.push_back(*it);
    // the blocks the factorisation touches (everything else in S stays zero from fba_create on)
    s.zero = at();
    for (int64_t k = 0; k < nb; ++k) {
        buf.push_back((int32_t)k);
        buf.push_back((int32_t)k);
        for (int32_t r : R[k]) { buf.push_back(r); buf.push_back((int32_t)k); }
    }
    s.nzero = (int)((at() - s.zero) / 2);
    s.n_tiles = ntile_total;
    // subtree split (Sched::split): cut the elimination tree.  parent(k) = the first block row below
    // column k; a subtree's columns touch only their own rows and their ancestors', so two subtrees never
    // share a block.  Starting from the roots, the subtree of the largest work (1 + r + r^2 block
    // products for a column of r panel blocks) moves its root column to the top until there are at least
    // w subtrees and none holds more than 1.25x the average (the balance cut for w).  The balance cuts for
    // w = 2 .. world are priced on the world ranks by a cost model of one iteration (split_cost below):
    // the ranks' linearisation and subtree flows side by side, then the top blocks' exchange, then the top
    // flow on every rank; per elimination-tree level max(LAT, work x TAU) -- a latency-bound chain where
    // the level is narrow, throughput where it is wide.  The cheapest is kept, so more ranks never take a
    // deeper cut than pays (a rank may then get no subtree: it only linearises its share of the top's
    // points).  Subtrees are dealt to the
    // ranks largest first, each to the least loaded (LPT).  The local inner-constraint border's block rows
    // must stay in a subtree (their weights come from one rank's diagonal); otherwise no split.
    s.split = false;
    std::vector<char> inc_own, inc_top;
    if (c.opt.split && c.opt.world > 1 && nb > 1) {
        const int W = c.opt.world;
        std::vector<int32_t> parent(nb, -1);
        std::vector<std::vector<int32_t>> kids(nb);
        for (int64_t k = 0; k < nb; ++k)
            for (int32_t r : R[k])
                if (r < nb) { parent[k] = r; kids[r].push_back((int32_t)k); break; }
        std::vector<double> sw(nb, 0.0), wk(nb, 0.0);  // children have smaller indices than their parents
        for (int64_t k = 0; k < nb; ++k) {
            const double r = (double)R[k].size();
            wk[k] = 1.0 + r + r * r;
            sw[k] += wk[k];
            if (parent[k] >= 0) sw[parent[k]] += sw[k];
        }
        // cost model constants (config 4 / 5 records): LAT = the critical chain of one
        // elimination-tree level (potrf + hand-offs), TAU = one 128^3 block product at the throughput the
        // wide levels reach (config 5: 22.5 TFLOP/s), BW = the all-reduce's algorithm bandwidth over xGMI,
        // LIN = linearising and reducing one block column's points (k_lin_reduce + k_red_blocks, config 4:
        // 47 columns in 235 us)
        constexpr double LAT = 30.0, TAU = 0.19, BW = 100e3, LIN = 5.0;  // us, us, bytes per us, us
        const int nlev = nb > 0 ? 1 + *std::max_element(level.begin(), level.end()) : 0;
        std::vector<int32_t> owner(nb);
        auto deal = [&](const std::vector<int32_t>& front, std::vector<double>& load, std::vector<int32_t>& root_rank) {
            std::vector<int32_t> f(front);
            std::stable_sort(f.begin(), f.end(), [&](int32_t a, int32_t b) { return sw[a] > sw[b]; });
            load.assign(W, 0.0);
            root_rank.assign(nb, -1);
            for (int32_t k : f) {
                const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                root_rank[k] = r;
                load[r] += sw[k];
            }
        };
        auto split_cost = [&](const std::vector<char>& top, const std::vector<int32_t>& front) {
            std::vector<double> load;
            std::vector<int32_t> rr;
            deal(front, load, rr);
            for (int64_t k = nb - 1; k >= 0; --k)
                owner[k] = top[k] ? -1 : (rr[k] >= 0 ? rr[k] : (parent[k] >= 0 ? owner[parent[k]] : -1));
            std::vector<double> lw((size_t)(W + 1) * nlev, 0.0);  // per rank (W: the top) and level: work
            std::vector<double> cols(W + 1, 0.0);
            double top_blocks = 0.0;
            for (int64_t k = 0; k < nb; ++k) {
                lw[(size_t)(owner[k] < 0 ? W : owner[k]) * nlev + level[k]] += wk[k];
                cols[owner[k] < 0 ? W : owner[k]] += 1.0;
                if (owner[k] < 0) top_blocks += 1.0 + (double)R[k].size();
            }
            auto flow = [&](int who) {
                double t = 0.0;
                for (int l = 0; l < nlev; ++l)
                    if (lw[(size_t)who * nlev + l] > 0.0) t += std::max(LAT, lw[(size_t)who * nlev + l] * TAU);
                return t;
            };
            double a = 0.0;
            for (int r = 0; r < W; ++r) a = std::max(a, LIN * (cols[r] + cols[W] / W) + flow(r));
            return a + 2.0 * (W - 1) / W * top_blocks * NB * NB * 8.0 / BW + flow(W);
        };
        std::vector<int32_t> roots;
        for (int64_t k = 0; k < nb; ++k)
            if (parent[k] < 0) roots.push_back((int32_t)k);
        // the balance cut for w subtrees: the largest subtree's root to the top until there are at least
        // w subtrees and none holds more than 1.25x the average
        auto balance_cut = [&](int w, std::vector<char>& tp, std::vector<int32_t>& fr) {
            fr = roots;
            tp.assign(nb, 0);
            for (;;) {
                double tot = 0.0, mx = -1.0;
                int imx = -1;
                for (size_t q = 0; q < fr.size(); ++q) {
                    tot += sw[fr[q]];
                    if (sw[fr[q]] > mx) { mx = sw[fr[q]]; imx = (int)q; }
                }
                if (imx < 0 || ((int)fr.size() >= w && mx <= 1.25 * tot / w)) break;
                const int32_t k = fr[imx];
                if (kids[k].empty()) break;  // one column: no further cut
                tp[k] = 1;
                fr.erase(fr.begin() + imx);
                fr.insert(fr.end(), kids[k].begin(), kids[k].end());
            }
        };
        // candidates: the balance cuts for w = 2 .. W subtrees, each priced on the W ranks; the cheapest
        // is kept (ties: the larger w)
        std::vector<int32_t> frontier;
        std::vector<char> top(nb, 0);
        double best = 1e300;
        int best_w = -1;
        for (int w = 2; w <= W; ++w) {
            std::vector<char> tp;
            std::vector<int32_t> fr;
            balance_cut(w, tp, fr);
            if (fr.size() < 2) continue;
            const double cst = split_cost(tp, fr);
            if (c.opt.verbose) {
                int nt = 0;
                for (char t : tp) nt += t;
                fprintf(stderr, "[fba] subtree split candidate w=%d: %d top columns, %zu subtrees, modelled %.0f us\n", w, nt,
                        fr.size(), cst);
            }
            if (cst <= best) { best = cst; best_w = w; frontier = fr; top = tp; }
        }
        const int best_step = best_w;
        if (best_step < 0) frontier.clear();
        std::vector<double> load;
        std::vector<int32_t> root_rank;
        deal(frontier, load, root_rank);
        std::vector<int32_t> br(nb, -1);
        for (int64_t k = nb - 1; k >= 0; --k)  // parents first
            br[k] = top[k] ? -1 : (root_rank[k] >= 0 ? root_rank[k] : (parent[k] >= 0 ? br[parent[k]] : -1));
        bool ok = !frontier.empty();
        if (c.n_loc > 0)
            for (int64_t i = 0; i <= (6 * (int64_t)c.n_loc - 1) / NB; ++i) ok = ok && br[i] >= 0;
        if (ok) {
            s.split = true;
            s.blk_rank = br;
            inc_own.assign(nb, 0);
            inc_top.assign(nb, 0);
            for (int64_t k = 0; k < nb; ++k) {
                inc_own[k] = br[k] == c.opt.rank;
                inc_top[k] = br[k] < 0;
            }
            // the top blocks the ranks sum: (b, b) and (a, b), a in R[b] (top rows and the RHS block row)
            s.top_blocks = at();
            for (int64_t b = 0; b < nb; ++b)
                if (br[b] < 0) {
                    buf.push_back((int32_t)b);
                    buf.push_back((int32_t)b);
                    for (int32_t a : R[b]) { buf.push_back(a); buf.push_back((int32_t)b); }
                }
            s.n_top_blocks = (int)((at() - s.top_blocks) / 2);
            if (c.opt.verbose) {
                int ntop = 0;
                for (int64_t k = 0; k < nb; ++k) ntop += br[k] < 0;
                fprintf(stderr, "[fba] subtree split: %d top columns (%d top blocks), %zu subtrees, modelled %.0f us per "
                        "factorisation; work per rank:", ntop, s.n_top_blocks, frontier.size(), best);
                for (double v : load) fprintf(stderr, " %.0f", v);
                fprintf(stderr, "; top columns:");
                for (int64_t k = 0; k < nb; ++k)
                    if (br[k] < 0) fprintf(stderr, " %ld", (long)k);
                fprintf(stderr, "\n");
            }
        } else if (c.opt.verbose) {
            fprintf(stderr, "[fba] subtree split not possible for this block pattern: replicated solve\n");
        }
    }
    if (s.split) {  // flow B (the top columns) first, saved; flow A (this rank's subtrees) in the main fields
        build_flow(s, buf, R, level, nb, real_rows, c.opt.verbose, &inc_top);
        Sched::FlowPart& T = s.top;
        T.rec = s.flow_rec;
        T.n = s.flow_n;
        T.nprog = s.flow_nprog;
        T.nuflag = s.flow_nuflag;
        T.ncounter = s.flow_ncounter;
        T.nscratch = s.flow_nscratch;
        for (int r = 0; r < 5; ++r) T.cnt[r] = s.flow_cnt[r];
        T.ok = s.flow_ok;
        T.flops = s.flow_flops;
        s.flow_flops = 0.0;
        build_flow(s, buf, R, level, nb, real_rows, c.opt.verbose, &inc_own);
        s.n_tflags = std::max(s.n_tflags, s.flow_nprog + s.flow_nuflag + T.nprog + T.nuflag);
        s.n_counters = std::max(s.n_counters, s.flow_ncounter + T.ncounter);
        s.n_scratch = std::max(s.n_scratch, s.flow_nscratch + T.nscratch);
    } else {
        build_flow(s, buf, R, level, nb, real_rows, c.opt.verbose);
        s.n_tflags = std::max(s.n_tflags, s.flow_nprog + s.flow_nuflag);
        s.n_counters = std::max(s.n_counters, s.flow_ncounter);
        s.n_scratch = std::max(s.n_scratch, s.flow_nscratch);
    }
    s.buf = std::move(buf);
    if (c.opt.verbose)
        fprintf(stderr, "[fba] camera system: %ld blocks, %d levels, %ld update tiles, %d images + %d padding slots\n",
                (long)nb, nw, (long)ntile_total, c.L.n_img_ref, c.L.n_img - c.L.n_img_ref);
}

}  // namespace fba
