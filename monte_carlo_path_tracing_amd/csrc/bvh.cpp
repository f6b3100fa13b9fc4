// Binned-SAH BVH for the GPU traversal kernels.
//
// Replaces the reference's uniform grid + 3D-DDA (Myobj.cpp:78-162 meshing, :334-474
// closet_ray_intersect, :476-622 closet_ray_intersect_light_triangle) as the acceleration
// structure; the closest-hit SEMANTICS are unchanged because the per-triangle test is the
// reference's fp64 Cramer rule (Myobj.cpp:165-192) applied to every candidate, and the BVH only
// prunes with conservatively enlarged fp32 boxes.
//
// Layout: each 64-byte node holds BOTH children's boxes, so one node fetch decides both
// children (one 64 B line per visited node; the Veach tree is ~6k nodes, L2-resident).
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <memory>
#include <system_error>
#include <thread>

#include "mcpt_internal.h"

namespace mcpt {

namespace {

struct Box {
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX};
    double hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    void grow(const double* p) {
        for (int c = 0; c < 3; c++) {
            lo[c] = std::min(lo[c], p[c]);
            hi[c] = std::max(hi[c], p[c]);
        }
    }
    void grow(const Box& b) {
        for (int c = 0; c < 3; c++) {
            lo[c] = std::min(lo[c], b.lo[c]);
            hi[c] = std::max(hi[c], b.hi[c]);
        }
    }
    double area() const {
        if (lo[0] > hi[0]) return 0;
        double d[3] = {hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]};
        return 2 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

struct Prim {
    Box box;
    double c[3];
    int32_t facet;
};

#ifndef MCPT_BVH_BINS
#define MCPT_BVH_BINS 32
#endif
#ifndef MCPT_BVH_ALL_AXES
#define MCPT_BVH_ALL_AXES 1  // binned SAH over all three centroid axes (0: the widest only, rounds 1-4)
#endif
#ifndef MCPT_BVH_SWEEP
#define MCPT_BVH_SWEEP 65536  // nodes of at most this many triangles: exact SAH sweep over all three axes
#endif
#ifndef MCPT_BVH_CTRAV
#define MCPT_BVH_CTRAV 0.0  // SAH: cost of an inner node in triangle tests (0: split whenever the children test fewer)
#endif
#ifndef MCPT_BVH_SPATIAL
#define MCPT_BVH_SPATIAL 1  // spatial splits (SBVH) where the object split's children overlap ...
#endif
#ifndef MCPT_BVH_SPATIAL_MIN
#define MCPT_BVH_SPATIAL_MIN 65536  // ... in trees of at least this many triangles (Cornell-1M +4%, Veach -7%)
#endif
#ifndef MCPT_BVH_SPATIAL_ALPHA
#define MCPT_BVH_SPATIAL_ALPHA 1e-5  // overlap (of the root's area) above which spatial splits are tried
#endif
#ifndef MCPT_BVH_SPATIAL_BUDGET
#define MCPT_BVH_SPATIAL_BUDGET 0.3  // at most this many duplicated references per triangle
#endif
constexpr int kBins = MCPT_BVH_BINS;
constexpr int kMaxDepth = 40;  // device traversal stack is 48 entries

// runs a() on a new thread and b() on this one, or both here if no thread can be started (a library call
// must not terminate its host process over a thread limit)
template <class A, class B>
void run_pair(A&& a, B&& b) {
    std::thread t;
    try {
        t = std::thread(a);  // a copy: `a` stays callable if the thread cannot start
    } catch (const std::system_error&) {
        a();
        b();
        return;
    }
    b();
    t.join();
}

struct Builder {
    std::vector<Prim> prims;
    Bvh* out;
    int max_leaf;
    double margin;

    void to_float_box(const Box& b, float* lo, float* hi) const {
        for (int c = 0; c < 3; c++) {
            lo[c] = std::nextafter(static_cast<float>(b.lo[c] - margin), -FLT_MAX);
            hi[c] = std::nextafter(static_cast<float>(b.hi[c] + margin), FLT_MAX);
        }
    }

    Box bounds(int b, int e) const {
        Box r;
        for (int i = b; i < e; i++) r.grow(prims[i].box);
        return r;
    }

    // emits a leaf: returns ~first_slot, count via out param
    int32_t make_leaf(int b, int e, int32_t& count) {
        int32_t first = static_cast<int32_t>(out->leaf_facets.size());
        for (int i = b; i < e; i++) out->leaf_facets.push_back(prims[i].facet);
        count = e - b;
        return ~first;
    }

    // partition [b, e) by binned SAH; returns split index or -1 (make a leaf)
    int split(std::vector<Prim>& prims, int b, int e, const Box& box) {
        const int n = e - b;
        if (n <= max_leaf) return -1;
        Box cb;
        for (int i = b; i < e; i++) cb.grow(prims[i].c);
        int widest = 0;
        for (int c = 1; c < 3; c++)
            if (cb.hi[c] - cb.lo[c] > cb.hi[widest] - cb.lo[widest]) widest = c;
        // the best binned split along one axis: (cost, first bin of the right side), bin index of a prim
        auto bin_of = [&](const Prim& p, int axis) {
            const double ext = cb.hi[axis] - cb.lo[axis];
            const int i = static_cast<int>((p.c[axis] - cb.lo[axis]) * (kBins * (1 - 1e-9) / ext));
            return std::min(kBins - 1, std::max(0, i));
        };
        auto sweep = [&](int axis, double* cost_out) {
            Box bb[kBins];
            int cnt[kBins] = {0};
            for (int i = b; i < e; i++) {
                const int q = bin_of(prims[i], axis);
                cnt[q]++;
                bb[q].grow(prims[i].box);
            }
            double best = DBL_MAX;
            int best_s = -1;
            double right_area[kBins];
            int right_cnt[kBins];
            Box acc;
            int ac = 0;
            for (int s = kBins - 1; s > 0; s--) {
                acc.grow(bb[s]);
                ac += cnt[s];
                right_area[s] = acc.area();
                right_cnt[s] = ac;
            }
            acc = Box();
            ac = 0;
            for (int s = 1; s < kBins; s++) {
                acc.grow(bb[s - 1]);
                ac += cnt[s - 1];
                if (ac == 0 || right_cnt[s] == 0) continue;
                const double cost = acc.area() * ac + right_area[s] * right_cnt[s];
                if (cost < best) {
                    best = cost;
                    best_s = s;
                }
            }
            *cost_out = best;
            return best_s;
        };
        if (n <= MCPT_BVH_SWEEP) {  // exact SAH: every split position of the centroid order on every axis
            struct AxisBest {
                double cost = DBL_MAX;
                int k = -1;
                std::vector<std::pair<double, int>> key;
            } ab[3];
            auto sweep_axis = [&](int c) {
                AxisBest& r = ab[c];
                r.key.resize(n);
                for (int i = 0; i < n; i++) r.key[i] = {prims[b + i].c[c], i};
                std::sort(r.key.begin(), r.key.end());  // ties by index: a stable order
                std::vector<double> right(n);
                Box acc;
                for (int i = n - 1; i > 0; i--) acc.grow(prims[b + r.key[i].second].box), right[i] = acc.area() * (n - i);
                acc = Box();
                for (int i = 1; i < n; i++) {
                    acc.grow(prims[b + r.key[i - 1].second].box);
                    const double cost = acc.area() * i + right[i];
                    if (cost < r.cost) r.cost = cost, r.k = i;
                }
            };
            if (n >= 8192) {  // large nodes: the three axes on three threads
                run_pair([&] { sweep_axis(1); }, [&] { run_pair([&] { sweep_axis(2); }, [&] { sweep_axis(0); }); });
            } else {
                for (int c = 0; c < 3; c++) sweep_axis(c);
            }
            int bax = -1;
            for (int c = 0; c < 3; c++)
                if (ab[c].k > 0 && (bax < 0 || ab[c].cost < ab[bax].cost)) bax = c;
            if (bax < 0 || !(ab[bax].cost + MCPT_BVH_CTRAV * box.area() < box.area() * n || n > 4 * max_leaf)) return -1;
            std::vector<Prim> tmp(n);
            for (int i = 0; i < n; i++) tmp[i] = prims[b + ab[bax].key[i].second];
            std::copy(tmp.begin(), tmp.end(), prims.begin() + b);
            return b + ab[bax].k;
        }
        int axis = widest, best_s = -1;
        double best = DBL_MAX;
        for (int c = 0; c < 3; c++) {
            if (!(cb.hi[c] - cb.lo[c] > 0) || (!MCPT_BVH_ALL_AXES && c != widest)) continue;
            double cost;
            const int s_c = sweep(c, &cost);
            if (s_c > 0 && cost < best) best = cost, best_s = s_c, axis = c;
        }
        int mid = -1;
        if (cb.hi[widest] - cb.lo[widest] > 0) {
            const double leaf_cost = box.area() * n;
            if (best_s > 0 && (best + MCPT_BVH_CTRAV * box.area() < leaf_cost || n > 4 * max_leaf)) {
                auto it = std::partition(prims.begin() + b, prims.begin() + e,
                                         [&](const Prim& p) { return bin_of(p, axis) < best_s; });
                mid = static_cast<int>(it - prims.begin());
            } else {
                return -1;
            }
        }
        if (mid <= b || mid >= e) {  // degenerate centroids: median split on index
            if (n <= max_leaf) return -1;
            std::nth_element(prims.begin() + b, prims.begin() + b + n / 2, prims.begin() + e,
                             [&](const Prim& x, const Prim& y) { return x.c[axis] < y.c[axis]; });
            mid = b + n / 2;
        }
        return mid;
    }

    // Two phases, so that the (dominant) split searches of disjoint ranges run in parallel while the
    // node / leaf order stays the serial DFS order: plan() decides every split of [b, e) (split() only
    // permutes prims[b, e)), ranges above kParallelPrims on their own thread; emit() writes the nodes.
    struct Plan {
        int mid = -1;  // < 0: leaf
        std::unique_ptr<Plan> l, r;
    };
    static constexpr int kParallelPrims = 1 << 17;
    std::unique_ptr<Plan> plan(int b, int e, int depth) {
        auto p = std::make_unique<Plan>();
        int mid = (depth >= kMaxDepth) ? -1 : split(prims, b, e, bounds(b, e));
        if (mid < 0) {
            if (e - b <= 64) return p;
            mid = b + (e - b) / 2;  // depth cap reached with a fat leaf: force a median split anyway
        }
        p->mid = mid;
        if (e - b > kParallelPrims) {
            run_pair([&] { p->l = plan(b, mid, depth + 1); }, [&] { p->r = plan(mid, e, depth + 1); });
        } else {
            p->l = plan(b, mid, depth + 1);
            p->r = plan(mid, e, depth + 1);
        }
        return p;
    }
    // ---- spatial splits (MCPT_BVH_SPATIAL; Stich, Friedrich & Dietrich, HPG 2009) ----
    // A node whose best object split leaves children that overlap by more than kSpatialAlpha of the root's
    // area also tries planes through space: a reference straddling the plane goes to both sides, each with
    // the box of its triangle clipped to that side (and to its own box).  The references live in vectors
    // owned by the plan nodes (a leaf keeps its facet list), so a facet may sit in several leaves; the
    // traversal's closest-hit rule (t, then the lower facet id) makes a repeated test a no-op.
    const HostScene* hs = nullptr;
    double root_area = 0;
    int64_t spatial_budget = 0;  // duplicates allowed over the whole tree (MCPT_BVH_SPATIAL_BUDGET per facet)
    static constexpr double kSpatialAlpha = MCPT_BVH_SPATIAL_ALPHA;
    static constexpr int kSBins = 32;
    // the box of facet f's part inside [lo, hi] along axis, intersected with `clip` (empty if none)
    Box clip_box(int32_t f, const Box& clip, int axis, double lo, double hi) const {
        double poly[9][3], tmp[9][3];
        int np = 3;
        for (int k = 0; k < 3; k++)
            for (int c = 0; c < 3; c++) poly[k][c] = hs->pos[9 * (size_t)f + 3 * k + c];
        auto cut = [&](double plane, bool keep_above) {  // Sutherland-Hodgman against one plane
            int nt = 0;
            for (int i = 0; i < np; i++) {
                const double* p = poly[i];
                const double* q = poly[(i + 1) % np];
                const double dp = keep_above ? p[axis] - plane : plane - p[axis];
                const double dq = keep_above ? q[axis] - plane : plane - q[axis];
                if (dp >= 0) std::memcpy(tmp[nt++], p, sizeof(tmp[0]));
                if ((dp >= 0) != (dq >= 0)) {
                    const double t = dp / (dp - dq);
                    for (int c = 0; c < 3; c++) tmp[nt][c] = p[c] + t * (q[c] - p[c]);
                    tmp[nt][axis] = plane;
                    nt++;
                }
            }
            np = nt;
            std::memcpy(poly, tmp, sizeof(double) * 3 * nt);
        };
        cut(lo, true);
        if (np) cut(hi, false);
        Box r;
        for (int i = 0; i < np; i++) r.grow(poly[i]);
        for (int c = 0; c < 3 && np; c++) r.lo[c] = std::max(r.lo[c], clip.lo[c]), r.hi[c] = std::min(r.hi[c], clip.hi[c]);
        if (np == 0 || r.lo[0] > r.hi[0] || r.lo[1] > r.hi[1] || r.lo[2] > r.hi[2]) return Box();
        return r;
    }
    // the best spatial split of refs in `box`: cost (A_L N_L + A_R N_R), axis and plane; false if none helps
    bool spatial_split(const std::vector<Prim>& refs, const Box& box, double* cost, int* axis, double* plane) const {
        const int n = static_cast<int>(refs.size());
        bool found = false;
        for (int a = 0; a < 3; a++) {
            const double lo = box.lo[a], ext = box.hi[a] - box.lo[a];
            if (!(ext > 0)) continue;
            Box bb[kSBins];
            int enter[kSBins] = {0}, leave[kSBins] = {0};
            auto bin = [&](double x) { return std::min(kSBins - 1, std::max(0, static_cast<int>((x - lo) * (kSBins / ext)))); };
            auto edge = [&](int i) { return i == kSBins ? box.hi[a] : lo + ext * i / kSBins; };
            for (const Prim& p : refs) {
                const int b0 = bin(p.box.lo[a]), b1 = bin(p.box.hi[a]);
                enter[b0]++, leave[b1]++;
                if (b0 == b1) {
                    bb[b0].grow(p.box);
                    continue;
                }
                for (int k = b0; k <= b1; k++) {
                    const Box c = clip_box(p.facet, p.box, a, edge(k), edge(k + 1));
                    if (c.lo[0] <= c.hi[0]) bb[k].grow(c);
                }
            }
            double right_area[kSBins];
            int right_cnt[kSBins];
            Box acc;
            int ac = 0;
            for (int k = kSBins - 1; k > 0; k--) acc.grow(bb[k]), ac += leave[k], right_area[k] = acc.area(), right_cnt[k] = ac;
            acc = Box();
            ac = 0;
            for (int k = 1; k < kSBins; k++) {
                acc.grow(bb[k - 1]);
                ac += enter[k - 1];
                if (ac == 0 || right_cnt[k] == 0 || ac >= n || right_cnt[k] >= n) continue;  // must shrink both sides
                const double c = acc.area() * ac + right_area[k] * right_cnt[k];
                if (!found || c < *cost) *cost = c, *axis = a, *plane = edge(k), found = true;
            }
        }
        return found;
    }
    struct SPlan {
        Box box;
        std::vector<int32_t> facets;  // a leaf's references
        std::unique_ptr<SPlan> l, r;
    };
    static Box vbounds(const std::vector<Prim>& v, int b, int e) {
        Box r;
        for (int i = b; i < e; i++) r.grow(v[i].box);
        return r;
    }
    // budget: the duplicates this subtree may still create.  It is passed down by value -- what a node does not
    // spend is shared between its children in proportion to their references -- so the tree depends only on the
    // scene, never on which builder thread got to a shared counter first, and the whole tree never exceeds the
    // budget it started with (a split that would is taken as the object split instead)
    std::unique_ptr<SPlan> splan(std::vector<Prim> refs, int depth, int64_t budget) {
        auto p = std::make_unique<SPlan>();
        const int n = static_cast<int>(refs.size());
        p->box = vbounds(refs, 0, n);
        int mid = (depth >= kMaxDepth) ? -1 : split(refs, 0, n, p->box);
        if (mid < 0 && n > 64) mid = n / 2;  // depth cap reached with a fat leaf: force a median split anyway
        if (mid < 0) {
            for (const Prim& q : refs) p->facets.push_back(q.facet);
            return p;
        }
        std::vector<Prim> L, R;
        const Box bl = vbounds(refs, 0, mid), br = vbounds(refs, mid, n);
        Box ov;
        for (int c = 0; c < 3; c++) ov.lo[c] = std::max(bl.lo[c], br.lo[c]), ov.hi[c] = std::min(bl.hi[c], br.hi[c]);
        const bool overlap = ov.lo[0] <= ov.hi[0] && ov.lo[1] <= ov.hi[1] && ov.lo[2] <= ov.hi[2];
        double scost = 0, plane = 0;
        int sax = 0;
        int64_t dup = 0;
        if (depth < kMaxDepth && overlap && ov.area() > kSpatialAlpha * root_area && budget > 0 &&
            spatial_split(refs, p->box, &scost, &sax, &plane) && scost < bl.area() * mid + br.area() * (n - mid)) {
            for (const Prim& q : refs) {
                if (q.box.hi[sax] <= plane) {
                    L.push_back(q);
                } else if (q.box.lo[sax] >= plane) {
                    R.push_back(q);
                } else {
                    Prim a = q, b = q;
                    a.box = clip_box(q.facet, q.box, sax, -DBL_MAX, plane);
                    b.box = clip_box(q.facet, q.box, sax, plane, DBL_MAX);
                    const bool ha = a.box.lo[0] <= a.box.hi[0], hb = b.box.lo[0] <= b.box.hi[0];
                    for (Prim* x : {&a, &b})
                        for (int c = 0; c < 3; c++) x->c[c] = 0.5 * (x->box.lo[c] + x->box.hi[c]);
                    if (ha) L.push_back(a);
                    if (hb) R.push_back(b);
                    if (!ha && !hb) L.push_back(q);  // (clipping lost it to rounding: keep it whole)
                    if (ha && hb) dup++;
                }
            }
            if (L.empty() || R.empty() || static_cast<int>(L.size()) >= n || static_cast<int>(R.size()) >= n ||
                dup > budget) {
                L.assign(refs.begin(), refs.begin() + mid);  // no progress, or over budget: the object split after all
                R.assign(refs.begin() + mid, refs.end());
                dup = 0;
            }
        } else {
            L.assign(refs.begin(), refs.begin() + mid);
            R.assign(refs.begin() + mid, refs.end());
        }
        std::vector<Prim>().swap(refs);
        const int64_t left = budget - dup;
        const int64_t bl_share = static_cast<int64_t>(static_cast<double>(left) * L.size() / (L.size() + R.size()));
        const int64_t br_share = left - bl_share;
        if (n > kParallelPrims) {
            run_pair([&] { p->l = splan(std::move(L), depth + 1, bl_share); },
                     [&] { p->r = splan(std::move(R), depth + 1, br_share); });
        } else {
            p->l = splan(std::move(L), depth + 1, bl_share);
            p->r = splan(std::move(R), depth + 1, br_share);
        }
        return p;
    }
    void semit(int32_t parent, int slot, const SPlan& p) {
        to_float_box(p.box, out->nodes[parent].lo[slot], out->nodes[parent].hi[slot]);
        if (!p.l) {
            out->nodes[parent].child[slot] = ~static_cast<int32_t>(out->leaf_facets.size());
            out->nodes[parent].count[slot] = static_cast<int32_t>(p.facets.size());
            out->leaf_facets.insert(out->leaf_facets.end(), p.facets.begin(), p.facets.end());
            return;
        }
        int32_t me = static_cast<int32_t>(out->nodes.size());
        out->nodes.push_back(BvhNode{});
        out->nodes[parent].child[slot] = me;
        out->nodes[parent].count[slot] = 0;
        semit(me, 0, *p.l);
        semit(me, 1, *p.r);
    }
    // writes the planned subtree of [b, e) as the child slot `slot` of node `parent`
    void emit(int b, int e, int32_t parent, int slot, const Plan& p) {
        to_float_box(bounds(b, e), out->nodes[parent].lo[slot], out->nodes[parent].hi[slot]);
        if (p.mid < 0) {
            int32_t cnt;
            int32_t leaf = make_leaf(b, e, cnt);
            out->nodes[parent].child[slot] = leaf;
            out->nodes[parent].count[slot] = cnt;
            return;
        }
        int32_t me = static_cast<int32_t>(out->nodes.size());
        out->nodes.push_back(BvhNode{});
        out->nodes[parent].child[slot] = me;
        out->nodes[parent].count[slot] = 0;
        emit(b, p.mid, me, 0, *p.l);
        emit(p.mid, e, me, 1, *p.r);
    }
};

}  // namespace

Bvh build_bvh(const HostScene& s, const std::vector<int32_t>& facets, int max_leaf) {
    Bvh bvh;
    Builder B;
    B.out = &bvh;
    B.max_leaf = max_leaf;
    Box scene;
    B.prims.resize(facets.size());
    for (size_t i = 0; i < facets.size(); i++) {
        Prim& p = B.prims[i];
        p.facet = facets[i];
        for (int k = 0; k < 3; k++) {
            double v[3] = {s.pos[9 * facets[i] + 3 * k], s.pos[9 * facets[i] + 3 * k + 1], s.pos[9 * facets[i] + 3 * k + 2]};
            p.box.grow(v);
        }
        for (int c = 0; c < 3; c++) p.c[c] = 0.5 * (p.box.lo[c] + p.box.hi[c]);
        scene.grow(p.box);
    }
    double ext = 0;
    for (int c = 0; c < 3; c++) ext = std::max(ext, scene.hi[c] - scene.lo[c]);
    B.margin = 1e-5 * ext + 1e-6;
    BvhNode root{};
    for (int k = 0; k < 2; k++) {
        for (int c = 0; c < 3; c++) {
            root.lo[k][c] = FLT_MAX;
            root.hi[k][c] = -FLT_MAX;
        }
        root.child[k] = ~0;
        root.count[k] = 0;
    }
    bvh.nodes.push_back(root);
    if (facets.empty()) return bvh;
    const int n = static_cast<int>(facets.size());
    Box all = B.bounds(0, n);
    if (MCPT_BVH_SPATIAL && n >= MCPT_BVH_SPATIAL_MIN) {
        B.hs = &s;
        B.root_area = all.area();
        B.spatial_budget = static_cast<int64_t>(MCPT_BVH_SPATIAL_BUDGET * n);
        std::unique_ptr<Builder::SPlan> root_plan = B.splan(std::move(B.prims), 0, B.spatial_budget);
        if (!root_plan->l) {  // one leaf: the root's slot 0 (slot 1 stays empty)
            B.to_float_box(root_plan->box, bvh.nodes[0].lo[0], bvh.nodes[0].hi[0]);
            bvh.nodes[0].child[0] = ~0;
            bvh.nodes[0].count[0] = static_cast<int32_t>(root_plan->facets.size());
            bvh.leaf_facets = root_plan->facets;
        } else {
            B.semit(0, 0, *root_plan->l);
            B.semit(0, 1, *root_plan->r);
        }
        return bvh;
    }
    int mid = B.split(B.prims, 0, n, all);
    if (mid < 0) {
        B.to_float_box(all, bvh.nodes[0].lo[0], bvh.nodes[0].hi[0]);
        int32_t cnt;
        bvh.nodes[0].child[0] = B.make_leaf(0, n, cnt);
        bvh.nodes[0].count[0] = cnt;
    } else {
        std::unique_ptr<Builder::Plan> pl, pr;
        run_pair([&] { pl = B.plan(0, mid, 1); }, [&] { pr = B.plan(mid, n, 1); });
        B.emit(0, mid, 0, 0, *pl);
        B.emit(mid, n, 0, 1, *pr);
    }
    return bvh;
}

namespace {
double box_area(const float* lo, const float* hi) {
    if (lo[0] > hi[0]) return 0;
    const double d[3] = {(double)hi[0] - lo[0], (double)hi[1] - lo[1], (double)hi[2] - lo[2]};
    return 2 * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
}
struct Cand {
    int32_t child, count;
    float lo[3], hi[3];
};
int32_t collapse(const Bvh& b, int32_t n2, std::vector<BvhNode4>& out) {
    const int32_t me = static_cast<int32_t>(out.size());
    out.push_back(BvhNode4{});
    std::vector<Cand> cs;
    auto add_children = [&](int32_t node) {
        const BvhNode& nd = b.nodes[node];
        for (int k = 0; k < 2; k++) {
            if (nd.child[k] < 0 && nd.count[k] == 0) continue;  // empty slot (single-leaf root)
            Cand c;
            c.child = nd.child[k];
            c.count = nd.count[k];
            for (int a = 0; a < 3; a++) {
                c.lo[a] = nd.lo[k][a];
                c.hi[a] = nd.hi[k][a];
            }
            cs.push_back(c);
        }
    };
    add_children(n2);
    while (cs.size() < 4) {
        int best = -1;
        double ba = -1;
        for (size_t i = 0; i < cs.size(); i++)
            if (cs[i].child >= 0 && box_area(cs[i].lo, cs[i].hi) > ba) {
                ba = box_area(cs[i].lo, cs[i].hi);
                best = static_cast<int>(i);
            }
        if (best < 0) break;
        const int32_t inner = cs[best].child;
        cs.erase(cs.begin() + best);
        add_children(inner);
    }
    int32_t child[4];
    for (size_t k = 0; k < 4; k++) child[k] = kBvh4Empty;
    for (size_t k = 0; k < cs.size(); k++) child[k] = cs[k].child >= 0 ? collapse(b, cs[k].child, out) : cs[k].child;
    BvhNode4& o = out[me];
    for (int k = 0; k < 4; k++) {
        const bool used = k < static_cast<int>(cs.size());
        for (int a = 0; a < 3; a++) {
            o.lo[a][k] = used ? cs[k].lo[a] : FLT_MAX;
            o.hi[a][k] = used ? cs[k].hi[a] : -FLT_MAX;
        }
        o.child[k] = child[k];
        o.count[k] = used ? cs[k].count : 0;
    }
    return me;
}

}  // namespace

std::vector<BvhNode4> collapse_bvh4(const Bvh& b) {
    std::vector<BvhNode4> out;
    if (!b.nodes.empty()) collapse(b, 0, out);
    return out;
}

namespace {
float decode_plane(int q, int bexp, float org) {
    uint32_t bits = (uint32_t)bexp << 23;
    float sc;
    std::memcpy(&sc, &bits, 4);
    return std::fmaf((float)q, sc, org);  // the traversal's v_fma_f32 (correctly rounded on both sides)
}
}  // namespace

std::vector<BvhNode4Q> quantize_bvh4(const std::vector<BvhNode4>& in) {
    std::vector<BvhNode4Q> out(in.size());
    for (size_t i = 0; i < in.size(); i++) {
        const BvhNode4& n = in[i];
        BvhNode4Q& o = out[i];
        std::memset(&o, 0, sizeof(o));
        bool used[4];
        for (int k = 0; k < 4; k++) {
            o.child[k] = n.child[k];
            used[k] = n.child[k] != kBvh4Empty && n.lo[0][k] <= n.hi[0][k];
        }
        for (int a = 0; a < 3; a++) {
            float lo = FLT_MAX, hi = -FLT_MAX;
            for (int k = 0; k < 4; k++)
                if (used[k]) {
                    lo = std::min(lo, n.lo[a][k]);
                    hi = std::max(hi, n.hi[a][k]);
                }
            if (lo > hi) lo = hi = 0.0f;  // no child: any planes (the traversal skips kBvh4Empty)
            o.org[a] = lo;
            // smallest scale 2^(b - 127) whose 255 steps from org reach hi in the decode arithmetic
            const double ext = (double)hi - (double)lo;
            int b = ext > 0 ? std::max(1, std::min(254, (int)std::ceil(std::log2(ext / 255.0)) + 127 - 1)) : 1;
            uint32_t qlo = 0, qhi = 0;
            for (;; b++) {
                if (b > 254) b = 254;
                bool ok = decode_plane(255, b, lo) >= hi || b == 254;
                qlo = qhi = 0;
                for (int k = 0; ok && k < 4; k++) {
                    if (!used[k]) {
                        qlo |= 255u << (8 * k);  // empty slot: lo > hi
                        continue;
                    }
                    const double scale = std::ldexp(1.0, b - 127);
                    int ql = std::max(0, std::min(255, (int)std::floor(((double)n.lo[a][k] - lo) / scale)));
                    while (ql > 0 && decode_plane(ql, b, lo) > n.lo[a][k]) ql--;
                    int qh = std::max(0, std::min(255, (int)std::ceil(((double)n.hi[a][k] - lo) / scale)));
                    while (qh < 255 && decode_plane(qh, b, lo) < n.hi[a][k]) qh++;
                    if (decode_plane(ql, b, lo) > n.lo[a][k] || decode_plane(qh, b, lo) < n.hi[a][k]) {
                        ok = false;  // needs a coarser scale
                        break;
                    }
                    qlo |= (uint32_t)ql << (8 * k);
                    qhi |= (uint32_t)qh << (8 * k);
                }
                if (ok || b == 254) break;
            }
            o.ex |= (uint32_t)b << (8 * a);
            o.q[2 * a] = qlo;
            o.q[2 * a + 1] = qhi;
        }
    }
    return out;
}

// ---- 8-wide compressed tree (BvhNode8Q) ----
namespace {
struct BN {  // binary node with its own box: inner (l, r >= 0) or leaf (first, count <= 2 after splitting)
    float lo[3], hi[3];
    int32_t l = -1, r = -1;
    int32_t first = 0, count = 0;
};
struct Bvh8Builder {
    const HostScene& s;
    const Bvh& b;
    double margin = 0;
    std::vector<BN> bn;
    Bvh8 out;
    Bvh8Builder(const HostScene& s_, const Bvh& b_) : s(s_), b(b_) {}

    // box of leaf slots [first, first + count): the triangles' float vertices, enlarged like Builder::to_float_box
    void leaf_box(int32_t first, int32_t count, float* lo, float* hi) const {
        double l[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, h[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int32_t i = first; i < first + count; i++) {
            const float* v = &s.pos[9 * (size_t)b.leaf_facets[i]];
            for (int k = 0; k < 3; k++)
                for (int c = 0; c < 3; c++) l[c] = std::min(l[c], (double)v[3 * k + c]), h[c] = std::max(h[c], (double)v[3 * k + c]);
        }
        for (int c = 0; c < 3; c++) {
            lo[c] = std::nextafter(static_cast<float>(l[c] - margin), -FLT_MAX);
            hi[c] = std::nextafter(static_cast<float>(h[c] + margin), FLT_MAX);
        }
    }
    // a leaf of the binary tree (box as stored there); more than two triangles: index halves, boxes of their own
    int32_t leaf(int32_t first, int32_t count, const float* lo, const float* hi) {
        const int32_t me = (int32_t)bn.size();
        bn.push_back(BN{});
        for (int c = 0; c < 3; c++) bn[me].lo[c] = lo[c], bn[me].hi[c] = hi[c];
        if (count <= 2) {
            bn[me].first = first, bn[me].count = count;
            return me;
        }
        const int32_t h = count / 2;
        float l0[3], h0[3], l1[3], h1[3];
        leaf_box(first, h, l0, h0);
        leaf_box(first + h, count - h, l1, h1);
        const int32_t a = leaf(first, h, l0, h0), c = leaf(first + h, count - h, l1, h1);
        bn[me].l = a, bn[me].r = c;
        return me;
    }
    // child k of binary node ni, or -1 for the single-leaf root's empty slot
    int32_t conv(int32_t ni, int k) {
        const BvhNode& nd = b.nodes[ni];
        if (nd.child[k] < 0 && nd.count[k] == 0) return -1;
        if (nd.child[k] < 0) return leaf(~nd.child[k], nd.count[k], nd.lo[k], nd.hi[k]);
        const int32_t me = (int32_t)bn.size();
        bn.push_back(BN{});
        for (int c = 0; c < 3; c++) bn[me].lo[c] = nd.lo[k][c], bn[me].hi[c] = nd.hi[k][c];
        const int32_t a = conv(nd.child[k], 0), c = conv(nd.child[k], 1);
        bn[me].l = a, bn[me].r = c;
        return me;
    }
    static double area(const BN& x) { return box_area(x.lo, x.hi); }

    // fills node `self` from the children of binary node `root` (collapsed up to eight)
    void node(int32_t root, int32_t self, int depth = 1) {
        out.depth = std::max(out.depth, depth);
        std::vector<int32_t> cand;
        for (int32_t c : {bn[root].l, bn[root].r})
            if (c >= 0) cand.push_back(c);
        while (cand.size() < 8) {  // expand the largest-area inner candidate (as collapse_bvh4)
            int best = -1;
            double ba = -1;
            for (size_t i = 0; i < cand.size(); i++)
                if (bn[cand[i]].l >= 0 && area(bn[cand[i]]) > ba) ba = area(bn[cand[i]]), best = (int)i;
            if (best < 0) break;
            const int32_t in = cand[best];
            cand.erase(cand.begin() + best);
            for (int32_t c : {bn[in].l, bn[in].r})
                if (c >= 0) cand.push_back(c);
        }
        // octant slots: greedy over (child, slot) by the child centre's offset from the node centre along
        // the slot's direction (bit a set: -a)
        double nlo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, nhi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
        for (int32_t c : cand)
            for (int a = 0; a < 3; a++) nlo[a] = std::min(nlo[a], (double)bn[c].lo[a]), nhi[a] = std::max(nhi[a], (double)bn[c].hi[a]);
        int32_t slot_of[8];
        for (int k = 0; k < 8; k++) slot_of[k] = -1;  // child at slot
        std::vector<bool> placed(cand.size(), false);
        for (size_t it = 0; it < cand.size(); it++) {
            double bs = -DBL_MAX;
            int bc = -1, bsl = -1;
            for (size_t i = 0; i < cand.size(); i++) {
                if (placed[i]) continue;
                for (int sl = 0; sl < 8; sl++) {
                    if (slot_of[sl] >= 0) continue;
                    double sc = 0;
                    for (int a = 0; a < 3; a++) {
                        const double off = 0.5 * ((double)bn[cand[i]].lo[a] + bn[cand[i]].hi[a]) - 0.5 * (nlo[a] + nhi[a]);
                        sc += ((sl >> a) & 1) ? -off : off;
                    }
                    if (sc > bs) bs = sc, bc = (int)i, bsl = sl;
                }
            }
            placed[bc] = true;
            slot_of[bsl] = (int32_t)bc;
        }
        // inner children contiguous in slot order; leaf triangles at base_tri + 2 slot + j
        int ninner = 0, kmin = 8, kmax = -1;
        for (int sl = 0; sl < 8; sl++) {
            if (slot_of[sl] < 0) continue;
            const BN& c = bn[cand[slot_of[sl]]];
            if (c.l >= 0) ninner++;
            else kmin = std::min(kmin, sl), kmax = std::max(kmax, sl);
        }
        // inner children at base_inner + slot (eight node slots reserved per node with inner children, the
        // unused ones never referenced): a stack entry is then (base, hit bits) in one word
        const int32_t base_inner = ninner > 0 ? (int32_t)out.nodes.size() : 0;
        if (ninner > 0) out.nodes.resize(out.nodes.size() + 8);
        int32_t base_tri = 0;
        uint32_t tvalid = 0, imask = 0;
        if (kmax >= 0) {
            const int32_t at = (int32_t)out.tri_facets.size();
            out.tri_facets.resize(out.tri_facets.size() + 2 * (kmax - kmin + 1), -1);
            base_tri = at - 2 * kmin;
        }
        std::vector<std::pair<int32_t, int32_t>> todo;  // (binary node, node index)
        for (int sl = 0; sl < 8; sl++) {
            if (slot_of[sl] < 0) continue;
            const BN& c = bn[cand[slot_of[sl]]];
            if (c.l >= 0) {
                imask |= 1u << sl;
                todo.emplace_back(cand[slot_of[sl]], base_inner + sl);
            } else {
                for (int j = 0; j < c.count; j++) {
                    out.tri_facets[base_tri + 2 * sl + j] = b.leaf_facets[c.first + j];
                    tvalid |= 1u << (2 * sl + j);
                }
            }
        }
        // quantized planes (as quantize_bvh4): per axis the union minimum and the smallest power-of-two
        // scale whose 255 steps reach the maximum, each plane rounded outward in the decode arithmetic
        BvhNode8Q o;
        std::memset(&o, 0, sizeof(o));
        for (int a = 0; a < 3; a++) {
            float lo = FLT_MAX, hi = -FLT_MAX;
            for (int sl = 0; sl < 8; sl++)
                if (slot_of[sl] >= 0) lo = std::min(lo, bn[cand[slot_of[sl]]].lo[a]), hi = std::max(hi, bn[cand[slot_of[sl]]].hi[a]);
            if (lo > hi) lo = hi = 0.0f;
            o.org[a] = lo;
            const double ext = (double)hi - (double)lo;
            int e = ext > 0 ? std::max(1, std::min(254, (int)std::ceil(std::log2(ext / 255.0)) + 127 - 1)) : 1;
            uint32_t ql[2], qh[2];
            for (;; e++) {
                if (e > 254) e = 254;
                bool ok = decode_plane(255, e, lo) >= hi || e == 254;
                ql[0] = ql[1] = qh[0] = qh[1] = 0;
                for (int sl = 0; ok && sl < 8; sl++) {
                    const int h = sl >> 2, sh = 8 * (sl & 3);
                    if (slot_of[sl] < 0) {
                        ql[h] |= 255u << sh;  // empty slot (the traversal masks it out)
                        continue;
                    }
                    const BN& c = bn[cand[slot_of[sl]]];
                    const double scale = std::ldexp(1.0, e - 127);
                    int q0 = std::max(0, std::min(255, (int)std::floor(((double)c.lo[a] - lo) / scale)));
                    while (q0 > 0 && decode_plane(q0, e, lo) > c.lo[a]) q0--;
                    int q1 = std::max(0, std::min(255, (int)std::ceil(((double)c.hi[a] - lo) / scale)));
                    while (q1 < 255 && decode_plane(q1, e, lo) < c.hi[a]) q1++;
                    if (decode_plane(q0, e, lo) > c.lo[a] || decode_plane(q1, e, lo) < c.hi[a]) {
                        ok = false;
                        break;
                    }
                    ql[h] |= (uint32_t)q0 << sh;
                    qh[h] |= (uint32_t)q1 << sh;
                }
                if (ok || e == 254) break;
            }
            o.ex |= (uint32_t)e << (8 * a);
            o.qlo[a][0] = ql[0], o.qlo[a][1] = ql[1];
            o.qhi[a][0] = qh[0], o.qhi[a][1] = qh[1];
        }
        o.ex |= imask << 24;
        o.base_inner = base_inner;
        o.base_tri = base_tri;
        o.tvalid = tvalid;
        out.nodes[self] = o;
        for (auto& t : todo) node(t.first, t.second, depth + 1);
    }
};
}  // namespace

Bvh8 build_bvh8(const HostScene& s, const Bvh& b) {
    Bvh8Builder B(s, b);
    double lo[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, hi[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX};
    for (int32_t f : b.leaf_facets)
        for (int k = 0; k < 9; k++) lo[k % 3] = std::min(lo[k % 3], (double)s.pos[9 * (size_t)f + k]), hi[k % 3] = std::max(hi[k % 3], (double)s.pos[9 * (size_t)f + k]);
    double ext = 0;
    for (int c = 0; c < 3; c++) ext = std::max(ext, hi[c] - lo[c]);
    B.margin = 1e-5 * ext + 1e-6;  // Builder::margin of the same facets
    B.out.nodes.resize(1);
    if (b.nodes.empty() || b.leaf_facets.empty()) {  // no facets: a root without children
        std::memset(&B.out.nodes[0], 0, sizeof(BvhNode8Q));
        return B.out;
    }
    BN root;
    root.l = -1, root.r = -1;
    B.bn.push_back(root);
    const int32_t a = B.conv(0, 0), c = B.conv(0, 1);
    B.bn[0].l = a, B.bn[0].r = c;
    if (B.bn[0].l < 0) std::swap(B.bn[0].l, B.bn[0].r);
    B.node(0, 0);
    return B.out;
}

}  // namespace mcpt
