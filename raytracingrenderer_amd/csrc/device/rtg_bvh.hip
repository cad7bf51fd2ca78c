// rtg_bvh.hip — host-side construction of the binary tree the wide nodes are cut from, with spatial
// splits (SBVH, Stich, Friedrich, Dietrich 2009): a triangle may be referenced by several leaf slots,
// each bounding the part of the triangle inside its region (the triangle clipped to the region's box).
//
// Exactness: k_trace accepts a candidate only through Triangle::rayIntersect on
// the full triangle record and the exact slab test on the triangle's reference leaf box (leafbox), so
// a slot's box only decides *whether* a triangle is tested. The fragments of a triangle cover it (the
// clip regions of a spatial split share only their plane), every fragment box is rounded outward to
// float and inflated by eta = 2^-17 of the scene scale like the single-triangle slots (item 3b), so
// every point within rounding of the triangle lies in some slot box, and a hit rayIntersect reports is
// reached through one of its slots. A triangle tested from two slots returns the same (t, id) twice,
// which the (t, id) minimum and the any-hit test absorb.
//
// Output: the descriptor's node format (links {left, right, start, end}, bounds {min xyz, max xyz};
// node 0 the root; a leaf is one triangle t: {-1, -1, t, t + 1}).
#include "rtg_internal.h"

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Ref {
    int tri;
    double lo[3], hi[3];  // the fragment's box (the clipped polygon's bounds, within the region)
};

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void add(const double* l, const double* h) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], l[a]); hi[a] = std::max(hi[a], h[a]); }
    }
    void add(const Ref& r) { add(r.lo, r.hi); }
    void add(const Box& b) { add(b.lo, b.hi); }
    bool empty() const { return lo[0] > hi[0]; }
    double area() const {
        if (empty()) return 0.0;
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return x * y + y * z + z * x;
    }
};

double overlap_area(const Box& a, const Box& b) {
    Box o;
    for (int k = 0; k < 3; ++k) {
        o.lo[k] = std::max(a.lo[k], b.lo[k]);
        o.hi[k] = std::min(a.hi[k], b.hi[k]);
        if (o.lo[k] > o.hi[k]) return 0.0;
    }
    return o.area();
}

// Bounds of triangle v clipped to the box [lo, hi] (Sutherland-Hodgman over the six planes), in
// double; false when nothing is left. The result is clamped to the box.
bool clip_bounds(const double v[3][3], const double* lo, const double* hi, double* out_lo, double* out_hi) {
    double a[12][3], b[12][3];
    int n = 3;
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) a[i][k] = v[i][k];
    for (int ax = 0; ax < 3; ++ax)
        for (int side = 0; side < 2; ++side) {
            const double c = side ? hi[ax] : lo[ax];
            auto inside = [&](const double* p) { return side ? p[ax] <= c : p[ax] >= c; };
            int m = 0;
            for (int i = 0; i < n; ++i) {
                const double* p = a[i];
                const double* q = a[(i + 1) % n];
                const bool pi = inside(p), qi = inside(q);
                if (pi) { std::memcpy(b[m++], p, sizeof(double) * 3); }
                if (pi != qi && m < 12) {
                    const double t = (c - p[ax]) / (q[ax] - p[ax]);
                    for (int k = 0; k < 3; ++k) b[m][k] = p[k] + t * (q[k] - p[k]);
                    b[m][ax] = c;
                    ++m;
                }
            }
            n = std::min(m, 9);
            if (n == 0) return false;
            std::memcpy(a, b, sizeof(double) * 3 * n);
        }
    for (int k = 0; k < 3; ++k) { out_lo[k] = INFINITY; out_hi[k] = -INFINITY; }
    for (int i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) {
            out_lo[k] = std::min(out_lo[k], a[i][k]);
            out_hi[k] = std::max(out_hi[k], a[i][k]);
        }
    for (int k = 0; k < 3; ++k) {
        out_lo[k] = std::max(out_lo[k], lo[k]);
        out_hi[k] = std::min(out_hi[k], hi[k]);
        if (out_lo[k] > out_hi[k]) return false;
    }
    return true;
}

struct Builder {
    const rtg_scene_desc* d;
    std::vector<int32_t> lk;    // links of this builder's nodes (node 0 = its root)
    std::vector<Ref> leaf_ref;  // per node: the leaf's reference (tri < 0: internal)
    double root_area = 0.0;
    long budget = 0;            // references that spatial splits may still add
    bool ok = true;
    int stop_depth = 1 << 30;   // build(): below this depth, hand the references to a sub-build
    std::vector<std::pair<int, std::vector<Ref>>> deferred;  // (node, references) of the sub-builds

    explicit Builder(const rtg_scene_desc* d_) : d(d_) {}

    void tri(int t, double v[3][3]) const {
        const float* P = d->positions + (size_t)t * 9;
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) v[i][k] = P[i * 3 + k];
    }

    int new_node() {
        lk.insert(lk.end(), {-1, -1, 0, 0});
        leaf_ref.push_back(Ref{-1, {0, 0, 0}, {0, 0, 0}});
        return (int)leaf_ref.size() - 1;
    }

    // object split over the references' centroids: the full SAH sweep up to RTG_SAH_SWEEP references
    // (sorted per axis), RTG_SAH_BINS bins per axis above. Sets `order` (the references by centroid on
    // the chosen axis, tie by triangle) and the split position in it; the two sides' boxes for the
    // overlap test.
    double object_split(const std::vector<Ref>& r, const Box& cb, std::vector<int>& order, size_t& cut, Box& bl,
                        Box& br) const {
        const size_t m = r.size();
        double best = INFINITY;
        int bax = -1;
        auto cen = [&](int i, int a) { return r[i].lo[a] + r[i].hi[a]; };
        std::vector<int> idx(m);
        if ((long)m <= RTG_SAH_SWEEP) {
            std::vector<Box> suf(m + 1);
            for (int a = 0; a < 3; ++a) {
                for (size_t i = 0; i < m; ++i) idx[i] = (int)i;
                std::sort(idx.begin(), idx.end(), [&](int x, int y) {
                    return cen(x, a) < cen(y, a) || (cen(x, a) == cen(y, a) && r[x].tri < r[y].tri);
                });
                suf[m] = Box();
                for (size_t p = m; p-- > 0;) { suf[p] = suf[p + 1]; suf[p].add(r[idx[p]]); }
                Box left;
                for (size_t p = 1; p < m; ++p) {
                    left.add(r[idx[p - 1]]);
                    const double c = left.area() * (double)p + suf[p].area() * (double)(m - p);
                    if (c < best) { best = c; bax = a; cut = p; bl = left; br = suf[p]; }
                }
            }
            if (bax >= 0) {
                order.resize(m);
                for (size_t i = 0; i < m; ++i) order[i] = (int)i;
                std::sort(order.begin(), order.end(), [&](int x, int y) {
                    return cen(x, bax) < cen(y, bax) || (cen(x, bax) == cen(y, bax) && r[x].tri < r[y].tri);
                });
            }
            return best;
        }
        const int NB = RTG_SAH_BINS;
        int bbin = 0;
        for (int a = 0; a < 3; ++a) {
            const double ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.0)) continue;
            std::vector<Box> bins(NB), right(NB + 1);
            std::vector<long> cnt(NB, 0), rc(NB + 1, 0);
            for (const Ref& x : r) {
                const double c = 0.5 * (x.lo[a] + x.hi[a]);
                const int b = std::min(NB - 1, (int)((c - cb.lo[a]) / ext * NB));
                bins[b].add(x);
                ++cnt[b];
            }
            for (int b = NB - 1; b >= 0; --b) { right[b] = right[b + 1]; right[b].add(bins[b]); rc[b] = rc[b + 1] + cnt[b]; }
            Box left;
            long lc = 0;
            for (int b = 1; b < NB; ++b) {
                left.add(bins[b - 1]);
                lc += cnt[b - 1];
                if (lc == 0 || rc[b] == 0) continue;
                const double c = left.area() * (double)lc + right[b].area() * (double)rc[b];
                if (c < best) { best = c; bax = a; bbin = b; bl = left; br = right[b]; }
            }
        }
        if (bax < 0) return best;
        // the binned split as an order + cut: the references of bins below bbin first
        const double ext = cb.hi[bax] - cb.lo[bax];
        order.clear();
        std::vector<int> hi_side;
        for (size_t i = 0; i < m; ++i) {
            const double c = 0.5 * (r[i].lo[bax] + r[i].hi[bax]);
            (std::min(NB - 1, (int)((c - cb.lo[bax]) / ext * NB)) < bbin ? order : hi_side).push_back((int)i);
        }
        cut = order.size();
        order.insert(order.end(), hi_side.begin(), hi_side.end());
        return best;
    }

    // binned spatial split (RTG_SBVH_BINS slabs per axis): each reference is clipped to every slab it
    // spans; entering / leaving counts give the two sides' reference counts at each plane
    double spatial_split(const std::vector<Ref>& r, const Box& nb, int& ax, double& plane) const {
        const int NB = RTG_SBVH_BINS;
        auto axis = [&](int a, double& pl) -> double {
            double best = INFINITY;
            const double lo = nb.lo[a], ext = nb.hi[a] - nb.lo[a];
            if (!(ext > 0.0)) return best;
            const double w = ext / NB;
            std::vector<Box> bins(NB);
            std::vector<long> enter(NB, 0), leave(NB, 0);
            for (const Ref& x : r) {
                int b0 = (int)((x.lo[a] - lo) / w), b1 = (int)((x.hi[a] - lo) / w);
                b0 = std::min(std::max(b0, 0), NB - 1);
                b1 = std::min(std::max(b1, b0), NB - 1);
                ++enter[b0];
                ++leave[b1];
                if (b0 == b1) {
                    bins[b0].add(x);
                    continue;
                }
                double v[3][3];
                tri(x.tri, v);
                for (int b = b0; b <= b1; ++b) {
                    double sl[3], sh[3], fl[3], fh[3];
                    for (int k = 0; k < 3; ++k) { sl[k] = x.lo[k]; sh[k] = x.hi[k]; }
                    sl[a] = std::max(x.lo[a], lo + w * b);
                    sh[a] = std::min(x.hi[a], b == NB - 1 ? nb.hi[a] : lo + w * (b + 1));
                    if (clip_bounds(v, sl, sh, fl, fh)) bins[b].add(fl, fh);
                }
            }
            std::vector<Box> right(NB + 1);
            std::vector<long> rc(NB + 1, 0);
            for (int b = NB - 1; b >= 0; --b) { right[b] = right[b + 1]; right[b].add(bins[b]); rc[b] = rc[b + 1] + leave[b]; }
            Box left;
            long lc = 0;
            for (int b = 1; b < NB; ++b) {
                left.add(bins[b - 1]);
                lc += enter[b - 1];
                if (lc == 0 || rc[b] == 0 || lc >= (long)r.size() || rc[b] >= (long)r.size()) continue;
                const double c = left.area() * (double)lc + right[b].area() * (double)rc[b];
                if (c < best) { best = c; pl = lo + w * b; }
            }
            return best;
        };
        double cost[3], pl[3] = {0, 0, 0};
        if (r.size() > 65536) {  // the top of the tree: the three axes on threads
            std::thread t1([&] { cost[1] = axis(1, pl[1]); }), t2([&] { cost[2] = axis(2, pl[2]); });
            cost[0] = axis(0, pl[0]);
            t1.join();
            t2.join();
        } else {
            for (int a = 0; a < 3; ++a) cost[a] = axis(a, pl[a]);
        }
        double best = INFINITY;
        ax = -1;
        for (int a = 0; a < 3; ++a)  // the first axis of the lowest cost, as a serial loop would pick
            if (cost[a] < best) { best = cost[a]; ax = a; plane = pl[a]; }
        return best;
    }

    int build(std::vector<Ref>& r, int depth) {
        const int node = new_node();
        if (!ok) return node;
        if (depth > 120) { ok = false; return node; }
        if (depth >= stop_depth && r.size() > 1) {  // a sub-build fills this node in
            deferred.emplace_back(node, std::move(r));
            return node;
        }
        if (r.size() == 1) {
            leaf_ref[node] = r[0];
            lk[(size_t)node * 4 + 2] = r[0].tri;
            lk[(size_t)node * 4 + 3] = r[0].tri + 1;
            return node;
        }
        Box nb, cb;
        for (const Ref& x : r) {
            nb.add(x);
            double c[3];
            for (int k = 0; k < 3; ++k) c[k] = 0.5 * (x.lo[k] + x.hi[k]);
            cb.add(c, c);
        }
        std::vector<int> order;
        size_t cut = 0;
        Box bl, br;
        const double co = object_split(r, cb, order, cut, bl, br);
        const bool have_o = !order.empty() && cut > 0 && cut < r.size();
        int sax = -1;
        double plane = 0.0;
        double cs = INFINITY;
        if (budget > 0 && (!have_o || overlap_area(bl, br) > RTG_SBVH_ALPHA * root_area))
            cs = spatial_split(r, nb, sax, plane);
        std::vector<Ref> L, R;
        if (sax >= 0 && cs < co) {
            long dup = 0;
            for (const Ref& x : r) {
                if (x.hi[sax] <= plane) { L.push_back(x); continue; }
                if (x.lo[sax] >= plane) { R.push_back(x); continue; }
                double v[3][3];
                tri(x.tri, v);
                Ref a = x, b = x;
                double sl[3], sh[3];
                for (int k = 0; k < 3; ++k) { sl[k] = x.lo[k]; sh[k] = x.hi[k]; }
                sh[sax] = plane;
                const bool ka = clip_bounds(v, sl, sh, a.lo, a.hi);
                for (int k = 0; k < 3; ++k) { sl[k] = x.lo[k]; sh[k] = x.hi[k]; }
                sl[sax] = plane;
                const bool kb = clip_bounds(v, sl, sh, b.lo, b.hi);
                if (ka) L.push_back(a);
                if (kb) R.push_back(b);
                if (!ka && !kb) L.push_back(x);  // (rounding: keep the reference whole)
                if (ka && kb) ++dup;
            }
            if (L.empty() || R.empty() || (L.size() >= r.size() && R.size() >= r.size())) {
                L.clear();
                R.clear();
            } else {
                budget -= dup;
            }
        }
        if (L.empty()) {
            // object split (or the median of the current order when every centroid coincides)
            if (have_o) {
                for (size_t i = 0; i < order.size(); ++i) (i < cut ? L : R).push_back(r[order[i]]);
            } else {
                L.assign(r.begin(), r.begin() + r.size() / 2);
                R.assign(r.begin() + r.size() / 2, r.end());
            }
        }
        std::vector<Ref>().swap(r);  // release the parent's list before the recursion
        const int l = build(L, depth + 1);
        const int rr = build(R, depth + 1);
        lk[(size_t)node * 4] = l;
        lk[(size_t)node * 4 + 1] = rr;
        return node;
    }
};

}  // namespace

// The own binary tree with spatial splits over the scene's triangles (rtg_kernels.hip calls it for
// prepare_scene when RTG_SBVH is set). The top levels are built first, down to a depth that leaves
// about 4 subtrees per host thread; the subtrees are then built on threads, each with a share of the
// duplication budget proportional to its references (so the tree does not depend on thread timing),
// and stitched in (a subtree's root takes its placeholder's id; children keep larger ids than their
// parents). false: non-finite input or a degenerate tree (the caller then keeps another tree).
bool build_sbvh(const rtg_scene_desc* d, std::vector<int32_t>& lk, std::vector<float>& bd) {
    const uint32_t nt = d->n_tris;
    if (nt < 2) return false;
    for (size_t k = 0; k < (size_t)nt * 9; ++k)
        if (!std::isfinite(d->positions[k])) return false;
    float scale = 0.0f;
    for (int k = 0; k < 6; ++k)
        if (std::isfinite(d->node_bounds[k])) scale = std::max(scale, std::fabs(d->node_bounds[k]));
    const double eta = std::ldexp((double)scale, -17);
    std::vector<Ref> refs(nt);
    Box root;
    for (uint32_t t = 0; t < nt; ++t) {
        const float* P = d->positions + (size_t)t * 9;
        refs[t].tri = (int)t;
        for (int k = 0; k < 3; ++k) {
            refs[t].lo[k] = std::min(std::min((double)P[k], (double)P[3 + k]), (double)P[6 + k]);
            refs[t].hi[k] = std::max(std::max((double)P[k], (double)P[3 + k]), (double)P[6 + k]);
        }
        root.add(refs[t]);
    }
    const int threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    Builder top(d);
    top.root_area = root.area();
    top.budget = (long)((double)nt * RTG_SBVH_DUP);
    top.stop_depth = nt < 50000 || threads == 1 ? (1 << 30) : 6;  // 2^6 = 64 subtrees at most
    top.build(refs, 0);
    if (!top.ok) return false;
    // the sub-builds: references as deferred, budget split by reference count
    const size_t nsub = top.deferred.size();
    std::vector<Builder> sub;
    sub.reserve(nsub);
    long deferred_refs = 0;
    for (auto& dr : top.deferred) deferred_refs += (long)dr.second.size();
    for (size_t k = 0; k < nsub; ++k) {
        sub.emplace_back(d);
        sub[k].root_area = top.root_area;
        sub[k].budget = deferred_refs ? (long)((double)top.budget * (double)top.deferred[k].second.size() / deferred_refs) : 0;
    }
    {
        std::atomic<size_t> next{0};
        std::vector<std::thread> pool;
        for (int t = 0; t < std::min<int>(threads, (int)nsub); ++t)
            pool.emplace_back([&]() {
                for (size_t k; (k = next.fetch_add(1)) < nsub;) sub[k].build(top.deferred[k].second, 6);
            });
        for (auto& t : pool) t.join();
    }
    for (const Builder& b : sub)
        if (!b.ok) return false;
    // stitch: the top nodes, then each sub-build's nodes 1.. after them; its node 0 is the placeholder
    std::vector<int32_t> L = std::move(top.lk);
    std::vector<Ref> R = std::move(top.leaf_ref);
    for (size_t k = 0; k < nsub; ++k) {
        const int ph = top.deferred[k].first;
        const int base = (int)R.size();
        auto id = [&](int j) { return j == 0 ? ph : base + j - 1; };
        const Builder& b = sub[k];
        for (size_t j = 0; j < b.leaf_ref.size(); ++j) {
            int32_t w[4] = {b.lk[j * 4], b.lk[j * 4 + 1], b.lk[j * 4 + 2], b.lk[j * 4 + 3]};
            if (w[0] >= 0) { w[0] = id(w[0]); w[1] = id(w[1]); }
            if (j == 0) {
                std::memcpy(&L[(size_t)ph * 4], w, sizeof(w));
                R[ph] = b.leaf_ref[0];
            } else {
                L.insert(L.end(), w, w + 4);
                R.push_back(b.leaf_ref[j]);
            }
        }
    }
    // bounds bottom-up (children have larger ids): a leaf's fragment box rounded outward to float and
    // inflated by eta; an internal node's the float union of its children's
    const size_t nn = R.size();
    bd.assign(nn * 6, 0.0f);
    for (size_t i = nn; i-- > 0;) {
        float* o = &bd[i * 6];
        const Ref& x = R[i];
        if (L[i * 4] < 0) {
            for (int k = 0; k < 3; ++k) {
                o[k] = std::nextafter((float)(x.lo[k] - eta), -INFINITY);
                o[3 + k] = std::nextafter((float)(x.hi[k] + eta), INFINITY);
            }
        } else {
            const float* a = &bd[(size_t)L[i * 4] * 6];
            const float* b = &bd[(size_t)L[i * 4 + 1] * 6];
            for (int k = 0; k < 3; ++k) {
                o[k] = std::min(a[k], b[k]);
                o[3 + k] = std::max(a[3 + k], b[3 + k]);
            }
        }
    }
    lk = std::move(L);
    return true;
}
