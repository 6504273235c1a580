// om_bvh.cpp — binned-SAH BVH over spheres, cubes, triangles, parallelograms.
#include "om_bvh.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

// SAH leaves: at most OM_BVH_MAX_LEAF records, always a leaf at OM_BVH_LEAF_FORCE or fewer; a tree
// whose compressed BVH2 does not fit the LDS budget (read through L2: S-10k) is rebuilt with the
// _L2 sizes: one record per leaf, so a ray reads fewer 64-B records and more 32-B half nodes (r05:
// C3 4258 / 4262 vs 4111 / 4119 Msamples/s at leaves <= 8, 4222 / 4240 at <= 2; C1, whose tree
// sits in LDS, 6558 / 6561 at 1 and 6950 / 7016 at 2 vs 7003 / 7016: profiles/r05_bvh2)
#ifndef OM_BVH_MAX_LEAF
#define OM_BVH_MAX_LEAF 8
#endif
#ifndef OM_BVH_LEAF_FORCE
#define OM_BVH_LEAF_FORCE 2
#endif
#ifndef OM_BVH_MAX_LEAF_L2
#define OM_BVH_MAX_LEAF_L2 1
#endif
#ifndef OM_BVH_LEAF_FORCE_L2
#define OM_BVH_LEAF_FORCE_L2 1
#endif
#ifndef OM_BVH_TRAV
#define OM_BVH_TRAV 1.0
#endif

namespace om {
namespace {

struct Box {
    double lo[3], hi[3];
    void empty() { for (int i = 0; i < 3; ++i) { lo[i] = 1e300; hi[i] = -1e300; } }
    void grow(const Box& b) { for (int i = 0; i < 3; ++i) { lo[i] = std::min(lo[i], b.lo[i]); hi[i] = std::max(hi[i], b.hi[i]); } }
    void grow_pt(const double* p) { for (int i = 0; i < 3; ++i) { lo[i] = std::min(lo[i], p[i]); hi[i] = std::max(hi[i], p[i]); } }
    double area() const {
        const double dx = std::max(0.0, hi[0] - lo[0]), dy = std::max(0.0, hi[1] - lo[1]), dz = std::max(0.0, hi[2] - lo[2]);
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
};

struct Item { Box b; double c[3]; uint32_t gi; };

// Inflate a box well beyond f32 rounding of the exact tests.
Box inflate(Box b) {
    double mag = 0.0;
    for (int i = 0; i < 3; ++i) mag = std::max(mag, std::max(std::fabs(b.lo[i]), std::fabs(b.hi[i])));
    for (int i = 0; i < 3; ++i) {
        const double ext = b.hi[i] - b.lo[i];
        const double m = 1e-3 * (1.0 + ext) + 1e-5 * mag;
        b.lo[i] -= m; b.hi[i] += m;
    }
    return b;
}

Box affine_box(const Mat4& l2w, double half) {
    Box b;
    for (int i = 0; i < 3; ++i) {
        const double a0 = l2w.r[i].e[0], a1 = l2w.r[i].e[1], a2 = l2w.r[i].e[2], c = l2w.r[i].e[3];
        // sphere (half < 0): exact ellipsoid extent = row norm; cube: 0.5 * L1 row norm
        const double h = half < 0 ? std::sqrt(a0 * a0 + a1 * a1 + a2 * a2) : half * (std::fabs(a0) + std::fabs(a1) + std::fabs(a2));
        b.lo[i] = c - h; b.hi[i] = c + h;
    }
    return inflate(b);
}

Box bary_box(const BaryPrim& p, bool para) {
    Box b; b.empty();
    double o[3], pu[3], pv[3], puv[3];
    for (int i = 0; i < 3; ++i) {
        o[i] = p.origin.e[i];
        pu[i] = o[i] + (double)p.u.e[i] * p.u_length;
        pv[i] = o[i] + (double)p.v.e[i] * p.v_length;
        puv[i] = pu[i] + (double)p.v.e[i] * p.v_length;
    }
    b.grow_pt(o); b.grow_pt(pu); b.grow_pt(pv);
    if (para) b.grow_pt(puv);
    return inflate(b);
}

struct Builder {
    std::vector<Item> items;
    std::vector<OmBvhNode> nodes;
    std::vector<uint32_t> order;
    uint32_t max_leaf = OM_BVH_MAX_LEAF, leaf_force = OM_BVH_LEAF_FORCE;

    uint32_t emit(const Box& b) {
        OmBvhNode n;
        for (int i = 0; i < 3; ++i) {
            n.lo[i] = std::nextafter((float)b.lo[i], -INFINITY);
            n.hi[i] = std::nextafter((float)b.hi[i], INFINITY);
        }
        n.left = 0; n.right = 0;
        nodes.push_back(n);
        return (uint32_t)(nodes.size() - 1);
    }

    // builds items[begin,end) ; returns node index
    // SAH down to depth kSahDepth, then median splits: depth <= kSahDepth + log2(n)
    // keeps every tree within the traversal stacks (24 entries, 64 for the global BVH).
    static constexpr uint32_t kSahDepth = 10;
    uint32_t build(uint32_t begin, uint32_t end, uint32_t depth = 0) {
        Box bb; bb.empty(); Box cb; cb.empty();
        for (uint32_t i = begin; i < end; ++i) { bb.grow(items[i].b); cb.grow_pt(items[i].c); }
        const uint32_t node = emit(bb);
        const uint32_t count = end - begin;
        auto make_leaf = [&]() {
            nodes[node].left = -(int32_t)(order.size() + 1);
            nodes[node].right = (int32_t)count;
            for (uint32_t i = begin; i < end; ++i) order.push_back(items[i].gi);
            return node;
        };
        if (count <= leaf_force) return make_leaf();
        // binned SAH over the centroid box
        const int NB = 16;
        double best_cost = 1e300; int best_axis = -1; int best_bin = -1;
        for (int ax = 0; ax < 3; ++ax) {
            const double lo = cb.lo[ax], hi = cb.hi[ax];
            if (!(hi - lo > 1e-12)) continue;
            Box bins[NB]; uint32_t cnt[NB] = {0};
            for (int k = 0; k < NB; ++k) bins[k].empty();
            for (uint32_t i = begin; i < end; ++i) {
                int k = (int)((items[i].c[ax] - lo) / (hi - lo) * NB);
                k = std::min(NB - 1, std::max(0, k));
                bins[k].grow(items[i].b); cnt[k]++;
            }
            Box lacc; lacc.empty(); uint32_t lc = 0;
            double la[NB]; uint32_t lcs[NB];
            for (int k = 0; k < NB - 1; ++k) { lacc.grow(bins[k]); lc += cnt[k]; la[k] = lacc.area(); lcs[k] = lc; }
            Box racc; racc.empty(); uint32_t rc = 0;
            for (int k = NB - 1; k > 0; --k) {
                racc.grow(bins[k]); rc += cnt[k];
                const uint32_t lcount = lcs[k - 1];
                if (lcount == 0 || rc == 0) continue;
                const double cost = la[k - 1] * lcount + racc.area() * rc;
                if (cost < best_cost) { best_cost = cost; best_axis = ax; best_bin = k; }
            }
        }
        const double leaf_cost = bb.area() * count;
        // traversal cost relative to one primitive test (OM_BVH_TRAV); leaves <= OM_BVH_MAX_LEAF (r01:
        // a sweep of cost 0.3-2 and max leaf 2-8 moved C1 by < 1%; r05 re-check in DESIGN.md §10)
        const double trav = OM_BVH_TRAV * bb.area();
        if (best_axis < 0 || depth >= kSahDepth) {
            if (count <= std::min(4u, max_leaf) || (best_axis < 0 && count <= 8)) return make_leaf();
            // degenerate centroids: median split on the longest box axis
            int ax = 0;
            for (int k = 1; k < 3; ++k) if (bb.hi[k] - bb.lo[k] > bb.hi[ax] - bb.lo[ax]) ax = k;
            std::nth_element(items.begin() + begin, items.begin() + begin + count / 2, items.begin() + end,
                             [ax](const Item& x, const Item& y) { return x.c[ax] < y.c[ax]; });
            const uint32_t mid = begin + count / 2;
            const uint32_t l = build(begin, mid, depth + 1);
            const uint32_t r = build(mid, end, depth + 1);
            nodes[node].left = (int32_t)l; nodes[node].right = (int32_t)r;
            return node;
        }
        if (count <= max_leaf && leaf_cost <= best_cost + trav) return make_leaf();
        const int ax = best_axis;
        const double lo = cb.lo[ax], hi = cb.hi[ax];
        auto mid_it = std::partition(items.begin() + begin, items.begin() + end, [&](const Item& it) {
            int k = (int)((it.c[ax] - lo) / (hi - lo) * NB);
            k = std::min(NB - 1, std::max(0, k));
            return k < best_bin;
        });
        uint32_t mid = (uint32_t)(mid_it - items.begin());
        if (mid == begin || mid == end) mid = begin + count / 2;
        const uint32_t l = build(begin, mid, depth + 1);
        const uint32_t r = build(mid, end, depth + 1);
        nodes[node].left = (int32_t)l; nodes[node].right = (int32_t)r;
        return node;
    }
};

}  // namespace

// IEEE half bits -> the value, exactly (every half is a float).
float half_value(uint16_t h) {
    const int e = (h >> 10) & 31, m = h & 1023;
    const float v = e == 0 ? std::ldexp((float)m, -24) : e == 31 ? INFINITY : std::ldexp((float)(1024 + m), e - 25);
    return (h & 0x8000u) ? -v : v;
}

// The half-precision plane that contains x on the outside: the largest half <= x (up = false, a
// box's lo) or the smallest half >= x (up = true, its hi); +-inf beyond the half range.  Binary
// search over the halves in value order (key k >= 0: bits k; k < 0: the negative half -k).
uint16_t half_out(float x, bool up) {
    auto bits = [](int k) { return (uint16_t)(k >= 0 ? k : (0x8000 | -k)); };
    if (std::isnan(x)) return bits(up ? 0x7C00 : -0x7C00);
    int lo = -0x7C00, hi = 0x7C00;                       // -inf .. +inf
    if (!up) {                                           // largest k with value(k) <= x
        while (lo < hi) { const int mid = lo + (hi - lo + 1) / 2; if (half_value(bits(mid)) <= x) lo = mid; else hi = mid - 1; }
        return bits(lo);
    }
    while (lo < hi) { const int mid = lo + (hi - lo) / 2; if (half_value(bits(mid)) >= x) hi = mid; else lo = mid + 1; }
    return bits(lo);
}


void build_bvh(const om_world& w, FrozenWorld& fw) {
    Builder b;
    std::vector<uint32_t> always;
    const double kHuge = 100.0;  // a bound larger than this is tested outside the BVH
    auto add = [&](const Box& box, uint32_t gi) {
        double ext = 0.0;
        for (int i = 0; i < 3; ++i) ext = std::max(ext, box.hi[i] - box.lo[i]);
        if (ext > 2.0 * kHuge) { always.push_back(gi); return; }
        Item it; it.b = box; it.gi = gi;
        for (int i = 0; i < 3; ++i) it.c[i] = 0.5 * (box.lo[i] + box.hi[i]);
        b.items.push_back(it);
    };
    for (size_t i = 0; i < w.spheres.size(); ++i) add(affine_box(w.spheres[i].l2w, -1.0), fw.offsets[K_SPHERE] + (uint32_t)i);
    for (size_t i = 0; i < w.cubes.size(); ++i) add(affine_box(w.cubes[i].l2w, 0.5), fw.offsets[K_CUBE] + (uint32_t)i);
    for (size_t i = 0; i < w.triangles.size(); ++i) add(bary_box(w.triangles[i], false), fw.offsets[K_TRI] + (uint32_t)i);
    for (size_t i = 0; i < w.planes.size(); ++i) always.push_back(fw.offsets[K_PLANE] + (uint32_t)i);
    for (size_t i = 0; i < w.parallelograms.size(); ++i) add(bary_box(w.parallelograms[i], true), fw.offsets[K_PARA] + (uint32_t)i);
    std::sort(always.begin(), always.end());
    fw.always = always;
    if (!b.items.empty()) b.build(0, (uint32_t)b.items.size());
    fw.bvh = b.nodes;
    fw.bvh_prims = b.order;
    build_skip_bvh(w, fw);
}

// Stackless layout: the SAH tree over the affine primitives (spheres,
// cubes) re-emitted in depth-first order with a skip ("miss") link per node, and the
// primitives' test records copied in leaf order so a leaf owns a contiguous run.
// Everything else (planes, triangles, parallelograms, huge bounds) goes to always2.
void build_bvh4(FrozenWorld& fw);

void build_skip_bvh(const om_world& w, FrozenWorld& fw) {
    Builder b;
    std::vector<uint32_t> always;
    const double kHuge = 100.0;
    auto add = [&](const Box& box, uint32_t gi) {
        double ext = 0.0;
        for (int i = 0; i < 3; ++i) ext = std::max(ext, box.hi[i] - box.lo[i]);
        if (ext > 2.0 * kHuge) { always.push_back(gi); return; }
        Item it; it.b = box; it.gi = gi;
        for (int i = 0; i < 3; ++i) it.c[i] = 0.5 * (box.lo[i] + box.hi[i]);
        b.items.push_back(it);
    };
    for (size_t i = 0; i < w.spheres.size(); ++i) add(affine_box(w.spheres[i].l2w, -1.0), fw.offsets[K_SPHERE] + (uint32_t)i);
    for (size_t i = 0; i < w.cubes.size(); ++i) add(affine_box(w.cubes[i].l2w, 0.5), fw.offsets[K_CUBE] + (uint32_t)i);
    for (size_t i = 0; i < w.triangles.size(); ++i) always.push_back(fw.offsets[K_TRI] + (uint32_t)i);
    for (size_t i = 0; i < w.planes.size(); ++i) always.push_back(fw.offsets[K_PLANE] + (uint32_t)i);
    for (size_t i = 0; i < w.parallelograms.size(); ++i) always.push_back(fw.offsets[K_PARA] + (uint32_t)i);
    std::sort(always.begin(), always.end());
    fw.always2 = always;
    fw.always2_rec.clear();
    for (uint32_t gi : always) {
        OmAlwaysRec r;
        r.gi = gi; r.pad = 0;
        if (gi < fw.offsets[K_SPHERE + 1]) {      // axis-aligned sphere: every off-diagonal entry of W2L is +-0
            const float* m = fw.sph_test[gi - fw.offsets[K_SPHERE]].w2l;
            if (m[1] == 0.0f && m[2] == 0.0f && m[4] == 0.0f && m[6] == 0.0f && m[8] == 0.0f && m[9] == 0.0f)
                r.pad = OM_ALWAYS_DIAG_SPHERE;
        }
        Box bx;
        bool bounded = true;
        if (gi >= fw.offsets[K_TRI] && gi < fw.offsets[K_TRI + 1]) bx = bary_box(w.triangles[gi - fw.offsets[K_TRI]], false);
        else if (gi >= fw.offsets[K_PARA] && gi < fw.offsets[K_PARA + 1]) bx = bary_box(w.parallelograms[gi - fw.offsets[K_PARA]], true);
        else bounded = false;   // planes; huge spheres/cubes (their inflation would cover the scene)
        for (int i = 0; i < 3; ++i) {
            r.lo[i] = bounded ? std::nextafter((float)bx.lo[i], -INFINITY) : -INFINITY;
            r.hi[i] = bounded ? std::nextafter((float)bx.hi[i], INFINITY) : INFINITY;
        }
        fw.always2_rec.push_back(r);
    }
    fw.snodes.clear();
    fw.srecs.clear();
    if (b.items.empty()) return;
    uint32_t root = b.build(0, (uint32_t)b.items.size());
    // internal nodes, leaves, and internal nodes on the deepest root-to-leaf path (the compressed
    // tree's lane-stack bound, fw.b2_depth below) of the built tree
    auto tree_stats = [&](uint32_t r, size_t& internal, size_t& leaves, uint32_t& tdepth) {
        internal = 0; leaves = 0; tdepth = 0;
        std::vector<std::pair<uint32_t, uint32_t>> st{{r, 1u}};
        while (!st.empty()) {
            const auto [n, d] = st.back();
            st.pop_back();
            const OmBvhNode& nd = b.nodes[n];
            if (nd.left < 0) { ++leaves; continue; }
            ++internal; tdepth = std::max(tdepth, d);
            st.push_back({(uint32_t)nd.left, d + 1u}); st.push_back({(uint32_t)nd.right, d + 1u});
        }
    };
    size_t internal, leaves;
    uint32_t tdepth;
    tree_stats(root, internal, leaves, tdepth);
    if (internal * sizeof(OmBvh2Node) + leaves * 4u > kB2LdsBudget) {    // read through L2: smaller leaves
        std::vector<OmBvhNode> nodes8;
        std::vector<uint32_t> order8;
        nodes8.swap(b.nodes); order8.swap(b.order);
        const uint32_t root8 = root;
        b.max_leaf = OM_BVH_MAX_LEAF_L2; b.leaf_force = OM_BVH_LEAF_FORCE_L2;
        root = b.build(0, (uint32_t)b.items.size());
        tree_stats(root, internal, leaves, tdepth);
        // the compressed BVH2 needs 15-bit node and leaf codes and a lane stack of <= 24 entries
        // (om_upload_world's b2_ok): one record per leaf gives one leaf per bounded primitive, which
        // breaks those limits from ~32k primitives on -- keep the max-leaf tree then
        if (!(internal < 32768u && leaves < 32768u && tdepth <= 24u)) {
            b.nodes.swap(nodes8); b.order.swap(order8);
            root = root8;
        }
    }
    // depth-first re-emission with skip links
    std::vector<uint32_t> leaf_first(b.nodes.size(), 0);
    struct Emit {
        const Builder& b; const FrozenWorld& fw; std::vector<OmSkipNode>& out; std::vector<OmAffineTest>& recs;
        std::vector<uint32_t>& leaf_first;
        void rec(uint32_t n) {
            const OmBvhNode& src = b.nodes[n];
            const uint32_t idx = (uint32_t)out.size();
            OmSkipNode o;
            for (int i = 0; i < 3; ++i) { o.lo[i] = src.lo[i]; o.hi[i] = src.hi[i]; }
            o.skip = 0; o.leaf = 0xFFFFFFFFu;
            out.push_back(o);
            if (src.left < 0) {
                const uint32_t first = (uint32_t)(-src.left - 1), cnt = (uint32_t)src.right;
                out[idx].leaf = ((uint32_t)recs.size() << 8) | cnt;
                leaf_first[n] = (uint32_t)recs.size();
                for (uint32_t k = 0; k < cnt; ++k) {
                    const uint32_t gi = b.order[first + k];
                    const bool cube = gi >= fw.offsets[K_CUBE];
                    OmAffineTest t = cube ? fw.cube_test[gi - fw.offsets[K_CUBE]] : fw.sph_test[gi];
                    const uint32_t tag = gi | (cube ? 0x80000000u : 0u);
                    std::memcpy(&t.pad, &tag, 4);
                    recs.push_back(t);
                }
            } else {
                rec((uint32_t)src.left);
                rec((uint32_t)src.right);
            }
            out[idx].skip = (uint32_t)out.size();
        }
    } e{b, fw, fw.snodes, fw.srecs, leaf_first};
    e.rec(root);

    // compressed BVH2: both child boxes in the parent (one 64-B read per visit), emitted
    // breadth-first so the top levels, which every ray visits, are the first nodes: a tree
    // too big for LDS stages that prefix there (om_wavefront.hip, OM_WF_HYB_BYTES).
    // direct leaf codes: when every record index fits 11 bits and every leaf holds
    // at most 15 records (S-traced: 485 records, leaves <= 8), a leaf child's 16-bit code is
    // OM_LEAF | first << 4 | count, so the traversal needs no leaf-table read to enter a leaf;
    // the table is still emitted (same order) for the other consumers.
    // (both conditions checked here, not assumed from the builder's leaf cap: a count above 15
    // would spill into the `first` bits)
    int32_t max_leaf = 0;
    for (const OmBvhNode& n : b.nodes)
        if (n.left < 0) max_leaf = std::max(max_leaf, n.right);
    const bool direct = fw.srecs.size() < 2048u && max_leaf <= 15;
    struct Emit2 {
        const Builder& b; const std::vector<uint32_t>& leaf_first; std::vector<OmBvh2Node>& out;
        std::vector<uint32_t>& leaves;
        bool direct;
        std::vector<std::pair<uint32_t, uint32_t>> q;   // (builder node, output index)
        uint32_t code(uint32_t c) {
            const OmBvhNode& n = b.nodes[c];
            if (n.left < 0) {
                leaves.push_back((leaf_first[c] << 8) | (uint32_t)n.right);
                if (direct) return OM_LEAF | (leaf_first[c] << 4) | (uint32_t)n.right;
                return OM_LEAF | (uint32_t)(leaves.size() - 1);
            }
            out.push_back(OmBvh2Node{});
            q.emplace_back(c, (uint32_t)(out.size() - 1));
            return (uint32_t)(out.size() - 1);
        }
        void rec(uint32_t root) {
            out.push_back(OmBvh2Node{});
            q.emplace_back(root, 0u);
            for (size_t h = 0; h < q.size(); ++h) {
                const uint32_t n = q[h].first, idx = q[h].second;
                const OmBvhNode& src = b.nodes[n];
                const OmBvhNode& L = b.nodes[(uint32_t)src.left];
                const OmBvhNode& R = b.nodes[(uint32_t)src.right];
                OmBvh2Node o{};
                for (int i = 0; i < 3; ++i) {
                    OM_B2_LO(o, 0, i) = L.lo[i]; OM_B2_HI(o, 0, i) = L.hi[i];
                    OM_B2_LO(o, 1, i) = R.lo[i]; OM_B2_HI(o, 1, i) = R.hi[i];
                }
                o.c0 = code((uint32_t)src.left);
                o.c1 = code((uint32_t)src.right);
                out[idx] = o;
            }
        }
    } e2{b, leaf_first, fw.b2nodes, fw.b2leaves, direct, {}};
    fw.b2nodes.clear();
    fw.b2leaves.clear();
    if (b.nodes[root].left < 0) {            // a single leaf: one node, second child an empty leaf
        OmBvh2Node o{};
        for (int i = 0; i < 3; ++i) {
            OM_B2_LO(o, 0, i) = b.nodes[root].lo[i]; OM_B2_HI(o, 0, i) = b.nodes[root].hi[i];
            OM_B2_LO(o, 1, i) = INFINITY; OM_B2_HI(o, 1, i) = -INFINITY;
        }
        fw.b2leaves.push_back((leaf_first[root] << 8) | (uint32_t)b.nodes[root].right);
        fw.b2leaves.push_back(0u);
        o.c0 = direct ? (OM_LEAF | (leaf_first[root] << 4) | (uint32_t)b.nodes[root].right) : (OM_LEAF | 0u);
        o.c1 = direct ? OM_LEAF : (OM_LEAF | 1u);          // empty leaf: no records
        fw.b2nodes.push_back(o);
    } else {
        e2.rec(root);
    }
    fw.b2_direct = direct ? 1u : 0u;
    fw.b2h.clear();
    for (const OmBvh2Node& n : fw.b2nodes) {
        OmBvh2NodeH h{};
        for (int i = 0; i < 3; ++i) {
            h.b[i] = half_out(OM_B2_LO(n, 0, i), false); h.b[3 + i] = half_out(OM_B2_HI(n, 0, i), true);
            h.b[6 + i] = half_out(OM_B2_LO(n, 1, i), false); h.b[9 + i] = half_out(OM_B2_HI(n, 1, i), true);
        }
        h.c0 = (uint16_t)n.c0; h.c1 = (uint16_t)n.c1; h.pad = 0u;
        fw.b2h.push_back(h);
    }
    // depth of the compressed tree (the traversal's stack bound)
    std::vector<uint32_t> depth(fw.b2nodes.size(), 1);
    fw.b2_depth = 1;
    for (uint32_t i = 0; i < fw.b2nodes.size(); ++i) {   // parents precede children (BFS)
        for (uint32_t c : {fw.b2nodes[i].c0, fw.b2nodes[i].c1})
            if (!(c & OM_LEAF)) { depth[c] = depth[i] + 1; fw.b2_depth = std::max(fw.b2_depth, depth[c]); }
    }
    // conservative world box of every leaf record (the tree's own item boxes)
    fw.srec_box.clear();
    for (const OmAffineTest& t : fw.srecs) {
        uint32_t tag;
        std::memcpy(&tag, &t.pad, 4);
        const uint32_t gi = tag & 0x7FFFFFFFu;
        const Box bx = (tag >> 31) ? affine_box(w.cubes[gi - fw.offsets[K_CUBE]].l2w, 0.5)
                                   : affine_box(w.spheres[gi].l2w, -1.0);
        for (int i = 0; i < 3; ++i) fw.srec_box.push_back(std::nextafter((float)bx.lo[i], -INFINITY));
        for (int i = 0; i < 3; ++i) fw.srec_box.push_back(std::nextafter((float)bx.hi[i], INFINITY));
    }
    build_bvh4(fw);
}

// BVH4: each wide node takes its BVH2 node's two children and keeps
// replacing the internal child of largest surface area by that child's two children, up
// to four.  Child boxes are the BVH2's (already conservative), so culling stays exact.
void build_bvh4(FrozenWorld& fw) {
    fw.b4nodes.clear();
    fw.b4_depth = 0;
    if (fw.b2nodes.empty()) return;
    struct Ch { uint32_t code; float lo[3], hi[3]; };
    auto kids = [&](uint32_t n, Ch* out) {
        const OmBvh2Node& N = fw.b2nodes[n];
        out[0].code = N.c0; out[1].code = N.c1;
        for (int i = 0; i < 3; ++i) {
            out[0].lo[i] = OM_B2_LO(N, 0, i); out[0].hi[i] = OM_B2_HI(N, 0, i);
            out[1].lo[i] = OM_B2_LO(N, 1, i); out[1].hi[i] = OM_B2_HI(N, 1, i);
        }
    };
    auto area = [](const Ch& c) {
        const double dx = std::max(0.0, (double)c.hi[0] - c.lo[0]), dy = std::max(0.0, (double)c.hi[1] - c.lo[1]),
                     dz = std::max(0.0, (double)c.hi[2] - c.lo[2]);
        return dx * dy + dy * dz + dz * dx;
    };
    struct Rec {
        FrozenWorld& fw; decltype(kids)& kids_of; decltype(area)& area_of;
        uint32_t go(uint32_t n2, uint32_t depth) {
            std::vector<Ch> ch(2);
            kids_of(n2, ch.data());
            while (ch.size() < 4) {
                int best = -1; double ba = -1.0;
                for (size_t i = 0; i < ch.size(); ++i)
                    if (!(ch[i].code & OM_LEAF) && area_of(ch[i]) > ba) { ba = area_of(ch[i]); best = (int)i; }
                if (best < 0) break;
                Ch two[2];
                kids_of(ch[best].code, two);
                ch[best] = two[0];
                ch.insert(ch.begin() + best + 1, two[1]);
            }
            const uint32_t idx = (uint32_t)fw.b4nodes.size();
            fw.b4nodes.push_back(OmBvh4Node{});
            fw.b4_depth = std::max(fw.b4_depth, depth);
            OmBvh4Node o{};
            for (int k = 0; k < 4; ++k) {
                if (k < (int)ch.size()) {
                    o.lox[k] = ch[k].lo[0]; o.loy[k] = ch[k].lo[1]; o.loz[k] = ch[k].lo[2];
                    o.hix[k] = ch[k].hi[0]; o.hiy[k] = ch[k].hi[1]; o.hiz[k] = ch[k].hi[2];
                    o.child[k] = (uint16_t)((ch[k].code & OM_LEAF) ? ch[k].code : go(ch[k].code, depth + 1));
                } else {
                    o.lox[k] = o.loy[k] = o.loz[k] = o.hix[k] = o.hiy[k] = o.hiz[k] = 0.0f;
                    o.child[k] = (uint16_t)OM_EMPTY;
                }
            }
            fw.b4nodes[idx] = o;
            return idx;
        }
    } r{fw, kids, area};
    r.go(0, 1);
    // breadth-first renumbering with half-precision planes (trees read through L2, §5.7)
    fw.b4h.clear();
    std::vector<uint32_t> order{0u}, pos(fw.b4nodes.size(), 0u);
    for (size_t h = 0; h < order.size(); ++h)
        for (uint16_t c : fw.b4nodes[order[h]].child)
            if (c != OM_EMPTY && !(c & OM_LEAF)) { pos[c] = (uint32_t)order.size(); order.push_back(c); }
    for (uint32_t n : order) {
        const OmBvh4Node& N = fw.b4nodes[n];
        OmBvh4NodeH o{};
        for (int k = 0; k < 4; ++k) {
            o.b[k] = half_out(N.lox[k], false); o.b[4 + k] = half_out(N.loy[k], false); o.b[8 + k] = half_out(N.loz[k], false);
            o.b[12 + k] = half_out(N.hix[k], true); o.b[16 + k] = half_out(N.hiy[k], true); o.b[20 + k] = half_out(N.hiz[k], true);
            const uint16_t c = N.child[k];
            o.child[k] = (c == OM_EMPTY || (c & OM_LEAF)) ? c : (uint16_t)pos[c];
        }
        fw.b4h.push_back(o);
    }
}

}  // namespace om
