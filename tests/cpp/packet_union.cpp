// packet_union.cpp — the case against a wave-coherent (packet) BVH2 traversal for bounce 1
// (VERDICT r05 #1c), measured on the product's own S-traced BVH2 (om_bvh.cpp).
//
// A wave of the bounce kernel traces 64 rays that leave one 8x8 tile's primary hits.  Traversed
// per ray (the shipped kernel), the node loop runs about as many iterations as its busiest lane
// needs; a packet traversal visits every node any lane needs, once per wave.  This program
// builds those bounce-1 rays on the host -- primary rays through pixel centres of the main.rs
// camera, their closest hit among the ellipsoids (the tree's leaf records) and the ground, a
// Lambertian bounce (n + unit sphere vector, materials.rs:52-61) as the most common scatter --
// traverses the BVH2 near-first per ray with closest-hit culling, and prints per tile: the busiest
// lane's node visits and leaf visits against the union over the tile's rays.  Host code only, an
// estimate: metal and glass bounces are more coherent, cubes and triangles are left out.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <set>
#include <vector>

#include "../../raytracingoneweekend_amd/csrc/om_world.h"
#include "ottomarcher.h"

namespace {

struct V { double x, y, z; };
V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V operator*(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
V unit(V a) { return a * (1.0 / std::sqrt(dot(a, a))); }

// closest t in (tmin, tmax] of the unit sphere in the record's local frame (W2L rows 3x4)
bool ellipsoid(const OmAffineTest& R, V o, V d, double tmin, double tmax, double& t, V& n) {
    const float* m = R.w2l;
    const V lo = {m[0] * o.x + m[1] * o.y + m[2] * o.z + m[3], m[4] * o.x + m[5] * o.y + m[6] * o.z + m[7],
                  m[8] * o.x + m[9] * o.y + m[10] * o.z + m[11]};
    const V ld = {m[0] * d.x + m[1] * d.y + m[2] * d.z, m[4] * d.x + m[5] * d.y + m[6] * d.z,
                  m[8] * d.x + m[9] * d.y + m[10] * d.z};
    const double a = dot(ld, ld), hb = dot(lo, ld), c = dot(lo, lo) - 1.0, disc = hb * hb - a * c;
    if (disc < 0) return false;
    const double sq = std::sqrt(disc);
    double r = (-hb - sq) / a;
    if (r <= tmin || r > tmax) { r = (-hb + sq) / a; if (r <= tmin || r > tmax) return false; }
    t = r;
    const V lp = lo + ld * r;                                     // gradient of |W2L p|^2: W2L^T lp
    n = unit({m[0] * lp.x + m[4] * lp.y + m[8] * lp.z, m[1] * lp.x + m[5] * lp.y + m[9] * lp.z,
              m[2] * lp.x + m[6] * lp.y + m[10] * lp.z});
    return true;
}

struct Trav { std::set<uint32_t> nodes, leaves; uint32_t node_visits = 0, leaf_visits = 0; };

// near-first BVH2 traversal with closest-hit culling over the leaf records; records visits
double trace(const om::FrozenWorld& fw, V o, V d, double tmax, Trav* tv, V* nrm) {
    double closest = tmax, t;
    V n{0, 1, 0};
    auto leaf = [&](uint32_t code) {
        const uint32_t first = fw.b2_direct ? ((code >> 4) & 0x7FFu) : fw.b2leaves[code & 0x7FFFu] >> 8;
        const uint32_t cnt = fw.b2_direct ? (code & 15u) : fw.b2leaves[code & 0x7FFFu] & 255u;
        if (tv) { tv->leaf_visits++; tv->leaves.insert(code); }
        for (uint32_t k = 0; k < cnt; ++k) {
            uint32_t tag;
            std::memcpy(&tag, &fw.srecs[first + k].pad, 4);
            if (tag >> 31) continue;                              // the cube: left out
            V nn;
            if (ellipsoid(fw.srecs[first + k], o, d, 1e-3, closest, t, nn)) { closest = t; n = nn; }
        }
    };
    // the ground (the first sphere, outside the tree, tested first as always2 is)
    V gn;
    if (ellipsoid(fw.sph_test[0], o, d, 1e-3, closest, t, gn)) { closest = t; n = gn; }
    auto slab = [&](const float* lo, const float* hi, double& near) {
        double t0 = 1e-3 * 0.5 - 1e-3, t1 = closest * 1.0001 + 1e-3;
        const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
        for (int a = 0; a < 3; ++a) {
            const double inv = 1.0 / (std::fabs(dd[a]) > 1e-20 ? dd[a] : std::copysign(1e-20, dd[a]));
            double ta = (lo[a] - oo[a]) * inv, tb = (hi[a] - oo[a]) * inv;
            if (ta > tb) std::swap(ta, tb);
            t0 = std::max(t0, ta); t1 = std::min(t1, tb);
        }
        near = t0;
        return t0 <= t1;
    };
    std::vector<uint32_t> stk;
    uint32_t cur = 0;
    for (;;) {
        if (cur & OM_LEAF) {
            leaf(cur);
            if (stk.empty()) break;
            cur = stk.back(); stk.pop_back();
            continue;
        }
        const OmBvh2Node& N = fw.b2nodes[cur];
        if (tv) { tv->node_visits++; tv->nodes.insert(cur); }
        double n0, n1;
        const bool h0 = slab(N.lo0, N.hi0, n0), h1 = slab(N.lo1, N.hi1, n1);
        if (h0 && h1) {
            const bool swap = n1 < n0;
            stk.push_back(swap ? N.c0 : N.c1);
            cur = swap ? N.c1 : N.c0;
        } else if (h0 || h1) {
            cur = h0 ? N.c0 : N.c1;
        } else {
            if (stk.empty()) break;
            cur = stk.back(); stk.pop_back();
        }
    }
    if (nrm) *nrm = n;
    return closest;
}

}  // namespace

int main() {
    om_world* w = nullptr;
    if (om_world_create(&w) != OM_OK || om_world_random_scene(w, 0x5EED, 0u, 11) != OM_OK) return 1;
    om::FrozenWorld fw;
    w->freeze(fw);
    const int W = 1920, H = 1080;
    const V from{13, 2, 3}, at{0, 0, 0}, vup{0, 1, 0};                      // main.rs:136-142
    const double vh = 2.0 * std::tan(20.0 * M_PI / 360.0), vw = vh * W / H;
    const V ww = unit(from - at), uu = unit(cross(vup, ww)), vv = cross(ww, uu);
    const V horiz = uu * (10.0 * vw), vert = vv * (10.0 * vh);
    const V llc = from - horiz * 0.5 - vert * 0.5 - ww * 10.0;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    double sum_max_nodes = 0, sum_union_nodes = 0, sum_mean_nodes = 0, sum_max_leaves = 0, sum_union_leaves = 0;
    int tiles = 0;
    for (int ty = 0; ty < H / 8; ty += 5)
        for (int tx = 0; tx < W / 8; tx += 5) {
            std::set<uint32_t> un, ul;
            uint32_t mx = 0, ml = 0, tot = 0, rays = 0;
            for (int k = 0; k < 64; ++k) {
                const int i = tx * 8 + (k & 7), j = ty * 8 + (k >> 3);
                const V d0 = unit(llc + horiz * ((i + 0.5) / (W - 1)) + vert * (1.0 - (j + 0.5) / (H - 1)) - from);
                V n;
                const double t = trace(fw, from, d0, 100.0, nullptr, &n);
                if (!(t < 100.0)) continue;                                     // sky: no bounce 1
                const V p = from + d0 * t;
                V r;
                do { r = {U(rng), U(rng), U(rng)}; } while (dot(r, r) >= 1.0);
                const V d1 = unit(n + unit(r));
                Trav tv;
                trace(fw, p, d1, 100.0, &tv, nullptr);
                mx = std::max(mx, tv.node_visits); ml = std::max(ml, tv.leaf_visits); tot += tv.node_visits; ++rays;
                un.insert(tv.nodes.begin(), tv.nodes.end()); ul.insert(tv.leaves.begin(), tv.leaves.end());
            }
            if (rays < 32) continue;                                            // tiles mostly on objects
            sum_max_nodes += mx; sum_union_nodes += un.size(); sum_mean_nodes += (double)tot / rays;
            sum_max_leaves += ml; sum_union_leaves += ul.size();
            ++tiles;
        }
    std::printf("tiles %d: bounce-1 node visits per ray %.1f, busiest lane %.1f, packet union %.1f; "
                "leaf visits busiest lane %.1f, packet union %.1f (of %zu nodes)\n", tiles, sum_mean_nodes / tiles,
                sum_max_nodes / tiles, sum_union_nodes / tiles, sum_max_leaves / tiles, sum_union_leaves / tiles,
                fw.b2nodes.size());
    om_world_destroy(w);
    return 0;
}
