// host_sanitize.cpp — drives the product's host C++ (om_world.cpp scene builders and freeze,
// om_bvh.cpp BVH/SBVH/BVH2/BVH4 builders, om_tiles.cpp primary-ray tile lists, om_multi.hip's
// host-side tile deal) and the CPU oracle (a small render of each scene) under ASan/UBSan.
// Built by `make -C tests/cpp sanitize` with -fsanitize=address,undefined (host code only, no
// device code: the library's GPU kernels are not part of this binary), run by
// tests/test_host_sanitize.py.  Any report aborts with a non-zero status.
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../raytracingoneweekend_amd/csrc/om_bvh.h"

#include "../../raytracingoneweekend_amd/csrc/om_shard.h"
#include "../../raytracingoneweekend_amd/csrc/om_tiles.h"
#include "../../raytracingoneweekend_amd/csrc/om_world.h"

// om_shard.cpp reports errors through om_render.hip's error channel, which is device-side
// code and not in this host-only binary: the test records the last message instead
namespace omi {
static std::string g_last;
om_status global_error(om_status code, const std::string& msg) { g_last = msg; return code; }
}

extern "C" {   // the oracle's C API (oracle/om_oracle.cpp), with its structs as there
struct OroCamera { float origin[3], horizontal[3], vertical[3], llc[3], u[3], v[3], w[3]; float lens_radius, aspect, focus, vw, vh; };
struct OroParams {
    uint32_t width, height, spp_total, sample_begin, sample_count, max_depth;
    float tmin, tmax;
    uint32_t march_steps, adaptive;
    uint64_t seed;
};
void* oro_world_new();
void oro_world_free(void* w);
void oro_world_random_scene(void* wp, uint64_t seed, uint32_t flags, int32_t grid_half);
void oro_world_marched_scene(void* wp);
void oro_camera_new(const float* lookfrom, const float* lookat, const float* vup, float vfov, float aspect,
                    float aperture, float focus, OroCamera* out);
void oro_render(void* wp, const OroCamera* c, const OroParams* p, void* stats_v, int32_t nthreads, uint64_t* counters);
void oro_render_pixels(void* wp, const OroCamera* c, const OroParams* p, void* stats_v, const uint32_t* pixels, uint32_t n);
}

static int g_fail = 0;
#define EXPECT(c) do { if (!(c)) { std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++g_fail; } } while (0)

struct Cam { float from[3], at[3], vup[3], vfov, aperture, focus; };

// The half-precision BVH2 planes (OmBvh2NodeH, om_bvh.cpp) must round every f32 plane OUTWARD, or
// an L2-resident tree could cull a box the exact test would hit: for every x,
// value(half_out(x, lo)) <= x <= value(half_out(x, hi)), tight (neighbouring halves, or x itself
// when x is a half), NaN -> the infinite planes, beyond +-65504 -> +-inf on the outer side.
static int half_key(uint16_t h) { return (h & 0x8000u) ? -(int)(h & 0x7FFFu) : (int)h; }
static void check_half_plane(float x) {
    const uint16_t hl = om::half_out(x, false), hh = om::half_out(x, true);
    const float lo = om::half_value(hl), hi = om::half_value(hh);
    if (std::isnan(x)) { EXPECT(lo == -INFINITY && hi == INFINITY); return; }
    EXPECT(lo <= x && x <= hi);
    if (lo == x) { EXPECT(hi == x); return; }
    EXPECT(half_key(hh) == half_key(hl) + 1 || (half_key(hl) == 0 && half_key(hh) == 1));
}
static void half_plane_sweep() {
    std::vector<float> xs = {0.0f, -0.0f, INFINITY, -INFINITY, NAN, -NAN, FLT_MAX, -FLT_MAX, FLT_MIN, -FLT_MIN,
                             1e-45f, -1e-45f, 65504.0f, -65504.0f, 65519.0f, 65520.0f, -65520.0f, 1e30f, -1e30f,
                             5.96e-8f, 2.98e-8f, -2.98e-8f, 6.1e-5f, 1.0f, -1.0f, 1000.5f, -999.999f};
    for (uint32_t h = 0; h < 0x10000u; ++h) {               // every half, and its f32 neighbours
        const float v = om::half_value((uint16_t)h);
        if (std::isinf(v)) continue;
        xs.push_back(v); xs.push_back(std::nextafter(v, INFINITY)); xs.push_back(std::nextafter(v, -INFINITY));
    }
    uint64_t z = 0x9E3779B97F4A7C15ull;                       // random f32 bit patterns
    for (int i = 0; i < 400000; ++i) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t b = (uint32_t)(z >> 32);
        float x;
        std::memcpy(&x, &b, 4);
        xs.push_back(x);
        xs.push_back(std::ldexp((float)(b & 0xFFFFFF) / 16777216.0f - 0.5f, (int)(b >> 27) - 10));   // |x| ~ 2^-11..2^21
    }
    for (float x : xs) check_half_plane(x);
    // an empty box (lo = +inf, hi = -inf) stays empty
    EXPECT(om::half_value(om::half_out(INFINITY, false)) == INFINITY && om::half_value(om::half_out(-INFINITY, true)) == -INFINITY);
    std::printf("half planes: %zu values round outward\n", xs.size());
}

// The half-precision BVH4 (om_bvh.cpp build_bvh4): breadth-first (every internal child after its
// parent, the root first), the same child codes as the f32 tree walked in step, and every half
// box containing its f32 box (planes rounded outward), so the L2 tree culls conservatively.
static void check_b4h(const om::FrozenWorld& fw) {
    EXPECT(fw.b4h.size() == fw.b4nodes.size());
    if (fw.b4nodes.empty()) return;
    std::vector<std::pair<uint32_t, uint32_t>> q{{0u, 0u}};   // (f32 DFS node, half BFS node)
    std::vector<uint32_t> seen(fw.b4h.size(), 0);
    for (size_t h = 0; h < q.size(); ++h) {
        const OmBvh4Node& F = fw.b4nodes[q[h].first];
        const OmBvh4NodeH& N = fw.b4h[q[h].second];
        seen[q[h].second]++;
        for (int k = 0; k < 4; ++k) {
            const uint16_t cf = F.child[k], ch = N.child[k];
            EXPECT((cf == OM_EMPTY) == (ch == OM_EMPTY));
            if (cf == OM_EMPTY) continue;
            const float f[6] = {F.lox[k], F.loy[k], F.loz[k], F.hix[k], F.hiy[k], F.hiz[k]};
            for (int a = 0; a < 3; ++a) {
                EXPECT(om::half_value(N.b[a * 4 + k]) <= f[a]);
                EXPECT(om::half_value(N.b[(3 + a) * 4 + k]) >= f[3 + a]);
            }
            if (cf & OM_LEAF) { EXPECT(ch == cf); continue; }
            EXPECT(!(ch & OM_LEAF) && ch > q[h].second && ch < fw.b4h.size());
            q.emplace_back(cf, ch);
        }
    }
    for (uint32_t v : seen) EXPECT(v == 1u);
}

int main() {
    half_plane_sweep();
    const Cam cams[] = {
        {{13.f, 2.f, 3.f}, {0.f, 0.f, 0.f}, {0.f, 1.f, 0.f}, 20.f, 0.1f, 10.f},          // main.rs:136-142
        {{0.3f, 0.35f, 0.2f}, {5.f, 0.2f, 2.f}, {0.f, 1.f, 0.f}, 70.f, 1.5f, 2.f},         // wide lens inside the field
    };
    const uint32_t sizes[][2] = {{1920, 1080}, {53, 37}, {1, 1}, {8, 8}};
    struct Scene { const char* name; int kind; uint32_t flags; int32_t grid; };
    const Scene scenes[] = {{"S-traced", 0, 0u, 11}, {"S-full", 0, 1u, 11}, {"S-10k", 0, 2u, 50},
                            {"S-marched", 1, 0u, 0}, {"basic", 2, 0u, 0}};
    for (const Scene& sc : scenes) {
        om_world* w = nullptr;
        EXPECT(om_world_create(&w) == OM_OK);
        if (sc.kind == 0) EXPECT(om_world_random_scene(w, 0x5EED, sc.flags, sc.grid) == OM_OK);
        else if (sc.kind == 1) EXPECT(om_world_marched_scene(w) == OM_OK);
        else EXPECT(om_world_basic_scene(w) == OM_OK);
        om::FrozenWorld fw;
        w->freeze(fw);                                          // BVH, SBVH, BVH2, BVH4 builders
        EXPECT(fw.offsets[8] > 0);
        check_b4h(fw);
        size_t lists = 0;
        for (const Cam& c : cams)
            for (const auto& sz : sizes) {
                om_camera cam;
                EXPECT(om_camera_new(c.from, c.at, c.vup, c.vfov, (float)sz[0] / (float)sz[1], c.aperture, c.focus, &cam) == OM_OK);
                omt::TileLists tl;
                if (omt::build(fw.srec_box, cam, sz[0], sz[1], tl)) {
                    EXPECT(tl.off.size() == (size_t)((sz[0] + 7) / 8) * ((sz[1] + 7) / 8) + 1);
                    EXPECT(tl.off.back() == tl.idx.size());
                    lists += tl.idx.size();
                }
            }
        std::printf("%s: %u prims, %zu BVH2 nodes, %zu tile-list entries\n", sc.name, fw.offsets[8], fw.b2nodes.size(), lists);
        om_world_destroy(w);
    }
    // a field of 40k spheres: one record per leaf would give ~40k leaves, past the compressed
    // BVH2's 15-bit codes, so the builder must keep a tree om_upload_world accepts
    {
        om_world* w = nullptr;
        EXPECT(om_world_create(&w) == OM_OK);
        EXPECT(om_world_random_scene(w, 0x5EED, 2u, 100) == OM_OK);
        om::FrozenWorld fw;
        w->freeze(fw);
        EXPECT(fw.offsets[8] >= 39000u);
        EXPECT(!fw.b2nodes.empty() && fw.b2nodes.size() < 32768u && fw.b2leaves.size() < 32768u && fw.b2_depth <= 24u);
        std::printf("S-40k: %u prims, %zu BVH2 nodes, %zu leaves, depth %u\n", fw.offsets[8], fw.b2nodes.size(),
                    fw.b2leaves.size(), fw.b2_depth);
        om_world_destroy(w);
    }
    // the tile deal of the multi-GPU path (om_multi.hip host side)
    for (uint32_t n : {1u, 2u, 3u, 8u}) {
        const uint32_t W = 37, H = 21, cap = om_shard_capacity(W, H, n);
        std::vector<uint32_t> seen(W * H, 0), lst(cap);
        std::vector<std::vector<om_pixel_stats>> shards(n);
        for (uint32_t r = 0; r < n; ++r) {
            uint32_t got = 0;
            EXPECT(om_shard_pixels(W, H, r, n, lst.data(), cap, &got) == OM_OK);
            shards[r].resize(got);
            for (uint32_t k = 0; k < got; ++k) { seen[lst[k]]++; shards[r][k].n = lst[k]; }
        }
        for (uint32_t v : seen) EXPECT(v == 1u);
        std::vector<const om_pixel_stats*> ptrs;
        for (auto& s : shards) ptrs.push_back(s.data());
        std::vector<om_pixel_stats> frame(W * H);
        EXPECT(om_shard_assemble_host(W, H, n, ptrs.data(), frame.data()) == OM_OK);
        for (uint32_t p = 0; p < W * H; ++p) EXPECT(frame[p].n == p);
    }
    // the oracle: a small frame of every scene, all threads, plus a pixel list
    for (const Scene& sc : scenes) {
        if (sc.kind == 2) continue;
        void* ow = oro_world_new();
        if (sc.kind == 0) oro_world_random_scene(ow, 0x5EED, sc.flags, sc.grid);
        else oro_world_marched_scene(ow);
        OroCamera oc;
        const float from[3] = {13.f, 2.f, 3.f}, at[3] = {0.f, 0.f, 0.f}, vup[3] = {0.f, 1.f, 0.f};
        const uint32_t W = 24, H = 16;
        oro_camera_new(from, at, vup, 20.f, (float)W / H, 0.1f, 10.f, &oc);
        OroParams p{W, H, 3, 0, 3, 50, 0.001f, 100.f, 256, 1, 5};
        std::vector<om_pixel_stats> st(W * H);
        uint64_t ctr[3] = {0, 0, 0};
        oro_render(ow, &oc, &p, st.data(), 3, ctr);
        EXPECT(ctr[0] > 0);
        const uint32_t px[3] = {0, W * H / 2, W * H - 1};
        std::vector<om_pixel_stats> sp(3);
        oro_render_pixels(ow, &oc, &p, sp.data(), px, 3);
        oro_world_free(ow);
    }
    if (g_fail == 0) std::printf("sanitize ok\n");
    return g_fail == 0 ? 0 : 1;
}
