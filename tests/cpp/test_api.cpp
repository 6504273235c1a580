// test_api.cpp — tests of the C++ mirror API (include/ottomarcher.hpp), driven by
// tests/test_cpp_api.py.
//
//   test_api cpu                  scene composition through the API == the native builders,
//                                 bit for bit; error behaviour (no device calls)
//   test_api gpu OUT_FIXED OUT_ADAPTIVE
//                                 renders S-traced through main.rs's thread scheme and the
//                                 C++ render(); writes the raw om_pixel_stats bytes, which
//                                 the Python side compares with the CPU oracle
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "ottomarcher.hpp"
#include "random_scene.hpp"

using namespace ottomarcher;

static int g_fail = 0;
#define EXPECT(c)                                                                  \
    do {                                                                           \
        if (!(c)) { std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); ++g_fail; } \
    } while (0)

// Every frozen primitive of `a` and `b` (om_world_export) has identical bits.
static bool same_world(const HittableList& a, const HittableList& b) {
    uint32_t ca[8], cb[8];
    check(om_world_counts(a.handle(), ca));
    check(om_world_counts(b.handle(), cb));
    if (std::memcmp(ca, cb, sizeof ca) != 0) { std::fprintf(stderr, "counts differ\n"); return false; }
    struct K { int kind, slot, floats; };
    const K kinds[] = {{0, 0, 32}, {1, 1, 32}, {2, 2, 29}, {4, 4, 29}, {7, 7, 43}};
    for (const K& k : kinds) {
        for (uint32_t i = 0; i < ca[k.slot]; ++i) {
            std::vector<float> x(k.floats), y(k.floats);
            check(om_world_export(a.handle(), k.kind, i, x.data(), k.floats));
            check(om_world_export(b.handle(), k.kind, i, y.data(), k.floats));
            if (std::memcmp(x.data(), y.data(), k.floats * sizeof(float)) != 0) {
                std::fprintf(stderr, "kind %d index %u differs\n", k.kind, i);
                return false;
            }
        }
    }
    return true;
}

static HittableList native_random_scene(uint64_t seed, uint32_t flags, int grid_half) {
    HittableList w = HittableList::new_();
    check(om_world_random_scene(w.handle(), seed, flags, grid_half));
    return w;
}

static int run_cpu() {
    // main.rs:37-100 composed through the API == om_world_random_scene, incl. torus and the 10k grid
    EXPECT(same_world(random_scene(0x5EED, false), native_random_scene(0x5EED, 0, 11)));
    EXPECT(same_world(random_scene(0x5EED, true), native_random_scene(0x5EED, 1, 11)));
    EXPECT(same_world(random_scene(42, false, 50, false), native_random_scene(42, 2, 50)));
    {
        HittableList n = HittableList::new_();
        check(om_world_basic_scene(n.handle()));
        EXPECT(same_world(basic_scene(), n));
    }
    // a different seed gives a different scene (the comparison is not vacuous)
    EXPECT(!same_world(random_scene(1, false), native_random_scene(2, 0, 11)));

    // Camera::new_ (camera.rs:38-59) is the library's: world_camera == new_ with its arguments
    {
        const Camera a = Camera::world_camera(90.0f, 1.5f);
        const Camera b = Camera::new_(Point3(0, 0, 0), Point3(0, 0, -1), Vec3(0, 1, 0), 90.0f, 1.5f, 0.0f, 1.0f);
        EXPECT(std::memcmp(&a.raw, &b.raw, sizeof a.raw) == 0);
        EXPECT(a.raw.lens_radius == 0.0f);
    }
    // Mat4x4: m4x4!(ID) is neutral for ^, and fast_homogenous_inverse undoes a translation
    {
        const Mat4x4 t = m4x4::TR(1.0f, 2.0f, 3.0f);
        const Mat4x4 ti = (t ^ m4x4::ID()).fast_homogenous_inverse();
        const Mat4x4 id = t ^ ti;
        EXPECT(std::memcmp(id.e, m4x4::ID().e, sizeof id.e) == 0);
    }
    // error behaviour: a bad material throws Error(OM_ERR_INVALID) with om_last_error's text
    {
        HittableList w = HittableList::new_();
        Material bad = Material::new_lambertian(Color(1, 1, 1));
        bad.raw.type = 7;
        bool threw = false;
        try {
            w += Sphere::new_with_radius(Point3(0, 0, 0), 1.0f, bad);
        } catch (const Error& e) {
            threw = e.status == OM_ERR_INVALID && std::string(e.what()).find("invalid material") != std::string::npos;
        }
        EXPECT(threw);
        uint32_t c[8];
        check(om_world_counts(w.handle(), c));
        EXPECT(c[0] == 0);  // nothing was appended
        w += Sphere::new_with_radius(Point3(0, 0, 0), 1.0f, Material::new_dielectric(1.5f));
        w.clear();
        check(om_world_counts(w.handle(), c));
        EXPECT(c[0] == 0);
    }
    // moved-from lists are empty handles; the destination owns the world
    {
        HittableList a = random_scene(3, false);
        HittableList b = std::move(a);
        EXPECT(a.handle() == nullptr && b.handle() != nullptr);
    }
    // main.rs:172-189 chunk deal: 2730-pixel chunks round-robin, leftover to the next thread
    {
        const std::vector<uint32_t> t = assign_threads(10000, 3);
        EXPECT(t.size() == 10000 && t[0] == 0 && t[2729] == 0 && t[2730] == 1 && t[5460] == 2 && t[8190] == 0);
        EXPECT(t[9999] == 0);  // 10000 / 2730 = 3 chunks -> leftover goes to 3 % 3 = 0
    }
    if (g_fail == 0) std::printf("cpu ok\n");
    return g_fail == 0 ? 0 : 1;
}

// Renders W x H x spp of S-traced with main.rs's thread scheme; returns the credited samples.
static uint64_t render_threads(const Camera& cam, const FrozenHittableList& frozen, uint32_t W, uint32_t H, uint32_t spp,
                               std::vector<Pixel>& pixels, const RenderOptions& opt, uint32_t num_threads) {
    const std::vector<uint32_t> assigned = assign_threads(W * H, num_threads);
    std::atomic<uint64_t> atom{0};
    std::vector<std::thread> th;
    std::vector<std::string> err(num_threads);
    for (uint32_t i = 0; i < num_threads; ++i)
        th.emplace_back([&, i]() {
            try {
                render(cam, frozen, 50, 0.001f, 100.0f, spp, W, H, PixelsBox{&pixels}, i, assigned, atom, opt);
            } catch (const std::exception& e) {
                err[i] = e.what();
            }
        });
    for (auto& t : th) t.join();
    for (const auto& e : err)
        if (!e.empty()) { std::fprintf(stderr, "render: %s\n", e.c_str()); ++g_fail; }
    return atom.load();
}

static void write_raw(const char* path, const std::vector<Pixel>& px) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(px.data()), (std::streamsize)(px.size() * sizeof(Pixel)));
}

static int run_gpu(const char* out_fixed, const char* out_adaptive) {
    const uint32_t W = 48, H = 32;
    const Camera cam = default_camera((float)W / (float)H);
    HittableList world = random_scene(0x5EED, false);
    const FrozenHittableList frozen = world.freeze(cam);
    std::vector<Pixel> fixed(W * H);
    {   // fixed spp (adaptive off), split into progressive calls of 3 samples
        RenderOptions opt;
        opt.adaptive = false;
        opt.samples_per_call = 3;
        opt.seed = 7;
        const uint64_t credited = render_threads(cam, frozen, W, H, 8, fixed, opt, 3);
        EXPECT(credited == (uint64_t)W * H * 8);
        write_raw(out_fixed, fixed);
    }
    {   // the default: one call for the frame, samples_atom fed by the live progress word
        std::vector<Pixel> px(W * H);
        RenderOptions opt;
        opt.adaptive = false;
        opt.seed = 7;
        const uint64_t credited = render_threads(cam, frozen, W, H, 8, px, opt, 2);
        EXPECT(credited == (uint64_t)W * H * 8);
        EXPECT(std::memcmp(px.data(), fixed.data(), px.size() * sizeof(Pixel)) == 0);
    }
    {   // the frame over 3 logical ranks on device 0 (MultiFrame: tile shards + gather)
        MultiFrame multi(world, {0, 0, 0});
        EXPECT(multi.transport() == OM_TRANSPORT_LOCAL);
        std::vector<Pixel> px(W * H);
        std::atomic<uint64_t> atom{0};
        RenderOptions opt;
        opt.adaptive = false;
        opt.seed = 7;
        opt.samples_per_call = 5;
        multi.render(cam, 50, 0.001f, 100.0f, 8, W, H, PixelsBox{&px}, atom, opt);
        EXPECT(atom.load() == (uint64_t)W * H * 8);
        EXPECT(std::memcmp(px.data(), fixed.data(), px.size() * sizeof(Pixel)) == 0);
    }
    {   // the reference's default: adaptive retirement, credits = every sample of the frame
        std::vector<Pixel> px(W * H);
        RenderOptions opt;
        opt.seed = 7;
        opt.samples_per_call = 5;
        const uint64_t credited = render_threads(cam, frozen, W, H, 24, px, opt, 4);
        EXPECT(credited == (uint64_t)W * H * 24);
        write_raw(out_adaptive, px);
    }
    {   // a framebuffer of the wrong size throws before any device work
        std::vector<Pixel> small(10);
        std::atomic<uint64_t> atom{0};
        bool threw = false;
        try {
            render(cam, frozen, 50, 0.001f, 100.0f, 4, W, H, PixelsBox{&small}, 0, {}, atom);
        } catch (const Error& e) {
            threw = e.status == OM_ERR_INVALID;
        }
        EXPECT(threw && atom.load() == 0);
    }
    if (g_fail == 0) std::printf("gpu ok\n");
    return g_fail == 0 ? 0 : 1;
}

int main(int argc, char** argv) {
    try {
        if (argc >= 2 && std::strcmp(argv[1], "cpu") == 0) return run_cpu();
        if (argc >= 4 && std::strcmp(argv[1], "gpu") == 0) return run_gpu(argv[2], argv[3]);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "uncaught: %s\n", e.what());
        return 1;
    }
    std::fprintf(stderr, "usage: %s cpu | gpu OUT_FIXED OUT_ADAPTIVE\n", argv[0]);
    return 2;
}
