// random_scene.hpp — the reference front-end's scene builders (main.rs:37-110) written
// statement for statement against the C++ mirror API (include/ottomarcher.hpp).
// Random draws come from om-rng's SplitMix64 host stream, which replaces
// rand::thread_rng (utils.rs:25) with the same 24-bit [0,1) grid and the same draw order,
// so the scene is bit-identical to the library's native om_world_random_scene.
#pragma once
#include <cstdint>

#include "ottomarcher.hpp"

namespace ottomarcher {

constexpr float PI = 3.1415926535897932385f;                                                  // utils.rs:29

struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next_u64() {
        s += 0x9E3779B97F4A7C15ULL;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    float rand() { return (float)(uint32_t)(next_u64() >> 40) * 5.9604644775390625e-8f; }    // f32::rand  utils.rs:25
    float rand_range(float lo, float hi) { const float r = rand(); return r * (hi - lo) + lo; }  // utils.rs:26
    Color color_rand() { const float x = rand(); const float y = rand(); const float z = rand(); return {x, y, z}; }  // vec3.rs:81
    Color color_rand_range(float lo, float hi) {                                              // vec3.rs:82-88
        const float x = rand_range(lo, hi); const float y = rand_range(lo, hi); const float z = rand_range(lo, hi);
        return {x, y, z};
    }
};

// main.rs:37-100.  with_torus: the marched torus block (main.rs:73-81), which the benchmark's
// S-traced scene omits; grid_half 11 = the reference grid, 50 = the 10k-sphere variant (C3).
// C++ leaves the evaluation order of `a ^ f(g)` operands unspecified, so every draw is taken
// into a local first, in the order Rust evaluates them (left to right).
inline HittableList random_scene(uint64_t seed = 0x5EED, bool with_torus = false, int grid_half = 11, bool extras = true) {
    SplitMix64 g(seed);
    HittableList world = HittableList::new_();
    const Material mat_ground = Material::new_lambertian(Color(0.5f, 0.5f, 0.5f));            // :39
    world += Sphere::new_with_radius(Point3(0.0f, -1000.0f, 0.0f), 1000.0f, mat_ground);      // :40-41
    for (int a = -grid_half; a < grid_half; ++a) {                                           // :42
        const float af = (float)a;
        for (int b = -grid_half; b < grid_half; ++b) {                                       // :44
            const float bf = (float)b;
            const float cx = af + 0.9f * g.rand();                                            // :46
            const float cz = bf + 0.9f * g.rand();
            const Point3 center(cx, 0.2f, cz);
            if (!((center - Point3(4.0f, 0.2f, 0.0f)).length() > 0.9f)) continue;            // :47
            Material sphere_material;
            const float mat_prob = g.rand();                                                  // :50
            if (mat_prob < 0.8f) {                                                            // :51-54
                const Color c1 = g.color_rand();
                const Color c2 = g.color_rand();
                sphere_material = Material::new_lambertian(c1 * c2);
            } else if (mat_prob < 0.95f) {                                                    // :55-59
                const Color albedo = g.color_rand_range(0.5f, 1.0f);
                const float fuzz = g.rand_range(0.0f, 0.5f);
                sphere_material = Material::new_metal_fuzz(albedo, fuzz);
            } else {                                                                          // :60-62
                sphere_material = Material::new_dielectric(1.5f);
            }
            const float rx = g.rand() * 2.0f * PI;                                            // :65-68
            const float ry = g.rand() * 2.0f * PI;
            const float rz = g.rand() * 2.0f * PI;
            const float sx = g.rand() + 1.0f;
            const float sy = g.rand() + 1.0f;
            const float sz = g.rand() + 1.0f;
            const Mat4x4 m = m4x4::TR(center) ^ m4x4::RX(rx) ^ m4x4::RY(ry) ^ m4x4::RZ(rz) ^ m4x4::SC(sx, sy, sz) ^
                             m4x4::SC(0.2f, 0.2f, 0.2f);
            world += Sphere::new_(m, sphere_material);                                       // :69
        }
    }
    if (with_torus) {                                                                         // :73-81
        const Material mat = Material::new_dielectric(1.5f);
        const Mat4x4 local_to_world = m4x4::TR(0.0f, 1.0f, 0.0f) ^ m4x4::RX(0.6f) ^ m4x4::RZ(1.33f * 2.0f * PI);
        world += MarchedTorus::new_(local_to_world, Vec3(0.5f, 0.1f, 0.1f), mat);
    }
    if (extras) {
        const Point3 p1(7.0f, 1.0f, 0.0f), p2(6.0f, 1.1f, 0.5f), p3(6.0f, 1.5f, 0.0f);        // :83-85
        world += Parallelogram::new3points(p1, p2, p3, Material::new_metal(Color(1.0f, 0.5f, 1.0f)));              // :86-88
        world += Triangle::new3points(p1 + Vec3(0.0f, 0.5f, 0.0f), p2, p3, Material::new_lambertian(Color(1.0f, 1.0f, 0.0f)));  // :89-91
        const Material mat = Material::new_metal(Color(0.7f, 0.6f, 0.5f));                   // :93-98
        const float rx = g.rand() * 2.0f * PI;
        const float ry = g.rand() * 2.0f * PI;
        const float rz = g.rand() * 2.0f * PI;
        world += Cube::new_(m4x4::TR(4.0f, 1.0f, 0.0f) ^ m4x4::RX(rx) ^ m4x4::RY(ry) ^ m4x4::RZ(rz), mat);
    }
    return world;
}

// main.rs:103-110
inline HittableList basic_scene() {
    HittableList world = HittableList::new_();
    const Material m = Material::new_lambertian(Color(0.5f, 0.5f, 0.5f));
    world += Sphere::new_with_radius(Point3(0.0f, 0.0f, -2.0f), 1.0f, m);
    world += Sphere::new_with_radius(Point3(-2.0f, 0.0f, -2.0f), 1.0f, m);
    world += Sphere::new_with_radius(Point3(2.0f, 0.0f, -2.0f), 1.0f, m);
    return world;
}

// main.rs:136-142
inline Camera default_camera(float aspect_ratio) {
    return Camera::new_(Point3(13.0f, 2.0f, 3.0f), Point3(0.0f, 0.0f, 0.0f), Vec3(0.0f, 1.0f, 0.0f), 20.0f, aspect_ratio,
                        0.1f, 10.0f);
}

// main.rs:170-189: CHUNK_SIZE = 32 KiB / size_of::<Color>() pixels per chunk, chunks dealt
// round-robin to the worker threads, the leftover to the next thread in turn.
inline std::vector<uint32_t> assign_threads(uint32_t image_size, uint32_t num_threads) {
    const uint32_t CHUNK_SIZE = 32u * 1024u / 12u;
    std::vector<uint32_t> assigned;
    assigned.reserve(image_size);
    for (uint32_t chunk = 0; chunk < image_size / CHUNK_SIZE; ++chunk)
        for (uint32_t i = 0; i < CHUNK_SIZE; ++i) assigned.push_back(chunk % num_threads);
    const uint32_t id = (image_size / CHUNK_SIZE) % num_threads;
    while (assigned.size() < image_size) assigned.push_back(id);
    return assigned;
}

}  // namespace ottomarcher
