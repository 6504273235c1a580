/*
 * ottomarcher.hpp — C++17 host-side mirror of the reference's scene/render API over the
 * C-ABI of ottomarcher.h.  Header-only; link libottomarcher.so.
 *
 * The reference's host code is Rust (compiled), and this image has no Rust toolchain, so
 * the host side above the C-ABI is C++: same type names, constructors, argument meaning
 * and call shape as the Rust crate, so a front-end reads like src/main.rs:
 *
 *     using namespace ottomarcher;
 *     HittableList world = HittableList::new_();
 *     world += Sphere::new_with_radius(Point3(0., -1000., 0.), 1000., Material::new_lambertian(Color(.5, .5, .5)));
 *     world += Sphere::new_(m4x4::TR(c) ^ m4x4::RX(a) ^ m4x4::SC(.2, .2, .2), mat);      // main.rs:65-68
 *     Camera camera = Camera::new_(lookfrom, lookat, vup, 20., 3. / 2., 0.1, 10.);       // camera.rs:38
 *     FrozenHittableList frozen = world.freeze(camera);                                  // hits.rs:87-89
 *     std::vector<Pixel> pixels(W * H);
 *     render(camera, frozen, 50, 0.001, 100., spp, W, H, PixelsBox{&pixels}, tid, assigned, atom);
 *
 * `new` is a C++ keyword, so the Rust `T::new` constructors are spelled `T::new_`; every
 * other name is the Rust one.  Errors: the reference panics on bugs (a panic kills that
 * worker); here a failed C-ABI call throws ottomarcher::Error carrying om_last_error().
 * All arithmetic (matrices, camera, scene freezing, rendering) happens inside the library
 * with the reference's f32 operation order, so scenes composed here are bit-identical to
 * the library's native builders (tests/cpp/test_api.cpp).
 */
#ifndef OTTOMARCHER_HPP
#define OTTOMARCHER_HPP

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "ottomarcher.h"

namespace ottomarcher {

struct Error : std::runtime_error {
    om_status status;
    Error(om_status s, const std::string& what) : std::runtime_error(what), status(s) {}
};

inline void check(om_status s, const om_ctx* ctx = nullptr) {
    if (s != OM_OK) {
        const char* e = om_last_error(ctx);
        throw Error(s, std::string("ottomarcher: ") + (e ? e : "error") + " (status " + std::to_string(s) + ")");
    }
}

// ------------------------------------------------------------ math/vec3.rs (host value type)
// Only what a front-end needs to compose scenes; component arithmetic is plain f32 in the
// reference's order (vec3.rs:150-260).
struct Vec3 {
    float e[3];
    Vec3() : e{0.0f, 0.0f, 0.0f} {}
    Vec3(float x, float y, float z) : e{x, y, z} {}
    float x() const { return e[0]; }
    float y() const { return e[1]; }
    float z() const { return e[2]; }
    const float* data() const { return e; }
    Vec3 operator+(const Vec3& o) const { return {e[0] + o.e[0], e[1] + o.e[1], e[2] + o.e[2]}; }
    Vec3 operator-(const Vec3& o) const { return {e[0] - o.e[0], e[1] - o.e[1], e[2] - o.e[2]}; }
    Vec3 operator*(const Vec3& o) const { return {e[0] * o.e[0], e[1] * o.e[1], e[2] * o.e[2]}; }
    Vec3 operator*(float f) const { return {e[0] * f, e[1] * f, e[2] * f}; }
    float length_squared() const { return e[0] * e[0] + e[1] * e[1] + e[2] * e[2]; }   // vec3.rs:29-31
    float length() const { return std::sqrt(length_squared()); }                         // vec3.rs:32-34
};
using Point3 = Vec3;
using Color = Vec3;

// ------------------------------------------------------------ materials.rs:27-38
struct Material {
    om_material raw;
    static Material new_lambertian(const Color& albedo) { return {om_material_lambertian(albedo.x(), albedo.y(), albedo.z())}; }
    static Material new_metal(const Color& albedo) { return {om_material_metal(albedo.x(), albedo.y(), albedo.z())}; }
    static Material new_metal_fuzz(const Color& albedo, float fuzz) {
        return {om_material_metal_fuzz(albedo.x(), albedo.y(), albedo.z(), fuzz)};
    }
    static Material new_dielectric(float index_of_refraction) { return {om_material_dielectric(index_of_refraction)}; }
};

// ------------------------------------------------------------ math/mat4x4.rs
// Row-major f32 4x4; `a ^ b` is dot_mat (mat4x4.rs:167-178).  Built by the library so the
// bits match the Rust op order.
struct Mat4x4 {
    float e[16];
    static Mat4x4 identity() { Mat4x4 m; check(om_mat4_identity(m.e)); return m; }                     // mat4x4.rs:16
    static Mat4x4 new_translate(const Vec3& v) { Mat4x4 m; check(om_mat4_translate(v.data(), m.e)); return m; }
    static Mat4x4 new_scale(const Vec3& v) { Mat4x4 m; check(om_mat4_scale(v.data(), m.e)); return m; }
    static Mat4x4 new_rotate_x(float f) { Mat4x4 m; check(om_mat4_rotate(0, f, m.e)); return m; }
    static Mat4x4 new_rotate_y(float f) { Mat4x4 m; check(om_mat4_rotate(1, f, m.e)); return m; }
    static Mat4x4 new_rotate_z(float f) { Mat4x4 m; check(om_mat4_rotate(2, f, m.e)); return m; }
    Mat4x4 dot_mat(const Mat4x4& o) const { Mat4x4 m; check(om_mat4_mul(e, o.e, m.e)); return m; }
    Mat4x4 operator^(const Mat4x4& o) const { return dot_mat(o); }
    Mat4x4 fast_homogenous_inverse() const { Mat4x4 m; check(om_mat4_fast_homogenous_inverse(e, m.e)); return m; }
};

// The m4x4! macro (mat4x4.rs:181-209).
namespace m4x4 {
inline Mat4x4 ID() { return Mat4x4::identity(); }
inline Mat4x4 RX(float a) { return Mat4x4::new_rotate_x(a); }
inline Mat4x4 RY(float a) { return Mat4x4::new_rotate_y(a); }
inline Mat4x4 RZ(float a) { return Mat4x4::new_rotate_z(a); }
inline Mat4x4 TR(const Vec3& v) { return Mat4x4::new_translate(v); }
inline Mat4x4 TR(float x, float y, float z) { return Mat4x4::new_translate(Vec3(x, y, z)); }
inline Mat4x4 SC(const Vec3& v) { return Mat4x4::new_scale(v); }
inline Mat4x4 SC(float x, float y, float z) { return Mat4x4::new_scale(Vec3(x, y, z)); }
}  // namespace m4x4

// ------------------------------------------------------------ camera.rs:10-59
struct Camera {
    om_camera raw;
    static Camera new_(const Point3& lookfrom, const Point3& lookat, const Vec3& vup, float vfov_in_degrees,
                       float aspect_ratio, float aperture, float focus_dist) {
        Camera c;
        check(om_camera_new(lookfrom.data(), lookat.data(), vup.data(), vfov_in_degrees, aspect_ratio, aperture,
                            focus_dist, &c.raw));
        return c;
    }
    static Camera world_camera(float vfov_in_degrees, float aspect_ratio) {                               // camera.rs:33-35
        return new_(Point3(0.0f, 0.0f, 0.0f), Point3(0.0f, 0.0f, -1.0f), Vec3(0.0f, 1.0f, 0.0f), vfov_in_degrees,
                    aspect_ratio, 0.0f, 1.0f);
    }
};

// ------------------------------------------------------------ traced.rs / marched.rs
// Value types holding the constructor arguments; `world += prim` hands them to the library,
// which derives W2L / bases exactly as the Rust constructors do.
struct Sphere {                                                                                          // traced.rs:13-32
    bool by_radius = false;
    Mat4x4 local_to_world{};
    Point3 center;
    float radius = 0.0f;
    Material material{};
    static Sphere new_(const Mat4x4& m_local_to_world, const Material& mat) {
        Sphere s; s.local_to_world = m_local_to_world; s.material = mat; return s;
    }
    static Sphere new_with_radius(const Point3& o, float r, const Material& mat) {
        Sphere s; s.by_radius = true; s.center = o; s.radius = r; s.material = mat; return s;
    }
};

struct Cube {                                                                                            // traced.rs:229-247
    bool by_length = false;
    Mat4x4 local_to_world{};
    Point3 center;
    float length = 0.0f;
    Material material{};
    static Cube new_(const Mat4x4& m_local_to_world, const Material& mat) {
        Cube c; c.local_to_world = m_local_to_world; c.material = mat; return c;
    }
    static Cube new_with_length(const Point3& o, float l, const Material& mat) {
        Cube c; c.by_length = true; c.center = o; c.length = l; c.material = mat; return c;
    }
};

template <int BT>  // Barycentric<BT> (traced.rs:118-226): 0 parallelogram, 1 triangle
struct Barycentric {
    bool three_points = false;
    Point3 origin;
    Vec3 u, v;
    float u_length = 0.0f, v_length = 0.0f;
    Material material{};
    static Barycentric new3points(const Point3& origin, const Point3& upoint, const Point3& vpoint, const Material& mat) {
        Barycentric b; b.three_points = true; b.origin = origin; b.u = upoint; b.v = vpoint; b.material = mat; return b;
    }
    static Barycentric new_(const Point3& origin, const Vec3& u, const Vec3& v, float u_length, float v_length,
                            const Material& mat) {
        Barycentric b; b.origin = origin; b.u = u; b.v = v; b.u_length = u_length; b.v_length = v_length; b.material = mat;
        return b;
    }
};
using Parallelogram = Barycentric<0>;
using Triangle = Barycentric<1>;

struct InfinitePlane {                                                                                   // traced.rs:77-116
    Point3 center;
    Vec3 normal;
    Material material{};
    static InfinitePlane new_(const Point3& center, const Vec3& normal, const Material& material) {
        return {center, normal, material};
    }
};

struct MarchedSphere { Point3 center; float radius; Material material; };                             // marched.rs:50-54
struct MarchedBox { Point3 center; Vec3 sizes; Material material; };                                  // marched.rs:79-83
struct MarchedTorus {                                                                                    // marched.rs:105-130
    Mat4x4 local_to_world;
    Vec3 local_sizes;
    Material material;
    static MarchedTorus new_(const Mat4x4& m_local_to_world, const Vec3& local_sizes, const Material& mat) {
        return {m_local_to_world, local_sizes, mat};
    }
};

// A user marched object: the device form of `HittableList += Arc<dyn Marched>` (hits.rs:96-100), its
// local_sdf a postfix program of om_sdf_op (ottomarcher.h) under MarchedTorus's transform.
struct MarchedSdf {
    Mat4x4 local_to_world;
    std::vector<om_sdf_op> ops;
    Material material;
    static MarchedSdf new_(const Mat4x4& m_local_to_world, std::vector<om_sdf_op> ops, const Material& mat) {
        return {m_local_to_world, std::move(ops), mat};
    }
};

// ------------------------------------------------------------ hits.rs
class FrozenHittableList;

// hits.rs:37-110: host list; `world += prim` appends in type order (hits.rs:370-371).
class HittableList {
public:
    HittableList() { check(om_world_create(&w_)); }
    static HittableList new_() { return HittableList(); }
    ~HittableList() { if (w_) om_world_destroy(w_); }
    HittableList(HittableList&& o) noexcept : w_(std::exchange(o.w_, nullptr)) {}
    HittableList& operator=(HittableList&& o) noexcept {
        if (this != &o) { if (w_) om_world_destroy(w_); w_ = std::exchange(o.w_, nullptr); }
        return *this;
    }
    HittableList(const HittableList&) = delete;
    HittableList& operator=(const HittableList&) = delete;

    HittableList& operator+=(const Sphere& s) {
        check(s.by_radius ? om_world_add_sphere_radius(w_, s.center.data(), s.radius, &s.material.raw)
                          : om_world_add_sphere(w_, s.local_to_world.e, &s.material.raw));
        return *this;
    }
    HittableList& operator+=(const Cube& c) {
        check(c.by_length ? om_world_add_cube_length(w_, c.center.data(), c.length, &c.material.raw)
                          : om_world_add_cube(w_, c.local_to_world.e, &c.material.raw));
        return *this;
    }
    HittableList& operator+=(const Triangle& t) {
        check(t.three_points ? om_world_add_triangle(w_, t.origin.data(), t.u.data(), t.v.data(), &t.material.raw)
                             : om_world_add_triangle_basis(w_, t.origin.data(), t.u.data(), t.v.data(), t.u_length,
                                                           t.v_length, &t.material.raw));
        return *this;
    }
    HittableList& operator+=(const Parallelogram& p) {
        check(p.three_points ? om_world_add_parallelogram(w_, p.origin.data(), p.u.data(), p.v.data(), &p.material.raw)
                             : om_world_add_parallelogram_basis(w_, p.origin.data(), p.u.data(), p.v.data(), p.u_length,
                                                                p.v_length, &p.material.raw));
        return *this;
    }
    HittableList& operator+=(const InfinitePlane& p) {
        check(om_world_add_plane(w_, p.center.data(), p.normal.data(), &p.material.raw));
        return *this;
    }
    HittableList& operator+=(const MarchedSphere& s) {
        check(om_world_add_marched_sphere(w_, s.center.data(), s.radius, &s.material.raw));
        return *this;
    }
    HittableList& operator+=(const MarchedBox& b) {
        check(om_world_add_marched_box(w_, b.center.data(), b.sizes.data(), &b.material.raw));
        return *this;
    }
    HittableList& operator+=(const MarchedTorus& t) {
        check(om_world_add_marched_torus(w_, t.local_to_world.e, t.local_sizes.data(), &t.material.raw));
        return *this;
    }
    HittableList& operator+=(const MarchedSdf& q) {
        check(om_world_add_marched_sdf(w_, q.local_to_world.e, q.ops.data(), (uint32_t)q.ops.size(), &q.material.raw));
        return *this;
    }
    void clear() { check(om_world_clear(w_)); }

    // hits.rs:87-89.  The camera only fed the reference's camera hash (out of scope,
    // DESIGN.md §9); the frozen world lives in HBM on `device`.
    inline FrozenHittableList freeze(const Camera& camera, int32_t device = 0) const;

    om_world* handle() const { return w_; }

private:
    om_world* w_ = nullptr;
};

// hits.rs:63-69: a world resident in device memory (one om_ctx: device + stream).
class FrozenHittableList {
public:
    FrozenHittableList(const HittableList& world, int32_t device = 0) {
        check(om_create(device, &ctx_));
        const om_status s = om_upload_world(ctx_, world.handle());
        if (s != OM_OK) {
            Error e(s, std::string("ottomarcher: ") + om_last_error(ctx_));
            om_destroy(ctx_);
            throw e;
        }
    }
    ~FrozenHittableList() { if (ctx_) om_destroy(ctx_); }
    FrozenHittableList(FrozenHittableList&& o) noexcept : ctx_(std::exchange(o.ctx_, nullptr)) {}
    FrozenHittableList& operator=(FrozenHittableList&& o) noexcept {
        if (this != &o) { if (ctx_) om_destroy(ctx_); ctx_ = std::exchange(o.ctx_, nullptr); }
        return *this;
    }
    FrozenHittableList(const FrozenHittableList&) = delete;
    FrozenHittableList& operator=(const FrozenHittableList&) = delete;

    void set_kernel(int32_t kernel) { check(om_set_kernel(ctx_, kernel), ctx_); }
    void set_pipeline(int32_t pipeline) { check(om_set_pipeline(ctx_, pipeline), ctx_); }
    om_ctx* ctx() const { return ctx_; }

private:
    om_ctx* ctx_ = nullptr;
};

inline FrozenHittableList HittableList::freeze(const Camera&, int32_t device) const { return FrozenHittableList(*this, device); }

// ------------------------------------------------------------ render_thread.rs
// Pixel = the reference's Stats (render_thread.rs:9-17, 40 bytes); the caller owns the
// framebuffer and passes a PixelsBox pointing at it (render_thread.rs:53-65, main.rs:192).
using Pixel = om_pixel_stats;
struct PixelsBox {
    std::vector<Pixel>* pixels;
};

// What the Rust signature cannot carry.  `adaptive` defaults to the reference's behaviour:
// render() always retires converged pixels (Stats::add's bad_avgs rule, render_thread.rs:31-38,
// 97-101); the benchmark's fixed-spp metric turns it off.  `samples_per_call` (0 = the whole
// frame in one call) splits the frame into progressive calls; progress does not need it:
// samples_atom advances while a call runs (om_progress).  `seed` keys om-rng (replaces thread_rng).
struct RenderOptions {
    bool adaptive = true;
    uint32_t samples_per_call = 0;
    uint64_t seed = 1;
    uint32_t march_steps = 1024;   // hits.rs:292
};

// render_thread::render (render_thread.rs:145-202).  The reference calls it from num_cpus-1
// threads with disjoint pixel sets (main.rs:200-214); here tid 0 renders every pixel on the
// device and the other tids return at once, so main.rs's thread loop stays correct.
// `assigned_thread` is accepted for signature parity and validated for size.  samples_atom
// receives the reference's credit (render_thread.rs:196-198) live: a poller copies the
// device-fed progress word (om_progress) into it every millisecond while the calls run, the
// way main.rs's log thread polls the atomic (main.rs:151-168).  The framebuffer is page-locked
// for the duration (om_host_register) so the per-call copies run at DMA speed.
inline void render(const Camera& camera, const FrozenHittableList& world, uint32_t max_depth, float tmin, float tmax,
                   uint32_t samples_per_pixel, uint32_t image_width, uint32_t image_height, PixelsBox pixels_box,
                   uint32_t tid, const std::vector<uint32_t>& assigned_thread, std::atomic<uint64_t>& samples_atom,
                   const RenderOptions& opt = RenderOptions()) {
    const uint64_t image_size = (uint64_t)image_width * image_height;
    if (!pixels_box.pixels || pixels_box.pixels->size() != image_size)
        throw Error(OM_ERR_INVALID, "ottomarcher: render: pixels must hold image_width*image_height entries");
    if (!assigned_thread.empty() && assigned_thread.size() != image_size)
        throw Error(OM_ERR_INVALID, "ottomarcher: render: assigned_thread must hold image_width*image_height entries");
    if (tid != 0 || samples_per_pixel == 0) return;
    const volatile uint64_t* prog = om_progress(world.ctx());
    if (!prog) throw Error(OM_ERR_DEVICE, std::string("ottomarcher: ") + om_last_error(world.ctx()));
    const uint64_t p0 = *prog;
    uint64_t credited = 0;                  // progress already added to samples_atom
    auto publish = [&]() {
        const uint64_t v = *prog - p0;
        if (v > credited) { samples_atom.fetch_add(v - credited, std::memory_order_relaxed); credited = v; }
    };
    void* const buf = pixels_box.pixels->data();
    const bool pinned = image_size && om_host_register(buf, image_size * sizeof(Pixel)) == OM_OK;
    std::atomic<bool> stop{false};
    std::thread poller([&]() {
        while (!stop.load(std::memory_order_relaxed)) {
            publish();
            std::this_thread::sleep_for(std::chrono::milliseconds(1));
        }
    });
    om_status st = OM_OK;
    const uint32_t per_call = opt.samples_per_call ? opt.samples_per_call : samples_per_pixel;
    for (uint32_t done = 0; done < samples_per_pixel && st == OM_OK; done += per_call) {
        om_render_params p{};
        p.width = image_width;
        p.height = image_height;
        p.spp_total = samples_per_pixel;
        p.sample_begin = done;
        p.sample_count = samples_per_pixel - done < per_call ? samples_per_pixel - done : per_call;
        p.max_depth = max_depth;
        p.tmin = tmin;
        p.tmax = tmax;
        p.march_steps = opt.march_steps;
        p.adaptive = opt.adaptive ? 1u : 0u;
        p.seed = opt.seed;
        st = om_render(world.ctx(), &camera.raw, &p, pixels_box.pixels->data(), nullptr);
    }
    stop = true;
    poller.join();
    publish();                              // the calls are synchronous: the word is final
    if (pinned) (void)om_host_unregister(buf);
    check(st, world.ctx());
}

// The render threads of main.rs:170-214 spread over GPUs: a ctx per device, 8x8 tiles dealt
// round-robin to them, the shards gathered into the caller's framebuffer (om_multi_*; RCCL
// between distinct devices).  render() has render_thread::render's meaning for the whole frame.
class MultiFrame {
public:
    MultiFrame(const HittableList& world, const std::vector<int32_t>& devices) {
        check(om_multi_create(devices.data(), (uint32_t)devices.size(), &m_));
        const om_status s = om_multi_upload_world(m_, world.handle());
        if (s != OM_OK) {
            Error e(s, std::string("ottomarcher: ") + om_multi_last_error(m_));
            om_multi_destroy(m_);
            throw e;
        }
    }
    ~MultiFrame() { if (m_) om_multi_destroy(m_); }
    MultiFrame(const MultiFrame&) = delete;
    MultiFrame& operator=(const MultiFrame&) = delete;
    int32_t transport() const { return om_multi_transport(m_); }
    om_ctx* ctx(uint32_t rank) const { return om_multi_ctx(m_, rank); }
    void render(const Camera& camera, uint32_t max_depth, float tmin, float tmax, uint32_t samples_per_pixel,
                uint32_t image_width, uint32_t image_height, PixelsBox pixels_box, std::atomic<uint64_t>& samples_atom,
                const RenderOptions& opt = RenderOptions()) {
        const uint64_t image_size = (uint64_t)image_width * image_height;
        if (!pixels_box.pixels || pixels_box.pixels->size() != image_size)
            throw Error(OM_ERR_INVALID, "ottomarcher: MultiFrame::render: pixels must hold image_width*image_height entries");
        const uint32_t per_call = opt.samples_per_call ? opt.samples_per_call : samples_per_pixel;
        for (uint32_t done = 0; done < samples_per_pixel; done += per_call) {
            om_render_params p{};
            p.width = image_width; p.height = image_height; p.spp_total = samples_per_pixel; p.sample_begin = done;
            p.sample_count = samples_per_pixel - done < per_call ? samples_per_pixel - done : per_call;
            p.max_depth = max_depth; p.tmin = tmin; p.tmax = tmax; p.march_steps = opt.march_steps;
            p.adaptive = opt.adaptive ? 1u : 0u; p.seed = opt.seed;
            om_counters c{};
            const om_status s = om_multi_render_host(m_, &camera.raw, &p, pixels_box.pixels->data(), &c);
            if (s != OM_OK) throw Error(s, std::string("ottomarcher: ") + om_multi_last_error(m_));
            samples_atom.fetch_add(c.credited, std::memory_order_relaxed);
        }
    }

private:
    om_multi* m_ = nullptr;
};

// draw_to_sdl views (main.rs:360-437) and the F12 save (main.rs:473-476), headless.
inline std::vector<uint8_t> display(const FrozenHittableList& world, const std::vector<Pixel>& pixels, uint32_t width,
                                    uint32_t height, int32_t view, std::vector<uint8_t> rgb = {}) {
    rgb.resize((size_t)width * height * 3);
    check(om_display(world.ctx(), pixels.data(), width, height, view, rgb.data()), world.ctx());
    return rgb;
}
inline void write_bmp(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t width, uint32_t height) {
    check(om_write_bmp(path.c_str(), rgb.data(), width, height));
}
inline void write_ppm(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t width, uint32_t height) {
    check(om_write_ppm(path.c_str(), rgb.data(), width, height));
}

}  // namespace ottomarcher
#endif  // OTTOMARCHER_HPP
