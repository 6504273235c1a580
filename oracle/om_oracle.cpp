// ============================================================================
// om_oracle.cpp — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
//
// A line-by-line C++ restatement of the reference hot path of
// octaviogarcia/RaytracingOneWeekend ("ottomarcher"), used ONLY by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
// Nothing in the product (raytracingoneweekend_amd/, include/) links, loads or
// calls this file.
//
// PARITY STATUS: "parity unpinned" against the real reference.
//   * The reference is Rust; no cargo/rustc exists in this image, its crates are
//     not vendored and there is no Cargo.lock, so it cannot be built or run here.
//   * The reference ships no tests, golden vectors or fixtures.
//   * Its RNG is rand 0.8 ThreadRng (ChaCha12, OS-seeded; utils.rs:25) and is not
//     reproducible, so the build defines its own counter-based RNG contract
//     (om-rng v2) at exactly the reference's draw sites.
//   This restatement is therefore anchored by analytic known-answer tests
//   (tests/test_oracle_kat.py) and by committed fixtures it generates
//   (tests/golden/, made by tests/golden/make_golden.py).
//
// Arithmetic contract: IEEE-754 binary32, no FMA contraction (-ffp-contract=off),
// no fast-math, same operation order as the Rust source (Rust never contracts or
// reassociates f32).  f32::max/min are NaN-ignoring (fmaxf/fminf); `as u8` is a
// saturating cast with NaN -> 0.
//
// Citations are file:line in /root/reference/src/.
// ============================================================================
#include <cmath>
#include <cstdint>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <thread>
#include <atomic>
#include <algorithm>

namespace oro {

static const float INF_F = INFINITY;
static const float PI_F = 3.1415926535897932385f;  // utils.rs:29

// ----------------------------------------------------------------------------
// om-rng v2 (replaces rand::thread_rng(); utils.rs:25).  Every draw maps 24 random
// bits to f32 * 2^-24 (rand 0.8's `Standard` f32 mapping, a 24-bit grid in [0,1)).
//   Rng      SplitMix64 — host-side streams: the scene generator and the jitter table.
//   PathRng  the per-path stream used inside ray_color: a 32-bit Weyl counter s and a
//            32-bit key k, both from one mix64 of (pixel << 32 | sample) ^ skey; a draw
//            is lowbias32((s += 0x9E3779B9) ^ k) >> 8.  Two 32-bit multiplies per draw
//            instead of SplitMix64's two 64-bit ones (~10% of the GPU bounce kernel);
//            the key keeps two paths whose counters overlap uncorrelated.
// ----------------------------------------------------------------------------
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
struct Rng {
    uint64_t s;
    inline uint64_t next_u64() { s += 0x9E3779B97F4A7C15ULL; return mix64(s); }
    // utils.rs:25  f32::rand()
    inline float rand() { return (float)(uint32_t)(next_u64() >> 40) * 5.9604644775390625e-8f; }
    // utils.rs:26  rand_range(min,max) = rand()*(max-min) + min
    inline float rand_range(float mn, float mx) { float r = rand(); return r * (mx - mn) + mn; }
};
struct PathRng {
    uint32_t s, k;
    static inline PathRng from_state(uint64_t st) { PathRng r; r.s = (uint32_t)st; r.k = (uint32_t)(st >> 32); return r; }
    inline uint32_t next_u32() {
        s += 0x9E3779B9u;
        uint32_t x = s ^ k;
        x ^= x >> 16; x *= 0x21F0AAADu;
        x ^= x >> 15; x *= 0x735A2D97u;
        return x ^ (x >> 15);
    }
    inline float rand() { return (float)(next_u32() >> 8) * 5.9604644775390625e-8f; }            // utils.rs:25
    inline float rand_range(float mn, float mx) { float r = rand(); return r * (mx - mn) + mn; }  // utils.rs:26
};
// Per-path stream: key = (pixel << 32) | sample, seed folded once.
static inline uint64_t seed_key(uint64_t seed) { return mix64(seed + 0x632BE59BD9B4E019ULL); }
static inline PathRng path_rng(uint64_t skey, uint32_t pixel, uint32_t sample) {
    return PathRng::from_state(mix64((((uint64_t)pixel << 32) | (uint64_t)sample) ^ skey));
}

// ----------------------------------------------------------------------------
// math/vec3.rs
// ----------------------------------------------------------------------------
struct V3 { float x, y, z; };
static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }                           // vec3.rs:118-121
static inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }       // vec3.rs:184-193
static inline V3 operator-(V3 a, V3 b) { return a + (-b); }                                  // vec3.rs:194-199
static inline V3 operator*(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }       // vec3.rs:200-209
static inline V3 operator*(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }          // vec3.rs:220-229
static inline V3 operator*(float s, V3 a) { return a * s; }                                  // vec3.rs:230-235
static inline V3 operator/(V3 a, float s) { return a * (1.0f / s); }                         // vec3.rs:236-240
static inline float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }            // vec3.rs:29-31
static inline float length_squared(V3 a) { return dot(a, a); }                               // vec3.rs:32-34
static inline float length(V3 a) { return std::sqrt(length_squared(a)); }                   // vec3.rs:35-37
static inline V3 unit(V3 a) { return a / length(a); }                                        // vec3.rs:38-40
static inline V3 vabs(V3 a) { return v3(std::fabs(a.x), std::fabs(a.y), std::fabs(a.z)); }  // vec3.rs:44-46
static inline float max_val(V3 a) { return std::fmax(a.x, std::fmax(a.y, a.z)); }           // vec3.rs:47-49
static inline float min_val(V3 a) { return std::fmin(a.x, std::fmin(a.y, a.z)); }           // vec3.rs:50-52
static inline V3 vmax(V3 a, V3 b) { return v3(std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)); }  // :53-55
static inline V3 cross(V3 a, V3 b) {                                                         // vec3.rs:62-68
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline bool near_zero(V3 a) {                                                         // vec3.rs:69-72
    const float eps = 1e-8f;
    return (std::fabs(a.x) < eps) && (std::fabs(a.y) < eps) && (std::fabs(a.z) < eps);
}
static inline float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
// Rust `f32 as u8`: saturating, NaN -> 0.
static inline uint8_t f32_as_u8(float f) {
    if (!(f > 0.0f)) return 0;           // NaN, negatives, zero
    if (f >= 255.0f) return 255;
    return (uint8_t)f;                   // truncation toward zero
}
// vec3.rs:74-76
static inline void to_u8x3(V3 c, uint8_t out[3]) {
    out[0] = f32_as_u8(c.x * 256.0f); out[1] = f32_as_u8(c.y * 256.0f); out[2] = f32_as_u8(c.z * 256.0f);
}
template <class G>
static inline V3 rand_v3_range(G& g, float mn, float mx) {                                 // vec3.rs:82-88
    float x = g.rand_range(mn, mx); float y = g.rand_range(mn, mx); float z = g.rand_range(mn, mx);
    return v3(x, y, z);
}
template <class G>
static inline V3 rand_v3(G& g) { float x = g.rand(); float y = g.rand(); float z = g.rand(); return v3(x, y, z); }  // vec3.rs:81
template <class G>
static inline V3 rand_in_unit_sphere(G& g) {                                               // vec3.rs:92-97
    for (;;) { V3 p = rand_v3_range(g, -1.0f, 1.0f); if (length_squared(p) < 1.0f) return p; }
}
template <class G>
static inline V3 rand_unit_vector(G& g) { return unit(rand_in_unit_sphere(g)); }          // vec3.rs:98-100
template <class G>
static inline V3 rand_in_unit_disc(G& g) {                                                 // vec3.rs:108-113
    for (;;) {
        float x = g.rand_range(-1.0f, 1.0f); float y = g.rand_range(-1.0f, 1.0f);
        V3 p = v3(x, y, 0.0f);
        if (length_squared(p) < 1.0f) return p;
    }
}

// ----------------------------------------------------------------------------
// math/vec4.rs, math/mat3x3.rs, math/mat4x4.rs
// ----------------------------------------------------------------------------
struct V4 { float x, y, z, w; };
static inline V4 v4(float x, float y, float z, float w) { V4 r = {x, y, z, w}; return r; }
static inline V4 v4_v3(V3 a) { return v4(a.x, a.y, a.z, 0.0f); }                            // vec4.rs:18
static inline V4 v4_p3(V3 a) { return v4(a.x, a.y, a.z, 1.0f); }                            // vec4.rs:19
static inline V3 xyz(V4 a) { return v3(a.x, a.y, a.z); }                                     // vec4.rs:54-56
static inline float dot4(V4 a, V4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }  // vec4.rs:27-29
static inline V4 operator-(V4 a) { return v4(-a.x, -a.y, -a.z, -a.w); }
static inline V4 operator+(V4 a, V4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }  // vec4.rs:111-121
static inline V4 operator-(V4 a, V4 b) { return a + (-b); }                                  // vec4.rs:122-127
static inline V4 operator*(V4 a, V4 b) { return v4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }  // vec4.rs:128-138
static inline V4 operator*(V4 a, float s) { return v4(a.x * s, a.y * s, a.z * s, a.w * s); }      // vec4.rs:150-160
static inline V4 operator*(float s, V4 a) { return a * s; }                                  // vec4.rs:161-166

struct M3 { V3 r[3]; };                                                                      // mat3x3.rs:6-8
static inline M3 m3_rows(V3 a, V3 b, V3 c) { M3 m; m.r[0] = a; m.r[1] = b; m.r[2] = c; return m; }
static inline M3 m3_cols(V3 a, V3 b, V3 c) {                                                 // mat3x3.rs:22-26
    return m3_rows(v3(a.x, b.x, c.x), v3(a.y, b.y, c.y), v3(a.z, b.z, c.z));
}
static inline float m3at(const M3& m, int i, int j) { return comp(m.r[i], j); }
static inline V3 m3_dot(const M3& m, V3 v) { return v3(dot(m.r[0], v), dot(m.r[1], v), dot(m.r[2], v)); }  // :27-29
static inline M3 m3_transpose(const M3& m) {                                                 // :49-51
    return m3_rows(v3(m.r[0].x, m.r[1].x, m.r[2].x), v3(m.r[0].y, m.r[1].y, m.r[2].y), v3(m.r[0].z, m.r[1].z, m.r[2].z));
}
static float m3_determinant(const M3& m) {                                                   // mat3x3.rs:52-68 (Kahan)
    volatile float sum = 0.0f, c = 0.0f;
    float in[6] = {
        (m3at(m, 0, 0) * m3at(m, 1, 1)) * m3at(m, 2, 2),
        (m3at(m, 0, 1) * m3at(m, 1, 2)) * m3at(m, 2, 0),
        (m3at(m, 0, 2) * m3at(m, 1, 0)) * m3at(m, 2, 1),
        ((-m3at(m, 0, 0)) * m3at(m, 1, 2)) * m3at(m, 2, 1),
        ((-m3at(m, 0, 1)) * m3at(m, 1, 0)) * m3at(m, 2, 2),
        ((-m3at(m, 0, 2)) * m3at(m, 1, 1)) * m3at(m, 2, 0)};
    for (int k = 0; k < 6; ++k) {
        float y = in[k] - c;
        float t = sum + y;
        c = (t - sum) - y;
        sum = t;
    }
    return sum;
}
static M3 m3_inverse(const M3& m) {                                                          // mat3x3.rs:69-81
    float det = m3_determinant(m);
    V3 r0 = v3(m3at(m, 1, 1) * m3at(m, 2, 2) - m3at(m, 1, 2) * m3at(m, 2, 1),
               m3at(m, 0, 2) * m3at(m, 2, 1) - m3at(m, 0, 1) * m3at(m, 2, 2),
               m3at(m, 0, 1) * m3at(m, 1, 2) - m3at(m, 0, 2) * m3at(m, 1, 1));
    V3 r1 = v3(m3at(m, 1, 2) * m3at(m, 2, 0) - m3at(m, 1, 0) * m3at(m, 2, 2),
               m3at(m, 0, 0) * m3at(m, 2, 2) - m3at(m, 0, 2) * m3at(m, 2, 0),
               m3at(m, 0, 2) * m3at(m, 1, 0) - m3at(m, 0, 0) * m3at(m, 1, 2));
    V3 r2 = v3(m3at(m, 1, 0) * m3at(m, 2, 1) - m3at(m, 1, 1) * m3at(m, 2, 0),
               m3at(m, 0, 1) * m3at(m, 2, 0) - m3at(m, 0, 0) * m3at(m, 2, 1),
               m3at(m, 0, 0) * m3at(m, 1, 1) - m3at(m, 0, 1) * m3at(m, 1, 0));
    float s = 1.0f / det;                                                                    // mat3x3.rs:92-96
    return m3_rows(r0 * s, r1 * s, r2 * s);
}

struct M4 { V4 r[4]; };                                                                      // mat4x4.rs:8-10
static inline M4 m4_rows(V4 a, V4 b, V4 c, V4 d) { M4 m; m.r[0] = a; m.r[1] = b; m.r[2] = c; m.r[3] = d; return m; }
static inline M4 m4_identity() { return m4_rows(v4(1, 0, 0, 0), v4(0, 1, 0, 0), v4(0, 0, 1, 0), v4(0, 0, 0, 1)); }
static inline float v4c(V4 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : (i == 2 ? a.z : a.w)); }
static inline V4 m4_col(const M4& m, int c) { return v4(v4c(m.r[0], c), v4c(m.r[1], c), v4c(m.r[2], c), v4c(m.r[3], c)); }  // :81-83
static inline M4 m4_cols(V4 a, V4 b, V4 c, V4 d) {                                           // mat4x4.rs:32-37
    return m4_rows(v4(a.x, b.x, c.x, d.x), v4(a.y, b.y, c.y, d.y), v4(a.z, b.z, c.z, d.z), v4(a.w, b.w, c.w, d.w));
}
static inline M4 m4_transpose(const M4& m) { return m4_rows(m4_col(m, 0), m4_col(m, 1), m4_col(m, 2), m4_col(m, 3)); }  // :85-87
static inline V4 m4_dot(const M4& m, V4 v) { return v4(dot4(m.r[0], v), dot4(m.r[1], v), dot4(m.r[2], v), dot4(m.r[3], v)); }  // :45-47
static inline V3 m4_dot_p3(const M4& m, V3 p) {                                              // mat4x4.rs:49-52
    V4 q = v4_p3(p); return v3(dot4(m.r[0], q), dot4(m.r[1], q), dot4(m.r[2], q));
}
static inline V3 m4_dot_v3(const M4& m, V3 p) {                                              // mat4x4.rs:54-57
    V4 q = v4_v3(p); return v3(dot4(m.r[0], q), dot4(m.r[1], q), dot4(m.r[2], q));
}
static M4 m4_dot_mat(const M4& a, const M4& b) {                                             // mat4x4.rs:66-72
    M4 t = m4_transpose(b); M4 o;
    for (int i = 0; i < 4; ++i)
        o.r[i] = v4(dot4(a.r[i], t.r[0]), dot4(a.r[i], t.r[1]), dot4(a.r[i], t.r[2]), dot4(a.r[i], t.r[3]));
    return o;
}
static inline M4 m4_from_m3(const M3& m) {                                                   // mat4x4.rs:38-43
    return m4_rows(v4_v3(m.r[0]), v4_v3(m.r[1]), v4_v3(m.r[2]), v4(0.0f, 0.0f, 0.0f, 1.0f));
}
static inline M4 m4_translate(V3 v) {                                                        // mat4x4.rs:88-93
    return m4_rows(v4(1, 0, 0, v.x), v4(0, 1, 0, v.y), v4(0, 0, 1, v.z), v4(0, 0, 0, 1));
}
static inline M4 m4_scale(V3 v) {                                                            // mat4x4.rs:94-99
    return m4_rows(v4(v.x, 0, 0, 0), v4(0, v.y, 0, 0), v4(0, 0, v.z, 0), v4(0, 0, 0, 1));
}
static inline M4 m4_rot_x(float f) { float c = std::cos(f), s = std::sin(f);                // mat4x4.rs:100-107
    return m4_rows(v4(1, 0, 0, 0), v4(0, c, s, 0), v4(0, -s, c, 0), v4(0, 0, 0, 1)); }
static inline M4 m4_rot_y(float f) { float c = std::cos(f), s = std::sin(f);                // mat4x4.rs:108-115
    return m4_rows(v4(c, 0, -s, 0), v4(0, 1, 0, 0), v4(s, 0, c, 0), v4(0, 0, 0, 1)); }
static inline M4 m4_rot_z(float f) { float c = std::cos(f), s = std::sin(f);                // mat4x4.rs:116-123
    return m4_rows(v4(c, -s, 0, 0), v4(s, c, 0, 0), v4(0, 0, 1, 0), v4(0, 0, 0, 1)); }
static M4 m4_fast_homogenous_inverse(const M4& m) {                                          // mat4x4.rs:59-64
    M4 s_inv = m4_from_m3(m3_inverse(m3_rows(xyz(m.r[0]), xyz(m.r[1]), xyz(m.r[2]))));
    M4 t_inv = m4_translate(-xyz(m4_col(m, 3)));
    return m4_dot_mat(s_inv, t_inv);
}
static void m4_decompose_trs(const M4& m, M4& t, M4& r, M4& s) {                            // mat4x4.rs:125-147
    V3 a = xyz(m4_col(m, 0)), b = xyz(m4_col(m, 1)), c = xyz(m4_col(m, 2)), d = xyz(m4_col(m, 3));
    float al = length(a), bl = length(b), cl = length(c);
    t = m4_cols(v4(1, 0, 0, 0), v4(0, 1, 0, 0), v4(0, 0, 1, 0), v4_p3(d));
    r = m4_cols(v4_v3(a / al), v4_v3(b / bl), v4_v3(c / cl), v4_p3(v3(0, 0, 0)));
    s = m4_rows(v4(al, 0, 0, 0), v4(0, bl, 0, 0), v4(0, 0, cl, 0), v4(0, 0, 0, 1));
}
static inline V4 m4_diag(const M4& m) { return v4(m.r[0].x, m.r[1].y, m.r[2].z, m.r[3].w); }  // mat4x4.rs:148-150
static inline M4 m4_load(const float* f) {
    return m4_rows(v4(f[0], f[1], f[2], f[3]), v4(f[4], f[5], f[6], f[7]), v4(f[8], f[9], f[10], f[11]), v4(f[12], f[13], f[14], f[15]));
}
static inline void m4_store(const M4& m, float* f) {
    for (int i = 0; i < 4; ++i) { f[4 * i] = m.r[i].x; f[4 * i + 1] = m.r[i].y; f[4 * i + 2] = m.r[i].z; f[4 * i + 3] = m.r[i].w; }
}

// ----------------------------------------------------------------------------
// ray.rs, materials.rs (data), hits.rs HitRecord
// ----------------------------------------------------------------------------
struct Ray { V3 orig, dir; };
static inline Ray ray_new(V3 o, V3 d) { Ray r; r.orig = o; r.dir = unit(d); return r; }     // ray.rs:11-13
static inline V3 ray_at(const Ray& r, float t) { return r.orig + t * r.dir; }               // ray.rs:14-16
static inline Ray ray_transform(const Ray& r, const M4& m) {                                 // ray.rs:17-19
    Ray o; o.orig = m4_dot_p3(m, r.orig); o.dir = m4_dot_v3(m, r.dir); return o;
}

enum { MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2 };                              // materials.rs:12-16
struct Material { float albedo[3]; float fuzz; float ior; int32_t type; };                   // materials.rs:18-24 (24 B)
static inline V3 albedo(const Material& m) { return v3(m.albedo[0], m.albedo[1], m.albedo[2]); }

struct HitRecord { V3 point; V3 normal; Material material; float t; uint64_t obj_id; };       // hits.rs:11-17

// ----------------------------------------------------------------------------
// traced.rs
// ----------------------------------------------------------------------------
struct Sphere { M4 l2w, w2l; Material mat; uint64_t id; };                                  // traced.rs:13-19
struct Cube { M4 l2w, w2l; Material mat; uint64_t id; };                                    // traced.rs:229-235
struct Plane { V3 center, normal; Material mat; uint64_t id; };                             // traced.rs:77-82
struct Bary { V3 origin, u; float u_length; V3 v; float v_length; V3 uxv, uxvxu; M3 base_inv; V3 v_in_base;  // traced.rs:118-131
              Material mat; uint64_t id; };

static bool sphere_hit(const Sphere& s, const Ray& r, float tmin, float tmax, HitRecord& hr) {  // traced.rs:39-62
    Ray nr = ray_transform(r, s.w2l);
    float a = length_squared(nr.dir);
    float half_b = dot(nr.orig, nr.dir);
    float c = length_squared(nr.orig) - 1.0f;
    float disc = half_b * half_b - a * c;
    if (disc < 0.0f) return false;
    float sqrtd = std::sqrt(disc);
    float root = (-half_b - sqrtd) / a;
    if (root < tmin || root > tmax) {
        root = (-half_b + sqrtd) / a;
        if (root < tmin || root > tmax) return false;
    }
    V3 lp = ray_at(nr, root);
    hr.point = m4_dot_p3(s.l2w, lp);
    hr.normal = unit(m4_dot_v3(s.l2w, lp));
    hr.material = s.mat; hr.t = root; hr.obj_id = s.id;
    return true;
}

static bool cube_hit(const Cube& cb, const Ray& r, float tmin, float tmax, HitRecord& hr) {  // traced.rs:266-298
    Ray nr = ray_transform(r, cb.w2l);
    float smallest_t = INF_F; int idx = -1;
    for (int i = 0; i < 3; ++i) {
        float di = comp(nr.dir, i), oi = comp(nr.orig, i);
        if (std::fabs(di) < 0.00001f) continue;
        float t1 = (0.5f - oi) / di;
        float t2 = (-0.5f - oi) / di;
        float t;
        if (t1 >= 0.0f && t2 >= 0.0f) t = std::fmin(t1, t2); else t = std::fmax(t1, t2);
        if (t > smallest_t || t > tmax || t < tmin) continue;
        float f = max_val(vabs(ray_at(nr, t)));
        bool is_solution = std::fabs(f - 0.5f) <= 0.00001f;
        if (!is_solution) continue;
        smallest_t = t; idx = i;
    }
    if (idx < 0) return false;
    V3 lp = ray_at(nr, smallest_t);
    V3 axis = idx == 0 ? v3(1, 0, 0) : (idx == 1 ? v3(0, 1, 0) : v3(0, 0, 1));
    V3 ln = axis * std::copysign(1.0f, comp(ray_at(nr, smallest_t), idx));
    hr.point = m4_dot_p3(cb.l2w, lp);
    hr.normal = m4_dot_v3(cb.l2w, ln);
    hr.material = cb.mat; hr.t = smallest_t; hr.obj_id = cb.id;
    return true;
}

static inline void ray_plane_intersect(const Ray& r, V3 n, V3 c, float& root, float& ndd) {  // traced.rs:92-99
    float div = dot(n, r.dir);
    if (std::fabs(div) < 0.000001f) { root = INF_F; ndd = 0.0f; return; }
    float num = -dot(n, r.orig - c);
    root = num / div; ndd = div;
}
static inline V3 normal_against_direction(V3 n, float ndd) { return n * std::copysign(1.0f, -ndd); }  // traced.rs:101-103

static bool plane_hit(const Plane& p, const Ray& r, float tmin, float tmax, HitRecord& hr) {  // traced.rs:106-114
    float root, ndd; ray_plane_intersect(r, p.normal, p.center, root, ndd);
    if (root == INF_F || root < tmin || root > tmax) return false;
    hr.normal = normal_against_direction(p.normal, ndd);
    hr.point = ray_at(r, root);
    hr.material = p.mat; hr.t = root; hr.obj_id = p.id;
    return true;
}

static bool bary_hit(const Bary& b, bool triangle, const Ray& r, float tmin, float tmax, HitRecord& hr) {  // traced.rs:176-200
    float root, ndd; ray_plane_intersect(r, b.uxv, b.origin, root, ndd);
    if (root == INF_F || root < tmin || root > tmax) return false;
    V3 point = ray_at(r, root);
    V3 pfo = point - b.origin;
    V3 c2 = m3_dot(b.base_inv, pfo);
    // calc_barycentric traced.rs:156-167
    float rx = c2.x, ry = c2.z, ux = 1.0f, uy = 0.0f, vx = b.v_in_base.x, vy = b.v_in_base.z;
    float det = ux * vy - vx * uy;
    float l1 = ((rx * vy - vx * ry) / det) / b.u_length;
    float l2 = (-(rx * uy - ux * ry) / det) / b.v_length;
    float l3 = 1.0f - l1 - l2;
    bool ok = triangle ? (l1 > 0.0f && l2 > 0.0f && l3 > 0.0f && l1 < 1.0f && l2 < 1.0f && l3 < 1.0f)   // :169-171
                       : (l1 > 0.0f && l2 > 0.0f && l1 < 1.0f && l2 < 1.0f);                          // :173-175
    if (!ok) return false;
    hr.normal = normal_against_direction(b.uxv, ndd);
    hr.point = point; hr.material = b.mat; hr.t = root; hr.obj_id = b.id;
    return true;
}

static Bary bary_new(V3 origin, V3 u, V3 v, float ul, float vl, const Material& m) {        // traced.rs:135-147
    Bary b;
    V3 uu = unit(u), vu = unit(v);
    V3 uxv = unit(cross(uu, vu));
    V3 uxvxu = unit(cross(uxv, uu));
    b.base_inv = m3_transpose(m3_cols(uu, uxv, uxvxu));
    b.v_in_base = m3_dot(b.base_inv, vu);
    b.origin = origin; b.u = uu; b.v = vu; b.u_length = ul; b.v_length = vl; b.uxv = uxv; b.uxvxu = uxvxu;
    b.mat = m; b.id = 0;
    return b;
}
static Bary bary_new3(V3 o, V3 up, V3 vp, const Material& m) {                              // traced.rs:148-154
    V3 ur = up - o; float ul = length(ur);
    V3 vr = vp - o; float vl = length(vr);
    return bary_new(o, ur, vr, ul, vl, m);
}

// ----------------------------------------------------------------------------
// marched.rs
// ----------------------------------------------------------------------------
struct MSphere { V3 center; float radius; Material mat; uint64_t id; };                      // marched.rs:50-54
struct MBox { V3 center, sizes; Material mat; uint64_t id; };                                // marched.rs:79-83
struct MTorus { M4 l2w_tr, w2l_tr; V4 l2w_s, w2l_s; V3 sizes; Material mat; uint64_t id; };  // marched.rs:105-113

static inline V4 center_to_local(V3 c, V4 p) { return p - p.w * v4_v3(c); }                 // marched.rs:67-69, 93-95
static inline V4 center_to_world(V3 c, V4 p) { return p + p.w * v4_v3(c); }                 // marched.rs:70-72, 96-98
static inline float msphere_local_sdf(const MSphere& s, V3 p) { return length(p) - s.radius; }  // :57-59
static inline float mbox_local_sdf(const MBox& b, V3 p) {                                    // :86-89
    V3 q = vabs(p) - b.sizes;
    return length(vmax(q, v3(0, 0, 0))) + std::fmin(std::fmax(q.x, std::fmax(q.y, q.z)), 0.0f);
}
static inline float mtorus_local_sdf(const MTorus& t, V3 p) {                                // :134-138
    V3 q = v3(length(v3(p.x, p.z, 0.0f)) - t.sizes.x, p.y, 0.0f);
    return length(q) - t.sizes.y;
}
static inline V4 mtorus_to_local(const MTorus& t, V4 p) { return m4_dot(t.w2l_tr, p * t.w2l_s); }   // :142-144
static inline V4 mtorus_to_world(const MTorus& t, V4 p) { return m4_dot(t.l2w_tr, p) * t.l2w_s; }   // :145-147
static inline float mtorus_to_world_f(const MTorus& t, float f) { return f * min_val(xyz(t.l2w_s)); }  // :148-150

// Marched::sdf marched.rs:14-18
static inline float msphere_sdf(const MSphere& s, V3 p) { return msphere_local_sdf(s, xyz(center_to_local(s.center, v4_p3(p)))); }
static inline float mbox_sdf(const MBox& b, V3 p) { return mbox_local_sdf(b, xyz(center_to_local(b.center, v4_p3(p)))); }
static inline float mtorus_sdf(const MTorus& t, V3 p) { return mtorus_to_world_f(t, mtorus_local_sdf(t, xyz(mtorus_to_local(t, v4_p3(p))))); }

// Marched::get_outward_local_normal marched.rs:25-44 (generic over the local sdf)
template <class F>
static V3 outward_local_normal(F local_sdf, V3 p) {
    const float eps = 0.0000001f;
    V3 ex = v3(eps, 0.0f, 0.0f), ey = v3(0.0f, eps, 0.0f), ez = v3(0.0f, 0.0f, eps);
    float x = local_sdf(p + ex) - local_sdf(p - ex);
    float y = local_sdf(p + ey) - local_sdf(p - ey);
    float z = local_sdf(p + ez) - local_sdf(p - ez);
    V3 normal = unit(v3(x, y, z));
    Ray tr = ray_new(v3(0, 0, 0), normal);
    V3 start = ray_at(tr, 0.0f);
    float start_val = local_sdf(start);
    V3 end = ray_at(tr, 1.0f);
    float end_val = local_sdf(end);
    float sign = (end_val > start_val) ? 1.0f : -1.0f;
    return normal * sign;
}
// MarchedSphere overrides get_outward_normal: marched.rs:60-63
static inline V3 msphere_normal(const MSphere& s, V3 p) { return unit(p - s.center); }
// default get_outward_normal marched.rs:19-24
static V3 mbox_normal(const MBox& b, V3 p) {
    V3 lp = xyz(center_to_local(b.center, v4_p3(p)));
    V4 n = v4_v3(outward_local_normal([&](V3 q) { return mbox_local_sdf(b, q); }, lp));
    return unit(xyz(center_to_world(b.center, n)));
}
static V3 mtorus_normal(const MTorus& t, V3 p) {
    V3 lp = xyz(mtorus_to_local(t, v4_p3(p)));
    V4 n = v4_v3(outward_local_normal([&](V3 q) { return mtorus_local_sdf(t, q); }, lp));
    return unit(xyz(mtorus_to_world(t, n)));
}
static MTorus mtorus_new(const M4& l2w, V3 sizes, const Material& m) {                       // marched.rs:116-130
    M4 t, r, s; m4_decompose_trs(l2w, t, r, s);
    M4 tr = m4_dot_mat(t, r);
    V4 sc = m4_diag(s);
    MTorus o;
    o.l2w_tr = tr; o.w2l_tr = m4_fast_homogenous_inverse(tr);
    o.l2w_s = sc; o.w2l_s = v4(1.0f / sc.x, 1.0f / sc.y, 1.0f / sc.z, 1.0f / sc.w);
    o.sizes = sizes; o.mat = m; o.id = 0;
    return o;
}

// A user marched object (`HittableList += Arc<dyn Marched>`, hits.rs:96-100), the form the product
// accepts (om_world_add_marched_sdf, include/ottomarcher.h): MarchedTorus's transform and default
// trait methods (marched.rs:14-44, 139-151) around a local_sdf given as a postfix program.
struct MSdfOp { int32_t op; float a[7]; };
struct MSdf { MTorus xf; std::vector<MSdfOp> ops; Material mat; uint64_t id; };
enum { SDF_SPHERE = 1, SDF_BOX = 2, SDF_TORUS = 3, SDF_UNION = 4, SDF_INTERSECT = 5, SDF_SUBTRACT = 6, SDF_ROUND = 7 };
static float msdf_local_sdf(const MSdf& q, V3 p) {
    float st[8]; int sp = 0;
    for (const MSdfOp& o : q.ops) {
        V3 c = v3(o.a[0], o.a[1], o.a[2]);
        float v;
        if (o.op == SDF_SPHERE) v = length(p - c) - o.a[3];                                  // as marched.rs:57-59
        else if (o.op == SDF_BOX) {                                                          // as marched.rs:86-89
            V3 b = vabs(p - c) - v3(o.a[3], o.a[4], o.a[5]);
            v = length(vmax(b, v3(0, 0, 0))) + std::fmin(std::fmax(b.x, std::fmax(b.y, b.z)), 0.0f);
        } else if (o.op == SDF_TORUS) {                                                      // as marched.rs:134-138
            V3 pc = p - c;
            V3 t = v3(length(v3(pc.x, pc.z, 0.0f)) - o.a[3], pc.y, 0.0f);
            v = length(t) - o.a[4];
        } else if (o.op == SDF_ROUND) v = st[--sp] - o.a[0];
        else {
            float b = st[--sp], a = st[--sp];
            v = o.op == SDF_UNION ? std::fmin(a, b) : o.op == SDF_INTERSECT ? std::fmax(a, b) : std::fmax(a, -b);
        }
        st[sp++] = v;
    }
    return st[0];
}
static inline float msdf_sdf(const MSdf& q, V3 p) { return mtorus_to_world_f(q.xf, msdf_local_sdf(q, xyz(mtorus_to_local(q.xf, v4_p3(p))))); }
static V3 msdf_normal(const MSdf& q, V3 p) {                                                 // default get_outward_normal
    V3 lp = xyz(mtorus_to_local(q.xf, v4_p3(p)));
    V4 n = v4_v3(outward_local_normal([&](V3 x) { return msdf_local_sdf(q, x); }, lp));
    return unit(xyz(mtorus_to_world(q.xf, n)));
}

// ----------------------------------------------------------------------------
// hits.rs: HittableList / FrozenHittableList::hit / unstuck
// ----------------------------------------------------------------------------
static const float HIT_SIZE = 0.001f;                                                        // hits.rs:113
struct World {
    // typed vecs in the reference order hits.rs:370-371
    std::vector<Sphere> spheres; std::vector<Cube> cubes; std::vector<Bary> triangles;
    std::vector<Plane> planes; std::vector<Bary> parallelograms;
    std::vector<MSphere> msph; std::vector<MBox> mbox; std::vector<MTorus> mtor;
    std::vector<MSdf> msdf;                                                                  // Arc<dyn Marched>, after the typed ones
    uint32_t march_steps = 1024;                                                             // hits.rs:292
    // obj_id = global type-order index + 1 (0 = sky); replaces the memory address of utils.rs:110.
    void assign_ids() {
        uint64_t k = 1;
        for (auto& o : spheres) o.id = k++;
        for (auto& o : cubes) o.id = k++;
        for (auto& o : triangles) o.id = k++;
        for (auto& o : planes) o.id = k++;
        for (auto& o : parallelograms) o.id = k++;
        for (auto& o : msph) o.id = k++;
        for (auto& o : mbox) o.id = k++;
        for (auto& o : mtor) o.id = k++;
        for (auto& o : msdf) o.id = k++;
    }
    bool has_marched() const { return !msph.empty() || !mbox.empty() || !mtor.empty() || !msdf.empty(); }
};

// 0 = sphere, 1 = box, 2 = torus, 3 = user object
static inline float marched_sdf_abs(const World& w, int kind, size_t i, V3 p) {
    if (kind == 0) return std::fabs(msphere_sdf(w.msph[i], p));
    if (kind == 1) return std::fabs(mbox_sdf(w.mbox[i], p));
    if (kind == 3) return std::fabs(msdf_sdf(w.msdf[i], p));
    return std::fabs(mtorus_sdf(w.mtor[i], p));
}

static const uint64_t UNSTUCK_CAP = 1u << 22;  // safety cap (not in the reference); see DESIGN.md

static float unstuck(const World& w, float t, const Ray& r) {                                // hits.rs:336-365
    const float MIN_STEP = HIT_SIZE / 2.0f;
    float new_t = t; float d = INF_F;
    V3 p = ray_at(r, t);
    int kind = -1; size_t idx = 0;
    for (size_t i = 0; i < w.msph.size(); ++i) { float nd = marched_sdf_abs(w, 0, i, p); if (nd < d) { d = nd; kind = 0; idx = i; } }
    for (size_t i = 0; i < w.mbox.size(); ++i) { float nd = marched_sdf_abs(w, 1, i, p); if (nd < d) { d = nd; kind = 1; idx = i; } }
    for (size_t i = 0; i < w.mtor.size(); ++i) { float nd = marched_sdf_abs(w, 2, i, p); if (nd < d) { d = nd; kind = 2; idx = i; } }
    for (size_t i = 0; i < w.msdf.size(); ++i) { float nd = marched_sdf_abs(w, 3, i, p); if (nd < d) { d = nd; kind = 3; idx = i; } }   // hits.rs:350-356
    float aux = d;
    if (kind < 0) return INF_F;
    uint64_t guard = 0;
    while (aux < HIT_SIZE && guard++ < UNSTUCK_CAP) {
        new_t += MIN_STEP;
        aux = marched_sdf_abs(w, kind, idx, ray_at(r, new_t));
    }
    return new_t;
}

static bool world_hit(const World& w, const Ray& r, float tmin, float tmax, HitRecord& rec) {  // hits.rs:270-334
    float closest = tmax; bool have = false; HitRecord hr;
    for (auto& o : w.spheres) if (sphere_hit(o, r, tmin, closest, hr)) { closest = hr.t; rec = hr; have = true; }
    for (auto& o : w.cubes) if (cube_hit(o, r, tmin, closest, hr)) { closest = hr.t; rec = hr; have = true; }
    for (auto& o : w.triangles) if (bary_hit(o, true, r, tmin, closest, hr)) { closest = hr.t; rec = hr; have = true; }
    for (auto& o : w.planes) if (plane_hit(o, r, tmin, closest, hr)) { closest = hr.t; rec = hr; have = true; }
    for (auto& o : w.parallelograms) if (bary_hit(o, false, r, tmin, closest, hr)) { closest = hr.t; rec = hr; have = true; }
    // (Arc<dyn Traced> objects hits.rs:280-285 are not representable across the C-ABI.)
    float t = unstuck(w, tmin, r);                                                           // hits.rs:288
    if (std::isinf(t)) return have;
    uint32_t iters = w.march_steps;
    while (t < tmax && t < closest && iters > 0) {                                           // hits.rs:294
        iters -= 1;
        V3 point = ray_at(r, t);
        float distance = INF_F; int kind = -1; size_t idx = 0;
        for (size_t i = 0; i < w.msph.size(); ++i) { float d = marched_sdf_abs(w, 0, i, point); if (d < distance) { distance = d; kind = 0; idx = i; } }
        for (size_t i = 0; i < w.mbox.size(); ++i) { float d = marched_sdf_abs(w, 1, i, point); if (d < distance) { distance = d; kind = 1; idx = i; } }
        for (size_t i = 0; i < w.mtor.size(); ++i) { float d = marched_sdf_abs(w, 2, i, point); if (d < distance) { distance = d; kind = 2; idx = i; } }
        for (size_t i = 0; i < w.msdf.size(); ++i) { float d = marched_sdf_abs(w, 3, i, point); if (d < distance) { distance = d; kind = 3; idx = i; } }   // hits.rs:312-319
        if (kind < 0) return have;                                                           // hits.rs:323
        if (distance < HIT_SIZE) {                                                           // hits.rs:325-327
            rec.t = t; rec.point = point;
            // the normal recomputed at every improvement (hits.rs:302-309) is a pure
            // function of (object, point): evaluating it once for the winner is identical.
            if (kind == 0) { rec.normal = msphere_normal(w.msph[idx], point); rec.material = w.msph[idx].mat; rec.obj_id = w.msph[idx].id; }
            else if (kind == 1) { rec.normal = mbox_normal(w.mbox[idx], point); rec.material = w.mbox[idx].mat; rec.obj_id = w.mbox[idx].id; }
            else if (kind == 2) { rec.normal = mtorus_normal(w.mtor[idx], point); rec.material = w.mtor[idx].mat; rec.obj_id = w.mtor[idx].id; }
            else { rec.normal = msdf_normal(w.msdf[idx], point); rec.material = w.msdf[idx].mat; rec.obj_id = w.msdf[idx].id; }
            return true;
        }
        t += distance;                                                                       // hits.rs:330
    }
    return have;
}

// ----------------------------------------------------------------------------
// materials.rs scatter
// ----------------------------------------------------------------------------
static inline V3 reflect(V3 v, V3 n) { return v - (2.0f * dot(v, n)) * n; }                 // materials.rs:98-100
static inline V3 refract(V3 uv, V3 n, float eta) {                                           // materials.rs:102-108
    float cos_theta = std::fmin(dot(-uv, n), 1.0f);
    V3 r_out_perp = eta * (uv + cos_theta * n);
    float aux = -std::sqrt(std::fabs(1.0f - length_squared(r_out_perp)));
    V3 r_out_parallel = aux * n;
    return r_out_perp + r_out_parallel;
}
static inline float reflectance(float cosv, float ref_idx) {                                 // materials.rs:110-116
    float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    float r0_2 = r0 * r0;
    float cos_5 = (1.0f - cosv) * (1.0f - cosv) * (1.0f - cosv) * (1.0f - cosv) * (1.0f - cosv);
    return r0_2 + (1.0f - r0_2) * cos_5;
}
static void scatter(const Ray& r_in, const HitRecord& hr, PathRng& g, V3& atten, Ray& out) {   // materials.rs:39-51
    const Material& m = hr.material;
    if (m.type == MAT_LAMBERTIAN) {                                                          // :52-61
        V3 nd = hr.normal + rand_unit_vector(g);
        if (near_zero(nd)) nd = hr.normal;
        out = ray_new(hr.point, nd); atten = albedo(m);
    } else if (m.type == MAT_METAL) {                                                        // :62-66
        V3 refl = reflect(r_in.dir, hr.normal);
        out = ray_new(hr.point, refl + m.fuzz * rand_in_unit_sphere(g)); atten = albedo(m);
    } else {                                                                                 // :68-95
        V3 du = r_in.dir;
        bool front = dot(du, hr.normal) < 0.0f;
        float rr; V3 n;
        if (front) { rr = 1.0f / m.ior; n = hr.normal; } else { rr = m.ior; n = -hr.normal; }
        float cos_theta = std::fmin(dot(-du, n), 1.0f);
        float sin_theta = std::sqrt(1.0f - cos_theta * cos_theta);
        bool cannot = (rr * sin_theta) > 1.0f;
        bool by_refl = reflectance(cos_theta, rr) > g.rand();                               // rand always drawn
        V3 nd = (cannot || by_refl) ? reflect(du, n) : refract(du, n, rr);
        out = ray_new(hr.point, nd); atten = v3(1.0f, 1.0f, 1.0f);
    }
}

// ----------------------------------------------------------------------------
// camera.rs
// ----------------------------------------------------------------------------
struct Camera { V3 origin, horizontal, vertical, llc, u, v, w; float lens_radius, aspect, focus, vw, vh; };  // camera.rs:10-29
static Camera camera_new(V3 lookfrom, V3 lookat, V3 vup, float vfov_deg, float aspect, float aperture, float focus) {  // :38-59
    float vfov = vfov_deg * PI_F / 180.0f;                                                   // utils.rs:33-35
    float height = std::tan(vfov / 2.0f) * focus;
    float vh = 2.0f * height;
    float vw = vh * aspect;
    V3 w = unit(lookfrom - lookat);
    V3 u = unit(cross(vup, w));
    V3 v = unit(cross(w, u));
    Camera c;
    c.origin = lookfrom; c.horizontal = vw * u; c.vertical = vh * v;
    c.llc = c.origin - c.horizontal / 2.0f - c.vertical / 2.0f - focus * w;
    c.u = u; c.v = v; c.w = w; c.lens_radius = aperture / 2.0f; c.aspect = aspect; c.focus = focus; c.vw = vw; c.vh = vh;
    return c;
}
static Ray camera_get_ray(const Camera& c, float s, float t, PathRng& g) {                      // camera.rs:60-65
    V3 rl = c.lens_radius * rand_in_unit_disc(g);
    V3 offset = c.u * rl.x + c.v * rl.y;
    // uv_to_dir camera.rs:67-74 = cols (H, V, 0, llc-origin); dot with (u, v, 0, 1)
    M4 m = m4_cols(v4_v3(c.horizontal), v4_v3(c.vertical), v4(0, 0, 0, 0), v4_p3(c.llc - c.origin));
    V3 direction = xyz(m4_dot(m, v4(s, t, 0.0f, 1.0f)));
    return ray_new(c.origin + offset, unit(direction - offset));
}

// ----------------------------------------------------------------------------
// utils.rs: lerp, normalize_color, scramble, BloomFilter
// ----------------------------------------------------------------------------
static inline V3 lerp(float t, V3 c1, V3 c2) { return (1.0f - t) * c1 + t * c2; }           // utils.rs:9-11
static inline float clampf(float x, float mn, float mx) { return std::fmin(std::fmax(x, mn), mx); }  // utils.rs:4-6
static inline V3 normalize_color(V3 c) {                                                     // utils.rs:12-17
    return v3(clampf(std::sqrt(c.x), 0.0f, 0.999f), clampf(std::sqrt(c.y), 0.0f, 0.999f), clampf(std::sqrt(c.z), 0.0f, 0.999f));
}
static inline uint64_t scramble(uint64_t id) {                                               // utils.rs:46-56
    uint64_t id1 = id & 0xFFFFFFFFULL;
    id1 ^= id1 << 13; id1 ^= id1 >> 7; id1 ^= id1 << 17;
    uint64_t id2 = id >> 32;
    id2 ^= id2 << 13; id2 ^= id2 >> 17; id2 ^= id2 << 5;
    return (id2 << 32) ^ id1 ^ (id1 * id2);
}
static inline uint64_t madd(uint64_t x, uint64_t m, uint64_t a) { return x * m + a; }       // utils.rs:71-73
static uint64_t bloom_hash(uint64_t id) {                                                    // utils.rs:94-107
    uint64_t ret = 0, bit = (id != 0) ? 1 : 0;
    ret |= bit << (scramble(madd(id, 456894789ULL, 348764781ULL) % 17287318477382145149ULL) % 64);
    ret |= bit << (scramble(madd(id, 56456ULL, 2345ULL) % 10520185020478678957ULL) % 64);
    ret |= bit << (scramble(madd(id, 12337ULL, 7878ULL) % 6100366985798845493ULL) % 64);
    ret |= bit << (scramble(madd(id, 7438554325ULL, 2554ULL) % 2581451885731034521ULL) % 64);
    ret |= bit << (scramble(madd(id, 12345ULL, 123123044ULL) % 2015400956511055807ULL) % 64);
    ret |= bit << (scramble(madd(id, 6373412378ULL, 12452ULL) % 8800267423223100703ULL) % 64);
    ret |= bit << (scramble(madd(id, 3453453ULL, 7874856378ULL) % 7039701875810786467ULL) % 64);
    ret |= bit << (scramble(madd(id, 999465ULL, 143ULL) % 3008457310659543551ULL) % 64);
    ret |= bit << (scramble(madd(id, 14444ULL, 111345ULL) % 5935720376112203207ULL) % 64);
    return ret;
}

// ----------------------------------------------------------------------------
// render_thread.rs
// ----------------------------------------------------------------------------
struct PixelStats {            // 40 B, same layout as om_pixel_stats
    uint64_t bloom; float sum[3]; uint32_t n; float avg_depth; uint32_t bad_avgs; uint8_t color[3]; uint8_t flags; uint32_t pad;
};
static_assert(sizeof(PixelStats) == 40, "layout");

// Stats::add render_thread.rs:23-39; returns `done`
static bool stats_add(PixelStats& st, V3 x, float depth, uint64_t obj_id) {
    uint8_t old[3] = {st.color[0], st.color[1], st.color[2]};
    st.sum[0] = st.sum[0] + x.x; st.sum[1] = st.sum[1] + x.y; st.sum[2] = st.sum[2] + x.z;
    st.n += 1;
    V3 avg = v3(st.sum[0], st.sum[1], st.sum[2]) / (float)st.n;
    to_u8x3(normalize_color(avg), st.color);
    uint32_t bad_run = (old[0] == st.color[0]) && (old[1] == st.color[1]) && (old[2] == st.color[2]);
    st.bad_avgs += bad_run;
    st.bad_avgs *= bad_run;
    float nf = (float)st.n;
    st.avg_depth = ((nf - 1.0f) * st.avg_depth + depth) / nf;
    st.bloom |= bloom_hash(obj_id);
    bool done = st.bad_avgs >= 5;
    if (done) st.flags |= 1;
    return done;
}


// ----------------------------------------------------------------------------
// main.rs:219-437 — the draw_to_sdl view modes over the pixel Stats (RGB24 out).
// Pixels apply_box_filter does not reach (W or H == 2: main.rs:322-341 loops) keep
// the caller's previous bytes, as the reference's persistent sdlpixels buffer does.
// ----------------------------------------------------------------------------
static const float SQRT2_INV_F = 0.7071067811865475244f;                                    // utils.rs:31
static inline V3 stats_sum(const PixelStats& p) { return v3(p.sum[0], p.sum[1], p.sum[2]); }
static inline void put_rgb(uint8_t* rgb, size_t px, V3 c) { to_u8x3(normalize_color(c), rgb + 3 * px); }
static inline void u64_to_color(uint64_t id, uint8_t* o) {                                  // utils.rs:59-70
    uint8_t b[8];
    for (int k = 0; k < 8; ++k) b[k] = (uint8_t)((id >> (8 * k)) & 0xFF);
    o[0] = b[0] ^ b[7] ^ b[3]; o[1] = b[1] ^ b[4] ^ b[5]; o[2] = b[2] ^ b[6];
}
// apply_box_filter_ij_samples / _depth / _id (main.rs:219-312)
static void box_filter_ij(int mode, const PixelStats* P, uint32_t W, uint8_t* rgb, uint32_t i, uint32_t j,
                          int min_x, int max_x, int min_y, int max_y) {
    const size_t me = (size_t)i + (size_t)j * W;
    const float di = P[me].avg_depth;
    if (mode == 1 && std::isinf(di)) {                                                      // :250-257
        std::memcpy(rgb + 3 * me, P[me].color, 3);
        return;
    }
    const uint64_t state = P[me].bloom;
    float total_weight = 0.0f;
    V3 color = v3(0.0f, 0.0f, 0.0f);
    for (int y = min_y; y <= max_y; ++y) {
        for (int x = min_x; x <= max_x; ++x) {
            const PixelStats& q = P[(size_t)((int)i + x) + (size_t)((int)j + y) * W];
            const float is_diagonal = (x != 0 && y != 0) ? 1.0f : 0.0f;
            if (mode == 0) {
                const float n = (float)q.n;
                const float diag_w = 1.0f - (1.0f - SQRT2_INV_F) * is_diagonal;
                total_weight = total_weight + n * diag_w;
                color = color + stats_sum(q) * diag_w;
            } else {
                float w;
                if (mode == 1) {
                    w = 1.0f / (1.0f + std::fabs(q.avg_depth - di));
                } else {
                    const float same_value = (q.bloom == state) ? 1.0f : 0.0f;
                    const float partial_value = ((q.bloom & state) == state) ? 1.0f : 0.0f;
                    w = same_value + partial_value;
                }
                const float diag_w = w * (1.0f - (1.0f - SQRT2_INV_F) * is_diagonal);
                total_weight = total_weight + diag_w;
                const V3 c = stats_sum(q) / (float)q.n;
                color = color + diag_w * c;
            }
        }
    }
    put_rgb(rgb, me, color / total_weight);
}
// apply_box_filter::<MODE> (main.rs:322-343), same visiting pattern
static void box_filter(int mode, const PixelStats* P, uint32_t H, uint32_t W, uint8_t* rgb) {
    for (uint32_t j = 1; j + 1 < H; ++j) {
        for (uint32_t i = 1; i + 1 < W; ++i) {
            if (j == 1) {
                box_filter_ij(mode, P, W, rgb, i, 0, -1, 1, 0, 1);
                box_filter_ij(mode, P, W, rgb, i, H - 1, -1, 1, -1, 0);
            }
            box_filter_ij(mode, P, W, rgb, i, j, -1, 1, -1, 1);
        }
        box_filter_ij(mode, P, W, rgb, 0, j, 0, 1, -1, 1);
        box_filter_ij(mode, P, W, rgb, W - 1, j, -1, 0, -1, 1);
    }
    box_filter_ij(mode, P, W, rgb, 0, 0, 0, 1, 0, 1);
    box_filter_ij(mode, P, W, rgb, W - 1, 0, -1, 0, 0, 1);
    box_filter_ij(mode, P, W, rgb, 0, H - 1, 0, 1, -1, 0);
    box_filter_ij(mode, P, W, rgb, W - 1, H - 1, -1, 0, -1, 0);
}
// draw_to_sdl's mode switch (main.rs:372-437)
static void display(const PixelStats* P, uint32_t W, uint32_t H, int mode, uint8_t* rgb) {
    const size_t N = (size_t)W * H;
    if (mode == 0) {                                                                        // MODE_NORMAL
        for (size_t k = 0; k < N; ++k) std::memcpy(rgb + 3 * k, P[k].color, 3);
    } else if (mode == 1) {                                                                 // MODE_SHOW_SAMPLES
        uint32_t max_samples = 1;
        for (size_t k = 0; k < N; ++k) if (P[k].n > max_samples) max_samples = P[k].n;
        for (size_t k = 0; k < N; ++k) {
            const float s = (float)P[k].n / (float)max_samples;
            put_rgb(rgb, k, v3(s, s, s));
        }
    } else if (mode == 3) {                                                                 // MODE_SHOW_DEPTH
        float max_depth = -1.0f;
        for (size_t k = 0; k < N; ++k) {
            const float d = P[k].avg_depth;
            if (d > max_depth && !std::isinf(d)) max_depth = d;
        }
        for (size_t k = 0; k < N; ++k) {
            const float d01 = P[k].avg_depth / max_depth;
            const bool is_inf = std::isinf(d01);
            const float rb = is_inf ? 0.0f : d01, g = is_inf ? 1.0f : d01;
            put_rgb(rgb, k, v3(rb, g, rb));
        }
    } else if (mode == 5) {                                                                 // MODE_SHOW_IDS
        for (size_t k = 0; k < N; ++k) u64_to_color(scramble(P[k].bloom), rgb + 3 * k);
    } else {                                                                                // 2 / 4 / 6: blurs
        box_filter(mode == 2 ? 0 : (mode == 4 ? 1 : 2), P, H, W, rgb);
    }
}

// handle_hit render_thread.rs:105-126 ; ray_color :128-143
struct SampleResult { V3 color; float depth; uint64_t id; uint32_t segments; };
static inline bool handle_hit(const World& w, Ray& r, V3& cur, float tmin, float tmax, PathRng& g, float& depth, uint64_t& id) {
    HitRecord hr;
    if (world_hit(w, r, tmin, tmax, hr)) {
        V3 att; Ray nr; scatter(r, hr, g, att, nr);
        cur = cur * att; r = nr; depth = hr.t; id = hr.obj_id;
    } else {
        float t = 0.5f * (r.dir.y + 1.0f);                                                   // :118
        cur = cur * lerp(t, v3(1.0f, 1.0f, 1.0f), v3(0.5f, 0.7f, 1.0f));                     // :119-120
        depth = INF_F; id = 0;
    }
    return true;
}
static SampleResult ray_color(const World& w, Ray r, uint32_t depth, float tmin, float tmax, PathRng& g) {
    SampleResult out; V3 cur = v3(1.0f, 1.0f, 1.0f); out.segments = 1;
    float depthf; uint64_t obj_id;
    handle_hit(w, r, cur, tmin, tmax, g, depthf, obj_id);                                    // :132 (first_hit == hit, F5)
    if (std::isinf(depthf)) { out.color = cur; out.depth = INF_F; out.id = 0; return out; }  // :133-135
    for (uint32_t i = 1; i < depth; ++i) {                                                   // :136
        float h; uint64_t hid; out.segments++;
        handle_hit(w, r, cur, tmin, tmax, g, h, hid);                                        // :137
        if (std::isinf(h)) { out.color = cur; out.depth = depthf; out.id = obj_id; return out; }  // :138-140
    }
    out.color = -v3(0.0f, 0.0f, 0.0f); out.depth = depthf; out.id = obj_id;                  // :142  -Color::ZERO
    return out;
}

struct RenderParams {          // mirrors om_render_params
    uint32_t width, height, spp_total, sample_begin, sample_count, max_depth;
    float tmin, tmax;
    uint32_t march_steps, adaptive;
    uint64_t seed;
};

static std::vector<float> jitter_table(uint64_t seed, uint32_t spp) {                       // render_thread.rs:164-174
    std::vector<float> jt(2 * (size_t)spp);
    for (uint32_t s = 0; s < spp; ++s) { jt[2 * s] = (float)((s / 2) & 1); jt[2 * s + 1] = (float)(s & 1); }
    Rng g; g.s = mix64(seed ^ 0x4A177E5B0C1D2E3FULL);
    for (uint32_t i = spp; i-- > 1;) {   // Fisher-Yates, i = spp-1 .. 1
        uint32_t j = (uint32_t)((g.next_u64() >> 32) % (uint64_t)(i + 1));
        std::swap(jt[2 * i], jt[2 * j]); std::swap(jt[2 * i + 1], jt[2 * j + 1]);
    }
    return jt;
}

struct Counters { uint64_t samples, segments, credited; };

// One pixel, samples [sample_begin, sample_begin+sample_count) — render_thread.rs:176-199
static void render_pixel(const World& w, const Camera& cam, const RenderParams& p, const float* jt, uint64_t skey,
                         uint32_t pxl, PixelStats& st, Counters& ctr) {
    uint32_t line = pxl / p.width, col = pxl - p.width * line;
    float j_f = (float)line, i_f = (float)col;
    float wf = (float)p.width, hf = (float)p.height;
    for (uint32_t k = 0; k < p.sample_count; ++k) {
        if (p.adaptive && (st.flags & 1)) break;                                             // ThreadPixels::add_run :97-101
        uint32_t s = st.n;
        if (s >= p.spp_total) break;
        PathRng g = path_rng(skey, pxl, s);
        float i_rand = (g.rand() + jt[2 * s]) / 2.0f;                                        // :188
        float j_rand = (g.rand() + jt[2 * s + 1]) / 2.0f;                                    // :189
        float u = (i_f + i_rand) / (wf - 1.0f);                                              // :190
        float v = 1.0f - (j_f + j_rand) / (hf - 1.0f);                                       // :191
        Ray r = camera_get_ray(cam, u, v, g);                                                // :192
        SampleResult sr = ray_color(w, r, p.max_depth, p.tmin, p.tmax, g);                   // :193
        bool done = stats_add(st, sr.color, sr.depth, sr.id);                                // :194
        ctr.samples += 1; ctr.segments += sr.segments;
        ctr.credited += (uint64_t)((done && p.adaptive) ? (p.spp_total - st.n) : 0) + 1;     // :196-198
    }
}

}  // namespace oro

// ============================================================================
// extern "C" surface for ctypes (tests / bench cpu_baseline only)
// ============================================================================
using namespace oro;

struct OroMaterial { float albedo[3]; float fuzz; float ior; int32_t type; };
struct OroCamera { float origin[3], horizontal[3], vertical[3], llc[3], u[3], v[3], w[3]; float lens_radius, aspect, focus, vw, vh; };

static inline Material to_mat(const OroMaterial* m) { Material o; std::memcpy(&o, m, sizeof(o)); return o; }
static inline V3 ld3(const float* f) { return v3(f[0], f[1], f[2]); }
static inline void st3(V3 a, float* f) { f[0] = a.x; f[1] = a.y; f[2] = a.z; }

extern "C" {

int oro_abi_version() { return 1; }

void* oro_world_new() { return new World(); }
void oro_world_free(void* w) { delete (World*)w; }
void oro_world_set_march_steps(void* w, uint32_t n) { ((World*)w)->march_steps = n; }

void oro_world_add_sphere(void* w, const float* l2w, const OroMaterial* m) {                 // traced.rs:22-25
    Sphere s; s.l2w = m4_load(l2w); s.w2l = m4_fast_homogenous_inverse(s.l2w); s.mat = to_mat(m); s.id = 0;
    ((World*)w)->spheres.push_back(s);
}
void oro_world_add_sphere_radius(void* w, const float* c, float r, const OroMaterial* m) {   // traced.rs:26-31
    Sphere s; s.l2w = m4_dot_mat(m4_translate(ld3(c)), m4_scale(v3(r, r, r))); s.w2l = m4_fast_homogenous_inverse(s.l2w);
    s.mat = to_mat(m); s.id = 0; ((World*)w)->spheres.push_back(s);
}
void oro_world_add_cube(void* w, const float* l2w, const OroMaterial* m) {                   // traced.rs:238-240
    Cube s; s.l2w = m4_load(l2w); s.w2l = m4_fast_homogenous_inverse(s.l2w); s.mat = to_mat(m); s.id = 0;
    ((World*)w)->cubes.push_back(s);
}
void oro_world_add_cube_length(void* w, const float* c, float len, const OroMaterial* m) {   // traced.rs:242-246
    Cube s; s.l2w = m4_dot_mat(m4_translate(ld3(c)), m4_scale(v3(len, len, len))); s.w2l = m4_fast_homogenous_inverse(s.l2w);
    s.mat = to_mat(m); s.id = 0; ((World*)w)->cubes.push_back(s);
}
// kind: 0 = parallelogram, 1 = triangle
void oro_world_add_bary3(void* w, int kind, const float* o, const float* up, const float* vp, const OroMaterial* m) {
    Bary b = bary_new3(ld3(o), ld3(up), ld3(vp), to_mat(m));
    if (kind == 1) ((World*)w)->triangles.push_back(b); else ((World*)w)->parallelograms.push_back(b);
}
void oro_world_add_bary(void* w, int kind, const float* o, const float* u, const float* v, float ul, float vl, const OroMaterial* m) {
    Bary b = bary_new(ld3(o), ld3(u), ld3(v), ul, vl, to_mat(m));
    if (kind == 1) ((World*)w)->triangles.push_back(b); else ((World*)w)->parallelograms.push_back(b);
}
void oro_world_add_plane(void* w, const float* c, const float* n, const OroMaterial* m) {    // traced.rs:86-88
    Plane p; p.center = ld3(c); p.normal = unit(ld3(n)); p.mat = to_mat(m); p.id = 0; ((World*)w)->planes.push_back(p);
}
void oro_world_add_marched_sphere(void* w, const float* c, float r, const OroMaterial* m) {
    MSphere s; s.center = ld3(c); s.radius = r; s.mat = to_mat(m); s.id = 0; ((World*)w)->msph.push_back(s);
}
void oro_world_add_marched_box(void* w, const float* c, const float* sz, const OroMaterial* m) {
    MBox b; b.center = ld3(c); b.sizes = ld3(sz); b.mat = to_mat(m); b.id = 0; ((World*)w)->mbox.push_back(b);
}
void oro_world_add_marched_sdf(void* w, const float* l2w, const void* ops, uint32_t n, const OroMaterial* m) {
    MSdf q;
    q.xf = mtorus_new(m4_load(l2w), v3(0, 0, 0), to_mat(m));
    q.ops.assign((const MSdfOp*)ops, (const MSdfOp*)ops + n);
    q.mat = to_mat(m); q.id = 0;
    ((World*)w)->msdf.push_back(q);
}
void oro_world_add_marched_torus(void* w, const float* l2w, const float* sz, const OroMaterial* m) {
    ((World*)w)->mtor.push_back(mtorus_new(m4_load(l2w), ld3(sz), to_mat(m)));
}

// Counts per type, in type order (8 entries).
void oro_world_counts(void* wp, uint32_t* out) {
    World* w = (World*)wp;
    out[0] = (uint32_t)w->spheres.size(); out[1] = (uint32_t)w->cubes.size(); out[2] = (uint32_t)w->triangles.size();
    out[3] = (uint32_t)w->planes.size(); out[4] = (uint32_t)w->parallelograms.size(); out[5] = (uint32_t)w->msph.size();
    out[6] = (uint32_t)w->mbox.size(); out[7] = (uint32_t)w->mtor.size();
}
// Derived (frozen) data for cross-checks with the product's scene builder.
// Affine prims (kind 0 sphere, 1 cube): 32 floats = l2w[16], w2l[16].
void oro_world_affine(void* wp, int kind, uint32_t i, float* out) {
    World* w = (World*)wp;
    if (kind == 0) { m4_store(w->spheres[i].l2w, out); m4_store(w->spheres[i].w2l, out + 16); }
    else { m4_store(w->cubes[i].l2w, out); m4_store(w->cubes[i].w2l, out + 16); }
}
// Barycentric (kind 0 parallelogram, 1 triangle): origin3 u3 ul v3 vl uxv3 uxvxu3 base_inv9 v_in_base3 = 29 floats
void oro_world_bary(void* wp, int kind, uint32_t i, float* out) {
    World* w = (World*)wp; const Bary& b = kind == 1 ? w->triangles[i] : w->parallelograms[i];
    st3(b.origin, out); st3(b.u, out + 3); out[6] = b.u_length; st3(b.v, out + 7); out[10] = b.v_length;
    st3(b.uxv, out + 11); st3(b.uxvxu, out + 14);
    for (int r = 0; r < 3; ++r) st3(b.base_inv.r[r], out + 17 + 3 * r);
    st3(b.v_in_base, out + 26);
}
// Torus: l2w_tr16 w2l_tr16 l2w_s4 w2l_s4 sizes3 = 43 floats
void oro_world_torus(void* wp, uint32_t i, float* out) {
    const MTorus& t = ((World*)wp)->mtor[i];
    m4_store(t.l2w_tr, out); m4_store(t.w2l_tr, out + 16);
    out[32] = t.l2w_s.x; out[33] = t.l2w_s.y; out[34] = t.l2w_s.z; out[35] = t.l2w_s.w;
    out[36] = t.w2l_s.x; out[37] = t.w2l_s.y; out[38] = t.w2l_s.z; out[39] = t.w2l_s.w;
    st3(t.sizes, out + 40);
}

// --- front-end scene builders (main.rs:37-110), with SplitMix64 (om-rng Rng) replacing thread_rng ---
// flags bit0: include the torus block main.rs:73-81 (S-full); S-traced omits it.
// grid_half: 11 for random_scene (a,b in -11..11); 50 gives the S-10k variant (a,b in -50..50).
// flags bit1: omit the parallelogram/triangle/cube blocks (S-10k: spheres + ground only).
void oro_world_random_scene(void* wp, uint64_t seed, uint32_t flags, int32_t grid_half) {
    World* w = (World*)wp;
    Rng g; g.s = seed;
    Material mat_ground = {{0.5f, 0.5f, 0.5f}, 0.0f, 0.0f, MAT_LAMBERTIAN};                   // main.rs:39
    {   Sphere s; s.l2w = m4_dot_mat(m4_translate(v3(0.0f, -1000.0f, 0.0f)), m4_scale(v3(1000.0f, 1000.0f, 1000.0f)));  // :41
        s.w2l = m4_fast_homogenous_inverse(s.l2w); s.mat = mat_ground; s.id = 0; w->spheres.push_back(s); }
    for (int32_t a = -grid_half; a < grid_half; ++a) {                                       // :42
        float af = (float)a;
        for (int32_t b = -grid_half; b < grid_half; ++b) {                                   // :44
            float bf = (float)b;
            float cx = af + 0.9f * g.rand();
            float cz = bf + 0.9f * g.rand();
            V3 center = v3(cx, 0.2f, cz);                                                    // :46
            bool add = length(center - v3(4.0f, 0.2f, 0.0f)) > 0.9f;                         // :47
            if (!add) continue;
            Material sm;
            float mat_prob = g.rand();                                                       // :50
            if (mat_prob < 0.8f) {                                                           // :51-54
                V3 c1 = rand_v3(g); V3 c2 = rand_v3(g); V3 alb = c1 * c2;
                sm = {{alb.x, alb.y, alb.z}, 0.0f, 0.0f, MAT_LAMBERTIAN};
            } else if (mat_prob < 0.95f) {                                                   // :55-59
                V3 alb = rand_v3_range(g, 0.5f, 1.0f); float fuzz = g.rand_range(0.0f, 0.5f);
                sm = {{alb.x, alb.y, alb.z}, fuzz, 0.0f, MAT_METAL};
            } else {                                                                         // :60-62
                sm = {{0.0f, 0.0f, 0.0f}, 0.0f, 1.5f, MAT_DIELECTRIC};
            }
            float rx = g.rand() * 2.0f * PI_F;                                               // :65-68 (left-to-right)
            float ry = g.rand() * 2.0f * PI_F;
            float rz = g.rand() * 2.0f * PI_F;
            float sx = g.rand() + 1.0f, sy = g.rand() + 1.0f, sz = g.rand() + 1.0f;
            M4 m = m4_dot_mat(m4_dot_mat(m4_dot_mat(m4_dot_mat(m4_dot_mat(m4_translate(center), m4_rot_x(rx)), m4_rot_y(ry)), m4_rot_z(rz)),
                                         m4_scale(v3(sx, sy, sz))), m4_scale(v3(0.2f, 0.2f, 0.2f)));
            Sphere s; s.l2w = m; s.w2l = m4_fast_homogenous_inverse(m); s.mat = sm; s.id = 0; w->spheres.push_back(s);  // :69
        }
    }
    if (flags & 1) {                                                                         // :73-81
        Material mat = {{0, 0, 0}, 0.0f, 1.5f, MAT_DIELECTRIC};
        M4 l2w = m4_dot_mat(m4_dot_mat(m4_translate(v3(0.0f, 1.0f, 0.0f)), m4_rot_x(0.6f)), m4_rot_z(1.33f * 2.0f * PI_F));
        w->mtor.push_back(mtorus_new(l2w, v3(0.5f, 0.1f, 0.1f), mat));
    }
    if (!(flags & 2)) {
        V3 p1 = v3(7.0f, 1.0f, 0.0f), p2 = v3(6.0f, 1.1f, 0.5f), p3 = v3(6.0f, 1.5f, 0.0f);  // :82-92
        Material m1 = {{1.0f, 0.5f, 1.0f}, 0.0f, 0.0f, MAT_METAL};
        Material m2 = {{1.0f, 1.0f, 0.0f}, 0.0f, 0.0f, MAT_LAMBERTIAN};
        w->parallelograms.push_back(bary_new3(p1, p2, p3, m1));
        w->triangles.push_back(bary_new3(p1 + v3(0.0f, 0.5f, 0.0f), p2, p3, m2));
        Material mc = {{0.7f, 0.6f, 0.5f}, 0.0f, 0.0f, MAT_METAL};                           // :93-98
        float rx = g.rand() * 2.0f * PI_F, ry = g.rand() * 2.0f * PI_F, rz = g.rand() * 2.0f * PI_F;
        M4 m = m4_dot_mat(m4_dot_mat(m4_dot_mat(m4_translate(v3(4.0f, 1.0f, 0.0f)), m4_rot_x(rx)), m4_rot_y(ry)), m4_rot_z(rz));
        Cube c; c.l2w = m; c.w2l = m4_fast_homogenous_inverse(m); c.mat = mc; c.id = 0; w->cubes.push_back(c);
    }
}

// Config C2 SDF scene: marched ground (main.rs:40's commented line), a
// MarchedSphere, a MarchedBox and random_scene's torus (main.rs:77-80).
void oro_world_marched_scene(void* wp) {
    World* w = (World*)wp;
    MSphere g; g.center = v3(0.0f, -1000.0f, 0.0f); g.radius = 1000.0f; g.mat = {{0.5f, 0.5f, 0.5f}, 0.0f, 0.0f, MAT_LAMBERTIAN}; g.id = 0;
    w->msph.push_back(g);
    MSphere s; s.center = v3(-4.0f, 1.0f, 0.0f); s.radius = 1.0f; s.mat = {{0.4f, 0.2f, 0.1f}, 0.0f, 0.0f, MAT_LAMBERTIAN}; s.id = 0;
    w->msph.push_back(s);
    MBox b; b.center = v3(4.0f, 1.0f, 0.0f); b.sizes = v3(0.5f, 0.5f, 0.5f); b.mat = {{0.7f, 0.6f, 0.5f}, 0.0f, 0.0f, MAT_METAL}; b.id = 0;
    w->mbox.push_back(b);
    M4 l2w = m4_dot_mat(m4_dot_mat(m4_translate(v3(0.0f, 1.0f, 0.0f)), m4_rot_x(0.6f)), m4_rot_z(1.33f * 2.0f * PI_F));
    w->mtor.push_back(mtorus_new(l2w, v3(0.5f, 0.1f, 0.1f), Material{{0, 0, 0}, 0.0f, 1.5f, MAT_DIELECTRIC}));
}

// camera.rs:38-59
void oro_camera_new(const float* lookfrom, const float* lookat, const float* vup, float vfov, float aspect,
                    float aperture, float focus, OroCamera* out) {
    Camera c = camera_new(ld3(lookfrom), ld3(lookat), ld3(vup), vfov, aspect, aperture, focus);
    st3(c.origin, out->origin); st3(c.horizontal, out->horizontal); st3(c.vertical, out->vertical); st3(c.llc, out->llc);
    st3(c.u, out->u); st3(c.v, out->v); st3(c.w, out->w);
    out->lens_radius = c.lens_radius; out->aspect = c.aspect; out->focus = c.focus; out->vw = c.vw; out->vh = c.vh;
}
static Camera cam_from(const OroCamera* c) {
    Camera o; o.origin = ld3(c->origin); o.horizontal = ld3(c->horizontal); o.vertical = ld3(c->vertical); o.llc = ld3(c->llc);
    o.u = ld3(c->u); o.v = ld3(c->v); o.w = ld3(c->w); o.lens_radius = c->lens_radius; o.aspect = c->aspect; o.focus = c->focus;
    o.vw = c->vw; o.vh = c->vh; return o;
}

// --- RNG KAT surface ---
void oro_rng_draws(uint64_t state, uint32_t n, float* out) { Rng g; g.s = state; for (uint32_t i = 0; i < n; ++i) out[i] = g.rand(); }
void oro_rng_path_draws(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, float* out) {
    PathRng g = path_rng(seed_key(seed), pixel, sample); for (uint32_t i = 0; i < n; ++i) out[i] = g.rand();
}
void oro_jitter_table(uint64_t seed, uint32_t spp, float* out) { auto jt = jitter_table(seed, spp); std::memcpy(out, jt.data(), jt.size() * 4); }
uint64_t oro_bloom_hash(uint64_t id) { return bloom_hash(id); }
uint64_t oro_scramble(uint64_t id) { return scramble(id); }
// draw_to_sdl view `mode` (0..6) of W*H stats into rgb (W*H*3, read-modify-write)
void oro_display(const void* stats, uint32_t W, uint32_t H, int32_t mode, uint8_t* rgb) {
    display((const PixelStats*)stats, W, H, mode, rgb);
}

// --- primitive KAT surface: out = t, point3, normal3, obj_id(as float) ; returns hit ---
static void hr_out(const HitRecord& h, float* out) { out[0] = h.t; st3(h.point, out + 1); st3(h.normal, out + 4); }
int oro_hit_world(void* wp, const float* ray6, float tmin, float tmax, float* out, uint64_t* id) {
    World* w = (World*)wp; w->assign_ids();
    Ray r; r.orig = ld3(ray6); r.dir = ld3(ray6 + 3);
    HitRecord h; bool hit = world_hit(*w, r, tmin, tmax, h);
    if (hit) { hr_out(h, out); *id = h.obj_id; }
    return hit ? 1 : 0;
}
// scatter with an explicit rng state; out = atten3, orig3, dir3
void oro_scatter(const float* ray6, const float* hit7 /*t,p3,n3*/, const OroMaterial* m, uint64_t state, float* out, uint64_t* state_out) {
    Ray r; r.orig = ld3(ray6); r.dir = ld3(ray6 + 3);
    HitRecord h; h.t = hit7[0]; h.point = ld3(hit7 + 1); h.normal = ld3(hit7 + 4); h.material = to_mat(m); h.obj_id = 0;
    PathRng g = PathRng::from_state(state); V3 att; Ray o; scatter(r, h, g, att, o);
    st3(att, out); st3(o.orig, out + 3); st3(o.dir, out + 6); *state_out = g.s;
}
void oro_get_ray(const OroCamera* c, float u, float v, uint64_t state, float* out6) {
    Camera cam = cam_from(c); PathRng g = PathRng::from_state(state); Ray r = camera_get_ray(cam, u, v, g);
    st3(r.orig, out6); st3(r.dir, out6 + 3);
}
void oro_stats_add(void* st, const float* color, float depth, uint64_t id) { stats_add(*(PixelStats*)st, ld3(color), depth, id); }
float oro_marched_sdf(void* wp, int kind, uint32_t i, const float* p) {
    World* w = (World*)wp;
    return kind == 0 ? msphere_sdf(w->msph[i], ld3(p)) : kind == 1 ? mbox_sdf(w->mbox[i], ld3(p))
         : kind == 3 ? msdf_sdf(w->msdf[i], ld3(p)) : mtorus_sdf(w->mtor[i], ld3(p));
}
void oro_marched_normal(void* wp, int kind, uint32_t i, const float* p, float* out) {
    World* w = (World*)wp;
    V3 n = kind == 0 ? msphere_normal(w->msph[i], ld3(p)) : kind == 1 ? mbox_normal(w->mbox[i], ld3(p))
         : kind == 3 ? msdf_normal(w->msdf[i], ld3(p)) : mtorus_normal(w->mtor[i], ld3(p));
    st3(n, out);
}

// --- render: the reference's thread scheme (main.rs:170-214) over pixel subsets ---
// stats: W*H PixelStats (in/out, caller-owned, like PixelsBox main.rs:192)
// nthreads == 0 -> num_cpus - 1 (main.rs:170).  counters (optional): samples, segments, credited.
void oro_render(void* wp, const OroCamera* c, const RenderParams* p, void* stats_v, int32_t nthreads, uint64_t* counters) {
    World* w = (World*)wp; w->assign_ids(); w->march_steps = p->march_steps;
    Camera cam = cam_from(c);
    PixelStats* stats = (PixelStats*)stats_v;
    uint32_t image_size = p->width * p->height;
    if (nthreads <= 0) { unsigned hc = std::thread::hardware_concurrency(); nthreads = hc > 1 ? (int32_t)hc - 1 : 1; }
    // assigned_thread main.rs:172-189: 2730-pixel chunks (32 KiB / sizeof(Color)) round-robin
    const uint32_t CHUNK = 32u * 1024u / 12u;
    std::vector<uint32_t> assigned(image_size);
    {   uint32_t nchunks = image_size / CHUNK, pos = 0;
        for (uint32_t ch = 0; ch < nchunks; ++ch) { uint32_t id = ch % (uint32_t)nthreads; for (uint32_t i = 0; i < CHUNK; ++i) assigned[pos++] = id; }
        uint32_t id = nchunks % (uint32_t)nthreads; while (pos < image_size) assigned[pos++] = id; }
    std::vector<float> jt = jitter_table(p->seed, p->spp_total);
    uint64_t skey = seed_key(p->seed);
    std::vector<Counters> ctrs(nthreads, Counters{0, 0, 0});
    auto worker = [&](int32_t tid) {                                                         // render_thread.rs:145-202
        std::vector<uint32_t> live, back;
        for (uint32_t pos = 0; pos < image_size; ++pos) if (assigned[pos] == (uint32_t)tid) live.push_back(pos);  // :155-159
        back.resize(live.size());
        for (uint32_t k = 0; k < p->sample_count; ++k) {                                     // :176 pass-major
            size_t blen = 0;
            RenderParams one = *p; one.sample_count = 1;
            for (size_t idx = 0; idx < live.size(); ++idx) {                                 // :178
                uint32_t pxl = live[idx];
                render_pixel(*w, cam, one, jt.data(), skey, pxl, stats[pxl], ctrs[tid]);
                bool retired = p->adaptive && (stats[pxl].flags & 1);
                back[blen] = pxl; blen += retired ? 0 : 1;                                   // add_run :97-101
            }
            back.resize(blen); live.swap(back); back.resize(live.size());                    // swap_buffers :92-96
        }
    };
    std::vector<std::thread> th;
    for (int32_t t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
    for (auto& t : th) t.join();
    if (counters) {
        counters[0] = counters[1] = counters[2] = 0;
        for (auto& c2 : ctrs) { counters[0] += c2.samples; counters[1] += c2.segments; counters[2] += c2.credited; }
    }
}

// Pixel-subset render (tile shards): stats[k] belongs to pixels[k].  Single thread.
void oro_render_pixels(void* wp, const OroCamera* c, const RenderParams* p, void* stats_v, const uint32_t* pixels, uint32_t n) {
    World* w = (World*)wp; w->assign_ids(); w->march_steps = p->march_steps;
    Camera cam = cam_from(c);
    PixelStats* stats = (PixelStats*)stats_v;
    std::vector<float> jt = jitter_table(p->seed, p->spp_total);
    uint64_t skey = seed_key(p->seed);
    Counters ctr{0, 0, 0};
    for (uint32_t k = 0; k < n; ++k) render_pixel(*w, cam, *p, jt.data(), skey, pixels[k], stats[k], ctr);
}

// The same over `nthreads` workers (pixel k to worker k % nthreads): pixels are independent, so
// the stats are those of the single-thread form.  Used for oracle windows of full-size frames.
void oro_render_pixels_mt(void* wp, const OroCamera* c, const RenderParams* p, void* stats_v, const uint32_t* pixels,
                          uint32_t n, int32_t nthreads) {
    World* w = (World*)wp; w->assign_ids(); w->march_steps = p->march_steps;
    Camera cam = cam_from(c);
    PixelStats* stats = (PixelStats*)stats_v;
    std::vector<float> jt = jitter_table(p->seed, p->spp_total);
    uint64_t skey = seed_key(p->seed);
    if (nthreads <= 0) { unsigned hc = std::thread::hardware_concurrency(); nthreads = hc > 0 ? (int32_t)hc : 1; }
    auto worker = [&](int32_t tid) {
        Counters ctr{0, 0, 0};
        for (uint32_t k = (uint32_t)tid; k < n; k += (uint32_t)nthreads)
            render_pixel(*w, cam, *p, jt.data(), skey, pixels[k], stats[k], ctr);
    };
    std::vector<std::thread> th;
    for (int32_t t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
    for (auto& t : th) t.join();
}

}  // extern "C"
