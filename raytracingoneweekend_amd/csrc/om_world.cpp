// om_world.cpp — HittableList (host), scene builders, and freeze() into the
// device layout of om_layout.h.  Host C++ only; compiled with -ffp-contract=off.
#include "om_world.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <string>

#include "om_bvh.h"

using namespace om;

namespace {

thread_local std::string g_last_error;

om_status fail(om_status code, const char* msg) {
    g_last_error = msg;
    return code;
}

// ---- om-rng SplitMix64 (host side: scene + jitter).  Replaces rand::thread_rng() (utils.rs:25).
struct SplitMix {
    uint64_t s;
    static uint64_t mix(uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    uint64_t next() { s += 0x9E3779B97F4A7C15ULL; return mix(s); }
    float f32() { return (float)(uint32_t)(next() >> 40) * 5.9604644775390625e-8f; }        // utils.rs:25
    float range(float lo, float hi) { const float r = f32(); return r * (hi - lo) + lo; }   // utils.rs:26
    Vec3 v3() { const float x = f32(); const float y = f32(); const float z = f32(); return Vec3::make(x, y, z); }  // vec3.rs:81
    Vec3 v3_range(float lo, float hi) {                                                      // vec3.rs:82-88
        const float x = range(lo, hi); const float y = range(lo, hi); const float z = range(lo, hi);
        return Vec3::make(x, y, z);
    }
};

inline om_material make_mat(float r, float g, float b, float fuzz, float ior, int32_t type) {
    om_material m;
    m.albedo[0] = r; m.albedo[1] = g; m.albedo[2] = b; m.fuzz = fuzz; m.ior = ior; m.type = type;
    return m;
}

bool valid_mat(const om_material* m) {
    return m && (m->type == OM_LAMBERTIAN || m->type == OM_METAL || m->type == OM_DIELECTRIC);
}

AffinePrim make_affine(const Mat4& l2w, const om_material& m) {                           // traced.rs:22-25, 238-240
    AffinePrim p;
    p.l2w = l2w;
    p.w2l = l2w.fast_homogenous_inverse();
    p.mat = m;
    return p;
}

BaryPrim make_bary(const Vec3& origin, const Vec3& u, const Vec3& v, float ul, float vl, const om_material& m) {  // traced.rs:135-147
    BaryPrim b;
    const Vec3 uu = u.unit();
    const Vec3 vu = v.unit();
    const Vec3 uxv = uu.cross(vu).unit();
    const Vec3 uxvxu = uxv.cross(uu).unit();
    b.base_inv = Mat3::cols(uu, uxv, uxvxu).transpose();
    b.v_in_base = b.base_inv.apply(vu);
    b.origin = origin; b.u = uu; b.u_length = ul; b.v = vu; b.v_length = vl; b.uxv = uxv; b.uxvxu = uxvxu; b.mat = m;
    return b;
}

BaryPrim make_bary3(const Vec3& o, const Vec3& up, const Vec3& vp, const om_material& m) {  // traced.rs:148-154
    const Vec3 ur = up.sub(o);
    const float ul = ur.length();
    const Vec3 vr = vp.sub(o);
    const float vl = vr.length();
    return make_bary(o, ur, vr, ul, vl, m);
}

MTorusPrim make_torus(const Mat4& l2w, const Vec3& sizes, const om_material& m) {         // marched.rs:116-130
    // decompose_into_translate_rotate_scale mat4x4.rs:125-147
    const Vec3 a = l2w.col(0).xyz(), b = l2w.col(1).xyz(), c = l2w.col(2).xyz(), d = l2w.col(3).xyz();
    const float al = a.length(), bl = b.length(), cl = c.length();
    const Mat4 t = Mat4::cols(Vec4::make(1, 0, 0, 0), Vec4::make(0, 1, 0, 0), Vec4::make(0, 0, 1, 0), Vec4::point(d));
    const Mat4 r = Mat4::cols(Vec4::vec(a.div(al)), Vec4::vec(b.div(bl)), Vec4::vec(c.div(cl)), Vec4::point(Vec3::make(0, 0, 0)));
    const Mat4 s = Mat4::rows(Vec4::make(al, 0, 0, 0), Vec4::make(0, bl, 0, 0), Vec4::make(0, 0, cl, 0), Vec4::make(0, 0, 0, 1));
    const Mat4 tr = t.mul(r);
    const Vec4 sc = Vec4::make(s.r[0].e[0], s.r[1].e[1], s.r[2].e[2], s.r[3].e[3]);         // diag mat4x4.rs:148-150
    MTorusPrim p;
    p.l2w_tr = tr;
    p.w2l_tr = tr.fast_homogenous_inverse();
    p.l2w_s = sc;
    p.w2l_s = Vec4::make(1.0f / sc.e[0], 1.0f / sc.e[1], 1.0f / sc.e[2], 1.0f / sc.e[3]);
    p.sizes = sizes;
    p.mat = m;
    return p;
}

void pack_affine(const AffinePrim& p, OmAffineTest& t, OmAffineHit& h) {
    for (int i = 0; i < 3; ++i) {
        for (int j = 0; j < 4; ++j) { t.w2l[4 * i + j] = p.w2l.r[i].e[j]; h.l2w[4 * i + j] = p.l2w.r[i].e[j]; }
        t.dz[i] = p.w2l.r[i].e[3] * 0.0f;   // w-term of dot_v3 (mat4x4.rs:54-57)
        h.lz[i] = p.l2w.r[i].e[3] * 0.0f;
    }
    t.pad = 0.0f; h.pad = 0.0f;
}

// Largest singular value of the 3x3 linear part (double-precision Jacobi on A^T A).
double sigma_max(const Mat4& l2w) {
    double a[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) a[i][j] = l2w.r[i].e[j];
    double s[3][3];
    for (int i = 0; i < 3; ++i) for (int j = 0; j < 3; ++j) { s[i][j] = 0; for (int k = 0; k < 3; ++k) s[i][j] += a[k][i] * a[k][j]; }
    for (int sweep = 0; sweep < 50; ++sweep) {
        double off = std::fabs(s[0][1]) + std::fabs(s[0][2]) + std::fabs(s[1][2]);
        if (off < 1e-300) break;
        for (int p = 0; p < 2; ++p) for (int q = p + 1; q < 3; ++q) {
            if (std::fabs(s[p][q]) < 1e-300) continue;
            const double theta = (s[q][q] - s[p][p]) / (2.0 * s[p][q]);
            const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
            const double c = 1.0 / std::sqrt(t * t + 1.0), sn = t * c;
            for (int k = 0; k < 3; ++k) { const double skp = s[k][p], skq = s[k][q]; s[k][p] = c * skp - sn * skq; s[k][q] = sn * skp + c * skq; }
            for (int k = 0; k < 3; ++k) { const double spk = s[p][k], sqk = s[q][k]; s[p][k] = c * spk - sn * sqk; s[q][k] = sn * spk + c * sqk; }
        }
    }
    const double ev = std::max(s[0][0], std::max(s[1][1], s[2][2]));
    return std::sqrt(std::max(ev, 0.0));
}

// Conservative bound: radius inflated well beyond f32 rounding.
OmBound make_bound(const Mat4& l2w, double local_radius) {
    OmBound b;
    const double cx = l2w.r[0].e[3], cy = l2w.r[1].e[3], cz = l2w.r[2].e[3];
    const double cn = std::sqrt(cx * cx + cy * cy + cz * cz);
    const double r = sigma_max(l2w) * local_radius;
    b.c[0] = (float)cx; b.c[1] = (float)cy; b.c[2] = (float)cz;
    b.r = (float)(r * (1.0 + 1e-3) + 1e-3 + 1e-5 * cn);
    return b;
}

}  // namespace

namespace om {

uint64_t bloom_hash(uint64_t id) {                                                         // utils.rs:94-107
    auto scramble = [](uint64_t v) -> uint64_t {                                           // utils.rs:46-56
        uint64_t lo = v & 0xFFFFFFFFULL;
        lo ^= lo << 13; lo ^= lo >> 7; lo ^= lo << 17;
        uint64_t hi = v >> 32;
        hi ^= hi << 13; hi ^= hi >> 17; hi ^= hi << 5;
        return (hi << 32) ^ lo ^ (lo * hi);
    };
    static const uint64_t K[9][3] = {
        {456894789ULL, 348764781ULL, 17287318477382145149ULL}, {56456ULL, 2345ULL, 10520185020478678957ULL},
        {12337ULL, 7878ULL, 6100366985798845493ULL},           {7438554325ULL, 2554ULL, 2581451885731034521ULL},
        {12345ULL, 123123044ULL, 2015400956511055807ULL},      {6373412378ULL, 12452ULL, 8800267423223100703ULL},
        {3453453ULL, 7874856378ULL, 7039701875810786467ULL},   {999465ULL, 143ULL, 3008457310659543551ULL},
        {14444ULL, 111345ULL, 5935720376112203207ULL}};
    const uint64_t bit = id != 0 ? 1 : 0;
    uint64_t h = 0;
    for (int i = 0; i < 9; ++i) h |= bit << (scramble((id * K[i][0] + K[i][1]) % K[i][2]) % 64);
    return h;
}

}  // namespace om

void om_world::freeze(FrozenWorld& fw) const {
    fw = FrozenWorld();
    fw.counts[0] = (uint32_t)spheres.size(); fw.counts[1] = (uint32_t)cubes.size(); fw.counts[2] = (uint32_t)triangles.size();
    fw.counts[3] = (uint32_t)planes.size(); fw.counts[4] = (uint32_t)parallelograms.size(); fw.counts[5] = (uint32_t)msph.size();
    fw.counts[6] = (uint32_t)mbox.size(); fw.counts[7] = (uint32_t)mtor.size(); fw.counts[8] = (uint32_t)msdf.size();
    fw.offsets[0] = 0;
    for (int k = 0; k < K_N; ++k) fw.offsets[k + 1] = fw.offsets[k] + fw.counts[k];
    const uint32_t total = fw.offsets[K_N];
    fw.mats.resize(total);
    fw.bloom.resize((size_t)total + 1);
    fw.bloom[0] = 0;
    for (uint32_t id = 1; id <= total; ++id) fw.bloom[id] = bloom_hash(id);
    auto put_mat = [&](uint32_t gi, const om_material& m) {
        OmMaterial& o = fw.mats[gi];
        o.albedo[0] = m.albedo[0]; o.albedo[1] = m.albedo[1]; o.albedo[2] = m.albedo[2];
        o.fuzz = m.fuzz; o.ior = m.ior; o.type = m.type; o.pad[0] = o.pad[1] = 0.0f;
    };
    fw.sph_test.resize(spheres.size()); fw.sph_hit.resize(spheres.size()); fw.sph_bound.resize(spheres.size());
    for (size_t i = 0; i < spheres.size(); ++i) {
        pack_affine(spheres[i], fw.sph_test[i], fw.sph_hit[i]);
        fw.sph_bound[i] = make_bound(spheres[i].l2w, 1.0);
        put_mat(fw.offsets[K_SPHERE] + (uint32_t)i, spheres[i].mat);
    }
    fw.cube_test.resize(cubes.size()); fw.cube_hit.resize(cubes.size()); fw.cube_bound.resize(cubes.size());
    for (size_t i = 0; i < cubes.size(); ++i) {
        pack_affine(cubes[i], fw.cube_test[i], fw.cube_hit[i]);
        fw.cube_bound[i] = make_bound(cubes[i].l2w, 0.8660254037844387);
        put_mat(fw.offsets[K_CUBE] + (uint32_t)i, cubes[i].mat);
    }
    auto pack_bary = [](const BaryPrim& b, OmBary& o) {
        b.origin.store(o.origin); o.u_length = b.u_length; b.uxv.store(o.uxv); o.v_length = b.v_length;
        for (int r = 0; r < 3; ++r) b.base_inv.r[r].store(o.base_inv + 3 * r);
        o.vx = b.v_in_base.x(); o.vy = b.v_in_base.z(); o.pad = 0.0f;
    };
    fw.tri.resize(triangles.size());
    for (size_t i = 0; i < triangles.size(); ++i) { pack_bary(triangles[i], fw.tri[i]); put_mat(fw.offsets[K_TRI] + (uint32_t)i, triangles[i].mat); }
    fw.plane.resize(planes.size());
    for (size_t i = 0; i < planes.size(); ++i) {
        planes[i].center.store(fw.plane[i].center); planes[i].normal.store(fw.plane[i].normal);
        fw.plane[i].pad0 = fw.plane[i].pad1 = 0.0f;
        put_mat(fw.offsets[K_PLANE] + (uint32_t)i, planes[i].mat);
    }
    fw.para.resize(parallelograms.size());
    for (size_t i = 0; i < parallelograms.size(); ++i) { pack_bary(parallelograms[i], fw.para[i]); put_mat(fw.offsets[K_PARA] + (uint32_t)i, parallelograms[i].mat); }
    fw.msph.resize(msph.size());
    for (size_t i = 0; i < msph.size(); ++i) {
        msph[i].center.store(fw.msph[i].center); fw.msph[i].radius = msph[i].radius;
        put_mat(fw.offsets[K_MSPHERE] + (uint32_t)i, msph[i].mat);
    }
    fw.mbox.resize(mbox.size());
    for (size_t i = 0; i < mbox.size(); ++i) {
        mbox[i].center.store(fw.mbox[i].center); mbox[i].sizes.store(fw.mbox[i].sizes); fw.mbox[i].pad0 = 0.0f;
        {   // |sdf| >= |p - center| - |sizes| (margins: f32 rounding of the SDF and of the test)
            const double sx = mbox[i].sizes.e[0], sy = mbox[i].sizes.e[1], sz = mbox[i].sizes.e[2];
            const double hd = std::sqrt(sx * sx + sy * sy + sz * sz);
            fw.mbox[i].br = std::isfinite(hd) ? (float)(hd * (1.0 + 1e-4) + 1e-4) : NAN;
        }
        put_mat(fw.offsets[K_MBOX] + (uint32_t)i, mbox[i].mat);
    }
    fw.mtor.resize(mtor.size());
    for (size_t i = 0; i < mtor.size(); ++i) {
        const MTorusPrim& t = mtor[i]; OmMTorus& o = fw.mtor[i];
        t.l2w_tr.store(o.l2w_tr); t.w2l_tr.store(o.w2l_tr);
        for (int k = 0; k < 4; ++k) { o.l2w_s[k] = t.l2w_s.e[k]; o.w2l_s[k] = t.w2l_s.e[k]; }
        t.sizes.store(o.sizes);
        o.min_scale = std::fmin(t.l2w_s.e[0], std::fmin(t.l2w_s.e[1], t.l2w_s.e[2]));     // Vec3::min_val vec3.rs:50-52
        // march cull: q = W2L_TR (p * w2l_s) with W2L_TR rigid, so |q| = |p * w2l_s - d|
        // >= |p - d * l2w_s| * min(w2l_s), and the torus lies within |q| <= R + r:
        // |sdf| >= (|p - bc| * kq - (R + r)) * min_scale.  A step skips the torus when
        // |p - bc| > (best / min_scale + R + r) / kq, i.e. |p - bc|^2 > (best * bk + br)^2.
        {
            const double kq = std::min({(double)t.w2l_s.e[0], (double)t.w2l_s.e[1], (double)t.w2l_s.e[2]}) * (1.0 - 1e-4);
            const double ms = (double)o.min_scale * (1.0 - 1e-4);
            const double rr = std::fabs((double)t.sizes.e[0]) + std::fabs((double)t.sizes.e[1]);
            const bool ok = kq > 0.0 && ms > 0.0 && std::isfinite(kq) && std::isfinite(ms) && std::isfinite(rr);
            for (int k = 0; k < 3; ++k) o.bc[k] = (float)((double)t.l2w_tr.r[k].e[3] * (double)t.l2w_s.e[k]);
            o.bk = ok ? (float)(1.0 / (ms * kq) * (1.0 + 1e-4)) : NAN;          // NaN: never cull
            o.br = ok ? (float)((rr * (1.0 + 1e-4) + 1e-4) / kq * (1.0 + 1e-4)) : NAN;
            o.pad_b[0] = o.pad_b[1] = o.pad_b[2] = 0.0f;
        }
        put_mat(fw.offsets[K_MTORUS] + (uint32_t)i, t.mat);
    }
    fw.msdf.resize(msdf.size());
    fw.msdf_ops.clear();
    for (size_t i = 0; i < msdf.size(); ++i) {
        const MSdfPrim& q = msdf[i]; OmMSdf& o = fw.msdf[i];
        q.xf.l2w_tr.store(o.l2w_tr); q.xf.w2l_tr.store(o.w2l_tr);
        for (int k = 0; k < 4; ++k) { o.l2w_s[k] = q.xf.l2w_s.e[k]; o.w2l_s[k] = q.xf.w2l_s.e[k]; }
        o.min_scale = std::fmin(q.xf.l2w_s.e[0], std::fmin(q.xf.l2w_s.e[1], q.xf.l2w_s.e[2]));   // as the torus
        o.op_first = (uint32_t)fw.msdf_ops.size(); o.op_count = (uint32_t)q.ops.size(); o.pad = 0;
        fw.msdf_ops.insert(fw.msdf_ops.end(), q.ops.begin(), q.ops.end());
        put_mat(fw.offsets[K_MSDF] + (uint32_t)i, q.mat);
    }
    build_bvh(*this, fw);
}

// ============================================================================
// C-ABI: materials, camera, world
// ============================================================================
extern "C" {

int32_t om_abi_version(void) { return OM_ABI_VERSION; }

om_material om_material_lambertian(float r, float g, float b) { return make_mat(r, g, b, 0.0f, 0.0f, OM_LAMBERTIAN); }  // materials.rs:27-29
om_material om_material_metal(float r, float g, float b) { return make_mat(r, g, b, 0.0f, 0.0f, OM_METAL); }            // :30-32
om_material om_material_metal_fuzz(float r, float g, float b, float fuzz) { return make_mat(r, g, b, fuzz, 0.0f, OM_METAL); }  // :33-35
om_material om_material_dielectric(float ior) { return make_mat(0.0f, 0.0f, 0.0f, 0.0f, ior, OM_DIELECTRIC); }          // :36-38

om_status om_mat4_identity(float out[16]) {
    if (!out) return fail(OM_ERR_INVALID, "om_mat4_identity: null out");
    Mat4::identity().store(out);
    return OM_OK;
}
om_status om_mat4_translate(const float v[3], float out[16]) {
    if (!v || !out) return fail(OM_ERR_INVALID, "om_mat4_translate: null pointer");
    Mat4::translate(Vec3::load(v)).store(out);
    return OM_OK;
}
om_status om_mat4_scale(const float v[3], float out[16]) {
    if (!v || !out) return fail(OM_ERR_INVALID, "om_mat4_scale: null pointer");
    Mat4::scale(Vec3::load(v)).store(out);
    return OM_OK;
}
om_status om_mat4_rotate(int32_t axis, float angle, float out[16]) {
    if (!out || axis < 0 || axis > 2) return fail(OM_ERR_INVALID, "om_mat4_rotate: bad axis or null out");
    (axis == 0 ? Mat4::rotate_x(angle) : axis == 1 ? Mat4::rotate_y(angle) : Mat4::rotate_z(angle)).store(out);
    return OM_OK;
}
om_status om_mat4_mul(const float a[16], const float b[16], float out[16]) {
    if (!a || !b || !out) return fail(OM_ERR_INVALID, "om_mat4_mul: null pointer");
    Mat4::load(a).mul(Mat4::load(b)).store(out);
    return OM_OK;
}
om_status om_mat4_fast_homogenous_inverse(const float m[16], float out[16]) {
    if (!m || !out) return fail(OM_ERR_INVALID, "om_mat4_fast_homogenous_inverse: null pointer");
    Mat4::load(m).fast_homogenous_inverse().store(out);
    return OM_OK;
}

om_status om_camera_new(const float lookfrom[3], const float lookat[3], const float vup[3], float vfov_deg, float aspect,
                        float aperture, float focus, om_camera* out) {                   // camera.rs:38-59
    if (!lookfrom || !lookat || !vup || !out) return fail(OM_ERR_INVALID, "om_camera_new: null pointer");
    const float vfov = vfov_deg * kPi / 180.0f;                                           // utils.rs:33-35
    const float height = std::tan(vfov / 2.0f) * focus;
    const float vh = 2.0f * height;
    const float vw = vh * aspect;
    const Vec3 from = Vec3::load(lookfrom), at = Vec3::load(lookat), up = Vec3::load(vup);
    const Vec3 w = from.sub(at).unit();
    const Vec3 u = up.cross(w).unit();
    const Vec3 v = w.cross(u).unit();
    const Vec3 h = u.scale(vw);
    const Vec3 vv = v.scale(vh);
    const Vec3 llc = from.sub(h.div(2.0f)).sub(vv.div(2.0f)).sub(w.scale(focus));
    from.store(out->origin); h.store(out->horizontal); vv.store(out->vertical); llc.store(out->lower_left_corner);
    u.store(out->u_of_plane); v.store(out->v_of_plane); w.store(out->w_of_plane);
    out->lens_radius = aperture / 2.0f; out->aspect_ratio = aspect; out->focus_dist = focus;
    out->viewport_width = vw; out->viewport_height = vh;
    return OM_OK;
}

om_status om_world_create(om_world** out) {
    if (!out) return fail(OM_ERR_INVALID, "om_world_create: null out");
    *out = new (std::nothrow) om_world();
    return *out ? OM_OK : fail(OM_ERR_NOMEM, "om_world_create: out of memory");
}
void om_world_destroy(om_world* w) { delete w; }
om_status om_world_clear(om_world* w) {                                                    // hits.rs:81-86
    if (!w) return fail(OM_ERR_INVALID, "om_world_clear: null world");
    *w = om_world();
    return OM_OK;
}

#define OM_CHECK_ADD(cond, name) \
    if (!(cond)) return fail(OM_ERR_INVALID, name ": null pointer or invalid material")

om_status om_world_add_sphere(om_world* w, const float l2w[16], const om_material* m) {
    OM_CHECK_ADD(w && l2w && valid_mat(m), "om_world_add_sphere");
    w->spheres.push_back(make_affine(Mat4::load(l2w), *m));
    return OM_OK;
}
om_status om_world_add_sphere_radius(om_world* w, const float c[3], float r, const om_material* m) {  // traced.rs:26-31
    OM_CHECK_ADD(w && c && valid_mat(m), "om_world_add_sphere_radius");
    w->spheres.push_back(make_affine(Mat4::translate(Vec3::load(c)).mul(Mat4::scale(Vec3::make(r, r, r))), *m));
    return OM_OK;
}
om_status om_world_add_cube(om_world* w, const float l2w[16], const om_material* m) {
    OM_CHECK_ADD(w && l2w && valid_mat(m), "om_world_add_cube");
    w->cubes.push_back(make_affine(Mat4::load(l2w), *m));
    return OM_OK;
}
om_status om_world_add_cube_length(om_world* w, const float c[3], float len, const om_material* m) {  // traced.rs:242-246
    OM_CHECK_ADD(w && c && valid_mat(m), "om_world_add_cube_length");
    w->cubes.push_back(make_affine(Mat4::translate(Vec3::load(c)).mul(Mat4::scale(Vec3::make(len, len, len))), *m));
    return OM_OK;
}
om_status om_world_add_triangle(om_world* w, const float o[3], const float up[3], const float vp[3], const om_material* m) {
    OM_CHECK_ADD(w && o && up && vp && valid_mat(m), "om_world_add_triangle");
    w->triangles.push_back(make_bary3(Vec3::load(o), Vec3::load(up), Vec3::load(vp), *m));
    return OM_OK;
}
om_status om_world_add_parallelogram(om_world* w, const float o[3], const float up[3], const float vp[3], const om_material* m) {
    OM_CHECK_ADD(w && o && up && vp && valid_mat(m), "om_world_add_parallelogram");
    w->parallelograms.push_back(make_bary3(Vec3::load(o), Vec3::load(up), Vec3::load(vp), *m));
    return OM_OK;
}
om_status om_world_add_triangle_basis(om_world* w, const float o[3], const float u[3], const float v[3], float ul, float vl, const om_material* m) {
    OM_CHECK_ADD(w && o && u && v && valid_mat(m), "om_world_add_triangle_basis");
    w->triangles.push_back(make_bary(Vec3::load(o), Vec3::load(u), Vec3::load(v), ul, vl, *m));
    return OM_OK;
}
om_status om_world_add_parallelogram_basis(om_world* w, const float o[3], const float u[3], const float v[3], float ul, float vl, const om_material* m) {
    OM_CHECK_ADD(w && o && u && v && valid_mat(m), "om_world_add_parallelogram_basis");
    w->parallelograms.push_back(make_bary(Vec3::load(o), Vec3::load(u), Vec3::load(v), ul, vl, *m));
    return OM_OK;
}
om_status om_world_add_plane(om_world* w, const float c[3], const float n[3], const om_material* m) {  // traced.rs:86-88
    OM_CHECK_ADD(w && c && n && valid_mat(m), "om_world_add_plane");
    PlanePrim p; p.center = Vec3::load(c); p.normal = Vec3::load(n).unit(); p.mat = *m;
    w->planes.push_back(p);
    return OM_OK;
}
om_status om_world_add_marched_sphere(om_world* w, const float c[3], float r, const om_material* m) {
    OM_CHECK_ADD(w && c && valid_mat(m), "om_world_add_marched_sphere");
    MSpherePrim p; p.center = Vec3::load(c); p.radius = r; p.mat = *m;
    w->msph.push_back(p);
    return OM_OK;
}
om_status om_world_add_marched_box(om_world* w, const float c[3], const float sz[3], const om_material* m) {
    OM_CHECK_ADD(w && c && sz && valid_mat(m), "om_world_add_marched_box");
    MBoxPrim p; p.center = Vec3::load(c); p.sizes = Vec3::load(sz); p.mat = *m;
    w->mbox.push_back(p);
    return OM_OK;
}
om_status om_world_add_marched_torus(om_world* w, const float l2w[16], const float sz[3], const om_material* m) {
    OM_CHECK_ADD(w && l2w && sz && valid_mat(m), "om_world_add_marched_torus");
    w->mtor.push_back(make_torus(Mat4::load(l2w), Vec3::load(sz), *m));
    return OM_OK;
}

om_status om_world_add_marched_sdf(om_world* w, const float l2w[16], const om_sdf_op* ops, uint32_t n, const om_material* m) {
    OM_CHECK_ADD(w && l2w && ops && valid_mat(m), "om_world_add_marched_sdf");
    if (n == 0 || n > OM_SDF_MAX_OPS) return fail(OM_ERR_INVALID, "om_world_add_marched_sdf: 1..OM_SDF_MAX_OPS ops");
    MSdfPrim p;
    int depth = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const om_sdf_op& q = ops[i];
        int params = 0, pops = 0;
        switch (q.op) {
            case OM_SDF_SPHERE: params = 4; break;
            case OM_SDF_BOX: params = 6; break;
            case OM_SDF_TORUS: params = 5; break;
            case OM_SDF_UNION: case OM_SDF_INTERSECT: case OM_SDF_SUBTRACT: pops = 2; break;
            case OM_SDF_ROUND: params = 1; pops = 1; break;
            default: return fail(OM_ERR_INVALID, "om_world_add_marched_sdf: unknown op");
        }
        for (int k = 0; k < params; ++k)
            if (!std::isfinite(q.a[k])) return fail(OM_ERR_INVALID, "om_world_add_marched_sdf: non-finite parameter");
        if (depth < pops) return fail(OM_ERR_INVALID, "om_world_add_marched_sdf: stack underflow");
        depth += (pops == 2 ? -1 : pops == 1 ? 0 : 1);
        if (depth > OM_SDF_MAX_STACK) return fail(OM_ERR_INVALID, "om_world_add_marched_sdf: stack deeper than OM_SDF_MAX_STACK");
        OmSdfOp o;
        o.op = (uint32_t)q.op;
        for (int k = 0; k < 7; ++k) o.a[k] = k < params ? q.a[k] : 0.0f;
        p.ops.push_back(o);
    }
    if (depth != 1) return fail(OM_ERR_INVALID, "om_world_add_marched_sdf: the program must leave exactly one value");
    p.xf = make_torus(Mat4::load(l2w), Vec3::make(0.0f, 0.0f, 0.0f), *m);     // MarchedTorus::new's decomposition
    p.mat = *m;
    w->msdf.push_back(std::move(p));
    return OM_OK;
}

om_status om_world_marched_sdf_count(const om_world* w, uint32_t* n) {
    if (!w || !n) return fail(OM_ERR_INVALID, "om_world_marched_sdf_count: null pointer");
    *n = (uint32_t)w->msdf.size();
    return OM_OK;
}

om_status om_world_counts(const om_world* w, uint32_t counts[8]) {
    if (!w || !counts) return fail(OM_ERR_INVALID, "om_world_counts: null pointer");
    counts[0] = (uint32_t)w->spheres.size(); counts[1] = (uint32_t)w->cubes.size(); counts[2] = (uint32_t)w->triangles.size();
    counts[3] = (uint32_t)w->planes.size(); counts[4] = (uint32_t)w->parallelograms.size(); counts[5] = (uint32_t)w->msph.size();
    counts[6] = (uint32_t)w->mbox.size(); counts[7] = (uint32_t)w->mtor.size();
    return OM_OK;
}

om_status om_world_export(const om_world* w, int32_t kind, uint32_t i, float* out, uint32_t n) {
    if (!w || !out) return fail(OM_ERR_INVALID, "om_world_export: null pointer");
    if (kind == K_SPHERE || kind == K_CUBE) {
        const auto& v = kind == K_SPHERE ? w->spheres : w->cubes;
        if (i >= v.size() || n < 32) return fail(OM_ERR_INVALID, "om_world_export: index/size");
        v[i].l2w.store(out); v[i].w2l.store(out + 16);
        return OM_OK;
    }
    if (kind == K_TRI || kind == K_PARA) {
        const auto& v = kind == K_TRI ? w->triangles : w->parallelograms;
        if (i >= v.size() || n < 29) return fail(OM_ERR_INVALID, "om_world_export: index/size");
        const BaryPrim& b = v[i];
        b.origin.store(out); b.u.store(out + 3); out[6] = b.u_length; b.v.store(out + 7); out[10] = b.v_length;
        b.uxv.store(out + 11); b.uxvxu.store(out + 14);
        for (int r = 0; r < 3; ++r) b.base_inv.r[r].store(out + 17 + 3 * r);
        b.v_in_base.store(out + 26);
        return OM_OK;
    }
    if (kind == K_MTORUS) {
        if (i >= w->mtor.size() || n < 43) return fail(OM_ERR_INVALID, "om_world_export: index/size");
        const MTorusPrim& t = w->mtor[i];
        t.l2w_tr.store(out); t.w2l_tr.store(out + 16);
        for (int k = 0; k < 4; ++k) { out[32 + k] = t.l2w_s.e[k]; out[36 + k] = t.w2l_s.e[k]; }
        t.sizes.store(out + 40);
        return OM_OK;
    }
    return fail(OM_ERR_INVALID, "om_world_export: unsupported kind");
}

// main.rs:37-100 with om-rng SplitMix64 in place of thread_rng.
om_status om_world_random_scene(om_world* w, uint64_t seed, uint32_t flags, int32_t grid_half) {
    if (!w || grid_half < 0 || grid_half > 4096) return fail(OM_ERR_INVALID, "om_world_random_scene: bad arguments");
    SplitMix g{seed};
    const om_material ground = make_mat(0.5f, 0.5f, 0.5f, 0.0f, 0.0f, OM_LAMBERTIAN);        // main.rs:39
    w->spheres.push_back(make_affine(Mat4::translate(Vec3::make(0.0f, -1000.0f, 0.0f)).mul(Mat4::scale(Vec3::make(1000.0f, 1000.0f, 1000.0f))), ground));  // :41
    const Vec3 excl = Vec3::make(4.0f, 0.2f, 0.0f);
    for (int32_t a = -grid_half; a < grid_half; ++a) {                                    // :42
        const float af = (float)a;
        for (int32_t b = -grid_half; b < grid_half; ++b) {                                // :44
            const float bf = (float)b;
            const float cx = af + 0.9f * g.f32();                                          // :46
            const float cz = bf + 0.9f * g.f32();
            const Vec3 center = Vec3::make(cx, 0.2f, cz);
            if (!(center.sub(excl).length() > 0.9f)) continue;                             // :47
            om_material m;
            const float prob = g.f32();                                                    // :50
            if (prob < 0.8f) {                                                             // :51-54
                const Vec3 c1 = g.v3();
                const Vec3 c2 = g.v3();
                const Vec3 alb = c1.mul(c2);
                m = make_mat(alb.x(), alb.y(), alb.z(), 0.0f, 0.0f, OM_LAMBERTIAN);
            } else if (prob < 0.95f) {                                                     // :55-59
                const Vec3 alb = g.v3_range(0.5f, 1.0f);
                const float fuzz = g.range(0.0f, 0.5f);
                m = make_mat(alb.x(), alb.y(), alb.z(), fuzz, 0.0f, OM_METAL);
            } else {                                                                       // :60-62
                m = make_mat(0.0f, 0.0f, 0.0f, 0.0f, 1.5f, OM_DIELECTRIC);
            }
            const float rx = g.f32() * 2.0f * kPi;                                         // :65-68, operands left to right
            const float ry = g.f32() * 2.0f * kPi;
            const float rz = g.f32() * 2.0f * kPi;
            const float sx = g.f32() + 1.0f;
            const float sy = g.f32() + 1.0f;
            const float sz = g.f32() + 1.0f;
            const Mat4 l2w = Mat4::translate(center).mul(Mat4::rotate_x(rx)).mul(Mat4::rotate_y(ry)).mul(Mat4::rotate_z(rz))
                                 .mul(Mat4::scale(Vec3::make(sx, sy, sz))).mul(Mat4::scale(Vec3::make(0.2f, 0.2f, 0.2f)));
            w->spheres.push_back(make_affine(l2w, m));                                     // :69
        }
    }
    if (flags & 1u) {                                                                      // :73-81
        const Mat4 l2w = Mat4::translate(Vec3::make(0.0f, 1.0f, 0.0f)).mul(Mat4::rotate_x(0.6f)).mul(Mat4::rotate_z(1.33f * 2.0f * kPi));
        w->mtor.push_back(make_torus(l2w, Vec3::make(0.5f, 0.1f, 0.1f), make_mat(0, 0, 0, 0.0f, 1.5f, OM_DIELECTRIC)));
    }
    if (!(flags & 2u)) {
        const Vec3 p1 = Vec3::make(7.0f, 1.0f, 0.0f), p2 = Vec3::make(6.0f, 1.1f, 0.5f), p3 = Vec3::make(6.0f, 1.5f, 0.0f);  // :83-85
        w->parallelograms.push_back(make_bary3(p1, p2, p3, make_mat(1.0f, 0.5f, 1.0f, 0.0f, 0.0f, OM_METAL)));         // :86-88
        w->triangles.push_back(make_bary3(p1.add(Vec3::make(0.0f, 0.5f, 0.0f)), p2, p3, make_mat(1.0f, 1.0f, 0.0f, 0.0f, 0.0f, OM_LAMBERTIAN)));  // :89-91
        const float rx = g.f32() * 2.0f * kPi;                                             // :93-98
        const float ry = g.f32() * 2.0f * kPi;
        const float rz = g.f32() * 2.0f * kPi;
        const Mat4 l2w = Mat4::translate(Vec3::make(4.0f, 1.0f, 0.0f)).mul(Mat4::rotate_x(rx)).mul(Mat4::rotate_y(ry)).mul(Mat4::rotate_z(rz));
        w->cubes.push_back(make_affine(l2w, make_mat(0.7f, 0.6f, 0.5f, 0.0f, 0.0f, OM_METAL)));
    }
    return OM_OK;
}

om_status om_world_basic_scene(om_world* w) {                                              // main.rs:103-110
    if (!w) return fail(OM_ERR_INVALID, "om_world_basic_scene: null world");
    const om_material m = make_mat(0.5f, 0.5f, 0.5f, 0.0f, 0.0f, OM_LAMBERTIAN);
    const float cs[3][3] = {{0.0f, 0.0f, -2.0f}, {-2.0f, 0.0f, -2.0f}, {2.0f, 0.0f, -2.0f}};
    for (auto& c : cs) w->spheres.push_back(make_affine(Mat4::translate(Vec3::load(c)).mul(Mat4::scale(Vec3::make(1.0f, 1.0f, 1.0f))), m));
    return OM_OK;
}

// Config C2: marched ground (main.rs:40's commented MarchedSphere),
// a MarchedBox, a MarchedSphere and random_scene's torus (main.rs:77-80).
om_status om_world_marched_scene(om_world* w) {
    if (!w) return fail(OM_ERR_INVALID, "om_world_marched_scene: null world");
    MSpherePrim ground; ground.center = Vec3::make(0.0f, -1000.0f, 0.0f); ground.radius = 1000.0f;
    ground.mat = make_mat(0.5f, 0.5f, 0.5f, 0.0f, 0.0f, OM_LAMBERTIAN);
    w->msph.push_back(ground);
    MSpherePrim s; s.center = Vec3::make(-4.0f, 1.0f, 0.0f); s.radius = 1.0f; s.mat = make_mat(0.4f, 0.2f, 0.1f, 0.0f, 0.0f, OM_LAMBERTIAN);
    w->msph.push_back(s);
    MBoxPrim b; b.center = Vec3::make(4.0f, 1.0f, 0.0f); b.sizes = Vec3::make(0.5f, 0.5f, 0.5f);
    b.mat = make_mat(0.7f, 0.6f, 0.5f, 0.0f, 0.0f, OM_METAL);
    w->mbox.push_back(b);
    const Mat4 l2w = Mat4::translate(Vec3::make(0.0f, 1.0f, 0.0f)).mul(Mat4::rotate_x(0.6f)).mul(Mat4::rotate_z(1.33f * 2.0f * kPi));
    w->mtor.push_back(make_torus(l2w, Vec3::make(0.5f, 0.1f, 0.1f), make_mat(0, 0, 0, 0.0f, 1.5f, OM_DIELECTRIC)));
    return OM_OK;
}

const char* om_world_last_error_internal(void) { return g_last_error.c_str(); }

}  // extern "C"
