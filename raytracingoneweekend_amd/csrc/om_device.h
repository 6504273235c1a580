// om_device.h — device functions of the hot path (gfx950).
//
// Bit-exactness contract: every expression below performs the same IEEE f32
// operations, in the same order, as the Rust reference (cited per function);
// the translation unit is compiled with -ffp-contract=off and HIP's default
// correctly-rounded f32 division and sqrt, denormals preserved.  Rust's
// f32::max/min are NaN-ignoring -> fmaxf/fminf (v_max_f32/v_min_f32, IEEE mode).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "om_layout.h"
#include "../../include/ottomarcher.h"

namespace omd {

struct F3 { float x, y, z; };
__device__ __forceinline__ F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ F3 ld3(const float* p) { return f3(p[0], p[1], p[2]); }
__device__ __forceinline__ F3 add(F3 a, F3 b) { return f3(a.x + b.x, a.y + b.y, a.z + b.z); }    // vec3.rs:184-193
__device__ __forceinline__ F3 sub(F3 a, F3 b) { return f3(a.x - b.x, a.y - b.y, a.z - b.z); }    // vec3.rs:194-199 (x+(-y) == x-y in IEEE)
__device__ __forceinline__ F3 mul(F3 a, F3 b) { return f3(a.x * b.x, a.y * b.y, a.z * b.z); }    // vec3.rs:200-209
__device__ __forceinline__ F3 scl(F3 a, float s) { return f3(a.x * s, a.y * s, a.z * s); }       // vec3.rs:220-235
__device__ __forceinline__ F3 neg(F3 a) { return f3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(F3 a, F3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }    // vec3.rs:29-31
// Square roots of the march SDFs: hipcc's correctly rounded f32 sqrt (v_sqrt_f32 plus a
// +-1-ulp correction and its range handling).  A bare-core variant (range test skipped when a
// whole wave is in range) was bit-exact but neutral on C2 and -13% on C1 in unit() (a uniform
// branch in the divergent leaf loop), so sqrtf stays.
__device__ __forceinline__ float march_sqrt(float x) { return sqrtf(x); }
__device__ __forceinline__ F3 unit(F3 a) {                                                        // vec3.rs:35-40, 236-240
    const float len = sqrtf(dot(a, a));
    return scl(a, 1.0f / len);
}
__device__ __forceinline__ F3 at(F3 o, F3 d, float t) { return add(o, scl(d, t)); }              // ray.rs:14-16 (t*dir == dir*t)

// Mat4x4::dot_p3 / dot_v3 over a row-major 3x4 block (mat4x4.rs:49-57).
__device__ __forceinline__ F3 xform_p(const float* m, F3 p) {
    return f3(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3],
              m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
              m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
__device__ __forceinline__ F3 xform_v(const float* m, const float* z, F3 p) {
    return f3(m[0] * p.x + m[1] * p.y + m[2] * p.z + z[0],
              m[4] * p.x + m[5] * p.y + m[6] * p.z + z[1],
              m[8] * p.x + m[9] * p.y + m[10] * p.z + z[2]);
}

// ---------------------------------------------------------------- om-rng v2
// Per-path stream (replaces rand::thread_rng(), utils.rs:25): 32-bit Weyl counter s and
// 32-bit key k from one mix64 of (pixel << 32 | sample) ^ skey; a draw is
// lowbias32((s += 0x9E3779B9) ^ k) >> 8, times 2^-24 (rand 0.8's 24-bit f32 grid).
// Same as PathRng in oracle/om_oracle.cpp.
struct Rng {
    uint32_t s, k;
    __device__ __forceinline__ float next() {
        s += 0x9E3779B9u;
        uint32_t x = s ^ k;
        x ^= x >> 16; x *= 0x21F0AAADu;
        x ^= x >> 15; x *= 0x735A2D97u;
        x ^= x >> 15;
        return (float)(x >> 8) * 5.9604644775390625e-8f;
    }
    __device__ __forceinline__ float range(float lo, float hi) { const float r = next(); return r * (hi - lo) + lo; }  // utils.rs:26
};
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ __forceinline__ Rng path_rng(uint64_t skey, uint32_t pixel, uint32_t sample) {
    const uint64_t z = mix64((((uint64_t)pixel << 32) | (uint64_t)sample) ^ skey);
    Rng r; r.s = (uint32_t)z; r.k = (uint32_t)(z >> 32); return r;
}
__device__ __forceinline__ F3 rand_in_unit_sphere(Rng& g) {                                      // vec3.rs:92-97
    for (;;) {
        const float x = g.range(-1.0f, 1.0f);
        const float y = g.range(-1.0f, 1.0f);
        const float z = g.range(-1.0f, 1.0f);
        if (x * x + y * y + z * z < 1.0f) return f3(x, y, z);
    }
}

// ---------------------------------------------------------------- traced.rs
// Sphere::hit (traced.rs:39-62) up to the accepted root, from the ray in local space.
// FASTREJ: the division-free rejection below (bounce 0's tile lists: coherent waves often reject
// an occluded candidate together; in the later bounces' divergent leaf loop it measured -0.4%).
template <bool FASTREJ = false>
__device__ __forceinline__ bool sphere_root_local(F3 lo, F3 ld, float tmin, float tmax, float& root) {
    const float a = dot(ld, ld);
    const float half_b = dot(lo, ld);
    const float c = dot(lo, lo) - 1.0f;
    const float disc = half_b * half_b - a * c;
    if (disc < 0.0f) return false;
    const float sqrtd = sqrtf(disc);
    const float n1 = -half_b - sqrtd, n2 = -half_b + sqrtd;
    if (FASTREJ) {
    // Both roots provably outside [tmin, tmax] without the two correctly rounded divisions
    // (~24 VALU): for a > 0 in the normal range, n < (tmin*a)(1-2^-18) implies
    // fl(n/a) < tmin and n > (tmax*a)(1+2^-18) implies fl(n/a) > tmax, whatever the f32
    // rounding of the products and of the quotient (each within 2^-24 relative), and
    // r1 <= r2 because n1 <= n2.  Only rejections the reference makes are skipped (a ray
    // leaving the surface it just hit, the ground sphere behind the current hit ...);
    // NaNs fail every compare and take the exact path.
    if (a >= 1e-30f && a <= 1e30f) {
        const float lo = (tmin * a) * (1.0f - 0x1p-18f), hi = (tmax * a) * (1.0f + 0x1p-18f);
        if (n2 < lo || n1 > hi || (n1 < lo && n2 > hi)) return false;
    }
    }
    float r = n1 / a;
    if (r < tmin || r > tmax) {
        r = n2 / a;
        if (r < tmin || r > tmax) return false;
    }
    root = r;
    return true;
}
template <bool FASTREJ = false>
__device__ __forceinline__ bool sphere_root(const OmAffineTest& T, F3 o, F3 d, float tmin, float tmax, float& root) {
    return sphere_root_local<FASTREJ>(xform_p(T.w2l, o), xform_v(T.w2l, T.dz, d), tmin, tmax, root);
}
// The same test for a sphere whose world-to-local block is diagonal (off-diagonal entries
// exactly +-0: an axis-aligned scaled sphere such as random_scene's ground, main.rs:38-40).
// Each dropped term of ((m0*x + m1*y) + m2*z) + m3 is a signed zero, and adding a signed zero
// leaves every nonzero value unchanged, so lo and ld equal the full transform's up to the
// sign of a zero component.  A zero's sign reaches the roots only as -(+-0) - sqrtd with
// sqrtd = 0, i.e. a root of +-0, which tmin > 0 rejects either way; everything else
// (dot products of squares and sums with a nonzero term) is sign-blind.  Callers use it only
// when tmin > 0; the winner's HitRecord is still built by the full transform.
template <bool FASTREJ = false>
__device__ __forceinline__ bool sphere_root_diag(const OmAffineTest& T, F3 o, F3 d, float tmin, float tmax, float& root) {
    const F3 lo = f3(T.w2l[0] * o.x + T.w2l[3], T.w2l[5] * o.y + T.w2l[7], T.w2l[10] * o.z + T.w2l[11]);
    const F3 ld = f3(T.w2l[0] * d.x + T.dz[0], T.w2l[5] * d.y + T.dz[1], T.w2l[10] * d.z + T.dz[2]);
    return sphere_root_local<FASTREJ>(lo, ld, tmin, tmax, root);
}
// Cube::hit (traced.rs:266-298) up to (smallest_t, idx).
__device__ __forceinline__ bool cube_root(const OmAffineTest& T, F3 o, F3 d, float tmin, float tmax, float& root, int& axis) {
    const F3 lo = xform_p(T.w2l, o);
    const F3 ld = xform_v(T.w2l, T.dz, d);
    float smallest = INFINITY; int idx = -1;
    const float oo[3] = {lo.x, lo.y, lo.z}, dd[3] = {ld.x, ld.y, ld.z};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (fabsf(dd[i]) < 0.00001f) continue;
        const float t1 = (0.5f - oo[i]) / dd[i];
        const float t2 = (-0.5f - oo[i]) / dd[i];
        const float t = (t1 >= 0.0f && t2 >= 0.0f) ? fminf(t1, t2) : fmaxf(t1, t2);
        if (t > smallest || t > tmax || t < tmin) continue;
        const F3 p = at(lo, ld, t);
        const float f = fmaxf(fabsf(p.x), fmaxf(fabsf(p.y), fabsf(p.z)));
        if (!(fabsf(f - 0.5f) <= 0.00001f)) continue;
        smallest = t; idx = i;
    }
    if (idx < 0) return false;
    root = smallest; axis = idx;
    return true;
}
// ray_plane_intersect (traced.rs:92-99)
__device__ __forceinline__ void plane_isect(F3 n, F3 c, F3 o, F3 d, float& root, float& ndd) {
    const float div = dot(n, d);
    if (fabsf(div) < 0.000001f) { root = INFINITY; ndd = 0.0f; return; }
    const float num = -dot(n, sub(o, c));
    root = num / div; ndd = div;
}
// InfinitePlane::hit (traced.rs:106-114)
__device__ __forceinline__ bool plane_root(const OmPlane& P, F3 o, F3 d, float tmin, float tmax, float& root, float& ndd) {
    plane_isect(ld3(P.normal), ld3(P.center), o, d, root, ndd);
    return !(root == INFINITY || root < tmin || root > tmax);
}
// Barycentric::hit_aux (traced.rs:176-200), TRI: check_lambdas_triangle else _parallelogram.
template <bool TRI>
__device__ __forceinline__ bool bary_root(const OmBary& B, F3 o, F3 d, float tmin, float tmax, float& root, float& ndd) {
    float r, nd;
    plane_isect(ld3(B.uxv), ld3(B.origin), o, d, r, nd);
    if (r == INFINITY || r < tmin || r > tmax) return false;
    const F3 pfo = sub(at(o, d, r), ld3(B.origin));
    const float rx = B.base_inv[0] * pfo.x + B.base_inv[1] * pfo.y + B.base_inv[2] * pfo.z;      // Mat3x3::dot row 0
    const float ry = B.base_inv[6] * pfo.x + B.base_inv[7] * pfo.y + B.base_inv[8] * pfo.z;      // row 2 (.z())
    const float ux = 1.0f, uy = 0.0f, vx = B.vx, vy = B.vy;                                      // calc_barycentric :156-167
    const float det = ux * vy - vx * uy;
    const float l1 = ((rx * vy - vx * ry) / det) / B.u_length;
    const float l2 = (-(rx * uy - ux * ry) / det) / B.v_length;
    const float l3 = 1.0f - l1 - l2;
    bool ok;
    if (TRI) ok = l1 > 0.0f && l2 > 0.0f && l3 > 0.0f && l1 < 1.0f && l2 < 1.0f && l3 < 1.0f;   // :169-171
    else ok = l1 > 0.0f && l2 > 0.0f && l1 < 1.0f && l2 < 1.0f;                                  // :173-175
    if (!ok) return false;
    root = r; ndd = nd;
    return true;
}

// ---------------------------------------------------------------- marched.rs
__device__ __forceinline__ float len3(F3 a) { return march_sqrt(dot(a, a)); }
// MarchedSphere (marched.rs:56-76): to_local = p - w*center (w = 1)
__device__ __forceinline__ float msphere_sdf(const OmMSphere& S, F3 p) {
    const F3 c = ld3(S.center);
    return len3(f3(p.x - c.x * 1.0f, p.y - c.y * 1.0f, p.z - c.z * 1.0f)) - S.radius;
}
__device__ __forceinline__ F3 msphere_normal(const OmMSphere& S, F3 p) { return unit(sub(p, ld3(S.center))); }  // :60-63
// MarchedBox (marched.rs:85-102)
__device__ __forceinline__ float mbox_local(const OmMBox& B, F3 p) {
    const F3 q = f3(fabsf(p.x) - B.sizes[0], fabsf(p.y) - B.sizes[1], fabsf(p.z) - B.sizes[2]);
    const F3 m = f3(fmaxf(q.x, 0.0f), fmaxf(q.y, 0.0f), fmaxf(q.z, 0.0f));
    return len3(m) + fminf(fmaxf(q.x, fmaxf(q.y, q.z)), 0.0f);
}
__device__ __forceinline__ F3 mbox_to_local(const OmMBox& B, F3 p) {
    return f3(p.x - B.center[0] * 1.0f, p.y - B.center[1] * 1.0f, p.z - B.center[2] * 1.0f);
}
__device__ __forceinline__ float mbox_sdf(const OmMBox& B, F3 p) { return mbox_local(B, mbox_to_local(B, p)); }
// MarchedTorus (marched.rs:133-151); TT = OmMTorus or the march's SDF-only copy (om_trace.h)
template <class TT>
__device__ __forceinline__ float mtorus_local(const TT& T, F3 p) {
    const float qx = march_sqrt((p.x * p.x + p.z * p.z) + 0.0f * 0.0f) - T.sizes[0];
    return march_sqrt((qx * qx + p.y * p.y) + 0.0f * 0.0f) - T.sizes[1];
}
template <class TT>
__device__ __forceinline__ F3 mtorus_to_local(const TT& T, F3 p) {
    // Mat4x4::dot(p4 * w2l_s), p4 = (p, 1); only xyz are used by sdf
    const float s0 = p.x * T.w2l_s[0], s1 = p.y * T.w2l_s[1], s2 = p.z * T.w2l_s[2], s3 = 1.0f * T.w2l_s[3];
    const float* m = T.w2l_tr;
    return f3(m[0] * s0 + m[1] * s1 + m[2] * s2 + m[3] * s3,
              m[4] * s0 + m[5] * s1 + m[6] * s2 + m[7] * s3,
              m[8] * s0 + m[9] * s1 + m[10] * s2 + m[11] * s3);
}
template <class TT>
__device__ __forceinline__ float mtorus_sdf(const TT& T, F3 p) { return mtorus_local(T, mtorus_to_local(T, p)) * T.min_scale; }

// get_outward_local_normal (marched.rs:25-44)
template <class F>
__device__ __forceinline__ F3 outward_local_normal(F sdf, F3 p) {
    const float eps = 0.0000001f;
    const float x = sdf(f3(p.x + eps, p.y + 0.0f, p.z + 0.0f)) - sdf(f3(p.x + (-eps), p.y + (-0.0f), p.z + (-0.0f)));
    const float y = sdf(f3(p.x + 0.0f, p.y + eps, p.z + 0.0f)) - sdf(f3(p.x + (-0.0f), p.y + (-eps), p.z + (-0.0f)));
    const float z = sdf(f3(p.x + 0.0f, p.y + 0.0f, p.z + eps)) - sdf(f3(p.x + (-0.0f), p.y + (-0.0f), p.z + (-eps)));
    const F3 n = unit(f3(x, y, z));
    const F3 tdir = unit(n);                                                                      // Ray::new normalises
    const F3 zero = f3(0.0f, 0.0f, 0.0f);
    const float start_val = sdf(at(zero, tdir, 0.0f));
    const float end_val = sdf(at(zero, tdir, 1.0f));
    const float sign = (end_val > start_val) ? 1.0f : -1.0f;
    return scl(n, sign);
}
// Marched::get_outward_normal default (marched.rs:19-24)
__device__ __forceinline__ F3 mbox_normal(const OmMBox& B, F3 p) {
    const F3 lp = mbox_to_local(B, p);
    const F3 n = outward_local_normal([&](F3 q) { return mbox_local(B, q); }, lp);
    // to_world(n4) with n4.w = 0: n + 0*center
    return unit(f3(n.x + B.center[0] * 0.0f, n.y + B.center[1] * 0.0f, n.z + B.center[2] * 0.0f));
}
__device__ __forceinline__ F3 mtorus_normal(const OmMTorus& T, F3 p) {
    const F3 lp = mtorus_to_local(T, p);
    const F3 n = outward_local_normal([&](F3 q) { return mtorus_local(T, q); }, lp);
    // to_world = (l2w_tr . n4) * l2w_s, n4.w = 0 (marched.rs:145-147)
    const float* m = T.l2w_tr;
    const float w0 = 0.0f;
    const F3 r = f3(m[0] * n.x + m[1] * n.y + m[2] * n.z + m[3] * w0,
                    m[4] * n.x + m[5] * n.y + m[6] * n.z + m[7] * w0,
                    m[8] * n.x + m[9] * n.y + m[10] * n.z + m[11] * w0);
    return unit(f3(r.x * T.l2w_s[0], r.y * T.l2w_s[1], r.z * T.l2w_s[2]));
}

// A user marched object (`Arc<dyn Marched>`, hits.rs:96-100; om_world_add_marched_sdf): its
// local_sdf is a postfix program over a float stack, evaluated in program order with the op
// formulas of the typed objects (marched.rs:56-58, 86-89, 133-138).  The stack is eight named
// registers selected by unrolled compares (a runtime-indexed array would live in scratch memory).
struct SdfStack {
    float v[OM_SDF_MAX_STACK];
    __device__ __forceinline__ float get(uint32_t i) const {
        float r = v[0];
#pragma unroll
        for (uint32_t k = 1; k < OM_SDF_MAX_STACK; ++k) r = i == k ? v[k] : r;
        return r;
    }
    __device__ __forceinline__ void set(uint32_t i, float x) {
#pragma unroll
        for (uint32_t k = 0; k < OM_SDF_MAX_STACK; ++k) v[k] = i == k ? x : v[k];
    }
};
__device__ __forceinline__ float msdf_local(const OmSdfOp* ops, uint32_t n, F3 p) {
    SdfStack st;
#pragma unroll
    for (uint32_t k = 0; k < OM_SDF_MAX_STACK; ++k) st.v[k] = 0.0f;
    uint32_t sp = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const OmSdfOp o = ops[i];
        const F3 q = f3(p.x - o.a[0], p.y - o.a[1], p.z - o.a[2]);
        float v;
        if (o.op == OM_SDF_SPHERE) {
            v = len3(q) - o.a[3];
        } else if (o.op == OM_SDF_BOX) {
            const F3 b = f3(fabsf(q.x) - o.a[3], fabsf(q.y) - o.a[4], fabsf(q.z) - o.a[5]);
            v = len3(f3(fmaxf(b.x, 0.0f), fmaxf(b.y, 0.0f), fmaxf(b.z, 0.0f))) + fminf(fmaxf(b.x, fmaxf(b.y, b.z)), 0.0f);
        } else if (o.op == OM_SDF_TORUS) {
            const float qx = march_sqrt((q.x * q.x + q.z * q.z) + 0.0f * 0.0f) - o.a[3];
            v = march_sqrt((qx * qx + q.y * q.y) + 0.0f * 0.0f) - o.a[4];
        } else if (o.op == OM_SDF_ROUND) {
            sp -= 1u;
            v = st.get(sp) - o.a[0];
        } else {                                          // UNION / INTERSECT / SUBTRACT: b = pop, a = pop
            const float b = st.get(sp - 1u), a = st.get(sp - 2u);
            sp -= 2u;
            v = o.op == OM_SDF_UNION ? fminf(a, b) : o.op == OM_SDF_INTERSECT ? fmaxf(a, b) : fmaxf(a, -b);
        }
        st.set(sp, v);
        sp += 1u;
    }
    return st.get(0);
}
__device__ __forceinline__ float msdf_sdf(const OmMSdf& Q, const OmSdfOp* ops, F3 p) {     // Marched::sdf marched.rs:14-18
    return msdf_local(ops + Q.op_first, Q.op_count, mtorus_to_local(Q, p)) * Q.min_scale;
}
__device__ __forceinline__ F3 msdf_normal(const OmMSdf& Q, const OmSdfOp* ops, F3 p) {    // default get_outward_normal
    const F3 lp = mtorus_to_local(Q, p);
    const F3 n = outward_local_normal([&](F3 q) { return msdf_local(ops + Q.op_first, Q.op_count, q); }, lp);
    const float* m = Q.l2w_tr;
    const float w0 = 0.0f;
    const F3 r = f3(m[0] * n.x + m[1] * n.y + m[2] * n.z + m[3] * w0,
                    m[4] * n.x + m[5] * n.y + m[6] * n.z + m[7] * w0,
                    m[8] * n.x + m[9] * n.y + m[10] * n.z + m[11] * w0);
    return unit(f3(r.x * Q.l2w_s[0], r.y * Q.l2w_s[1], r.z * Q.l2w_s[2]));
}

// ---------------------------------------------------------------- materials.rs
__device__ __forceinline__ F3 reflect(F3 v, F3 n) { return sub(v, scl(n, 2.0f * dot(v, n))); }  // materials.rs:98-100
__device__ __forceinline__ F3 refract(F3 uv, F3 n, float eta) {                                 // materials.rs:102-108
    const float cos_theta = fminf(dot(neg(uv), n), 1.0f);
    const F3 perp = scl(add(uv, scl(n, cos_theta)), eta);
    const float aux = -sqrtf(fabsf(1.0f - dot(perp, perp)));
    return add(perp, scl(n, aux));
}
__device__ __forceinline__ float reflectance(float c, float ref_idx) {                          // materials.rs:110-116
    const float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    const float r0_2 = r0 * r0;
    const float cos_5 = (1.0f - c) * (1.0f - c) * (1.0f - c) * (1.0f - c) * (1.0f - c);
    return r0_2 + (1.0f - r0_2) * cos_5;
}
// Material::scatter (materials.rs:39-95); returns the unnormalised new direction
// (Ray::new normalises it, ray.rs:11-13) and the attenuation.
// Lambertian and Metal both draw one rand_in_unit_sphere before anything else that consumes the
// stream (reflect draws nothing), so a wave holding both kinds runs ONE rejection loop for them
// instead of one per kind (C1 +2.4%); each path's draws are unchanged.
__device__ __forceinline__ void scatter(const OmMaterial& m, F3 dir, F3 normal, Rng& g, F3& new_dir, F3& atten) {
    if (m.type != 2) {
        const F3 r = rand_in_unit_sphere(g);                                                     // materials.rs:54 / :64
        if (m.type == 0) {                                                                       // lambertian :52-61
            F3 nd = add(normal, unit(r));
            if (fabsf(nd.x) < 1e-8f && fabsf(nd.y) < 1e-8f && fabsf(nd.z) < 1e-8f) nd = normal;  // near_zero vec3.rs:69-72
            new_dir = nd;
        } else {                                                                                 // metal :62-66
            const F3 refl = reflect(dir, normal);
            new_dir = add(refl, scl(r, m.fuzz));
        }
        atten = ld3(m.albedo);
    } else {                                                                                     // dielectric :68-95
        const bool front = dot(dir, normal) < 0.0f;
        const float rr = front ? 1.0f / m.ior : m.ior;
        const F3 n = front ? normal : neg(normal);
        const float cos_theta = fminf(dot(neg(dir), n), 1.0f);
        const float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
        const bool cannot = (rr * sin_theta) > 1.0f;
        const bool by_refl = reflectance(cos_theta, rr) > g.next();                             // rand always drawn
        new_dir = (cannot || by_refl) ? reflect(dir, n) : refract(dir, n, rr);
        atten = f3(1.0f, 1.0f, 1.0f);
    }
}

// ---------------------------------------------------------------- Stats (render_thread.rs:23-39)
__device__ __forceinline__ uint8_t f32_as_u8(float f) {                                        // Rust `as u8`: saturating, NaN -> 0
    if (!(f > 0.0f)) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)f;
}
__device__ __forceinline__ uint8_t quantize(float c) {                                           // normalize_color + to_u8x3 (utils.rs:12-17, vec3.rs:74-76)
    return f32_as_u8(fminf(fmaxf(sqrtf(c), 0.0f), 0.999f) * 256.0f);
}
struct PixelState {
    uint64_t bloom; float sx, sy, sz; uint32_t n; float avg_depth; uint32_t bad; uint32_t rgbf;  // rgbf = color[3] | flags << 24
};
__device__ __forceinline__ bool stats_add(PixelState& st, F3 x, float depth, uint64_t bloom_bits) {
    const uint32_t old = st.rgbf & 0x00FFFFFFu;
    st.sx = st.sx + x.x; st.sy = st.sy + x.y; st.sz = st.sz + x.z;
    st.n += 1;
    const float inv = 1.0f / (float)st.n;                                                        // Vec3 / f32 = * (1/x)
    const uint32_t r = quantize(st.sx * inv), gq = quantize(st.sy * inv), b = quantize(st.sz * inv);
    const uint32_t col = r | (gq << 8) | (b << 16);
    const uint32_t bad_run = (old == col) ? 1u : 0u;
    st.bad = (st.bad + bad_run) * bad_run;
    const float nf = (float)st.n;
    st.avg_depth = ((nf - 1.0f) * st.avg_depth + depth) / nf;
    st.bloom |= bloom_bits;
    const bool done = st.bad >= 5;
    st.rgbf = col | (st.rgbf & 0xFF000000u) | (done ? 0x01000000u : 0u);
    return done;
}

}  // namespace omd
