// om_trace.h — closest-hit query over the frozen world (hits.rs:270-365) and the
// HitRecord of the winner; shared by the megakernel (om_render.hip) and the
// wavefront pipeline (om_wavefront.hip).
#pragma once
#include "om_device.h"
#include "om_layout.h"
#include "om_tuning.h"

namespace omd {

// Box plane k of a device BVH2 node (k: child 0 lo xyz, hi xyz; child 1 lo xyz, hi xyz).
template <int K> __device__ __forceinline__ float b2p(const OmBvh2NodeH& N);
template <int K> __device__ __forceinline__ float b2p(const OmBvh2Node& N) {
    return K < 3 ? N.lo0[K % 3] : K < 6 ? N.hi0[K % 3] : K < 9 ? N.lo1[K % 3] : N.hi1[K % 3];
}
// A half-precision box plane (OmBvh2NodeH) as f32, exactly.
__device__ __forceinline__ float h2f(uint16_t b) { return (float)__builtin_bit_cast(_Float16, b); }
template <int K> __device__ __forceinline__ float b2p(const OmBvh2NodeH& N) { return h2f(N.b[K]); }
// Plane P (lox loy loz hix hiy hiz) of child k of a 4-wide node, f32 or half.
template <int P> __device__ __forceinline__ float b4p(const OmBvh4Node& N, int k) {
    return P == 0 ? N.lox[k] : P == 1 ? N.loy[k] : P == 2 ? N.loz[k] : P == 3 ? N.hix[k] : P == 4 ? N.hiy[k] : N.hiz[k];
}
template <int P> __device__ __forceinline__ float b4p(const OmBvh4NodeH& N, int k) { return h2f(N.b[P * 4 + k]); }

// Slab-test min/max as IEEE minimum/maximum (NaN-propagating): gfx950's v_minimum3_f32 /
// v_maximum3_f32 need no canonicalising v_max x,x of the loop-carried t_lo / t_hi that fminf /
// fmaxf cost per node visit (an inline-asm v_min/v_max variant lost 12%: the compiler drains
// every outstanding load before an asm statement).  Culling only: a NaN slab value
// reaches near or far and every `!(near > far)` test then visits the box.
__device__ __forceinline__ float smin(float a, float b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ float smax(float a, float b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ float smin3(float a, float b, float c) { return smin(smin(a, b), c); }
__device__ __forceinline__ float smax3(float a, float b, float c) { return smax(smax(a, b), c); }
// near / far slab distances of one box: max(min(x), min(y), min(z), t_lo), min(max(x), max(y), max(z), t_hi)
__device__ __forceinline__ float slab_near(float x0, float x1, float y0, float y1, float z0, float z1, float t_lo) {
    return smax3(smin(x0, x1), smin(y0, y1), smax(smin(z0, z1), t_lo));
}
__device__ __forceinline__ float slab_far(float x0, float x1, float y0, float y1, float z0, float z1, float t_hi) {
    return smin3(smax(x0, x1), smax(y0, y1), smin(smax(z0, z1), t_hi));
}

// Inverse direction component for the conservative slab tests only (never an output value):
// the hardware reciprocal (1 ulp) instead of the correctly rounded division, ~10 VALU each.
// Boxes are inflated by 1e-3*(1+extent) and the t window is loosened by 1e-4 relative, far
// beyond its error; the component is kept >= 1e-20 in magnitude, so the result is finite.
__device__ __forceinline__ float inv_dir(float c) {
    const float k = fabsf(c) > 1e-20f ? c : copysignf(1e-20f, c);
    return __builtin_amdgcn_rcpf(k);
}

// Work counters (om_counters); compiled out (COUNT=false) of the production kernels so
// they cost no registers — the bench counts work in a separate, identical launch.
template <bool COUNT>
struct WorkT {
    uint32_t prim = 0, pre = 0, march = 0;
    __device__ __forceinline__ void add_prim() { if (COUNT) prim++; }
    __device__ __forceinline__ void add_pre(uint32_t k = 1) { if (COUNT) pre += k; }
    __device__ __forceinline__ void add_march() { if (COUNT) march++; }
};

// Exact test of global primitive gi with the brute-force acceptance (root <= tmax).
__device__ __forceinline__ bool test_prim(const OmSceneDev& S, uint32_t gi, F3 o, F3 d, float tmin, float tmax, float& t) {
    if (gi < S.off_cube) return sphere_root(S.sph_test[gi], o, d, tmin, tmax, t);
    if (gi < S.off_tri) { int ax; return cube_root(S.cube_test[gi - S.off_cube], o, d, tmin, tmax, t, ax); }
    float ndd;
    if (gi < S.off_plane) return bary_root<true>(S.tri[gi - S.off_tri], o, d, tmin, tmax, t, ndd);
    if (gi < S.off_para) return plane_root(S.plane[gi - S.off_plane], o, d, tmin, tmax, t, ndd);
    return bary_root<false>(S.para[gi - S.off_para], o, d, tmin, tmax, t, ndd);
}

// Reference order brute force: FrozenHittableList::hit traced section (hits.rs:272-285).
// CULL: skip spheres whose conservative bounding sphere proves the exact test
// would return None — the accepted sequence is unchanged.
template <bool CULL, class Wk>
__device__ __forceinline__ int traced_brute(const OmSceneDev& S, F3 o, F3 d, float tmin, float& closest, Wk& w) {
    int best = -1;
    float t;
    for (uint32_t i = 0; i < S.n_sph; ++i) {
        if (CULL) {
            const OmBound B = S.sph_bound[i];
            const float ocx = o.x - B.c[0], ocy = o.y - B.c[1], ocz = o.z - B.c[2];
            const float b = ocx * d.x + ocy * d.y + ocz * d.z;
            const float px = ocx - b * d.x, py = ocy - b * d.y, pz = ocz - b * d.z;
            const float q = px * px + py * py + pz * pz;
            w.add_pre();
            // every comparison is false for NaN -> the exact test decides
            if (q > B.r * B.r || -b + B.r < tmin || -b - B.r > closest) continue;
        }
        w.add_prim();
        if (sphere_root(S.sph_test[i], o, d, tmin, closest, t)) { closest = t; best = (int)i; }
    }
    for (uint32_t i = 0; i < S.n_cube; ++i) {
        int ax; w.add_prim();
        if (cube_root(S.cube_test[i], o, d, tmin, closest, t, ax)) { closest = t; best = (int)(S.off_cube + i); }
    }
    float ndd;
    for (uint32_t i = 0; i < S.n_tri; ++i) {
        w.add_prim();
        if (bary_root<true>(S.tri[i], o, d, tmin, closest, t, ndd)) { closest = t; best = (int)(S.off_tri + i); }
    }
    for (uint32_t i = 0; i < S.n_plane; ++i) {
        w.add_prim();
        if (plane_root(S.plane[i], o, d, tmin, closest, t, ndd)) { closest = t; best = (int)(S.off_plane + i); }
    }
    for (uint32_t i = 0; i < S.n_para; ++i) {
        w.add_prim();
        if (bary_root<false>(S.para[i], o, d, tmin, closest, t, ndd)) { closest = t; best = (int)(S.off_para + i); }
    }
    return best;
}

// BVH traversal with the brute-force tie rule: the reference keeps the smallest
// accepted root and, on equal roots, the later object in type order.
template <class Wk>
__device__ __forceinline__ void offer(const OmSceneDev& S, uint32_t gi, F3 o, F3 d, float tmin, float& closest, int& best, Wk& w) {
    float t;
    w.add_prim();
    if (test_prim(S, gi, o, d, tmin, closest, t)) {
        if (t < closest || (int)gi > best) { closest = t; best = (int)gi; }
    }
}

template <class Wk>
__device__ __forceinline__ int traced_bvh(const OmSceneDev& S, F3 o, F3 d, float tmin, float& closest, Wk& w) {
    // Non-finite rays take the reference loop (NaN roots are accepted there).
    if (!isfinite(o.x + o.y + o.z + d.x + d.y + d.z)) return traced_brute<false, Wk>(S, o, d, tmin, closest, w);
    int best = -1;
    for (uint32_t k = 0; k < S.n_always; ++k) offer(S, S.always[k], o, d, tmin, closest, best, w);
    if (S.n_bvh_nodes == 0) return best;
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    const float t_lo = tmin * 0.5f - 1e-3f;
    uint32_t stack[64];
    int sp = 0;
    uint32_t node = 0;
    for (;;) {
        const OmBvhNode N = S.bvh[node];
        if (N.left < 0) {
            const uint32_t first = (uint32_t)(-N.left - 1), cnt = (uint32_t)N.right;
            for (uint32_t k = 0; k < cnt; ++k) offer(S, S.bvh_prims[first + k], o, d, tmin, closest, best, w);
        } else {
            const OmBvhNode L = S.bvh[N.left], R = S.bvh[N.right];
            w.add_pre(2);
            // Slab tests on inflated boxes, (lo - o) * (1/d): a zero direction component
            // gives +-inf (correct containment) or NaN (dropped by fminf/fmaxf = unconstrained).
            const float t_hi = closest * 1.0001f + 1e-3f;
            float x0 = (L.lo[0] - o.x) * ix, x1 = (L.hi[0] - o.x) * ix;
            float y0 = (L.lo[1] - o.y) * iy, y1 = (L.hi[1] - o.y) * iy;
            float z0 = (L.lo[2] - o.z) * iz, z1 = (L.hi[2] - o.z) * iz;
            const float ln = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
            const float lf = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
            x0 = (R.lo[0] - o.x) * ix; x1 = (R.hi[0] - o.x) * ix;
            y0 = (R.lo[1] - o.y) * iy; y1 = (R.hi[1] - o.y) * iy;
            z0 = (R.lo[2] - o.z) * iz; z1 = (R.hi[2] - o.z) * iz;
            const float rn = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
            const float rf = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
            const bool hl = !(ln > lf), hr = !(rn > rf);
            if (hl && hr) {
                const bool left_first = ln <= rn;
                stack[sp++] = left_first ? (uint32_t)N.right : (uint32_t)N.left;
                node = left_first ? (uint32_t)N.left : (uint32_t)N.right;
                continue;
            }
            if (hl) { node = (uint32_t)N.left; continue; }
            if (hr) { node = (uint32_t)N.right; continue; }
        }
        if (sp == 0) break;
        node = stack[--sp];
    }
    return best;
}

// A record at a wave-uniform address, read through the constant address space: scalar loads
// (s_load, the scalar cache) instead of vector loads, which the compiler must otherwise use
// because the kernels' global stores may alias the scene arrays (they never do: the scene is
// immutable while a kernel runs, om_upload_world happens between calls).  The always2 records
// are read by every ray of every wave: through the vector path each one was a dependent L2
// round trip queued behind the path-state streams (C1 +3.1%).
template <class T>
__device__ __forceinline__ T uniform_load(const T* p) {
    static_assert(sizeof(T) % 4 == 0, "dword records");
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    cu32* q = (cu32*)p;
    T r;
    uint32_t* d = (uint32_t*)&r;
#pragma unroll
    for (uint32_t i = 0; i < sizeof(T) / 4; ++i) d[i] = q[i];
    return r;
}

// Exact test of global primitive gi (wave-uniform) with the reference's acceptance, the record
// read by uniform_load.
template <class Wk>
__device__ __forceinline__ void offer_uniform(const OmSceneDev& S, uint32_t gi, F3 o, F3 d, float tmin, float& closest, int& best,
                                             Wk& w) {
    float t, ndd;
    bool h;
    w.add_prim();
    if (gi < S.off_cube) h = sphere_root(uniform_load(S.sph_test + gi), o, d, tmin, closest, t);
    else if (gi < S.off_tri) { int ax; h = cube_root(uniform_load(S.cube_test + (gi - S.off_cube)), o, d, tmin, closest, t, ax); }
    else if (gi < S.off_plane) h = bary_root<true>(uniform_load(S.tri + (gi - S.off_tri)), o, d, tmin, closest, t, ndd);
    else if (gi < S.off_para) h = plane_root(uniform_load(S.plane + (gi - S.off_plane)), o, d, tmin, closest, t, ndd);
    else h = bary_root<false>(uniform_load(S.para + (gi - S.off_para)), o, d, tmin, closest, t, ndd);
    if (h && (t < closest || (int)gi > best)) { closest = t; best = (int)gi; }
}

// The primitives outside the BVH trees (always2), in index order: conservative box first, then
// the exact test with the brute-force tie rule.  An unbounded record (huge primitives, planes:
// lo = -inf) passes every slab test, so it skips it (+0.6% on C1); one flagged as an
// axis-aligned sphere (the ground) takes sphere_root_diag (same accepted root, 24 fewer VALU).
template <class Wk>
__device__ __forceinline__ void offer_always2(const OmSceneDev& S, F3 o, F3 d, float tmin, float ix, float iy, float iz,
                                              float nox, float noy, float noz, float t_lo, float& closest, int& best, Wk& w) {
    for (uint32_t k = 0; k < S.n_always2; ++k) {
        const OmAlwaysRec A = uniform_load(S.always2_rec + k);
        if (A.lo[0] == -INFINITY) {
            if (A.pad == OM_ALWAYS_DIAG_SPHERE && tmin > 0.0f) {
                float t;
                w.add_prim();
                if (sphere_root_diag(uniform_load(S.sph_test + A.gi), o, d, tmin, closest, t) && (t < closest || (int)A.gi > best)) {
                    closest = t; best = (int)A.gi;
                }
            } else {
                offer_uniform(S, A.gi, o, d, tmin, closest, best, w);
            }
            continue;
        }
        w.add_pre();
        const float t_hi = closest * 1.0001f + 1e-3f;
        const float x0 = __builtin_fmaf(A.lo[0], ix, nox), x1 = __builtin_fmaf(A.hi[0], ix, nox);
        const float y0 = __builtin_fmaf(A.lo[1], iy, noy), y1 = __builtin_fmaf(A.hi[1], iy, noy);
        const float z0 = __builtin_fmaf(A.lo[2], iz, noz), z1 = __builtin_fmaf(A.hi[2], iz, noz);
        const float n0 = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
        const float f0 = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
        if (!(n0 > f0)) offer_uniform(S, A.gi, o, d, tmin, closest, best, w);
    }
}

// One leaf record (Sphere/Cube test record, tag bit 31 = cube), brute-force tie rule.
template <bool FASTREJ = false, class Wk>
__device__ __forceinline__ void test_rec(const OmAffineTest& R, F3 o, F3 d, float tmin, float& closest, int& best, Wk& w) {
    uint32_t tag;
    __builtin_memcpy(&tag, &R.pad, 4);
    const uint32_t gi = tag & 0x7FFFFFFFu;
    float t;
    int ax;
    w.add_prim();
    const bool h = (tag >> 31) ? cube_root(R, o, d, tmin, closest, t, ax) : sphere_root<FASTREJ>(R, o, d, tmin, closest, t);
    if (h && (t < closest || (int)gi > best)) { closest = t; best = (int)gi; }
}

// (first record << 8) | count of the leaf with child code `code`: straight from a direct code
// (OM_LEAF | first << 4 | count, om_bvh.cpp), else from the leaf table.
__device__ __forceinline__ uint32_t leaf_payload(const OmSceneDev& S, uint32_t code, const uint32_t* leaves) {
    return S.b2_direct ? ((((code >> 4) & 0x7FFu) << 8) | (code & 15u)) : leaves[code & (OM_LEAF - 1u)];
}

// Leaf of the BVH2/BVH4: its records, tested in place.
template <class Wk>
__device__ __forceinline__ void test_leaf(const OmAffineTest* recs, uint32_t lf, F3 o, F3 d, float tmin, float& closest,
                                          int& best, Wk& w) {
    const uint32_t first = lf >> 8, cnt = lf & 255u;
    for (uint32_t k = 0; k < cnt; ++k) test_rec(recs[first + k], o, d, tmin, closest, best, w);
}


// Stackless BVH traversal.  Nodes are visited in depth-first
// order: box hit -> next node (internal) or the leaf's records then `skip`; miss ->
// `skip`.  No per-lane stack (no scratch), one 32-B node read per step.  The box test
// only decides which exact tests run, so it may use FMA (it never touches output bits):
// boxes are inflated far beyond its rounding, the direction is kept away from 0 so
// every slab value is finite, and NaN compares fall through to "visit".
// NODES/RECS point into LDS (staged once per workgroup) or into global memory.
template <class Wk>
__device__ __forceinline__ int traced_sbvh(const OmSceneDev& S, const OmSkipNode* nodes, const OmAffineTest* recs,
                                           F3 o, F3 d, float tmin, float& closest, Wk& w) {
    if (!isfinite(o.x + o.y + o.z + d.x + d.y + d.z)) return traced_brute<false, Wk>(S, o, d, tmin, closest, w);
    int best = -1;
    const float ix = inv_dir(d.x);
    const float iy = inv_dir(d.y);
    const float iz = inv_dir(d.z);
    const float nox = -o.x * ix, noy = -o.y * iy, noz = -o.z * iz;
    const float t_lo = tmin * 0.5f - 1e-3f;
    offer_always2(S, o, d, tmin, ix, iy, iz, nox, noy, noz, t_lo, closest, best, w);
    const uint32_t n = S.n_snodes;
    uint32_t node = 0;
    while (node < n) {
        const OmSkipNode N = nodes[node];
        w.add_pre();
        const float t_hi = closest * 1.0001f + 1e-3f;
        const float x0 = __builtin_fmaf(N.lo[0], ix, nox), x1 = __builtin_fmaf(N.hi[0], ix, nox);
        const float y0 = __builtin_fmaf(N.lo[1], iy, noy), y1 = __builtin_fmaf(N.hi[1], iy, noy);
        const float z0 = __builtin_fmaf(N.lo[2], iz, noz), z1 = __builtin_fmaf(N.hi[2], iz, noz);
        const float tn = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
        const float tf = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
        if (!(tn > tf)) {
            if (N.leaf == 0xFFFFFFFFu) { node++; continue; }
            const uint32_t first = N.leaf >> 8, cnt = N.leaf & 255u;
            for (uint32_t k = 0; k < cnt; ++k) {
                const OmAffineTest R = recs[first + k];
                uint32_t tag;
                __builtin_memcpy(&tag, &R.pad, 4);
                const uint32_t gi = tag & 0x7FFFFFFFu;
                float t;
                int ax;
                w.add_prim();
                const bool h = (tag >> 31) ? cube_root(R, o, d, tmin, closest, t, ax) : sphere_root(R, o, d, tmin, closest, t);
                if (h && (t < closest || (int)gi > best)) { closest = t; best = (int)gi; }
            }
        }
        node = N.skip;
    }
    return best;
}

// The marched objects of a world, seen by the march loop through one of three views:
//  MarchedArrays  the scene arrays, any count (each step reloads every object's parameters
//                 with scalar loads: runtime-bounded loops over memory);
//  MarchedRegs    a copy of at most KS spheres, KB boxes and KT tori taken once before the
//                 loop, so the parameters stay in (scalar) registers across the steps;
//  MarchedExact   a copy of EXACTLY NS spheres, NB boxes and NT tori with only the fields the
//                 march reads (a torus: 24 of its 43 floats), taken once per kernel: fully
//                 unrolled steps with no count guards, the parameters in SGPRs.
// All visit the objects in the same order with the same arithmetic.  INDEXED: the view may be
// indexed at run time (arrays); the register views are only ever indexed by unrolled counters.
struct MarchedArrays {
    static constexpr uint32_t KS = 0u, KB = 0u, KT = 0u;      // 0: unbounded
    static constexpr bool INDEXED = true;
    static constexpr bool RELOAD = false;
    static constexpr bool USER = true;                         // visits the user objects (OmMSdf) too
    const OmMSphere* s; const OmMBox* b; const OmMTorus* t;
    const OmMSdf* q; const OmSdfOp* qo;
    uint32_t ns, nb, nt, nq;
    __device__ explicit MarchedArrays(const OmSceneDev& S)
        : s(S.msph), b(S.mbox), t(S.mtor), q(S.msdf), qo(S.msdf_ops), ns(S.n_msph), nb(S.n_mbox), nt(S.n_mtor),
          nq(S.n_msdf) {}
};
template <uint32_t KS_, uint32_t KB_, uint32_t KT_>
struct MarchedRegs {
    static constexpr uint32_t KS = KS_, KB = KB_, KT = KT_;
    static constexpr bool INDEXED = false;
    static constexpr bool RELOAD = false;
    static constexpr bool USER = false;
    OmMSphere s[KS]; OmMBox b[KB]; OmMTorus t[KT];
    uint32_t ns, nb, nt;
    __device__ explicit MarchedRegs(const OmSceneDev& S) : ns(S.n_msph), nb(S.n_mbox), nt(S.n_mtor) {
#pragma unroll
        for (uint32_t i = 0; i < KS; ++i) if (i < ns) s[i] = S.msph[i];
#pragma unroll
        for (uint32_t i = 0; i < KB; ++i) if (i < nb) b[i] = S.mbox[i];
#pragma unroll
        for (uint32_t i = 0; i < KT; ++i) if (i < nt) t[i] = S.mtor[i];
    }
    __device__ static bool fits(const OmSceneDev& S) {
        return S.n_msph <= KS && S.n_mbox <= KB && S.n_mtor <= KT && S.n_msdf == 0u;
    }
};
using MarchedSmall = MarchedRegs<4, 2, 1>;   // S-marched (2, 1, 1), S-full (0, 0, 1)

// What mtorus_sdf and the march cull read of a torus (mtorus_to_local uses the first three
// rows of W2L_TR and all of w2l_s, mtorus_local the two sizes): 24 floats of the 43.
struct MTorusSdf {
    float w2l_tr[12]; float w2l_s[4]; float sizes[2]; float min_scale, bk, br; float bc[3];
    __device__ void load(const OmMTorus& T) {
#pragma unroll
        for (int k = 0; k < 12; ++k) w2l_tr[k] = T.w2l_tr[k];
#pragma unroll
        for (int k = 0; k < 4; ++k) w2l_s[k] = T.w2l_s[k];
        sizes[0] = T.sizes[0]; sizes[1] = T.sizes[1];
        min_scale = T.min_scale; bk = T.bk; br = T.br;
        bc[0] = T.bc[0]; bc[1] = T.bc[1]; bc[2] = T.bc[2];
    }
};
// An exact-count view: EXACTLY NS spheres, NB boxes and NT tori with only the fields the march
// reads (a torus: 24 of its 43 floats, MTorusSdf), staged in LDS once per workgroup (the
// north_star's "LDS-staged SDF params", k_march): fully unrolled steps with no
// count guards, every step reads them with broadcast ds_reads at constant offsets.
template <uint32_t NS, uint32_t NB, uint32_t NT>
struct MarchedExactLds {
    static constexpr uint32_t KS = NS, KB = NB, KT = NT;
    static constexpr bool INDEXED = false;
    // re-read every step (a compiler-only fence in nearest_marched): hoisted out of the march loop
    // the parameters would sit in VGPRs (64 + 23 spilled) instead of LDS
    static constexpr bool RELOAD = true;
    static constexpr bool USER = false;                        // (run_batch picks it only without user objects)
    static constexpr uint32_t ns = NS, nb = NB, nt = NT;
    struct Block { OmMSphere s[NS ? NS : 1]; OmMBox b[NB ? NB : 1]; MTorusSdf t[NT ? NT : 1]; };
    const OmMSphere* s; const OmMBox* b; const MTorusSdf* t;
    __host__ __device__ static bool matches(uint32_t n_s, uint32_t n_b, uint32_t n_t) { return n_s == NS && n_b == NB && n_t == NT; }
    // every thread of the block calls it (it ends with a barrier)
    __device__ MarchedExactLds(const OmSceneDev& S, Block* lds) : s(lds->s), b(lds->b), t(lds->t) {
        const uint32_t i = threadIdx.x;
        if (i < NS) lds->s[i] = S.msph[i];
        else if (i < NS + NB) lds->b[i - NS] = S.mbox[i - NS];
        else if (i < NS + NB + NT) lds->t[i - NS - NB].load(S.mtor[i - NS - NB]);
        __syncthreads();
    }
};

// for (i < n) body(i): unrolled over the register view's bound, a plain loop otherwise (K = 0:
// the arrays view's runtime count, or an exact view's constant 0, which folds away)
template <uint32_t K, class F>
__device__ __forceinline__ void for_objects(uint32_t n, F body) {
    if constexpr (K == 0u) {
        for (uint32_t i = 0; i < n; ++i) body(i);
    } else {
#pragma unroll
        for (uint32_t i = 0; i < K; ++i) if (i < n) body(i);
    }
}

// Nearest marched object at p: min |sdf| over the marched objects in type order, strict '<'
// (the first minimum wins; hits.rs:296-322, 341-358).  An object whose conservative lower
// bound (om_world.cpp) proves |sdf| > best cannot be the new minimum and is skipped: the
// result is bit-identical to evaluating every SDF.  -> best (INFINITY if none), kind, index.

template <class M>
__device__ __forceinline__ float nearest_marched(const M& m, F3 p, int& bk, uint32_t& bi) {
    if constexpr (M::RELOAD) __atomic_signal_fence(__ATOMIC_SEQ_CST);
    float best = INFINITY;
    bk = -1; bi = 0;
    for_objects<M::KS>(m.ns, [&](uint32_t i) {
        const float v = fabsf(msphere_sdf(m.s[i], p));
        if (v < best) { best = v; bk = 0; bi = i; }
    });
    // The cull skips an object only when no active lane of the wave needs it (a scalar branch on
    // the ballot, no exec-mask split); the lanes that do not need it then evaluate it too, and
    // their `need` keeps the result as the cull would (r06: C2 +2.0%, SALU -16%, r06_ab4)
    for_objects<M::KB>(m.nb, [&](uint32_t i) {
        const OmMBox& B = m.b[i];
        const float dx = p.x - B.center[0], dy = p.y - B.center[1], dz = p.z - B.center[2];
        const float thr = (best + B.br) * 1.0001f;                             // inf/NaN -> evaluate
        const bool need = !(dx * dx + dy * dy + dz * dz > thr * thr);
        if (__ballot(need) == 0) return;
        const float v = fabsf(mbox_sdf(B, p));
        if (need && v < best) { best = v; bk = 1; bi = i; }
    });
    for_objects<M::KT>(m.nt, [&](uint32_t i) {
        const auto& T = m.t[i];
        const float dx = p.x - T.bc[0], dy = p.y - T.bc[1], dz = p.z - T.bc[2];
        const float thr = best * T.bk + T.br;                                  // inf/NaN -> evaluate
        const bool need = !(dx * dx + dy * dy + dz * dz > thr * thr);
        if (__ballot(need) == 0) return;
        const float v = fabsf(mtorus_sdf(T, p));
        if (need && v < best) { best = v; bk = 2; bi = i; }
    });
    if constexpr (M::USER) {                                   // Arc<dyn Marched> objects last (hits.rs:312-319)
        for (uint32_t i = 0; i < m.nq; ++i) {
            const float v = fabsf(msdf_sdf(m.q[i], m.qo, p));
            if (v < best) { best = v; bk = 3; bi = i; }
        }
    }
    return best;
}

// |sdf| of the one marched object (kind, idx) at q.  The register view is only ever indexed
// by unrolled loop counters (a runtime index would move it to scratch memory).
template <class M>
__device__ __forceinline__ float sdf_one(const M& m, int kind, uint32_t idx, F3 q) {
    if constexpr (M::INDEXED) {
        if constexpr (M::USER) if (kind == 3) return fabsf(msdf_sdf(m.q[idx], m.qo, q));
        return kind == 0 ? fabsf(msphere_sdf(m.s[idx], q)) : kind == 1 ? fabsf(mbox_sdf(m.b[idx], q)) : fabsf(mtorus_sdf(m.t[idx], q));
    } else {
        float v = 0.0f;
        if (kind == 0) for_objects<M::KS>(m.ns, [&](uint32_t i) { if (i == idx) v = fabsf(msphere_sdf(m.s[i], q)); });
        else if (kind == 1) for_objects<M::KB>(m.nb, [&](uint32_t i) { if (i == idx) v = fabsf(mbox_sdf(m.b[i], q)); });
        else for_objects<M::KT>(m.nt, [&](uint32_t i) { if (i == idx) v = fabsf(mtorus_sdf(m.t[i], q)); });
        return v;
    }
}

// unstuck (hits.rs:336-365): the start of the sphere-tracing loop.  Returns false when the
// world has no marched objects (hits.rs:359); otherwise t is where the march starts.
template <class M>
__device__ __forceinline__ bool march_begin(const M& m, F3 o, F3 d, float tmin, float& t) {
    const float HIT = 0.001f;
    int kind;
    uint32_t idx;
    const float dist = nearest_marched(m, at(o, d, tmin), kind, idx);     // r.at(tmin)
    if (kind < 0) return false;                                                // hits.rs:359
    t = tmin;
    float aux = dist;
    uint32_t guard = 0;
    while (aux < HIT && guard++ < (1u << 22)) {                                // hits.rs:360-363 (+ safety cap)
        t += HIT / 2.0f;
        const F3 q = at(o, d, t);
        aux = sdf_one(m, kind, idx, q);
    }
    return true;
}

// One iteration of the sphere-tracing loop (hits.rs:294-332).  Returns 0 to continue, 1 on
// a hit (gi = the marched winner's global index, the hit is at t), 2 when the march ends
// without one.
template <class M, class Wk>
__device__ __forceinline__ int march_step(const OmSceneDev& S, const M& m, F3 o, F3 d, float tmax, float closest, float& t,
                                          uint32_t& iters, int& gi, Wk& w) {
    const float HIT = 0.001f;
    if (!(t < tmax && t < closest && iters > 0)) return 2;                    // hits.rs:294
    const F3 p = at(o, d, t);
    iters -= 1;
    w.add_march();
    int bk;
    uint32_t bi;
    const float best = nearest_marched(m, p, bk, bi);
    if (bk < 0) return 2;                                                      // hits.rs:323
    if (best < HIT) {                                                          // hits.rs:325-327
        gi = (int)(bk == 0 ? S.off_msph + bi : bk == 1 ? S.off_mbox + bi : bk == 2 ? S.off_mtor + bi : S.off_msdf + bi);
        return 1;
    }
    t += best;                                                                 // hits.rs:330
    return 0;
}

template <class M, class Wk>
__device__ __forceinline__ int march_with(const OmSceneDev& S, const M& m, F3 o, F3 d, float tmin, float tmax, float closest,
                                          uint32_t steps, float& t_hit, Wk& w) {
    float t;
    if (!march_begin(m, o, d, tmin, t)) return -1;
    uint32_t iters = steps;
    int gi = -1, r;
    while ((r = march_step(S, m, o, d, tmax, closest, t, iters, gi, w)) == 0) {}
    if (r == 1) { t_hit = t; return gi; }
    return -1;
}

// unstuck + sphere-tracing loop (hits.rs:287-365).  Returns the marched winner's global
// index or -1; `t_hit` receives the hit t.  Small marched sets (every reference scene) are
// copied to registers once per call instead of reloaded at every step.
template <class Wk>
__device__ __forceinline__ int march(const OmSceneDev& S, F3 o, F3 d, float tmin, float tmax, float closest,
                                     uint32_t steps, float& t_hit, Wk& w) {
    if (MarchedSmall::fits(S)) return march_with(S, MarchedSmall(S), o, d, tmin, tmax, closest, steps, t_hit, w);
    return march_with(S, MarchedArrays(S), o, d, tmin, tmax, closest, steps, t_hit, w);
}

// Build the HitRecord of the winner (point, normal) — the winner's own exact
// test re-run with tmax = its root reproduces the same root bit for bit.
// MARCH = false (worlds without marched primitives, a compile-time split like the trace's):
// the marched winners' normal code (central differences, ~60 sqrt/div) is left out.
// USER: the world may hold user marched objects (OmMSdf): their normal runs the SDF program 7 times,
// whose registers must not weigh on the kernels of worlds without them (C2's shade and tail).
template <bool MARCH = true, bool USER = MARCH>
__device__ __forceinline__ void finalize(const OmSceneDev& S, int gi, F3 o, F3 d, float tmin, float t, F3& point, F3& normal) {
    const uint32_t g = (uint32_t)gi;
    if (g < S.off_tri) {                                                       // Sphere / Cube
        const bool cube = g >= S.off_cube;
        const OmAffineTest& T = cube ? S.cube_test[g - S.off_cube] : S.sph_test[g];
        const OmAffineHit& H = cube ? S.cube_hit[g - S.off_cube] : S.sph_hit[g];
        const F3 lo = xform_p(T.w2l, o), ld = xform_v(T.w2l, T.dz, d);
        const F3 lp = at(lo, ld, t);
        point = xform_p(H.l2w, lp);
        if (!cube) {
            normal = unit(xform_v(H.l2w, H.lz, lp));                           // traced.rs:59
        } else {
            float r; int ax = 0;
            cube_root(T, o, d, tmin, t, r, ax);
            // traced.rs:293-296: axis * copysign(1, p[idx]); normal NOT normalised
            const float comp = ax == 0 ? lp.x : (ax == 1 ? lp.y : lp.z);
            const float s = copysignf(1.0f, comp);
            const F3 ln = f3((ax == 0 ? 1.0f : 0.0f) * s, (ax == 1 ? 1.0f : 0.0f) * s, (ax == 2 ? 1.0f : 0.0f) * s);
            normal = xform_v(H.l2w, H.lz, ln);
        }
        return;
    }
    if (g < S.off_msph) {                                                      // plane / barycentric
        F3 n, c;
        if (g < S.off_plane) { n = ld3(S.tri[g - S.off_tri].uxv); c = ld3(S.tri[g - S.off_tri].origin); }
        else if (g < S.off_para) { n = ld3(S.plane[g - S.off_plane].normal); c = ld3(S.plane[g - S.off_plane].center); }
        else { n = ld3(S.para[g - S.off_para].uxv); c = ld3(S.para[g - S.off_para].origin); }
        float r, ndd;
        plane_isect(n, c, o, d, r, ndd);
        point = at(o, d, t);
        normal = scl(n, copysignf(1.0f, -ndd));                                // traced.rs:101-103
        return;
    }
    point = at(o, d, t);                                                       // marched (hits.rs:326)
    if (!MARCH) { normal = f3(0.0f, 0.0f, 0.0f); return; }                    // unreachable: no marched winner
    if (g < S.off_mbox) normal = msphere_normal(S.msph[g - S.off_msph], point);
    else if (g < S.off_mtor) normal = mbox_normal(S.mbox[g - S.off_mbox], point);
    else if (!USER || g < S.off_msdf) normal = mtorus_normal(S.mtor[g - S.off_mtor], point);
    else normal = msdf_normal(S.msdf[g - S.off_msdf], S.msdf_ops, point);
}

}  // namespace omd

namespace omd {

// render_thread.rs:183-192 + Camera::get_ray (camera.rs:60-65): the primary ray of
// sample s of pixel (i_f, j_f); g is the path's fresh om-rng stream.
__device__ __forceinline__ void gen_camera_ray(const OmCamDev& C, const OmParamsDev& P, const float2* jitter,
                                               float i_f, float j_f, uint32_t s, Rng& g, F3& o, F3& d) {
    const float2 jt = jitter[s];
    const float i_rand = (g.next() + jt.x) / 2.0f;
    const float j_rand = (g.next() + jt.y) / 2.0f;
    const float u = (i_f + i_rand) / P.wf_m1;
    const float v = 1.0f - (j_f + j_rand) / P.hf_m1;
    float dx, dy;
    for (;;) {                                                     // rand_in_unit_disc vec3.rs:108-113
        dx = g.range(-1.0f, 1.0f);
        dy = g.range(-1.0f, 1.0f);
        if (dx * dx + dy * dy < 1.0f) break;
    }
    const float rlx = dx * C.lens_radius, rly = dy * C.lens_radius;
    const F3 off = f3(C.u[0] * rlx + C.v[0] * rly, C.u[1] * rlx + C.v[1] * rly, C.u[2] * rlx + C.v[2] * rly);
    // uv_to_dir . (u, v, 0, 1): ((H*u + V*v) + 0*0) + D*1
    const F3 dir = f3((C.horizontal[0] * u + C.vertical[0] * v) + 0.0f * 0.0f + C.llc_minus_origin[0],
                      (C.horizontal[1] * u + C.vertical[1] * v) + 0.0f * 0.0f + C.llc_minus_origin[1],
                      (C.horizontal[2] * u + C.vertical[2] * v) + 0.0f * 0.0f + C.llc_minus_origin[2]);
    o = add(ld3(C.origin), off);
    d = unit(unit(sub(dir, off)));                                 // camera.rs:64 + ray.rs:12
}

}  // namespace omd

namespace omd {

// Compressed-BVH2 traversal: one 64-B node read gives both child
// boxes; near child first, the far one pushed on a per-lane u16 stack that lives in
// LDS (stk[level * STRIDE]) — no scratch memory.  Leaves hold only Sphere/Cube
// records (everything else is in always2).  Box tests only choose which exact tests
// run (FMA allowed, conservative, see traced_sbvh); the acceptance keeps the
// brute-force tie rule, so the winner is bit-identical to hits.rs:274-285.
// The stack needs one entry per internal level (om_upload_world sizes it to the tree).
// The reference loop's answer for a non-finite ray, in closed form (hits.rs:274-285):
// every Sphere::hit accepts a NaN root (`disc < 0` and the range checks are all false
// for NaN, traced.rs:46-55) and so does InfinitePlane::hit (traced.rs:108), while Cube
// (is_solution false) and Barycentric (lambda checks false) reject.  The last accepted
// object in type order wins: the last plane, else the last sphere; t is NaN.
__device__ __forceinline__ int nonfinite_hit(const OmSceneDev& S, float& closest) {
    if (S.n_plane) { closest = __int_as_float(0x7FC00000); return (int)(S.off_plane + S.n_plane - 1u); }
    if (S.n_sph) { closest = __int_as_float(0x7FC00000); return (int)(S.n_sph - 1u); }
    return -1;
}

// Primary ray with a per-tile candidate list (om_tiles.h): always2, then
// every record the conservative lens-aware frustum of its 8x8 tile can reach — the
// brute-force loop of hits.rs:274-285 over a superset of the records it could accept.
// UNIFORM: every lane of the wave is in tile `tile` (the caller checked it; a bounce-0 wave is one
// 8x8 tile of one sample except where partial tiles meet), so the list and its records are read
// with scalar loads (uniform_load) instead of vector loads.
// tnear (UNIFORM): the lists are sorted by a lower bound of the t at which any primary ray can
// reach the record's box (om_tiles.cpp); once every lane's closest is below the next record's
// bound, that record and all later ones would be rejected (root >= bound > closest = tmax), so
// the wave stops (C1 +0.6%).  NaN closest keeps testing.  The candidates take sphere_root's
// division-free rejection (FASTREJ): coherent waves often reject an occluded candidate together.
template <bool UNIFORM = false, class Wk>
__device__ __forceinline__ int traced_tiles(const OmSceneDev& S, const uint32_t* toff, const uint16_t* tidx, uint32_t tile,
                                            F3 o, F3 d, float tmin, float& closest, Wk& w, const float* tnear = nullptr) {
    if (!isfinite(o.x + o.y + o.z + d.x + d.y + d.z)) return nonfinite_hit(S, closest);
    int best = -1;
    const float ix = inv_dir(d.x);
    const float iy = inv_dir(d.y);
    const float iz = inv_dir(d.z);
    const float nox = -o.x * ix, noy = -o.y * iy, noz = -o.z * iz;
    offer_always2(S, o, d, tmin, ix, iy, iz, nox, noy, noz, tmin * 0.5f - 1e-3f, closest, best, w);
    if constexpr (UNIFORM) {
        const uint32_t b = uniform_load(toff + tile), e = uniform_load(toff + tile + 1);
        const uint32_t* tw = (const uint32_t*)tidx;                 // u16 entries, read as the dword holding them
        auto rec_at = [&](uint32_t k) {
            const uint32_t pair = uniform_load(tw + (k >> 1));
            return (k & 1u) ? pair >> 16 : pair & 0xFFFFu;
        };
        uint32_t k = b;
        for (; k < e; ++k) {
            const uint32_t r = rec_at(k);
            if (tnear && __ballot(!(closest < uniform_load(tnear + r))) == 0) break;
            test_rec<true>(uniform_load(S.srecs + r), o, d, tmin, closest, best, w);
        }
    } else {
        const uint32_t e = toff[tile + 1];
        for (uint32_t k = toff[tile]; k < e; ++k) test_rec(S.srecs[tidx[k]], o, d, tmin, closest, best, w);
    }
    return best;
}

// HYB: only nodes [0, nl) are in `nodes` (the breadth-first prefix staged in LDS); the
// others are read from `gnodes` (global memory, through L2).
// CUNIT: bytes per unit of an internal node's code: sizeof(Node) when codes are node indices;
// 16 for the LDS copy at the padded 80-B stride, whose codes stage_scene pre-multiplies (a shift
// instead of the quarter-rate v_mul_lo_u32 of cur * 80: +0.7% on C1 and C4, r06).
// (Pop culling -- u32 entries carrying the pushed child's near distance, popped entries beyond
// the current closest dropped unread -- removed only 1.8% of the box tests on C1 and cost LDS
// occupancy on C3: DESIGN.md §8, r06.)
template <int DEPTH, int STRIDE, class Wk, bool HYB = false, class Node = OmBvh2Node, int CUNIT = (int)sizeof(Node)>
__device__ __forceinline__ int traced_bvh2(const OmSceneDev& S, const Node* nodes, const uint32_t* leaves,
                                           const OmAffineTest* recs, uint16_t* stk,
                                           F3 o, F3 d, float tmin, float& closest, Wk& w,
                                           const Node* gnodes = nullptr, uint32_t nl = 0) {
    if (!isfinite(o.x + o.y + o.z + d.x + d.y + d.z)) return nonfinite_hit(S, closest);
    int best = -1;
    const float ix = inv_dir(d.x);
    const float iy = inv_dir(d.y);
    const float iz = inv_dir(d.z);
    const float nox = -o.x * ix, noy = -o.y * iy, noz = -o.z * iz;
    const float t_lo = tmin * 0.5f - 1e-3f;
    offer_always2(S, o, d, tmin, ix, iy, iz, nox, noy, noz, t_lo, closest, best, w);
    // slab tests of node N's two child boxes: -> h0, h1 (hit), and whether child 1 is nearer
    auto slabs = [&](const Node& N, bool& h0, bool& h1, bool& swap) {
        w.add_pre(2);
        const float t_hi = closest * 1.0001f + 1e-3f;
        // half planes (OmBvh2NodeH): the (float) conversion folds into v_fma_mix_f32
        float x0 = __builtin_fmaf(b2p<0>(N), ix, nox), x1 = __builtin_fmaf(b2p<3>(N), ix, nox);
        float y0 = __builtin_fmaf(b2p<1>(N), iy, noy), y1 = __builtin_fmaf(b2p<4>(N), iy, noy);
        float z0 = __builtin_fmaf(b2p<2>(N), iz, noz), z1 = __builtin_fmaf(b2p<5>(N), iz, noz);
        const float n0 = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
        const float f0 = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
        x0 = __builtin_fmaf(b2p<6>(N), ix, nox); x1 = __builtin_fmaf(b2p<9>(N), ix, nox);
        y0 = __builtin_fmaf(b2p<7>(N), iy, noy); y1 = __builtin_fmaf(b2p<10>(N), iy, noy);
        z0 = __builtin_fmaf(b2p<8>(N), iz, noz); z1 = __builtin_fmaf(b2p<11>(N), iz, noz);
        const float n1 = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
        const float f1 = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
        h0 = !(n0 > f0); h1 = !(n1 > f1); swap = n1 < n0;
    };
    uint32_t cur = 0;                                   // 16-bit code: node index | OM_LEAF + leaf index
    int sp = 0;                                         // lane stack: one entry per internal level
    // next entry off the stack -> cur; false when the stack is empty
    auto pop = [&]() -> bool {
        if (sp == 0) return false;
        --sp;
        cur = stk[sp * STRIDE];
        return true;
    };
    // the leaf and node steps of one loop, each ending in `continue`: the structurizer turns
    // this shape into a node loop nested in the leaf loop (a lane descends until it reaches a
    // leaf, then the wave's leaves are tested) -- written as one flat if/else loop instead,
    // C1 ran 14% slower (r04)
    for (;;) {
        if (cur >= OM_LEAF) {                       // the single leaf site (16-bit codes: one compare, no and)
            test_leaf(recs, leaf_payload(S, cur, leaves), o, d, tmin, closest, best, w);
            if (!pop()) break;
            continue;
        }
        const Node N = (HYB && cur >= nl) ? gnodes[cur] : *(const Node*)((const char*)nodes + cur * (uint32_t)CUNIT);
        bool h0, h1, swap;
        slabs(N, h0, h1, swap);
        if (h0 && h1) {                             // near child next, far child pushed
            stk[sp * STRIDE] = (uint16_t)(swap ? N.c0 : N.c1);   // sp < depth: om_upload_world sizes the stack
            ++sp;
            cur = swap ? N.c1 : N.c0;
        } else if (h0 || h1) {
            cur = h0 ? N.c0 : N.c1;
        } else {
            if (!pop()) break;
            continue;
        }
    }
    return best;
}


// 4-wide BVH traversal: one 112-B node read gives four slab tests; the
// hit children are ordered near-first by a 5-compare sorting network, the nearest is
// visited next and the others go on the lane's LDS stack with three unconditional u16
// writes (no divergent push branches; the stack holds 3 spare entries for them).
// HYB (half nodes, trees read through L2): nodes [0, nl) are the breadth-first prefix in LDS.
template <int STRIDE, class Wk, bool HYB = false, class Node = OmBvh4Node>
__device__ __forceinline__ int traced_bvh4(const OmSceneDev& S, const Node* nodes, const uint32_t* leaves,
                                           const OmAffineTest* recs, uint16_t* stk,
                                           F3 o, F3 d, float tmin, float& closest, Wk& w,
                                           const Node* gnodes = nullptr, uint32_t nl = 0) {
    if (!isfinite(o.x + o.y + o.z + d.x + d.y + d.z)) return nonfinite_hit(S, closest);
    int best = -1;
    const float ix = inv_dir(d.x);
    const float iy = inv_dir(d.y);
    const float iz = inv_dir(d.z);
    const float nox = -o.x * ix, noy = -o.y * iy, noz = -o.z * iz;
    const float t_lo = tmin * 0.5f - 1e-3f;
    offer_always2(S, o, d, tmin, ix, iy, iz, nox, noy, noz, t_lo, closest, best, w);
    uint32_t cur = 0;
    int sp = 0;
    for (;;) {
        if (cur >= OM_LEAF) {
            test_leaf(recs, leaf_payload(S, cur, leaves), o, d, tmin, closest, best, w);
            if (sp == 0) break;
            --sp;
            cur = stk[sp * STRIDE];
            continue;
        }
        const Node N = (HYB && cur >= nl) ? gnodes[cur] : nodes[cur];
        w.add_pre(4);
        const float t_hi = closest * 1.0001f + 1e-3f;
        float key[4];
        uint32_t code[4];
        int n = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float x0 = __builtin_fmaf(b4p<0>(N, k), ix, nox), x1 = __builtin_fmaf(b4p<3>(N, k), ix, nox);
            const float y0 = __builtin_fmaf(b4p<1>(N, k), iy, noy), y1 = __builtin_fmaf(b4p<4>(N, k), iy, noy);
            const float z0 = __builtin_fmaf(b4p<2>(N, k), iz, noz), z1 = __builtin_fmaf(b4p<5>(N, k), iz, noz);
            const float tn = slab_near(x0, x1, y0, y1, z0, z1, t_lo);
            const float tf = slab_far(x0, x1, y0, y1, z0, z1, t_hi);
            const uint32_t c = N.child[k];
            const bool h = !(tn > tf) && c != OM_EMPTY;
            // a NaN slab counts as a hit but sorts by t_lo: the network needs ordered keys (a NaN
            // key compares false both ways and could leave a missed child ahead of the hit one)
            key[k] = h ? fmaxf(tn, t_lo) : INFINITY;
            code[k] = c;
            n += h ? 1 : 0;
        }
        if (n == 0) {
            if (sp == 0) break;
            --sp;
            cur = stk[sp * STRIDE];
            continue;
        }
#define OM_CAS(a, b)                                                                          \
        {                                                                                     \
            const bool sw = key[b] < key[a];                                                  \
            const float ka = key[a], kb = key[b];                                             \
            const uint32_t ca = code[a], cb = code[b];                                        \
            key[a] = sw ? kb : ka; key[b] = sw ? ka : kb;                                     \
            code[a] = sw ? cb : ca; code[b] = sw ? ca : cb;                                   \
        }
        OM_CAS(0, 1) OM_CAS(2, 3) OM_CAS(0, 2) OM_CAS(1, 3) OM_CAS(1, 2)
#undef OM_CAS
        // stack, bottom -> top: the n-1 far children, farthest first (nearest popped first)
        const uint32_t w0 = n == 4 ? code[3] : (n == 3 ? code[2] : code[1]);
        const uint32_t w1 = n == 4 ? code[2] : code[1];
        stk[sp * STRIDE] = (uint16_t)w0;
        stk[(sp + 1) * STRIDE] = (uint16_t)w1;
        stk[(sp + 2) * STRIDE] = (uint16_t)code[1];
        sp += n - 1;
        cur = code[0];
    }
    return best;
}

}  // namespace omd
