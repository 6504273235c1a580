// om_render.hip — the hot path on MI355X (gfx950): per-pixel ray_color
// integrator (render_thread.rs:105-202) with closest-hit over the frozen world
// (hits.rs:270-365), as one persistent-path megakernel.
//
// Execution model: one lane owns one pixel for the whole call
// and walks that pixel's samples in order (so Stats::add sees samples in the
// reference's order, bit for bit).  The bounce recursion is flattened into a
// segment loop with path REGENERATION: when a lane's path ends, the same loop
// iteration starts that pixel's next sample, so every active lane runs the
// closest-hit query of some live ray each iteration — the SIMD-utilisation
// benefit of wavefront compaction without the HBM ray queues.  A wave owns an
// 8x8 pixel tile for ray coherence.  Scene records are read at wave-uniform
// addresses (scalar loads) and stay L2/LDS resident.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"
#include "om_device.h"
#include "om_layout.h"
#include "om_world.h"

using namespace omd;

static_assert(sizeof(om_pixel_stats) == 40, "om_pixel_stats layout");
static_assert(sizeof(OmAffineTest) == 64 && sizeof(OmBvhNode) == 32, "layout");

namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// closest hit over the traced primitives
// ---------------------------------------------------------------------------
enum { MODE_BRUTE = 1, MODE_CULLED = 2, MODE_BVH = 3 };

struct Work { uint32_t prim, pre, march; };

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
template <bool CULL>
__device__ __forceinline__ int traced_brute(const OmSceneDev& S, F3 o, F3 d, float tmin, float& closest, Work& w) {
    int best = -1;
    float t;
    for (uint32_t i = 0; i < S.n_sph; ++i) {
        if (CULL) {
            const OmBound B = S.sph_bound[i];
            const float ocx = o.x - B.c[0], ocy = o.y - B.c[1], ocz = o.z - B.c[2];
            const float b = ocx * d.x + ocy * d.y + ocz * d.z;
            const float px = ocx - b * d.x, py = ocy - b * d.y, pz = ocz - b * d.z;
            const float q = px * px + py * py + pz * pz;
            w.pre++;
            // every comparison is false for NaN -> the exact test decides
            if (q > B.r * B.r || -b + B.r < tmin || -b - B.r > closest) continue;
        }
        w.prim++;
        if (sphere_root(S.sph_test[i], o, d, tmin, closest, t)) { closest = t; best = (int)i; }
    }
    for (uint32_t i = 0; i < S.n_cube; ++i) {
        int ax; w.prim++;
        if (cube_root(S.cube_test[i], o, d, tmin, closest, t, ax)) { closest = t; best = (int)(S.off_cube + i); }
    }
    float ndd;
    for (uint32_t i = 0; i < S.n_tri; ++i) {
        w.prim++;
        if (bary_root<true>(S.tri[i], o, d, tmin, closest, t, ndd)) { closest = t; best = (int)(S.off_tri + i); }
    }
    for (uint32_t i = 0; i < S.n_plane; ++i) {
        w.prim++;
        if (plane_root(S.plane[i], o, d, tmin, closest, t, ndd)) { closest = t; best = (int)(S.off_plane + i); }
    }
    for (uint32_t i = 0; i < S.n_para; ++i) {
        w.prim++;
        if (bary_root<false>(S.para[i], o, d, tmin, closest, t, ndd)) { closest = t; best = (int)(S.off_para + i); }
    }
    return best;
}

// BVH traversal with the brute-force tie rule: the reference keeps the smallest
// accepted root and, on equal roots, the later object in type order.
__device__ __forceinline__ void offer(const OmSceneDev& S, uint32_t gi, F3 o, F3 d, float tmin, float& closest, int& best, Work& w) {
    float t;
    w.prim++;
    if (test_prim(S, gi, o, d, tmin, closest, t)) {
        if (t < closest || (int)gi > best) { closest = t; best = (int)gi; }
    }
}

__device__ __forceinline__ int traced_bvh(const OmSceneDev& S, F3 o, F3 d, float tmin, float& closest, Work& w) {
    // Non-finite rays take the reference loop (NaN roots are accepted there).
    if (!isfinite(o.x + o.y + o.z + d.x + d.y + d.z)) return traced_brute<false>(S, o, d, tmin, closest, w);
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
            w.pre += 2;
            // Slab tests on inflated boxes, (lo - o) * (1/d): a zero direction component
            // gives +-inf (correct containment) or NaN (dropped by fminf/fmaxf = unconstrained).
            const float t_hi = closest * 1.0001f + 1e-3f;
            float x0 = (L.lo[0] - o.x) * ix, x1 = (L.hi[0] - o.x) * ix;
            float y0 = (L.lo[1] - o.y) * iy, y1 = (L.hi[1] - o.y) * iy;
            float z0 = (L.lo[2] - o.z) * iz, z1 = (L.hi[2] - o.z) * iz;
            const float ln = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), t_lo));
            const float lf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t_hi));
            x0 = (R.lo[0] - o.x) * ix; x1 = (R.hi[0] - o.x) * ix;
            y0 = (R.lo[1] - o.y) * iy; y1 = (R.hi[1] - o.y) * iy;
            z0 = (R.lo[2] - o.z) * iz; z1 = (R.hi[2] - o.z) * iz;
            const float rn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), t_lo));
            const float rf = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fminf(fmaxf(z0, z1), t_hi));
            const bool hl = ln <= lf, hr = rn <= rf;
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

// unstuck (hits.rs:336-365) + sphere-tracing loop (hits.rs:287-333).
// Returns the marched winner's global index or -1; `t` receives the hit t.
__device__ __forceinline__ int march(const OmSceneDev& S, F3 o, F3 d, float tmin, float tmax, float closest,
                                     uint32_t steps, float& t_hit, Work& w) {
    const float HIT = 0.001f;
    // nearest marched object at r.at(tmin), strict '<' (first minimum wins)
    F3 p = at(o, d, tmin);
    float dist = INFINITY; int kind = -1; uint32_t idx = 0;
    for (uint32_t i = 0; i < S.n_msph; ++i) { const float v = fabsf(msphere_sdf(S.msph[i], p)); if (v < dist) { dist = v; kind = 0; idx = i; } }
    for (uint32_t i = 0; i < S.n_mbox; ++i) { const float v = fabsf(mbox_sdf(S.mbox[i], p)); if (v < dist) { dist = v; kind = 1; idx = i; } }
    for (uint32_t i = 0; i < S.n_mtor; ++i) { const float v = fabsf(mtorus_sdf(S.mtor[i], p)); if (v < dist) { dist = v; kind = 2; idx = i; } }
    if (kind < 0) return -1;                                                   // hits.rs:359
    float t = tmin;
    float aux = dist;
    uint32_t guard = 0;
    while (aux < HIT && guard++ < (1u << 22)) {                                // hits.rs:360-363 (+ safety cap)
        t += HIT / 2.0f;
        const F3 q = at(o, d, t);
        aux = kind == 0 ? fabsf(msphere_sdf(S.msph[idx], q)) : kind == 1 ? fabsf(mbox_sdf(S.mbox[idx], q)) : fabsf(mtorus_sdf(S.mtor[idx], q));
    }
    uint32_t iters = steps;
    while (t < tmax && t < closest && iters > 0) {                            // hits.rs:294
        iters -= 1;
        w.march++;
        p = at(o, d, t);
        float best = INFINITY; int bk = -1; uint32_t bi = 0;
        for (uint32_t i = 0; i < S.n_msph; ++i) { const float v = fabsf(msphere_sdf(S.msph[i], p)); if (v < best) { best = v; bk = 0; bi = i; } }
        for (uint32_t i = 0; i < S.n_mbox; ++i) { const float v = fabsf(mbox_sdf(S.mbox[i], p)); if (v < best) { best = v; bk = 1; bi = i; } }
        for (uint32_t i = 0; i < S.n_mtor; ++i) { const float v = fabsf(mtorus_sdf(S.mtor[i], p)); if (v < best) { best = v; bk = 2; bi = i; } }
        if (bk < 0) return -1;                                                 // hits.rs:323
        if (best < HIT) {                                                      // hits.rs:325-327
            t_hit = t;
            return (int)(bk == 0 ? S.off_msph + bi : bk == 1 ? S.off_mbox + bi : S.off_mtor + bi);
        }
        t += best;                                                             // hits.rs:330
    }
    return -1;
}

// Build the HitRecord of the winner (point, normal) — the winner's own exact
// test re-run with tmax = its root reproduces the same root bit for bit.
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
    if (g < S.off_mbox) normal = msphere_normal(S.msph[g - S.off_msph], point);
    else if (g < S.off_mtor) normal = mbox_normal(S.mbox[g - S.off_mbox], point);
    else normal = mtorus_normal(S.mtor[g - S.off_mtor], point);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void render_kernel(OmSceneDev S, OmCamDev C, OmParamsDev P,
                                                        const float2* __restrict__ jitter,
                                                        om_pixel_stats* __restrict__ stats,
                                                        const uint32_t* __restrict__ pixel_list,
                                                        unsigned long long* __restrict__ counters) {
    const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
    uint32_t pixel, slot;
    bool valid;
    if (pixel_list) {
        valid = tid < P.n_pixels;
        pixel = valid ? pixel_list[tid] : 0u;
        slot = tid;
    } else {
        const uint32_t wave = tid >> 6, lane = tid & 63u;
        const uint32_t tx = wave % P.tiles_x, ty = wave / P.tiles_x;
        const uint32_t px = tx * 8u + (lane & 7u), py = ty * 8u + (lane >> 3);
        valid = px < P.width && py < P.height;
        pixel = py * P.width + px;
        slot = pixel;
    }
    PixelState st;
    if (valid) {
        const om_pixel_stats in = stats[slot];
        st.bloom = in.bloom; st.sx = in.sum[0]; st.sy = in.sum[1]; st.sz = in.sum[2]; st.n = in.n;
        st.avg_depth = in.avg_depth; st.bad = in.bad_avgs;
        st.rgbf = (uint32_t)in.color[0] | ((uint32_t)in.color[1] << 8) | ((uint32_t)in.color[2] << 16) | ((uint32_t)in.flags << 24);
    } else {
        st.bloom = 0; st.sx = st.sy = st.sz = 0.0f; st.n = 0; st.avg_depth = 0.0f; st.bad = 0; st.rgbf = 0;
    }
    const uint32_t line = valid ? pixel / P.width : 0u;
    const float j_f = (float)line, i_f = (float)(pixel - P.width * line);
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    const bool has_marched = (S.n_msph + S.n_mbox + S.n_mtor) != 0u;

    uint32_t todo = valid ? P.sample_count : 0u;
    bool live = false;
    F3 o = f3(0, 0, 0), d = f3(0, 0, 0), cur = f3(1, 1, 1);
    Rng g; g.s = 0;
    uint32_t seg = 0, first_id = 0;
    float depthf = 0.0f;
    Work w = {0, 0, 0};
    uint32_t n_samples = 0, n_segments = 0, credited = 0;

    for (;;) {
        if (!live && todo > 0u) {
            if ((P.adaptive && (st.rgbf & 0x01000000u)) || st.n >= P.spp_total) {
                todo = 0u;
            } else {
                // render_thread.rs:183-192 + Camera::get_ray camera.rs:60-65
                const uint32_t s = st.n;
                g = path_rng(P.skey, pixel, s);
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
                cur = f3(1.0f, 1.0f, 1.0f);
                seg = 0; live = true; todo--;
            }
        }
        if (__ballot(live) == 0ull) break;
        if (!live) continue;

        // ---- one segment: handle_hit(world.hit(ray)) render_thread.rs:105-126
        n_segments++;
        float closest = P.tmax;
        int best;
        if (MODE == MODE_BVH) best = traced_bvh(S, o, d, P.tmin, closest, w);
        else best = traced_brute<MODE == MODE_CULLED>(S, o, d, P.tmin, closest, w);
        if (has_marched) {
            float tm;
            const int mg = march(S, o, d, P.tmin, P.tmax, closest, P.march_steps, tm, w);
            if (mg >= 0) { best = mg; closest = tm; }
        }
        float seg_depth; uint32_t seg_id;
        if (best >= 0) {
            F3 point, normal;
            finalize(S, best, o, d, P.tmin, closest, point, normal);
            F3 nd, att;
            scatter(S.mats[best], d, normal, g, nd, att);
            cur = mul(cur, att);
            o = point; d = unit(nd);
            seg_depth = closest; seg_id = (uint32_t)best + 1u;
        } else {
            const float t = 0.5f * (d.y + 1.0f);                               // render_thread.rs:118-120
            cur = mul(cur, f3((1.0f - t) + 0.5f * t, (1.0f - t) + 0.7f * t, (1.0f - t) + 1.0f * t));
            seg_depth = INFINITY; seg_id = 0u;
        }
        bool finished = false;
        F3 result = cur;
        float rdepth = 0.0f; uint32_t rid = 0;
        if (seg == 0u) {
            depthf = seg_depth; first_id = seg_id;
            if (isinf(seg_depth)) { finished = true; rdepth = INFINITY; rid = 0u; }     // :133-135
        } else if (isinf(seg_depth)) {
            finished = true; rdepth = depthf; rid = first_id;                       // :138-140
        }
        if (!finished && seg + 1u >= depth_cap) {                              // :142  -Color::ZERO
            finished = true; result = f3(-0.0f, -0.0f, -0.0f); rdepth = depthf; rid = first_id;
        }
        seg++;
        if (finished) {
            const bool done = stats_add(st, result, rdepth, S.bloom[rid]);
            n_samples++;
            credited += ((done && P.adaptive) ? (P.spp_total - st.n) : 0u) + 1u; // :196-198
            live = false;
        }
    }

    if (valid) {
        om_pixel_stats out;
        out.bloom = st.bloom; out.sum[0] = st.sx; out.sum[1] = st.sy; out.sum[2] = st.sz; out.n = st.n;
        out.avg_depth = st.avg_depth; out.bad_avgs = st.bad;
        out.color[0] = (uint8_t)(st.rgbf & 0xFFu); out.color[1] = (uint8_t)((st.rgbf >> 8) & 0xFFu);
        out.color[2] = (uint8_t)((st.rgbf >> 16) & 0xFFu); out.flags = (uint8_t)(st.rgbf >> 24); out.reserved = 0u;
        stats[slot] = out;
    }
    if (counters) {
        const uint32_t c0 = wave_sum(n_samples), c1 = wave_sum(n_segments), c2 = wave_sum(w.prim), c3 = wave_sum(w.pre),
                       c4 = wave_sum(w.march), c5 = wave_sum(credited);
        if ((threadIdx.x & 63u) == 0u) {
            atomicAdd(&counters[OMC_SAMPLES], (unsigned long long)c0);
            atomicAdd(&counters[OMC_SEGMENTS], (unsigned long long)c1);
            atomicAdd(&counters[OMC_PRIM_TESTS], (unsigned long long)c2);
            atomicAdd(&counters[OMC_PRE_TESTS], (unsigned long long)c3);
            atomicAdd(&counters[OMC_MARCH], (unsigned long long)c4);
            atomicAdd(&counters[OMC_CREDITED], (unsigned long long)c5);
        }
    }
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
thread_local std::string g_err;

struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    void release() { if (p) (void)hipFree(p); p = nullptr; n = 0; }
};

}  // namespace

struct om_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    std::vector<DevBuf> scene_bufs;
    OmSceneDev scene{};
    bool have_world = false;
    int kernel = OM_KERNEL_AUTO;
    DevBuf counters, jitter, stats, pixels;
    uint64_t jitter_seed = 0; uint32_t jitter_spp = 0;
    hipStream_t last_stream = nullptr;
    ~om_ctx() {
        for (auto& b : scene_bufs) b.release();
        counters.release(); jitter.release(); stats.release(); pixels.release();
        if (stream) (void)hipStreamDestroy(stream);
    }
};

namespace {

om_status set_err(om_ctx* c, om_status code, const std::string& msg) {
    g_err = msg;
    if (c) c->err = msg;
    return code;
}
#define OM_HIP(ctx, call)                                                                       \
    do {                                                                                        \
        hipError_t e_ = (call);                                                                 \
        if (e_ != hipSuccess) return set_err(ctx, OM_ERR_DEVICE, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

template <class T>
om_status upload(om_ctx* c, const std::vector<T>& v, const T** out) {
    *out = nullptr;
    if (v.empty()) return OM_OK;
    DevBuf b;
    b.n = v.size() * sizeof(T);
    OM_HIP(c, hipMalloc(&b.p, b.n));
    c->scene_bufs.push_back(b);
    OM_HIP(c, hipMemcpyAsync(b.p, v.data(), b.n, hipMemcpyHostToDevice, c->stream));
    *out = (const T*)b.p;
    return OM_OK;
}

om_status ensure(om_ctx* c, DevBuf& b, size_t n) {
    if (b.n >= n) return OM_OK;
    b.release();
    OM_HIP(c, hipMalloc(&b.p, n));
    b.n = n;
    return OM_OK;
}

// jitter table render_thread.rs:164-174: ((s/2)&1, s&1) shuffled once (om-rng v1 Fisher-Yates)
om_status prepare_jitter(om_ctx* c, uint64_t seed, uint32_t spp) {
    if (c->jitter.p && c->jitter_seed == seed && c->jitter_spp == spp) return OM_OK;
    std::vector<float> jt(2 * (size_t)spp);
    for (uint32_t s = 0; s < spp; ++s) { jt[2 * s] = (float)((s / 2) & 1u); jt[2 * s + 1] = (float)(s & 1u); }
    auto mix = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    uint64_t st = mix(seed ^ 0x4A177E5B0C1D2E3FULL);
    for (uint32_t i = spp; i-- > 1;) {
        st += 0x9E3779B97F4A7C15ULL;
        const uint32_t j = (uint32_t)((mix(st) >> 32) % (uint64_t)(i + 1));
        std::swap(jt[2 * i], jt[2 * j]);
        std::swap(jt[2 * i + 1], jt[2 * j + 1]);
    }
    om_status s = ensure(c, c->jitter, jt.size() * sizeof(float) + 16);
    if (s) return s;
    OM_HIP(c, hipMemcpyAsync(c->jitter.p, jt.data(), jt.size() * sizeof(float), hipMemcpyHostToDevice, c->stream));
    OM_HIP(c, hipStreamSynchronize(c->stream));  // jt is a host temporary
    c->jitter_seed = seed; c->jitter_spp = spp;
    return OM_OK;
}

om_status validate(om_ctx* c, const om_camera* cam, const om_render_params* p) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (!cam || !p) return set_err(c, OM_ERR_INVALID, "null camera/params");
    if (!c->have_world) return set_err(c, OM_ERR_STATE, "om_upload_world must precede rendering");
    if (p->width < 2 || p->height < 2) return set_err(c, OM_ERR_INVALID, "width/height must be >= 2");
    if ((uint64_t)p->width * p->height > (1ull << 31)) return set_err(c, OM_ERR_INVALID, "image too large");
    if (p->spp_total == 0) return set_err(c, OM_ERR_INVALID, "spp_total must be > 0");
    return OM_OK;
}

om_status launch(om_ctx* c, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_stats,
                 const uint32_t* dev_pixels, uint32_t n_pixels, hipStream_t stream) {
    om_status s = prepare_jitter(c, p->seed, p->spp_total);
    if (s) return s;
    if (!c->counters.p) {
        s = ensure(c, c->counters, OMC_N * sizeof(unsigned long long));
        if (s) return s;
        OM_HIP(c, hipMemsetAsync(c->counters.p, 0, OMC_N * sizeof(unsigned long long), stream));
    }
    c->last_stream = stream;
    OmCamDev C;
    for (int i = 0; i < 3; ++i) {
        C.origin[i] = cam->origin[i]; C.horizontal[i] = cam->horizontal[i]; C.vertical[i] = cam->vertical[i];
        C.llc_minus_origin[i] = cam->lower_left_corner[i] - cam->origin[i];          // camera.rs:72
        C.u[i] = cam->u_of_plane[i]; C.v[i] = cam->v_of_plane[i];
    }
    C.lens_radius = cam->lens_radius;
    OmParamsDev P;
    P.width = p->width; P.height = p->height; P.spp_total = p->spp_total; P.sample_count = p->sample_count;
    P.max_depth = p->max_depth; P.march_steps = p->march_steps; P.adaptive = p->adaptive ? 1u : 0u;
    P.tmin = p->tmin; P.tmax = p->tmax;
    P.wf_m1 = (float)p->width - 1.0f; P.hf_m1 = (float)p->height - 1.0f;             // render_thread.rs:190-191
    const uint64_t sk = p->seed + 0x632BE59BD9B4E019ULL;
    uint64_t z = sk;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    P.skey = z ^ (z >> 31);
    P.tiles_x = (p->width + 7u) / 8u;
    uint64_t threads;
    if (dev_pixels) {
        P.n_pixels = n_pixels;
        threads = n_pixels;
    } else {
        const uint64_t tiles = (uint64_t)P.tiles_x * ((p->height + 7u) / 8u);
        P.n_pixels = p->width * p->height;
        threads = tiles * 64u;
    }
    if (threads == 0) return OM_OK;
    const uint32_t blocks = (uint32_t)((threads + kBlock - 1) / kBlock);
    int mode = c->kernel;
    if (mode == OM_KERNEL_AUTO) mode = OM_KERNEL_BVH;
    const float2* jt = (const float2*)c->jitter.p;
    unsigned long long* ctr = (unsigned long long*)c->counters.p;
    if (mode == OM_KERNEL_BRUTE)
        hipLaunchKernelGGL(render_kernel<MODE_BRUTE>, dim3(blocks), dim3(kBlock), 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    else if (mode == OM_KERNEL_CULLED)
        hipLaunchKernelGGL(render_kernel<MODE_CULLED>, dim3(blocks), dim3(kBlock), 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    else
        hipLaunchKernelGGL(render_kernel<MODE_BVH>, dim3(blocks), dim3(kBlock), 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    OM_HIP(c, hipGetLastError());
    return OM_OK;
}

}  // namespace

extern "C" {

const char* om_world_last_error_internal(void);

om_status om_create(int32_t device, om_ctx** out) {
    if (!out) return set_err(nullptr, OM_ERR_INVALID, "om_create: null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return set_err(nullptr, OM_ERR_DEVICE, "om_create: no HIP device available");
    if (device < 0 || device >= n) return set_err(nullptr, OM_ERR_INVALID, "om_create: device index out of range");
    om_ctx* c = new (std::nothrow) om_ctx();
    if (!c) return set_err(nullptr, OM_ERR_NOMEM, "om_create: out of memory");
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_err(nullptr, OM_ERR_DEVICE, "om_create: stream creation failed");
    }
    *out = c;
    return OM_OK;
}

void om_destroy(om_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    delete c;
}

const char* om_last_error(const om_ctx* c) {
    if (c) return c->err.c_str();
    if (!g_err.empty()) return g_err.c_str();
    return om_world_last_error_internal();
}

om_status om_upload_world(om_ctx* c, const om_world* w) {
    if (!c || !w) return set_err(c, OM_ERR_INVALID, "om_upload_world: null pointer");
    OM_HIP(c, hipSetDevice(c->device));
    OM_HIP(c, hipStreamSynchronize(c->stream));
    for (auto& b : c->scene_bufs) b.release();
    c->scene_bufs.clear();
    c->have_world = false;
    om::FrozenWorld fw;
    w->freeze(fw);
    OmSceneDev& S = c->scene;
    S = OmSceneDev{};
    om_status s = OM_OK;
#define UP(vec, field) if ((s = upload(c, fw.vec, &S.field)) != OM_OK) return s
    UP(sph_test, sph_test); UP(sph_hit, sph_hit); UP(sph_bound, sph_bound);
    UP(cube_test, cube_test); UP(cube_hit, cube_hit); UP(cube_bound, cube_bound);
    UP(tri, tri); UP(plane, plane); UP(para, para);
    UP(msph, msph); UP(mbox, mbox); UP(mtor, mtor);
    UP(mats, mats); UP(bloom, bloom); UP(bvh, bvh); UP(bvh_prims, bvh_prims); UP(always, always);
#undef UP
    S.n_sph = fw.counts[0]; S.n_cube = fw.counts[1]; S.n_tri = fw.counts[2]; S.n_plane = fw.counts[3]; S.n_para = fw.counts[4];
    S.n_msph = fw.counts[5]; S.n_mbox = fw.counts[6]; S.n_mtor = fw.counts[7];
    S.off_cube = fw.offsets[1]; S.off_tri = fw.offsets[2]; S.off_plane = fw.offsets[3]; S.off_para = fw.offsets[4];
    S.off_msph = fw.offsets[5]; S.off_mbox = fw.offsets[6]; S.off_mtor = fw.offsets[7]; S.n_total = fw.offsets[8];
    S.n_bvh_nodes = (uint32_t)fw.bvh.size();
    S.n_always = (uint32_t)fw.always.size();
    OM_HIP(c, hipStreamSynchronize(c->stream));
    c->have_world = true;
    return OM_OK;
}

om_status om_set_kernel(om_ctx* c, int32_t k) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (k < OM_KERNEL_AUTO || k > OM_KERNEL_BVH) return set_err(c, OM_ERR_INVALID, "om_set_kernel: unknown kernel");
    c->kernel = k;
    return OM_OK;
}

om_status om_render_device(om_ctx* c, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_stats, void* stream) {
    om_status s = validate(c, cam, p);
    if (s) return s;
    if (!dev_stats) return set_err(c, OM_ERR_INVALID, "null dev_stats");
    OM_HIP(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    return launch(c, cam, p, dev_stats, nullptr, 0, st);
}

om_status om_render_device_pixels(om_ctx* c, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_stats,
                                  const uint32_t* dev_pixels, uint32_t n_pixels, void* stream) {
    om_status s = validate(c, cam, p);
    if (s) return s;
    if (!dev_stats || (!dev_pixels && n_pixels)) return set_err(c, OM_ERR_INVALID, "null dev_stats/dev_pixels");
    OM_HIP(c, hipSetDevice(c->device));
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    if (n_pixels == 0) return OM_OK;
    return launch(c, cam, p, dev_stats, dev_pixels, n_pixels, st);
}

om_status om_render(om_ctx* c, const om_camera* cam, const om_render_params* p, om_pixel_stats* stats, om_counters* counters) {
    om_status s = validate(c, cam, p);
    if (s) return s;
    if (!stats) return set_err(c, OM_ERR_INVALID, "null stats");
    OM_HIP(c, hipSetDevice(c->device));
    const size_t bytes = (size_t)p->width * p->height * sizeof(om_pixel_stats);
    if ((s = ensure(c, c->stats, bytes)) != OM_OK) return s;
    OM_HIP(c, hipMemcpyAsync(c->stats.p, stats, bytes, hipMemcpyHostToDevice, c->stream));
    if ((s = om_reset_counters(c, c->stream)) != OM_OK) return s;
    if ((s = launch(c, cam, p, (om_pixel_stats*)c->stats.p, nullptr, 0, c->stream)) != OM_OK) return s;
    OM_HIP(c, hipMemcpyAsync(stats, c->stats.p, bytes, hipMemcpyDeviceToHost, c->stream));
    OM_HIP(c, hipStreamSynchronize(c->stream));
    if (counters) return om_get_counters(c, counters);
    return OM_OK;
}

om_status om_get_counters(om_ctx* c, om_counters* out) {
    if (!c || !out) return set_err(c, OM_ERR_INVALID, "null pointer");
    std::memset(out, 0, sizeof(*out));
    if (!c->counters.p) return OM_OK;
    OM_HIP(c, hipSetDevice(c->device));
    unsigned long long h[OMC_N];
    OM_HIP(c, hipStreamSynchronize(c->stream));
    if (c->last_stream && c->last_stream != c->stream) OM_HIP(c, hipStreamSynchronize(c->last_stream));
    OM_HIP(c, hipMemcpy(h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost));
    out->samples = h[OMC_SAMPLES]; out->segments = h[OMC_SEGMENTS]; out->prim_tests = h[OMC_PRIM_TESTS];
    out->pre_tests = h[OMC_PRE_TESTS]; out->march_steps = h[OMC_MARCH]; out->credited = h[OMC_CREDITED];
    return OM_OK;
}

om_status om_reset_counters(om_ctx* c, void* stream) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    OM_HIP(c, hipSetDevice(c->device));
    om_status s = ensure(c, c->counters, OMC_N * sizeof(unsigned long long));
    if (s) return s;
    OM_HIP(c, hipMemsetAsync(c->counters.p, 0, OMC_N * sizeof(unsigned long long), stream ? (hipStream_t)stream : c->stream));
    return OM_OK;
}

}  // extern "C"
