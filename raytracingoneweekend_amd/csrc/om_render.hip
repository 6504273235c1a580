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

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"
#include "om_device.h"
#include "om_layout.h"
#include "om_display.h"
#include "om_tiles.h"
#include "om_wavefront.h"
#include "om_world.h"
#include "om_internal.h"

using namespace omd;

static_assert(sizeof(om_pixel_stats) == 40, "om_pixel_stats layout");
static_assert(sizeof(OmAffineTest) == 64 && sizeof(OmBvhNode) == 32, "layout");

namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// closest hit over the traced primitives
// ---------------------------------------------------------------------------
enum { MODE_BRUTE = 1, MODE_CULLED = 2, MODE_BVH = 3, MODE_SBVH_LDS = 4, MODE_SBVH_GLOBAL = 5, MODE_BVH2 = 6 };
constexpr int kStack2 = 24;                    // BVH2 lane-stack bound (om_upload_world checks the depth)
constexpr int kBlockLds = 512;
constexpr uint32_t kLdsBudget = 96u * 1024u;   // staged scene per workgroup (160 KiB per CU)

}  // namespace

#include "om_trace.h"

namespace {

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

extern __shared__ __attribute__((aligned(16))) uint4 om_lds[];

// MARCH is a compile-time split (as in the wavefront): traced-only scenes do not carry
// the sphere-tracing code's registers.
template <int MODE, int BLOCK, bool COUNT, bool MARCH>
__global__ __launch_bounds__(BLOCK, (BLOCK >= 512 ? 4 : 1)) void render_kernel(OmSceneDev S, OmCamDev C, OmParamsDev P,
                                                       const float2* __restrict__ jitter,
                                                       om_pixel_stats* __restrict__ stats,
                                                       const uint32_t* __restrict__ pixel_list,
                                                       unsigned long long* __restrict__ counters) {
    if (MODE == MODE_SBVH_LDS) {
        // stage the stackless BVH + its records once per workgroup (uint4 chunks)
        const uint32_t nn = S.n_snodes * 2u, nr = S.n_srecs * 4u;
        const uint4* sn = (const uint4*)S.snodes;
        const uint4* sr = (const uint4*)S.srecs;
        for (uint32_t i = threadIdx.x; i < nn; i += BLOCK) om_lds[i] = sn[i];
        for (uint32_t i = threadIdx.x; i < nr; i += BLOCK) om_lds[nn + i] = sr[i];
        __syncthreads();
    }
    const OmSkipNode* lds_nodes = (const OmSkipNode*)om_lds;
    const OmAffineTest* lds_recs = (const OmAffineTest*)(om_lds + S.n_snodes * 2u);
    // BVH2: [lane stack][nodes][leaf table] in LDS (nodes through L2 when they exceed the budget)
    uint16_t* b2_stk = (uint16_t*)om_lds + threadIdx.x;
    const OmBvh2Node* b2_nodes = S.b2nodes;
    const uint32_t* b2_leaves = S.b2leaves;
    if (MODE == MODE_BVH2 && S.b2_lds_bytes) {
        uint4* dst = om_lds + (BLOCK * S.b2_stack * 2u) / 16u;
        const uint32_t nn = S.n_b2nodes * (uint32_t)(sizeof(OmBvh2Node) / 16u);
        const uint4* sn = (const uint4*)S.b2nodes;
        for (uint32_t i = threadIdx.x; i < nn; i += BLOCK) dst[i] = sn[i];
        uint32_t* ldst = (uint32_t*)(dst + nn);
        for (uint32_t i = threadIdx.x; i < S.n_b2leaves; i += BLOCK) ldst[i] = S.b2leaves[i];
        __syncthreads();
        b2_nodes = (const OmBvh2Node*)dst;
        b2_leaves = ldst;
    }
    const uint32_t tid = blockIdx.x * BLOCK + threadIdx.x;
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

    uint32_t todo = valid ? P.sample_count : 0u;
    bool live = false;
    F3 o = f3(0, 0, 0), d = f3(0, 0, 0), cur = f3(1, 1, 1);
    Rng g; g.s = 0; g.k = 0;
    uint32_t seg = 0, first_id = 0;
    float depthf = 0.0f;
    WorkT<COUNT> w;
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
        if (COUNT) n_segments++;
        float closest = P.tmax;
        int best;
        if (MODE == MODE_SBVH_LDS) best = traced_sbvh(S, lds_nodes, lds_recs, o, d, P.tmin, closest, w);
        else if (MODE == MODE_SBVH_GLOBAL) best = traced_sbvh(S, S.snodes, S.srecs, o, d, P.tmin, closest, w);
        else if (MODE == MODE_BVH) best = traced_bvh(S, o, d, P.tmin, closest, w);
        else if (MODE == MODE_BVH2) best = traced_bvh2<kStack2, BLOCK>(S, b2_nodes, b2_leaves, S.srecs, b2_stk, o, d, P.tmin, closest, w);
        else best = traced_brute<MODE == MODE_CULLED>(S, o, d, P.tmin, closest, w);
        if (MARCH) {
            float tm;
            const int mg = march(S, o, d, P.tmin, P.tmax, closest, P.march_steps, tm, w);
            if (mg >= 0) { best = mg; closest = tm; }
        }
        float seg_depth; uint32_t seg_id;
        if (best >= 0) {
            F3 point, normal;
            finalize<MARCH>(S, best, o, d, P.tmin, closest, point, normal);
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
            if (COUNT) n_samples++;
            credited += ((done && P.adaptive) ? (P.spp_total - st.n) : 0u) + 1u;     // :196-198
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
    if (COUNT) {
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
    if (P.progress) {                                                          // live samples_atom (om_progress)
        const uint32_t c = wave_sum(credited);
        if ((threadIdx.x & 63u) == 0u && c) atomicAdd(&counters[OMC_PROGRESS], (unsigned long long)c);
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
    DevBuf counters, stats, pixels, view_scratch, view_rgb;
    // jitter tables, one immutable device buffer per (seed, spp_total): a table that queued
    // kernels may still read is never rewritten in place (most recent first, kMaxJitterTables)
    struct JitterTable { uint64_t seed; uint32_t spp; DevBuf buf; };
    std::vector<JitterTable> jitters;
    hipStream_t last_stream = nullptr;
    bool count_work = true;
    int pipeline = OM_PIPELINE_AUTO;
    uint32_t tail_bounce = 0;
    uint32_t wf_streams = 2;            // wavefront calls: batches in flight (om_set_streams)
    uint32_t ad_batches = 0, ad_paths_log2 = 0;   // adaptive wavefront schedule (om_set_adaptive_batches; 0 = default)
    // primary-ray tile lists (om_tiles.h): host record boxes of the uploaded world, the
    // device lists of the last (camera, frame, world) and the policy (om_set_primary_lists)
    std::vector<float> srec_box;
    uint64_t world_gen = 0;
    int primary_lists = OM_PRIMARY_LISTS_AUTO;
    DevBuf tile_off, tile_idx, tile_tnear;
    bool tiles_valid = false, tiles_use = false;
    om_camera tiles_cam{};
    uint32_t tiles_w = 0, tiles_h = 0;
    uint64_t tiles_gen = 0;
    double tiles_avg = 0.0;
    omw::Timer timer;
    omw::Buffers wf;
    unsigned long long* progress_host = nullptr;   // om_progress: pinned host word (null: progress off)
    DevBuf frame_list;                  // tile-ordered pixel list of the full frame (wavefront path)
    uint32_t frame_w = 0, frame_h = 0;
    ~om_ctx() {
        for (auto& b : scene_bufs) b.release();
        for (auto& j : jitters) j.buf.release();
        counters.release(); stats.release(); pixels.release(); frame_list.release();
        view_scratch.release(); view_rgb.release(); tile_off.release(); tile_idx.release(); tile_tnear.release();
        wf.release();
        timer.release();
        if (progress_host) (void)hipHostFree(progress_host);
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

// jitter table render_thread.rs:164-174: ((s/2)&1, s&1) shuffled once (om-rng SplitMix64 Fisher-Yates).
// Each (seed, spp) gets its own device buffer, written once before any kernel can read it,
// so an asynchronous call with another seed never races a queued one.
constexpr size_t kMaxJitterTables = 8;
om_status prepare_jitter(om_ctx* c, uint64_t seed, uint32_t spp, const float2** out) {
    *out = nullptr;
    for (size_t i = 0; i < c->jitters.size(); ++i)
        if (c->jitters[i].seed == seed && c->jitters[i].spp == spp) {
            if (i) std::rotate(c->jitters.begin(), c->jitters.begin() + i, c->jitters.begin() + i + 1);
            *out = (const float2*)c->jitters[0].buf.p;
            return OM_OK;
        }
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
    if (c->jitters.size() >= kMaxJitterTables) {      // evict the least recent once the device is idle
        OM_HIP(c, hipDeviceSynchronize());
        c->jitters.back().buf.release();
        c->jitters.pop_back();
    }
    om_ctx::JitterTable t{seed, spp, DevBuf{}};
    om_status s = ensure(c, t.buf, jt.size() * sizeof(float) + 16);
    if (s) return s;
    const hipError_t e = hipMemcpyAsync(t.buf.p, jt.data(), jt.size() * sizeof(float), hipMemcpyHostToDevice, c->stream);
    const hipError_t e2 = e == hipSuccess ? hipStreamSynchronize(c->stream) : e;   // jt is a host temporary
    if (e2 != hipSuccess) {
        t.buf.release();
        return set_err(c, OM_ERR_DEVICE, std::string("jitter upload: ") + hipGetErrorString(e2));
    }
    c->jitters.insert(c->jitters.begin(), t);
    *out = (const float2*)t.buf.p;
    return OM_OK;
}

om_status validate(om_ctx* c, const om_camera* cam, const om_render_params* p) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (!cam || !p) return set_err(c, OM_ERR_INVALID, "null camera/params");
    if (!c->have_world) return set_err(c, OM_ERR_STATE, "om_upload_world must precede rendering");
    if (p->width == 0 || p->height == 0) return set_err(c, OM_ERR_INVALID, "width/height must be > 0");
    if ((uint64_t)p->width * p->height > (1ull << 31)) return set_err(c, OM_ERR_INVALID, "image too large");
    return OM_OK;
}

template <int MODE, int BLOCK>
void go(bool count, uint64_t threads, uint32_t lds, hipStream_t stream, const OmSceneDev& S, const OmCamDev& C,
        const OmParamsDev& P, const float2* jt, om_pixel_stats* st, const uint32_t* px, unsigned long long* ctr) {
    const uint32_t blocks = (uint32_t)((threads + BLOCK - 1) / BLOCK);
    const bool march = (S.n_msph + S.n_mbox + S.n_mtor + S.n_msdf) != 0u;
    if (count && march)
        hipLaunchKernelGGL((render_kernel<MODE, BLOCK, true, true>), dim3(blocks), dim3(BLOCK), lds, stream, S, C, P, jt, st, px, ctr);
    else if (count)
        hipLaunchKernelGGL((render_kernel<MODE, BLOCK, true, false>), dim3(blocks), dim3(BLOCK), lds, stream, S, C, P, jt, st, px, ctr);
    else if (march)
        hipLaunchKernelGGL((render_kernel<MODE, BLOCK, false, true>), dim3(blocks), dim3(BLOCK), lds, stream, S, C, P, jt, st, px, ctr);
    else
        hipLaunchKernelGGL((render_kernel<MODE, BLOCK, false, false>), dim3(blocks), dim3(BLOCK), lds, stream, S, C, P, jt, st, px, ctr);
}

// Primary-ray candidate lists for (camera, frame, world), rebuilt only when one changes.
// AUTO uses them when a pixel sees <= 12 candidates on average (a primary BVH2 traversal
// costs ~11 node visits + 3.5 exact tests); S-traced at 1080p sees 3.2 (max 14 per tile).
constexpr double kTileListMaxAvg = 12.0;
om_status ensure_tile_lists(om_ctx* c, const om_camera* cam, uint32_t W, uint32_t H, hipStream_t stream) {
    if (c->primary_lists == OM_PRIMARY_LISTS_OFF) { c->tiles_use = false; return OM_OK; }
    const bool same = c->tiles_valid && c->tiles_gen == c->world_gen && c->tiles_w == W && c->tiles_h == H &&
                      std::memcmp(&c->tiles_cam, cam, sizeof(om_camera)) == 0;
    if (!same) {
        omt::TileLists tl;
        const bool ok = omt::build(c->srec_box, *cam, W, H, tl);
        // the cache keys are set only once the device lists are complete: a failed upload
        // leaves tiles_valid false, so the next call rebuilds instead of reading stale lists
        c->tiles_valid = false;
        c->tiles_use = false;
        if (ok) {
            om_status s = ensure(c, c->tile_off, tl.off.size() * 4u);
            // +1 entry: the uniform (scalar) reader loads whole dwords (traced_tiles<true>, om_trace.h)
            if (s == OM_OK) s = ensure(c, c->tile_idx, (tl.idx.size() + 2u) * 2u);
            if (s == OM_OK) s = ensure(c, c->tile_tnear, std::max<size_t>(tl.tnear.size(), 1u) * 4u);
            if (s != OM_OK) return s;
            OM_HIP(c, hipStreamSynchronize(stream));        // the previous lists may still be read
            OM_HIP(c, hipMemcpy(c->tile_off.p, tl.off.data(), tl.off.size() * 4u, hipMemcpyHostToDevice));
            if (!tl.idx.empty()) OM_HIP(c, hipMemcpy(c->tile_idx.p, tl.idx.data(), tl.idx.size() * 2u, hipMemcpyHostToDevice));
            if (!tl.tnear.empty())
                OM_HIP(c, hipMemcpy(c->tile_tnear.p, tl.tnear.data(), tl.tnear.size() * 4u, hipMemcpyHostToDevice));
        }
        c->tiles_valid = true; c->tiles_gen = c->world_gen; c->tiles_w = W; c->tiles_h = H; c->tiles_cam = *cam;
        c->tiles_avg = ok ? tl.avg_per_pixel : -1.0;
    }
    c->tiles_use = c->tiles_avg >= 0.0 &&
                   (c->primary_lists == OM_PRIMARY_LISTS_ON || c->tiles_avg <= kTileListMaxAvg);
    return OM_OK;
}

om_status launch(om_ctx* c, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_stats,
                 const uint32_t* dev_pixels, uint32_t n_pixels, hipStream_t stream) {
    // samples_per_pixel = 0: render()'s pass loop never runs (render_thread.rs:176), Stats untouched
    if (p->spp_total == 0 || p->sample_count == 0) return OM_OK;
    const float2* jitter = nullptr;
    om_status s = prepare_jitter(c, p->seed, p->spp_total, &jitter);
    if (s) return s;
    if (!c->counters.p) {
        s = ensure(c, c->counters, OMC_SLOTS * sizeof(unsigned long long));
        if (s) return s;
        OM_HIP(c, hipMemsetAsync(c->counters.p, 0, OMC_SLOTS * sizeof(unsigned long long), stream));
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
    P.progress = c->progress_host ? 1u : 0u;
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
    int pipeline = c->pipeline;
    // AUTO: the wavefront, the faster pipeline on every measured config since r04:
    // C1 6100 vs 3142 Msamples/s, C2 with one stream 2377 vs 1180-1202 (r04_ad), C2 adaptive 2939 vs
    // 1041 credited (16-sample calls), C1 adaptive 3466 vs 2832 (16-sample calls), 4199 vs 3388 (64),
    // all counting build; production build, C1 adaptive 64 spp in one call: 7171 vs 3392-3507 (r04_q7).
    if (pipeline == OM_PIPELINE_AUTO) pipeline = OM_PIPELINE_WAVEFRONT;
    int mode = c->kernel;
    if (mode == OM_KERNEL_AUTO) mode = OM_KERNEL_BVH2;
    if (pipeline == OM_PIPELINE_WAVEFRONT) {
        omw::Launch L;
        L.S = c->scene; L.C = C; L.P = P;
        L.jitter = jitter;
        L.stats = dev_stats;
        L.counters = (unsigned long long*)c->counters.p;
        L.count = c->count_work;
        L.tail_bounce = c->tail_bounce;
        L.streams = c->wf_streams;
        L.ad_batches = c->ad_batches; L.ad_paths_log2 = c->ad_paths_log2;
        L.timer = &c->timer;
        L.tile_off = nullptr; L.tile_idx = nullptr; L.tile_tnear = nullptr;
        L.progress_host = c->progress_host;
        if (mode == OM_KERNEL_BVH2 && c->scene.n_b2nodes) {
            if ((s = ensure_tile_lists(c, cam, p->width, p->height, stream)) != OM_OK) return s;
            if (c->tiles_use) {
                L.tile_off = (const uint32_t*)c->tile_off.p; L.tile_idx = (const uint16_t*)c->tile_idx.p;
                L.tile_tnear = (const float*)c->tile_tnear.p;
            }
        }
        L.trace_mode = mode == OM_KERNEL_BRUTE ? MODE_BRUTE : mode == OM_KERNEL_CULLED ? MODE_CULLED
                     : mode == OM_KERNEL_BVH ? MODE_BVH : mode == OM_KERNEL_BVH2 ? 6
                     : mode == OM_KERNEL_BVH4 ? 8 : MODE_SBVH_LDS;
        if (dev_pixels) {
            L.pixels = dev_pixels; L.n_pixels = n_pixels; L.stats_by_pixel = false;
        } else {
            if (c->frame_w != p->width || c->frame_h != p->height || !c->frame_list.p) {
                // 8x8 tiles in row-major tile order, lanes row-major inside a tile
                std::vector<uint32_t> lst;
                lst.reserve((size_t)p->width * p->height);
                const uint32_t tx = (p->width + 7u) / 8u, ty = (p->height + 7u) / 8u;
                for (uint32_t t = 0; t < tx * ty; ++t)
                    for (uint32_t l = 0; l < 64u; ++l) {
                        const uint32_t px = (t % tx) * 8u + (l & 7u), py = (t / tx) * 8u + (l >> 3);
                        if (px < p->width && py < p->height) lst.push_back(py * p->width + px);
                    }
                if ((s = ensure(c, c->frame_list, lst.size() * 4)) != OM_OK) return s;
                OM_HIP(c, hipMemcpyAsync(c->frame_list.p, lst.data(), lst.size() * 4, hipMemcpyHostToDevice, stream));
                OM_HIP(c, hipStreamSynchronize(stream));
                c->frame_w = p->width; c->frame_h = p->height;
            }
            L.pixels = (const uint32_t*)c->frame_list.p; L.n_pixels = p->width * p->height; L.stats_by_pixel = true;
        }
        std::string err;
        const hipError_t e = omw::render(c->wf, L, stream, err);
        if (e != hipSuccess) return set_err(c, OM_ERR_DEVICE, err + ": " + hipGetErrorString(e));
        return OM_OK;
    }
    const float2* jt = jitter;
    unsigned long long* ctr = (unsigned long long*)c->counters.p;
    const bool count = c->count_work;
    const int mk_ti = c->timer.begin(stream);
    if (mode == OM_KERNEL_SBVH) {
        if (c->scene.lds_bytes)
            go<MODE_SBVH_LDS, kBlockLds>(count, threads, c->scene.lds_bytes, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
        else
            go<MODE_SBVH_GLOBAL, kBlockLds>(count, threads, 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    } else if (mode == OM_KERNEL_BRUTE) {
        go<MODE_BRUTE, kBlock>(count, threads, 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    } else if (mode == OM_KERNEL_CULLED) {
        go<MODE_CULLED, kBlock>(count, threads, 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    } else if ((mode == OM_KERNEL_BVH2 || mode == OM_KERNEL_BVH4) && c->scene.n_b2nodes) {
        const uint32_t lds = kBlock * c->scene.b2_stack * 2u + c->scene.b2_lds_bytes;
        go<MODE_BVH2, kBlock>(count, threads, lds, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    } else if ((mode == OM_KERNEL_BVH2 || mode == OM_KERNEL_BVH4) && c->scene.n_bvh_nodes <= 1u) {
        // empty BVH2 and at most one leaf in the old BVH (marched-only worlds): the reference
        // loop, without MODE_BVH's scratch-memory stack
        go<MODE_BRUTE, kBlock>(count, threads, 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    } else {
        go<MODE_BVH, kBlock>(count, threads, 0, stream, c->scene, C, P, jt, dev_stats, dev_pixels, ctr);
    }
    c->timer.end(mk_ti, OM_KT_MEGAKERNEL, stream);
    OM_HIP(c, hipGetLastError());
    if (c->progress_host)   // one launch per call: the word advances when it ends
        OM_HIP(c, hipMemcpyAsync(c->progress_host, ctr + OMC_PROGRESS, sizeof(unsigned long long), hipMemcpyDeviceToHost, stream));
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
    UP(msph, msph); UP(mbox, mbox); UP(mtor, mtor); UP(msdf, msdf); UP(msdf_ops, msdf_ops);
    UP(mats, mats); UP(bloom, bloom); UP(bvh, bvh); UP(bvh_prims, bvh_prims); UP(always, always);
    UP(snodes, snodes); UP(srecs, srecs); UP(always2, always2); UP(always2_rec, always2_rec); UP(b2nodes, b2nodes); UP(b2h, b2h); UP(b2leaves, b2leaves);
#undef UP
    c->srec_box = fw.srec_box;
    c->world_gen++;
    c->tiles_valid = false;
    S.n_sph = fw.counts[0]; S.n_cube = fw.counts[1]; S.n_tri = fw.counts[2]; S.n_plane = fw.counts[3]; S.n_para = fw.counts[4];
    S.n_msph = fw.counts[5]; S.n_mbox = fw.counts[6]; S.n_mtor = fw.counts[7]; S.n_msdf = fw.counts[om::K_MSDF];
    S.off_cube = fw.offsets[1]; S.off_tri = fw.offsets[2]; S.off_plane = fw.offsets[3]; S.off_para = fw.offsets[4];
    S.off_msph = fw.offsets[5]; S.off_mbox = fw.offsets[6]; S.off_mtor = fw.offsets[7];
    S.off_msdf = fw.offsets[om::K_MSDF]; S.n_total = fw.offsets[om::K_N];
    S.n_bvh_nodes = (uint32_t)fw.bvh.size();
    S.n_always = (uint32_t)fw.always.size();
    S.n_snodes = (uint32_t)fw.snodes.size(); S.n_srecs = (uint32_t)fw.srecs.size(); S.n_always2 = (uint32_t)fw.always2.size();
    const size_t lds = fw.snodes.size() * sizeof(OmSkipNode) + fw.srecs.size() * sizeof(OmAffineTest);
    S.lds_bytes = lds <= kLdsBudget ? (uint32_t)(lds < 16 ? 16 : lds) : 0u;
    // compressed BVH2: usable when node and leaf ids fit the 15-bit codes and its depth fits
    // the lane-stack bound (otherwise the wavefront path uses the global-memory BVH)
    const bool b2_ok = !fw.b2nodes.empty() && fw.b2nodes.size() < 32768u && fw.b2leaves.size() < 32768u &&
                       fw.b2_depth <= 24u;   // lane stack bound (om_wavefront.hip kStackDepth)
    S.n_b2nodes = b2_ok ? (uint32_t)fw.b2nodes.size() : 0u;
    S.n_b2leaves = b2_ok ? (uint32_t)fw.b2leaves.size() : 0u;
    S.b2_direct = b2_ok ? fw.b2_direct : 0u;
    S.b2_stack = b2_ok ? fw.b2_depth : 0u;   // one push per internal level on the current path, deepest included
    const size_t b2_bytes = fw.b2nodes.size() * sizeof(OmBvh2Node) + fw.b2leaves.size() * 4u;
    S.b2_lds_bytes = (b2_ok && b2_bytes <= kB2LdsBudget) ? (uint32_t)((b2_bytes + 15u) & ~(size_t)15u) : 0u;
    // BVH4 (same leaf table): up to 3 pushes per level + 3 spare entries for the
    // unconditional pushes, within the 48-entry bound of om_wavefront.hip
    const uint32_t b4_stack = 3u * fw.b4_depth + 3u;
    const bool b4_ok = b2_ok && !fw.b4nodes.empty() && fw.b4nodes.size() < 32768u && b4_stack <= 48u;
    if (b4_ok && (s = upload(c, fw.b4nodes, &S.b4nodes)) != OM_OK) return s;
    if (b4_ok && (s = upload(c, fw.b4h, &S.b4h)) != OM_OK) return s;
    S.n_b4nodes = b4_ok ? (uint32_t)fw.b4nodes.size() : 0u;
    S.b4_stack = b4_ok ? b4_stack : 0u;
    const size_t b4_bytes = fw.b4nodes.size() * sizeof(OmBvh4Node) + fw.b2leaves.size() * 4u;
    S.b4_lds_bytes = (b4_ok && b4_bytes <= 40u * 1024u) ? (uint32_t)((b4_bytes + 15u) & ~(size_t)15u) : 0u;
    OM_HIP(c, hipStreamSynchronize(c->stream));
    c->have_world = true;
    return OM_OK;
}

om_status om_set_kernel(om_ctx* c, int32_t k) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (k < OM_KERNEL_AUTO || k > OM_KERNEL_BVH4) return set_err(c, OM_ERR_INVALID, "om_set_kernel: unknown kernel");
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

om_status om_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return set_err(nullptr, OM_ERR_INVALID, "om_host_register: null/empty buffer");
    const hipError_t e = hipHostRegister(p, bytes, hipHostRegisterDefault);
    if (e != hipSuccess) return set_err(nullptr, OM_ERR_DEVICE, std::string("om_host_register: ") + hipGetErrorString(e));
    return OM_OK;
}

om_status om_host_unregister(void* p) {
    if (!p) return set_err(nullptr, OM_ERR_INVALID, "om_host_unregister: null buffer");
    const hipError_t e = hipHostUnregister(p);
    if (e != hipSuccess) return set_err(nullptr, OM_ERR_DEVICE, std::string("om_host_unregister: ") + hipGetErrorString(e));
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

om_status om_set_pipeline(om_ctx* c, int32_t pipeline) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (pipeline != OM_PIPELINE_MEGAKERNEL && pipeline != OM_PIPELINE_WAVEFRONT && pipeline != OM_PIPELINE_AUTO)
        return set_err(c, OM_ERR_INVALID, "om_set_pipeline: unknown pipeline");
    c->pipeline = pipeline;
    return OM_OK;
}

om_status om_set_primary_lists(om_ctx* c, int32_t mode) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (mode < OM_PRIMARY_LISTS_OFF || mode > OM_PRIMARY_LISTS_ON)
        return set_err(c, OM_ERR_INVALID, "om_set_primary_lists: unknown mode");
    c->primary_lists = mode;
    return OM_OK;
}

om_status om_set_tail_bounce(om_ctx* c, uint32_t bounce) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    c->tail_bounce = bounce;
    return OM_OK;
}

om_status om_set_streams(om_ctx* c, uint32_t streams) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (streams < 1 || streams > (uint32_t)omw::kMaxSets) return set_err(c, OM_ERR_INVALID, "om_set_streams: streams must be 1..4");
    c->wf_streams = streams;
    return OM_OK;
}

om_status om_set_adaptive_batches(om_ctx* c, uint32_t batches, uint32_t paths_log2) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    // every planned batch is launched whether or not the device plan leaves it any pixel (the host
    // never reads the live count back): ~10 launches of ~5 us each per empty batch and stream, so
    // the knob is capped at a few dozen batches
    if (batches > 64u || paths_log2 > 27u)
        return set_err(c, OM_ERR_INVALID, "om_set_adaptive_batches: batches <= 64, paths_log2 <= 27");
    c->ad_batches = batches; c->ad_paths_log2 = paths_log2;
    return OM_OK;
}

om_status om_set_timing(om_ctx* c, int32_t mode) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (mode < 0 || mode > 2) return set_err(c, OM_ERR_INVALID, "om_set_timing: mode must be 0, 1 or 2");
    OM_HIP(c, hipSetDevice(c->device));
    for (size_t i = 0; c->timer.on() && i < c->timer.cls.size(); ++i)
        if (c->timer.cls[i] >= 0) OM_HIP(c, hipEventSynchronize(c->timer.ev[2 * i + 1]));
    c->timer.mode = mode;
    c->timer.clear();
    return OM_OK;
}

om_status om_get_kernel_times(om_ctx* c, om_kernel_times* out) {
    if (!c || !out) return set_err(c, OM_ERR_INVALID, "om_get_kernel_times: null argument");
    OM_HIP(c, hipSetDevice(c->device));
    *out = om_kernel_times{};
    omw::Timer& t = c->timer;
    for (size_t i = 0; i < t.cls.size(); ++i) {
        if (t.cls[i] < 0) continue;
        OM_HIP(c, hipEventSynchronize(t.ev[2 * i + 1]));
        float ms = 0.0f;
        OM_HIP(c, hipEventElapsedTime(&ms, t.ev[2 * i], t.ev[2 * i + 1]));
        out->launches[t.cls[i]] += t.nl[i];
        out->ms[t.cls[i]] += (double)ms;
    }
    t.clear();
    return OM_OK;
}

om_status om_display_device(om_ctx* c, const om_pixel_stats* dev_stats, uint32_t width, uint32_t height, int32_t view,
                            uint8_t* dev_rgb, void* stream) {
    if (!c || !dev_stats || !dev_rgb) return set_err(c, OM_ERR_INVALID, "om_display_device: null argument");
    if (view < OM_VIEW_NORMAL || view > OM_VIEW_ID_BLUR) return set_err(c, OM_ERR_INVALID, "om_display_device: unknown view");
    if (width == 0 || height == 0 || (uint64_t)width * height > 0xFFFFFFFFull / 3u)
        return set_err(c, OM_ERR_INVALID, "om_display_device: bad frame size");
    const bool blur = view == OM_VIEW_SAMPLE_BLUR || view == OM_VIEW_DEPTH_BLUR || view == OM_VIEW_ID_BLUR;
    if (blur && (width < 2 || height < 2))   // apply_box_filter indexes a 2x2 corner neighbourhood
        return set_err(c, OM_ERR_INVALID, "om_display_device: blur views need width, height >= 2");
    OM_HIP(c, hipSetDevice(c->device));
    om_status s = ensure(c, c->view_scratch, omv::scratch_bytes(width, height));
    if (s != OM_OK) return s;
    hipStream_t st = stream ? (hipStream_t)stream : c->stream;
    const hipError_t e = omv::render(dev_stats, width, height, view, dev_rgb, c->view_scratch.p, st);
    if (e != hipSuccess) return set_err(c, OM_ERR_DEVICE, std::string("om_display_device: ") + hipGetErrorString(e));
    c->last_stream = st;
    return OM_OK;
}

om_status om_display(om_ctx* c, const om_pixel_stats* stats, uint32_t width, uint32_t height, int32_t view, uint8_t* rgb) {
    if (!c || !stats || !rgb) return set_err(c, OM_ERR_INVALID, "om_display: null argument");
    if (width == 0 || height == 0 || (uint64_t)width * height > 0xFFFFFFFFull / 3u)
        return set_err(c, OM_ERR_INVALID, "om_display: bad frame size");
    OM_HIP(c, hipSetDevice(c->device));
    const size_t npx = (size_t)width * height;
    om_status s = ensure(c, c->stats, npx * sizeof(om_pixel_stats));
    if (s != OM_OK) return s;
    if ((s = ensure(c, c->view_rgb, npx * 3)) != OM_OK) return s;
    OM_HIP(c, hipMemcpyAsync(c->stats.p, stats, npx * sizeof(om_pixel_stats), hipMemcpyHostToDevice, c->stream));
    OM_HIP(c, hipMemcpyAsync(c->view_rgb.p, rgb, npx * 3, hipMemcpyHostToDevice, c->stream));
    if ((s = om_display_device(c, (const om_pixel_stats*)c->stats.p, width, height, view, (uint8_t*)c->view_rgb.p, c->stream)) != OM_OK)
        return s;
    OM_HIP(c, hipMemcpyAsync(rgb, c->view_rgb.p, npx * 3, hipMemcpyDeviceToHost, c->stream));
    OM_HIP(c, hipStreamSynchronize(c->stream));
    return OM_OK;
}

const volatile uint64_t* om_progress(om_ctx* c) {
    if (!c) { set_err(nullptr, OM_ERR_INVALID, "om_progress: null ctx"); return nullptr; }
    if (c->progress_host) return (const volatile uint64_t*)c->progress_host;
    if (hipSetDevice(c->device) != hipSuccess) { set_err(c, OM_ERR_DEVICE, "om_progress: hipSetDevice"); return nullptr; }
    if (!c->counters.p) {
        if (ensure(c, c->counters, OMC_SLOTS * sizeof(unsigned long long)) != OM_OK) return nullptr;
        if (hipMemset(c->counters.p, 0, OMC_SLOTS * sizeof(unsigned long long)) != hipSuccess) {
            set_err(c, OM_ERR_DEVICE, "om_progress: hipMemset");
            return nullptr;
        }
    }
    unsigned long long* h = nullptr;
    if (hipHostMalloc((void**)&h, sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess) {
        set_err(c, OM_ERR_NOMEM, "om_progress: hipHostMalloc");
        return nullptr;
    }
    *h = 0;
    if (hipStreamSynchronize(c->stream) != hipSuccess ||
        hipMemcpy(h, (unsigned long long*)c->counters.p + OMC_PROGRESS, sizeof(*h), hipMemcpyDeviceToHost) != hipSuccess) {
        (void)hipHostFree(h);
        set_err(c, OM_ERR_DEVICE, "om_progress: reading the device word");
        return nullptr;
    }
    c->progress_host = h;
    return (const volatile uint64_t*)h;
}

om_status om_reset_progress(om_ctx* c) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    if (!c->progress_host) return OM_OK;
    OM_HIP(c, hipSetDevice(c->device));
    OM_HIP(c, hipDeviceSynchronize());
    OM_HIP(c, hipMemset((unsigned long long*)c->counters.p + OMC_PROGRESS, 0, sizeof(unsigned long long)));
    *(volatile unsigned long long*)c->progress_host = 0;
    return OM_OK;
}

om_status om_set_counting(om_ctx* c, int32_t enable) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    c->count_work = enable != 0;
    return OM_OK;
}

om_status om_reset_counters(om_ctx* c, void* stream) {
    if (!c) return set_err(nullptr, OM_ERR_INVALID, "null ctx");
    OM_HIP(c, hipSetDevice(c->device));
    const bool fresh = !c->counters.p;
    om_status s = ensure(c, c->counters, OMC_SLOTS * sizeof(unsigned long long));
    if (s) return s;
    // the counters only; the progress word after them keeps counting (om_reset_progress)
    OM_HIP(c, hipMemsetAsync(c->counters.p, 0, (fresh ? OMC_SLOTS : OMC_N) * sizeof(unsigned long long),
                             stream ? (hipStream_t)stream : c->stream));
    return OM_OK;
}

}  // extern "C"

namespace omi {
int ctx_device(const om_ctx* c) { return c->device; }
hipStream_t ctx_stream(const om_ctx* c) { return c->stream; }
om_status ctx_error(om_ctx* c, om_status code, const std::string& msg) { return set_err(c, code, msg); }
om_status global_error(om_status code, const std::string& msg) { return set_err(nullptr, code, msg); }
}  // namespace omi
