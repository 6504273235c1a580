// om_wavefront.hip — wavefront path tracer: the bounce recursion of
// ray_color (render_thread.rs:128-143) flattened into per-bounce launches over SoA
// path queues in HBM:
//
//   bounce 0    one lane per (sample, pixel): camera ray (render_thread.rs:183-192),
//               closest hit (hits.rs:270-365), HitRecord + Material::scatter / sky
//               (render_thread.rs:105-126); survivors are compacted into queue 1,
//               finished paths write (colour, depth, id) to their result slot
//   bounce b    the same from queue b: trace + shade + compaction in ONE kernel (the
//               path state is read once and written once per bounce; no hit buffer)
//   tail        from bounce T on the queues hold a few thousand paths: one persistent
//               launch runs every remaining path to completion, lanes stealing paths
//               from a per-workgroup LDS counter (no ~40 near-empty launch pairs)
//   accumulate  one lane per pixel: Stats::add over the batch's samples IN SAMPLE
//               ORDER (render_thread.rs:23-39): bit-identical to the sequential
//               reference and to the megakernel.
//
// Queues are SEGMENTED: workgroup s owns segment s of every queue and compacts its
// survivors into segment s of the next queue with a ballot + LDS scan — no global
// atomics (one contended queue counter capped the first version at ~88 wave-appends
// per microsecond, MI355X_MICROARCH.md row 'dequeue').  Paths are sample-major
// (slot = s_local * n_pixels + k over a tile-ordered pixel list), so a wave holds 64
// neighbouring pixels of one sample: coherent rays.
#include "om_wavefront.h"

#include <algorithm>

#include "om_device.h"
#include "om_trace.h"
#include "om_tuning.h"

using namespace omd;

namespace omw {

void QueueSet::release() {
    for (int a = 0; a < 2; ++a) {
        for (int b = 0; b < 3; ++b) { if (q[a][b]) (void)hipFree(q[a][b]); q[a][b] = nullptr; }
        if (qr[a]) (void)hipFree(qr[a]); qr[a] = nullptr;
    }
    if (res) (void)hipFree(res);
    if (res_id) (void)hipFree(res_id);
    if (counts) (void)hipFree(counts);
    if (hit) (void)hipFree(hit);
    res = nullptr; res_id = nullptr; counts = nullptr; hit = nullptr;
}

void Buffers::release() {
    for (auto& s : set) s.release();
    if (n0) (void)hipFree(n0);
    n0 = nullptr; n0_cap = 0;
    for (auto& st : side) { if (st) (void)hipStreamDestroy(st); st = nullptr; }

    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
    cap = 0; counts_n = 0; nsets = 0;
}

namespace {

constexpr uint32_t kNoSample = 0xFFFFFFFFu;
enum { TR_BRUTE = 1, TR_CULLED = 2, TR_BVH = 3, TR_SBVH_LDS = 4, TR_SBVH_GLOBAL = 5, TR_BVH2_LDS = 6, TR_BVH2_GLOBAL = 7,
       TR_BVH4_LDS = 8, TR_BVH4_GLOBAL = 9 };
#define OM_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(OM_WF_WAVES, OM_WF_WAVES)))   // occupancy request (waves per SIMD)
constexpr int kBlk = OM_WF_BLOCK;                                 // workgroup = one queue segment
constexpr int kStackDepth = 24;                                   // BVH2 per-lane LDS stack bound (entries)
// f32 BVH2 nodes staged in LDS sit OM_B2_NODE_STRIDE bytes apart (om_tuning.h)
constexpr uint32_t kB2Stride = OM_B2_NODE_STRIDE;
static_assert(kB2Stride % 16u == 0u && kB2Stride >= sizeof(OmBvh2Node), "16-B aligned node slots");
// LDS bytes of the lane stack: S.b2_stack entries per lane (the tree's internal depth, 9 for
// S-traced: 9 KiB per 512-lane workgroup instead of 24 KiB at the 24-entry bound).
template <int TR>
__host__ __device__ inline uint32_t stack_bytes(const OmSceneDev& S) {
    return kBlk * ((TR == TR_BVH4_LDS || TR == TR_BVH4_GLOBAL) ? S.b4_stack : S.b2_stack) * 2u;
}
// LDS bytes of a BVH2 staged whole (TR_BVH2_LDS): padded nodes + leaf table
__host__ __device__ inline uint32_t b2_stage_bytes(const OmSceneDev& S) {
    return (S.n_b2nodes * kB2Stride + S.n_b2leaves * 4u + 15u) & ~15u;
}
constexpr uint32_t kTailSpb = OM_WF_TAIL_SPB;                     // queue segments per tail workgroup
constexpr uint32_t kTailDefault = 16;                             // first bounce handled by the tail kernel
// marched worlds: bounce 0 as k_march + k_bounce<HIT>, every later segment in the lane-refilling
// tail (om_tuning.h)
constexpr uint32_t kTailMarched = OM_WF_TAIL_MARCHED;
// BVH2s read through L2 (S-10k): 10 (C3, r03_v24/v25: T = 6 / 8 / 10 / 12 / 16 / 20 -> 3318 / 3523 /
// 3553 / 3517 / 3416 / 3351 Msamples/s, means of two to four runs)
constexpr uint32_t kTailL2 = 10;
// batches above 2^25 paths (C4's 4K frame: 16 spp = 133M paths) keep more paths per late bounce,
// so the per-bounce launches stay efficient longer: 24 (C4, r03_v26: T = 12 / 16 / 20 / 24 ->
// 6956 / 7240 / 7304 / 7374 Msamples/s, means of two runs)
constexpr uint32_t kTailBigBatch = 24;
__host__ __device__ inline uint32_t hyb_nodes(const OmSceneDev& S) {
    constexpr uint32_t kCap = OM_WF_HYB_BYTES / (uint32_t)sizeof(OmBvh2NodeH);
    return S.b2_lds_bytes ? 0u : (S.n_b2nodes < kCap ? S.n_b2nodes : kCap);
}
__host__ __device__ inline uint32_t hyb4_nodes(const OmSceneDev& S) {
    constexpr uint32_t kCap = OM_WF_HYB4_BYTES / (uint32_t)sizeof(OmBvh4NodeH);
    return S.b4_lds_bytes ? 0u : (S.n_b4nodes < kCap ? S.n_b4nodes : kCap);
}
// k_march's instance for a marched set of exactly C2's shape (2 spheres, 1 box, 1 torus: S-marched):
// the SDF-only fields staged in LDS once per workgroup, every march step unrolled with no count
// guards; other marched sets read the scene arrays.  Traced parts TR_BRUTE /
// TR_BVH2_LDS only.
using MarchedC2Lds = MarchedExactLds<2, 1, 1>;
enum { MV_ARRAYS = 0, MV_EXACT_C2_LDS = 1 };
template <int TR>
__host__ __device__ constexpr bool exact_view_built() { return TR == TR_BRUTE || TR == TR_BVH2_LDS; }
// Segment capacity rounded up to whole waves, so that a bounce-0 wave is exactly one 8x8 tile of
// one sample (tile-ordered pixel lists hold whole tiles).
__host__ __device__ inline uint32_t seg_capacity(uint64_t paths, uint32_t nseg) {
    const uint64_t c = (paths + nseg - 1) / nseg;
    return (uint32_t)((c + 63u) / 64u * 64u);
}

extern __shared__ __attribute__((aligned(16))) uint4 wf_lds[];

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ void flush_counter(unsigned long long* ctr, int slot, uint32_t v) {
    v = wave_sum32(v);
    if (__lane_id() == 0 && v) atomicAdd(&ctr[slot], (unsigned long long)v);
}

struct Seg {
    uint32_t nseg;    // segments (= bounce workgroups)
    uint32_t segcap;  // paths per segment
};

// Adaptive calls: per stream and batch, the stream's live pixels listed for the
// batch (c, counted by the previous k_accumulate's compaction) and the call's samples rendered
// before it (done).  The batch's sample count is a function of the two, evaluated by every kernel
// of the batch (ad_batch), so the host never reads the count back.
struct AdPlan { uint32_t c, done; };
struct AdCfg {
    uint32_t sample_count;   // samples of the call
    uint32_t batches;        // batches per stream per call
    uint32_t paths;          // target paths per batch (c x b)
};
__host__ __device__ inline uint32_t ad_batch(uint32_t c, uint32_t done, uint32_t j, const AdCfg& A) {
    if (c == 0u || done >= A.sample_count || j >= A.batches) return 0u;
    const uint32_t rem = A.sample_count - done, left = A.batches - j;
    const uint32_t even = (rem + left - 1u) / left, want = A.paths / c;
    const uint32_t b = even > want ? even : want;
    return b < rem ? b : rem;
}
// a batch's adaptive list: the live list, its plan, the stream's next list and plan
struct AdList {
    const uint32_t* list;    // null: fixed-spp batch over the whole pixel list
    const AdPlan* plan;
    uint32_t* list_next;
    AdPlan* plan_next;
    AdCfg A;
    uint32_t j;              // batch index within the stream's call
};

// One SoA path queue: o|depthf, d|first_id, throughput|segment, rng s|rng k|slot|-.
// (SoA, not 64-B AoS records: AoS measured -22% on C1, r05_sort)
struct Queue {
    float4* q0; float4* q1; float4* q2; uint4* qr;
};

// Primary-ray source of bounce 0 (render_thread.rs:176-192).
struct Gen {
    OmCamDev C;
    const float2* jitter;
    const om_pixel_stats* stats;
    const uint32_t* pixels;      // tile-ordered pixel list
    uint32_t n_pixels, by_pixel, batch;
    const uint32_t* n0;          // concurrent fixed-spp calls: per listed pixel, Stats.n at the call start
    uint32_t done;               // samples of the call before this batch (with n0)
    AdList ad;                   // adaptive calls: the stream's live list (ad.list null otherwise)
    const uint32_t* tile_off;    // primary-ray candidate lists (null: traverse)
    const uint16_t* tile_idx;
    const float* tile_tnear;
};

// A path between bounces: ray_color's loop state (render_thread.rs:128-143).
struct Path {
    F3 o, d, cur;
    float depthf;
    uint32_t first_id, seg, slot;
    Rng g;
};

// The path-state loads and stores carry the non-temporal hint: each 16-B lane record is read
// once per bounce and written once, so the streaming queues do not evict the leaf records and
// nodes the trace re-reads from the vector L1.  Component loads keep the scalar register shapes
// (a native 4-vector load moved k_bounce into scratch spills in r01); the compiler still merges
// them into global_load/store_dwordx4 ... nt.  C1: 7096 / 7114 vs 7094 / 7068 Msamples/s (r03_v13).
template <class V>
__device__ __forceinline__ V ld4(const V* q) {
    V v;
    v.x = __builtin_nontemporal_load(&q->x); v.y = __builtin_nontemporal_load(&q->y);
    v.z = __builtin_nontemporal_load(&q->z); v.w = __builtin_nontemporal_load(&q->w);
    return v;
}
__device__ __forceinline__ void load_ray(const Queue& Q, uint64_t i, Path& p) {
    const float4 a = ld4(Q.q0 + i), b = ld4(Q.q1 + i);
    p.o = f3(a.x, a.y, a.z); p.depthf = a.w;
    p.d = f3(b.x, b.y, b.z); p.first_id = __float_as_uint(b.w);
}
__device__ __forceinline__ void load_rest(const Queue& Q, uint64_t i, Path& p) {
    const float4 c = ld4(Q.q2 + i);
    const uint4 r = ld4(Q.qr + i);
    p.cur = f3(c.x, c.y, c.z); p.seg = __float_as_uint(c.w);
    p.g.s = r.x; p.g.k = r.y; p.slot = r.z;
}
template <class V>
__device__ __forceinline__ void st4(V* q, V v) {
    __builtin_nontemporal_store(v.x, &q->x); __builtin_nontemporal_store(v.y, &q->y);
    __builtin_nontemporal_store(v.z, &q->z); __builtin_nontemporal_store(v.w, &q->w);
}
__device__ __forceinline__ void store_path(const Queue& Q, uint64_t i, const Path& p) {
    st4(Q.q0 + i, make_float4(p.o.x, p.o.y, p.o.z, p.depthf));
    st4(Q.q1 + i, make_float4(p.d.x, p.d.y, p.d.z, __uint_as_float(p.first_id)));
    st4(Q.q2 + i, make_float4(p.cur.x, p.cur.y, p.cur.z, __uint_as_float(p.seg)));
    st4(Q.qr + i, make_uint4(p.g.s, p.g.k, p.slot, 0u));
}

// Scene data a workgroup traces against: the BVH2/BVH4 nodes + leaf table staged in LDS behind
// the per-lane stack ([stack][nodes][leaf table]), or (TR_BVH2_GLOBAL) the breadth-first prefix
// of the half-precision nodes in LDS and the rest read through L2.
struct Tracer {
    const OmBvh2Node* b2n;   // TR_BVH2_LDS: f32 nodes in LDS
    const OmBvh2NodeH* h2l;  // TR_BVH2_GLOBAL: half nodes [0, nl) staged in LDS
    const OmBvh2NodeH* h2g;  //                 every half node, through L2
    uint32_t nl;
    const OmBvh4Node* b4n;
    const OmBvh4NodeH* h4l;  // TR_BVH4_GLOBAL: half nodes [0, nl) staged in LDS
    const OmBvh4NodeH* h4g;  //                 every half node, through L2
    const uint32_t* bl;
    const OmAffineTest* recs;
    uint16_t* stk;
};

template <int TR, uint32_t STACKS = 1>
__device__ __forceinline__ Tracer stage_scene(const OmSceneDev& S) {   // every thread of the block calls it
    Tracer t;
    t.stk = (uint16_t*)wf_lds + threadIdx.x;
    t.b2n = S.b2nodes; t.b4n = S.b4nodes; t.bl = S.b2leaves; t.recs = S.srecs;
    t.h2l = S.b2h; t.h2g = S.b2h; t.nl = 0;
    t.h4l = S.b4h; t.h4g = S.b4h;
    if (TR == TR_BVH4_GLOBAL && hyb4_nodes(S)) {
        t.nl = hyb4_nodes(S);
        uint4* dst = wf_lds + STACKS * stack_bytes<TR>(S) / 16u;
        const uint4* sn = (const uint4*)S.b4h;
        for (uint32_t i = threadIdx.x; i < t.nl * (uint32_t)(sizeof(OmBvh4NodeH) / 16u); i += kBlk) dst[i] = sn[i];
        __syncthreads();
        t.h4l = (const OmBvh4NodeH*)dst;
    }
    if (TR == TR_BVH2_GLOBAL && hyb_nodes(S)) {
        t.nl = hyb_nodes(S);
        uint4* dst = wf_lds + STACKS * stack_bytes<TR>(S) / 16u;
        const uint4* sn = (const uint4*)S.b2h;
        for (uint32_t i = threadIdx.x; i < t.nl * (uint32_t)(sizeof(OmBvh2NodeH) / 16u); i += kBlk) dst[i] = sn[i];
        __syncthreads();
        t.h2l = (const OmBvh2NodeH*)dst;
    }
    if (TR == TR_BVH2_LDS || TR == TR_BVH4_LDS) {
        // uint4 words per node in memory / per node slot in LDS (BVH2: padded to kB2Stride)
        constexpr uint32_t wn = TR == TR_BVH2_LDS ? (uint32_t)(sizeof(OmBvh2Node) / 16u) : (uint32_t)(sizeof(OmBvh4Node) / 16u);
        constexpr uint32_t ws = TR == TR_BVH2_LDS ? kB2Stride / 16u : wn;
        const uint32_t nn = (TR == TR_BVH2_LDS ? S.n_b2nodes : S.n_b4nodes) * wn;
        const uint4* sn = TR == TR_BVH2_LDS ? (const uint4*)S.b2nodes : (const uint4*)S.b4nodes;
        uint4* dst = wf_lds + STACKS * stack_bytes<TR>(S) / 16u;
        for (uint32_t i = threadIdx.x; i < nn; i += kBlk) {
            uint4 v = sn[i];
            // BVH2 child codes (words 0 and 2: c0, c1) of internal nodes become slot offsets in
            // 16-B units, so the traversal addresses a node with a shift (traced_bvh2's CUNIT)
            if (TR == TR_BVH2_LDS && (i % wn) % 2u == 0u && v.w < OM_LEAF) v.w *= ws;
            dst[(i / wn) * ws + i % wn] = v;
        }
        uint32_t* ldst = (uint32_t*)(dst + nn / wn * ws);
        for (uint32_t i = threadIdx.x; i < S.n_b2leaves; i += kBlk) ldst[i] = S.b2leaves[i];
        __syncthreads();
        t.b2n = (const OmBvh2Node*)dst; t.b4n = (const OmBvh4Node*)dst; t.bl = ldst;
    }
    return t;
}

// Closest hit of one ray (hits.rs:270-365): -> (closest, global prim index or -1).
// MARCH is a compile-time split: the sphere-tracing code (3 SDFs + unstuck) would
// otherwise set the register budget of every traced-only scene.
template <int TR, bool MARCH, class Wk>
__device__ __forceinline__ int trace(const OmSceneDev& S, const OmParamsDev& P, const Tracer& T, F3 o, F3 d,
                                     float& closest, Wk& w) {
    closest = P.tmax;
    int best;
    if (TR == TR_BVH4_LDS) best = traced_bvh4<kBlk>(S, T.b4n, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w);
    else if (TR == TR_BVH4_GLOBAL)
        best = traced_bvh4<kBlk, Wk, true>(S, T.h4l, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w, T.h4g, T.nl);
    else if (TR == TR_BVH2_LDS)
        best = traced_bvh2<kStackDepth, kBlk, Wk, false, OmBvh2Node, 16>(S, T.b2n, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w);
    else if (TR == TR_BVH2_GLOBAL)
        best = traced_bvh2<kStackDepth, kBlk, Wk, true>(S, T.h2l, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w, T.h2g, T.nl);
    else if (TR == TR_SBVH_GLOBAL) best = traced_sbvh(S, S.snodes, S.srecs, o, d, P.tmin, closest, w);
    else if (TR == TR_BVH) best = traced_bvh(S, o, d, P.tmin, closest, w);
    else best = traced_brute<TR == TR_CULLED>(S, o, d, P.tmin, closest, w);
    if (MARCH) {
        float tm;
        const int mg = march(S, o, d, P.tmin, P.tmax, closest, P.march_steps, tm, w);
        if (mg >= 0) { best = mg; closest = tm; }
    }
    return best;
}

// handle_hit + ray_color's termination rules (render_thread.rs:105-143) for one
// segment.  Returns true when the path continues (p advanced to the next segment);
// otherwise the sample's (colour, depth, id) is written to its result slot.
template <bool MARCH, bool USER = MARCH>
__device__ __forceinline__ bool shade_path(const OmSceneDev& S, const OmParamsDev& P, uint32_t depth_cap, Path& p,
                                           float closest, int best, float4* __restrict__ res,
                                           uint32_t* __restrict__ res_id) {
    float seg_depth; uint32_t seg_id;
    if (best >= 0) {                                                   // handle_hit, Some(hr)
        F3 point, normal;
        finalize<MARCH, USER>(S, best, p.o, p.d, P.tmin, closest, point, normal);
        F3 nd, att;
        scatter(S.mats[best], p.d, normal, p.g, nd, att);
        p.cur = mul(p.cur, att);
        p.o = point; p.d = unit(nd);
        seg_depth = closest; seg_id = (uint32_t)best + 1u;
    } else {                                                           // None: sky (render_thread.rs:118-120)
        const float t = 0.5f * (p.d.y + 1.0f);
        p.cur = mul(p.cur, f3((1.0f - t) + 0.5f * t, (1.0f - t) + 0.7f * t, (1.0f - t) + 1.0f * t));
        seg_depth = INFINITY; seg_id = 0u;
    }
    bool finished = false;
    F3 result = p.cur;
    float rdepth = 0.0f; uint32_t rid = 0;
    if (p.seg == 0u) {
        p.depthf = seg_depth; p.first_id = seg_id;
        if (isinf(seg_depth)) { finished = true; rdepth = INFINITY; rid = 0u; }         // :133-135
    } else if (isinf(seg_depth)) {
        finished = true; rdepth = p.depthf; rid = p.first_id;                            // :138-140
    }
    if (!finished && p.seg + 1u >= depth_cap) {                                          // :142 -Color::ZERO
        finished = true; result = f3(-0.0f, -0.0f, -0.0f); rdepth = p.depthf; rid = p.first_id;
    }
    if (finished) {
        res[p.slot] = make_float4(result.x, result.y, result.z, rdepth);
        res_id[p.slot] = rid;
        return false;
    }
    p.seg += 1u;
    return true;
}

// Camera sample i of the batch (render_thread.rs:176-192): -> p (a fresh path) and its
// pixel; false (and no sample recorded in res_id) when the sample is not taken.
// `stride` is the batch's pixel count: the whole list (fixed spp) or the stream's live list.
__device__ __forceinline__ bool gen_path(const OmParamsDev& P, const Gen& R, uint32_t stride, uint64_t i, Path& p,
                                         uint32_t& pixel, uint32_t* __restrict__ res_id) {
    const uint32_t s_local = (uint32_t)i / stride, kk = (uint32_t)i - s_local * stride;
    const uint32_t k = R.ad.list ? R.ad.list[kk] : kk;
    pixel = R.pixels[k];
    // the sample index is the pixel's Stats.n (jitters[pixel.stats.n], render_thread.rs:188).
    // Concurrent fixed-spp calls take it from the call-start snapshot plus the samples of the
    // batches before this one, so a batch never waits for the previous batch's accumulate.
    // Serial and adaptive calls read the live Stats: an adaptive stream's pixels are its own, and
    // its previous batch's accumulate has run on the same stream.
    uint32_t s;
    bool live;
    if (R.n0) {
        const uint32_t v = R.n0[k];
        s = (v & 0x7FFFFFFFu) + R.done + s_local;
        live = s < P.spp_total && !(v >> 31);
    } else {
        const om_pixel_stats& ps = R.stats[R.by_pixel ? pixel : k];
        s = ps.n + s_local;
        live = s < P.spp_total && !(P.adaptive && (ps.flags & 1u));
    }
    if (!live) {
        res_id[i] = kNoSample;
        return false;
    }
    p.g = path_rng(P.skey, pixel, s);
    const uint32_t line = pixel / P.width;
    gen_camera_ray(R.C, P, R.jitter, (float)(pixel - P.width * line), (float)line, s, p.g, p.o, p.d);
    p.cur = f3(1.0f, 1.0f, 1.0f); p.depthf = 0.0f; p.first_id = 0u; p.seg = 0u; p.slot = (uint32_t)i;
    return true;
}

// ---------------------------------------------------------------- bounce
// Workgroup s: the paths of segment s of queue `in` (FIRST: the camera samples
// [s*segcap, (s+1)*segcap) of the batch) -> survivors into segment s of `out`.
// HIT (split march pipeline): no trace here; the (closest, winner) of every path of the
// segment was written to `hitbuf` (queue-slot order) by k_march.
// Work distribution: every wave takes 64-path chunks of the segment from an
// LDS counter and appends its survivors with one LDS atomic, so the 8 waves never wait for each
// other.  Queue order within a segment then depends on which wave finishes first; results are
// keyed by slot and the RNG by (pixel, sample), never by queue position.
template <int TR, bool COUNT, bool MARCH, bool FIRST, bool HIT = false, bool USER = MARCH>
__global__ __launch_bounds__(kBlk) OM_WAVES_ATTR void k_bounce(OmSceneDev S, OmParamsDev P, Seg G, Gen R, Queue in,
                                                 const uint32_t* __restrict__ count_in, Queue out,
                                                 uint32_t* __restrict__ count_out, float4* __restrict__ res,
                                                 uint32_t* __restrict__ res_id, unsigned long long* __restrict__ counters,
                                                 const float2* __restrict__ hitbuf) {
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    uint32_t n, stride = R.n_pixels;
    uint64_t first0 = seg0;                 // FIRST: the batch's first sample of this workgroup
    if (FIRST) {
        uint64_t paths = (uint64_t)R.n_pixels * R.batch;
        if (R.ad.list) {                    // adaptive: the stream's live list x the planned samples
            const AdPlan pl = uniform_load(R.ad.plan);
            stride = pl.c;
            paths = (uint64_t)pl.c * ad_batch(pl.c, pl.done, R.ad.j, R.ad.A);
            first0 = (uint64_t)blockIdx.x * seg_capacity(paths, G.nseg);
            n = first0 < paths ? (uint32_t)std::min<uint64_t>(seg_capacity(paths, G.nseg), paths - first0) : 0u;
        } else {
            n = seg0 < paths ? (uint32_t)std::min<uint64_t>(G.segcap, paths - seg0) : 0u;
        }
    } else {
        n = count_in[blockIdx.x];
    }
    if (n == 0) {
        if (threadIdx.x == 0) count_out[blockIdx.x] = 0u;
        return;
    }
    __shared__ uint32_t q_next, q_out;
    if (threadIdx.x == 0) { q_next = kBlk / 64u; q_out = 0u; }
    __syncthreads();
    const Tracer T = HIT ? Tracer{} : stage_scene<TR>(S);
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    WorkT<COUNT> w;
    uint32_t segs = 0;
    const uint32_t lane = __lane_id();
    for (uint32_t chunk = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); chunk * 64u < n;) {   // wave-uniform
        const uint32_t jj = chunk * 64u + lane;
        bool keep = false;
        Path p;
        uint32_t p_pixel = 0;
        if (jj < n) {
            const uint64_t i = seg0 + jj;
            bool live = true;
            if (FIRST) {
                live = gen_path(P, R, stride, first0 + jj, p, p_pixel, res_id);
            } else {
                load_ray(in, i, p);
                load_rest(in, i, p);       // issued before the trace: its latency hides behind it
            }
            if (live) {
                float closest;
                int best;
                if (HIT) {
                    const float2 h = hitbuf[i];
                    closest = h.x; best = __float_as_int(h.y);
                } else if (FIRST && (TR == TR_BVH2_LDS || TR == TR_BVH2_GLOBAL) && R.tile_off) {
                    const uint32_t line = p_pixel / P.width;
                    const uint32_t tile = (p_pixel - line * P.width) / 8u + (line / 8u) * P.tiles_x;
                    closest = P.tmax;
                    // a wave within one tile (all but where partial tiles meet) reads its list
                    // and records with scalar loads
                    const uint32_t t0 = __builtin_amdgcn_readfirstlane(tile);
                    if (__ballot(tile != t0) == 0)
                        best = traced_tiles<true>(S, R.tile_off, R.tile_idx, t0, p.o, p.d, P.tmin, closest, w, R.tile_tnear);
                    else
                        best = traced_tiles(S, R.tile_off, R.tile_idx, tile, p.o, p.d, P.tmin, closest, w);
                    if (MARCH) {
                        float tm;
                        const int mg = march(S, p.o, p.d, P.tmin, P.tmax, closest, P.march_steps, tm, w);
                        if (mg >= 0) { best = mg; closest = tm; }
                    }
                } else {
                    best = trace<TR, MARCH>(S, P, T, p.o, p.d, closest, w);
                }
                keep = shade_path<MARCH, USER>(S, P, depth_cap, p, closest, best, res, res_id);
                if (COUNT) segs++;
            }
        }
        const uint64_t m = __ballot(keep);
        uint32_t obase = 0u, nc = 0u;
        if (lane == 0) {
            obase = m ? atomicAdd(&q_out, (uint32_t)__popcll(m)) : 0u;
            nc = atomicAdd(&q_next, 1u);
        }
        obase = __builtin_amdgcn_readfirstlane(obase);
        chunk = __builtin_amdgcn_readfirstlane(nc);
        if (keep) store_path(out, seg0 + obase + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), p);
    }
    __syncthreads();
    if (threadIdx.x == 0) count_out[blockIdx.x] = q_out;
    if (COUNT) {
        flush_counter(counters, OMC_SEGMENTS, segs);
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- split march pipeline
// k_raygen: the camera samples [s*segcap, (s+1)*segcap) of the batch; the taken ones are
// compacted into segment s of `out` (bounce 0 of the split pipeline reads them from there).
template <bool COUNT>
__global__ __launch_bounds__(kBlk) OM_WAVES_ATTR void k_raygen(OmParamsDev P, Seg G, Gen R, Queue out,
                                                 uint32_t* __restrict__ count_out, uint32_t* __restrict__ res_id) {
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    uint64_t paths = (uint64_t)R.n_pixels * R.batch, first0 = seg0;
    uint32_t n, stride = R.n_pixels;
    if (R.ad.list) {                        // adaptive: the stream's live list x the planned samples
        const AdPlan pl = uniform_load(R.ad.plan);
        stride = pl.c;
        paths = (uint64_t)pl.c * ad_batch(pl.c, pl.done, R.ad.j, R.ad.A);
        first0 = (uint64_t)blockIdx.x * seg_capacity(paths, G.nseg);
        n = first0 < paths ? (uint32_t)std::min<uint64_t>(seg_capacity(paths, G.nseg), paths - first0) : 0u;
    } else {
        n = seg0 < paths ? (uint32_t)std::min<uint64_t>(G.segcap, paths - seg0) : 0u;
    }
    __shared__ uint32_t q_out;
    if (threadIdx.x == 0) q_out = 0u;
    __syncthreads();
    const uint32_t lane = __lane_id();
    for (uint32_t base = 0; base < n; base += kBlk) {
        const uint32_t jj = base + threadIdx.x;
        Path p;
        uint32_t pixel;
        const bool keep = jj < n && gen_path(P, R, stride, first0 + jj, p, pixel, res_id);
        const uint64_t m = __ballot(keep);
        uint32_t obase = 0u;
        if (lane == 0 && m) obase = atomicAdd(&q_out, (uint32_t)__popcll(m));
        obase = __builtin_amdgcn_readfirstlane(obase);
        if (keep) store_path(out, seg0 + obase + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), p);
    }
    __syncthreads();
    if (threadIdx.x == 0) count_out[blockIdx.x] = q_out;
}

// k_march: closest traced hit + unstuck + sphere tracing (hits.rs:270-365) of every path of
// segment s of `in`, with LANE REFILL: a lane whose march ends writes (closest, winner) to
// hit[slot] and waits until OM_WF_REFILL lanes of its wave are idle; they then take the
// segment's next paths together (wave-aggregated LDS counter).  The wave's march iterations
// are then no longer the max over 64 paths' step counts.
template <int TR, bool COUNT, class M, class Wk>
__device__ __forceinline__ void march_lanes(const OmSceneDev& S, const OmParamsDev& P, const Tracer& T, const M& m,
                                            const Queue& in, uint64_t seg0, uint32_t n, uint32_t& next,
                                            float2* __restrict__ hit, Wk& w) {
    const uint32_t lane = __lane_id();
    uint32_t j = threadIdx.x;
    bool act = j < n, marching = false;
    bool dry = !act;                                   // the segment has no path left for this lane
    F3 o = f3(0.0f, 0.0f, 0.0f), d = o;
    float t = 0.0f, closest = 0.0f;
    int best = -1;
    uint32_t iters = 0;
    auto start = [&]() {
        const float4 a = in.q0[seg0 + j], b = in.q1[seg0 + j];
        o = f3(a.x, a.y, a.z); d = f3(b.x, b.y, b.z);
        best = trace<TR, false>(S, P, T, o, d, closest, w);
        marching = march_begin(m, o, d, P.tmin, t);
        iters = P.march_steps;
    };
    if (act) start();
    for (;;) {
#pragma unroll
        for (int u = 0; u < OM_MARCH_UNROLL; ++u) {     // march steps between refill checks
            if (act) {
                int gi = -1;
                const int r = marching ? march_step(S, m, o, d, P.tmax, closest, t, iters, gi, w) : 2;
                if (r != 0) {
                    if (r == 1) { best = gi; closest = t; }
                    hit[seg0 + j] = make_float2(closest, __int_as_float(best));
                    act = false;
                }
            }
        }
        // refill the idle lanes together once enough of them wait (or nothing else runs):
        // a refill runs the trace and unstuck, which costs several march steps
        const uint64_t want = __ballot(!act && !dry), busy = __ballot(act);
        if (want && (__popcll(want) >= OM_WF_REFILL || busy == 0)) {
            uint32_t base = 0u;
            if (lane == 0) base = atomicAdd(&next, (uint32_t)__popcll(want));
            base = __builtin_amdgcn_readfirstlane(base);
            if (!act && !dry) {
                j = base + (uint32_t)__popcll(want & ((1ull << lane) - 1ull));
                if (j < n) { act = true; start(); } else dry = true;
            }
        }
        if (__ballot(act) == 0) break;
    }
}

template <int TR, bool COUNT, int VIEW>
__global__ __launch_bounds__(kBlk) OM_WAVES_ATTR void k_march(OmSceneDev S, OmParamsDev P, Seg G, Queue in,
                                                const uint32_t* __restrict__ count_in, float2* __restrict__ hit,
                                                unsigned long long* __restrict__ counters) {
    const uint32_t n = count_in[blockIdx.x];
    if (n == 0) return;
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    __shared__ uint32_t next;
    if (threadIdx.x == 0) next = kBlk;
    __syncthreads();
    const Tracer T = stage_scene<TR>(S);
    WorkT<COUNT> w;
    if constexpr (VIEW == MV_EXACT_C2_LDS) {
        __shared__ MarchedC2Lds::Block mblock;
        march_lanes<TR, COUNT>(S, P, T, MarchedC2Lds(S, &mblock), in, seg0, n, next, hit, w);
    } else {
        march_lanes<TR, COUNT>(S, P, T, MarchedArrays(S), in, seg0, n, next, hit, w);
    }
    if (COUNT) {
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- tail
// Workgroup b: every path of segments [b*kTailSpb, (b+1)*kTailSpb) of queue `in`, each run to
// completion.  Lanes are refilled from an LDS counter as their paths end, in a single loop:
//   traced worlds  one segment (trace + shade) per iteration; a lane whose path ended takes the
//                  next path at once, so it never waits for the longest path of its wave (a
//                  nested per-path loop holds every finished lane until the whole wave leaves it);
//   marched worlds the k_march scheme (march_lanes) inside the tail: OM_MARCH_UNROLL march steps
//                  per iteration, a lane whose march ended shades and starts its next segment,
//                  lanes whose path ended are refilled together once OM_WF_REFILL of them wait.
// (r04: C2 +8.3% over the r03 nested loop, in which every lane ran its path to completion before
// it took another; C1 and C3 within 0.3%.)
struct TailSrc {
    const Queue& in;
    const uint32_t* pre;
    uint32_t s0, segcap;
    __device__ __forceinline__ bool load(uint32_t idx, Path& p) const {
        uint32_t k = 0;
        while (idx >= pre[k + 1]) ++k;
        const uint64_t i = (uint64_t)(s0 + k) * segcap + (idx - pre[k]);
        load_ray(in, i, p);
        load_rest(in, i, p);
        return true;                                        // (a queued path is always live)
    }
};
template <int TR, bool COUNT, class M, class Src, class Wk>
__device__ __forceinline__ uint32_t tail_march_lanes(const OmSceneDev& S, const OmParamsDev& P, const Tracer& T, const M& m,
                                                     const Src& src, uint32_t total, uint32_t& next,
                                                     float4* __restrict__ res, uint32_t* __restrict__ res_id, Wk& w) {
    const uint32_t lane = __lane_id();
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    uint32_t idx = threadIdx.x, segs = 0, iters = 0;
    bool have = idx < total, dry = !have, marching = false, act = false;
    // The march steps need only the ray; the rest of the path (throughput, first hit, segment,
    // slot, RNG) is parked in LDS until the next shade (18 KB per workgroup), so it does not sit
    // in registers across the march loop: C2's tail spilled 40 B per lane with it in registers,
    // 12 B parked (C2 3301 vs 3275 Msamples/s, r04_ab8).
    __shared__ uint32_t rest[9][kBlk];
    Path p;
    float t = 0.0f, closest = 0.0f;
    int best = -1;
    auto park = [&]() {
        const uint32_t i = threadIdx.x;
        rest[0][i] = __float_as_uint(p.cur.x); rest[1][i] = __float_as_uint(p.cur.y); rest[2][i] = __float_as_uint(p.cur.z);
        rest[3][i] = __float_as_uint(p.depthf); rest[4][i] = p.first_id; rest[5][i] = p.seg; rest[6][i] = p.slot;
        rest[7][i] = p.g.s; rest[8][i] = p.g.k;
    };
    auto unpark = [&]() {
        const uint32_t i = threadIdx.x;
        p.cur = f3(__uint_as_float(rest[0][i]), __uint_as_float(rest[1][i]), __uint_as_float(rest[2][i]));
        p.depthf = __uint_as_float(rest[3][i]); p.first_id = rest[4][i]; p.seg = rest[5][i]; p.slot = rest[6][i];
        p.g.s = rest[7][i]; p.g.k = rest[8][i];
    };
    auto begin = [&]() {                                    // closest traced hit + unstuck of the segment
        park();
        best = trace<TR, false>(S, P, T, p.o, p.d, closest, w);
        marching = march_begin(m, p.o, p.d, P.tmin, t);
        iters = P.march_steps;
        act = true;
    };
    if (have) { have = src.load(idx, p); if (have) begin(); }
    for (;;) {
#pragma unroll
        for (int u = 0; u < OM_WF_TAIL_UNROLL; ++u) {         // march steps between checks
            if (act) {
                int gi = -1;
                const int r = marching ? march_step(S, m, p.o, p.d, P.tmax, closest, t, iters, gi, w) : 2;
                if (r != 0) {
                    if (r == 1) { best = gi; closest = t; }
                    act = false;
                }
            }
        }
        // march ended: handle_hit, next segment or done -- for the wave's ended lanes together, once
        // OM_WF_TAIL_SHADE of them wait or none marches
        // (the ballots are taken before the branch, with every lane active: inside it only the
        // ended lanes run, whose act is false, so a ballot of act there would always be 0)
        const bool ended = have && !act;
        const uint64_t em = __ballot(ended), am = __ballot(act);
        if (ended && (OM_WF_TAIL_SHADE <= 1 || __popcll(em) >= OM_WF_TAIL_SHADE || am == 0)) {
            if (COUNT) segs++;
            unpark();
            if (shade_path<true, M::USER>(S, P, depth_cap, p, closest, best, res, res_id)) begin();
            else have = false;
        }
        const uint64_t want = __ballot(!have && !dry), busy = __ballot(have);
        if (want && (__popcll(want) >= OM_WF_TAIL_REFILL || busy == 0)) {
            uint32_t base = 0u;
            if (lane == 0) base = atomicAdd(&next, (uint32_t)__popcll(want));
            base = __builtin_amdgcn_readfirstlane(base);
            if (!have && !dry) {
                idx = base + (uint32_t)__popcll(want & ((1ull << lane) - 1ull));
                if (idx < total) { have = src.load(idx, p); if (have) begin(); } else dry = true;
            }
        }
        if (__ballot(have || !dry) == 0) break;             // (a lane not dry is refilled next time round)
    }
    return segs;
}

template <int TR, bool COUNT, bool MARCH, int VIEW = MV_ARRAYS, uint32_t SPB = kTailSpb>
__global__ __launch_bounds__(kBlk) __attribute__((amdgpu_waves_per_eu(MARCH ? OM_WF_TAIL_MARCH_WAVES : OM_WF_WAVES,
                                                                      MARCH ? OM_WF_TAIL_MARCH_WAVES : OM_WF_WAVES)))
void k_tail(OmSceneDev S, OmParamsDev P, Seg G, Queue in,
                                               const uint32_t* __restrict__ count_in, float4* __restrict__ res,
                                               uint32_t* __restrict__ res_id, unsigned long long* __restrict__ counters) {
    __shared__ uint32_t pre[SPB + 1];
    __shared__ uint32_t next;
    const uint32_t s0 = blockIdx.x * SPB;
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t k = 0; k < SPB; ++k) {
            pre[k] = acc;
            acc += s0 + k < G.nseg ? count_in[s0 + k] : 0u;
        }
        pre[SPB] = acc;
        next = kBlk;
    }
    __syncthreads();
    const uint32_t total = pre[SPB];
    if (total == 0) return;
    const Tracer T = stage_scene<TR>(S);
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    const TailSrc src{in, pre, s0, G.segcap};
    WorkT<COUNT> w;
    uint32_t segs = 0;
    if constexpr (MARCH) {
        if constexpr (VIEW == MV_EXACT_C2_LDS) {
            __shared__ MarchedC2Lds::Block mblock;
            segs = tail_march_lanes<TR, COUNT>(S, P, T, MarchedC2Lds(S, &mblock), src, total, next, res, res_id, w);
        } else {
            segs = tail_march_lanes<TR, COUNT>(S, P, T, MarchedArrays(S), src, total, next, res, res_id, w);
        }
    } else {
        uint32_t idx = threadIdx.x;
        bool have = idx < total;
        Path p;
        if (have) src.load(idx, p);
        for (;;) {
            if (have) {
                float closest;
                const int best = trace<TR, false>(S, P, T, p.o, p.d, closest, w);
                if (COUNT) segs++;
                if (!shade_path<false>(S, P, depth_cap, p, closest, best, res, res_id)) {
                    idx = atomicAdd(&next, 1u);                 // the path ended: the next one at once
                    have = idx < total;
                    if (have) src.load(idx, p);
                }
            }
            if (__ballot(have) == 0) break;
        }
    }
    if (COUNT) {
        flush_counter(counters, OMC_SEGMENTS, segs);
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- accumulate
// Adaptive batches (ad.list): lane kk owns live-list entry kk, and a pixel that is still live after
// the batch, with samples of the call left, is appended to the stream's next list (one ballot and
// one atomic per workgroup: ThreadPixels::add_run / swap_buffers, render_thread.rs:68-102).  The list's
// order then depends on which wave appends first; a result's slot and a path's RNG never do.
template <bool COUNT>
__global__ __launch_bounds__(kBlk) void k_accumulate(OmParamsDev P, om_pixel_stats* __restrict__ stats,
                                                     const uint32_t* __restrict__ pixels, uint32_t n_pixels, uint32_t by_pixel,
                                                     uint32_t batch, const float4* __restrict__ res,
                                                     const uint32_t* __restrict__ res_id, const uint64_t* __restrict__ bloom,
                                                     AdList ad, unsigned long long* __restrict__ counters) {
    const uint32_t kk = blockIdx.x * kBlk + threadIdx.x;
    uint32_t n_samples = 0, credited = 0;
    uint32_t done0 = 0;
    if (ad.list) {
        const AdPlan pl = uniform_load(ad.plan);
        n_pixels = pl.c;
        batch = ad_batch(pl.c, pl.done, ad.j, ad.A);
        done0 = pl.done;
        if (kk == 0) ad.plan_next->done = pl.done + batch;
    }
    bool relist = false;
    uint32_t k = kk;
    if (kk < n_pixels) {
        if (ad.list) k = ad.list[kk];
        const uint32_t slot = by_pixel ? pixels[k] : k;
        const om_pixel_stats in = stats[slot];
        PixelState st;
        st.bloom = in.bloom; st.sx = in.sum[0]; st.sy = in.sum[1]; st.sz = in.sum[2]; st.n = in.n;
        st.avg_depth = in.avg_depth; st.bad = in.bad_avgs;
        st.rgbf = (uint32_t)in.color[0] | ((uint32_t)in.color[1] << 8) | ((uint32_t)in.color[2] << 16) | ((uint32_t)in.flags << 24);
        // the loads of OM_ACC_GROUP samples are issued together (ids, then results and bloom
        // words), then added in sample order: one lane's samples no longer cost a chain of
        // dependent global round trips each (r03: 0.2-0.85 ms per 1080p x 16-spp launch before)
        bool retired = P.adaptive && (st.rgbf & 0x01000000u);          // retired before the batch: no loads
        for (uint32_t s0 = 0; s0 < batch && !retired; s0 += OM_ACC_GROUP) {
            const uint32_t m = batch - s0 < OM_ACC_GROUP ? batch - s0 : OM_ACC_GROUP;
            uint32_t id[OM_ACC_GROUP];
            float4 rr[OM_ACC_GROUP];
            uint64_t bl[OM_ACC_GROUP];
#pragma unroll
            for (uint32_t j = 0; j < OM_ACC_GROUP; ++j) id[j] = j < m ? res_id[(uint64_t)(s0 + j) * n_pixels + kk] : kNoSample;
#pragma unroll
            for (uint32_t j = 0; j < OM_ACC_GROUP; ++j) {
                if (j < m) rr[j] = res[(uint64_t)(s0 + j) * n_pixels + kk];
                bl[j] = bloom[id[j] == kNoSample ? 0u : id[j]];
            }
#pragma unroll
            for (uint32_t j = 0; j < OM_ACC_GROUP; ++j) {                  // sample order == reference order
                if (j >= m) break;
                // adaptive batches of several samples: a pixel that retires at sample j takes no more
                // (ThreadPixels::add_run, render_thread.rs:68-102); the batch's later samples of it
                // were rendered speculatively and are dropped here
                if (P.adaptive && (st.rgbf & 0x01000000u)) { retired = true; break; }
                if (id[j] == kNoSample) continue;
                const bool done = stats_add(st, f3(rr[j].x, rr[j].y, rr[j].z), rr[j].w, bl[j]);
                if (COUNT) n_samples++;
                credited += ((done && P.adaptive) ? (P.spp_total - st.n) : 0u) + 1u;   // render_thread.rs:196-198
            }
        }
        om_pixel_stats out;
        out.bloom = st.bloom; out.sum[0] = st.sx; out.sum[1] = st.sy; out.sum[2] = st.sz; out.n = st.n;
        out.avg_depth = st.avg_depth; out.bad_avgs = st.bad;
        out.color[0] = (uint8_t)(st.rgbf & 0xFFu); out.color[1] = (uint8_t)((st.rgbf >> 8) & 0xFFu);
        out.color[2] = (uint8_t)((st.rgbf >> 16) & 0xFFu); out.flags = (uint8_t)(st.rgbf >> 24); out.reserved = 0u;
        stats[slot] = out;
        relist = ad.list && !(st.rgbf & 0x01000000u) && st.n < P.spp_total && done0 + batch < ad.A.sample_count;
    }
    if (ad.list) {                                                  // the stream's next live list
        const uint64_t m = __ballot(relist);
        uint32_t base = 0u;
        // one global atomic per workgroup (the waves' counts summed in LDS first): the ~16k
        // contended atomics on one word of a 1M-pixel accumulate become ~2k (r06: C1_adaptive
        // +3.8%, profiles/r06_adaptive)
        __shared__ uint32_t wg_n, wg_base;
        if (threadIdx.x == 0) wg_n = 0u;
        __syncthreads();
        if (__lane_id() == 0 && m) base = atomicAdd(&wg_n, (uint32_t)__popcll(m));
        __syncthreads();
        if (threadIdx.x == 0) wg_base = wg_n ? atomicAdd(&ad.plan_next->c, wg_n) : 0u;
        __syncthreads();
        base = __builtin_amdgcn_readfirstlane(base) + wg_base;
        if (relist) ad.list_next[base + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull))] = k;
    }
    if (COUNT) {
        flush_counter(counters, OMC_SAMPLES, n_samples);
        flush_counter(counters, OMC_CREDITED, credited);
    }
    if (P.progress) {                                               // live samples_atom (om_progress)
        // summed per workgroup first: one contended atomic per workgroup, not per wave
        __shared__ unsigned long long wg_credit;
        if (threadIdx.x == 0) wg_credit = 0ull;
        __syncthreads();
        const uint32_t v = wave_sum32(credited);
        if (__lane_id() == 0 && v) atomicAdd(&wg_credit, (unsigned long long)v);
        __syncthreads();
        if (threadIdx.x == 0 && wg_credit) atomicAdd(&counters[OMC_PROGRESS], wg_credit);
    }
}

// k_snapshot: n0[k] = Stats.n of listed pixel k at the start of a concurrent fixed-spp call.
__global__ __launch_bounds__(256) void k_snapshot(const om_pixel_stats* __restrict__ stats, const uint32_t* __restrict__ pixels,
                                                  uint32_t n_pixels, uint32_t by_pixel, uint32_t* __restrict__ n0) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k >= n_pixels) return;
    n0[k] = stats[by_pixel ? pixels[k] : k].n;
}

// k_ad_init: the first live list of every stream of an adaptive call.  Chunk q of 64 list entries
// (a tile of a frame list) belongs to stream q % ns; its pixels that are not retired and have
// samples left are appended to that stream's list (one ballot per wave, one atomic per workgroup and stream: a wave is one
// chunk).  plans (zeroed by the caller) get the counts.
constexpr uint32_t kAdInitBlk = 1024u;
__global__ __launch_bounds__(kAdInitBlk) void k_ad_init(const om_pixel_stats* __restrict__ stats, const uint32_t* __restrict__ pixels,
                                                 uint32_t n_pixels, uint32_t by_pixel, uint32_t spp_total, uint32_t ns,
                                                 uint32_t* __restrict__ lists, uint64_t list_stride, AdPlan* __restrict__ plans,
                                                 uint32_t plan_stride) {
    const uint32_t k = blockIdx.x * kAdInitBlk + threadIdx.x;
    bool live = false;
    if (k < n_pixels) {
        const om_pixel_stats& ps = stats[by_pixel ? pixels[k] : k];
        live = !(ps.flags & 1u) && ps.n < spp_total;
    }
    const uint32_t s = (k >> 6) % ns;                                // wave-uniform
    const uint64_t m = __ballot(live);
    uint32_t base = 0u;
    // per stream, one global atomic per workgroup (the waves' counts summed in LDS first)
    __shared__ uint32_t wg_n[4], wg_base[4];
    if (threadIdx.x < 4u) wg_n[threadIdx.x] = 0u;
    __syncthreads();
    if (__lane_id() == 0 && m) base = atomicAdd(&wg_n[s], (uint32_t)__popcll(m));
    __syncthreads();
    if (threadIdx.x < ns && wg_n[threadIdx.x])
        wg_base[threadIdx.x] = atomicAdd(&plans[(uint64_t)threadIdx.x * plan_stride].c, wg_n[threadIdx.x]);
    __syncthreads();
    base = __builtin_amdgcn_readfirstlane(base) + (m ? wg_base[s] : 0u);
    if (live) lists[s * list_stride + base + (uint32_t)__popcll(m & ((1ull << __lane_id()) - 1ull))] = k;
}

hipError_t grow(Buffers& B, uint64_t cap, uint32_t counts_n, int nsets) {
    hipError_t e;
    if (cap > B.cap || nsets > B.nsets) {
        for (auto& s : B.set) s.release();
        B.cap = 0; B.nsets = 0; B.counts_n = 0;
        for (int k = 0; k < nsets; ++k) {
            QueueSet& S = B.set[k];
            for (int a = 0; a < 2; ++a) {
                for (int b = 0; b < 3; ++b) if ((e = hipMalloc(&S.q[a][b], cap * sizeof(float4))) != hipSuccess) return e;
                if ((e = hipMalloc(&S.qr[a], cap * sizeof(uint4))) != hipSuccess) return e;
            }
            if ((e = hipMalloc(&S.res, cap * sizeof(float4))) != hipSuccess) return e;
            if ((e = hipMalloc(&S.res_id, cap * sizeof(uint32_t))) != hipSuccess) return e;
            if ((e = hipMalloc(&S.hit, cap * sizeof(float2))) != hipSuccess) return e;
        }
        B.cap = cap; B.nsets = nsets;
    }
    if (counts_n > B.counts_n) {
        for (int k = 0; k < B.nsets; ++k) {
            QueueSet& S = B.set[k];
            if (S.counts) (void)hipFree(S.counts);
            S.counts = nullptr;
            if ((e = hipMalloc(&S.counts, (size_t)counts_n * sizeof(uint32_t))) != hipSuccess) return e;
        }
        B.counts_n = counts_n;
    }
    return hipSuccess;
}

Queue queue(QueueSet& B, int k) { return Queue{B.q[k][0], B.q[k][1], B.q[k][2], B.qr[k]}; }

// One batch: bounce 0 .. tail_at-1 as per-bounce launches, then the tail launch, all on `st`;
// returns the number of bounce-family launches.
template <int TR, bool COUNT, bool MARCH>
uint32_t run_batch(QueueSet& B, const Launch& L, hipStream_t st, Seg G, const Gen& R, uint32_t depth_cap,
                   uint32_t tail_at, uint32_t lds) {
    Timer& tm = *L.timer;
    const bool each = tm.mode == 1;
    uint32_t launches = 0;
    const bool exact = MARCH && L.S.n_msdf == 0u && MarchedC2Lds::matches(L.S.n_msph, L.S.n_mbox, L.S.n_mtor);
    auto tail = [&](const Queue& in, const uint32_t* cin) {
        const int ti = each ? tm.begin(st) : -1;
        const uint32_t grid = (G.nseg + kTailSpb - 1u) / kTailSpb;
        if (exact && exact_view_built<TR>())
            hipLaunchKernelGGL((k_tail<TR, COUNT, MARCH, MARCH && exact_view_built<TR>() ? MV_EXACT_C2_LDS : MV_ARRAYS>), dim3(grid),
                               dim3(kBlk), lds, st, L.S, L.P, G, in, cin, B.res, B.res_id, L.counters);
        else
            hipLaunchKernelGGL((k_tail<TR, COUNT, MARCH>), dim3(grid), dim3(kBlk), lds, st, L.S, L.P, G, in, cin,
                               B.res, B.res_id, L.counters);
        tm.end(ti, OM_KT_TAIL, st);
        return launches + 1u;
    };
    if constexpr (MARCH) {
        // split march pipeline: k_raygen compacts the camera paths into queue 0;
        // per bounce, the lane-refilling k_march writes every path's (closest, winner) to the hit
        // buffer and k_bounce<HIT> shades and compacts
        {
            const int ti = each ? tm.begin(st) : -1;
            hipLaunchKernelGGL((k_raygen<COUNT>), dim3(G.nseg), dim3(kBlk), 0, st, L.P, G, R, queue(B, 0), B.counts, B.res_id);
            tm.end(ti, OM_KT_BOUNCE0, st);
            ++launches;
        }
        for (uint32_t bounce = 0; bounce < depth_cap; ++bounce) {
            const Queue in = queue(B, bounce & 1u), out = queue(B, (bounce + 1u) & 1u);
            const uint32_t* cin = B.counts + (size_t)bounce * G.nseg;
            if (bounce >= tail_at) return tail(in, cin);   // (tail_at 0: k_raygen's camera paths too)
            uint32_t* cout = B.counts + (size_t)(bounce + 1u) * G.nseg;
            const int kc = bounce == 0 ? OM_KT_BOUNCE0 : OM_KT_BOUNCE;
            int ti = each ? tm.begin(st) : -1;
            if (exact && exact_view_built<TR>())
                hipLaunchKernelGGL((k_march<TR, COUNT, exact_view_built<TR>() ? MV_EXACT_C2_LDS : MV_ARRAYS>), dim3(G.nseg),
                                   dim3(kBlk), lds, st, L.S, L.P, G, in, cin, B.hit, L.counters);
            else
                hipLaunchKernelGGL((k_march<TR, COUNT, MV_ARRAYS>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, in, cin,
                                   B.hit, L.counters);
            tm.end(ti, kc, st);
            ti = each ? tm.begin(st) : -1;
            if (exact && exact_view_built<TR>())                       // no user objects (OmMSdf) in the world
                hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, false, true, false>), dim3(G.nseg), dim3(kBlk), 0, st, L.S, L.P, G,
                                   R, in, cin, out, cout, B.res, B.res_id, L.counters, (const float2*)B.hit);
            else
                hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, false, true>), dim3(G.nseg), dim3(kBlk), 0, st, L.S, L.P, G, R, in,
                                   cin, out, cout, B.res, B.res_id, L.counters, (const float2*)B.hit);
            tm.end(ti, kc, st);
            launches += 2u;
        }
        return launches;
    } else {
    for (uint32_t bounce = 0; bounce < depth_cap; ++bounce) {
        const Queue in = queue(B, bounce & 1u), out = queue(B, (bounce + 1u) & 1u);
        const uint32_t* cin = B.counts + (size_t)bounce * G.nseg;
        if (bounce > 0 && bounce >= tail_at) return tail(in, cin);
        uint32_t* cout = B.counts + (size_t)(bounce + 1u) * G.nseg;
        const int ti = each ? tm.begin(st) : -1;
        if (bounce == 0)
            hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, true>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, R, in,
                               cin, out, cout, B.res, B.res_id, L.counters, (const float2*)nullptr);
        else
            hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, false>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, R, in,
                               cin, out, cout, B.res, B.res_id, L.counters, (const float2*)nullptr);
        tm.end(ti, bounce == 0 ? OM_KT_BOUNCE0 : OM_KT_BOUNCE, st);
        ++launches;
    }
    return launches;
    }
}

template <int TR>
uint32_t run_tr(bool count, bool march, QueueSet& B, const Launch& L, hipStream_t st, Seg G, const Gen& R,
                uint32_t depth_cap, uint32_t tail_at, uint32_t lds) {
    if (count && march) return run_batch<TR, true, true>(B, L, st, G, R, depth_cap, tail_at, lds);
    if (count) return run_batch<TR, true, false>(B, L, st, G, R, depth_cap, tail_at, lds);
    if (march) return run_batch<TR, false, true>(B, L, st, G, R, depth_cap, tail_at, lds);
    return run_batch<TR, false, false>(B, L, st, G, R, depth_cap, tail_at, lds);
}

hipError_t ensure_events(Buffers& B, size_t n) {
    while (B.ev.size() < n) {
        hipEvent_t e = nullptr;
        const hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) return r;
        B.ev.push_back(e);
    }
    return hipSuccess;
}

}  // namespace

// Schedules:
//   fixed spp, serial      (L.streams == 1) one batch after another on `st`.
//   fixed spp, concurrent  (default) the call's samples split into batches of at most half the
//               call, dealt round-robin to L.streams streams (`st` + side streams), each with its
//               own queue set: two batches are in flight at once, so one batch's latency-bound
//               phases (the drain of every launch, the late bounces, the tail) run beside the
//               other's full ones.  Sample indices come from the call-start Stats.n snapshot (n0).
//   adaptive    the listed pixels are dealt to the streams by 64-entry chunks; each stream runs
//               up to ad_batches batches over ITS live pixels, from a live list its own
//               k_accumulate compacts, with the batch's sample count planned on the device from
//               the live count (ad_batch): nothing is rendered for a retired pixel, and samples
//               past a retirement inside a batch are dropped in sample order by k_accumulate.
// In both concurrent forms the accumulates run in batch order through events (acc i after
// acc i-1) and the call ends joined on `st`.
// Timing: mode 2 brackets the call once on `st` (OM_KT_BOUNCE_SPAN, with the call's
// bounce-family launch count); mode 1 brackets every launch on its stream and the call.
hipError_t render(Buffers& B, const Launch& L, hipStream_t st, std::string& err) {
    const uint32_t n_px = L.n_pixels;
    if (n_px == 0 || L.P.sample_count == 0) return hipSuccess;
    const bool adaptive = L.P.adaptive != 0u;
    const uint32_t want = std::max<uint32_t>(1u, std::min<uint32_t>(L.streams, (uint32_t)kMaxSets));
    // fixed spp: paths per batch 2^25 (33.5M, ~4.9 GB of queues per set; 16 spp of 1080p, the
    // measured sweet spot, §5.5), raised up to 16 spp of the frame for frames above 2M pixels,
    // within 2^27 (~21 GB per set, two sets; MI355X has 288 GB): a 4K frame (C4, 8.3M pixels) then
    // runs 16-spp batches like 1080p instead of 4-spp ones, whose 4x launches and 4x Stats
    // read-modify-write per sample cost C4 ~11% in k_accumulate alone (r03)
    const uint64_t kMaxPaths = std::min<uint64_t>(1ull << OM_WF_MAX_PATHS_LOG2,
                                                  std::max<uint64_t>(1ull << OM_WF_MIN_PATHS_LOG2, (uint64_t)OM_WF_BATCH_SPP * n_px));
    uint32_t ns, nb, batch = 0, ad_k = 0, cmax = 0;
    uint64_t max_paths;
    std::vector<uint32_t> done_at(1, 0u);                          // fixed spp: samples of the call before batch i
    AdCfg A{};
    if (adaptive) {
        const uint32_t chunks = (n_px + 63u) / 64u;
        ns = std::min<uint32_t>(want, chunks);
        cmax = std::min<uint32_t>(n_px, (chunks + ns - 1u) / ns * 64u);   // entries of the fullest stream
        // batches per stream: OM_WF_ADAPTIVE_BATCHES, more when the forced even share of a large
        // call would exceed 2^OM_WF_ADAPTIVE_CAP_LOG2 paths
        const uint64_t capmax = 1ull << OM_WF_ADAPTIVE_CAP_LOG2;
        uint64_t k = L.ad_batches ? L.ad_batches : OM_WF_ADAPTIVE_BATCHES;
        while (k < L.P.sample_count && (uint64_t)cmax * ((L.P.sample_count + k - 1u) / k) > capmax) ++k;
        ad_k = (uint32_t)std::min<uint64_t>(k, L.P.sample_count);
        A.sample_count = L.P.sample_count; A.batches = ad_k;
        A.paths = 1u << (L.ad_paths_log2 ? L.ad_paths_log2 : OM_WF_ADAPTIVE_PATHS_LOG2);
        max_paths = std::max<uint64_t>(std::min<uint64_t>(A.paths, (uint64_t)cmax * L.P.sample_count),
                                       (uint64_t)cmax * ((L.P.sample_count + ad_k - 1u) / ad_k));
        nb = ad_k * ns;
    } else {
        const bool concurrent = want >= 2u && L.P.sample_count >= 2u;
        batch = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(L.P.sample_count, kMaxPaths / n_px));
        // at most 1/want of the call per batch, so every call has batches in flight together
        if (concurrent) batch = std::min<uint32_t>(batch, (L.P.sample_count + want - 1u) / want);
        while (done_at.back() < L.P.sample_count)
            done_at.push_back(done_at.back() + std::min(batch, L.P.sample_count - done_at.back()));
        nb = (uint32_t)done_at.size() - 1u;
        ns = concurrent ? std::min<uint32_t>(want, nb) : 1u;
        max_paths = (uint64_t)n_px * batch;
    }
    const uint32_t depth_cap = L.P.max_depth > 1u ? L.P.max_depth : 1u;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int tr = L.trace_mode == TR_SBVH_LDS ? TR_SBVH_GLOBAL : L.trace_mode;
    if (tr == TR_BVH4_LDS) tr = L.S.n_b4nodes == 0 ? TR_BVH2_LDS : (L.S.b4_lds_bytes ? TR_BVH4_LDS : TR_BVH4_GLOBAL);
    // an empty BVH2 (no bounded sphere/cube: marched-only worlds, C2) takes the reference loop
    // when the old BVH holds at most one leaf: TR_BVH's 64-entry stack lives in scratch memory,
    // which every k_march / k_tail wave would then carry for nothing (C2: 1785 vs 1649, r02_v8)
    if (tr == TR_BVH2_LDS)
        tr = L.S.n_b2nodes == 0 ? (L.S.n_bvh_nodes <= 1u ? TR_BRUTE : TR_BVH) : (L.S.b2_lds_bytes ? TR_BVH2_LDS : TR_BVH2_GLOBAL);
    // segments, a multiple of the tail grouping: 4096 lanes per CU (8 workgroups of 512) for
    // traced worlds whose BVH2 sits in LDS, 8192 for marched worlds and L2-resident trees
    const bool march = (L.S.n_msph + L.S.n_mbox + L.S.n_mtor + L.S.n_msdf) != 0u;
    const uint32_t tail_at = L.tail_bounce ? L.tail_bounce
                           : march ? kTailMarched : (tr == TR_BVH2_GLOBAL || tr == TR_BVH4_GLOBAL) ? kTailL2
                           : adaptive ? OM_WF_ADAPTIVE_TAIL
                           : max_paths > (1ull << 25) ? kTailBigBatch : kTailDefault;
    const uint32_t lanes_per_cu = (march || tr == TR_BVH2_GLOBAL || tr == TR_BVH4_GLOBAL) ? OM_WF_LANES_PER_CU_WIDE
                                                                                          : OM_WF_LANES_PER_CU;
    uint32_t nseg = (uint32_t)std::min<uint64_t>((max_paths + kBlk - 1) / kBlk, (uint64_t)cus * (lanes_per_cu / kBlk));
    nseg = (nseg + kTailSpb - 1) / kTailSpb * kTailSpb;
    const uint32_t segcap = seg_capacity(max_paths, nseg);
    hipError_t e = grow(B, (uint64_t)nseg * segcap, (depth_cap + 1u) * nseg, (int)ns);
    if (e != hipSuccess) { err = "wavefront buffer allocation failed"; return e; }
    const uint32_t lds = tr == TR_BVH2_LDS ? stack_bytes<TR_BVH2_LDS>(L.S) + b2_stage_bytes(L.S)
                       : tr == TR_BVH2_GLOBAL ? stack_bytes<TR_BVH2_GLOBAL>(L.S) + hyb_nodes(L.S) * (uint32_t)sizeof(OmBvh2NodeH)
                       : tr == TR_BVH4_LDS ? stack_bytes<TR_BVH4_LDS>(L.S) + L.S.b4_lds_bytes
                       : tr == TR_BVH4_GLOBAL ? stack_bytes<TR_BVH4_GLOBAL>(L.S) + hyb4_nodes(L.S) * (uint32_t)sizeof(OmBvh4NodeH)
                       : 0u;
    Gen R;
    R.C = L.C; R.jitter = L.jitter; R.stats = L.stats; R.pixels = L.pixels; R.n_pixels = n_px;
    R.by_pixel = L.stats_by_pixel ? 1u : 0u;
    R.tile_off = L.tile_off; R.tile_idx = L.tile_idx; R.tile_tnear = L.tile_tnear;
    R.n0 = nullptr; R.done = 0; R.ad = AdList{};
    hipStream_t streams[kMaxSets] = {st, st, st, st};
    Timer& tm = *L.timer;
    const int call_ti = tm.begin(st);
    // device words: fixed spp, the call-start Stats.n snapshot (n0, concurrent calls); adaptive, per
    // stream two live lists (ping-pong) of cmax entries and ad_k + 1 plans
    const uint32_t plan_stride = ad_k + 1u;
    const uint64_t words = adaptive ? (uint64_t)ns * 2u * cmax + (uint64_t)ns * plan_stride * 2u : (ns > 1 ? n_px : 0u);
    if (words > B.n0_cap) {
        if (B.n0) (void)hipFree(B.n0);
        B.n0 = nullptr; B.n0_cap = 0;
        if ((e = hipMalloc(&B.n0, (size_t)words * sizeof(uint32_t))) != hipSuccess) { err = "n0 allocation failed"; return e; }
        B.n0_cap = words;
    }
    uint32_t* lists = B.n0;
    AdPlan* plans = adaptive ? (AdPlan*)(B.n0 + (uint64_t)ns * 2u * cmax) : nullptr;
    if (adaptive) {
        (void)hipMemsetAsync(plans, 0, (size_t)ns * plan_stride * sizeof(AdPlan), st);
        hipLaunchKernelGGL(k_ad_init, dim3((n_px + kAdInitBlk - 1u) / kAdInitBlk), dim3(kAdInitBlk), 0, st, L.stats, L.pixels, n_px, R.by_pixel,
                           L.P.spp_total, ns, lists, (uint64_t)2u * cmax, plans, plan_stride);
    } else if (ns > 1) {
        hipLaunchKernelGGL(k_snapshot, dim3((n_px + 255u) / 256u), dim3(256), 0, st, L.stats, L.pixels, n_px, R.by_pixel, B.n0);
        R.n0 = B.n0;
    }
    // events: [0] call start on `st`, [k] side stream k joined, [kMaxSets + i] batch i accumulated
    if (ns > 1) {
        if ((e = ensure_events(B, kMaxSets + nb)) != hipSuccess) { err = "event creation failed"; return e; }
        (void)hipEventRecord(B.ev[0], st);                       // side streams start after everything before the call
        for (uint32_t k = 1; k < ns; ++k) {
            if (!B.side[k] && (e = hipStreamCreateWithFlags(&B.side[k], hipStreamNonBlocking)) != hipSuccess) {
                err = "side stream creation failed"; return e;
            }
            streams[k] = B.side[k];
            (void)hipStreamWaitEvent(streams[k], B.ev[0], 0);
        }
    }
    uint32_t launches = 0;
    for (uint32_t i = 0; i < nb; ++i) {
        const uint32_t sidx = i % ns;                             // stream (and queue set) of batch i
        hipStream_t si = streams[sidx];
        QueueSet& QS = B.set[sidx];
        Seg G;
        G.nseg = nseg;
        uint32_t b = 0, grid_a;
        AdList ad{};
        if (adaptive) {
            // batch j of stream sidx: its live list and plan, the next ones written by its accumulate
            const uint32_t j = i / ns;
            uint32_t* lbase = lists + (uint64_t)sidx * 2u * cmax;
            ad.list = lbase + (uint64_t)(j & 1u) * cmax;
            ad.list_next = lbase + (uint64_t)((j + 1u) & 1u) * cmax;
            ad.plan = plans + (uint64_t)sidx * plan_stride + j;
            ad.plan_next = plans + (uint64_t)sidx * plan_stride + j + 1u;
            ad.A = A; ad.j = j;
            G.segcap = segcap;                                    // queue capacity of the largest batch
            grid_a = (cmax + kBlk - 1) / kBlk;
        } else {
            const uint32_t done = done_at[i];
            b = done_at[i + 1] - done;
            G.segcap = seg_capacity((uint64_t)n_px * b, nseg);
            R.done = done;
            grid_a = (n_px + kBlk - 1) / kBlk;
        }
        R.batch = b;
        R.ad = ad;
        switch (tr) {
            case TR_BRUTE: launches += run_tr<TR_BRUTE>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            case TR_CULLED: launches += run_tr<TR_CULLED>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            case TR_BVH: launches += run_tr<TR_BVH>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            case TR_SBVH_GLOBAL: launches += run_tr<TR_SBVH_GLOBAL>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            case TR_BVH2_LDS: launches += run_tr<TR_BVH2_LDS>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            case TR_BVH4_LDS: launches += run_tr<TR_BVH4_LDS>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            case TR_BVH4_GLOBAL: launches += run_tr<TR_BVH4_GLOBAL>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
            default: launches += run_tr<TR_BVH2_GLOBAL>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds); break;
        }
        // accumulates in batch order: fixed spp needs it (Stats::add in sample order); an adaptive
        // stream's pixels are its own, so there it only keeps the streams in step and the progress
        // copies in order (unchained streams measured the same: 49.3 vs 49.2 ms per frame, r05_p6)
        if (ns > 1 && i > 0) (void)hipStreamWaitEvent(si, B.ev[kMaxSets + i - 1u], 0);
        const int ati = tm.mode == 1 ? tm.begin(si) : -1;
        if (L.count)
            hipLaunchKernelGGL(k_accumulate<true>, dim3(grid_a), dim3(kBlk), 0, si, L.P, L.stats, L.pixels, n_px,
                               L.stats_by_pixel ? 1u : 0u, b, QS.res, QS.res_id, L.S.bloom, ad, L.counters);
        else
            hipLaunchKernelGGL(k_accumulate<false>, dim3(grid_a), dim3(kBlk), 0, si, L.P, L.stats, L.pixels, n_px,
                               L.stats_by_pixel ? 1u : 0u, b, QS.res, QS.res_id, L.S.bloom, ad, L.counters);
        tm.end(ati, OM_KT_ACCUMULATE, si);
        // live progress: the cumulative credit after this batch, to the host word om_progress
        // hands out; ahead of the event the next batch's accumulate waits on, so the copies
        // land in order and the word only grows
        if (L.progress_host)
            (void)hipMemcpyAsync(L.progress_host, L.counters + OMC_PROGRESS, sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, si);
        if (ns > 1) (void)hipEventRecord(B.ev[kMaxSets + i], si);
        if ((e = hipGetLastError()) != hipSuccess) { err = "wavefront launch failed"; return e; }
    }
    for (uint32_t k = 1; k < ns; ++k) {
        (void)hipEventRecord(B.ev[k], streams[k]);
        (void)hipStreamWaitEvent(st, B.ev[k], 0);
    }
    tm.end(call_ti, OM_KT_BOUNCE_SPAN, st, launches);
    return hipSuccess;
}

}  // namespace omw
