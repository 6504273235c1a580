// om_wavefront.hip — wavefront path tracer: the bounce recursion of
// ray_color (render_thread.rs:128-143) flattened into per-bounce kernels over SoA ray
// queues in HBM:
//
//   raygen      one lane per (sample, pixel): camera ray (render_thread.rs:183-192)
//   intersect   one lane per live ray: closest hit (hits.rs:270-365) -> (t, gi)
//   shade       one lane per live ray: HitRecord + Material::scatter / sky
//               (render_thread.rs:105-126); survivors are compacted into the next
//               queue, finished paths write (colour, depth, id) to their result slot
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

using namespace omd;

namespace omw {

void Buffers::release() {
    for (int a = 0; a < 2; ++a) {
        for (int b = 0; b < 3; ++b) { if (q[a][b]) (void)hipFree(q[a][b]); q[a][b] = nullptr; }
        if (qr[a]) (void)hipFree(qr[a]); qr[a] = nullptr;
    }
    if (hits) (void)hipFree(hits);
    if (res) (void)hipFree(res);
    if (res_id) (void)hipFree(res_id);
    if (counts) (void)hipFree(counts);
    hits = nullptr; res = nullptr; res_id = nullptr; counts = nullptr; cap = 0; counts_n = 0;
}

namespace {

constexpr uint32_t kNoSample = 0xFFFFFFFFu;
enum { TR_BRUTE = 1, TR_CULLED = 2, TR_BVH = 3, TR_SBVH_LDS = 4, TR_SBVH_GLOBAL = 5, TR_BVH2_LDS = 6, TR_BVH2_GLOBAL = 7 };
constexpr int kBlk = 256;          // raygen / shade / intersect workgroup = one queue segment
constexpr int kStackDepth = 24;                                   // BVH2 per-lane LDS stack (u16 entries)
constexpr uint32_t kStackBytes = kBlk * kStackDepth * 2u;         // 12 KiB per 256-lane workgroup
constexpr int kBlkLds = 1024;      // LDS-staged intersect workgroup = kSpbLds segments
constexpr int kSpbLds = kBlkLds / kBlk;

extern __shared__ __attribute__((aligned(16))) uint4 wf_lds[];

// Block-wide stream compaction: returns this lane's rank among the block's keep=true
// lanes (lane order), and the block total.  Every thread of the block must call it.
__device__ __forceinline__ uint32_t block_scan(bool keep, uint32_t& total) {
    __shared__ uint32_t wc[kBlk / 64];
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    const uint64_t m = __ballot(keep);
    const uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wc[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBlk / 64; ++w) {
        const uint32_t c = wc[w];
        off += w < wave ? c : 0u;
        tot += c;
    }
    __syncthreads();
    total = tot;
    return off + pre;
}

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
    uint32_t nseg;    // segments (= shade/raygen workgroups)
    uint32_t segcap;  // rays per segment
};

// ---------------------------------------------------------------- raygen
__global__ __launch_bounds__(kBlk) void k_raygen(OmCamDev C, OmParamsDev P, const float2* __restrict__ jitter,
                                                 const om_pixel_stats* __restrict__ stats, const uint32_t* __restrict__ pixels,
                                                 uint32_t n_pixels, uint32_t by_pixel, uint32_t batch, Seg G,
                                                 float4* __restrict__ q0, float4* __restrict__ q1, float4* __restrict__ q2,
                                                 uint4* __restrict__ qr, uint32_t* __restrict__ count,
                                                 uint32_t* __restrict__ res_id) {
    const uint64_t paths = (uint64_t)n_pixels * batch;
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    const uint64_t end = std::min<uint64_t>(seg0 + G.segcap, paths);
    uint32_t run = 0;
    for (uint64_t base = seg0; base < end; base += kBlk) {
        const uint64_t t = base + threadIdx.x;
        bool ok = false;
        F3 o = f3(0, 0, 0), d = f3(0, 0, 0);
        Rng g; g.s = 0;
        if (t < end) {
            const uint32_t s_local = (uint32_t)(t / n_pixels), k = (uint32_t)(t - (uint64_t)s_local * n_pixels);
            const uint32_t pixel = pixels[k];
            const uint32_t slot = by_pixel ? pixel : k;
            const uint32_t s = stats[slot].n + s_local;
            ok = s < P.spp_total && !(P.adaptive && (stats[slot].flags & 1u));
            res_id[t] = kNoSample;
            if (ok) {
                g = path_rng(P.skey, pixel, s);
                const uint32_t line = pixel / P.width;
                gen_camera_ray(C, P, jitter, (float)(pixel - P.width * line), (float)line, s, g, o, d);
            }
        }
        uint32_t tot;
        const uint32_t j = block_scan(ok, tot);
        if (ok) {
            const uint64_t at_ = seg0 + run + j;
            q0[at_] = make_float4(o.x, o.y, o.z, 0.0f);
            q1[at_] = make_float4(d.x, d.y, d.z, __uint_as_float(0u));
            q2[at_] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(0u));
            qr[at_] = make_uint4((uint32_t)g.s, (uint32_t)(g.s >> 32), (uint32_t)t, 0u);
        }
        run += tot;
    }
    if (threadIdx.x == 0) count[blockIdx.x] = run;
}

// ---------------------------------------------------------------- intersect
// Workgroup b traces segments [b*SPB, b*SPB+SPB).
template <int TR, int BLOCK, bool COUNT, bool MARCH>
__global__ __launch_bounds__(BLOCK) void k_intersect(OmSceneDev S, OmParamsDev P, Seg G, const float4* __restrict__ q0,
                                                     const float4* __restrict__ q1, const uint32_t* __restrict__ count,
                                                     float2* __restrict__ hits, unsigned long long* __restrict__ counters) {
    constexpr uint32_t SPB = BLOCK / kBlk;
    const uint32_t s0 = blockIdx.x * SPB;
    uint32_t work = 0;
    for (uint32_t k = 0; k < SPB && s0 + k < G.nseg; ++k) work += count[s0 + k];
    if (work == 0) return;
    if (TR == TR_BVH2_LDS) {                                      // [stack][nodes][leaf table]
        const uint32_t nn = S.n_b2nodes * 4u;
        const uint4* sn = (const uint4*)S.b2nodes;
        uint4* dst = wf_lds + kStackBytes / 16u;
        for (uint32_t i = threadIdx.x; i < nn; i += BLOCK) dst[i] = sn[i];
        uint32_t* ldst = (uint32_t*)(dst + nn);
        for (uint32_t i = threadIdx.x; i < S.n_b2leaves; i += BLOCK) ldst[i] = S.b2leaves[i];
        __syncthreads();
    }
    uint16_t* stk = (uint16_t*)wf_lds + threadIdx.x;
    const OmBvh2Node* b2_lds = (const OmBvh2Node*)(wf_lds + kStackBytes / 16u);
    const uint32_t* b2_leaves_lds = (const uint32_t*)(wf_lds + kStackBytes / 16u + S.n_b2nodes * 4u);
    if (TR == TR_SBVH_LDS) {
        const uint32_t nn = S.n_snodes * 2u, nr = S.n_srecs * 4u;
        const uint4* sn = (const uint4*)S.snodes;
        const uint4* sr = (const uint4*)S.srecs;
        for (uint32_t i = threadIdx.x; i < nn; i += BLOCK) wf_lds[i] = sn[i];
        for (uint32_t i = threadIdx.x; i < nr; i += BLOCK) wf_lds[nn + i] = sr[i];
        __syncthreads();
    }
    const OmSkipNode* lds_nodes = (const OmSkipNode*)wf_lds;
    const OmAffineTest* lds_recs = (const OmAffineTest*)(wf_lds + S.n_snodes * 2u);
    // MARCH is a compile-time split: the sphere-tracing code (3 SDFs + unstuck) would
    // otherwise set the register budget of every traced-only scene.
    WorkT<COUNT> w;
    for (uint32_t k = 0; k < SPB && s0 + k < G.nseg; ++k) {
        const uint32_t n = count[s0 + k];
        const uint64_t seg0 = (uint64_t)(s0 + k) * G.segcap;
        for (uint32_t j = threadIdx.x; j < n; j += BLOCK) {
            const uint64_t i = seg0 + j;
            const float4 a = q0[i], b = q1[i];
            const F3 o = f3(a.x, a.y, a.z), d = f3(b.x, b.y, b.z);
            float closest = P.tmax;
            int best;
            if (TR == TR_BVH2_LDS) best = traced_bvh2<kStackDepth, BLOCK>(S, b2_lds, b2_leaves_lds, stk, o, d, P.tmin, closest, w);
            else if (TR == TR_BVH2_GLOBAL)
                best = traced_bvh2<kStackDepth, BLOCK>(S, S.b2nodes, S.b2leaves, stk, o, d, P.tmin, closest, w);
            else if (TR == TR_SBVH_LDS) best = traced_sbvh(S, lds_nodes, lds_recs, o, d, P.tmin, closest, w);
            else if (TR == TR_SBVH_GLOBAL) best = traced_sbvh(S, S.snodes, S.srecs, o, d, P.tmin, closest, w);
            else if (TR == TR_BVH) best = traced_bvh(S, o, d, P.tmin, closest, w);
            else best = traced_brute<TR == TR_CULLED>(S, o, d, P.tmin, closest, w);
            if (MARCH) {
                float tm;
                const int mg = march(S, o, d, P.tmin, P.tmax, closest, P.march_steps, tm, w);
                if (mg >= 0) { best = mg; closest = tm; }
            }
            hits[i] = make_float2(closest, __int_as_float(best));
        }
    }
    if (COUNT) {
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- shade
template <bool COUNT>
__global__ __launch_bounds__(kBlk) void k_shade(OmSceneDev S, OmParamsDev P, Seg G,
                                                const float4* __restrict__ i0, const float4* __restrict__ i1,
                                                const float4* __restrict__ i2, const uint4* __restrict__ ir,
                                                const uint32_t* __restrict__ count_in, const float2* __restrict__ hits,
                                                float4* __restrict__ o0, float4* __restrict__ o1, float4* __restrict__ o2,
                                                uint4* __restrict__ orr, uint32_t* __restrict__ count_out,
                                                float4* __restrict__ res, uint32_t* __restrict__ res_id,
                                                unsigned long long* __restrict__ counters) {
    const uint32_t n = count_in[blockIdx.x];
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    uint32_t segs = 0, run = 0;
    for (uint32_t base = 0; base < n; base += kBlk) {
        const uint32_t jj = base + threadIdx.x;
        const bool valid = jj < n;
        const uint64_t i = seg0 + jj;
        bool keep = false;
        float4 a = make_float4(0, 0, 0, 0), b = a, c = a;
        uint4 r = make_uint4(0, 0, 0, 0);
        if (valid) {
            a = i0[i]; b = i1[i]; c = i2[i]; r = ir[i];
            const float2 h = hits[i];
            const int best = __float_as_int(h.y);
            const float closest = h.x;
            F3 o = f3(a.x, a.y, a.z), d = f3(b.x, b.y, b.z), cur = f3(c.x, c.y, c.z);
            float depthf = a.w;
            uint32_t first_id = __float_as_uint(b.w);
            const uint32_t seg = __float_as_uint(c.w);
            Rng g; g.s = ((uint64_t)r.y << 32) | r.x;
            float seg_depth; uint32_t seg_id;
            if (best >= 0) {                                                   // handle_hit, Some(hr)
                F3 point, normal;
                finalize(S, best, o, d, P.tmin, closest, point, normal);
                F3 nd, att;
                scatter(S.mats[best], d, normal, g, nd, att);
                cur = mul(cur, att);
                o = point; d = unit(nd);
                seg_depth = closest; seg_id = (uint32_t)best + 1u;
            } else {                                                           // None: sky (render_thread.rs:118-120)
                const float t = 0.5f * (d.y + 1.0f);
                cur = mul(cur, f3((1.0f - t) + 0.5f * t, (1.0f - t) + 0.7f * t, (1.0f - t) + 1.0f * t));
                seg_depth = INFINITY; seg_id = 0u;
            }
            bool finished = false;
            F3 result = cur;
            float rdepth = 0.0f; uint32_t rid = 0;
            if (seg == 0u) {
                depthf = seg_depth; first_id = seg_id;
                if (isinf(seg_depth)) { finished = true; rdepth = INFINITY; rid = 0u; }       // :133-135
            } else if (isinf(seg_depth)) {
                finished = true; rdepth = depthf; rid = first_id;                         // :138-140
            }
            if (!finished && seg + 1u >= depth_cap) {                                        // :142 -Color::ZERO
                finished = true; result = f3(-0.0f, -0.0f, -0.0f); rdepth = depthf; rid = first_id;
            }
            if (finished) {
                res[r.z] = make_float4(result.x, result.y, result.z, rdepth);
                res_id[r.z] = rid;
            } else {
                keep = true;
                a = make_float4(o.x, o.y, o.z, depthf);
                b = make_float4(d.x, d.y, d.z, __uint_as_float(first_id));
                c = make_float4(cur.x, cur.y, cur.z, __uint_as_float(seg + 1u));
                r = make_uint4((uint32_t)g.s, (uint32_t)(g.s >> 32), r.z, 0u);
            }
            if (COUNT) segs++;
        }
        uint32_t tot;
        const uint32_t j = block_scan(keep, tot);
        if (keep) {
            const uint64_t at_ = seg0 + run + j;
            o0[at_] = a; o1[at_] = b; o2[at_] = c; orr[at_] = r;
        }
        run += tot;
    }
    if (threadIdx.x == 0) count_out[blockIdx.x] = run;
    if (COUNT) flush_counter(counters, OMC_SEGMENTS, segs);
}

// ---------------------------------------------------------------- accumulate
template <bool COUNT>
__global__ __launch_bounds__(kBlk) void k_accumulate(OmParamsDev P, om_pixel_stats* __restrict__ stats,
                                                     const uint32_t* __restrict__ pixels, uint32_t n_pixels, uint32_t by_pixel,
                                                     uint32_t batch, const float4* __restrict__ res,
                                                     const uint32_t* __restrict__ res_id, const uint64_t* __restrict__ bloom,
                                                     unsigned long long* __restrict__ counters) {
    const uint32_t k = blockIdx.x * kBlk + threadIdx.x;
    uint32_t n_samples = 0, credited = 0;
    if (k < n_pixels) {
        const uint32_t slot = by_pixel ? pixels[k] : k;
        const om_pixel_stats in = stats[slot];
        PixelState st;
        st.bloom = in.bloom; st.sx = in.sum[0]; st.sy = in.sum[1]; st.sz = in.sum[2]; st.n = in.n;
        st.avg_depth = in.avg_depth; st.bad = in.bad_avgs;
        st.rgbf = (uint32_t)in.color[0] | ((uint32_t)in.color[1] << 8) | ((uint32_t)in.color[2] << 16) | ((uint32_t)in.flags << 24);
        for (uint32_t s = 0; s < batch; ++s) {                                 // sample order == reference order
            const uint64_t t = (uint64_t)s * n_pixels + k;
            const uint32_t id = res_id[t];
            if (id == kNoSample) continue;
            const float4 rr = res[t];
            const bool done = stats_add(st, f3(rr.x, rr.y, rr.z), rr.w, bloom[id]);
            if (COUNT) {
                n_samples++;
                credited += ((done && P.adaptive) ? (P.spp_total - st.n) : 0u) + 1u;   // render_thread.rs:196-198
            }
        }
        om_pixel_stats out;
        out.bloom = st.bloom; out.sum[0] = st.sx; out.sum[1] = st.sy; out.sum[2] = st.sz; out.n = st.n;
        out.avg_depth = st.avg_depth; out.bad_avgs = st.bad;
        out.color[0] = (uint8_t)(st.rgbf & 0xFFu); out.color[1] = (uint8_t)((st.rgbf >> 8) & 0xFFu);
        out.color[2] = (uint8_t)((st.rgbf >> 16) & 0xFFu); out.flags = (uint8_t)(st.rgbf >> 24); out.reserved = 0u;
        stats[slot] = out;
    }
    if (COUNT) {
        flush_counter(counters, OMC_SAMPLES, n_samples);
        flush_counter(counters, OMC_CREDITED, credited);
    }
}

hipError_t grow(Buffers& B, uint64_t cap, uint32_t counts_n) {
    if (cap > B.cap) {
        uint32_t* cnt = B.counts;
        const uint32_t cn = B.counts_n;
        B.counts = nullptr;
        B.release();
        B.counts = cnt; B.counts_n = cn;
        hipError_t e;
        for (int a = 0; a < 2; ++a) {
            for (int b = 0; b < 3; ++b) if ((e = hipMalloc(&B.q[a][b], cap * sizeof(float4))) != hipSuccess) return e;
            if ((e = hipMalloc(&B.qr[a], cap * sizeof(uint4))) != hipSuccess) return e;
        }
        if ((e = hipMalloc(&B.hits, cap * sizeof(float2))) != hipSuccess) return e;
        if ((e = hipMalloc(&B.res, cap * sizeof(float4))) != hipSuccess) return e;
        if ((e = hipMalloc(&B.res_id, cap * sizeof(uint32_t))) != hipSuccess) return e;
        B.cap = cap;
    }
    if (counts_n > B.counts_n) {
        if (B.counts) (void)hipFree(B.counts);
        B.counts = nullptr;
        hipError_t e = hipMalloc(&B.counts, (size_t)counts_n * sizeof(uint32_t));
        if (e != hipSuccess) return e;
        B.counts_n = counts_n;
    }
    return hipSuccess;
}

template <int TR, int BLOCK>
void launch_intersect(bool count, uint32_t lds, hipStream_t st, const Launch& L, Seg G, const float4* q0,
                      const float4* q1, const uint32_t* cnt, float2* hits) {
    constexpr uint32_t SPB = BLOCK / kBlk;
    const uint32_t grid = (G.nseg + SPB - 1) / SPB;
    const bool march = (L.S.n_msph + L.S.n_mbox + L.S.n_mtor) != 0u;
    if (count && march)
        hipLaunchKernelGGL((k_intersect<TR, BLOCK, true, true>), dim3(grid), dim3(BLOCK), lds, st, L.S, L.P, G, q0, q1, cnt, hits, L.counters);
    else if (count)
        hipLaunchKernelGGL((k_intersect<TR, BLOCK, true, false>), dim3(grid), dim3(BLOCK), lds, st, L.S, L.P, G, q0, q1, cnt, hits, L.counters);
    else if (march)
        hipLaunchKernelGGL((k_intersect<TR, BLOCK, false, true>), dim3(grid), dim3(BLOCK), lds, st, L.S, L.P, G, q0, q1, cnt, hits, L.counters);
    else
        hipLaunchKernelGGL((k_intersect<TR, BLOCK, false, false>), dim3(grid), dim3(BLOCK), lds, st, L.S, L.P, G, q0, q1, cnt, hits, L.counters);
}

}  // namespace

hipError_t render(Buffers& B, const Launch& L, hipStream_t st, std::string& err) {
    const uint32_t n_px = L.n_pixels;
    if (n_px == 0 || L.P.sample_count == 0) return hipSuccess;
    const uint64_t kMaxPaths = 1ull << 25;   // 33.5M paths per batch (~5.3 GB of queues)
    const uint32_t batch = L.P.adaptive ? 1u : (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(L.P.sample_count, kMaxPaths / n_px));
    const uint32_t depth_cap = L.P.max_depth > 1u ? L.P.max_depth : 1u;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t max_paths = (uint64_t)n_px * batch;
    // segments: a multiple of the LDS-intersect grouping, ~16 workgroups per CU
    uint32_t nseg = (uint32_t)std::min<uint64_t>((max_paths + kBlk - 1) / kBlk, (uint64_t)cus * 16u);
    nseg = (nseg + kSpbLds - 1) / kSpbLds * kSpbLds;
    const uint32_t segcap = (uint32_t)((max_paths + nseg - 1) / nseg);
    hipError_t e = grow(B, (uint64_t)nseg * segcap, (depth_cap + 1u) * nseg);
    if (e != hipSuccess) { err = "wavefront buffer allocation failed"; return e; }
    const bool lds_path = L.trace_mode == TR_SBVH_LDS && L.S.lds_bytes;
    int tr = (L.trace_mode == TR_SBVH_LDS && !L.S.lds_bytes) ? TR_SBVH_GLOBAL : L.trace_mode;
    if (tr == TR_BVH2_LDS) tr = L.S.n_b2nodes == 0 ? TR_BVH : (L.S.b2_lds_bytes ? TR_BVH2_LDS : TR_BVH2_GLOBAL);
    for (uint32_t done = 0; done < L.P.sample_count;) {
        const uint32_t b = std::min(batch, L.P.sample_count - done);
        const uint64_t paths = (uint64_t)n_px * b;
        Seg G;
        G.nseg = nseg;
        G.segcap = (uint32_t)((paths + nseg - 1) / nseg);
        hipLaunchKernelGGL(k_raygen, dim3(nseg), dim3(kBlk), 0, st, L.C, L.P, L.jitter, L.stats, L.pixels, n_px,
                           L.stats_by_pixel ? 1u : 0u, b, G, B.q[0][0], B.q[0][1], B.q[0][2], B.qr[0], B.counts, B.res_id);
        int cur = 0;
        for (uint32_t bounce = 0; bounce < depth_cap; ++bounce) {
            const uint32_t* cnt = B.counts + (size_t)bounce * nseg;
            if (lds_path) launch_intersect<TR_SBVH_LDS, kBlkLds>(L.count, L.S.lds_bytes, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            else if (tr == TR_BRUTE) launch_intersect<TR_BRUTE, kBlk>(L.count, 0, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            else if (tr == TR_CULLED) launch_intersect<TR_CULLED, kBlk>(L.count, 0, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            else if (tr == TR_BVH) launch_intersect<TR_BVH, kBlk>(L.count, 0, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            else if (tr == TR_BVH2_LDS)
                launch_intersect<TR_BVH2_LDS, kBlk>(L.count, kStackBytes + L.S.b2_lds_bytes, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            else if (tr == TR_BVH2_GLOBAL)
                launch_intersect<TR_BVH2_GLOBAL, kBlk>(L.count, kStackBytes, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            else launch_intersect<TR_SBVH_GLOBAL, kBlk>(L.count, 0, st, L, G, B.q[cur][0], B.q[cur][1], cnt, B.hits);
            const int nx = 1 - cur;
            uint32_t* cnt_out = B.counts + (size_t)(bounce + 1) * nseg;
            if (L.count)
                hipLaunchKernelGGL(k_shade<true>, dim3(nseg), dim3(kBlk), 0, st, L.S, L.P, G, B.q[cur][0], B.q[cur][1],
                                   B.q[cur][2], B.qr[cur], cnt, B.hits, B.q[nx][0], B.q[nx][1], B.q[nx][2], B.qr[nx], cnt_out,
                                   B.res, B.res_id, L.counters);
            else
                hipLaunchKernelGGL(k_shade<false>, dim3(nseg), dim3(kBlk), 0, st, L.S, L.P, G, B.q[cur][0], B.q[cur][1],
                                   B.q[cur][2], B.qr[cur], cnt, B.hits, B.q[nx][0], B.q[nx][1], B.q[nx][2], B.qr[nx], cnt_out,
                                   B.res, B.res_id, L.counters);
            cur = nx;
        }
        const uint32_t grid_a = (n_px + kBlk - 1) / kBlk;
        if (L.count)
            hipLaunchKernelGGL(k_accumulate<true>, dim3(grid_a), dim3(kBlk), 0, st, L.P, L.stats, L.pixels, n_px,
                               L.stats_by_pixel ? 1u : 0u, b, B.res, B.res_id, L.S.bloom, L.counters);
        else
            hipLaunchKernelGGL(k_accumulate<false>, dim3(grid_a), dim3(kBlk), 0, st, L.P, L.stats, L.pixels, n_px,
                               L.stats_by_pixel ? 1u : 0u, b, B.res, B.res_id, L.S.bloom, L.counters);
        if ((e = hipGetLastError()) != hipSuccess) { err = "wavefront launch failed"; return e; }
        done += b;
    }
    return hipSuccess;
}

}  // namespace omw
