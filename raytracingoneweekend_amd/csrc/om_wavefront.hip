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
    for (auto& st : tail) { if (st) (void)hipStreamDestroy(st); st = nullptr; }
    if (acc) (void)hipStreamDestroy(acc);
    acc = nullptr;
    for (int k = 0; k < kMaxSets; ++k) {
        if (alt_res[k]) (void)hipFree(alt_res[k]);
        if (alt_id[k]) (void)hipFree(alt_id[k]);
        alt_res[k] = nullptr; alt_id[k] = nullptr;
    }
    alt_cap = 0;
    for (auto e : ev) (void)hipEventDestroy(e);
    ev.clear();
    cap = 0; counts_n = 0; nsets = 0;
}

namespace {

constexpr uint32_t kNoSample = 0xFFFFFFFFu;
#ifndef OM_EMPTY_B2_BRUTE
#define OM_EMPTY_B2_BRUTE 1
#endif
enum { TR_BRUTE = 1, TR_CULLED = 2, TR_BVH = 3, TR_SBVH_LDS = 4, TR_SBVH_GLOBAL = 5, TR_BVH2_LDS = 6, TR_BVH2_GLOBAL = 7,
       TR_BVH4_LDS = 8, TR_BVH4_GLOBAL = 9 };
// Workgroup = one queue segment.  512 lanes share one LDS copy of the BVH2 nodes between 8
// waves, so LDS stops capping occupancy, and 8 waves/SIMD (<= 64 VGPRs; bounce 0 spills
// 8 B/lane) hide the incoherent bounces' latency.  Measured on C1 (tools/ablate.sh):
// 256/no hint 3770, 256/8 3671, 512/- 3802, 512/8 3929, 1024/8 3368 Msamples/s.
#ifndef OM_WF_BLOCK
#define OM_WF_BLOCK 512
#endif
#ifndef OM_WF_WAVES
#define OM_WF_WAVES 8
#endif
// bounce 0 (coherent camera rays, VALU-issue-bound) may ask for fewer waves, and so more
// registers, than the latency-bound later bounces
#ifndef OM_WF_WAVES_FIRST
#define OM_WF_WAVES_FIRST OM_WF_WAVES
#endif
#if OM_WF_WAVES > 0 && OM_WF_WAVES_FIRST > 0
#define OM_WAVES_ATTR_B(FIRST) __attribute__((amdgpu_waves_per_eu((FIRST) ? OM_WF_WAVES_FIRST : OM_WF_WAVES, (FIRST) ? OM_WF_WAVES_FIRST : OM_WF_WAVES)))
#else
#define OM_WAVES_ATTR_B(FIRST)
#endif
#if OM_WF_WAVES > 0                                               // occupancy request (waves per SIMD)
#define OM_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(OM_WF_WAVES, OM_WF_WAVES)))
#else
#define OM_WAVES_ATTR
#endif
constexpr int kBlk = OM_WF_BLOCK;                                 // workgroup = one queue segment
constexpr int kStackDepth = 24;                                   // BVH2 per-lane LDS stack bound (u16 entries)
// LDS bytes of the lane stack: S.b2_stack entries per lane (the tree's internal depth, 9 for
// S-traced: 4.5 KiB per 256-lane workgroup instead of 12 KiB at the 24-entry bound, which
// lifts the LDS-limited occupancy from 5 to 6 workgroups per CU).
template <int TR>
__host__ __device__ inline uint32_t stack_bytes(const OmSceneDev& S) {
    return kBlk * ((TR == TR_BVH4_LDS || TR == TR_BVH4_GLOBAL) ? S.b4_stack : S.b2_stack) * 2u;
}
#ifndef OM_WF_TAIL_SPB
#define OM_WF_TAIL_SPB 2
#endif
constexpr uint32_t kTailSpb = OM_WF_TAIL_SPB;                     // queue segments per tail workgroup
// Async tails (OM_WF_ASYNC_TAIL, fixed-spp calls): each batch's tail runs on the context's tail
// stream while its main stream already starts the call's next batch on another queue set, so
// the latency-bound tails (a chain of up to max_depth - T serial bounces of the longest paths)
// overlap the heavy early bounces instead of leaving the chip idle at every batch boundary.
// The tail grid is narrow (kTailSpbAsync segments per workgroup) so it holds few CU slots.
#ifndef OM_WF_ASYNC_TAIL
#define OM_WF_ASYNC_TAIL 0
#endif
#ifndef OM_WF_TAIL_SPB_ASYNC
#define OM_WF_TAIL_SPB_ASYNC 2
#endif
#ifndef OM_WF_TAIL_PRIO
#define OM_WF_TAIL_PRIO 1
#endif
// With async tails: the bounce from which a batch moves to its tail stream (0: only the tail).
#ifndef OM_WF_DRAIN_AT
#define OM_WF_DRAIN_AT 0
#endif
// Concurrent batches: 1 runs every k_accumulate on the context's accumulate stream with two
// result buffers per queue set, so a stream starts its next batch right after its tail instead
// of waiting for its own accumulate, which waits for the other stream's (sample order): that
// chain held the two streams in lockstep, both draining at once (r03 kernel trace).
#ifndef OM_WF_ACC_STREAM
#define OM_WF_ACC_STREAM 0
#endif
// Late bounces (b >= OM_WF_LATE_GLOBAL, 0: never) of a world whose BVH2 sits in LDS read its nodes
// through the caches instead of staging them: a late-bounce workgroup traces a chunk or two per
// wave, for which the 19 KB copy into LDS (and its barrier) is a large part of its life.
#ifndef OM_WF_LATE_GLOBAL
#define OM_WF_LATE_GLOBAL 0
#endif
// Concurrent batches: stream 1's first batch starts once stream 0's first batch has launched
// bounce OM_WF_STAGGER (0: at once), so one batch's light late bounces meet the other's heavy ones.
#ifndef OM_WF_STAGGER
#define OM_WF_STAGGER 0
#endif
constexpr uint32_t kTailSpbAsync = OM_WF_TAIL_SPB_ASYNC;
constexpr uint32_t kTailDefault = 16;                             // first bounce handled by the tail kernel
// marched worlds: 12 (C2, 8 march steps per refill check, r03_v22/v23: T = 6 / 8 / 10 / 12 / 16 / 20
// / 24 -> 2579 / 2647 / 2674 / 2668 / 2655 / 2605 / 2541 Msamples/s, means of two or four runs)
constexpr uint32_t kTailMarched = 12;
// BVH2s read through L2 (S-10k): 10 (C3, r03_v24/v25: T = 6 / 8 / 10 / 12 / 16 / 20 -> 3318 / 3523 /
// 3553 / 3517 / 3416 / 3351 Msamples/s, means of two to four runs)
constexpr uint32_t kTailL2 = 10;
// batches above 2^25 paths (C4's 4K frame: 16 spp = 133M paths) keep more paths per late bounce,
// so the per-bounce launches stay efficient longer: 24 (C4, r03_v26: T = 12 / 16 / 20 / 24 ->
// 6956 / 7240 / 7304 / 7374 Msamples/s, means of two runs)
constexpr uint32_t kTailBigBatch = 24;
// Merged late bounces (traced worlds): from bounce OM_WF_MERGE_AT on (0: never), a bounce
// workgroup handles OM_WF_MERGE consecutive queue segments.  The late bounces carry few paths
// per segment, yet each launch filled every CU with whole 512-lane workgroups (8 wave slots
// each, mostly idle) that the other batch's heavy launches then lacked; merging divides those
// launches' workgroups by OM_WF_MERGE.  Segment k's paths stay within merged segment k / F, so
// nothing else changes (results are keyed by slot and (pixel, sample)).
#ifndef OM_WF_MERGE_AT
#define OM_WF_MERGE_AT 0
#endif
#ifndef OM_WF_MERGE
#define OM_WF_MERGE 4
#endif
constexpr uint32_t kMergeMax = 16;
static_assert(OM_WF_MERGE >= 1 && OM_WF_MERGE <= kMergeMax, "OM_WF_MERGE in [1, 16]");
// Work distribution inside a bounce workgroup.  1 (default): every wave takes 64-path
// chunks of the segment from an LDS counter and appends its survivors with one LDS atomic,
// so the 8 waves never wait for each other; 0: the block walks the segment in 512-path
// steps with a block-wide ballot scan (two barriers per step, every wave waits for the
// slowest).  Both produce identical bits: a path's results are keyed by its slot and its
// RNG by (pixel, sample), never by its queue position.
#ifndef OM_WF_WAVEQ
#define OM_WF_WAVEQ 1
#endif
#ifndef OM_WF_MAX_PATHS_LOG2
#define OM_WF_MAX_PATHS_LOG2 27
#endif
// samples per pixel per batch for frames above 2M pixels (within 2^OM_WF_MAX_PATHS_LOG2 paths)
#ifndef OM_WF_BATCH_SPP
#define OM_WF_BATCH_SPP 16
#endif
#ifndef OM_WF_MIN_PATHS_LOG2
#define OM_WF_MIN_PATHS_LOG2 25
#endif
// Bounce 0 with primary tile lists: a wave whose lanes all lie in one 8x8 tile (every wave but
// those where partial tiles meet) reads the tile's list and records with scalar loads.
#ifndef OM_TILES_UNIFORM
#define OM_TILES_UNIFORM 1
#endif
// Segment capacity rounded up to whole waves (0: exact split), so that a bounce-0 wave is
// exactly one 8x8 tile of one sample (tile-ordered pixel lists hold whole tiles).
// A BVH2 too big for LDS (S-10k: 213 KB) stages its breadth-first prefix, up to this many
// bytes of nodes, into LDS; deeper nodes are read through L2 (0 = every node from L2).
#ifndef OM_WF_HYB_BYTES
#define OM_WF_HYB_BYTES 24576
#endif
__host__ __device__ inline uint32_t hyb_nodes(const OmSceneDev& S) {
    return S.b2_lds_bytes ? 0u : (S.n_b2nodes < OM_WF_HYB_BYTES / 64u ? S.n_b2nodes : OM_WF_HYB_BYTES / 64u);
}
// Worlds with marched primitives: 1 (default) runs each bounce as a lane-refilling march
// launch (k_march: lanes whose march ended take the segment's next paths together once
// OM_WF_REFILL of them wait, so a wave no longer runs as long as its longest march) followed
// by the shade+compact launch reading the (closest, winner) it wrote; 0 keeps the fused
// trace+march+shade bounce kernel.
#ifndef OM_WF_MARCH_SPLIT
#define OM_WF_MARCH_SPLIT 1
#endif
// k_march instances: SMALL = keep a marched set that fits MarchedSmall in registers (chosen on
// the host, one copy of the march code per instance) instead of reading the scene arrays.
// Off by default: on C2 the register instance measured 1419-1454 Msamples/s against 1618-1624
// for the arrays (one instance holding both views: 1437-1451), although the same view speeds
// up the megakernel's march() (983 -> 1080).
#ifndef OM_WF_MARCH_REGS
#define OM_WF_MARCH_REGS 0
#endif
// k_march instance for a marched set of exactly C2's shape (2 spheres, 1 box, 1 torus: S-marched),
// every march step unrolled with no count guards: 2 (default) the SDF-only fields
// staged in LDS once per workgroup (MarchedExactLds), 1 copied to SGPRs (MarchedExact; C2 -1.4%),
// 0 the arrays view.  Traced parts TR_BRUTE / TR_BVH2_LDS only.
#ifndef OM_WF_MARCH_EXACT
#define OM_WF_MARCH_EXACT 2
#endif
using MarchedC2 = MarchedExact<2, 1, 1>;
using MarchedC2Lds = MarchedExactLds<2, 1, 1>;
enum { MV_ARRAYS = 0, MV_SMALL = 1, MV_EXACT_C2 = 2, MV_EXACT_C2_LDS = 3 };
template <int TR>
__host__ __device__ constexpr bool exact_view_built() { return OM_WF_MARCH_EXACT && (TR == TR_BRUTE || TR == TR_BVH2_LDS); }
// k_march refills its idle lanes once at least this many of a wave's 64 wait.
#ifndef OM_WF_REFILL
#define OM_WF_REFILL 16
#endif
// k_march: march steps per refill check (the check costs three ballots and its branches).
// C2 (r03_v16/v17): 1 / 2 / 4 / 6 / 8 steps -> 2500 / 2587 / 2650 / 2661 / 2682 Msamples/s.
#ifndef OM_MARCH_UNROLL
#define OM_MARCH_UNROLL 8
#endif
// Adaptive calls: samples per pixel per (serial) batch.  Bounce 0 reads each pixel's retirement
// flag at the batch start; a pixel that retires inside a batch has its remaining samples of
// that batch rendered and dropped by k_accumulate (the result is the sequential one).  C1
// adaptive, 16 spp per call (tools/adaptive_sweep.sh): 1 / 4 / 8 / 16 -> 564 / 1519 / 2376 /
// 3190 credited Msamples/s (megakernel: 2749).
#ifndef OM_WF_ADAPTIVE_BATCH
#define OM_WF_ADAPTIVE_BATCH 16
#endif
// k_bounce b >= 1: load the path's throughput/RNG/slot lanes before the trace (1: their latency hides
// behind it, +1.3% on C1 over five A/B pairs) or after it (0).
#ifndef OM_WF_EARLY_REST
#define OM_WF_EARLY_REST 1
#endif
// Queue segments (= bounce workgroups) per CU: OM_WF_LANES_PER_CU / OM_WF_BLOCK.
#ifndef OM_WF_LANES_PER_CU
#define OM_WF_LANES_PER_CU 4096
#endif
// Marched worlds (split march pipeline) and BVH2s read through L2 (S-10k)
// use twice the segments: k_march's lane refill and the L2-bound traversal both drain a
// segment at their own pace, and halving each workgroup's share shortens the last round of
// workgroups in every launch.  C2 / C3 / C1 measurements in DESIGN.md §5.8.
#ifndef OM_WF_LANES_PER_CU_WIDE
#define OM_WF_LANES_PER_CU_WIDE 8192
#endif
#ifndef OM_WF_ALIGN
#define OM_WF_ALIGN 64
#endif
__host__ __device__ inline uint32_t seg_capacity(uint64_t paths, uint32_t nseg) {
    const uint64_t c = (paths + nseg - 1) / nseg;
    return OM_WF_ALIGN > 1 ? (uint32_t)((c + OM_WF_ALIGN - 1) / OM_WF_ALIGN * OM_WF_ALIGN) : (uint32_t)c;
}

extern __shared__ __attribute__((aligned(16))) uint4 wf_lds[];

// Diagnostic build only (OM_PHASE_STAMPS=1, tools/phase_stamps.py): every wave sums the shader
// cycles (s_memtime) its lanes spend in each phase of a path chunk, and lane 0 adds the sums to
// g_phase[kernel * 8 + phase] at exit.  Production builds compile none of it.
#ifndef OM_PHASE_STAMPS
#define OM_PHASE_STAMPS 0
#endif
#if OM_PHASE_STAMPS
__device__ unsigned long long g_phase[64];
enum { PHK_BOUNCE0 = 0, PHK_BOUNCE = 8, PHK_TAIL = 16, PHK_MARCH = 24, PHK_HIT = 32 };
struct PhaseClock {
    uint64_t t, begin, acc[6] = {0, 0, 0, 0, 0, 0};
    __device__ PhaseClock() { t = begin = __builtin_amdgcn_s_memtime(); }
    __device__ void lap(int k) { const uint64_t n = __builtin_amdgcn_s_memtime(); acc[k] += n - t; t = n; }
    __device__ void flush(int base) {
        const uint64_t life = __builtin_amdgcn_s_memtime() - begin;
        if (__lane_id() == 0) {
            for (int k = 0; k < 6; ++k) atomicAdd(&g_phase[base + k], (unsigned long long)acc[k]);
            atomicAdd(&g_phase[base + 6], (unsigned long long)life);
            atomicAdd(&g_phase[base + 7], 1ull);                    // waves
        }
    }
};
// OM_PHASE_STAMPS=2: the trace's laps (WorkT::lap, om_trace.h), summed over the lanes of every
// wave (a lane's sums cover the steps it took part in) -> g_phase[40 + k] cycles, [48 + k] laps
template <class Wk>
__device__ void flush_laps(const Wk& w) {
#if OM_PHASE_STAMPS == 2
    for (int k = 0; k < LAP_N; ++k) {
        atomicAdd(&g_phase[40 + k], (unsigned long long)w.lacc[k]);
        atomicAdd(&g_phase[48 + k], (unsigned long long)w.lcnt[k]);
    }
#endif
}
#define PH_DECL PhaseClock ph_
#define PH_LAP(k) ph_.lap(k)
#define PH_WAIT_LAP(k) do { __builtin_amdgcn_s_waitcnt(0); ph_.lap(k); } while (0)
#define PH_FLUSH(base) ph_.flush(base)
#else
#define PH_DECL
#define PH_LAP(k)
#define PH_WAIT_LAP(k)
#define PH_FLUSH(base)
#endif

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
    uint32_t nseg;    // segments (= bounce workgroups)
    uint32_t segcap;  // paths per segment
    // merged read (OM_WF_MERGE_AT, k_bounce b >= 1 only): workgroup s reads the input segments
    // [s*fin, min((s+1)*fin, nseg_in)) of capacity segcap_in each and writes output segment s
    // (capacity segcap = fin * segcap_in, so its survivors always fit); fin = 1: no merge
    uint32_t fin = 1;
    uint32_t segcap_in = 0;
    uint32_t nseg_in = 0;
};

// One SoA path queue: o|depthf, d|first_id, throughput|segment, rng s|rng k|slot|-.
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
    const uint32_t* n0;          // fixed-spp calls: Stats.n per listed pixel at the call's start
    uint32_t done;               // samples of the call before this batch (with n0)
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

// OM_WF_NT_LOADS: the path-state loads carry the non-temporal hint (each 16-B lane record is read
// once per bounce), so the streaming queues do not evict the leaf records and nodes the trace
// re-reads from the vector L1.  Component loads keep the scalar register shapes (a native
// 4-vector load moved k_bounce into scratch spills in r01); the compiler still merges them into
// global_load_dwordx4 ... nt.  C1 with both hints: 7096 / 7114 vs 7094 / 7068 Msamples/s (r03_v13).
#ifndef OM_WF_NT_LOADS
#define OM_WF_NT_LOADS 1
#endif
template <class V>
__device__ __forceinline__ V ld4(const V* q) {
#if OM_WF_NT_LOADS
    V v;
    v.x = __builtin_nontemporal_load(&q->x); v.y = __builtin_nontemporal_load(&q->y);
    v.z = __builtin_nontemporal_load(&q->z); v.w = __builtin_nontemporal_load(&q->w);
    return v;
#else
    return *q;
#endif
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
// OM_WF_NT_STORES: the same hint on the path-state stores (read back only by the next launch).
#ifndef OM_WF_NT_STORES
#define OM_WF_NT_STORES 1
#endif
template <class V>
__device__ __forceinline__ void st4(V* q, V v) {
#if OM_WF_NT_STORES
    __builtin_nontemporal_store(v.x, &q->x); __builtin_nontemporal_store(v.y, &q->y);
    __builtin_nontemporal_store(v.z, &q->z); __builtin_nontemporal_store(v.w, &q->w);
#else
    *q = v;
#endif
}
__device__ __forceinline__ void store_path(const Queue& Q, uint64_t i, const Path& p) {
    st4(Q.q0 + i, make_float4(p.o.x, p.o.y, p.o.z, p.depthf));
    st4(Q.q1 + i, make_float4(p.d.x, p.d.y, p.d.z, __uint_as_float(p.first_id)));
    st4(Q.q2 + i, make_float4(p.cur.x, p.cur.y, p.cur.z, __uint_as_float(p.seg)));
    st4(Q.qr + i, make_uint4(p.g.s, p.g.k, p.slot, 0u));
}

// Scene data a workgroup traces against: BVH2/BVH4 nodes + leaf table staged in LDS behind
// the per-lane stack ([stack][nodes][leaf table]), or read through L2.
struct Tracer {
    const OmBvh2Node* b2n;
    uint32_t nl;             // TR_BVH2_GLOBAL: nodes [0, nl) staged in LDS at b2l
    const OmBvh2Node* b2l;
    const OmBvh4Node* b4n;
    const uint32_t* bl;
    const OmAffineTest* recs;
    uint16_t* stk;
};

template <int TR, uint32_t STACKS = 1>
__device__ __forceinline__ Tracer stage_scene(const OmSceneDev& S) {   // every thread of the block calls it
    Tracer t;
    t.stk = (uint16_t*)wf_lds + threadIdx.x;
    t.b2n = S.b2nodes; t.b4n = S.b4nodes; t.bl = S.b2leaves; t.recs = S.srecs;
    t.nl = 0; t.b2l = S.b2nodes;
    if (TR == TR_BVH2_GLOBAL && hyb_nodes(S)) {
        t.nl = hyb_nodes(S);
        uint4* dst = wf_lds + STACKS * stack_bytes<TR>(S) / 16u;
        const uint4* sn = (const uint4*)S.b2nodes;
        for (uint32_t i = threadIdx.x; i < t.nl * 4u; i += kBlk) dst[i] = sn[i];
        __syncthreads();
        t.b2l = (const OmBvh2Node*)dst;
    }
    if (TR == TR_BVH2_LDS || TR == TR_BVH4_LDS) {
        const uint32_t nn = TR == TR_BVH2_LDS ? S.n_b2nodes * 4u : S.n_b4nodes * 7u;   // uint4 per node
        const uint4* sn = TR == TR_BVH2_LDS ? (const uint4*)S.b2nodes : (const uint4*)S.b4nodes;
        uint4* dst = wf_lds + STACKS * stack_bytes<TR>(S) / 16u;
        for (uint32_t i = threadIdx.x; i < nn; i += kBlk) dst[i] = sn[i];
        uint32_t* ldst = (uint32_t*)(dst + nn);
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
    if (TR == TR_BVH4_LDS || TR == TR_BVH4_GLOBAL) best = traced_bvh4<kBlk>(S, T.b4n, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w);
    else if (TR == TR_BVH2_LDS) best = traced_bvh2<kStackDepth, kBlk>(S, T.b2n, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w);
    else if (TR == TR_BVH2_GLOBAL)
        best = traced_bvh2<kStackDepth, kBlk, Wk, true>(S, T.b2l, T.bl, T.recs, T.stk, o, d, P.tmin, closest, w, T.b2n, T.nl);
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
template <bool MARCH>
__device__ __forceinline__ bool shade_path(const OmSceneDev& S, const OmParamsDev& P, uint32_t depth_cap, Path& p,
                                           float closest, int best, float4* __restrict__ res,
                                           uint32_t* __restrict__ res_id) {
    float seg_depth; uint32_t seg_id;
    if (best >= 0) {                                                   // handle_hit, Some(hr)
        F3 point, normal;
        finalize<MARCH>(S, best, p.o, p.d, P.tmin, closest, point, normal);
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
__device__ __forceinline__ bool gen_path(const OmParamsDev& P, const Gen& R, uint64_t i, Path& p, uint32_t& pixel,
                                         uint32_t* __restrict__ res_id) {
    const uint32_t s_local = (uint32_t)(i / R.n_pixels), k = (uint32_t)(i - (uint64_t)s_local * R.n_pixels);
    pixel = R.pixels[k];
    // the sample index is the pixel's Stats.n (jitters[pixel.stats.n], render_thread.rs:188).
    // Fixed-spp calls take it from the call-start snapshot plus the samples of earlier
    // batches, so a batch never waits for the previous batch's accumulate; adaptive
    // calls (serial batches) read the live Stats for n and the done flag.
    uint32_t s;
    bool live;
    if (R.n0) {
        s = R.n0[k] + R.done + s_local;
        live = s < P.spp_total;
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
template <int TR, bool COUNT, bool MARCH, bool FIRST, bool HIT = false>
__global__ __launch_bounds__(kBlk) OM_WAVES_ATTR_B(FIRST) void k_bounce(OmSceneDev S, OmParamsDev P, Seg G, Gen R, Queue in,
                                                 const uint32_t* __restrict__ count_in, Queue out,
                                                 uint32_t* __restrict__ count_out, float4* __restrict__ res,
                                                 uint32_t* __restrict__ res_id, unsigned long long* __restrict__ counters,
                                                 const float2* __restrict__ hitbuf) {
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    uint32_t n;
    __shared__ uint32_t mpre[kMergeMax + 1];          // merged read: prefix of the input segments' counts
    const bool merged = !FIRST && !HIT && G.fin > 1u;
    if (FIRST) {
        const uint64_t paths = (uint64_t)R.n_pixels * R.batch;
        n = seg0 < paths ? (uint32_t)std::min<uint64_t>(G.segcap, paths - seg0) : 0u;
    } else if (merged) {
        if (threadIdx.x == 0) {
            uint32_t acc = 0;
            for (uint32_t k = 0; k < G.fin; ++k) {
                mpre[k] = acc;
                const uint32_t si = blockIdx.x * G.fin + k;
                acc += si < G.nseg_in ? count_in[si] : 0u;
            }
            mpre[G.fin] = acc;
        }
        __syncthreads();
        n = mpre[G.fin];
    } else {
        n = count_in[blockIdx.x];
    }
    if (n == 0) {
        if (threadIdx.x == 0) count_out[blockIdx.x] = 0u;
        return;
    }
#if OM_WF_WAVEQ
    __shared__ uint32_t q_next, q_out;
    if (threadIdx.x == 0) { q_next = kBlk / 64u; q_out = 0u; }
    __syncthreads();
#endif
    const Tracer T = HIT ? Tracer{} : stage_scene<TR>(S);
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    WorkT<COUNT> w;
    uint32_t segs = 0, run = 0;
    PH_DECL;
#if OM_WF_WAVEQ
    const uint32_t lane = __lane_id();
    for (uint32_t chunk = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); chunk * 64u < n;) {   // wave-uniform
        const uint32_t jj = chunk * 64u + lane;
#else
    for (uint32_t base = 0; base < n; base += kBlk) {
        const uint32_t jj = base + threadIdx.x;
#endif
        bool keep = false;
        Path p;
        uint32_t p_pixel = 0;
        if (jj < n) {
            uint64_t i = seg0 + jj;
            if (merged) {                                 // input segment k of the workgroup's fin
                uint32_t k = 0;
                while (jj >= mpre[k + 1]) ++k;
                i = (uint64_t)(blockIdx.x * G.fin + k) * G.segcap_in + (jj - mpre[k]);
            }
            bool live = true;
            if (FIRST) {
                live = gen_path(P, R, i, p, p_pixel, res_id);
            } else {
                load_ray(in, i, p);
#if OM_WF_EARLY_REST
                load_rest(in, i, p);       // issued before the trace: its latency hides behind it
#endif
            }
            PH_WAIT_LAP(0);
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
#if OM_TILES_UNIFORM
                    // a wave within one tile reads its list with scalar loads
                    const uint32_t t0 = __builtin_amdgcn_readfirstlane(tile);
                    if (__ballot(tile != t0) == 0)
                        best = traced_tiles<true>(S, R.tile_off, R.tile_idx, t0, p.o, p.d, P.tmin, closest, w, R.tile_tnear);
                    else
#endif
                        best = traced_tiles(S, R.tile_off, R.tile_idx, tile, p.o, p.d, P.tmin, closest, w);
                    if (MARCH) {
                        float tm;
                        const int mg = march(S, p.o, p.d, P.tmin, P.tmax, closest, P.march_steps, tm, w);
                        if (mg >= 0) { best = mg; closest = tm; }
                    }
                } else {
                    best = trace<TR, MARCH>(S, P, T, p.o, p.d, closest, w);
                }
#ifdef OM_ABLATE_TRACE2X   // timing ablation (tools/ablate.sh): the trace runs twice, same answer
                {
                    F3 o2 = p.o;
                    o2.x += P.march_steps == 0xDEADBEEFu ? 1.0f : 0.0f;
                    float c2;
                    const int b2 = trace<TR, MARCH>(S, P, T, o2, p.d, c2, w);
                    if (b2 != best || c2 != closest) res_id[0] = 0xDEADu;
                }
#endif
#if !OM_WF_EARLY_REST
                if (!FIRST) load_rest(in, i, p);
#endif
                PH_WAIT_LAP(1);
#ifdef OM_ABLATE_SHADE2X   // timing ablation: shade a copy first (same result slot, same values)
                {
                    Path p2 = p;
                    p2.cur.x *= P.march_steps == 0xDEADBEEFu ? 2.0f : 1.0f;
                    if (shade_path<MARCH>(S, P, depth_cap, p2, closest, best, res, res_id) && p2.seg == 0xFFFFFFu) res_id[1] = 0u;
                }
#endif
                keep = shade_path<MARCH>(S, P, depth_cap, p, closest, best, res, res_id);
                if (COUNT) segs++;
                PH_WAIT_LAP(2);
            }
        }
#if OM_WF_WAVEQ
        const uint64_t m = __ballot(keep);
        uint32_t obase = 0u, nc = 0u;
        if (lane == 0) {
            obase = m ? atomicAdd(&q_out, (uint32_t)__popcll(m)) : 0u;
            nc = atomicAdd(&q_next, 1u);
        }
        obase = __builtin_amdgcn_readfirstlane(obase);
        chunk = __builtin_amdgcn_readfirstlane(nc);
        if (keep) store_path(out, seg0 + obase + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), p);
        PH_WAIT_LAP(3);
    }
    PH_FLUSH(HIT ? PHK_HIT : FIRST ? PHK_BOUNCE0 : PHK_BOUNCE);
#if OM_PHASE_STAMPS
    if (!FIRST && !HIT) flush_laps(w);
#endif
    __syncthreads();
    run = q_out;
#else
        uint32_t tot;
        const uint32_t j = block_scan(keep, tot);
        if (keep) store_path(out, seg0 + run + j, p);
        run += tot;
    }
#endif
    if (threadIdx.x == 0) count_out[blockIdx.x] = run;
    if (COUNT) {
        flush_counter(counters, OMC_SEGMENTS, segs);
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- two paths per lane
// OM_WF_DUAL: bounces b >= 1 of traced worlds whose BVH2 sits in LDS run
// k_bounce2 instead of k_bounce: a wave takes 128-path chunks, lane l holds paths l and l + 64
// of its chunk and traces both at once (traced_bvh2_x2: each iteration fetches the next node or
// leaf record of BOTH rays before advancing either), then shades both and appends the survivors
// of both with one LDS atomic.  The lane stack is doubled (second half: the B rays).  Results
// are keyed by slot and (pixel, sample) as everywhere, so the bits are unchanged.
#ifndef OM_WF_DUAL
#define OM_WF_DUAL 0
#endif
#if OM_WF_DUAL && OM_B2_DIRECT
#error "OM_WF_DUAL's b2_enter reads the leaf table: build it with -DOM_B2_DIRECT=0"
#endif
#ifndef OM_WF_DUAL_WAVES
#define OM_WF_DUAL_WAVES 0
#endif
#if OM_WF_DUAL_WAVES > 0
#define OM_WAVES_ATTR_DUAL __attribute__((amdgpu_waves_per_eu(OM_WF_DUAL_WAVES, OM_WF_DUAL_WAVES)))
#else
#define OM_WAVES_ATTR_DUAL
#endif
template <bool COUNT>
__global__ __launch_bounds__(kBlk) OM_WAVES_ATTR_DUAL void k_bounce2(OmSceneDev S, OmParamsDev P, Seg G, Queue in,
                                                           const uint32_t* __restrict__ count_in, Queue out,
                                                           uint32_t* __restrict__ count_out, float4* __restrict__ res,
                                                           uint32_t* __restrict__ res_id,
                                                           unsigned long long* __restrict__ counters) {
    const uint64_t seg0 = (uint64_t)blockIdx.x * G.segcap;
    const uint32_t n = count_in[blockIdx.x];
    if (n == 0) {
        if (threadIdx.x == 0) count_out[blockIdx.x] = 0u;
        return;
    }
    __shared__ uint32_t q_next, q_out;
    if (threadIdx.x == 0) { q_next = kBlk / 64u; q_out = 0u; }
    __syncthreads();
    const Tracer T = stage_scene<TR_BVH2_LDS, 2>(S);
    uint16_t* stkB = T.stk + S.b2_stack * kBlk;
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    WorkT<COUNT> w;
    uint32_t segs = 0;
    const uint32_t lane = __lane_id();
    for (uint32_t chunk = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); chunk * 128u < n;) {   // wave-uniform
        const uint32_t ja = chunk * 128u + lane, jb = ja + 64u;
        const bool ina = ja < n, inb = jb < n;
        Path pa, pb;
        B2Ray A, B;
        A.sp = -1; B.sp = -1;
        if (ina) load_ray(in, seg0 + ja, pa);
        if (inb) load_ray(in, seg0 + jb, pb);
        if (ina) b2_begin(S, A, pa.o, pa.d, P.tmin, P.tmax, w);
        if (inb) b2_begin(S, B, pb.o, pb.d, P.tmin, P.tmax, w);
        traced_bvh2_x2<kStackDepth, kBlk>(S, T.b2n, T.bl, T.recs, T.stk, stkB, P.tmin, A, B, w);
        bool ka = false, kb = false;
        if (ina) {
            load_rest(in, seg0 + ja, pa);
            ka = shade_path<false>(S, P, depth_cap, pa, A.closest, A.best, res, res_id);
            if (COUNT) segs++;
        }
        if (inb) {
            load_rest(in, seg0 + jb, pb);
            kb = shade_path<false>(S, P, depth_cap, pb, B.closest, B.best, res, res_id);
            if (COUNT) segs++;
        }
        const uint64_t ma = __ballot(ka), mb = __ballot(kb);
        uint32_t obase = 0u, nc = 0u;
        if (lane == 0) {
            const uint32_t c = (uint32_t)(__popcll(ma) + __popcll(mb));
            obase = c ? atomicAdd(&q_out, c) : 0u;
            nc = atomicAdd(&q_next, 1u);
        }
        obase = __builtin_amdgcn_readfirstlane(obase);
        chunk = __builtin_amdgcn_readfirstlane(nc);
        const uint64_t below = (1ull << lane) - 1ull;
        if (ka) store_path(out, seg0 + obase + (uint32_t)__popcll(ma & below), pa);
        if (kb) store_path(out, seg0 + obase + (uint32_t)__popcll(ma) + (uint32_t)__popcll(mb & below), pb);
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
    const uint64_t paths = (uint64_t)R.n_pixels * R.batch;
    const uint32_t n = seg0 < paths ? (uint32_t)std::min<uint64_t>(G.segcap, paths - seg0) : 0u;
    __shared__ uint32_t q_out;
    if (threadIdx.x == 0) q_out = 0u;
    __syncthreads();
    const uint32_t lane = __lane_id();
    for (uint32_t base = 0; base < n; base += kBlk) {
        const uint32_t jj = base + threadIdx.x;
        Path p;
        uint32_t pixel;
        const bool keep = jj < n && gen_path(P, R, seg0 + jj, p, pixel, res_id);
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
    PH_DECL;
    auto start = [&]() {
        const float4 a = in.q0[seg0 + j], b = in.q1[seg0 + j];
        o = f3(a.x, a.y, a.z); d = f3(b.x, b.y, b.z);
        best = trace<TR, false>(S, P, T, o, d, closest, w);
        marching = march_begin(m, o, d, P.tmin, t);
        iters = P.march_steps;
    };
    if (act) start();
    PH_WAIT_LAP(0);
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
        PH_WAIT_LAP(1);
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
            PH_WAIT_LAP(0);
        }
        PH_LAP(3);
        if (__ballot(act) == 0) break;
    }
    PH_FLUSH(PHK_MARCH);
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
    } else if constexpr (VIEW == MV_EXACT_C2) march_lanes<TR, COUNT>(S, P, T, MarchedC2(S), in, seg0, n, next, hit, w);
    else if constexpr (VIEW == MV_SMALL) march_lanes<TR, COUNT>(S, P, T, MarchedSmall(S), in, seg0, n, next, hit, w);
    else march_lanes<TR, COUNT>(S, P, T, MarchedArrays(S), in, seg0, n, next, hit, w);
    if (COUNT) {
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- tail
#ifndef OM_WF_TAIL_SETPRIO
#define OM_WF_TAIL_SETPRIO 0
#endif
// Workgroup b: every path of segments [b*kTailSpb, (b+1)*kTailSpb) of queue `in`, each
// run to completion; a lane whose path ends takes the next one from an LDS counter.
template <int TR, bool COUNT, bool MARCH, uint32_t SPB = kTailSpb>
__global__ __launch_bounds__(kBlk) OM_WAVES_ATTR void k_tail(OmSceneDev S, OmParamsDev P, Seg G, Queue in,
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
    // the tail is a few long chains beside the other stream's full launches: a raised wave
    // priority lets its waves issue first on the SIMDs they share (OM_WF_TAIL_SETPRIO, 0 = off)
    if (OM_WF_TAIL_SETPRIO > 0) __builtin_amdgcn_s_setprio(OM_WF_TAIL_SETPRIO);
    const Tracer T = stage_scene<TR>(S);
    const uint32_t depth_cap = P.max_depth > 1u ? P.max_depth : 1u;
    WorkT<COUNT> w;
    uint32_t segs = 0;
    PH_DECL;
    for (uint32_t idx = threadIdx.x; idx < total; idx = atomicAdd(&next, 1u)) {
        uint32_t k = 0;
        while (idx >= pre[k + 1]) ++k;
        const uint64_t i = (uint64_t)(s0 + k) * G.segcap + (idx - pre[k]);
        Path p;
        load_ray(in, i, p);
        load_rest(in, i, p);
        PH_WAIT_LAP(0);
        for (;;) {
            float closest;
            const int best = trace<TR, MARCH>(S, P, T, p.o, p.d, closest, w);
            if (COUNT) segs++;
            PH_WAIT_LAP(1);
            const bool more = shade_path<MARCH>(S, P, depth_cap, p, closest, best, res, res_id);
            PH_WAIT_LAP(2);
            if (!more) break;
        }
    }
    PH_FLUSH(PHK_TAIL);
    if (COUNT) {
        flush_counter(counters, OMC_SEGMENTS, segs);
        flush_counter(counters, OMC_PRIM_TESTS, w.prim);
        flush_counter(counters, OMC_PRE_TESTS, w.pre);
        flush_counter(counters, OMC_MARCH, w.march);
    }
}

// ---------------------------------------------------------------- accumulate
#ifndef OM_ACC_SETPRIO
#define OM_ACC_SETPRIO 0
#endif
#ifndef OM_ACC_GROUP
#define OM_ACC_GROUP 8
#endif
template <bool COUNT>
__global__ __launch_bounds__(kBlk) void k_accumulate(OmParamsDev P, om_pixel_stats* __restrict__ stats,
                                                     const uint32_t* __restrict__ pixels, uint32_t n_pixels, uint32_t by_pixel,
                                                     uint32_t batch, const float4* __restrict__ res,
                                                     const uint32_t* __restrict__ res_id, const uint64_t* __restrict__ bloom,
                                                     unsigned long long* __restrict__ counters) {
    if (OM_ACC_SETPRIO > 0) __builtin_amdgcn_s_setprio(OM_ACC_SETPRIO);
    const uint32_t k = blockIdx.x * kBlk + threadIdx.x;
    uint32_t n_samples = 0, credited = 0;
    if (k < n_pixels) {
        const uint32_t slot = by_pixel ? pixels[k] : k;
        const om_pixel_stats in = stats[slot];
        PixelState st;
        st.bloom = in.bloom; st.sx = in.sum[0]; st.sy = in.sum[1]; st.sz = in.sum[2]; st.n = in.n;
        st.avg_depth = in.avg_depth; st.bad = in.bad_avgs;
        st.rgbf = (uint32_t)in.color[0] | ((uint32_t)in.color[1] << 8) | ((uint32_t)in.color[2] << 16) | ((uint32_t)in.flags << 24);
#if OM_ACC_GROUP > 1
        // the loads of OM_ACC_GROUP samples are issued together (ids, then results and bloom
        // words), then added in sample order: one lane's samples no longer cost a chain of
        // dependent global round trips each (r03: 0.2-0.85 ms per 1080p x 16-spp launch before)
        bool retired = false;
        for (uint32_t s0 = 0; s0 < batch && !retired; s0 += OM_ACC_GROUP) {
            const uint32_t m = batch - s0 < OM_ACC_GROUP ? batch - s0 : OM_ACC_GROUP;
            uint32_t id[OM_ACC_GROUP];
            float4 rr[OM_ACC_GROUP];
            uint64_t bl[OM_ACC_GROUP];
#pragma unroll
            for (uint32_t j = 0; j < OM_ACC_GROUP; ++j) id[j] = j < m ? res_id[(uint64_t)(s0 + j) * n_pixels + k] : kNoSample;
#pragma unroll
            for (uint32_t j = 0; j < OM_ACC_GROUP; ++j) {
                if (j < m) rr[j] = res[(uint64_t)(s0 + j) * n_pixels + k];
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
#else
        for (uint32_t s = 0; s < batch; ++s) {                                 // sample order == reference order
            // adaptive batches of several samples: a pixel that retires at sample j takes no more
            // (ThreadPixels::add_run, render_thread.rs:68-102); the batch's later samples of it
            // were rendered speculatively and are dropped here
            if (P.adaptive && (st.rgbf & 0x01000000u)) break;
            const uint64_t t = (uint64_t)s * n_pixels + k;
            const uint32_t id = res_id[t];
            if (id == kNoSample) continue;
            const float4 rr = res[t];
            const bool done = stats_add(st, f3(rr.x, rr.y, rr.z), rr.w, bloom[id]);
            if (COUNT) n_samples++;
            credited += ((done && P.adaptive) ? (P.spp_total - st.n) : 0u) + 1u;   // render_thread.rs:196-198
        }
#endif
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
    if (P.progress) flush_counter(counters, OMC_PROGRESS, credited);      // live samples_atom (om_progress)
}

// k_snapshot: n0[k] = Stats.n of listed pixel k at the start of a fixed-spp call.
__global__ __launch_bounds__(256) void k_snapshot(const om_pixel_stats* __restrict__ stats, const uint32_t* __restrict__ pixels,
                                                  uint32_t n_pixels, uint32_t by_pixel, uint32_t* __restrict__ n0) {
    const uint32_t k = blockIdx.x * 256u + threadIdx.x;
    if (k < n_pixels) n0[k] = stats[by_pixel ? pixels[k] : k].n;
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

// One batch: bounce 0 .. tail_at-1 as per-bounce launches, then the tail launch; returns
// the number of bounce-family launches.
// Async tails (Tail.ev set): the bounce launches go on `st`; the event is recorded after the
// last of them, and the tail launch (narrow: kTailSpbAsync segments per workgroup, so it holds
// few CU slots while it trickles) goes on Tail.st behind it.  Otherwise the tail follows on st.
struct Tail {
    hipStream_t st;
    hipEvent_t ev;
    hipEvent_t stag = nullptr;   // recorded on the batch's stream after its bounce stag_at launch
    uint32_t stag_at = 0;
};
template <int TR, bool COUNT, bool MARCH>
__host__ inline void launch_tail(const Launch& L, QueueSet& B, Seg G, const Queue& in, const uint32_t* cin, uint32_t lds,
                                 hipStream_t st, const Tail& T, Timer& tm, bool each) {
    hipStream_t ts = st;
    if (T.ev) {
        (void)hipEventRecord(T.ev, st);
        (void)hipStreamWaitEvent(T.st, T.ev, 0);
        ts = T.st;
    }
    const int ti = each ? tm.begin(ts) : -1;
    if (T.ev) {
        const uint32_t grid = (G.nseg + kTailSpbAsync - 1u) / kTailSpbAsync;
        hipLaunchKernelGGL((k_tail<TR, COUNT, MARCH, kTailSpbAsync>), dim3(grid), dim3(kBlk), lds, ts, L.S, L.P, G, in, cin,
                           B.res, B.res_id, L.counters);
    } else {
        const uint32_t grid = (G.nseg + kTailSpb - 1u) / kTailSpb;
        hipLaunchKernelGGL((k_tail<TR, COUNT, MARCH>), dim3(grid), dim3(kBlk), lds, ts, L.S, L.P, G, in, cin,
                           B.res, B.res_id, L.counters);
    }
    tm.end(ti, OM_KT_TAIL, ts);
}
template <int TR, bool COUNT, bool MARCH>
uint32_t run_batch(QueueSet& B, const Launch& L, hipStream_t st, Seg G, const Gen& R, uint32_t depth_cap,
                   uint32_t tail_at, uint32_t lds, const Tail& T) {
    Timer& tm = *L.timer;
    const bool each = tm.mode == 1;
    uint32_t launches = 0;
    if (MARCH && OM_WF_MARCH_SPLIT) {
        {
            const int ti = each ? tm.begin(st) : -1;
            hipLaunchKernelGGL((k_raygen<COUNT>), dim3(G.nseg), dim3(kBlk), 0, st, L.P, G, R, queue(B, 0), B.counts, B.res_id);
            tm.end(ti, OM_KT_BOUNCE0, st);
            ++launches;
        }
        for (uint32_t bounce = 0; bounce < depth_cap; ++bounce) {
            const Queue in = queue(B, bounce & 1u), out = queue(B, (bounce + 1u) & 1u);
            const uint32_t* cin = B.counts + (size_t)bounce * G.nseg;
            if (bounce > 0 && bounce >= tail_at) {
                launch_tail<TR, COUNT, MARCH>(L, B, G, in, cin, lds, st, T, tm, each);
                return launches + 1u;
            }
            uint32_t* cout = B.counts + (size_t)(bounce + 1u) * G.nseg;
            const int kc = bounce == 0 ? OM_KT_BOUNCE0 : OM_KT_BOUNCE;
            int ti = each ? tm.begin(st) : -1;
            const bool small = OM_WF_MARCH_REGS && L.S.n_msph <= MarchedSmall::KS && L.S.n_mbox <= MarchedSmall::KB &&
                               L.S.n_mtor <= MarchedSmall::KT;
            const bool exact = MarchedC2::matches(L.S.n_msph, L.S.n_mbox, L.S.n_mtor);
            if constexpr (exact_view_built<TR>()) {
                if (exact) {
                    if (OM_WF_MARCH_EXACT == 2)
                        hipLaunchKernelGGL((k_march<TR, COUNT, MV_EXACT_C2_LDS>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G,
                                           in, cin, B.hit, L.counters);
                    else
                        hipLaunchKernelGGL((k_march<TR, COUNT, MV_EXACT_C2>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, in,
                                           cin, B.hit, L.counters);
                    goto launched;
                }
            }
            if (small)
                hipLaunchKernelGGL((k_march<TR, COUNT, MV_SMALL>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, in, cin, B.hit, L.counters);
            else
                hipLaunchKernelGGL((k_march<TR, COUNT, MV_ARRAYS>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, in, cin, B.hit, L.counters);
        launched:
            tm.end(ti, kc, st);
            ti = each ? tm.begin(st) : -1;
            hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, false, true>), dim3(G.nseg), dim3(kBlk), 0, st, L.S, L.P, G, R, in,
                               cin, out, cout, B.res, B.res_id, L.counters, (const float2*)B.hit);
            tm.end(ti, kc, st);
            launches += 2u;
        }
        if (T.ev) { (void)hipEventRecord(T.ev, st); (void)hipStreamWaitEvent(T.st, T.ev, 0); }
        return launches;
    }
    Tail TT = T;
    const uint32_t cstride = G.nseg;                   // count arrays: one block of nseg per bounce
    for (uint32_t bounce = 0; bounce < depth_cap; ++bounce) {
        const Queue in = queue(B, bounce & 1u), out = queue(B, (bounce + 1u) & 1u);
        const uint32_t* cin = B.counts + (size_t)bounce * cstride;
        if (bounce > 0 && bounce >= tail_at) {
            launch_tail<TR, COUNT, MARCH>(L, B, G, in, cin, lds, st, TT, tm, each);
            return launches + 1u;
        }
        // async drain (OM_WF_DRAIN_AT, with async tails): from this bounce on, the batch's light
        // late bounces, its tail and its accumulate run on the tail stream, so the main stream
        // already starts the next batch's heavy bounces on another queue set
        if (OM_WF_DRAIN_AT > 0 && TT.ev && bounce == (uint32_t)OM_WF_DRAIN_AT) {
            (void)hipEventRecord(TT.ev, st);
            (void)hipStreamWaitEvent(TT.st, TT.ev, 0);
            st = TT.st;
            TT.ev = nullptr;
        }
        uint32_t* cout = B.counts + (size_t)(bounce + 1u) * cstride;
        // merged late bounces: this launch reads F segments per workgroup and writes the merged
        // geometry, which every later launch of the batch (and its tail) then uses
        Seg GL = G;
        if (OM_WF_MERGE_AT > 0 && OM_WF_MERGE > 1 && !OM_WF_DUAL && bounce == (uint32_t)OM_WF_MERGE_AT &&
            G.nseg >= 2u * OM_WF_MERGE) {
            // the last merged segment may take fewer input segments: its survivors still fit
            // the queue, as they never outnumber its inputs
            GL.nseg = (G.nseg + OM_WF_MERGE - 1u) / OM_WF_MERGE; GL.segcap = G.segcap * OM_WF_MERGE;
            GL.fin = OM_WF_MERGE; GL.segcap_in = G.segcap; GL.nseg_in = G.nseg;
            G.nseg = GL.nseg; G.segcap = GL.segcap;    // (k_tail takes any segment count)
        }
        const int ti = each ? tm.begin(st) : -1;
        if (bounce == 0)
            hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, true>), dim3(G.nseg), dim3(kBlk), lds, st, L.S, L.P, G, R, in,
                               cin, out, cout, B.res, B.res_id, L.counters, (const float2*)nullptr);
#if OM_WF_DUAL
        else if (TR == TR_BVH2_LDS && !MARCH)
            hipLaunchKernelGGL((k_bounce2<COUNT>), dim3(G.nseg), dim3(kBlk), lds + stack_bytes<TR_BVH2_LDS>(L.S), st, L.S,
                               L.P, G, in, cin, out, cout, B.res, B.res_id, L.counters);
#endif
        else if (OM_WF_LATE_GLOBAL > 0 && TR == TR_BVH2_LDS && bounce >= (uint32_t)OM_WF_LATE_GLOBAL)
            hipLaunchKernelGGL((k_bounce<TR_BVH2_GLOBAL, COUNT, MARCH, false>), dim3(GL.nseg), dim3(kBlk),
                               stack_bytes<TR_BVH2_GLOBAL>(L.S), st, L.S, L.P, GL, R, in, cin, out, cout, B.res, B.res_id,
                               L.counters, (const float2*)nullptr);
        else
            hipLaunchKernelGGL((k_bounce<TR, COUNT, MARCH, false>), dim3(GL.nseg), dim3(kBlk), lds, st, L.S, L.P, GL, R, in,
                               cin, out, cout, B.res, B.res_id, L.counters, (const float2*)nullptr);
        tm.end(ti, bounce == 0 ? OM_KT_BOUNCE0 : OM_KT_BOUNCE, st);
        if (T.stag && bounce == T.stag_at) (void)hipEventRecord(T.stag, st);
        ++launches;
    }
    if (TT.ev) { (void)hipEventRecord(TT.ev, st); (void)hipStreamWaitEvent(TT.st, TT.ev, 0); }
    return launches;
}

template <int TR>
uint32_t run_tr(bool count, bool march, QueueSet& B, const Launch& L, hipStream_t st, Seg G, const Gen& R,
                uint32_t depth_cap, uint32_t tail_at, uint32_t lds, const Tail& T) {
    if (count && march) return run_batch<TR, true, true>(B, L, st, G, R, depth_cap, tail_at, lds, T);
    if (count) return run_batch<TR, true, false>(B, L, st, G, R, depth_cap, tail_at, lds, T);
    if (march) return run_batch<TR, false, true>(B, L, st, G, R, depth_cap, tail_at, lds, T);
    return run_batch<TR, false, false>(B, L, st, G, R, depth_cap, tail_at, lds, T);
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
//   serial      (adaptive calls, or L.streams == 1) one batch after another on `st`; an
//               adaptive batch's bounce 0 reads the Stats its predecessor's accumulate wrote.
//   concurrent  (fixed spp, default) the call's samples split into batches of at most half
//               the call, dealt round-robin to L.streams streams (`st` + side streams), each
//               with its own queue set: two batches are in flight at once, so one batch's
//               latency-bound phases (the drain of every launch, the late bounces, the tail)
//               run beside the other's full ones.  Accumulates stay in sample order through
//               events (acc i after acc i-1) and the call ends joined on `st`.  Sample indices
//               come from the call-start Stats.n snapshot (n0), so every schedule renders
//               identical bits.
// Timing: mode 2 brackets the call once on `st` (OM_KT_BOUNCE_SPAN, with the call's
// bounce-family launch count); mode 1 brackets every launch on its stream and the call.
hipError_t render(Buffers& B, const Launch& L, hipStream_t st, std::string& err) {
    const uint32_t n_px = L.n_pixels;
    if (n_px == 0 || L.P.sample_count == 0) return hipSuccess;
    // paths per batch: 2^25 (33.5M, ~4.9 GB of queues per set; 16 spp of 1080p, the measured sweet
    // spot, §5.5), raised up to 16 spp of the frame for frames above 2M pixels, within 2^27 (~21 GB
    // per set, two sets; MI355X has 288 GB): a 4K frame (C4, 8.3M pixels) then runs 16-spp batches
    // like 1080p instead of 4-spp ones, whose 4x launches and 4x Stats read-modify-write per sample
    // cost C4 ~11% in k_accumulate alone (r03)
    const uint64_t kMaxPaths = std::min<uint64_t>(1ull << OM_WF_MAX_PATHS_LOG2,
                                                  std::max<uint64_t>(1ull << OM_WF_MIN_PATHS_LOG2, (uint64_t)OM_WF_BATCH_SPP * n_px));
    const uint32_t want = std::max<uint32_t>(1u, std::min<uint32_t>(L.streams, (uint32_t)kMaxSets));
    const bool concurrent = !L.P.adaptive && want >= 2u && L.P.sample_count >= 2u;
    uint32_t batch = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(L.P.sample_count, kMaxPaths / n_px));
    if (L.P.adaptive) batch = std::min<uint32_t>(batch, OM_WF_ADAPTIVE_BATCH);
    if (concurrent) batch = std::min<uint32_t>(batch, (L.P.sample_count + want - 1u) / want);
    const uint32_t nb = (L.P.sample_count + batch - 1u) / batch;
    const uint32_t ns = concurrent ? std::min<uint32_t>(want, nb) : 1u;
    // async tails (fixed spp, concurrent batches): each main stream alternates between two queue
    // sets, so a batch's tail and accumulate (on a tail stream) overlap the next batch's bounces
    const bool async_tail = OM_WF_ASYNC_TAIL && concurrent && ns >= 2u && 2u * ns <= (uint32_t)kMaxSets;
    const uint32_t nsets = async_tail ? std::min<uint32_t>(2u * ns, nb) : ns;
    const uint32_t depth_cap = L.P.max_depth > 1u ? L.P.max_depth : 1u;
    int dev = 0;
    (void)hipGetDevice(&dev);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t max_paths = (uint64_t)n_px * batch;
    int tr = L.trace_mode == TR_SBVH_LDS ? TR_SBVH_GLOBAL : L.trace_mode;
    if (tr == TR_BVH4_LDS) tr = L.S.n_b4nodes == 0 ? TR_BVH2_LDS : (L.S.b4_lds_bytes ? TR_BVH4_LDS : TR_BVH4_GLOBAL);
    // an empty BVH2 (no bounded sphere/cube: marched-only worlds, C2) takes the reference loop
    // when the old BVH holds at most one leaf: TR_BVH's 64-entry stack lives in scratch memory,
    // which every k_march / k_tail wave would then carry for nothing
    if (tr == TR_BVH2_LDS)
        tr = L.S.n_b2nodes == 0 ? (OM_EMPTY_B2_BRUTE && L.S.n_bvh_nodes <= 1u ? TR_BRUTE : TR_BVH) : (L.S.b2_lds_bytes ? TR_BVH2_LDS : TR_BVH2_GLOBAL);
    // segments, a multiple of the tail grouping: 4096 lanes per CU (8 workgroups of 512) for
    // traced worlds whose BVH2 sits in LDS, 8192 for marched worlds and L2-resident trees
    const bool march = (L.S.n_msph + L.S.n_mbox + L.S.n_mtor) != 0u;
    const uint32_t tail_at = L.tail_bounce ? L.tail_bounce
                           : march ? kTailMarched : tr == TR_BVH2_GLOBAL ? kTailL2
                           : max_paths > (1ull << 25) ? kTailBigBatch : kTailDefault;
    const uint32_t lanes_per_cu = (march || tr == TR_BVH2_GLOBAL) ? OM_WF_LANES_PER_CU_WIDE : OM_WF_LANES_PER_CU;
    uint32_t nseg = (uint32_t)std::min<uint64_t>((max_paths + kBlk - 1) / kBlk, (uint64_t)cus * (lanes_per_cu / kBlk));
    nseg = (nseg + kTailSpb - 1) / kTailSpb * kTailSpb;
    const uint32_t segcap = seg_capacity(max_paths, nseg);
    hipError_t e = grow(B, (uint64_t)nseg * segcap, (depth_cap + 1u) * nseg, (int)nsets);
    if (e != hipSuccess) { err = "wavefront buffer allocation failed"; return e; }
    const uint32_t lds = tr == TR_BVH2_LDS ? stack_bytes<TR_BVH2_LDS>(L.S) + L.S.b2_lds_bytes
                       : tr == TR_BVH2_GLOBAL ? stack_bytes<TR_BVH2_GLOBAL>(L.S) + hyb_nodes(L.S) * 64u
                       : tr == TR_BVH4_LDS ? stack_bytes<TR_BVH4_LDS>(L.S) + L.S.b4_lds_bytes
                       : tr == TR_BVH4_GLOBAL ? stack_bytes<TR_BVH4_GLOBAL>(L.S) : 0u;
    Gen R;
    R.C = L.C; R.jitter = L.jitter; R.stats = L.stats; R.pixels = L.pixels; R.n_pixels = n_px;
    R.by_pixel = L.stats_by_pixel ? 1u : 0u;
    R.tile_off = L.tile_off; R.tile_idx = L.tile_idx; R.tile_tnear = L.tile_tnear;
    R.n0 = nullptr; R.done = 0;
    hipStream_t streams[kMaxSets] = {st, st, st, st};
    Timer& tm = *L.timer;
    const int call_ti = tm.begin(st);
    if (!L.P.adaptive) {
        if (n_px > B.n0_cap) {
            if (B.n0) (void)hipFree(B.n0);
            B.n0 = nullptr; B.n0_cap = 0;
            if ((e = hipMalloc(&B.n0, (size_t)n_px * sizeof(uint32_t))) != hipSuccess) { err = "n0 allocation failed"; return e; }
            B.n0_cap = n_px;
        }
        hipLaunchKernelGGL(k_snapshot, dim3((n_px + 255u) / 256u), dim3(256), 0, st, L.stats, L.pixels, n_px,
                           R.by_pixel, B.n0);
        R.n0 = B.n0;
    }
    // events: [0] call start on `st`, [k] side stream k joined (or, async tails: [1], [2] tail
    // streams done), [kMaxSets + i] batch i accumulated; async tails: [kMaxSets + nb + i] batch
    // i's bounces launched (its tail waits on it)
    // accumulate stream: events [kMaxSets + i] batch i accumulated (as before), [kMaxSets + nb + i]
    // batch i rendered, [kMaxSets + 2nb] the stagger point, [kMaxSets + 2nb + 1] the accumulate
    // stream's end of call
    const bool acc_stream = OM_WF_ACC_STREAM && concurrent && ns >= 2u && !async_tail;
    const size_t ev_stag = kMaxSets + 2u * (size_t)nb, ev_accend = ev_stag + 1u;
    if (ns > 1) {
        if ((e = ensure_events(B, kMaxSets + 2u * nb + 2u)) != hipSuccess) { err = "event creation failed"; return e; }
        (void)hipEventRecord(B.ev[0], st);                       // side streams start after everything before the call
        for (uint32_t k = 1; k < ns; ++k) {
            if (!B.side[k] && (e = hipStreamCreateWithFlags(&B.side[k], hipStreamNonBlocking)) != hipSuccess) {
                err = "side stream creation failed"; return e;
            }
            streams[k] = B.side[k];
            (void)hipStreamWaitEvent(streams[k], B.ev[0], 0);
        }
        for (uint32_t k = 0; async_tail && k < 2u; ++k) {
            if (!B.tail[k]) {
                // high priority: the tail + accumulate chain is latency-bound and gates the reuse of
                // its queue set; the dispatcher serves its workgroups ahead of the bounce launches'.
                // Its own HW queue pool also keeps it off the main streams' in-order queues.
                int lo = 0, hi = 0;
                (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
                if ((e = hipStreamCreateWithPriority(&B.tail[k], hipStreamNonBlocking, OM_WF_TAIL_PRIO ? hi : lo)) != hipSuccess) {
                    err = "tail stream creation failed"; return e;
                }
            }
            (void)hipStreamWaitEvent(B.tail[k], B.ev[0], 0);
        }
    }
    if (acc_stream) {
        if (!B.acc && (e = hipStreamCreateWithFlags(&B.acc, hipStreamNonBlocking)) != hipSuccess) {
            err = "accumulate stream creation failed"; return e;
        }
        bool have = B.alt_cap >= B.cap;
        for (uint32_t k = 0; k < ns; ++k) have = have && B.alt_res[k] && B.alt_id[k];
        if (!have) {
            for (int k = 0; k < kMaxSets; ++k) {
                if (B.alt_res[k]) (void)hipFree(B.alt_res[k]);
                if (B.alt_id[k]) (void)hipFree(B.alt_id[k]);
                B.alt_res[k] = nullptr; B.alt_id[k] = nullptr;
            }
            B.alt_cap = 0;
            for (uint32_t k = 0; k < ns; ++k) {
                if ((e = hipMalloc(&B.alt_res[k], B.cap * sizeof(float4))) != hipSuccess ||
                    (e = hipMalloc(&B.alt_id[k], B.cap * sizeof(uint32_t))) != hipSuccess) {
                    err = "result buffer allocation failed"; return e;
                }
            }
            B.alt_cap = B.cap;
        }
        (void)hipStreamWaitEvent(B.acc, B.ev[0], 0);
    }
    uint32_t launches = 0;
    for (uint32_t i = 0, done = 0; i < nb; ++i) {
        const uint32_t b = std::min(batch, L.P.sample_count - done);
        const uint64_t paths = (uint64_t)n_px * b;
        hipStream_t si = streams[i % ns];
        // accumulate stream: odd rounds of a stream write the set's second result buffer, and a
        // result buffer is rewritten only once the batch that last wrote it is accumulated
        QueueSet QS = B.set[i % nsets];                          // (a shallow copy: pointers only)
        if (acc_stream) {
            if ((i / ns) & 1u) { QS.res = B.alt_res[i % ns]; QS.res_id = B.alt_id[i % ns]; }
            if (i >= 2u * ns) (void)hipStreamWaitEvent(si, B.ev[kMaxSets + i - 2u * ns], 0);
        }
        // async tails: batch i's tail + accumulate go on tail stream i % 2, behind its bounces; the
        // queue set is reused by batch i + nsets only after batch i is accumulated
        Tail TT{async_tail ? B.tail[i % 2u] : si, async_tail ? B.ev[kMaxSets + nb + i] : nullptr};
        if (OM_WF_STAGGER > 0 && ns > 1) {
            if (i == 0) { TT.stag = B.ev[ev_stag]; TT.stag_at = OM_WF_STAGGER; }
            if (i == 1) (void)hipStreamWaitEvent(si, B.ev[ev_stag], 0);
        }
        if (async_tail && i >= nsets) (void)hipStreamWaitEvent(si, B.ev[kMaxSets + i - nsets], 0);
        Seg G;
        G.nseg = nseg;
        G.segcap = seg_capacity(paths, nseg);
        R.batch = b;
        R.done = done;
        switch (tr) {
            case TR_BRUTE: launches += run_tr<TR_BRUTE>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            case TR_CULLED: launches += run_tr<TR_CULLED>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            case TR_BVH: launches += run_tr<TR_BVH>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            case TR_SBVH_GLOBAL: launches += run_tr<TR_SBVH_GLOBAL>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            case TR_BVH2_LDS: launches += run_tr<TR_BVH2_LDS>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            case TR_BVH4_LDS: launches += run_tr<TR_BVH4_LDS>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            case TR_BVH4_GLOBAL: launches += run_tr<TR_BVH4_GLOBAL>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
            default: launches += run_tr<TR_BVH2_GLOBAL>(L.count, march, QS, L, si, G, R, depth_cap, tail_at, lds, TT); break;
        }
        if (acc_stream) {                                            // accumulate stream: in order by itself
            (void)hipEventRecord(B.ev[kMaxSets + nb + i], si);
            (void)hipStreamWaitEvent(B.acc, B.ev[kMaxSets + nb + i], 0);
            si = B.acc;
        } else {
            if (async_tail) si = TT.st;                              // accumulate behind the tail
            if (ns > 1 && i > 0) (void)hipStreamWaitEvent(si, B.ev[kMaxSets + i - 1u], 0);   // Stats::add in sample order
        }
        const uint32_t grid_a = (n_px + kBlk - 1) / kBlk;
        const int ati = tm.mode == 1 ? tm.begin(si) : -1;
        if (L.count)
            hipLaunchKernelGGL(k_accumulate<true>, dim3(grid_a), dim3(kBlk), 0, si, L.P, L.stats, L.pixels, n_px,
                               L.stats_by_pixel ? 1u : 0u, b, QS.res, QS.res_id, L.S.bloom, L.counters);
        else
            hipLaunchKernelGGL(k_accumulate<false>, dim3(grid_a), dim3(kBlk), 0, si, L.P, L.stats, L.pixels, n_px,
                               L.stats_by_pixel ? 1u : 0u, b, QS.res, QS.res_id, L.S.bloom, L.counters);
        tm.end(ati, OM_KT_ACCUMULATE, si);
        // live progress: the cumulative credit after this batch, to the host word om_progress
        // hands out; ahead of the event the next batch's accumulate waits on, so the copies
        // land in order and the word only grows
        if (L.progress_host)
            (void)hipMemcpyAsync(L.progress_host, L.counters + OMC_PROGRESS, sizeof(unsigned long long),
                                 hipMemcpyDeviceToHost, si);
        if (ns > 1) (void)hipEventRecord(B.ev[kMaxSets + i], si);
        if ((e = hipGetLastError()) != hipSuccess) { err = "wavefront launch failed"; return e; }
        done += b;
    }
    if (async_tail) {                                             // the call ends joined on `st`: the
        for (uint32_t k = 0; k < 2u; ++k) {                       // tail streams end every batch (its
            (void)hipEventRecord(B.ev[1u + k], B.tail[k]);        // accumulate), behind its bounces
            (void)hipStreamWaitEvent(st, B.ev[1u + k], 0);
        }
        for (uint32_t k = 1; k < ns; ++k) {
            (void)hipEventRecord(B.ev[2u + k], streams[k]);
            (void)hipStreamWaitEvent(st, B.ev[2u + k], 0);
        }
    } else {
        for (uint32_t k = 1; k < ns; ++k) {
            (void)hipEventRecord(B.ev[k], streams[k]);
            (void)hipStreamWaitEvent(st, B.ev[k], 0);
        }
        if (acc_stream) {
            (void)hipEventRecord(B.ev[ev_accend], B.acc);
            (void)hipStreamWaitEvent(st, B.ev[ev_accend], 0);
        }
    }
    tm.end(call_ti, OM_KT_BOUNCE_SPAN, st, launches);
    return hipSuccess;
}

}  // namespace omw

#if OM_PHASE_STAMPS
// diagnostic build only: copy (and optionally clear) the phase sums
extern "C" int om_debug_phase_stamps(unsigned long long* out64, int reset) {
    if (hipMemcpyFromSymbol(out64, HIP_SYMBOL(omw::g_phase), sizeof(omw::g_phase)) != hipSuccess) return -1;
    if (reset) {
        static const unsigned long long zero[64] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(omw::g_phase), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
