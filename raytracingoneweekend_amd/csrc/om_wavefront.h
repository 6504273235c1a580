// om_wavefront.h — host interface of the wavefront pipeline.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"
#include "om_layout.h"

namespace omw {

// One batch's device work buffers: ping-pong path queues, result slots, per-bounce counts.
struct QueueSet {
    float4* q[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};  // ping-pong queues: o|depthf, d|first_id, cur|seg
    uint4* qr[2] = {nullptr, nullptr};   // rng lo, rng hi, path slot, pad
    float4* res = nullptr;       // colour.xyz, depth
    uint32_t* res_id = nullptr;  // obj id (0xFFFFFFFF = no sample)
    uint32_t* counts = nullptr;  // per bounce, per queue segment: live rays
    float2* hit = nullptr;       // split march pipeline: (closest, winner) per queue slot
    void release();
};

// Device work buffers of one context; grown on demand, never shrunk.  kMaxSets queue sets
// let that many batches be in flight at once (overlapped schedule): batch
// i uses set i % S on stream i % S (stream 0 = the caller's stream, the others `side`).
constexpr int kMaxSets = 4;
struct Buffers {
    uint64_t cap = 0;            // paths per batch (per set)
    uint32_t counts_n = 0;       // count words per set
    int nsets = 0;               // sets allocated at `cap`
    QueueSet set[kMaxSets];
    uint32_t* n0 = nullptr;      // fixed spp: per listed pixel, the call-start Stats.n (Gen::n0); adaptive: live lists + plans
    uint64_t n0_cap = 0;
    hipStream_t side[kMaxSets] = {};  // streams 1.. of the overlapped schedule
    std::vector<hipEvent_t> ev;  // cross-stream ordering events (timing disabled)
    void release();
};

// Optional device timing (om_set_timing): HIP event pairs on the launch stream.  Mode 1
// brackets every launch (tagged with its OM_KT_* class) and the call; mode 2 brackets only
// the call (OM_KT_BOUNCE_SPAN, with its bounce-family launch count): two events per call.
struct Timer {
    int mode = 0;
    std::vector<hipEvent_t> ev;   // pool, pairs (2i, 2i+1)
    std::vector<int> cls;         // class of pair i since the last read (-1: open)
    std::vector<uint32_t> nl;     // launches inside pair i
    bool on() const { return mode != 0; }
    // Opens pair i (recorded on `st`) and returns i; pairs may nest (a call around its launches).
    int begin(hipStream_t st) {
        if (!on()) return -1;
        const size_t i = cls.size();
        while (ev.size() < 2 * i + 2) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) { mode = 0; return -1; }
            ev.push_back(e);
        }
        (void)hipEventRecord(ev[2 * i], st);
        cls.push_back(-1);
        nl.push_back(0);
        return (int)i;
    }
    void end(int i, int c, hipStream_t st, uint32_t launches = 1) {
        if (!on() || i < 0) return;
        (void)hipEventRecord(ev[2 * i + 1], st);
        cls[i] = c;
        nl[i] = launches;
    }
    void clear() { cls.clear(); nl.clear(); }
    void release() { for (auto e : ev) (void)hipEventDestroy(e); ev.clear(); clear(); }
};

struct Launch {
    OmSceneDev S;
    OmCamDev C;
    OmParamsDev P;
    const float2* jitter;
    om_pixel_stats* stats;
    const uint32_t* pixels;      // device list of row-major pixel indices (tile order)
    uint32_t n_pixels;
    bool stats_by_pixel;         // stats[pixel] (full frame) instead of stats[k]
    unsigned long long* counters;
    bool count;
    int trace_mode;              // closest-hit kernel variant (om_render.hip MODE_*)
    uint32_t tail_bounce;        // first bounce run by the persistent tail kernel (0 = default)
    uint32_t streams;            // batches in flight (queue sets, streams), 1 = serial, <= kMaxSets
    uint32_t ad_batches;         // adaptive calls: batches per stream per call (0 = OM_WF_ADAPTIVE_BATCHES)
    uint32_t ad_paths_log2;      // adaptive calls: log2 of the target paths per batch (0 = OM_WF_ADAPTIVE_PATHS_LOG2)
    Timer* timer;                // per-launch event timing (may be off)
    const uint32_t* tile_off;    // primary-ray candidate lists per 8x8 tile (null = traverse the BVH)
    const uint16_t* tile_idx;
    const float* tile_tnear;     // per leaf record: lower bound of a primary ray's t to its box (lists sorted by it)
    unsigned long long* progress_host;   // om_progress word (pinned host) or null; device side counters[OMC_PROGRESS]
};

// Renders P.sample_count samples of every listed pixel; returns 0 or a HIP error text.
hipError_t render(Buffers& B, const Launch& L, hipStream_t stream, std::string& err);

}  // namespace omw
