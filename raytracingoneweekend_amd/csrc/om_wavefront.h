// om_wavefront.h — host interface of the wavefront pipeline.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"
#include "om_layout.h"

namespace omw {

// Device work buffers of one context; grown on demand, never shrunk.
struct Buffers {
    uint64_t cap = 0;            // paths per batch
    float4* q[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};  // ping-pong queues: o|depthf, d|first_id, cur|seg
    uint4* qr[2] = {nullptr, nullptr};   // rng lo, rng hi, path slot, pad
    float4* res = nullptr;       // colour.xyz, depth
    uint32_t* res_id = nullptr;  // obj id (0xFFFFFFFF = no sample)
    uint32_t* counts = nullptr;  // per bounce, per queue segment: live rays
    uint32_t counts_n = 0;       // words allocated
    void release();
};

// Optional device timing (om_set_timing): HIP event pairs on the launch stream.  Mode 1
// brackets every launch (tagged with its OM_KT_* class); mode 2 brackets the whole
// bounce-kernel family of a batch once (OM_KT_BOUNCE_SPAN, with its launch count), which
// costs two events per batch instead of two per launch.
struct Timer {
    int mode = 0;
    std::vector<hipEvent_t> ev;   // pool, pairs (2i, 2i+1)
    std::vector<int> cls;         // class of pair i since the last read
    std::vector<uint32_t> nl;     // launches inside pair i
    bool on() const { return mode != 0; }
    void begin(hipStream_t st) {
        if (!on()) return;
        const size_t i = 2 * cls.size();
        while (ev.size() < i + 2) {
            hipEvent_t e = nullptr;
            if (hipEventCreate(&e) != hipSuccess) { mode = 0; return; }
            ev.push_back(e);
        }
        (void)hipEventRecord(ev[i], st);
    }
    void end(int c, hipStream_t st, uint32_t launches = 1) {
        if (!on()) return;
        (void)hipEventRecord(ev[2 * cls.size() + 1], st);
        cls.push_back(c);
        nl.push_back(launches);
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
    Timer* timer;                // per-launch event timing (may be off)
    const uint32_t* tile_off;    // primary-ray candidate lists per 8x8 tile (null = traverse the BVH)
    const uint16_t* tile_idx;
};

// Renders P.sample_count samples of every listed pixel; returns 0 or a HIP error text.
hipError_t render(Buffers& B, const Launch& L, hipStream_t stream, std::string& err);

}  // namespace omw
