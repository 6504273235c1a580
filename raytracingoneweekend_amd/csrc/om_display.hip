// om_display.hip — the reference's display modes (draw_to_sdl, main.rs:345-484, and
// apply_box_filter, main.rs:219-343) as image-space kernels: one lane per output pixel,
// reading the 40-B Stats of its 3x3 neighbourhood (served from L2 after the first
// touch), writing 3 bytes.  HBM-bound: ~40 B read + 3 B written per pixel.
// Bit-exact against oracle/om_oracle.cpp `display`: same f32 operation order, no FMA
// contraction, correctly rounded division, Rust `as u8` saturation.
#include "om_display.h"

#include <algorithm>

#include "om_device.h"

using namespace omd;

namespace omv {
namespace {

constexpr int kB = 256;
constexpr uint32_t kMaxBlocks = 1024;
constexpr float kSqrt2Inv = 0.7071067811865475244f;                         // utils.rs:31

__device__ __forceinline__ uint64_t scramble_d(uint64_t id) {              // utils.rs:46-56
    uint64_t id1 = id & 0xFFFFFFFFull;
    id1 ^= id1 << 13; id1 ^= id1 >> 7; id1 ^= id1 << 17;
    uint64_t id2 = id >> 32;
    id2 ^= id2 << 13; id2 ^= id2 >> 17; id2 ^= id2 << 5;
    return (id2 << 32) ^ id1 ^ (id1 * id2);
}

__device__ __forceinline__ void put(uint8_t* rgb, size_t k, F3 c) {       // normalize_color + to_u8x3
    rgb[3 * k + 0] = quantize(c.x);
    rgb[3 * k + 1] = quantize(c.y);
    rgb[3 * k + 2] = quantize(c.z);
}

// ---- max samples / max finite depth (main.rs:378-383, 397-403) -------------------------
// The reference scans pixels in order and replaces on strictly greater, so among equal
// maxima the first pixel wins (it matters for +-0): the reduction carries the index.
struct Part {
    uint32_t n;        // max Stats.n (starts at 1)
    float d;           // max finite avg_depth (starts at -1)
    uint32_t di;       // pixel index of d (0xFFFFFFFF = the initial -1, before every pixel)
    uint32_t pad;
};

__device__ __forceinline__ void merge(Part& a, const Part& b) {
    a.n = a.n > b.n ? a.n : b.n;
    const bool take = b.d > a.d || (b.d == a.d && (b.di + 1u) < (a.di + 1u));   // 0xFFFFFFFF + 1 = 0: the init is first
    if (take) { a.d = b.d; a.di = b.di; }
}

__global__ __launch_bounds__(kB) void k_maxes(const om_pixel_stats* __restrict__ st, uint32_t npx, Part* __restrict__ out) {
    __shared__ Part sh[kB];
    Part p; p.n = 1u; p.d = -1.0f; p.di = 0xFFFFFFFFu; p.pad = 0u;
    for (uint32_t k = blockIdx.x * kB + threadIdx.x; k < npx; k += gridDim.x * kB) {   // increasing k per lane
        const uint32_t n = st[k].n;
        if (n > p.n) p.n = n;
        const float d = st[k].avg_depth;
        if (d > p.d && !isinf(d)) { p.d = d; p.di = k; }
    }
    sh[threadIdx.x] = p;
    __syncthreads();
    for (int s = kB / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) { Part a = sh[threadIdx.x]; merge(a, sh[threadIdx.x + s]); sh[threadIdx.x] = a; }
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

__global__ __launch_bounds__(kB) void k_maxes_final(Part* __restrict__ parts, uint32_t nparts) {
    __shared__ Part sh[kB];
    Part p; p.n = 1u; p.d = -1.0f; p.di = 0xFFFFFFFFu; p.pad = 0u;
    for (uint32_t k = threadIdx.x; k < nparts; k += kB) merge(p, parts[k]);
    sh[threadIdx.x] = p;
    __syncthreads();
    for (int s = kB / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) { Part a = sh[threadIdx.x]; merge(a, sh[threadIdx.x + s]); sh[threadIdx.x] = a; }
        __syncthreads();
    }
    if (threadIdx.x == 0) parts[nparts] = sh[0];
}

// ---- per-pixel views: MODE_NORMAL 0, MODE_SHOW_SAMPLES 1, MODE_SHOW_DEPTH 3, MODE_SHOW_IDS 5
template <int MODE>
__global__ __launch_bounds__(kB) void k_view(const om_pixel_stats* __restrict__ st, uint32_t npx, const Part* __restrict__ mx,
                                             uint8_t* __restrict__ rgb) {
    const uint32_t k = blockIdx.x * kB + threadIdx.x;
    if (k >= npx) return;
    const om_pixel_stats& p = st[k];
    if (MODE == 0) {                                                                   // main.rs:374-381
        rgb[3 * k + 0] = p.color[0]; rgb[3 * k + 1] = p.color[1]; rgb[3 * k + 2] = p.color[2];
    } else if (MODE == 1) {                                                            // :384-394
        const float s = (float)p.n / (float)mx->n;
        put(rgb, k, f3(s, s, s));
    } else if (MODE == 3) {                                                            // :404-414
        const float d01 = p.avg_depth / mx->d;
        const bool inf = isinf(d01);
        const float rb = inf ? 0.0f : d01, g = inf ? 1.0f : d01;
        put(rgb, k, f3(rb, g, rb));
    } else {                                                                           // :425-433, utils.rs:59-70
        const uint64_t id = scramble_d(p.bloom);
        uint8_t b[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) b[i] = (uint8_t)((id >> (8 * i)) & 0xFFu);
        rgb[3 * k + 0] = b[0] ^ b[7] ^ b[3];
        rgb[3 * k + 1] = b[1] ^ b[4] ^ b[5];
        rgb[3 * k + 2] = b[2] ^ b[6];
    }
}

// ---- the three 3x3 blurs (apply_box_filter_ij_samples/_depth/_id, main.rs:219-312) --------
// Coverage and neighbourhoods of apply_box_filter (main.rs:322-343): interior pixels use
// the full 3x3; top/bottom lines only exist when H >= 3 (they are visited inside the j
// loop), left/right lines for 1 <= j <= H-2, the four corners always.
template <int F>
__global__ __launch_bounds__(kB) void k_blur(const om_pixel_stats* __restrict__ st, uint32_t W, uint32_t H,
                                             uint8_t* __restrict__ rgb) {
    const uint32_t k = blockIdx.x * kB + threadIdx.x;
    if (k >= W * H) return;
    const uint32_t j = k / W, i = k - j * W;
    const bool ie = i == 0 || i == W - 1, je = j == 0 || j == H - 1;
    const bool covered = (ie && je) || (!je && H >= 3) || (je && !ie && H >= 3);
    if (!covered) return;
    const int min_x = i == 0 ? 0 : -1, max_x = i == W - 1 ? 0 : 1;
    const int min_y = j == 0 ? 0 : -1, max_y = j == H - 1 ? 0 : 1;
    const om_pixel_stats& me = st[k];
    const float di = me.avg_depth;
    if (F == 1 && isinf(di)) {                                                         // main.rs:250-257
        rgb[3 * k + 0] = me.color[0]; rgb[3 * k + 1] = me.color[1]; rgb[3 * k + 2] = me.color[2];
        return;
    }
    const uint64_t state = me.bloom;
    float total_weight = 0.0f;
    F3 color = f3(0.0f, 0.0f, 0.0f);
    for (int y = min_y; y <= max_y; ++y) {
        for (int x = min_x; x <= max_x; ++x) {
            const om_pixel_stats& q = st[(size_t)((int)i + x) + (size_t)((int)j + y) * W];
            const float is_diagonal = (x != 0 && y != 0) ? 1.0f : 0.0f;
            const F3 sum = f3(q.sum[0], q.sum[1], q.sum[2]);
            if (F == 0) {
                const float n = (float)q.n;
                const float diag_w = 1.0f - (1.0f - kSqrt2Inv) * is_diagonal;
                total_weight = total_weight + n * diag_w;
                color = add(color, scl(sum, diag_w));
            } else {
                float w;
                if (F == 1) {
                    w = 1.0f / (1.0f + fabsf(q.avg_depth - di));
                } else {
                    const float same_value = q.bloom == state ? 1.0f : 0.0f;
                    const float partial_value = (q.bloom & state) == state ? 1.0f : 0.0f;
                    w = same_value + partial_value;
                }
                const float diag_w = w * (1.0f - (1.0f - kSqrt2Inv) * is_diagonal);
                total_weight = total_weight + diag_w;
                const F3 c = scl(sum, 1.0f / (float)q.n);                              // Vec3 / f32 (vec3.rs:236-240)
                color = add(color, scl(c, diag_w));
            }
        }
    }
    put(rgb, k, scl(color, 1.0f / total_weight));
}

uint32_t max_blocks(uint32_t npx) { return std::max(1u, std::min(kMaxBlocks, (npx + kB - 1) / kB)); }

}  // namespace

size_t scratch_bytes(uint32_t width, uint32_t height) {
    return (size_t)(max_blocks(width * height) + 1u) * sizeof(Part);
}

hipError_t render(const om_pixel_stats* st, uint32_t W, uint32_t H, int mode, uint8_t* rgb, void* scratch, hipStream_t s) {
    const uint32_t npx = W * H;
    const uint32_t grid = (npx + kB - 1) / kB;
    Part* parts = (Part*)scratch;
    if (mode == OM_VIEW_SAMPLES || mode == OM_VIEW_DEPTH) {
        const uint32_t nb = max_blocks(npx);
        hipLaunchKernelGGL(k_maxes, dim3(nb), dim3(kB), 0, s, st, npx, parts);
        hipLaunchKernelGGL(k_maxes_final, dim3(1), dim3(kB), 0, s, parts, nb);
        parts += nb;                                                                   // the final Part
    }
    switch (mode) {
        case OM_VIEW_NORMAL: hipLaunchKernelGGL(k_view<0>, dim3(grid), dim3(kB), 0, s, st, npx, parts, rgb); break;
        case OM_VIEW_SAMPLES: hipLaunchKernelGGL(k_view<1>, dim3(grid), dim3(kB), 0, s, st, npx, parts, rgb); break;
        case OM_VIEW_DEPTH: hipLaunchKernelGGL(k_view<3>, dim3(grid), dim3(kB), 0, s, st, npx, parts, rgb); break;
        case OM_VIEW_IDS: hipLaunchKernelGGL(k_view<5>, dim3(grid), dim3(kB), 0, s, st, npx, parts, rgb); break;
        case OM_VIEW_SAMPLE_BLUR: hipLaunchKernelGGL(k_blur<0>, dim3(grid), dim3(kB), 0, s, st, W, H, rgb); break;
        case OM_VIEW_DEPTH_BLUR: hipLaunchKernelGGL(k_blur<1>, dim3(grid), dim3(kB), 0, s, st, W, H, rgb); break;
        default: hipLaunchKernelGGL(k_blur<2>, dim3(grid), dim3(kB), 0, s, st, W, H, rgb); break;
    }
    return hipGetLastError();
}

}  // namespace omv
