// om_multi.hip — multi-GPU frames: 8x8 pixel-tile shards dealt round-robin to ranks and the
// framebuffer gathered to rank 0 over RCCL (xGMI).  Re-design of the reference's pixel deal to
// its render threads (main.rs:170-214: 2730-pixel chunks round-robin, one shared framebuffer);
// DESIGN.md §6.
//
// Data path of one frame (C4: 3840x2160, 8 ranks):
//   every rank renders its tiles into a compact shard (40-B om_pixel_stats in list order,
//   om_shard_capacity entries, HBM-resident across progressive calls);
//   gather: one RCCL group of send/recv per rank (rank 0 receives all shards, its own
//   included, into a staging buffer of nranks x capacity), then one scatter launch per rank
//   on rank 0 moves each shard to its pixels (k_shard_to_frame: 40 B read + 40 B written per
//   pixel, HBM-bound, coalesced 8-B words).
// The 332-MB C4 frame puts 41.5 MB on each peer's own xGMI link into rank 0 (~0.3 ms at
// ~150 GB/s), against seconds of rendering.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"
#include "om_internal.h"
#include "om_shard.h"

using oms::capacity;
using oms::deal;

namespace {

constexpr uint32_t kWords = sizeof(om_pixel_stats) / 8;   // 5 u64 words per pixel
static_assert(sizeof(om_pixel_stats) == 40, "om_pixel_stats layout");

// one lane per 8-B word: the shard side is read/written fully coalesced; the frame side in
// runs of 8 pixels (320 B) per tile row
__global__ void __launch_bounds__(256) k_shard_to_frame(const uint64_t* __restrict__ shard, const uint32_t* __restrict__ list,
                                                        uint32_t n, uint64_t* __restrict__ frame) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)n * kWords) return;
    const uint32_t k = (uint32_t)(i / kWords), w = (uint32_t)(i % kWords);
    frame[(uint64_t)list[k] * kWords + w] = shard[i];
}

__global__ void __launch_bounds__(256) k_frame_to_shard(const uint64_t* __restrict__ frame, const uint32_t* __restrict__ list,
                                                        uint32_t n, uint64_t* __restrict__ shard) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)n * kWords) return;
    const uint32_t k = (uint32_t)(i / kWords), w = (uint32_t)(i % kWords);
    shard[i] = frame[(uint64_t)list[k] * kWords + w];
}

hipError_t launch_move(bool to_frame, const void* src, const uint32_t* list, uint32_t n, void* dst, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t words = (uint64_t)n * kWords;
    const uint32_t blocks = (uint32_t)((words + 255) / 256);
    if (to_frame)
        hipLaunchKernelGGL(k_shard_to_frame, dim3(blocks), dim3(256), 0, st, (const uint64_t*)src, list, n, (uint64_t*)dst);
    else
        hipLaunchKernelGGL(k_frame_to_shard, dim3(blocks), dim3(256), 0, st, (const uint64_t*)src, list, n, (uint64_t*)dst);
    return hipGetLastError();
}

// Test hook (tests/test_multi_gpu.py): OM_DEBUG_FAIL_ALLOC=<bytes> makes every DBuf allocation
// of at least that many bytes fail as if the device were out of memory, so the error and retry
// paths of the shard bookkeeping can be exercised without exhausting 288 GB of HBM.
bool debug_fail_alloc(size_t bytes) {
    const char* v = std::getenv("OM_DEBUG_FAIL_ALLOC");
    return v && *v && bytes >= (size_t)std::strtoull(v, nullptr, 10);
}

struct DBuf {
    void* p = nullptr;
    size_t n = 0;
    int dev = -1;
    hipError_t ensure(int device, size_t bytes) {
        if (p && n >= bytes && dev == device) return hipSuccess;
        release();
        if (debug_fail_alloc(bytes)) return hipErrorOutOfMemory;
        hipError_t e = hipSetDevice(device);
        if (e == hipSuccess) e = hipMalloc(&p, std::max<size_t>(bytes, 16));
        if (e != hipSuccess) { p = nullptr; return e; }
        n = bytes; dev = device;
        return hipSuccess;
    }
    void release() {
        if (p) { (void)hipSetDevice(dev); (void)hipFree(p); }
        p = nullptr; n = 0; dev = -1;
    }
};

// The tile deal of one (W, H, nranks), as device lists: rank `mine`'s list on its device and,
// on rank 0, every rank's list (for the scatter/cut launches).
struct Deal {
    uint32_t w = 0, h = 0, nranks = 0, cap = 0;
    std::vector<uint32_t> count, offset;   // per rank: pixels, offset into `all`
    DBuf all;                              // every rank's list, rank-major (root device)
    bool valid(uint32_t W, uint32_t H, uint32_t N) const { return all.p && w == W && h == H && nranks == N; }
    hipError_t build(uint32_t W, uint32_t H, uint32_t N, int root_dev) {
        w = W; h = H; nranks = N; cap = capacity(W, H, N);
        count.assign(N, 0); offset.assign(N, 0);
        std::vector<uint32_t> lst, cat;
        cat.reserve((size_t)W * H);
        for (uint32_t r = 0; r < N; ++r) {
            deal(W, H, r, N, lst);
            offset[r] = (uint32_t)cat.size();
            count[r] = (uint32_t)lst.size();
            cat.insert(cat.end(), lst.begin(), lst.end());
        }
        hipError_t e = all.ensure(root_dev, cat.size() * 4);
        if (e == hipSuccess) e = hipMemcpy(all.p, cat.data(), cat.size() * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) all.release();
        return e;
    }
    const uint32_t* list(uint32_t r) const { return (const uint32_t*)all.p + offset[r]; }
};

std::string nccl_msg(const char* what, ncclResult_t r) { return std::string(what) + ": " + ncclGetErrorString(r); }

}  // namespace

// ---------------------------------------------------------------------------
// one rank per process
// ---------------------------------------------------------------------------
struct om_comm {
    om_ctx* ctx = nullptr;
    int device = 0;
    uint32_t nranks = 1, rank = 0;
    ncclComm_t nc = nullptr;
    Deal deal;                // every rank's list on this rank's device (root scatters with all of them)
    DBuf staging;             // root: nranks x capacity shards
};

namespace {

om_status comm_lists(om_comm* c, uint32_t W, uint32_t H) {
    if (c->deal.valid(W, H, c->nranks)) return OM_OK;
    const hipError_t e = c->deal.build(W, H, c->nranks, c->device);
    if (e != hipSuccess) return omi::ctx_error(c->ctx, OM_ERR_DEVICE, std::string("shard lists: ") + hipGetErrorString(e));
    return OM_OK;
}

om_status check_frame(om_ctx* ctx, uint32_t W, uint32_t H) {
    if (W == 0 || H == 0 || (uint64_t)W * H > (1ull << 31)) return omi::ctx_error(ctx, OM_ERR_INVALID, "bad frame size");
    return OM_OK;
}

}  // namespace

extern "C" {

om_status om_rccl_library(char* path, uint32_t path_bytes, int32_t* version) {
    if (path && path_bytes) {
        Dl_info info{};
        const char* f = dladdr((void*)&ncclGetUniqueId, &info) && info.dli_fname ? info.dli_fname : "";
        std::strncpy(path, f, path_bytes - 1);
        path[path_bytes - 1] = '\0';
    }
    if (version) {
        int v = 0;
        const ncclResult_t r = ncclGetVersion(&v);
        if (r != ncclSuccess) return omi::global_error(OM_ERR_DEVICE, nccl_msg("ncclGetVersion", r));
        *version = v;
    }
    return OM_OK;
}

om_status om_comm_unique_id(uint8_t id[OM_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == OM_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id) return omi::global_error(OM_ERR_INVALID, "om_comm_unique_id: null id");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return omi::global_error(OM_ERR_DEVICE, nccl_msg("ncclGetUniqueId", r));
    std::memcpy(id, &u, sizeof(u));
    return OM_OK;
}

om_status om_comm_init_rank(om_ctx* ctx, uint32_t nranks, uint32_t rank, const uint8_t id[OM_COMM_ID_BYTES], om_comm** out) {
    if (!ctx || !id || !out || nranks == 0 || rank >= nranks)
        return omi::global_error(OM_ERR_INVALID, "om_comm_init_rank: bad argument");
    *out = nullptr;
    om_comm* c = new (std::nothrow) om_comm();
    if (!c) return omi::ctx_error(ctx, OM_ERR_NOMEM, "om_comm_init_rank: out of memory");
    c->ctx = ctx; c->device = omi::ctx_device(ctx); c->nranks = nranks; c->rank = rank;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) { delete c; return omi::ctx_error(ctx, OM_ERR_DEVICE, hipGetErrorString(e)); }
    const ncclResult_t r = ncclCommInitRank(&c->nc, (int)nranks, u, (int)rank);
    if (r != ncclSuccess) { delete c; return omi::ctx_error(ctx, OM_ERR_DEVICE, nccl_msg("ncclCommInitRank", r)); }
    *out = c;
    return OM_OK;
}

void om_comm_destroy(om_comm* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->nc) (void)ncclCommDestroy(c->nc);
    c->deal.all.release(); c->staging.release();
    delete c;
}

om_status om_comm_info(const om_comm* c, int32_t* nranks, int32_t* rank) {
    if (!c || !nranks || !rank) return omi::global_error(OM_ERR_INVALID, "om_comm_info: null argument");
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(c->nc, &n);
    if (e == ncclSuccess) e = ncclCommUserRank(c->nc, &r);
    if (e != ncclSuccess) return omi::ctx_error(c->ctx, OM_ERR_DEVICE, nccl_msg("om_comm_info", e));
    *nranks = n; *rank = r;
    return OM_OK;
}

om_status om_render_shard(om_comm* c, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_shard, void* stream) {
    if (!c || !p) return omi::global_error(OM_ERR_INVALID, "om_render_shard: null argument");
    om_status s = check_frame(c->ctx, p->width, p->height);
    if (s || (s = comm_lists(c, p->width, p->height))) return s;
    const uint32_t n = c->deal.count[c->rank];
    // device list of this rank's pixels on its own device (root: the rank-major table)
    return om_render_device_pixels(c->ctx, cam, p, dev_shard, c->deal.list(c->rank), n, stream);
}

om_status om_gather_frame(om_comm* c, const om_pixel_stats* dev_shard, uint32_t W, uint32_t H, om_pixel_stats* dev_frame,
                          void* stream) {
    if (!c) return omi::global_error(OM_ERR_INVALID, "om_gather_frame: null comm");
    om_status s = check_frame(c->ctx, W, H);
    if (s || (s = comm_lists(c, W, H))) return s;
    const bool root = c->rank == 0;
    if ((!dev_shard && c->deal.count[c->rank]) || (root && !dev_frame))
        return omi::ctx_error(c->ctx, OM_ERR_INVALID, "om_gather_frame: null shard/frame");
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return omi::ctx_error(c->ctx, OM_ERR_DEVICE, hipGetErrorString(e));
    hipStream_t st = stream ? (hipStream_t)stream : omi::ctx_stream(c->ctx);
    const size_t cap_b = (size_t)c->deal.cap * sizeof(om_pixel_stats);
    if (root && (e = c->staging.ensure(c->device, cap_b * c->nranks)) != hipSuccess)
        return omi::ctx_error(c->ctx, OM_ERR_DEVICE, std::string("gather staging: ") + hipGetErrorString(e));
    ncclResult_t r = ncclGroupStart();
    const size_t mine_b = (size_t)c->deal.count[c->rank] * sizeof(om_pixel_stats);
    if (r == ncclSuccess && mine_b) r = ncclSend(dev_shard, mine_b, ncclUint8, 0, c->nc, st);
    for (uint32_t q = 0; root && r == ncclSuccess && q < c->nranks; ++q) {
        const size_t b = (size_t)c->deal.count[q] * sizeof(om_pixel_stats);
        if (b) r = ncclRecv((char*)c->staging.p + q * cap_b, b, ncclUint8, (int)q, c->nc, st);
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return omi::ctx_error(c->ctx, OM_ERR_DEVICE, nccl_msg("om_gather_frame send/recv", r != ncclSuccess ? r : r2));
    for (uint32_t q = 0; root && q < c->nranks; ++q)
        if ((e = launch_move(true, (char*)c->staging.p + q * cap_b, c->deal.list(q), c->deal.count[q], dev_frame, st)) != hipSuccess)
            return omi::ctx_error(c->ctx, OM_ERR_DEVICE, std::string("k_shard_to_frame: ") + hipGetErrorString(e));
    return OM_OK;
}

om_status om_scatter_frame(om_comm* c, const om_pixel_stats* dev_frame, uint32_t W, uint32_t H, om_pixel_stats* dev_shard,
                           void* stream) {
    if (!c) return omi::global_error(OM_ERR_INVALID, "om_scatter_frame: null comm");
    om_status s = check_frame(c->ctx, W, H);
    if (s || (s = comm_lists(c, W, H))) return s;
    const bool root = c->rank == 0;
    if ((!dev_shard && c->deal.count[c->rank]) || (root && !dev_frame))
        return omi::ctx_error(c->ctx, OM_ERR_INVALID, "om_scatter_frame: null shard/frame");
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) return omi::ctx_error(c->ctx, OM_ERR_DEVICE, hipGetErrorString(e));
    hipStream_t st = stream ? (hipStream_t)stream : omi::ctx_stream(c->ctx);
    const size_t cap_b = (size_t)c->deal.cap * sizeof(om_pixel_stats);
    if (root) {
        if ((e = c->staging.ensure(c->device, cap_b * c->nranks)) != hipSuccess)
            return omi::ctx_error(c->ctx, OM_ERR_DEVICE, std::string("scatter staging: ") + hipGetErrorString(e));
        for (uint32_t q = 0; q < c->nranks; ++q)
            if ((e = launch_move(false, dev_frame, c->deal.list(q), c->deal.count[q], (char*)c->staging.p + q * cap_b, st)) != hipSuccess)
                return omi::ctx_error(c->ctx, OM_ERR_DEVICE, std::string("k_frame_to_shard: ") + hipGetErrorString(e));
    }
    ncclResult_t r = ncclGroupStart();
    for (uint32_t q = 0; root && r == ncclSuccess && q < c->nranks; ++q) {
        const size_t b = (size_t)c->deal.count[q] * sizeof(om_pixel_stats);
        if (b) r = ncclSend((char*)c->staging.p + q * cap_b, b, ncclUint8, (int)q, c->nc, st);
    }
    const size_t mine_b = (size_t)c->deal.count[c->rank] * sizeof(om_pixel_stats);
    if (r == ncclSuccess && mine_b) r = ncclRecv(dev_shard, mine_b, ncclUint8, 0, c->nc, st);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return omi::ctx_error(c->ctx, OM_ERR_DEVICE, nccl_msg("om_scatter_frame send/recv", r != ncclSuccess ? r : r2));
    return OM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// one process, several GPUs
// ---------------------------------------------------------------------------
// The shards stay resident on their GPUs across progressive calls, as the reference's render
// threads keep writing one shared framebuffer with no per-pass copy (main.rs:192-214): a
// frame is dealt out once, when om_multi_render first sees it (its device pointer and size),
// and comes back only when om_multi_gather asks for it.
struct om_multi {
    std::vector<om_ctx*> ctx;
    std::vector<int> dev;
    int transport = OM_TRANSPORT_RCCL;
    std::vector<ncclComm_t> nc;        // RCCL: one communicator per rank (ncclCommInitAll)
    Deal deal;                          // every rank's list on devices[0]
    std::vector<DBuf> list;             // per rank r > 0: its list on its device
    std::vector<DBuf> shard;            // per rank: its shard on its device (HBM-resident)
    std::vector<DBuf> staging;          // per rank r > 0: its shard's image on devices[0]
    std::vector<hipEvent_t> ev;         // [0] on devices[0]: frame cut / gather done; [r]: rank r's stream
    bool ev0_live = false;              // ev[0] has been recorded (the ranks' streams wait on it)
    hipEvent_t done0 = nullptr;         // on devices[0]: rank 0's last render
    bool renders_live = false;          // done0 and ev[r >= 1] have been recorded by a render
    const void* bound = nullptr;        // the device frame whose shards are resident
    uint32_t bw = 0, bh = 0;
    DBuf host_frame;                    // om_multi_render_host: the frame on devices[0]
    std::string err;
};

namespace {

om_status merr(om_multi* m, om_status code, const std::string& msg) {
    if (m) m->err = msg;
    return omi::global_error(code, msg);
}

#define OM_MHIP(m, call)                                                                                 \
    do {                                                                                                 \
        hipError_t e_ = (call);                                                                          \
        if (e_ != hipSuccess) return merr(m, OM_ERR_DEVICE, std::string(#call ": ") + hipGetErrorString(e_)); \
    } while (0)

om_status multi_lists_build(om_multi* m, uint32_t W, uint32_t H) {
    const uint32_t N = (uint32_t)m->ctx.size();
    OM_MHIP(m, m->deal.build(W, H, N, m->dev[0]));
    std::vector<uint32_t> lst;
    const size_t cap_b = (size_t)m->deal.cap * sizeof(om_pixel_stats);
    for (uint32_t r = 0; r < N; ++r) {
        OM_MHIP(m, m->shard[r].ensure(m->dev[r], cap_b));
        OM_MHIP(m, hipMemset(m->shard[r].p, 0, cap_b));
        if (r == 0) continue;
        deal(W, H, r, N, lst);
        OM_MHIP(m, m->list[r].ensure(m->dev[r], std::max<size_t>(lst.size(), 1) * 4));
        if (!lst.empty()) OM_MHIP(m, hipMemcpy(m->list[r].p, lst.data(), lst.size() * 4, hipMemcpyHostToDevice));
        OM_MHIP(m, m->staging[r].ensure(m->dev[0], cap_b));
    }
    return OM_OK;
}

// The deal's lists, shards and staging buffers for (W, H).  The deal counts as built only once
// every per-rank buffer is in place: a failure part-way (an allocation, a copy) releases the
// rank-major table, so the next call rebuilds everything instead of launching on missing or
// undersized buffers.  A new deal forgets the resident frame.
om_status multi_lists(om_multi* m, uint32_t W, uint32_t H) {
    if (m->deal.valid(W, H, (uint32_t)m->ctx.size())) return OM_OK;
    m->bound = nullptr;
    const om_status s = multi_lists_build(m, W, H);
    if (s != OM_OK) m->deal.all.release();
    return s;
}

std::vector<hipStream_t> rank_streams(om_multi* m, void* stream) {
    std::vector<hipStream_t> st(m->ctx.size());
    for (size_t r = 0; r < st.size(); ++r) st[r] = omi::ctx_stream(m->ctx[r]);
    if (stream) st[0] = (hipStream_t)stream;
    return st;
}

// ev[0] on st[0], and every rank's stream waits on it.
om_status fence_from_root(om_multi* m, const std::vector<hipStream_t>& st) {
    OM_MHIP(m, hipSetDevice(m->dev[0]));
    OM_MHIP(m, hipEventRecord(m->ev[0], st[0]));
    m->ev0_live = true;
    for (size_t r = 1; r < st.size(); ++r) {
        OM_MHIP(m, hipSetDevice(m->dev[r]));
        OM_MHIP(m, hipStreamWaitEvent(st[r], m->ev[0], 0));
    }
    return OM_OK;
}

// Rank 0 cuts dev_frame into the shards (its own in place, the others' into staging) and deals
// them out: the frame becomes the resident one.  The shards and staging buffers it overwrites
// may still be in use by the previous frame's work: every rank's last render (a frame re-dealt
// with no gather in between: render(A), render(B)) and the last gather's reads of staging, on
// whatever stream those calls were given.  So st[0] first waits on all of them.
om_status deal_frame(om_multi* m, const om_pixel_stats* dev_frame, const std::vector<hipStream_t>& st) {
    const uint32_t N = (uint32_t)m->ctx.size();
    const Deal& D = m->deal;
    OM_MHIP(m, hipSetDevice(m->dev[0]));
    if (m->renders_live) {
        OM_MHIP(m, hipStreamWaitEvent(st[0], m->done0, 0));
        for (uint32_t r = 1; r < N; ++r) OM_MHIP(m, hipStreamWaitEvent(st[0], m->ev[r], 0));
    }
    if (m->ev0_live) OM_MHIP(m, hipStreamWaitEvent(st[0], m->ev[0], 0));
    for (uint32_t r = 0; r < N; ++r)
        OM_MHIP(m, launch_move(false, dev_frame, D.list(r), D.count[r], r ? m->staging[r].p : m->shard[0].p, st[0]));
    if (m->transport == OM_TRANSPORT_RCCL && N > 1) {
        ncclResult_t e = ncclGroupStart();
        for (uint32_t r = 1; e == ncclSuccess && r < N; ++r) {
            const size_t b = (size_t)D.count[r] * sizeof(om_pixel_stats);
            if (!b) continue;
            e = ncclSend(m->staging[r].p, b, ncclUint8, (int)r, m->nc[0], st[0]);
            if (e == ncclSuccess) e = ncclRecv(m->shard[r].p, b, ncclUint8, 0, m->nc[r], st[r]);
        }
        const ncclResult_t e2 = ncclGroupEnd();
        if (e != ncclSuccess || e2 != ncclSuccess) return merr(m, OM_ERR_DEVICE, nccl_msg("om_multi deal", e != ncclSuccess ? e : e2));
    } else {
        for (uint32_t r = 1; r < N; ++r)
            if (D.count[r])
                OM_MHIP(m, hipMemcpyPeerAsync(m->shard[r].p, m->dev[r], m->staging[r].p, m->dev[0],
                                              (size_t)D.count[r] * sizeof(om_pixel_stats), st[0]));
    }
    return fence_from_root(m, st);
}

bool frame_bound(const om_multi* m, const void* f, uint32_t W, uint32_t H) {
    return m->bound && m->bound == f && m->bw == W && m->bh == H;
}

}  // namespace

extern "C" {

om_status om_multi_create(const int32_t* devices, uint32_t n, om_multi** out) {
    if (!devices || !out || n == 0) return merr(nullptr, OM_ERR_INVALID, "om_multi_create: bad argument");
    *out = nullptr;
    om_multi* m = new (std::nothrow) om_multi();
    if (!m) return merr(nullptr, OM_ERR_NOMEM, "om_multi_create: out of memory");
    m->dev.assign(devices, devices + n);
    m->ctx.assign(n, nullptr);
    m->list.resize(n); m->shard.resize(n); m->staging.resize(n);
    m->ev.assign(n, nullptr);
    if (hipSetDevice(devices[0]) != hipSuccess || hipEventCreateWithFlags(&m->done0, hipEventDisableTiming) != hipSuccess) {
        om_multi_destroy(m);
        return merr(nullptr, OM_ERR_DEVICE, "om_multi_create: event creation failed");
    }
    for (uint32_t r = 0; r < n; ++r) {
        om_status s = om_create(devices[r], &m->ctx[r]);
        if (s != OM_OK) { const std::string msg = om_last_error(nullptr); om_multi_destroy(m); return merr(nullptr, s, msg); }
        if (hipSetDevice(devices[r]) != hipSuccess || hipEventCreateWithFlags(&m->ev[r], hipEventDisableTiming) != hipSuccess) {
            om_multi_destroy(m);
            return merr(nullptr, OM_ERR_DEVICE, "om_multi_create: event creation failed");
        }
    }
    std::vector<int> sorted(m->dev);
    std::sort(sorted.begin(), sorted.end());
    const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    m->transport = distinct ? OM_TRANSPORT_RCCL : OM_TRANSPORT_LOCAL;
    if (distinct) {
        m->nc.assign(n, nullptr);
        const ncclResult_t r = ncclCommInitAll(m->nc.data(), (int)n, m->dev.data());
        if (r != ncclSuccess) {
            m->nc.clear();
            om_multi_destroy(m);
            return merr(nullptr, OM_ERR_DEVICE, nccl_msg("ncclCommInitAll", r));
        }
    }
    *out = m;
    return OM_OK;
}

void om_multi_destroy(om_multi* m) {
    if (!m) return;
    for (size_t r = 0; r < m->dev.size(); ++r) {
        (void)hipSetDevice(m->dev[r]);
        (void)hipDeviceSynchronize();
    }
    for (auto c : m->nc) if (c) (void)ncclCommDestroy(c);
    for (auto& b : m->list) b.release();
    for (auto& b : m->shard) b.release();
    for (auto& b : m->staging) b.release();
    m->deal.all.release();
    m->host_frame.release();
    for (size_t r = 0; r < m->ev.size(); ++r)
        if (m->ev[r]) { (void)hipSetDevice(m->dev[r]); (void)hipEventDestroy(m->ev[r]); }
    if (m->done0) { (void)hipSetDevice(m->dev[0]); (void)hipEventDestroy(m->done0); }
    for (auto c : m->ctx) om_destroy(c);
    delete m;
}

int32_t om_multi_transport(const om_multi* m) { return m ? m->transport : -1; }

om_ctx* om_multi_ctx(om_multi* m, uint32_t rank) { return (m && rank < m->ctx.size()) ? m->ctx[rank] : nullptr; }

const char* om_multi_last_error(const om_multi* m) { return m ? m->err.c_str() : om_last_error(nullptr); }

om_status om_multi_upload_world(om_multi* m, const om_world* w) {
    if (!m || !w) return merr(m, OM_ERR_INVALID, "om_multi_upload_world: null argument");
    for (size_t r = 0; r < m->ctx.size(); ++r) {
        const om_status s = om_upload_world(m->ctx[r], w);
        if (s != OM_OK) return merr(m, s, std::string("rank ") + std::to_string(r) + ": " + om_last_error(m->ctx[r]));
    }
    return OM_OK;
}

om_status om_multi_render(om_multi* m, const om_camera* cam, const om_render_params* p, om_pixel_stats* dev_frame, void* stream) {
    if (!m || !cam || !p || !dev_frame) return merr(m, OM_ERR_INVALID, "om_multi_render: null argument");
    if (p->width == 0 || p->height == 0 || (uint64_t)p->width * p->height > (1ull << 31))
        return merr(m, OM_ERR_INVALID, "om_multi_render: width/height must be > 0");
    const uint32_t N = (uint32_t)m->ctx.size();
    om_status s = multi_lists(m, p->width, p->height);
    if (s) return s;
    const std::vector<hipStream_t> st = rank_streams(m, stream);
    if (!frame_bound(m, dev_frame, p->width, p->height)) {
        // a new frame (first use, another buffer or size, or after om_multi_reset): deal it out
        m->bound = nullptr;
        if ((s = deal_frame(m, dev_frame, st))) return s;
        m->bound = dev_frame; m->bw = p->width; m->bh = p->height;
    } else if (m->ev0_live) {
        // resident shards: the ranks start after rank 0's last deal or gather (which read them);
        // rank 0 too, as the caller may pass this render another stream than the gather's
        for (uint32_t r = 0; r < N; ++r) {
            OM_MHIP(m, hipSetDevice(m->dev[r]));
            OM_MHIP(m, hipStreamWaitEvent(st[r], m->ev[0], 0));
        }
    }
    // every rank renders its tiles into its resident shard on its own stream (all devices at once)
    const Deal& D = m->deal;
    for (uint32_t r = 0; r < N; ++r) {
        if (D.count[r]) {
            const uint32_t* lst = r ? (const uint32_t*)m->list[r].p : D.list(0);
            s = om_render_device_pixels(m->ctx[r], cam, p, (om_pixel_stats*)m->shard[r].p, lst, D.count[r], st[r]);
            if (s != OM_OK) return merr(m, s, std::string("rank ") + std::to_string(r) + ": " + om_last_error(m->ctx[r]));
        }
        OM_MHIP(m, hipSetDevice(m->dev[r]));
        OM_MHIP(m, hipEventRecord(r ? m->ev[r] : m->done0, st[r]));
    }
    m->renders_live = true;
    return OM_OK;
}

om_status om_multi_gather(om_multi* m, om_pixel_stats* dev_frame, uint32_t W, uint32_t H, void* stream) {
    if (!m || !dev_frame) return merr(m, OM_ERR_INVALID, "om_multi_gather: null argument");
    if (!m->bound || m->bw != W || m->bh != H || !m->deal.valid(W, H, (uint32_t)m->ctx.size()))
        return merr(m, OM_ERR_INVALID, "om_multi_gather: no resident frame of this size (om_multi_render first)");
    const uint32_t N = (uint32_t)m->ctx.size();
    const Deal& D = m->deal;
    const std::vector<hipStream_t> st = rank_streams(m, stream);
    OM_MHIP(m, hipSetDevice(m->dev[0]));
    OM_MHIP(m, hipStreamWaitEvent(st[0], m->done0, 0));                // rank 0's last render (any stream)
    if (m->transport == OM_TRANSPORT_RCCL && N > 1) {
        ncclResult_t e = ncclGroupStart();
        for (uint32_t r = 1; e == ncclSuccess && r < N; ++r) {
            const size_t b = (size_t)D.count[r] * sizeof(om_pixel_stats);
            if (!b) continue;
            e = ncclSend(m->shard[r].p, b, ncclUint8, 0, m->nc[r], st[r]);   // after rank r's render on st[r]
            if (e == ncclSuccess) e = ncclRecv(m->staging[r].p, b, ncclUint8, (int)r, m->nc[0], st[0]);
        }
        const ncclResult_t e2 = ncclGroupEnd();
        if (e != ncclSuccess || e2 != ncclSuccess) return merr(m, OM_ERR_DEVICE, nccl_msg("om_multi_gather", e != ncclSuccess ? e : e2));
    } else if (N > 1) {
        OM_MHIP(m, hipSetDevice(m->dev[0]));
        for (uint32_t r = 1; r < N; ++r) {
            OM_MHIP(m, hipStreamWaitEvent(st[0], m->ev[r], 0));       // rank r's last render
            if (D.count[r])
                OM_MHIP(m, hipMemcpyPeerAsync(m->staging[r].p, m->dev[0], m->shard[r].p, m->dev[r],
                                              (size_t)D.count[r] * sizeof(om_pixel_stats), st[0]));
        }
    }
    // rank 0 puts every shard into the frame
    OM_MHIP(m, hipSetDevice(m->dev[0]));
    for (uint32_t r = 0; r < N; ++r)
        OM_MHIP(m, launch_move(true, r ? m->staging[r].p : m->shard[0].p, D.list(r), D.count[r], dev_frame, st[0]));
    // the next render call's ranks overwrite their shards only after this read them
    OM_MHIP(m, hipEventRecord(m->ev[0], st[0]));
    m->ev0_live = true;
    return OM_OK;
}

void om_multi_reset(om_multi* m) {
    if (!m) return;
    m->bound = nullptr;
}

om_status om_multi_render_host(om_multi* m, const om_camera* cam, const om_render_params* p, om_pixel_stats* stats,
                               om_counters* counters) {
    if (!m || !cam || !p || !stats) return merr(m, OM_ERR_INVALID, "om_multi_render_host: null argument");
    if (p->width == 0 || p->height == 0 || (uint64_t)p->width * p->height > (1ull << 31))
        return merr(m, OM_ERR_INVALID, "om_multi_render_host: width/height must be > 0");
    const size_t bytes = (size_t)p->width * p->height * sizeof(om_pixel_stats);
    hipStream_t st = omi::ctx_stream(m->ctx[0]);
    for (auto c : m->ctx) {
        const om_status s = om_reset_counters(c, nullptr);
        if (s != OM_OK) return merr(m, s, om_last_error(c));
    }
    OM_MHIP(m, hipSetDevice(m->dev[0]));
    // The host framebuffer is the caller's (render_thread.rs:145-147): it may have been zeroed to
    // restart, rewritten, or freed and reallocated at the same address since the last call, so
    // every call mirrors it on devices[0] and deals it out again.  This form is a
    // synchronous round trip with two whole-frame copies anyway; om_multi_render keeps the
    // shards resident across calls for device frames.
    OM_MHIP(m, m->host_frame.ensure(m->dev[0], bytes));
    m->bound = nullptr;
    OM_MHIP(m, hipMemcpyAsync(m->host_frame.p, stats, bytes, hipMemcpyHostToDevice, st));
    om_status s = om_multi_render(m, cam, p, (om_pixel_stats*)m->host_frame.p, st);
    if (s == OM_OK) s = om_multi_gather(m, (om_pixel_stats*)m->host_frame.p, p->width, p->height, st);
    if (s != OM_OK) return s;
    OM_MHIP(m, hipSetDevice(m->dev[0]));
    OM_MHIP(m, hipMemcpyAsync(stats, m->host_frame.p, bytes, hipMemcpyDeviceToHost, st));
    OM_MHIP(m, hipStreamSynchronize(st));
    if (counters) {
        *counters = om_counters{};
        for (auto c : m->ctx) {
            om_counters k{};
            if ((s = om_get_counters(c, &k)) != OM_OK) return merr(m, s, om_last_error(c));
            counters->samples += k.samples; counters->segments += k.segments; counters->prim_tests += k.prim_tests;
            counters->pre_tests += k.pre_tests; counters->march_steps += k.march_steps; counters->credited += k.credited;
        }
    }
    return OM_OK;
}

}  // extern "C"
