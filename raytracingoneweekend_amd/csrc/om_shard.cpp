// om_shard.cpp — the tile deal of multi-GPU frames: 8x8 pixel tiles dealt
// round-robin to ranks, the re-design of main.rs:172-189's 2730-pixel chunk round-robin over
// the render threads.  Host C++; om_multi.hip moves the shards on the device.
#include "om_shard.h"

#include <cstring>

namespace oms {

uint64_t n_tiles(uint32_t w, uint32_t h) { return (uint64_t)((w + kTile - 1) / kTile) * ((h + kTile - 1) / kTile); }

uint32_t capacity(uint32_t w, uint32_t h, uint32_t nranks) {
    return (uint32_t)((n_tiles(w, h) + nranks - 1) / nranks * kTile * kTile);
}

void deal(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks, std::vector<uint32_t>& out) {
    out.clear();
    const uint32_t tx = (w + kTile - 1) / kTile;
    for (uint64_t t = rank; t < n_tiles(w, h); t += nranks)
        for (uint32_t l = 0; l < kTile * kTile; ++l) {
            const uint32_t px = (uint32_t)(t % tx) * kTile + (l % kTile), py = (uint32_t)(t / tx) * kTile + l / kTile;
            if (px < w && py < h) out.push_back(py * w + px);
        }
}

}  // namespace oms

extern "C" {

uint32_t om_shard_capacity(uint32_t width, uint32_t height, uint32_t nranks) {
    if (nranks == 0) return 0;
    return oms::capacity(width, height, nranks);
}

om_status om_shard_pixels(uint32_t width, uint32_t height, uint32_t rank, uint32_t nranks, uint32_t* out, uint32_t cap,
                          uint32_t* n_out) {
    if (!n_out || nranks == 0 || rank >= nranks) return omi::global_error(OM_ERR_INVALID, "om_shard_pixels: bad rank/nranks");
    if ((uint64_t)width * height > (1ull << 31)) return omi::global_error(OM_ERR_INVALID, "om_shard_pixels: frame too large");
    std::vector<uint32_t> lst;
    oms::deal(width, height, rank, nranks, lst);
    *n_out = (uint32_t)lst.size();
    if (lst.size() > cap || (!out && !lst.empty()))
        return omi::global_error(OM_ERR_INVALID, "om_shard_pixels: output too small (see om_shard_capacity)");
    if (!lst.empty()) std::memcpy(out, lst.data(), lst.size() * 4);
    return OM_OK;
}

om_status om_shard_assemble_host(uint32_t width, uint32_t height, uint32_t nranks, const om_pixel_stats* const* shards,
                                 om_pixel_stats* frame) {
    if (!shards || !frame || nranks == 0) return omi::global_error(OM_ERR_INVALID, "om_shard_assemble_host: null argument");
    if ((uint64_t)width * height > (1ull << 31)) return omi::global_error(OM_ERR_INVALID, "om_shard_assemble_host: frame too large");
    std::vector<uint32_t> lst;
    for (uint32_t r = 0; r < nranks; ++r) {
        oms::deal(width, height, r, nranks, lst);
        if (!lst.empty() && !shards[r]) return omi::global_error(OM_ERR_INVALID, "om_shard_assemble_host: null shard");
        for (size_t k = 0; k < lst.size(); ++k) frame[lst[k]] = shards[r][k];
    }
    return OM_OK;
}

}  // extern "C"
