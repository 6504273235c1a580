// om_shard.h — the host-side tile deal of multi-GPU frames (om_shard.cpp), shared by the
// C-ABI entry points and om_multi.hip.  Host C++ only (no HIP types).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/ottomarcher.h"

namespace oms {
constexpr uint32_t kTile = 8;
uint64_t n_tiles(uint32_t w, uint32_t h);
// pixels of the largest rank's shard
uint32_t capacity(uint32_t w, uint32_t h, uint32_t nranks);
// rank's pixels: tiles t = rank, rank + nranks, ... in row-major tile order, lane order inside
void deal(uint32_t w, uint32_t h, uint32_t rank, uint32_t nranks, std::vector<uint32_t>& out);
}  // namespace oms

namespace omi {
om_status global_error(om_status code, const std::string& msg);   // om_render.hip
}
