// om_tiles.h — primary-ray candidate lists per 8x8 pixel tile.
//
// The reference's camera hash (camera_hash.rs, hits.rs:116-185) meant to cull primary
// rays by screen cell but overflows on random_scene.  This is the same idea
// made conservative: a leaf record joins a tile's list when some primary ray of that
// tile — from any lens point through any jittered position of its pixels — can reach
// the record's (inflated) box.  Bounce 0 then tests the tile's list brute force with the
// reference tie rule instead of traversing the BVH, so the answer is unchanged.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/ottomarcher.h"

namespace omt {

struct TileLists {
    std::vector<uint32_t> off;   // tiles + 1 prefix offsets into idx
    std::vector<uint16_t> idx;   // srec indices, each tile's sorted by tnear (ascending)
    std::vector<float> tnear;    // per srec: a lower bound of the t at which any primary ray can reach its box
    double avg_per_pixel = 0.0;  // mean list length seen by a pixel
};

// srec_box: 6 floats per leaf record (lo xyz, hi xyz).  Returns false when lists cannot
// be built (frame < 2 pixels in a dimension, > 65535 records, a degenerate camera).
bool build(const std::vector<float>& srec_box, const om_camera& cam, uint32_t width, uint32_t height, TileLists& out);

}  // namespace omt
