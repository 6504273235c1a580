// om_display.h — draw_to_sdl view modes (main.rs:219-437) as image-space kernels over
// the per-pixel Stats in HBM.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/ottomarcher.h"

namespace omv {

// Device scratch (bytes) `render` needs for a W x H frame (the max reductions of modes 1/3).
size_t scratch_bytes(uint32_t width, uint32_t height);

// RGB24 view `mode` (OM_VIEW_*) of W*H stats into rgb (W*H*3, read-modify-write: pixels the
// reference's box filter does not visit keep their bytes).  Asynchronous on `stream`.
hipError_t render(const om_pixel_stats* stats, uint32_t width, uint32_t height, int mode, uint8_t* rgb, void* scratch,
                  hipStream_t stream);

}  // namespace omv
