// om_internal.h — what other translation units of libottomarcher.so need from an om_ctx
// (defined in om_render.hip); not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <string>

#include "../../include/ottomarcher.h"

namespace omi {
int ctx_device(const om_ctx* c);
hipStream_t ctx_stream(const om_ctx* c);
// records `msg` as om_last_error(c) (and the global last error) and returns `code`
om_status ctx_error(om_ctx* c, om_status code, const std::string& msg);
om_status global_error(om_status code, const std::string& msg);
}  // namespace omi
