"""Latency floor of one bounce (GPU box, under rocprofv3 --kernel-trace): an 8x8 frame (one
wave per bounce launch) of S-traced at max_depth 50, serial batches, no persistent tail, so
every bounce is its own launch holding at most 64 paths.  The launch durations in the trace are
the per-bounce latency of one wave (plus the launch overhead).
    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/lone_latency.py"""
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402

W, H = int(os.environ.get("LL_W", 8)), int(os.environ.get("LL_H", 8))
world = om.random_scene(0x5EED)
cam = om.default_camera(16 / 9)            # the C1 camera; the 8x8 frame is its top-left corner region
fz = world.freeze(cam, pipeline="wavefront")
L.check(L.lib.om_set_streams(fz.ctx, 1), fz.ctx)
L.check(L.lib.om_set_tail_bounce(fz.ctx, int(os.environ.get("LL_TAIL", 50))), fz.ctx)
L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)
st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
for spp in (1, 1, 1, 1):
    p = om.make_params(50, 0.001, 100.0, 64, W, H, sample_count=spp, seed=3)
    L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()),
                                   C.c_void_p(s.cuda_stream)), fz.ctx)
    s.synchronize()
print("ok")
