"""Where the persistent tail's time goes (GPU box): C1's 1080p frame, one 32-spp call (two
concurrent 16-spp batches, the bench's batch shape) per max_depth, every launch timed on its own
stream (om_set_timing mode 1).  With max_depth = tail + 1 the tail runs exactly one segment per
path (pure throughput); with 50 it runs the deepest paths' chains.  Also the lone-wave floor: an
8x8 frame whose only paths all go to the tail at bounce 1.
    python tools/tail_probe.py [OM_LIB=...]   -> one JSON line per case"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402

TAIL = int(os.environ.get("TP_TAIL", 16))
world = om.random_scene(0x5EED)


def run(W, H, depth, spp, tail, streams, reps=3):
    cam = om.default_camera(16 / 9)
    fz = world.freeze(cam, pipeline="wavefront")
    L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
    L.check(L.lib.om_set_tail_bounce(fz.ctx, tail), fz.ctx)
    st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    kt = L.om_kernel_times()
    out = None
    for rep in range(reps + 1):
        st.zero_()
        torch.cuda.synchronize()
        L.check(L.lib.om_set_timing(fz.ctx, 1), fz.ctx)
        p = om.make_params(depth, 0.001, 100.0, spp, W, H, sample_count=spp, seed=1)
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()),
                                       C.c_void_p(s.cuda_stream)), fz.ctx)
        s.synchronize()
        L.check(L.lib.om_get_kernel_times(fz.ctx, C.byref(kt)), fz.ctx)
        if rep:                                               # rep 0 warms up
            r = {c: (int(kt.launches[i]), round(kt.ms[i] / max(1, kt.launches[i]), 4))
                 for i, c in enumerate(L.KT_CLASSES) if kt.launches[i]}
            out = r if out is None else {c: (r[c][0], min(r[c][1], out[c][1])) for c in r}
    fz.close()
    return out


for depth in (TAIL + 1, TAIL + 2, TAIL + 4, TAIL + 8, 34, 50):
    print(json.dumps({"case": "C1 32spp", "tail": TAIL, "max_depth": depth, "per_launch_ms": run(1920, 1080, depth, 32, TAIL, 2)}),
          flush=True)
for depth in (2, 3, 5, 9, 17, 50):
    print(json.dumps({"case": "8x8 lone wave", "tail": 1, "max_depth": depth, "per_launch_ms": run(8, 8, depth, 1, 1, 1)}),
          flush=True)
