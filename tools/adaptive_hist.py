"""Per-pixel sample counts of an adaptive frame (render_thread.rs:31-38, 68-102): renders C1's
1080p frame at SPP spp adaptive in STEP-spp calls and prints the histogram of Stats.n (how many
samples each pixel took before it retired) as one JSON line.  Used to model adaptive batch
schedules on the host.  argv: [SPP [STEP [scene]]].
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402


def main():
    W, H = 1920, 1080
    SPP = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    STEP = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    scene = sys.argv[3] if len(sys.argv) > 3 else "C1"
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = C.c_void_p(stream.cuda_stream)
    cam = om.default_camera(W / H)
    world = om.random_scene(0x5EED) if scene == "C1" else om.marched_scene()
    fz = world.freeze(cam)
    st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, SPP, W, H, sample_count=STEP, seed=1, adaptive=True, march_steps=256)
    for _ in range(SPP // STEP):
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz.ctx)
    torch.cuda.synchronize()
    n = st.view(W * H, 40)[:, 20:24].contiguous().view(torch.int32).cpu().flatten()
    hist = torch.bincount(n.long(), minlength=SPP + 1).tolist()
    print(json.dumps({"scene": scene, "W": W, "H": H, "spp": SPP, "step": STEP, "taken": int(n.sum()), "hist": hist}))


if __name__ == "__main__":
    main()
