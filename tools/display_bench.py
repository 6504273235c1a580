"""Time the display views (om_display_device) on a rendered 1920x1080 frame: per view the
average kernel time over N launches (HIP events on a dedicated stream) and the achieved
rate against the algorithmic bytes (40-B Stats read once + 3-B RGB written per pixel).

    python tools/display_bench.py [--reps 50]   (GPU box)  -> one JSON line
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    W, H = 1920, 1080
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = C.c_void_p(stream.cuda_stream)
    cam = om.default_camera(W / H)
    fz = om.random_scene(0x5EED).freeze(cam)
    stats = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, 8, W, H, seed=1)
    L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(stats.data_ptr()), sp), fz.ctx)
    rgb = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    out = {"frame": f"{W}x{H} S-traced 8 spp", "views": {}}
    for v, name in enumerate(L.VIEWS):
        for _ in range(3):
            L.check(L.lib.om_display_device(fz.ctx, C.c_void_p(stats.data_ptr()), W, H, v, C.c_void_p(rgb.data_ptr()), sp), fz.ctx)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(args.reps):
            L.check(L.lib.om_display_device(fz.ctx, C.c_void_p(stats.data_ptr()), W, H, v, C.c_void_p(rgb.data_ptr()), sp), fz.ctx)
        b.record(stream)
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / args.reps
        out["views"][name] = {"ms": round(ms, 4), "algorithmic_gbs": round(W * H * 43 / (ms / 1e3) / 1e9, 1)}
    host = om.display(fz, stats.cpu().numpy().view(L.PIXEL_STATS_DTYPE), W, H, "sample_blur")
    out["host_path_ok"] = bool(host.shape == (H, W, 3))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
