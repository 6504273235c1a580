"""Adaptive sampling (render_thread.rs:31-38, 68-102, 196-198) on C1: a pixel retires after
5 consecutive samples leave its 8-bit colour unchanged, and the progress counter credits
the skipped samples.  Per pipeline: wall time for a 64-spp frame in 16-spp calls, samples
actually taken, samples credited (the reference's samples_atom) -> one JSON line.
"""
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402


def main():
    W, H, SPP, STEP = 1920, 1080, 64, 16
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = C.c_void_p(stream.cuda_stream)
    cam = om.default_camera(W / H)
    world = om.random_scene(0x5EED)
    out = {"frame": f"C1 {W}x{H}, {SPP} spp adaptive, {STEP} spp per call"}
    frames = {}
    for pipe in ("wavefront", "megakernel"):
        fz = world.freeze(cam, pipeline=pipe)
        st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
        p = om.make_params(50, 0.001, 100.0, SPP, W, H, sample_count=STEP, seed=1, adaptive=True)
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz.ctx)
        torch.cuda.synchronize()
        st.zero_()
        L.check(L.lib.om_reset_counters(fz.ctx, sp), fz.ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(SPP // STEP):
            L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz.ctx)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ctr = L.om_counters()
        L.check(L.lib.om_get_counters(fz.ctx, C.byref(ctr)), fz.ctx)
        frames[pipe] = st.cpu()
        out[pipe] = {"s": round(dt, 4), "taken_msamples_s": round(ctr.samples / dt / 1e6, 1),
                     "credited_msamples_s": round(ctr.credited / dt / 1e6, 1),
                     "taken_frac": round(ctr.samples / (W * H * SPP), 4)}
    out["pipelines_bit_identical"] = bool(torch.equal(frames["wavefront"], frames["megakernel"]))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
