"""Secondary measurements for DESIGN.md (GPU box):
  * C1 through the HOST framebuffer entry point om_render (stats copied host -> device ->
    host every call: the PCIe-inclusive rate; bench.py's `value` keeps stats in HBM), with
    the framebuffer page-locked (PixelsBox, om_host_register) or pageable, at 512 / 32 / 16
    spp per call, beside the device-resident rate of the same frame;
  * C0, the reference's own CPU case (400x225, 64 spp, depth 8): GPU (om_render_device)
    and the CPU oracle on this host's cores (the reference's num_cpus-1 thread scheme).
One JSON line.  python tools/host_path.py
"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402


def c1_host(per_call, pinned, spp=512):
    """C1 through om_render (host Stats: the PCIe-inclusive rate), `per_call` spp per call."""
    W, H = 1920, 1080
    cam = om.default_camera(W / H)
    fz = om.random_scene(0x5EED).freeze(cam)
    L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)
    box = om.PixelsBox.new(W * H)
    target = box if pinned else box.pixels                   # a bare array stays pageable
    om.render(cam, fz, 50, 0.001, 100.0, spp, W, H, target, seed=1, sample_count=per_call, adaptive=False)  # warm-up
    box.pixels[:] = 0
    t0 = time.perf_counter()
    for _ in range(spp // per_call):
        om.render(cam, fz, 50, 0.001, 100.0, spp, W, H, target, seed=1, sample_count=per_call, adaptive=False)
    dt = time.perf_counter() - t0
    assert int(box.pixels["n"].min()) == spp
    return {"msamples_s": round(W * H * spp / dt / 1e6, 1), "calls": spp // per_call, "spp_per_call": per_call,
            "pinned": pinned, "stats_bytes_each_way_per_call": W * H * 40}


def c1_device(per_call=32, spp=512):
    """The same frame with device-resident Stats (om_render_device): bench.py's value."""
    W, H = 1920, 1080
    cam = om.default_camera(W / H)
    fz = om.random_scene(0x5EED).freeze(cam)
    L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)
    st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    p = om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=per_call, seed=1)
    go = lambda: L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()),
                                                C.c_void_p(s.cuda_stream)), fz.ctx)
    go()
    torch.cuda.synchronize()
    st.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(spp // per_call):
        go()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"msamples_s": round(W * H * spp / dt / 1e6, 1), "calls": spp // per_call, "spp_per_call": per_call}


def main():
    out = {}
    dev = c1_device()
    out["c1_device_resident"] = dev
    for per_call, pinned in ((512, True), (32, True), (32, False), (16, True)):
        r = c1_host(per_call, pinned)
        r["of_device_resident"] = round(r["msamples_s"] / dev["msamples_s"], 3)
        out[f"c1_host_{per_call}spp_{'pinned' if pinned else 'pageable'}"] = r
    # ---- C0 on the GPU (device stats) and on the CPU oracle
    W0, H0, SPP0, D0 = 400, 225, 64, 8
    cam0 = om.default_camera(W0 / H0)
    fz0 = om.random_scene(0x5EED).freeze(cam0)
    stream = torch.cuda.Stream()
    sp = C.c_void_p(stream.cuda_stream)
    st = torch.zeros(W0 * H0 * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(D0, 0.001, 100.0, SPP0, W0, H0, seed=1)
    L.check(L.lib.om_render_device(fz0.ctx, C.byref(cam0.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz0.ctx)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        st.zero_()
        L.check(L.lib.om_render_device(fz0.ctx, C.byref(cam0.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz0.ctx)
    torch.cuda.synchronize()
    gpu_s = (time.perf_counter() - t0) / reps
    from oracle import oracle as O                              # CPU baseline only
    cores = max(1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 2)) - 1)
    t0 = time.perf_counter()
    cpu_stats, _ = O.render(O.random_scene(0x5EED), O.default_camera(W0 / H0), O.params(W0, H0, SPP0, max_depth=D0, seed=1),
                            nthreads=cores)
    cpu_s = time.perf_counter() - t0
    same = np.array_equal(cpu_stats.view(np.uint8).reshape(-1), st.cpu().numpy())
    out["c0"] = {"frame": f"{W0}x{H0}x{SPP0} depth {D0}", "gpu_ms": round(gpu_s * 1e3, 2),
                 "gpu_msamples_s": round(W0 * H0 * SPP0 / gpu_s / 1e6, 1), "cpu_s": round(cpu_s, 2),
                 "cpu_msamples_s": round(W0 * H0 * SPP0 / cpu_s / 1e6, 3), "cpu_threads": cores,
                 "bit_identical": bool(same)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
