"""Secondary measurements for DESIGN.md (GPU box):
  * C1 through the HOST framebuffer entry point om_render (stats copied host -> device ->
    host every call: the PCIe-inclusive rate; bench.py's `value` keeps stats in HBM);
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


def main():
    out = {}
    # ---- C1 host path: 4 calls of 16 spp through om_render (host stats, includes PCIe)
    W, H = 1920, 1080
    cam = om.default_camera(W / H)
    fz = om.random_scene(0x5EED).freeze(cam)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, 64, W, H, pix, seed=1, sample_count=16, adaptive=False)          # warm-up
    pix = om.PixelsBox.new(W * H)
    t0 = time.perf_counter()
    for _ in range(4):
        om.render(cam, fz, 50, 0.001, 100.0, 64, W, H, pix, seed=1, sample_count=16, adaptive=False)
    dt = time.perf_counter() - t0
    assert int(pix.pixels["n"].min()) == 64
    out["c1_host_path"] = {"msamples_s": round(W * H * 64 / dt / 1e6, 1), "calls": 4, "spp_per_call": 16,
                           "stats_bytes_each_way": W * H * 40}
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
