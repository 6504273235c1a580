"""Where a bounce-family wave's time goes (diagnostic build only: tools/ablate.sh variant
`phase`, -DOM_PHASE_STAMPS=1).  Renders a config the way bench.py's step does (32 spp per
call, timing off) and prints, per kernel, the share of wave lifetime spent in each phase of
a path chunk (s_memtime sums over waves, om_wavefront.hip PhaseClock):

  bounce0 / bounce / hit   0 path load or camera ray (+ forced wait), 1 trace, 2 shade,
                           3 compaction + store + next-chunk claim
  tail                     0 path load, 1 trace, 2 shade
  march                    0 refill (queue load + traced part + unstuck), 1 march steps,
                           3 refill vote

    OM_LIB=$PWD/_abl/lib_phase.so python tools/phase_stamps.py --config C1 > out.json

With the `phase2` build (-DOM_PHASE_STAMPS=2) the later bounces' trace is split further
(WorkT::lap, om_trace.h): always2, node read wait, slab + choice, stack pop, leaf record read
wait, record test; per lane, so a lane's step also carries the time the wave spent on other
lanes' diverged steps since its previous lap.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402

KERNELS = {0: "bounce0", 8: "bounce", 16: "tail", 24: "march", 32: "hit"}
PHASES = {"bounce0": ["gen", "trace", "shade", "compact"], "bounce": ["load", "trace", "shade", "compact"],
          "hit": ["load", "hitbuf", "shade", "compact"], "tail": ["load", "trace", "shade"],
          "march": ["refill", "step", "-", "vote"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1", choices=["C1", "C2", "C3"])
    ap.add_argument("--calls", type=int, default=4)
    a = ap.parse_args()
    fn = L.lib.om_debug_phase_stamps
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    W, H = 1920, 1080
    world = {"C1": lambda: om.random_scene(0x5EED), "C2": om.marched_scene,
             "C3": lambda: om.random_scene(0x5EED, grid_half=50, extras=False)}[a.config]()
    steps = 256 if a.config == "C2" else 1024
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, 32 * (a.calls + 1), W, H, sample_count=32, seed=1, march_steps=steps)
    buf = (C.c_uint64 * 64)()

    def call():
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(frame.data_ptr()), None), fz.ctx)

    call()                                                   # warm-up
    torch.cuda.synchronize()
    assert fn(buf, 1) == 0
    for _ in range(a.calls):
        call()
    torch.cuda.synchronize()
    assert fn(buf, 0) == 0
    out = {"config": a.config, "calls": a.calls, "kernels": {}}
    for base, name in KERNELS.items():
        acc = [buf[base + k] for k in range(8)]
        life, waves = acc[6], acc[7]
        if not waves:
            continue
        ph = {PHASES[name][k]: round(acc[k] / life, 4) for k in range(len(PHASES[name])) if PHASES[name][k] != "-"}
        out["kernels"][name] = {"waves": waves, "mean_wave_cycles": round(life / waves), "share_of_wave_life": ph,
                                "unaccounted": round(1 - sum(acc[:6]) / life, 4)}
    laps = ["always2", "node_wait", "node_slab", "pop", "rec_wait", "rec_test"]
    if any(buf[48 + k] for k in range(len(laps))):       # OM_PHASE_STAMPS=2: the later bounces' trace laps
        tot = sum(buf[40 + k] for k in range(len(laps)))
        out["bounce_trace_laps"] = {n: {"lane_cycles_share": round(buf[40 + k] / tot, 4), "events": buf[48 + k],
                                        "cycles_per_event": round(buf[40 + k] / max(1, buf[48 + k]), 1)}
                                    for k, n in enumerate(laps)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
