"""Adaptive sampling (render_thread.rs:31-38, 68-102, 196-198) on C1: a pixel retires after
5 consecutive samples leave its 8-bit colour unchanged, and the progress counter credits
the skipped samples.  Per schedule (wavefront with two concurrent batches, wavefront serial,
megakernel): wall time for a 64-spp frame in STEP-spp calls (argv[1], default 16), samples
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
    W, H = 1920, 1080
    STEP = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    SPP = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    scene = sys.argv[2] if len(sys.argv) > 2 else "C1"            # C1 (S-traced) or C2 (S-marched, 256 steps)
    REPS = 5
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sp = C.c_void_p(stream.cuda_stream)
    cam = om.default_camera(W / H)
    world = om.random_scene(0x5EED) if scene == "C1" else om.marched_scene()
    out = {"frame": f"{scene} {W}x{H}, {SPP} spp adaptive, {STEP} spp per call"}
    frames = {}
    extra = [int(x) for x in sys.argv[4].split(",")] if len(sys.argv) > 4 else []   # more stream counts
    # AD_SCHEDS="K,P;K,P": more wavefront runs with om_set_adaptive_batches(K, P) (2 streams)
    scheds = [tuple(int(v) for v in x.split(",")) for x in os.environ.get("AD_SCHEDS", "").split(";") if x]
    runs = ([("wavefront", "wavefront", 2, (0, 0))]
            + ([] if os.environ.get("AD_NO_SERIAL") else [("wavefront_serial", "wavefront", 1, (0, 0))])
            + ([] if os.environ.get("AD_NO_MEGA") else [("megakernel", "megakernel", 1, (0, 0))])
            + [(f"wavefront_s{k}", "wavefront", k, (0, 0)) for k in extra]
            + [(f"wavefront_k{a}_p{b}", "wavefront", 2, (a, b)) for a, b in scheds])
    for name, pipe, streams, sched in runs:
        fz = world.freeze(cam, pipeline=pipe)
        L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
        L.check(L.lib.om_set_adaptive_batches(fz.ctx, *sched), fz.ctx)
        L.check(L.lib.om_set_tail_bounce(fz.ctx, int(os.environ.get("AD_TAIL", "0"))), fz.ctx)
        st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
        p = om.make_params(50, 0.001, 100.0, SPP, W, H, sample_count=STEP, seed=1, adaptive=True,
                           march_steps=256)
        L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)          # timed: the production build
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz.ctx)
        torch.cuda.synchronize()
        reps = []
        for _ in range(REPS):                                     # REPS frames, each from zeroed Stats
            st.zero_()
            L.check(L.lib.om_reset_counters(fz.ctx, sp), fz.ctx)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(SPP // STEP):
                L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz.ctx)
            torch.cuda.synchronize()
            reps.append(time.perf_counter() - t0)
        dt = sorted(reps)[len(reps) // 2]                         # median frame
        timed = st.clone()
        st.zero_()                                                # counting pass: samples taken, credit
        L.check(L.lib.om_set_counting(fz.ctx, 1), fz.ctx)
        L.check(L.lib.om_reset_counters(fz.ctx, sp), fz.ctx)
        for _ in range(SPP // STEP):
            L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp), fz.ctx)
        torch.cuda.synchronize()
        assert torch.equal(st, timed), "counting build changed the frame"
        ctr = L.om_counters()
        L.check(L.lib.om_get_counters(fz.ctx, C.byref(ctr)), fz.ctx)
        frames[name] = st.cpu()
        out[name] = {"s": round(dt, 4), "frames_s": [round(x, 4) for x in reps], "taken_msamples_s": round(ctr.samples / dt / 1e6, 1),
                     "credited_msamples_s": round(ctr.credited / dt / 1e6, 1),
                     "taken_frac": round(ctr.samples / (W * H * SPP), 4),
                     "segments_g": round(ctr.segments / 1e9, 4), "gseg_s": round(ctr.segments / dt / 1e9, 2)}
    out["schedules_bit_identical"] = all(bool(torch.equal(frames["wavefront"], f)) for f in frames.values())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
