"""CPU baseline timing of the oracle (bench.py's `cpu_baseline` leg; test infrastructure, never
the product).  Runs the reference's thread scheme (num_cpus-1 workers over 2730-pixel
round-robin chunks, main.rs:170-189) over full 1-spp passes of a config's frame until a time
budget is spent, and prints one JSON object.  Which build is timed is chosen by ORO_LIB
(liboro.so: -O3, default x86-64 target; liboro_v3.so: -O3 -march=x86-64-v3), so bench.py runs
this as a subprocess once per build.

    ORO_LIB=liboro_v3.so python oracle/cpu_bench.py --config C1 --budget 12 [--threads N]

With --window W,H,X0,Y0,SIZE,SPP it instead renders the SIZE x SIZE window at (X0, Y0) of the
config's W x H frame at SPP samples (render seed 1) and saves its Stats to --dump: the oracle side
of bench.py's per-config window parity check (the GPU frame it times vs this restatement).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path[0] = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # the repo root, not oracle/
from oracle import oracle as O  # noqa: E402

SCENES = {"C0": "S-traced", "C1": "S-traced", "C2": "S-marched", "C3": "S-10k", "C4": "S-traced"}
MARCH = {"C2": 256}
FRAMES = {"C0": (400, 225), "C1": (1920, 1080), "C2": (1920, 1080), "C3": (240, 135), "C4": (1920, 1080)}
DEPTH = {"C0": 8}


def scene(cfg):
    s = SCENES[cfg]
    if s == "S-traced":
        return O.random_scene(0x5EED)
    if s == "S-marched":
        return O.marched_scene()
    return O.random_scene(0x5EED, grid_half=50, extras=False)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cgroup_quota_cpus():
    """The cgroup CPU quota in CPUs, rounded up (cgroup v2 cpu.max, else v1 cfs_quota/period),
    or None when there is none."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
        return None
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return max(1, -(-q // per)) if q > 0 else None
    except (OSError, ValueError):
        return None


def num_cpus():
    """num_cpus::get() on Linux (num_cpus 1.x, what main.rs:170 calls): the cgroup CPU quota when
    one is set, else the CPUs of the affinity mask.  -> (num_cpus, affinity count, quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_quota_cpus()
    return (min(aff, quota) if quota else aff), aff, quota


def run(cfg, budget_s, threads, spp_total=64, seed=1, dump=None):
    """Full 1-spp passes of the config's frame (C3: a 1/64-area frame of the same scene and camera,
    since the oracle is brute force over 10k spheres and the per-sample cost does not depend on
    the resolution; C0: its whole 400x225x64 frame at depth 8)."""
    w, h = FRAMES[cfg]
    depth = DEPTH.get(cfg, 50)
    ow, cam = scene(cfg), O.default_camera(w / h)
    stats = np.zeros(w * h, dtype=O.PIXEL_STATS_DTYPE)
    done, t_total, passes = 0, 0.0, 0
    full = cfg == "C0"                                         # the CPU config: the whole frame
    while passes == 0 or (passes < spp_total and (full or t_total < budget_s)):
        p = O.params(w, h, spp_total, sample_count=1, max_depth=depth, seed=seed,
                     march_steps=MARCH.get(cfg, 1024))
        t0 = time.perf_counter()
        _, ctr = O.render(ow, cam, p, stats=stats, nthreads=threads)
        t_total += time.perf_counter() - t0
        done += ctr["samples"]
        passes += 1
    if dump:
        np.save(dump, stats, allow_pickle=False)           # the frame, for bench.py's C0 bit-exactness check
    nc, aff, quota = num_cpus()
    return {"value": done / t_total / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "build": os.path.basename(O.LIB), "seconds": round(t_total, 3), "samples": int(done),
            "num_cpus": nc, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
            "threads_rule": "num_cpus::get() - 1 (main.rs:170): the cgroup quota if set, else the affinity mask",
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "sample": f"{cfg} frame {w}x{h}, {passes} spp (full 1-spp passes), depth {depth}, {SCENES[cfg]}, "
                      f"{threads} threads ({os.path.basename(O.LIB)}), {t_total:.1f} s"}


def window(cfg, spec, threads, dump, seed=1):
    """The oracle's Stats of one window of the config's frame (bench.py's window parity); a 7th
    field 1 renders it adaptively (render_thread.rs:31-38, 68-102)."""
    v = [int(x) for x in spec.split(",")]
    w, h, x0, y0, size, spp = v[:6]
    adaptive = len(v) > 6 and v[6] == 1
    p = O.params(w, h, spp, max_depth=DEPTH.get(cfg, 50), seed=seed, march_steps=MARCH.get(cfg, 1024), adaptive=adaptive)
    t0 = time.perf_counter()
    st = O.render_pixels(scene(cfg), O.default_camera(w / h), p, O.window_pixels(w, h, x0, y0, size), nthreads=threads)
    np.save(dump, st, allow_pickle=False)
    return {"seconds": round(time.perf_counter() - t0, 3), "threads": threads, "window": [x0, y0, size], "spp": spp,
            "adaptive": adaptive}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C1", choices=list(SCENES))
    ap.add_argument("--budget", type=float, default=12.0)
    ap.add_argument("--threads", type=int, default=0,
                    help="0: num_cpus::get() - 1 as main.rs:170; -1: num_cpus::get() (the all-cores point)")
    ap.add_argument("--dump", default=None, help="save the rendered Stats (.npy) here")
    ap.add_argument("--window", default=None, help="W,H,X0,Y0,SIZE,SPP[,ADAPTIVE]: render one window into --dump")
    a = ap.parse_args()
    n = num_cpus()[0]
    t = a.threads if a.threads > 0 else (n if a.threads < 0 else max(1, n - 1))
    if a.window:
        print(json.dumps(window(a.config, a.window, t, a.dump)))
    else:
        print(json.dumps(run(a.config, a.budget, t, dump=a.dump)))
