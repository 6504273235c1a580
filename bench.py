"""bench.py — MI355X benchmark of the ray_color hot path (BASELINE.json metric).

Workload (config C1, BASELINE.json configs[1]): the S-traced random_scene (main.rs:37-100
minus the torus block, om-rng scene seed 0x5EED), camera of main.rs:136-142, 1920x1080,
max_depth 50, tmin 0.001, tmax 100, fixed spp (adaptive off).  One STEP = one progressive
pass of SPP_PER_STEP samples over every pixel this rank owns, accumulated into the
per-pixel Stats in HBM (render_thread.rs:176-199, batched).  4 steps of 128 spp at N=1 =
the full 512-spp frame; the library runs each step as 16-spp batches, two in flight
(om_set_streams).

Every rank (N = 1 included) goes through the product's multi-GPU path: its
8x8-tile shard of the frame (om_shard_pixels: main.rs:172-189's chunk round-robin, re-designed
for GPUs) is rendered into an HBM-resident shard (om_render_shard), and the timed region ends
with om_gather_frame, the RCCL grouped send/recv of every shard to rank 0 over xGMI plus the
scatter into the W*H frame there.  N>1 (torch.distributed.run, one process per GPU): each rank
renders its tiles at SPP_PER_STEP*N samples per step (fixed per-GPU work: weak scaling).
torch.distributed (gloo, host memory) is the harness's control plane only: it hands RCCL's
unique id from rank 0 to the others, and carries the barriers and the max-over-ranks time.

At N=1 the line also carries `configs`: C2 (marched SDF scene, 256 march steps) and C3 (10k
spheres, BVH) at full spp with their own roofline and CPU baseline, C4's 3840x2160 frame at
256 spp (the N=1 leg of the 8-GPU config), and C0 (the reference's CPU case, 400x225x64 at
depth 8) timed on the GPU and on the host cores.

Output: ONE JSON line on rank 0 (see DESIGN.md §7 for every field).
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402
from raytracingoneweekend_amd import shard  # noqa: E402

MAX_DEPTH, TMIN, TMAX, SEED, SCENE_SEED = 50, 0.001, 100.0, 1, 0x5EED
# 128 spp per call: 8 batches of 16 spp on two streams; a call boundary drains both batches, so
# fewer, larger calls measured +0.8% over 32 spp per call (profiles/r03_v7/ab_drain_ab*_C1.jsonl, base rows)
SPP_PER_STEP = 128
# BASELINE.json configs: C1 is the metric's workload (the default line); C2/C3 ride along in
# the line's `configs` at N=1; C4 is the 4K frame of the multi-GPU config (--config C4).
CONFIGS = {
    "C0": {"scene": "S-traced", "spp": 64, "march_steps": 1024, "size": (400, 225), "depth": 8},
    "C1": {"scene": "S-traced", "spp": 512, "march_steps": 1024},
    "C2": {"scene": "S-marched", "spp": 256, "march_steps": 256},
    "C3": {"scene": "S-10k", "spp": 256, "march_steps": 1024},
    # BASELINE.json configs[4]: 3840x2160, 4096 spp, 8 GPUs; each rank renders its 1/N of the
    # tiles at 4096 spp: the fixed frame (strong scaling)
    "C4": {"scene": "S-traced", "spp": 4096, "march_steps": 1024, "size": (3840, 2160)},
}


def make_scene(name, om_or_oracle):
    if name == "S-traced":
        return om_or_oracle.random_scene(SCENE_SEED)
    if name == "S-marched":
        return om_or_oracle.marched_scene()
    return om_or_oracle.random_scene(SCENE_SEED, grid_half=50, extras=False)


PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md; FMA = 2 flop)
ISSUE_PEAK_TFLOPS = 78.6  # one f32 op per lane per cycle: 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz (no FMA)
PEAK_HBM_GBS = 8000.0

# Algorithmic FP32 work per counted unit, counted from om_device.h /
# om_trace.h in the reference's op order (no FMA: every add/mul/div/sqrt/min/max/cmp = 1).
FLOP_EXACT_TEST = 56      # Sphere::hit miss path: 2 affine xforms (36) + a, half_b, c, disc, cmp (20)
FLOP_BOX_TEST = 25        # slab test of one BVH child box
FLOP_SEGMENT = 110        # finalize (point + normal) + scatter + throughput + loop bookkeeping
FLOP_CAMERA_RAY = 50      # jitter/uv + lens disc + get_ray (bounce 0, once per sample)
FLOP_MARCH_STEP = 60      # one sphere-tracing iteration over the marched objects (S-traced: none)
# Algorithmic HBM bytes of the bounce-family kernels (SoA path queues).
# Fused pipeline (traced worlds): a segment after the first reads its 64-B path and the
# previous bounce wrote it (128 B); a sample reads its pixel id + Stats.n/flags (12 B) and
# writes its result (20 B).  Split march pipeline (marched worlds, §5.8): k_raygen writes every
# sample's 64-B camera path, so every segment is written and read once (128 B), k_march reads
# its origin + direction (32 B) and writes an 8-B hit record that k_bounce<HIT> reads (16 B).
BYTES_PER_LATER_SEGMENT = 128
BYTES_PER_SAMPLE = 32
BYTES_PER_SEGMENT_SPLIT = 128 + 32 + 16
BOUNCE_FAMILY = ("bounce0", "bounce", "tail")            # trace+shade launches (+ k_raygen/k_march: split)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")          # C1; other configs: pmc_traffic_<config>.json
# per-kernel PMC summaries of the same bench command (tools/pmc_final.sh -> tools/pmc_summary.py),
# committed per config: the roofline carries the family's VALU lane utilisation and wait fraction
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary_{}.json")
# bench.py's window parity (after the timed region, untimed): the oracle renders one window of the
# timed frame in the cpu_baseline subprocess (oracle/cpu_bench.py --window), compared byte for byte
WINDOW = {"C1": 16, "C2": 16, "C3": 8, "C4": 16}


def cpu_baseline(cfg, budget_s, lib="liboro.so", threads=0, dump=None):
    """The oracle (CPU restatement, `port`) on the host cores, in a child process
    (oracle/cpu_bench.py, which never touches the GPU): the reference's thread scheme on the
    config's frame for about `budget_s` seconds of full 1-spp passes.  `lib` picks the build
    (liboro.so: -O3 default x86-64; liboro_v3.so: -O3 -march=x86-64-v3).  threads: 0 =
    num_cpus::get() - 1 as main.rs:170 (the cgroup quota if set, else the affinity mask);
    -1 = num_cpus::get()."""
    env = dict(os.environ, ORO_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_bench.py"), "--config", cfg,
                        "--budget", str(budget_s), "--threads", str(threads)] + (["--dump", dump] if dump else []),
                       env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"cpu baseline {cfg}/{lib} failed: {r.stderr[-2000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def pmc_fields(name):
    """VALU lane utilisation and wait fractions of the bounce family from the committed per-kernel
    PMC summary of this config ("also report ... VALU utilization"), or None.
    The summary names the library build it profiled (om_build_id); `matches_timed_build` says
    whether that is the build timed here (an A/B build must not carry another build's
    counters as its own, so the caller reports them at the top level only when it matches)."""
    f = PMC_SUMMARY.format(name)
    if not os.path.exists(f):
        return None
    pm = json.load(open(f))
    comb = pm["combined"]["derived"]
    per = {k: {"valu_lane_utilisation": round(v["derived"]["valu_lane_utilisation"], 4),
               "wait_any_frac": round(v["derived"]["wait_any_frac"], 4),
               "wave_cycle_share": None}
           for k, v in pm["kernels"].items() if "valu_lane_utilisation" in v.get("derived", {})}
    # a kernel's share of the family's wave-cycles: mean per dispatch x dispatches
    wc = {k: v["counters"].get("SQ_WAVE_CYCLES", 0.0) * v["dispatches"].get("SQ_WAVE_CYCLES", 0)
          for k, v in pm["kernels"].items()}
    tot = sum(wc.values()) or 1.0
    for k in per:
        per[k]["wave_cycle_share"] = round(wc.get(k, 0.0) / tot, 4)
    build = pm.get("build_id")
    return {"valu_lane_utilisation": round(comb["valu_lane_utilisation"], 4),
            "wait_any_frac": round(comb["wait_any_frac"], 4), "wait_inst_frac": round(comb["wait_inst_frac"], 4),
            "per_kernel": per, "source": pm.get("source"), "file": os.path.relpath(f, ROOT),
            "build_id": build, "matches_timed_build": build is not None and build == L.build_id()}


def pmc_top(pmc, key):
    """A PMC field for the top level of a roofline: only when the summary profiled this build."""
    return pmc[key] if pmc and pmc["matches_timed_build"] else None


def window_parity(name, frame_u8, W, H, spp, depth, march_steps, adaptive=False):
    """One window of the timed frame (rank 0, after the timed region) vs the oracle's render of it
    (oracle/cpu_bench.py --window in a child process: the oracle never enters this process)."""
    import tempfile
    size = WINDOW[name]
    x0, y0 = W // 2 - size // 2, H // 2 - size // 2
    with tempfile.TemporaryDirectory() as td:
        dump = os.path.join(td, "window.npy")
        r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_bench.py"), "--config", name,
                            "--window", f"{W},{H},{x0},{y0},{size},{spp},{int(adaptive)}", "--dump", dump,
                            "--threads", "-1"],
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"oracle window {name} failed: {r.stderr[-2000:]}")
        info = json.loads(r.stdout.strip().splitlines()[-1])
        exp = np.load(dump, allow_pickle=False).view(np.uint8).reshape(-1, 40)
    pix = ((np.arange(y0, y0 + size)[:, None] * W) + np.arange(x0, x0 + size)[None, :]).reshape(-1)
    got = frame_u8.reshape(W * H, 40)[pix]
    bad = int(np.any(got != exp, axis=1).sum())
    if bad:
        print(f"bench: {name} window parity FAILED: {bad}/{pix.size} pixels differ from the oracle", file=sys.stderr)
    return {"window": [int(x0), int(y0), size], "spp": spp, "depth": depth, "pixels": int(pix.size), "adaptive": adaptive,
            "bit_exact_vs_oracle": bad == 0, "pixels_differ": bad, "oracle_s": info["seconds"],
            "objects_hit": int(np.count_nonzero(got.view(np.uint64)[:, 0]))}


class Control:
    """Harness control plane (gloo over host memory; absent at N=1): RCCL id hand-off,
    barriers, max over ranks.  No frame data goes through it."""

    def __init__(self, world_size, rank):
        self.n, self.rank = world_size, rank
        if world_size > 1:
            dist.init_process_group("gloo")

    def unique_id(self):
        uid = [shard.unique_id() if self.rank == 0 else None]
        if self.n > 1:
            dist.broadcast_object_list(uid, src=0)
        return uid[0]

    def barrier(self):
        if self.n > 1:
            dist.barrier()

    def max(self, x):
        if self.n == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.n > 1:
            dist.barrier()
            dist.destroy_process_group()


def layout(name, n, rank, spp_per_step, steps):
    """The rank's share of a config's job: (W, H, depth, spp_step, spp_total, cap, n_mine).  Every
    config but C4 is weak scaling (a rank renders its 1/n of the tiles at spp_per_step * n samples
    per step: fixed per-GPU work); C4 renders the fixed 4K frame (strong scaling)."""
    cfg = CONFIGS[name]
    W, H = cfg.get("size", (1920, 1080))
    depth = cfg.get("depth", MAX_DEPTH)
    spp_step = spp_per_step * (1 if name == "C4" else n)
    cap = shard.shard_capacity(W, H, n)
    n_mine = shard.tile_pixels(W, H, rank, n).size
    return W, H, depth, spp_step, spp_step * steps, cap, n_mine


def check_gathered(shard_u8, n_mine, frame_u8, W, H, n, rank, spp_total):
    """The timed job is complete: every pixel of the rank's shard took every sample, and on rank 0
    the gathered frame is complete and equal to rank 0's shard where they overlap."""
    mine = shard_u8[: n_mine * 40].view(L.PIXEL_STATS_DTYPE)
    assert int(mine["n"].min()) == spp_total and int(mine["n"].max()) == spp_total, "every pixel must take every sample"
    if rank == 0:
        fr = frame_u8.view(L.PIXEL_STATS_DTYPE)
        assert int(fr["n"].min()) == spp_total and int(fr["n"].max()) == spp_total, "gathered frame incomplete"
        assert np.array_equal(fr[shard.tile_pixels(W, H, 0, n)].view(np.uint8).reshape(-1), shard_u8[: n_mine * 40]), \
            "gathered frame differs from rank 0's shard"


def timed_region(ctl, steps, step, gather, sync):
    """K steps plus the gather, bracketed by a barrier + device synchronisation on both sides;
    -> the max over ranks of the wall time."""
    ctl.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    gather()
    sync()
    ctl.barrier()
    return ctl.max(time.perf_counter() - t0)


class HostComm:
    """--host-rehearsal only (tests/test_bench_cpu.py): a stand-in for shard.Comm over the gloo
    group, so that bench.py's N>1 control flow -- unique-id hand-off, RCCL's rank check, the spp
    split, shard capacities, the timed region's barriers and max, the gather into rank 0 and the
    checks on the gathered frame -- runs on CPU processes.  It renders nothing: a step adds its
    samples to every pixel of the shard with a pixel-keyed sum, and the gather moves the host
    shards to rank 0 and places them with the product's own om_shard_assemble_host."""

    def __init__(self, uid):
        assert len(uid) == L.OM_COMM_ID_BYTES
        self.n = dist.get_world_size() if dist.is_initialized() else 1
        self.rank = dist.get_rank() if dist.is_initialized() else 0

    def info(self):
        return self.n, self.rank

    def render_shard(self, pixels, shard_arr, spp):
        st = shard_arr[: pixels.size]
        st["n"] += spp
        st["sum"] += (pixels.astype(np.float32) * spp)[:, None]

    def gather_frame(self, shard_arr, W, H):
        shards = [None] * self.n if self.rank == 0 else None
        if self.n > 1:
            dist.gather_object(shard_arr.view(np.uint8), shards, dst=0)
        else:
            shards = [shard_arr.view(np.uint8)]
        return shard.assemble(W, H, shards).view(np.uint8) if self.rank == 0 else np.zeros(40, np.uint8)


def run_host_rehearsal(name, ctl, steps, warmup, spp_per_step):
    """bench.py's N>1 harness on CPU processes (--host-rehearsal, gloo): the run_config control flow
    with HostComm in place of RCCL and no device.  Returns the fields run_config returns (the
    roofline, work and window parity are device measurements: None)."""
    n, rank = ctl.n, ctl.rank
    comm = HostComm(ctl.unique_id())
    nranks_seen = check_comm_ranks(comm.info(), n, rank)
    W, H, depth, spp_step, spp_total, cap, n_mine = layout(name, n, rank, spp_per_step, steps)
    pixels = shard.tile_pixels(W, H, rank, n)
    sh = np.zeros(cap, dtype=L.PIXEL_STATS_DTYPE)
    for _ in range(warmup):
        comm.render_shard(pixels, sh, spp_step)
    sh[:] = 0
    out = {}
    elapsed = timed_region(ctl, steps, lambda i: comm.render_shard(pixels, sh, spp_step),
                           lambda: out.__setitem__("frame", comm.gather_frame(sh, W, H)), lambda: None)
    check_gathered(sh.view(np.uint8), n_mine, out["frame"], W, H, n, rank, spp_total)
    if rank == 0:
        fr = out["frame"].view(L.PIXEL_STATS_DTYPE)
        assert np.array_equal(fr["sum"][:, 0], np.arange(W * H, dtype=np.float32) * spp_total), "pixels misplaced"
    return {"value": round(W * H * spp_total / elapsed / 1e6, 3), "elapsed_s": elapsed, "steps": steps, "W": W, "H": H,
            "depth": depth, "spp_total": spp_total, "spp_step": spp_step, "mega": False, "roofline": None,
            "window_parity": None, "nranks_seen": nranks_seen, "work": None, "shard_capacity": cap, "shard_pixels": n_mine}


def run_config(name, args, ctl, local_rank, steps, warmup, spp_per_step, timing_mode, pmc_ok=True):
    """One config through the product path; returns the measured fields (value, roofline, work)."""
    if args.host_rehearsal:
        return run_host_rehearsal(name, ctl, steps, warmup, spp_per_step)
    cfg = CONFIGS[name]
    n, rank = ctl.n, ctl.rank
    # a dedicated (non-NULL) stream: the kernels, their HIP events and the RCCL gather run on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = stream.cuda_stream
    assert sptr, "need a non-default stream handle"
    world = make_scene(cfg["scene"], om)
    W, H = cfg.get("size", (1920, 1080))
    cam = om.default_camera(W / H)
    frozen = world.freeze(cam, device=local_rank, kernel=args.kernel, pipeline=args.pipeline)
    ctx = frozen.ctx
    L.check(L.lib.om_set_tail_bounce(ctx, args.tail), ctx)
    L.check(L.lib.om_set_streams(ctx, args.streams), ctx)
    L.check(L.lib.om_set_primary_lists(ctx, {"off": 0, "auto": 1, "on": 2}[args.primary_lists]), ctx)
    comm = shard.Comm(ctx, n, rank, ctl.unique_id())
    nranks_seen = check_comm_ranks(comm.info(), n, rank)     # RCCL's own view of the communicator
    W, H, depth, spp_step, spp_total, cap, n_mine = layout(name, n, rank, spp_per_step, steps)
    sh = torch.zeros(cap * 40, dtype=torch.uint8, device="cuda")
    frame = torch.zeros((W * H if rank == 0 else 1) * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(depth, TMIN, TMAX, spp_total, W, H, sample_count=spp_step, seed=SEED,
                       march_steps=cfg["march_steps"])

    def step():
        comm.render_shard(cam, p, sh.data_ptr(), sptr)

    for count in (1, 0):                                      # warm the counting and the production build
        L.check(L.lib.om_set_counting(ctx, count), ctx)
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        sh.zero_()
    torch.cuda.synchronize()

    kt = L.om_kernel_times()
    timing = timing_mode != "off"
    # region (default): two HIP events on `stream` around the K render calls and nothing inside
    # them (every call joins its side stream back to `stream`, so the pair spans all its work);
    # span / launch: the library's own events, once per call / around every launch
    L.check(L.lib.om_set_timing(ctx, {"off": 0, "region": 0, "launch": 1, "span": 2}[timing_mode]), ctx)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    # ---- timed region: ev0 before the first call, ev1 after the last, then the gather
    def timed_step(i):
        if i == 0:
            ev0.record(stream)
        step()

    def gather():
        ev1.record(stream)
        comm.gather_frame(sh.data_ptr(), W, H, frame.data_ptr(), sptr)   # RCCL: every shard to rank 0
    elapsed = timed_region(ctl, steps, timed_step, gather, torch.cuda.synchronize)
    # ---- end timed region
    region_s = ev0.elapsed_time(ev1) / 1e3                    # device time of the K calls
    L.check(L.lib.om_get_kernel_times(ctx, C.byref(kt)), ctx)
    L.check(L.lib.om_set_timing(ctx, 0), ctx)
    host = sh.cpu().numpy().copy()
    frame_u8 = frame.cpu().numpy()
    check_gathered(host, n_mine, frame_u8, W, H, n, rank, spp_total)
    parity = None
    if rank == 0 and not args.no_window_parity:
        parity = window_parity(name, frame_u8, W, H, spp_total, depth, cfg["march_steps"])

    # per-launch durations (untimed): the same K steps again, production build, every launch
    # bracketed by events on its stream (om_set_timing 1) -> the rocprof-comparable average
    # launch duration and the launch concurrency inside a call; same shard, bit for bit
    kl = L.om_kernel_times()
    if timing:
        sh.zero_()
        L.check(L.lib.om_set_timing(ctx, 1), ctx)
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        L.check(L.lib.om_get_kernel_times(ctx, C.byref(kl)), ctx)
        L.check(L.lib.om_set_timing(ctx, 0), ctx)
        assert np.array_equal(sh.cpu().numpy(), host), "per-launch timing changed the result"
    mega = kl.launches[L.KT_CLASSES.index("megakernel")] > 0     # the pipeline that actually ran (auto)
    fam = [L.KT_CLASSES.index("megakernel")] if mega else [L.KT_CLASSES.index(k) for k in BOUNCE_FAMILY]
    span_i = L.KT_CLASSES.index("megakernel" if mega else "bounce_span")

    # work counting (untimed): the same K steps again with the counting build; the shard it
    # produces must equal the timed one bit for bit (counters change nothing)
    sh.zero_()
    L.check(L.lib.om_reset_counters(ctx, C.c_void_p(sptr)), ctx)
    L.check(L.lib.om_set_counting(ctx, 1), ctx)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ctr = L.om_counters()
    L.check(L.lib.om_get_counters(ctx, C.byref(ctr)), ctx)
    assert np.array_equal(sh.cpu().numpy(), host), "counting build changed the result"
    comm.close()
    frozen.close()

    total_samples = W * H * spp_total        # all ranks together (each renders its 1/N of the pixels)
    value = total_samples / elapsed / 1e6
    marched = cfg["scene"] == "S-marched"

    # roofline of the dominant kernel: the trace+shade bounce family (all its launches: bounce 0,
    # bounces 1.., tail; marched worlds also k_raygen and k_march), algorithmic flops from the
    # live counters.  Its launches run two at a time (concurrent batches), so the rate is the
    # family's flops over the time it holds the GPU: the timed region's call spans.
    launches = sum(kl.launches[i] for i in fam) if timing else 0
    roof = None
    if timing and launches:
        # the timed region's device time of the calls: the event pair (region), or the sum of the
        # library's per-call spans (span / launch modes)
        span_s = region_s if timing_mode == "region" else kt.ms[span_i] / 1e3
        per_launch_s = sum(kl.ms[i] for i in fam) / 1e3 / launches  # rerun: mean launch duration
        rerun_span_s = kl.ms[span_i] / 1e3
        flops = (FLOP_EXACT_TEST * ctr.prim_tests + FLOP_BOX_TEST * ctr.pre_tests + FLOP_SEGMENT * ctr.segments
                 + FLOP_CAMERA_RAY * ctr.samples + FLOP_MARCH_STEP * ctr.march_steps)
        if marched and not mega:
            # split march pipeline with the tail from bounce 1 (the default for marched worlds, r04):
            # bounce 0 as the split pair (176 B per camera segment), then every later segment in the
            # lane-refilling tail, whose paths stay in registers: a path entering the tail is written
            # once and read once (128 B), bounded here by the later segments themselves
            nbytes = (BYTES_PER_SEGMENT_SPLIT + BYTES_PER_SAMPLE) * ctr.samples \
                + BYTES_PER_LATER_SEGMENT * (ctr.segments - ctr.samples)
        else:
            nbytes = BYTES_PER_LATER_SEGMENT * (ctr.segments - ctr.samples) + BYTES_PER_SAMPLE * ctr.samples
        achieved_tflops = flops / span_s / 1e12
        traffic, traffic_src = None, None
        pmc_file = PMC_TRAFFIC if name == "C1" else PMC_TRAFFIC.replace(".json", f"_{name}.json")
        if pmc_ok and os.path.exists(pmc_file) and not mega and args.kernel == "auto":
            pm = json.load(open(pmc_file))
            traffic, traffic_src = pm["hbm_bytes_per_launch"], pm["source"]
        pmc = pmc_fields(name) if (pmc_ok and not mega and args.kernel == "auto") else None
        roof = {"bound": "valu", "achieved": round(achieved_tflops, 3), "peak": PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved_tflops / PEAK_TFLOPS, 4), "traffic": traffic,
                "issue_peak": ISSUE_PEAK_TFLOPS, "frac_of_issue_peak": round(achieved_tflops / ISSUE_PEAK_TFLOPS, 4),
                "kernel": "render_kernel (megakernel)" if mega else
                          ("k_raygen+k_march+k_bounce<HIT> (bounce 0) + lane-refilling k_tail" if marched else
                           "k_bounce0+k_bounce+k_tail (fused trace+shade)"),
                "launches_per_step": round(launches / steps, 2),
                "avg_launch_ms": round(per_launch_s * 1e3, 4),
                "effective_ms_per_launch": round(span_s / launches * 1e3, 4),
                "launch_concurrency": round(per_launch_s * launches / rerun_span_s, 3) if rerun_span_s else None,
                "flop_per_launch": round(flops / launches), "algorithmic_bytes_per_launch": round(nbytes / launches),
                "hbm_achieved_gbs": round(nbytes / span_s / 1e9, 2), "traffic_source": traffic_src,
                "traffic_over_algorithmic": round(traffic / (nbytes / launches), 3) if traffic else None,
                "kernel_share_of_step": round(span_s / elapsed, 4), "timing": timing_mode,
                "valu_lane_utilisation": pmc_top(pmc, "valu_lane_utilisation"),
                "wait_any_frac": pmc_top(pmc, "wait_any_frac"), "pmc": pmc,
                "all_kernels_ms_per_step": {k: round(kl.ms[i] / steps, 4) for i, k in enumerate(L.KT_CLASSES)
                                            if kl.launches[i]}}
    return {
        "value": round(value, 3), "elapsed_s": elapsed, "steps": steps, "W": W, "H": H, "depth": depth,
        "spp_total": spp_total, "spp_step": spp_step, "mega": mega, "roofline": roof,
        "window_parity": parity, "nranks_seen": nranks_seen,
        "work": {"segments_per_sample": round(ctr.segments / max(1, ctr.samples), 4),
                 "prim_tests_per_segment": round(ctr.prim_tests / max(1, ctr.segments), 3),
                 "box_tests_per_segment": round(ctr.pre_tests / max(1, ctr.segments), 3),
                 "march_steps_per_segment": round(ctr.march_steps / max(1, ctr.segments), 3),
                 "gsegments_per_s": round(ctr.segments * n / elapsed / 1e9, 4)},
    }


def check_comm_ranks(seen, world_size, rank):
    """RCCL's (nranks, rank) for the bench's communicator must be the launcher's (WORLD_SIZE, RANK):
    a silently smaller communicator would time a fraction of the job.  Returns nranks."""
    n_seen, r_seen = seen
    if n_seen != world_size or r_seen != rank:
        raise SystemExit(f"bench: RCCL communicator has {n_seen} ranks (this is rank {r_seen}), "
                         f"but WORLD_SIZE={world_size} RANK={rank}")
    return n_seen


def config_entry(name, e, note=""):
    return {"metric": "Msamples/s", "value": e["value"], "ms_per_step": round(e["elapsed_s"] / e["steps"] * 1e3, 4),
            "workload": workload(name, e) + note, "pipeline": "megakernel" if e["mega"] else "wavefront",
            "roofline": e["roofline"], "work": e["work"], "window_parity": e["window_parity"]}


def workload(name, r):
    cfg = CONFIGS[name]
    return (f"{name} {cfg['scene']} {r['W']}x{r['H']}, {r['spp_total']} spp timed ({r['spp_step']} spp/step), "
            f"depth {r['depth']}" + (f", {cfg['march_steps']} march steps" if name == "C2" else ""))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C1", choices=[c for c in CONFIGS if c != "C0"])
    ap.add_argument("--steps", type=int, default=None, help="default: the config's spp / spp-per-step (C1: 4)")
    ap.add_argument("--spp-per-step", type=int, default=SPP_PER_STEP, help="samples per pixel per step (one render call)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kernel", default="auto", choices=list(L.KERNELS))
    ap.add_argument("--pipeline", default="auto", choices=list(L.PIPELINES))
    ap.add_argument("--tail", type=int, default=0, help="first bounce of the persistent tail launch (0 = library default)")
    ap.add_argument("--streams", type=int, default=2, help="wavefront batches in flight per call (om_set_streams; 1 = serial)")
    ap.add_argument("--kernel-timing", default="region", choices=["region", "span", "launch", "off"],
                    help="HIP events in the timed region: region = one pair around all K calls (default), "
                         "span = the library's pair around each call's bounce kernels (2 events/step), "
                         "launch = around every launch (per-kernel breakdown); off = none and no roofline")
    ap.add_argument("--primary-lists", default="auto", choices=["off", "auto", "on"],
                    help="bounce-0 per-tile candidate lists (DESIGN.md §5.10); auto = when they average <= 12")
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="quick mode: the headline config only (no CPU baselines, no `configs` block)")
    ap.add_argument("--no-extras", action="store_true", help="no `configs` block (C2/C3/C0) at N=1")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--host-rehearsal", action="store_true",
                    help="tests only: run the N>1 control flow on CPU processes (gloo), RCCL replaced by HostComm; "
                         "renders nothing, prints no measurement")
    ap.add_argument("--no-window-parity", action="store_true",
                    help="skip the oracle window of each timed frame (untimed; a few seconds of host CPU)")
    args = ap.parse_args()
    cfg = CONFIGS[args.config]

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}")
    if world_size > 1 and int(os.environ.get("LOCAL_WORLD_SIZE", world_size)) == world_size:
        # one node: RCCL's bootstrap (the unique id rank 0 hands out) over loopback, whatever the
        # container's hostname and interfaces; the frame data goes over xGMI, not sockets
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    if not args.host_rehearsal:
        torch.cuda.set_device(local_rank)
    ctl = Control(world_size, rank)
    steps = args.steps
    if steps is None:
        steps = cfg["spp"] // args.spp_per_step if args.config != "C4" else cfg["spp"] // args.spp_per_step
    r = run_config(args.config, args, ctl, local_rank, steps, args.warmup, args.spp_per_step, args.kernel_timing)
    if args.host_rehearsal:                  # no device ran: a rehearsal record, never a metric line
        if rank == 0:
            print(json.dumps({"host_rehearsal": True, "config": args.config, "n_ranks": world_size, "steps": steps,
                              **{k: r[k] for k in ("spp_step", "spp_total", "W", "H", "nranks_seen", "shard_capacity",
                                                   "shard_pixels", "elapsed_s")}}))
        ctl.close()
        return

    extras = None
    quick = args.no_cpu_baseline or args.no_extras
    if rank == 0 and world_size == 1 and not quick and args.config == "C1":
        extras = {}
        # C1_frame: exactly the quoted "1080p@512spp" frame, one fresh frame of 4 x 128-spp calls
        # timed alone (its end-of-call drains included), beside the driver's --steps run
        c1 = CONFIGS["C1"]
        e = run_config("C1", args, ctl, local_rank, c1["spp"] // args.spp_per_step, 1, args.spp_per_step, "region")
        extras["C1_frame"] = config_entry("C1", e, " (one fresh 512-spp frame)")
        extras["C1_frame"]["ms_per_frame"] = round(e["elapsed_s"] * 1e3, 4)
        for name in ("C2", "C3"):
            c = CONFIGS[name]
            e = run_config(name, args, ctl, local_rank, c["spp"] // args.spp_per_step, 1, args.spp_per_step, "region")
            extras[name] = config_entry(name, e)
            extras[name]["cpu_baseline"] = cpu_baseline(name, min(8.0, args.cpu_budget))
        # C4's 4K frame at N=1: 256 of the config's 4096 spp (the full frame is the multi-GPU run,
        # --config C4), so the driver's line exercises the 3840x2160 frame too
        e = run_config("C4", args, ctl, local_rank, max(1, 256 // args.spp_per_step), 1, args.spp_per_step, "region")
        extras["C4"] = config_entry("C4", e, " (N=1 leg of the 8-GPU config: 256 of its 4096 spp)")
        extras["C4"]["cpu_baseline"] = cpu_baseline("C4", min(6.0, args.cpu_budget))
        extras["C0"] = run_c0(args)
        extras["C1_adaptive"] = run_adaptive(args)
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.config, args.cpu_budget)
        cpu["second"] = cpu_baseline(args.config, args.cpu_budget, "liboro_v3.so")
        cpu["all_cores"] = cpu_baseline(args.config, args.cpu_budget, threads=-1)   # nproc-1 and nproc

    rccl = shard.rccl_library()       # the RCCL om_gather_frame ran on (torch's, by soname: DESIGN.md §6)
    if rank == 0:
        out = {
            "metric": "Msamples/s (W×H×spp/s) + achieved HBM GB/s, 1080p@512spp traced scene",
            "value": r["value"],
            "unit": "Msamples/s",
            "n_gpus": world_size,
            "steps": steps,
            "warmup": args.warmup,
            "ms_per_step": round(r["elapsed_s"] / steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "C4" else "weak",   # C4: the fixed 4K x 4096-spp frame
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: {cfg['scene']} (om-rng scene seed 0x5EED), render seed 1",
            "config": {"workload": workload(args.config, r), "width": r["W"], "height": r["H"],
                       "spp_per_step": r["spp_step"], "max_depth": r["depth"],
                       "parallelism": f"tile{world_size}", "gather": "RCCL send/recv (om_gather_frame)",
                       "rccl_library": rccl[0], "rccl_version": rccl[1],
                       "kernel": args.kernel,
                       "pipeline": args.pipeline + (("->megakernel" if r["mega"] else "->wavefront")
                                                    if args.pipeline == "auto" else ""),
                       "tail_bounce": args.tail or "default", "streams": args.streams},
            "nranks_seen": r["nranks_seen"],
            "window_parity": r["window_parity"],
            "hbm_gbs": r["roofline"]["hbm_achieved_gbs"] if r["roofline"] else None,
            "roofline": r["roofline"],
            "work": r["work"],
            "cpu_baseline": cpu,
            "configs": extras,
        }
        print(json.dumps(out))
    ctl.close()


def run_adaptive(args, spp=512, per_call=128, reps=3):
    """C1's 1080p frame in the reference's default mode, adaptive sampling (render_thread.rs:31-38,
    68-102, 196-198): a pixel retires after 5 samples that leave its 8-bit colour unchanged, and
    the progress counter credits its skipped samples.  value = credited Msamples/s (the
    reference's samples_atom rate), beside the samples actually taken.  One fresh 512-spp frame in
    128-spp calls per rep (each call: the live pixels dealt to the streams, each stream's batches
    planned on the device from its live list); the frame must be identical across
    reps and to the serial schedule, and its centre window to the oracle's adaptive render
    (window_parity); the roofline is the counting pass's executed work over the median frame."""
    W, H = CONFIGS["C1"].get("size", (1920, 1080))
    stream = torch.cuda.Stream()
    sp = C.c_void_p(stream.cuda_stream)
    world = make_scene("S-traced", om)
    cam = om.default_camera(W / H)
    frames = {}
    out = {}
    ctrs = {}
    launches = {}
    for label, streams in (("concurrent", args.streams), ("serial", 1)):
        fz = world.freeze(cam, kernel=args.kernel, pipeline=args.pipeline)
        L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
        st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
        p = om.make_params(MAX_DEPTH, TMIN, TMAX, spp, W, H, sample_count=per_call, seed=SEED, adaptive=True)

        def frame():
            for _ in range(spp // per_call):
                L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()), sp),
                        fz.ctx)
        L.check(L.lib.om_set_counting(fz.ctx, 1), fz.ctx)          # counting pass: samples taken, credit, work
        L.check(L.lib.om_reset_counters(fz.ctx, sp), fz.ctx)
        frame()
        torch.cuda.synchronize()
        ctr = L.om_counters()
        L.check(L.lib.om_get_counters(fz.ctx, C.byref(ctr)), fz.ctx)
        ctrs[label] = ctr
        ref = st.clone()
        L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)          # production build, timed
        times = []
        for _ in range(reps):
            st.zero_()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            frame()
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            assert torch.equal(st, ref), "adaptive frame differs between reps / builds"
        # bounce-family launches of one frame (the library's own count, timing mode 2), for the
        # PMC traffic per frame; the same frame again, bit for bit
        kt = L.om_kernel_times()
        st.zero_()
        L.check(L.lib.om_set_timing(fz.ctx, 2), fz.ctx)
        frame()
        torch.cuda.synchronize()
        L.check(L.lib.om_get_kernel_times(fz.ctx, C.byref(kt)), fz.ctx)
        L.check(L.lib.om_set_timing(fz.ctx, 0), fz.ctx)
        assert torch.equal(st, ref), "timing changed the adaptive frame"
        launches[label] = int(kt.launches[L.KT_CLASSES.index("bounce_span")])
        fz.close()
        dt = sorted(times)[len(times) // 2]
        frames[label] = ref
        out[label] = {"credited_msamples_s": round(ctr.credited / dt / 1e6, 3),
                      "taken_msamples_s": round(ctr.samples / dt / 1e6, 3), "ms_per_frame": round(dt * 1e3, 4),
                      "taken_frac": round(ctr.samples / (W * H * spp), 4),
                      "gsegments_per_s": round(ctr.segments / dt / 1e9, 3)}
    assert torch.equal(frames["concurrent"], frames["serial"]), "adaptive schedules differ"
    c = out["concurrent"]
    ctr = ctrs["concurrent"]
    dt = c["ms_per_frame"] / 1e3
    parity = None
    if not args.no_window_parity:
        parity = window_parity("C1", frames["concurrent"].cpu().numpy(), W, H, spp, MAX_DEPTH, 1024, adaptive=True)
    # executed work of the frame (counting pass; speculative samples included in the segments and
    # tests, camera rays priced at the samples taken: a lower bound) over the median frame time
    flops = (FLOP_EXACT_TEST * ctr.prim_tests + FLOP_BOX_TEST * ctr.pre_tests + FLOP_SEGMENT * ctr.segments
             + FLOP_CAMERA_RAY * ctr.samples)
    nbytes = BYTES_PER_LATER_SEGMENT * max(0, ctr.segments - ctr.samples) + BYTES_PER_SAMPLE * ctr.samples
    pmc = pmc_fields("C1_adaptive")
    # HBM traffic per frame: the PMC mean per bounce-family launch (profiles/pmc_traffic_C1_adaptive.json,
    # empty planned batches included) x the frame's launches
    traffic, traffic_src = None, None
    tf = PMC_TRAFFIC.replace(".json", "_C1_adaptive.json")
    if os.path.exists(tf) and args.kernel == "auto":
        pm = json.load(open(tf))
        traffic, traffic_src = pm["hbm_bytes_per_launch"] * launches["concurrent"], pm["source"]
    achieved = flops / dt / 1e12
    roof = {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_TFLOPS, 4), "frac_of_issue_peak": round(achieved / ISSUE_PEAK_TFLOPS, 4),
            "kernel": "k_bounce0+k_bounce+k_tail (fused trace+shade), adaptive live-list batches",
            "timing": "median frame wall time (host clock around the 4 calls)",
            "flop_per_frame": round(flops), "algorithmic_bytes_per_frame": round(nbytes),
            "launches_per_frame": launches["concurrent"], "traffic_per_frame": round(traffic) if traffic else None,
            "traffic_source": traffic_src, "traffic_over_algorithmic": round(traffic / nbytes, 3) if traffic else None,
            "hbm_achieved_gbs": round(nbytes / dt / 1e9, 2),
            "valu_lane_utilisation": pmc_top(pmc, "valu_lane_utilisation"),
            "wait_any_frac": pmc_top(pmc, "wait_any_frac"), "pmc": pmc}
    return {"metric": "credited Msamples/s", "value": c["credited_msamples_s"], "taken_msamples_s": c["taken_msamples_s"],
            "taken_frac": c["taken_frac"], "ms_per_frame": c["ms_per_frame"],
            "workload": f"C1 S-traced {W}x{H}, {spp} spp adaptive (the reference's default), {per_call}-spp calls, "
                        f"depth {MAX_DEPTH}, median of {reps} fresh frames",
            "work": {"segments_per_taken_sample": round(ctr.segments / max(1, ctr.samples), 4),
                     "prim_tests_per_segment": round(ctr.prim_tests / max(1, ctr.segments), 3),
                     "box_tests_per_segment": round(ctr.pre_tests / max(1, ctr.segments), 3),
                     "gsegments_per_s": c["gsegments_per_s"]},
            "roofline": roof, "window_parity": parity,
            "serial_batches": out["serial"], "schedules_bit_identical": True}


def run_c0(args, reps=20):
    """C0, the reference's CPU case (BASELINE.json configs[0]: 400x225, 64 spp, depth 8): the
    whole 64-spp frame per step on the GPU (device-resident Stats, zeroed before each frame)
    beside the CPU oracle rendering the same frame (the frame tests/test_golden.py and the
    parity tests hold bit-identical between the two)."""
    cfg = CONFIGS["C0"]
    W, H = cfg["size"]
    world = make_scene(cfg["scene"], om)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    L.check(L.lib.om_set_counting(fz.ctx, 0), fz.ctx)
    stream = torch.cuda.Stream()
    frames = [torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda") for _ in range(reps + 1)]
    p = om.make_params(cfg["depth"], TMIN, TMAX, cfg["spp"], W, H, seed=SEED)

    def frame(buf):
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(buf.data_ptr()),
                                       C.c_void_p(stream.cuda_stream)), fz.ctx)
    frame(frames[-1])                                                      # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in frames[:reps]:
        frame(b)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    got = frames[0].cpu().numpy()
    same = all(torch.equal(b, frames[0]) for b in frames[1:])
    fz.close()
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        dump = os.path.join(td, "c0_oracle.npy")
        cpu = cpu_baseline("C0", 0.0, dump=dump)                        # the oracle renders the same frame
        exp = np.load(dump, allow_pickle=False)
    bad = int(np.any(got.reshape(-1, 40) != exp.view(np.uint8).reshape(-1, 40), axis=1).sum())
    assert bad == 0, f"C0: {bad} pixels of the GPU frame differ from the oracle's"
    return {"metric": "Msamples/s", "value": round(W * H * cfg["spp"] / dt / 1e6, 3), "ms_per_frame": round(dt * 1e3, 4),
            "workload": f"C0 S-traced {W}x{H}, {cfg['spp']} spp, depth {cfg['depth']} (whole frame per step, {reps} frames)",
            "frame_n_ok": bool((got.view(L.PIXEL_STATS_DTYPE)["n"] == cfg["spp"]).all()),
            "frame_bit_exact_vs_oracle": bad == 0, "frames_identical": bool(same),
            "cpu_baseline": cpu, "gpu_over_cpu": round(W * H * cfg["spp"] / dt / 1e6 / cpu["value"], 1)}


if __name__ == "__main__":
    main()
