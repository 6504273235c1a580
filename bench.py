"""bench.py — MI355X benchmark of the ray_color hot path (BASELINE.json metric).

Workload (config C1, BASELINE.json configs[1]): the S-traced random_scene (main.rs:37-100
minus the torus block, om-rng scene seed 0x5EED), camera of main.rs:136-142, 1920x1080,
max_depth 50, tmin 0.001, tmax 100, fixed spp (adaptive off).  One STEP = one progressive
pass of SPP_PER_STEP samples over every pixel this rank owns, accumulated into the
per-pixel Stats in HBM (render_thread.rs:176-199, batched).  16 steps of 32 spp at N=1 =
the full 512-spp frame; the library runs each step as two concurrent 16-spp batches
(om_set_streams).

N>1 (torch.distributed.run, one rank per GPU): 8x8 pixel tiles are dealt round-robin to
ranks (main.rs:172-189's chunk round-robin); every rank renders its tiles at
SPP_PER_STEP*N samples per step (fixed per-GPU work: weak scaling) and one RCCL gather
of the finished f32 framebuffer to rank 0 closes the timed region.

Output: ONE JSON line on rank 0 (see DESIGN.md §7 for every field).
"""
import argparse
import ctypes as C
import json
import os
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

W, H, MAX_DEPTH, TMIN, TMAX, SEED, SCENE_SEED = 1920, 1080, 50, 0.001, 100.0, 1, 0x5EED
SPP_PER_STEP = 32
# BASELINE.json configs: C1 is the metric's workload (the default line); C2/C3/C4 are measured
# with --config for DESIGN.md (the marched SDF scene at 256 march steps, the 10k-sphere BVH,
# the 4K frame of the multi-GPU config).
CONFIGS = {
    "C1": {"scene": "S-traced", "spp": 512, "march_steps": 1024},
    "C2": {"scene": "S-marched", "spp": 256, "march_steps": 256},
    "C3": {"scene": "S-10k", "spp": 256, "march_steps": 1024},
    # the multi-GPU config (BASELINE.json configs[4]: 3840x2160, 4096 spp, 8 GPUs); weak scaling
    # as for C1: each rank renders its 1/N of the tiles at spp_per_step * N per step
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
# Algorithmic HBM bytes of the bounce kernels (SoA path queue): a segment
# after the first reads its 64-B path and writes the 64-B survivor; a sample reads its
# pixel id + Stats.n/flags (12 B) and writes its result (20 B).
BYTES_PER_LATER_SEGMENT = 128
BYTES_PER_SAMPLE = 32
BOUNCE_FAMILY = ("bounce0", "bounce", "tail")            # one fused trace+shade kernel body
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")          # C1; other configs: pmc_traffic_<config>.json


def cpu_baseline(budget_s=12.0, cfg="C1"):
    """Oracle (CPU restatement, `port`) on the host: the reference's thread scheme
    (num_cpus-1 workers, 2730-px round-robin chunks, main.rs:170-189) on the same frame."""
    from oracle import oracle as O  # checker / baseline only
    cores = max(1, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 2)) - 1)
    ow = make_scene(CONFIGS[cfg]["scene"], O)
    # the oracle is brute force: for the 10k-sphere scene a 1/64-area frame of the same
    # scene and camera (per-sample cost does not depend on the resolution)
    w, h = (W // 8, H // 8) if cfg == "C3" else (W, H)
    cam = O.default_camera(w / h)
    done, t_total, passes = 0, 0.0, 0
    stats = np.zeros(w * h, dtype=O.PIXEL_STATS_DTYPE)
    spp_total = 64
    while passes == 0 or (t_total < budget_s and passes < spp_total):
        p = O.params(w, h, spp_total, sample_count=1, max_depth=MAX_DEPTH, seed=SEED,
                     march_steps=CONFIGS[cfg]["march_steps"])
        t0 = time.perf_counter()
        _, ctr = O.render(ow, cam, p, stats=stats, nthreads=cores)
        t_total += time.perf_counter() - t0
        done += ctr["samples"]
        passes += 1
    return {"value": done / t_total / 1e6, "unit": "Msamples/s", "cores": cores, "kind": "port",
            "sample": f"{cfg} frame {w}x{h}, {passes} spp (full passes), depth {MAX_DEPTH}, {CONFIGS[cfg]['scene']}, "
                      f"{cores} threads, {t_total:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--config", default="C1", choices=list(CONFIGS))
    ap.add_argument("--steps", type=int, default=None, help="default: the config's spp / spp-per-step (C1: 32)")
    ap.add_argument("--spp-per-step", type=int, default=SPP_PER_STEP, help="samples per pixel per step (one render call)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--kernel", default="auto", choices=list(L.KERNELS))
    ap.add_argument("--pipeline", default="auto", choices=list(L.PIPELINES))
    ap.add_argument("--tail", type=int, default=0, help="first bounce of the persistent tail launch (0 = library default)")
    ap.add_argument("--streams", type=int, default=2, help="wavefront batches in flight per call (om_set_streams; 1 = serial)")
    ap.add_argument("--kernel-timing", default="span", choices=["span", "launch", "off"],
                    help="HIP events in the timed region: span = once around each batch's bounce kernels "
                         "(2 events/step, default), launch = around every launch (per-kernel breakdown)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the measured path); gloo gathers through host memory and maps "
                         "ranks onto the visible GPUs (a functional rehearsal of N>1 on a 1-GPU box)")
    ap.add_argument("--primary-lists", default="auto", choices=["off", "auto", "on"],
                    help="bounce-0 per-tile candidate lists (DESIGN.md §5.10); auto = when they average <= 12")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    args = ap.parse_args()
    cfg = CONFIGS[args.config]
    global W, H
    W, H = cfg.get("size", (W, H))
    if args.steps is None:
        args.steps = cfg["spp"] // (args.spp_per_step * args.gpus) if args.config == "C4" else cfg["spp"] // args.spp_per_step

    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world_size}")
    gloo = args.dist_backend == "gloo"
    if gloo:
        local_rank = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    if world_size > 1:
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    # ---- setup (not timed): scene build + freeze/upload, camera, tile lists
    # a dedicated (non-NULL) stream: the kernel, its HIP events and the collectives all run on it
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sptr = C.c_void_p(stream.cuda_stream)
    assert sptr.value, "need a non-default stream handle"
    world = make_scene(cfg["scene"], om)
    cam = om.default_camera(W / H)
    frozen = world.freeze(cam, device=local_rank, kernel=args.kernel, pipeline=args.pipeline)
    ctx = frozen.ctx
    L.check(L.lib.om_set_tail_bounce(ctx, args.tail), ctx)
    L.check(L.lib.om_set_streams(ctx, args.streams), ctx)
    L.check(L.lib.om_set_primary_lists(ctx, {"off": 0, "auto": 1, "on": 2}[args.primary_lists]), ctx)
    spp_step = args.spp_per_step * world_size                # fixed per-GPU samples per step
    spp_total = spp_step * args.steps
    pix = shard.tile_pixels(W, H, rank, world_size)
    n_px = int(pix.size)
    dev_pix = torch.from_numpy(pix.view(np.int32)).cuda()
    stats = torch.zeros(n_px * 40, dtype=torch.uint8, device="cuda")

    def step(p):
        L.check(L.lib.om_render_device_pixels(ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(stats.data_ptr()),
                                              C.c_void_p(dev_pix.data_ptr()), n_px, sptr), ctx)

    p = om.make_params(MAX_DEPTH, TMIN, TMAX, spp_total, W, H, sample_count=spp_step, seed=SEED,
                       march_steps=cfg["march_steps"])
    for _ in range(args.warmup):
        step(p)
    torch.cuda.synchronize()
    stats.zero_()                                            # timed frame starts from empty Stats
    L.check(L.lib.om_set_counting(ctx, 0), ctx)              # production build: counters compiled out
    for _ in range(args.warmup):                             # warm the non-counting kernel too
        step(p)
    torch.cuda.synchronize()
    stats.zero_()
    gathered, send = None, None
    if world_size > 1:                                       # gather buffers (equal-size shards), allocated untimed
        n_max = shard.shard_capacity(W, H, world_size) * 40
        send = torch.zeros(n_max, dtype=torch.uint8, device="cpu" if gloo else "cuda")
        gathered = [torch.empty_like(send) for _ in range(world_size)] if rank == 0 else None
    torch.cuda.synchronize()

    kt = L.om_kernel_times()
    timing = args.kernel_timing != "off"
    L.check(L.lib.om_set_timing(ctx, {"off": 0, "launch": 1, "span": 2}[args.kernel_timing]), ctx)   # events on `stream`

    # ---- timed region
    if world_size > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(p)
    if world_size > 1:                                       # RCCL gather of the f32 framebuffer to rank 0
        send[: stats.numel()] = stats.cpu() if gloo else stats
        dist.gather(send, gathered, dst=0)
    torch.cuda.synchronize()
    if world_size > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # ---- end timed region

    t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else "cuda")
    if world_size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    L.check(L.lib.om_get_kernel_times(ctx, C.byref(kt)), ctx)
    L.check(L.lib.om_set_timing(ctx, 0), ctx)
    host = stats.cpu().numpy().view(L.PIXEL_STATS_DTYPE).copy()
    assert int(host["n"].min()) == spp_total and int(host["n"].max()) == spp_total, "every pixel must take every sample"

    # per-launch durations (untimed): the same K steps again, production build, every launch
    # bracketed by events on its stream (om_set_timing 1) -> the rocprof-comparable average
    # launch duration and the launch concurrency inside a call; same frame, bit for bit
    mega = kt.launches[L.KT_CLASSES.index("megakernel")] > 0     # the pipeline that actually ran (auto)
    fam = [L.KT_CLASSES.index("megakernel")] if mega else [L.KT_CLASSES.index(k) for k in BOUNCE_FAMILY]
    span_i = L.KT_CLASSES.index("megakernel" if mega else "bounce_span")
    kl = L.om_kernel_times()
    if timing:
        stats.zero_()
        L.check(L.lib.om_set_timing(ctx, 1), ctx)
        for _ in range(args.steps):
            step(p)
        torch.cuda.synchronize()
        L.check(L.lib.om_get_kernel_times(ctx, C.byref(kl)), ctx)
        L.check(L.lib.om_set_timing(ctx, 0), ctx)
        assert np.array_equal(stats.cpu().numpy(), host.view(np.uint8)), "per-launch timing changed the result"

    # work counting (untimed): the same K steps again with the counting build; the
    # frame it produces must equal the timed one bit for bit (counters change nothing)
    stats.zero_()
    L.check(L.lib.om_reset_counters(ctx, sptr), ctx)
    L.check(L.lib.om_set_counting(ctx, 1), ctx)
    for _ in range(args.steps):
        step(p)
    torch.cuda.synchronize()
    ctr = L.om_counters()
    L.check(L.lib.om_get_counters(ctx, C.byref(ctr)), ctx)
    assert np.array_equal(stats.cpu().numpy(), host.view(np.uint8)), "counting build changed the result"

    total_samples = W * H * spp_total                          # all ranks together
    value = total_samples / elapsed / 1e6

    # roofline of the dominant kernel: the fused trace+shade bounce kernel (all its launches:
    # bounce 0, bounces 1.., tail), algorithmic flops from the live counters.  Its launches run
    # two at a time (concurrent batches), so the rate is the family's flops over the time it
    # holds the GPU: the timed region's call spans (events on the call's stream).
    launches = sum(kl.launches[i] for i in fam) if timing else 0
    roof = None
    if timing and launches:
        span_s = kt.ms[span_i] / 1e3                               # timed region: the calls' device time
        per_launch_s = sum(kl.ms[i] for i in fam) / 1e3 / launches  # rerun: mean launch duration
        rerun_span_s = kl.ms[span_i] / 1e3
        flops = (FLOP_EXACT_TEST * ctr.prim_tests + FLOP_BOX_TEST * ctr.pre_tests + FLOP_SEGMENT * ctr.segments
                 + FLOP_CAMERA_RAY * ctr.samples + FLOP_MARCH_STEP * ctr.march_steps)
        nbytes = BYTES_PER_LATER_SEGMENT * (ctr.segments - ctr.samples) + BYTES_PER_SAMPLE * ctr.samples
        achieved_tflops = flops / span_s / 1e12
        traffic, traffic_src = None, None
        pmc_file = PMC_TRAFFIC if args.config == "C1" else PMC_TRAFFIC.replace(".json", f"_{args.config}.json")
        if os.path.exists(pmc_file) and not mega and args.kernel == "auto":
            pm = json.load(open(pmc_file))
            traffic, traffic_src = pm["hbm_bytes_per_launch"], pm["source"]
        roof = {"bound": "valu", "achieved": round(achieved_tflops, 3), "peak": PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved_tflops / PEAK_TFLOPS, 4), "traffic": traffic,
                "issue_peak": ISSUE_PEAK_TFLOPS, "frac_of_issue_peak": round(achieved_tflops / ISSUE_PEAK_TFLOPS, 4),
                "kernel": "render_kernel (megakernel)" if mega else "k_bounce0+k_bounce+k_tail (fused trace+shade)",
                "launches_per_step": round(launches / args.steps, 2),
                "avg_launch_ms": round(per_launch_s * 1e3, 4),
                "effective_ms_per_launch": round(span_s / launches * 1e3, 4),
                "launch_concurrency": round(per_launch_s * launches / rerun_span_s, 3) if rerun_span_s else None,
                "flop_per_launch": round(flops / launches), "algorithmic_bytes_per_launch": round(nbytes / launches),
                "hbm_achieved_gbs": round(nbytes / span_s / 1e9, 2), "traffic_source": traffic_src,
                "kernel_share_of_step": round(span_s / elapsed, 4), "timing": args.kernel_timing,
                "all_kernels_ms_per_step": {k: round(kl.ms[i] / args.steps, 4) for i, k in enumerate(L.KT_CLASSES)
                                            if kl.launches[i]}}
    hbm_gbs = roof["hbm_achieved_gbs"] if roof else None

    if rank == 0:
        if gathered is not None:                             # assemble + verify the gathered frame (untimed)
            frame = shard.assemble(W, H, [g.cpu().numpy() for g in gathered])
            assert int(frame["n"].min()) == spp_total, "gathered frame incomplete"
        cpu = None
        if world_size == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_budget, args.config)
        out = {
            "metric": "Msamples/s (W×H×spp/s) + achieved HBM GB/s, 1080p@512spp traced scene",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "C4" else "weak",   # C4: the fixed 4K x 4096-spp frame
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic: {cfg['scene']} (om-rng scene seed 0x5EED), render seed 1",
            "config": {"workload": f"{args.config} {cfg['scene']} {W}x{H}, {spp_total} spp timed ({spp_step} spp/step), "
                                   f"depth {MAX_DEPTH}" + (f", {cfg['march_steps']} march steps" if args.config == "C2" else ""),
                       "width": W, "height": H, "spp_per_step": spp_step, "max_depth": MAX_DEPTH,
                       "parallelism": f"tile{world_size}" + ("/gloo" if gloo and world_size > 1 else ""),
                       "kernel": args.kernel,
                       "pipeline": args.pipeline + (("->megakernel" if mega else "->wavefront") if args.pipeline == "auto" else ""),
                       "tail_bounce": args.tail or "default", "streams": args.streams},
            "hbm_gbs": hbm_gbs,
            "roofline": roof,
            "work": {"segments_per_sample": round(ctr.segments / max(1, ctr.samples), 4),
                     "prim_tests_per_segment": round(ctr.prim_tests / max(1, ctr.segments), 3),
                     "box_tests_per_segment": round(ctr.pre_tests / max(1, ctr.segments), 3),
                     "march_steps_per_segment": round(ctr.march_steps / max(1, ctr.segments), 3),
                     "gsegments_per_s": round(ctr.segments * world_size / elapsed / 1e9, 4)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world_size > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
