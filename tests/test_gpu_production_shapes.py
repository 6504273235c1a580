"""Parity at the batch shapes the bench times (VERDICT r03 "next" #1).

The numbers bench.py posts come from size-dependent schedules that the small oracle tests never
reach: 16-spp batches of 133 M paths with the persistent tail from bounce 24 (C4's 4K frame,
om_wavefront.hip `kTailBigBatch`), 128-spp calls over a tile shard (C1's call), the L2-resident
BVH2 with tail 10 and 8192 lanes per CU (C3), and the split march pipeline at 1080p (C2).  Each
test renders the config's frame in ONE call of the production shape, checks with the library's
own launch counts that the call really ran that schedule, and then compares it

  * bit for bit with the same frame rendered as 1-spp calls (2-8 M-path batches, one stream,
    the default tail: a different schedule whose bits must not differ, render_thread.rs:176-199
    renders a pixel's samples in order whatever the thread split), and
  * bit for bit with the CPU oracle on windows of the frame (sky, the sphere field, the ground;
    hits.rs:270-334 + render_thread.rs:105-143 restated in oracle/om_oracle.cpp).
"""
import ctypes as C

import numpy as np
import pytest

from scenes_common import compare_stats, compare_stats_nan_payload

pytestmark = pytest.mark.gpu

SEED = 1                      # bench.py's render seed


def _scene(om_or_oracle, name):
    if name == "S-traced":
        return om_or_oracle.random_scene(0x5EED)
    if name == "S-marched":
        return om_or_oracle.marched_scene()
    return om_or_oracle.random_scene(0x5EED, grid_half=50, extras=False)   # S-10k


def _render_calls(om, fz, cam, W, H, spp, per_call, march_steps, timing=False, adaptive=False):
    """`spp // per_call` om_render_device calls of `per_call` samples into a fresh device frame;
    returns (frame, kernel times of the calls when `timing`)."""
    import torch
    from raytracingoneweekend_amd import _lib as L
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=per_call, seed=SEED, march_steps=march_steps,
                       adaptive=adaptive)
    L.check(L.lib.om_set_timing(fz.ctx, 1 if timing else 0), fz.ctx)
    for _ in range(spp // per_call):
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(frame.data_ptr()), None), fz.ctx)
    torch.cuda.synchronize()
    kt = None
    if timing:
        kt = L.om_kernel_times()
        L.check(L.lib.om_get_kernel_times(fz.ctx, C.byref(kt)), fz.ctx)
        L.check(L.lib.om_set_timing(fz.ctx, 0), fz.ctx)
    return frame, kt


def _launches(kt, cls):
    from raytracingoneweekend_amd import _lib as L
    return int(kt.launches[L.KT_CLASSES.index(cls)])


def _windows(W, H, size):
    """Sky (top rows), the sphere field around the big glass sphere (centre), ground (bottom left)."""
    return [(W // 2 - size // 2, 4), (W // 2 - size // 2, H // 2 - size // 2), (W // 8, H - size - 8)]


def _check_windows(oracle, name, frame_u8, W, H, spp, size, march_steps, nan_ok=False, adaptive=False):
    oworld = _scene(oracle, name)
    ocam = oracle.default_camera(W / H)
    p = oracle.params(W, H, spp, seed=SEED, march_steps=march_steps, adaptive=adaptive)
    stats = frame_u8.view(np.uint8).reshape(W * H, 40)
    hit_any = 0
    for (x0, y0) in _windows(W, H, size):
        pix = oracle.window_pixels(W, H, x0, y0, size)
        exp = oracle.render_pixels(oworld, ocam, p, pix, nthreads=0)
        got = stats[pix].copy().view(oracle.PIXEL_STATS_DTYPE).reshape(-1)
        nb, msg = (compare_stats_nan_payload if nan_ok else compare_stats)(got, exp, f"{name} window {x0},{y0}")
        assert nb == 0, msg
        assert (got["n"] <= spp).all() if adaptive else (got["n"] == spp).all()
        hit_any += int((got["bloom"] != 0).sum())
    assert hit_any > 0, "no window saw an object"


def test_c4_shape_4k_32spp_one_call(om, oracle):
    """C4: 3840x2160 S-traced, one 32-spp call = two concurrent 16-spp batches of 133 M paths
    (above 2^25: tail from bounce 24) == 32 one-spp calls (8.3 M-path batches, tail 16) == oracle."""
    W, H, SPP = 3840, 2160, 32
    world = _scene(om, "S-traced")
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    big, kt = _render_calls(om, fz, cam, W, H, SPP, SPP, 1024, timing=True)
    assert _launches(kt, "bounce0") == 2 and _launches(kt, "tail") == 2, "expected two 16-spp batches"
    assert _launches(kt, "bounce") == 2 * 23, "expected the big-batch tail threshold (24)"
    small, kt1 = _render_calls(om, fz, cam, W, H, SPP, 1, 1024, timing=True)
    assert _launches(kt1, "bounce") == SPP * 15, "expected the default tail threshold (16) for 1-spp calls"
    fz.close()
    diff = int((big != small).view(-1, 40).any(1).sum())
    assert diff == 0, f"{diff} pixels differ between the 32-spp call and 32 one-spp calls"
    _check_windows(oracle, "S-traced", big.cpu().numpy(), W, H, SPP, 24, 1024)


def test_max_frame_8k_one_call(om, oracle):
    """The largest frame the bench family reaches, and then some: 7680x4320 (33.2 M pixels, 4x C4),
    one 4-spp call = two concurrent 2-spp batches of 66 M paths (the 2^27-path cap on a batch
    decides the split; above 2^25 paths: tail from bounce 24) == 4 one-spp calls == oracle windows.
    Path slots, pixel indices and queue offsets stay 32-bit clean at this size."""
    W, H, SPP = 7680, 4320, 4
    world = _scene(om, "S-traced")
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    big, kt = _render_calls(om, fz, cam, W, H, SPP, SPP, 1024, timing=True)
    assert _launches(kt, "bounce0") == 2 and _launches(kt, "tail") == 2, "expected two concurrent 2-spp batches"
    assert _launches(kt, "bounce") == 2 * 23, "expected the big-batch tail threshold (24)"
    small, _ = _render_calls(om, fz, cam, W, H, SPP, 1, 1024)
    fz.close()
    diff = int((big != small).view(-1, 40).any(1).sum())
    assert diff == 0, f"{diff} pixels differ between the 4-spp call and 4 one-spp calls"
    _check_windows(oracle, "S-traced", big.cpu().numpy(), W, H, SPP, 16, 1024)


def test_c1_shape_1080p_128spp_shard_call(om, oracle):
    """C1: bench.py's step itself -- om_render_shard of 128 spp over the (N=1) tile shard, eight
    16-spp batches of 33 M paths on two streams, then the RCCL gather -- == 128 one-spp calls
    over the whole frame == oracle windows."""
    import torch
    from raytracingoneweekend_amd import shard
    W, H, SPP = 1920, 1080, 128
    world = _scene(om, "S-traced")
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    comm = shard.Comm(fz.ctx, 1, 0, shard.unique_id())
    sh = torch.zeros(shard.shard_capacity(W, H, 1) * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, SPP, W, H, sample_count=SPP, seed=SEED)
    s = torch.cuda.Stream()
    from raytracingoneweekend_amd import _lib as L
    L.check(L.lib.om_set_timing(fz.ctx, 1), fz.ctx)
    comm.render_shard(cam, p, sh.data_ptr(), s.cuda_stream)
    s.synchronize()
    kt = L.om_kernel_times()
    L.check(L.lib.om_get_kernel_times(fz.ctx, C.byref(kt)), fz.ctx)
    L.check(L.lib.om_set_timing(fz.ctx, 0), fz.ctx)
    assert _launches(kt, "bounce0") == 8 and _launches(kt, "bounce") == 8 * 15, "expected 8 x 16-spp batches, tail 16"
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    comm.gather_frame(sh.data_ptr(), W, H, frame.data_ptr(), s.cuda_stream)
    s.synchronize()
    comm.close()
    small, _ = _render_calls(om, fz, cam, W, H, SPP, 1, 1024)
    fz.close()
    diff = int((frame != small).view(-1, 40).any(1).sum())
    assert diff == 0, f"{diff} pixels differ between the bench's 128-spp shard call and 128 one-spp calls"
    _check_windows(oracle, "S-traced", frame.cpu().numpy(), W, H, SPP, 24, 1024)


def test_c3_shape_1080p_10k_bvh2_l2(om, oracle):
    """C3: 1080p S-10k on the auto kernel (BVH2 read through L2 past its LDS top, tail 10, 8192
    lanes per CU), one 16-spp call (two 8-spp batches) == 16 one-spp calls == oracle windows."""
    W, H, SPP = 1920, 1080, 16
    world = _scene(om, "S-10k")
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    big, kt = _render_calls(om, fz, cam, W, H, SPP, SPP, 1024, timing=True)
    assert _launches(kt, "bounce0") == 2 and _launches(kt, "bounce") == 2 * 9, "expected 2 batches, tail 10"
    small, _ = _render_calls(om, fz, cam, W, H, SPP, 1, 1024)
    fz.close()
    diff = int((big != small).view(-1, 40).any(1).sum())
    assert diff == 0, f"{diff} pixels differ between the 16-spp call and 16 one-spp calls"
    _check_windows(oracle, "S-10k", big.cpu().numpy(), W, H, SPP, 16, 1024)


def test_c2_shape_1080p_marched_split_pipeline(om, oracle):
    """C2: 1080p S-marched (256 march steps) on the split march pipeline: bounce 0 as k_raygen +
    lane-refilling k_march + k_bounce<HIT>, every later segment in the lane-refilling marched tail
    (from bounce 1, om_tuning.h OM_WF_TAIL_MARCHED); one 16-spp call == 16 one-spp calls == oracle
    windows."""
    W, H, SPP, STEPS = 1920, 1080, 16, 256
    world = _scene(om, "S-marched")
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    big, kt = _render_calls(om, fz, cam, W, H, SPP, SPP, STEPS, timing=True)
    assert _launches(kt, "megakernel") == 0 and _launches(kt, "tail") == 2, "expected the wavefront, 2 batches"
    # per batch: k_raygen + k_march + k_bounce<HIT> (bounce 0), no per-bounce launch after it
    assert _launches(kt, "bounce0") == 6 and _launches(kt, "bounce") == 0, "expected the marched tail from bounce 1"
    small, _ = _render_calls(om, fz, cam, W, H, SPP, 1, STEPS)
    fz.close()
    diff = int((big != small).view(-1, 40).any(1).sum())
    assert diff == 0, f"{diff} pixels differ between the 16-spp call and 16 one-spp calls"
    _check_windows(oracle, "S-marched", big.cpu().numpy(), W, H, SPP, 24, STEPS)


def test_c1_adaptive_shape_1080p_512spp(om, oracle):
    """C1_adaptive, the bench's adaptive frame (the reference's default mode, render_thread.rs:31-38,
    68-102, 176-199): 1920x1080 S-traced, 512 spp adaptive in 4 x 128-spp calls on two streams, each
    stream running its live pixels in 3 device-planned batches per call from the live lists its
    accumulates compact == the same frame in 16-spp calls on one stream (a different deal and other
    batch sizes) == the sequential oracle on three 16x16 windows."""
    import torch
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 1920, 1080, 512
    world = _scene(om, "S-traced")
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    big, kt = _render_calls(om, fz, cam, W, H, SPP, 128, 1024, timing=True, adaptive=True)
    assert _launches(kt, "bounce0") == 4 * 2 * 3, "expected 4 calls x 2 streams x 3 planned batches"
    assert _launches(kt, "accumulate") == 4 * 2 * 3
    L.check(L.lib.om_set_streams(fz.ctx, 1), fz.ctx)
    small, kt1 = _render_calls(om, fz, cam, W, H, SPP, 16, 1024, timing=True, adaptive=True)
    assert _launches(kt1, "bounce0") == 32 * 1 * 3, "expected 32 calls x 1 stream x 3 batches"
    fz.close()
    diff = int((big != small).view(-1, 40).any(1).sum())
    assert diff == 0, f"{diff} pixels differ between 128-spp calls on 2 streams and 16-spp calls on 1"
    n = big.view(-1, 40)[:, 20:24].contiguous().view(-1).view(torch.int32)
    assert int(n.min()) < 16 and 0 < int(n.max()) < SPP, "expected early and late retirements"
    _check_windows(oracle, "S-traced", big.cpu().numpy(), W, H, SPP, 16, 1024, adaptive=True)
