"""Multi-GPU frames through the native path (om_multi_*, om_comm_*), on the
one GPU of the test box: C4's 3840x2160 frame rendered as N logical ranks (device copies:
RCCL refuses two ranks on one GPU) and through RCCL itself (one rank, whose shard still
travels through an RCCL send/recv), each bit-identical to the single-device render of the
same frame, and a window of it bit-identical to the CPU oracle."""
import ctypes as C

import numpy as np
import pytest

from scenes_common import compare_stats

pytestmark = pytest.mark.gpu

W4K, H4K = 3840, 2160          # BASELINE.json configs[4] (C4)


def _full_frame(om, world, cam, W, H, spp, calls, seed, spp_total=None):
    """Single-device reference: one ctx, `calls` om_render_device calls of spp // calls samples
    (of spp_total, default spp: the jitter table's size) over the whole frame."""
    import torch
    from raytracingoneweekend_amd import _lib as L
    fz = world.freeze(cam)
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, spp_total or spp, W, H, sample_count=spp // calls, seed=seed)
    for _ in range(calls):
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(frame.data_ptr()), None), fz.ctx)
    torch.cuda.synchronize()
    fz.close()
    return frame


def _window_vs_oracle(oracle, frame_u8, W, H, spp, seed, x0, y0, size=24, sample_count=None):
    pix = np.array([(y0 + j) * W + x0 + i for j in range(size) for i in range(size)], dtype=np.uint32)
    exp = oracle.render_pixels(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                               oracle.params(W, H, spp, sample_count=sample_count, seed=seed), pix)
    got = frame_u8.view(np.uint8).reshape(W * H, 40)[pix].copy().view(oracle.PIXEL_STATS_DTYPE).reshape(-1)
    return compare_stats(got, exp, f"window {x0},{y0}")


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_multi_local_ranks_4k_frame_bit_identical(om, oracle, nranks):
    """om_multi over `nranks` logical ranks on device 0 (OM_TRANSPORT_LOCAL): C4's 4K frame dealt
    out once, three progressive calls into the ranks' resident shards, ONE gather == one ctx.
    Then a second frame buffer already holding those samples is dealt out (a frame rendered
    elsewhere), one more call and gather == one ctx at the higher sample count."""
    import torch
    from raytracingoneweekend_amd import shard
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W4K / H4K)
    spp, seed = 3, 41
    ref = _full_frame(om, world, cam, W4K, H4K, spp, 3, seed, spp_total=spp + 1)
    mf = shard.MultiFrame([0] * nranks, world)
    assert mf.transport == "local"
    s = torch.cuda.Stream()
    frame = torch.zeros(W4K * H4K * 40, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    p = om.make_params(50, 0.001, 100.0, spp + 1, W4K, H4K, sample_count=1, seed=seed)
    for _ in range(spp):
        mf.render(cam, p, frame.data_ptr(), s.cuda_stream)
    mf.gather(frame.data_ptr(), W4K, H4K, s.cuda_stream)
    s.synchronize()
    assert torch.equal(frame, ref), f"{int((frame != ref).view(-1, 40).any(1).sum())} pixels differ"
    host = frame.cpu().numpy()
    assert int(host.view(om.PIXEL_STATS_DTYPE)["n"].min()) == spp
    nb, msg = _window_vs_oracle(oracle, host, W4K, H4K, spp + 1, seed, 1800, 1000, sample_count=spp)
    assert nb == 0, msg
    # a second buffer (a frame rendered elsewhere): dealt out on first sight
    ref4 = _full_frame(om, world, cam, W4K, H4K, spp + 1, spp + 1, seed)
    frame2 = frame.clone()
    torch.cuda.synchronize()
    mf.render(cam, p, frame2.data_ptr(), s.cuda_stream)
    mf.gather(frame2.data_ptr(), W4K, H4K, s.cuda_stream)
    s.synchronize()
    assert torch.equal(frame2, ref4)
    mf.close()


def test_multi_gather_stale_frame_and_reset(om):
    """The frame only changes on gather; om_multi_reset re-deals a frame the caller rewrote."""
    import torch
    from raytracingoneweekend_amd import shard
    W, H, seed = 200, 120, 44
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    mf = shard.MultiFrame([0, 0, 0], world)
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, 4, W, H, sample_count=2, seed=seed)
    mf.render(cam, p, frame.data_ptr())
    torch.cuda.synchronize()
    assert not frame.any(), "om_multi_render must not write the frame"
    mf.gather(frame.data_ptr(), W, H)
    torch.cuda.synchronize()
    first = frame.clone()
    frame.zero_()                                   # the caller restarts the frame ...
    mf.reset()                                      # ... and says so
    mf.render(cam, p, frame.data_ptr())
    mf.gather(frame.data_ptr(), W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, first)
    with pytest.raises(Exception, match="no resident frame"):
        mf.gather(frame.data_ptr(), W + 8, H)
    mf.close()


def test_multi_failed_allocation_then_retry(om, monkeypatch):
    """a shard allocation that fails part-way through the deal's bookkeeping returns
    an error and leaves no half-built deal behind; the retried call rebuilds it and renders the
    same frame as one ctx (OM_DEBUG_FAIL_ALLOC: every shard-buffer allocation of >= N bytes
    fails, om_multi.hip)."""
    import torch
    from raytracingoneweekend_amd import _lib as L
    from raytracingoneweekend_amd import shard
    W, H, spp, seed = W4K, H4K, 1, 45
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    ref = _full_frame(om, world, cam, W, H, spp, 1, seed)
    mf = shard.MultiFrame([0, 0, 0], world)
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    p = om.make_params(50, 0.001, 100.0, spp, W, H, seed=seed)
    # the rank-major list table (33 MB) fits, every shard (110 MB) fails
    monkeypatch.setenv("OM_DEBUG_FAIL_ALLOC", str(64 << 20))
    for _ in range(2):
        with pytest.raises(L.OmError, match="out of memory|ensure"):
            mf.render(cam, p, frame.data_ptr())
    monkeypatch.delenv("OM_DEBUG_FAIL_ALLOC")
    mf.render(cam, p, frame.data_ptr())
    mf.gather(frame.data_ptr(), W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, ref)
    mf.close()


def test_multi_rccl_transport_one_device(om):
    """om_multi on distinct devices uses RCCL (ncclCommInitAll); with one GPU that is one rank."""
    import torch
    from raytracingoneweekend_amd import shard
    W, H, spp, seed = 480, 270, 3, 42
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    ref = _full_frame(om, world, cam, W, H, spp, 1, seed)
    mf = shard.MultiFrame([0], world)
    assert mf.transport == "rccl"
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    mf.render(cam, om.make_params(50, 0.001, 100.0, spp, W, H, seed=seed), frame.data_ptr())
    mf.gather(frame.data_ptr(), W, H)
    torch.cuda.synchronize()
    assert torch.equal(frame, ref)
    mf.close()


def test_rccl_library_is_reported(om):
    """om_rccl_library names the RCCL the comm paths run on (bench.py records it in the line)."""
    from raytracingoneweekend_amd import shard
    path, version = shard.rccl_library()
    assert "rccl" in path and version >= 20000


def test_comm_rank_render_gather_scatter_through_rccl(om, oracle):
    """The per-process API bench.py drives on every GPU: om_comm_init_rank (RCCL), progressive
    om_render_shard calls into an HBM-resident shard, om_gather_frame (rank 0's shard goes
    through an RCCL send/recv to itself) == the single-device frame; om_scatter_frame cuts it
    back into the same shard."""
    import torch
    from raytracingoneweekend_amd import shard
    W, H, spp, seed = W4K, H4K, 2, 43
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    ref = _full_frame(om, world, cam, W, H, spp, 2, seed)
    fz = world.freeze(cam)
    comm = shard.Comm(fz.ctx, 1, 0, shard.unique_id())
    cap = shard.shard_capacity(W, H, 1)
    sh = torch.zeros(cap * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=1, seed=seed)
    s = torch.cuda.Stream()
    for _ in range(2):
        comm.render_shard(cam, p, sh.data_ptr(), s.cuda_stream)
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    comm.gather_frame(sh.data_ptr(), W, H, frame.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert torch.equal(frame, ref)
    back = torch.zeros_like(sh)
    comm.scatter_frame(frame.data_ptr(), W, H, back.data_ptr(), s.cuda_stream)
    s.synchronize()
    assert torch.equal(back, sh)
    nb, msg = _window_vs_oracle(oracle, frame.cpu().numpy(), W, H, spp, seed, 0, 2136)
    assert nb == 0, msg
    comm.close()
    fz.close()


def test_multi_redeal_without_gather(om):
    """render(A) then render(B) with no gather between -- B's deal overwrites the
    shards A's renders may still be writing, on another stream -- then gather(B) == one ctx."""
    import torch
    from raytracingoneweekend_amd import shard
    W, H, spp, seed = W4K, H4K, 4, 46
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    ref = _full_frame(om, world, cam, W, H, 2, 1, seed, spp_total=spp)
    mf = shard.MultiFrame([0, 0, 0], world)
    a = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    b = torch.zeros_like(a)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    mf.render(cam, om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=spp, seed=seed), a.data_ptr(), s1.cuda_stream)
    mf.render(cam, om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=2, seed=seed), b.data_ptr(), s2.cuda_stream)
    mf.gather(b.data_ptr(), W, H, s2.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(b, ref), f"{int((b != ref).view(-1, 40).any(1).sum())} pixels differ"
    mf.close()


def test_multi_render_host_sees_a_rewritten_buffer(om, oracle):
    """the host form copies the caller's buffer on every call, so zeroing it restarts
    the frame (no om_multi_reset needed) -- the same two calls give the same frame twice."""
    import ctypes as C
    from raytracingoneweekend_amd import _lib as L
    from raytracingoneweekend_amd import shard
    W, H, spp, seed = 160, 96, 3, 47
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    mf = shard.MultiFrame([0, 0], world)
    buf = np.zeros(W * H, dtype=om.PIXEL_STATS_DTYPE)
    p = om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=spp, seed=seed)
    mf._check(L.lib.om_multi_render_host(mf._m, C.byref(cam.raw), C.byref(p), buf.ctypes.data_as(C.c_void_p), None))
    first = buf.copy()
    assert (first["n"] == spp).all()
    buf[:] = np.zeros(1, dtype=om.PIXEL_STATS_DTYPE)           # the caller restarts the frame in place
    mf._check(L.lib.om_multi_render_host(mf._m, C.byref(cam.raw), C.byref(p), buf.ctypes.data_as(C.c_void_p), None))
    assert np.array_equal(buf.view(np.uint8), first.view(np.uint8))
    exp, _ = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H), oracle.params(W, H, spp, seed=seed))
    nb, msg = compare_stats(buf, exp, "render_host")
    assert nb == 0, msg
    mf.close()


@pytest.mark.parametrize("sched", [(0, 0), (5, 8)])
def test_multi_adaptive_shards_bit_identical(om, oracle, sched):
    """Adaptive calls on shards: each logical rank renders its listed pixels
    with the live-list schedule over ITS shard (its streams' chunks of the shard's list, the
    batches planned from the live counts; `sched` = om_set_adaptive_batches on every rank, (5, 8):
    several batches per stream); the gathered frame == one ctx rendering the whole frame
    adaptively, and a window of it == the sequential oracle."""
    import torch
    from raytracingoneweekend_amd import _lib as L
    from raytracingoneweekend_amd import shard
    W, H, SPP, seed = 160, 96, 40, 17
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    p = om.make_params(50, 0.001, 100.0, SPP, W, H, sample_count=SPP, seed=seed, adaptive=True)
    fz = world.freeze(cam)
    ref = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(ref.data_ptr()), None), fz.ctx)
    torch.cuda.synchronize()
    fz.close()
    mf = shard.MultiFrame([0, 0, 0], world)
    for r in range(3):
        L.check(L.lib.om_set_adaptive_batches(mf.ctx(r), *sched), mf.ctx(r))
    s = torch.cuda.Stream()
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    mf.render(cam, p, frame.data_ptr(), s.cuda_stream)
    mf.gather(frame.data_ptr(), W, H, s.cuda_stream)
    s.synchronize()
    mf.close()
    assert torch.equal(frame, ref), f"{int((frame != ref).view(-1, 40).any(1).sum())} pixels differ"
    host = frame.cpu().numpy()
    assert int(host.view(om.PIXEL_STATS_DTYPE)["n"].min()) < SPP          # pixels retired early
    pix = np.array([(40 + j) * W + 60 + i for j in range(16) for i in range(16)], dtype=np.uint32)
    exp = oracle.render_pixels(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                               oracle.params(W, H, SPP, seed=seed, adaptive=True), pix)
    got = host.reshape(W * H, 40)[pix].copy().view(oracle.PIXEL_STATS_DTYPE).reshape(-1)
    nb, msg = compare_stats(got, exp, "adaptive shards window")
    assert nb == 0, msg
