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


def _full_frame(om, world, cam, W, H, spp, calls, seed):
    """Single-device reference: one ctx, om_render_device over the whole frame."""
    import torch
    from raytracingoneweekend_amd import _lib as L
    fz = world.freeze(cam)
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, spp, W, H, sample_count=spp // calls, seed=seed)
    for _ in range(calls):
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(frame.data_ptr()), None), fz.ctx)
    torch.cuda.synchronize()
    fz.close()
    return frame


def _window_vs_oracle(oracle, frame_u8, W, H, spp, seed, x0, y0, size=24):
    pix = np.array([(y0 + j) * W + x0 + i for j in range(size) for i in range(size)], dtype=np.uint32)
    exp = oracle.render_pixels(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                               oracle.params(W, H, spp, seed=seed), pix)
    got = frame_u8.view(np.uint8).reshape(W * H, 40)[pix].copy().view(oracle.PIXEL_STATS_DTYPE).reshape(-1)
    return compare_stats(got, exp, f"window {x0},{y0}")


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_multi_local_ranks_4k_frame_bit_identical(om, oracle, nranks):
    """om_multi over `nranks` logical ranks on device 0 (OM_TRANSPORT_LOCAL): two progressive
    calls of C4's 4K frame (the second one deals a partly rendered frame back out) == one ctx."""
    import torch
    from raytracingoneweekend_amd import shard
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W4K / H4K)
    spp, seed = 2, 41
    ref = _full_frame(om, world, cam, W4K, H4K, spp, 2, seed)
    mf = shard.MultiFrame([0] * nranks, world)
    assert mf.transport == "local"
    frame = torch.zeros(W4K * H4K * 40, dtype=torch.uint8, device="cuda")
    p = om.make_params(50, 0.001, 100.0, spp, W4K, H4K, sample_count=1, seed=seed)
    for _ in range(2):
        mf.render(cam, p, frame.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(frame, ref), f"{int((frame != ref).view(-1, 40).any(1).sum())} pixels differ"
    host = frame.cpu().numpy()
    assert int(host.view(om.PIXEL_STATS_DTYPE)["n"].min()) == spp
    nb, msg = _window_vs_oracle(oracle, host, W4K, H4K, spp, seed, 1800, 1000)
    assert nb == 0, msg
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
    torch.cuda.synchronize()
    assert torch.equal(frame, ref)
    mf.close()


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
