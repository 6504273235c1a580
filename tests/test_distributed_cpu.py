"""N>1 path on CPU: world_size-2/3 gloo ranks take their 8x8-tile shards from the product's
deal (om_shard_pixels), render them, send them to rank 0, and rank 0 assembles the frame with
the product's om_shard_assemble_host; the frame must be bit-identical to a single-rank render
(om-rng is keyed by pixel and sample, not by rank).  There is no GPU here, so the per-rank
render is the CPU oracle's render_pixels and gloo carries the bytes RCCL carries on the GPU
(om_gather_frame, tested on the GPU in test_multi_gpu.py)."""
import os
import socket

import numpy as np
import pytest

W, H, SPP = 40, 24, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world_size, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    from raytracingoneweekend_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    pix = shard.tile_pixels(W, H, rank, world_size)                       # the product's tile deal
    st = O.render_pixels(O.random_scene(0x5EED), O.default_camera(W / H), O.params(W, H, SPP, seed=9), pix)
    cap = shard.shard_capacity(W, H, world_size) * 40
    send = torch.zeros(cap, dtype=torch.uint8)
    send[: pix.size * 40] = torch.from_numpy(st.view(np.uint8).copy())
    bufs = [torch.empty_like(send) for _ in range(world_size)] if rank == 0 else None
    dist.gather(send, bufs, dst=0)
    if rank == 0:                                                          # the product's assembly
        sizes = [shard.tile_pixels(W, H, r, world_size).size for r in range(world_size)]
        frame = shard.assemble(W, H, [b.numpy()[: n * 40] for b, n in zip(bufs, sizes)])
        np.save(out_path, frame.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world_size", [2, 3])
def test_tile_sharded_gather_is_bit_identical(oracle, tmp_path, world_size):
    import torch.multiprocessing as mp
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world_size, _free_port(), out), nprocs=world_size, join=True)
    got = np.load(out)
    ref, _ = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H), oracle.params(W, H, SPP, seed=9),
                           nthreads=2)
    assert np.array_equal(got, ref.view(np.uint8))


def _deal_restated(w, h, rank, ws):
    """Independent restatement of the deal: tiles t % ws == rank, row-major, lanes row-major."""
    tx, ty = (w + 7) // 8, (h + 7) // 8
    out = []
    for t in range(rank, tx * ty, ws):
        for lane in range(64):
            px, py = (t % tx) * 8 + lane % 8, (t // tx) * 8 + lane // 8
            if px < w and py < h:
                out.append(py * w + px)
    return np.array(out, dtype=np.uint32)


def test_native_deal_matches_restatement():
    from raytracingoneweekend_amd import shard
    for (w, h) in [(37, 21), (8, 8), (1, 1), (3, 50), (64, 9)]:
        for ws in (1, 2, 3, 8, 20):
            for r in range(ws):
                assert np.array_equal(shard.tile_pixels(w, h, r, ws), _deal_restated(w, h, r, ws)), (w, h, ws, r)


def test_shard_argument_errors(om):
    from raytracingoneweekend_amd import _lib as L
    import ctypes as C
    n = C.c_uint32()
    assert L.lib.om_shard_pixels(16, 16, 2, 2, None, 0, C.byref(n)) == L.OM_ERR_INVALID      # rank >= nranks
    assert L.lib.om_shard_pixels(16, 16, 0, 2, None, 0, C.byref(n)) == L.OM_ERR_INVALID      # no room
    assert n.value == 128
    assert L.lib.om_shard_capacity(16, 16, 0) == 0
    assert L.lib.om_comm_init_rank(None, 2, 0, None, None) == L.OM_ERR_INVALID
    assert L.lib.om_multi_create(None, 0, None) == L.OM_ERR_INVALID
    assert L.lib.om_multi_transport(None) == -1


def test_assemble_round_trip():
    from raytracingoneweekend_amd import _lib as L
    from raytracingoneweekend_amd import shard
    w, h, ws = 45, 19, 3
    rng = np.random.default_rng(1)
    frame = rng.integers(0, 256, size=w * h * 40, dtype=np.uint8).view(L.PIXEL_STATS_DTYPE)
    shards = [frame[shard.tile_pixels(w, h, r, ws)] for r in range(ws)]
    assert np.array_equal(shard.assemble(w, h, shards).view(np.uint8), frame.view(np.uint8))


def test_tiles_partition_the_frame():
    from raytracingoneweekend_amd import shard
    for (w, h) in [(1920, 1080), (37, 21), (8, 8)]:
        for ws in (1, 2, 3, 8):
            parts = [shard.tile_pixels(w, h, r, ws) for r in range(ws)]
            allp = np.concatenate(parts)
            assert allp.size == w * h and np.unique(allp).size == w * h
            assert max(p.size for p in parts) <= shard.shard_capacity(w, h, ws)


@pytest.mark.parametrize("W,H", [(1, 1), (7, 5), (13, 9), (53, 37), (641, 359), (3840, 2160)])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 7, 8])
def test_tile_deal_partitions_the_frame(om, W, H, n):
    """the product's deal (om_shard_pixels) over all ranks covers every pixel exactly
    once, for odd frame sizes and rank counts; every shard fits om_shard_capacity, so the gather's
    staging offsets q * capacity (om_gather_frame, om_multi_gather) never overlap; each rank's
    pixels come in its tile order (t % n == rank, row-major tiles, lane order 8*y + x inside)."""
    from raytracingoneweekend_amd import shard
    cap = shard.shard_capacity(W, H, n)
    seen = np.zeros(W * H, dtype=np.int32)
    counts = []
    for r in range(n):
        pix = shard.tile_pixels(W, H, r, n)
        counts.append(pix.size)
        assert pix.size <= cap
        np.add.at(seen, pix.astype(np.int64), 1)
        x, y = pix % W, pix // W
        tiles_x = (W + 7) // 8
        t = (y // 8) * tiles_x + x // 8
        assert np.all(t % n == r)
        key = t.astype(np.int64) * 64 + (y % 8) * 8 + (x % 8)
        assert np.all(np.diff(key) > 0)                                 # tile order, lane order inside
    assert np.all(seen == 1)
    assert sum(counts) == W * H and max(counts) <= cap
    # the gather's staging layout: rank q's shard at q * cap, no overlap, all within n * cap
    ends = [q * cap + counts[q] for q in range(n)]
    assert all(ends[q] <= (q + 1) * cap for q in range(n))
