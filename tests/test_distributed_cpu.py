"""N>1 path on CPU: world_size-2 gloo ranks shard the frame by 8x8 tiles
(raytracingoneweekend_amd.shard), render their tiles (CPU oracle stands in for the
device here) and gather to rank 0 with one collective; the assembled frame must be
bit-identical to a single-rank render (RNG keyed by pixel and sample, not by rank)."""
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
    pix = shard.tile_pixels(W, H, rank, world_size)
    st = O.render_pixels(O.random_scene(0x5EED), O.default_camera(W / H), O.params(W, H, SPP, seed=9), pix)
    frame = shard.gather_frame(dist, torch.from_numpy(st.view(np.uint8).copy()), W, H, rank, world_size)
    if rank == 0:
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


def test_tiles_partition_the_frame():
    from raytracingoneweekend_amd import shard
    for (w, h) in [(1920, 1080), (37, 21), (8, 8)]:
        for ws in (1, 2, 3, 8):
            parts = [shard.tile_pixels(w, h, r, ws) for r in range(ws)]
            allp = np.concatenate(parts)
            assert allp.size == w * h and np.unique(allp).size == w * h
            assert max(p.size for p in parts) <= shard.shard_capacity(w, h, ws)
