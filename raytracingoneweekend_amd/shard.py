"""Pixel-tile sharding of a frame across ranks (one process per GPU) and the
framebuffer gather.

Reference analogue: main.rs:172-189 deals 2730-pixel chunks round-robin to CPU
threads.  Here 8x8 tiles (one wavefront each) are dealt round-robin to ranks, so
every rank gets a spatially interleaved, cost-balanced share.  Pixels are
independent and om-rng is keyed by (pixel, sample), so a sharded render is
bit-identical to a single-device render.
"""
import numpy as np

from ._lib import PIXEL_STATS_DTYPE

TILE = 8


def tile_pixels(width, height, rank, world_size):
    """Row-major pixel indices of the tiles t with t % world_size == rank, tile-major,
    each tile in lane order (lane = 8*y + x).  Out-of-frame lanes of edge tiles are dropped."""
    tx, ty = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    lane = np.arange(TILE * TILE)
    lx, ly = lane % TILE, lane // TILE
    tiles = np.arange(rank, tx * ty, world_size)
    px = (tiles[:, None] % tx) * TILE + lx[None, :]
    py = (tiles[:, None] // tx) * TILE + ly[None, :]
    ok = (px < width) & (py < height)
    return (py * width + px)[ok].astype(np.uint32)


def shard_capacity(width, height, world_size):
    """Upper bound of any rank's pixel count (equal-size buffers for the collective)."""
    tx, ty = (width + TILE - 1) // TILE, (height + TILE - 1) // TILE
    return ((tx * ty + world_size - 1) // world_size) * TILE * TILE


def assemble(width, height, shards):
    """Scatter per-rank compact om_pixel_stats shards (rank order) back into a W*H frame."""
    frame = np.zeros(width * height, dtype=PIXEL_STATS_DTYPE)
    ws = len(shards)
    for r, sh in enumerate(shards):
        idx = tile_pixels(width, height, r, ws)
        frame[idx] = np.asarray(sh).view(PIXEL_STATS_DTYPE)[: idx.size]
    return frame


def gather_frame(dist, stats_u8, width, height, rank, world_size, device=None):
    """Gather every rank's compact uint8 stats tensor (torch) to rank 0 and assemble the
    frame there (numpy om_pixel_stats[W*H]); other ranks return None.  One collective."""
    import torch
    cap = shard_capacity(width, height, world_size) * PIXEL_STATS_DTYPE.itemsize
    send = torch.zeros(cap, dtype=torch.uint8, device=stats_u8.device if device is None else device)
    send[: stats_u8.numel()] = stats_u8
    bufs = [torch.empty_like(send) for _ in range(world_size)] if rank == 0 else None
    dist.gather(send, bufs, dst=0)
    if rank != 0:
        return None
    return assemble(width, height, [b.cpu().numpy() for b in bufs])
