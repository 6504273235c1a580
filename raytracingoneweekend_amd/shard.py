"""Multi-GPU frames: pixel-tile shards and the RCCL gather, over the C-ABI.

Reference analogue: main.rs:170-214 deals 2730-pixel chunks round-robin to num_cpus-1 render
threads sharing one framebuffer.  Here 8x8 tiles (one wavefront each) are dealt round-robin to
ranks (om_shard_pixels), every rank renders its tiles into a compact shard, and the shards are
gathered to rank 0 with one RCCL group of send/recv (om_gather_frame) or, for one process
driving several GPUs, inside om_multi_render.  Pixels are independent and om-rng is keyed by
(pixel, sample), so a sharded frame is bit-identical to a single-device render.

Everything here marshals arguments to libottomarcher.so; nothing is computed in Python.
"""
import contextlib
import ctypes as C
import os
import sys

import numpy as np

from . import _lib as L
from ._lib import PIXEL_STATS_DTYPE, check, lib

TILE = 8


def shard_capacity(width, height, world_size):
    """Pixels of the largest rank's shard (om_shard_capacity): every shard buffer's size."""
    return int(lib.om_shard_capacity(int(width), int(height), int(world_size)))


def tile_pixels(width, height, rank, world_size):
    """Row-major pixel indices of rank's tiles (om_shard_pixels): tiles t with
    t % world_size == rank in row-major tile order, each tile's in-frame pixels in lane order."""
    cap = shard_capacity(width, height, world_size)
    out = np.empty(max(cap, 1), dtype=np.uint32)
    n = C.c_uint32()
    check(lib.om_shard_pixels(int(width), int(height), int(rank), int(world_size), out.ctypes.data, cap, C.byref(n)))
    return out[: n.value].copy()


def assemble(width, height, shards):
    """Frame (om_pixel_stats[W*H]) from every rank's host shard in rank order (om_shard_assemble_host)."""
    ws = len(shards)
    arrs = [np.ascontiguousarray(np.asarray(s).view(np.uint8)).view(PIXEL_STATS_DTYPE) for s in shards]
    ptrs = (C.c_void_p * ws)(*[a.ctypes.data for a in arrs])
    frame = np.zeros(int(width) * int(height), dtype=PIXEL_STATS_DTYPE)
    check(lib.om_shard_assemble_host(int(width), int(height), ws, ptrs, frame.ctypes.data))
    return frame


@contextlib.contextmanager
def _stdout_to_stderr():
    """RCCL prints a version banner on stdout when a communicator is created; a front-end whose
    stdout is data (bench.py's one JSON line) keeps it on stderr."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def rccl_library():
    """(path, version) of the RCCL library serving om_comm_* / om_multi_* in this process."""
    buf = C.create_string_buffer(4096)
    v = C.c_int32()
    check(lib.om_rccl_library(buf, len(buf), C.byref(v)))
    return buf.value.decode(), v.value


def unique_id():
    """om_comm_unique_id: the 128 bytes rank 0 hands to every rank before Comm()."""
    buf = (C.c_uint8 * L.OM_COMM_ID_BYTES)()
    check(lib.om_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """One rank of a frame shard communicator (om_comm: RCCL over xGMI), bound to `ctx`'s device.
    Every rank must construct it (it blocks until all ranks joined)."""

    def __init__(self, ctx, world_size, rank, uid):
        if len(uid) != L.OM_COMM_ID_BYTES:
            raise ValueError("unique id must be OM_COMM_ID_BYTES long")
        self.ctx, self.world_size, self.rank = ctx, int(world_size), int(rank)
        self._c = C.c_void_p()
        idbuf = (C.c_uint8 * L.OM_COMM_ID_BYTES).from_buffer_copy(uid)
        with _stdout_to_stderr():
            check(lib.om_comm_init_rank(ctx, self.world_size, self.rank, idbuf, C.byref(self._c)), ctx)

    def info(self):
        """(nranks, rank) as RCCL reports them for this communicator (om_comm_info)."""
        n, r = C.c_int32(), C.c_int32()
        check(lib.om_comm_info(self._c, C.byref(n), C.byref(r)), self.ctx)
        return n.value, r.value

    def render_shard(self, cam, params, dev_shard_ptr, stream=None):
        check(lib.om_render_shard(self._c, C.byref(cam.raw if hasattr(cam, "raw") else cam), C.byref(params),
                                  C.c_void_p(dev_shard_ptr), C.c_void_p(stream)), self.ctx)

    def gather_frame(self, dev_shard_ptr, width, height, dev_frame_ptr, stream=None):
        check(lib.om_gather_frame(self._c, C.c_void_p(dev_shard_ptr), int(width), int(height),
                                  C.c_void_p(dev_frame_ptr), C.c_void_p(stream)), self.ctx)

    def scatter_frame(self, dev_frame_ptr, width, height, dev_shard_ptr, stream=None):
        check(lib.om_scatter_frame(self._c, C.c_void_p(dev_frame_ptr), int(width), int(height),
                                   C.c_void_p(dev_shard_ptr), C.c_void_p(stream)), self.ctx)

    def close(self):
        if getattr(self, "_c", None) and self._c.value:
            lib.om_comm_destroy(self._c)
            self._c = C.c_void_p()

    def __del__(self):
        self.close()


class MultiFrame:
    """One process driving several GPUs (om_multi): a ctx per device, tile shards, and the
    gather (RCCL for distinct devices; device copies when a device repeats)."""

    def __init__(self, devices, world, kernel="auto", pipeline="auto"):
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        self._m = C.c_void_p()
        with _stdout_to_stderr():
            st = lib.om_multi_create(devs, len(devices), C.byref(self._m))
        if st != L.OM_OK:
            raise L.OmError(f"om_multi_create failed ({st}): {lib.om_multi_last_error(None).decode()}")
        self.n = len(devices)
        self._check(lib.om_multi_upload_world(self._m, world.handle))
        for r in range(self.n):
            ctx = self.ctx(r)
            check(lib.om_set_kernel(ctx, L.KERNELS[kernel]), ctx)
            check(lib.om_set_pipeline(ctx, L.PIPELINES[pipeline]), ctx)

    def _check(self, st):
        if st != L.OM_OK:
            raise L.OmError(f"ottomarcher multi error {st}: {lib.om_multi_last_error(self._m).decode()}")

    @property
    def transport(self):
        return {L.OM_TRANSPORT_RCCL: "rccl", L.OM_TRANSPORT_LOCAL: "local"}[lib.om_multi_transport(self._m)]

    def ctx(self, rank):
        return C.c_void_p(lib.om_multi_ctx(self._m, rank))

    @staticmethod
    def _stream(stream):
        """The caller's stream; by default torch's current one, so the calls are ordered after the
        work that produced dev_frame.  torch's legacy default stream has the NULL handle, which
        the C-ABI reads as "the ctx's own stream" (not ordered with it): synchronise instead."""
        if stream is not None:
            return stream
        import torch
        s = torch.cuda.current_stream().cuda_stream
        if not s:
            torch.cuda.synchronize()
        return s or None

    def render(self, cam, params, dev_frame_ptr, stream=None):
        """One progressive call into the ranks' resident shards (om_multi_render); the first call
        on a frame deals it out.  dev_frame is brought up to date by gather()."""
        self._check(lib.om_multi_render(self._m, C.byref(cam.raw), C.byref(params), C.c_void_p(dev_frame_ptr),
                                        C.c_void_p(self._stream(stream))))

    def gather(self, dev_frame_ptr, width, height, stream=None):
        """The resident shards back into dev_frame (om_multi_gather)."""
        self._check(lib.om_multi_gather(self._m, C.c_void_p(dev_frame_ptr), int(width), int(height),
                                        C.c_void_p(self._stream(stream))))

    def reset(self):
        """Forget the resident frame (after writing dev_frame yourself)."""
        lib.om_multi_reset(self._m)

    def close(self):
        if getattr(self, "_m", None) and self._m.value:
            lib.om_multi_destroy(self._m)
            self._m = C.c_void_p()

    def __del__(self):
        self.close()
