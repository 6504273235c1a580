"""GPU parity on the reference's edge cases that random scenes never reach:

* exact ties — traced.rs:51-53 accepts root == t_max, so in hits.rs:274-285 the LATER object
  of two with the same root wins.  Every HIP traversal re-orders the tests and implements this
  as `t < closest || gi > best` (om_trace.h); here duplicated primitives tie exactly, inside one
  BVH leaf and across leaves, and a triangle and a parallelogram built from the same three
  points tie across the type order;
* the NaN marched normal — marched.rs:25-44's eps = 1e-7 central differences round to zero on
  a face at |x| >= 2 (ulp 2.4e-7), so unit((0,0,0)) is NaN and the path carries NaN into the
  pixel's running sum;
* C0, the reference's CPU case (BASELINE.json configs[0]: 400x225, 64 spp, max_depth 8), whole
  frame, against the oracle.

Bar: every byte of om_pixel_stats equals the oracle's, except the payload (sign and mantissa
bits) of a NaN in `sum`, where only NaN-ness is compared.
"""
import numpy as np
import pytest

from scenes_common import compare_stats, compare_stats_nan_payload, nan_normal_world, tie_scene

pytestmark = pytest.mark.gpu

KERNELS = ["brute", "culled", "bvh", "sbvh", "bvh2", "bvh4"]
PIPELINES = ["megakernel", "wavefront"]
COMBOS = [(k, p) for p in PIPELINES for k in KERNELS]
def _render(om, world, cam, W, H, spp, kernel, pipeline, seed, max_depth=50, lists=None, march_steps=1024):
    from raytracingoneweekend_amd import _lib as L
    fz = world.freeze(cam, kernel=kernel, pipeline=pipeline)
    if lists is not None:
        L.check(L.lib.om_set_primary_lists(fz.ctx, lists), fz.ctx)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, max_depth, 0.001, 100.0, spp, W, H, pix, seed=seed, adaptive=False, march_steps=march_steps)
    fz.close()
    return pix.pixels


@pytest.mark.parametrize("kernel", COMBOS)
def test_exact_ties_bit_exact(om, oracle, kernel):
    W, H, SPP = 64, 40, 4
    w, ow = tie_scene(om, oracle)
    cam, ocam = om.default_camera(W / H), oracle.default_camera(W / H)
    exp, _ = oracle.render(ow, ocam, oracle.params(W, H, SPP, seed=17))
    got = _render(om, w, cam, W, H, SPP, kernel[0], kernel[1], seed=17)
    nb, msg = compare_stats(got, exp, f"ties/{kernel}")
    assert nb == 0, msg


@pytest.mark.parametrize("lists", [0, 1, 2])
def test_exact_ties_primary_tile_lists(om, oracle, lists):
    """Bounce 0 over per-tile candidate lists (forced off / auto / forced on)
    keeps the later-object rule on the duplicated records."""
    W, H, SPP = 53, 37, 3
    w, ow = tie_scene(om, oracle)
    cam, ocam = om.default_camera(W / H), oracle.default_camera(W / H)
    exp, _ = oracle.render(ow, ocam, oracle.params(W, H, SPP, seed=23))
    got = _render(om, w, cam, W, H, SPP, "bvh2", "wavefront", seed=23, lists=lists)
    nb, msg = compare_stats(got, exp, f"ties/lists{lists}")
    assert nb == 0, msg


def test_ties_are_exercised(om, oracle):
    """The duplicates decide real pixels: the GPU frame's winning ids (bloom) differ from the
    frame where the first copy wins (the scene without the later copies) on many pixels, and
    the first-copy frame is itself the oracle's."""
    W, H, SPP = 64, 40, 2
    cam, ocam = om.default_camera(W / H), oracle.default_camera(W / H)
    w, _ = tie_scene(om, oracle)
    w1, ow1 = tie_scene(om, oracle, duplicates=False)
    got = _render(om, w, cam, W, H, SPP, "auto", "wavefront", seed=29)
    first = _render(om, w1, cam, W, H, SPP, "auto", "wavefront", seed=29)
    exp1, _ = oracle.render(ow1, ocam, oracle.params(W, H, SPP, seed=29))
    nb, msg = compare_stats(first, exp1, "ties/first-copy scene")
    assert nb == 0, msg
    differ = int((got["bloom"] != first["bloom"]).sum())
    assert differ > W * H // 20, f"only {differ} pixels see a duplicate"


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_nan_marched_normal(om, oracle, pipeline):
    W, H, SPP = 64, 40, 4
    w, ow = nan_normal_world(om, oracle)
    cam, ocam = om.default_camera(W / H), oracle.default_camera(W / H)
    exp, _ = oracle.render(ow, ocam, oracle.params(W, H, SPP, seed=31, march_steps=256))
    n_nan = int(np.isnan(exp["sum"]).any(axis=1).sum())
    assert n_nan > 0, "the scene must reach the NaN normal of marched.rs:25-44"
    got = _render(om, w, cam, W, H, SPP, "auto", pipeline, seed=31, march_steps=256)
    nb, msg = compare_stats_nan_payload(got, exp, f"nan-normal/{pipeline}")
    assert nb == 0, msg
    assert int(np.isnan(got["sum"]).any(axis=1).sum()) == n_nan


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_c0_frame_bit_exact(om, oracle, pipeline):
    """BASELINE.json configs[0] (the reference's CPU case), the whole 400x225x64 frame at
    max_depth 8, render seed 1 as in bench.py."""
    W, H, SPP = 400, 225, 64
    cam, ocam = om.default_camera(W / H), oracle.default_camera(W / H)
    exp, _ = oracle.render(oracle.random_scene(0x5EED), ocam, oracle.params(W, H, SPP, max_depth=8, seed=1))
    got = _render(om, om.random_scene(0x5EED), cam, W, H, SPP, "auto", pipeline, seed=1, max_depth=8)
    nb, msg = compare_stats(got, exp, f"C0/{pipeline}")
    assert nb == 0, msg
    assert (got["n"] == SPP).all()

