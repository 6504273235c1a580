"""GPU parity: the HIP hot path (through the C-ABI) vs the CPU oracle on the same
scene, camera, params and om-rng seed.  Bar: bit-identical om_pixel_stats
(sum, n, avg_depth, bad_avgs, color, flags, bloom) for every pixel, every kernel."""
import numpy as np
import pytest

from scenes_common import compare_stats, kitchen_sink

pytestmark = pytest.mark.gpu

KERNELS = ["brute", "culled", "bvh", "sbvh", "bvh2", "bvh4"]
PIPELINES = ["megakernel", "wavefront"]
COMBOS = [(k, p) for p in PIPELINES for k in KERNELS]


def _render_both(om, O, world, oworld, cam, ocam, W, H, spp, kernel, seed=3, max_depth=50, adaptive=False,
                 sample_count=None, march_steps=1024, pipeline="wavefront"):
    if isinstance(kernel, tuple):
        kernel, pipeline = kernel
    frozen = world.freeze(cam, kernel=kernel, pipeline=pipeline)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, frozen, max_depth, 0.001, 100.0, spp, W, H, pix, seed=seed, adaptive=adaptive,
              sample_count=sample_count, march_steps=march_steps)
    p = O.params(W, H, spp, sample_count=sample_count, max_depth=max_depth, adaptive=adaptive, seed=seed,
                 march_steps=march_steps)
    exp, _ = O.render(oworld, ocam, p)
    return pix.pixels, exp, frozen


@pytest.mark.parametrize("kernel", COMBOS)
def test_traced_scene_bit_exact(om, oracle, kernel):
    W, H, SPP = 64, 40, 6
    got, exp, _ = _render_both(om, oracle, om.random_scene(0x5EED), oracle.random_scene(0x5EED),
                               om.default_camera(W / H), oracle.default_camera(W / H), W, H, SPP, kernel)
    nb, msg = compare_stats(got, exp, f"S-traced/{kernel}")
    assert nb == 0, msg
    assert (got["n"] == SPP).all()


@pytest.mark.parametrize("kernel", COMBOS)
def test_full_scene_with_torus_bit_exact(om, oracle, kernel):
    W, H, SPP = 40, 28, 3
    got, exp, _ = _render_both(om, oracle, om.random_scene(0x5EED, with_torus=True),
                               oracle.random_scene(0x5EED, with_torus=True),
                               om.default_camera(W / H), oracle.default_camera(W / H), W, H, SPP, kernel)
    nb, msg = compare_stats(got, exp, f"S-full/{kernel}")
    assert nb == 0, msg


@pytest.mark.parametrize("kernel", COMBOS)
def test_kitchen_sink_every_primitive_bit_exact(om, oracle, kernel):
    W, H, SPP = 48, 32, 4
    w, ow, cam, ocam = kitchen_sink(om, oracle)
    got, exp, _ = _render_both(om, oracle, w, ow, cam, ocam, W, H, SPP, kernel, seed=11)
    nb, msg = compare_stats(got, exp, f"kitchen/{kernel}")
    assert nb == 0, msg


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_marched_scene_bit_exact(om, oracle, pipeline):
    W, H, SPP = 32, 20, 2
    got, exp, _ = _render_both(om, oracle, om.marched_scene(), oracle.marched_scene(), om.default_camera(W / H),
                               oracle.default_camera(W / H), W, H, SPP, "auto", march_steps=256, pipeline=pipeline)
    nb, msg = compare_stats(got, exp, "S-marched")
    assert nb == 0, msg


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_marched_scene_many_rays_bit_exact(om, oracle, pipeline):
    """C2's scene on 0.46 M samples: the lazy march steps (a leading marched sphere alone while
    every other object's bound stays above it) decide the same winner and the
    same distance as the full loop of hits.rs:294-332 on every step of every ray."""
    W, H, SPP = 240, 135, 14
    got, exp, _ = _render_both(om, oracle, om.marched_scene(), oracle.marched_scene(), om.default_camera(W / H),
                               oracle.default_camera(W / H), W, H, SPP, "auto", march_steps=256, pipeline=pipeline,
                               seed=21)
    nb, msg = compare_stats(got, exp, f"S-marched large/{pipeline}")
    assert nb == 0, msg


def _marched_zoo(om, O):
    """Marched spheres nested, overlapping and tiny; a box; a NON-uniformly scaled torus (its
    cull factor bk != 1); the camera inside the big sphere's shell region."""
    w, ow = om.HittableList.new(), O.World()
    mats = [(om.Material.new_lambertian((0.6, 0.6, 0.6)), O.material("lambertian", (0.6, 0.6, 0.6))),
            (om.Material.new_metal_fuzz((0.8, 0.7, 0.5), 0.3), O.material("metal", (0.8, 0.7, 0.5), fuzz=0.3)),
            (om.Material.new_dielectric(1.5), O.material("dielectric", ior=1.5))]
    for (c, r, k) in [((0., -100., 0.), 100., 0), ((0., 0.6, 0.), 0.6, 2), ((0., 0.6, 0.), 0.3, 1),
                      ((0.9, 0.3, 0.2), 0.3, 0), ((-0.7, 0.05, 0.6), 0.05, 1), ((0.35, 0.6, 0.), 0.4, 0)]:
        w += om.MarchedSphere(c, r, mats[k][0]); ow.add_marched_sphere(c, r, mats[k][1])
    w += om.MarchedBox((-1.0, 0.4, -0.3), (0.2, 0.4, 0.3), mats[1][0])
    ow.add_marched_box((-1.0, 0.4, -0.3), (0.2, 0.4, 0.3), mats[1][1])
    l2w = om.m4x4("TR", 0.2, 1.5, -0.8) ^ om.m4x4("RX", 0.7) ^ om.m4x4("SC", 1.6, 0.6, 1.1)
    w += om.MarchedTorus.new(l2w, (0.5, 0.12, 0.12), mats[0][0]); ow.add_marched_torus(l2w.to_numpy(), (0.5, 0.12, 0.12), mats[0][1])
    cam = om.Camera.new((2.2, 1.1, 2.6), (0., 0.5, 0.), (0., 1., 0.), 45., 1.6, 0.05, 3.)
    ocam = O.camera((2.2, 1.1, 2.6), (0., 0.5, 0.), (0., 1., 0.), 45., 1.6, 0.05, 3.)
    return w, ow, cam, ocam


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_marched_zoo_bit_exact(om, oracle, pipeline):
    w, ow, cam, ocam = _marched_zoo(om, oracle)
    W, H, SPP = 96, 60, 6
    got, exp, _ = _render_both(om, oracle, w, ow, cam, ocam, W, H, SPP, "auto", march_steps=512, pipeline=pipeline,
                               seed=5)
    nb, msg = compare_stats(got, exp, f"marched zoo/{pipeline}")
    assert nb == 0, msg


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_adaptive_retirement_bit_exact(om, oracle, pipeline):
    W, H, SPP = 32, 24, 24
    got, exp, _ = _render_both(om, oracle, om.random_scene(0x5EED), oracle.random_scene(0x5EED),
                               om.default_camera(W / H), oracle.default_camera(W / H), W, H, SPP, "auto",
                               adaptive=True, pipeline=pipeline)
    nb, msg = compare_stats(got, exp, "adaptive")
    assert nb == 0, msg
    assert got["n"].min() < SPP  # some pixels (sky) retired early, like the reference


@pytest.mark.parametrize("sample_count", [1, 5, 24])
def test_adaptive_speculative_batches_bit_exact(om, oracle, sample_count):
    """Wavefront adaptive calls render several samples per live pixel per batch and drop those
    past a pixel's retirement: progressive calls of 1 / 5 / 24 samples ==
    the sequential oracle, on a frame bigger than one workgroup's segment."""
    W, H, SPP = 72, 40, 24
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, pipeline="wavefront")
    pix = om.PixelsBox.new(W * H)
    for _ in range((SPP + sample_count - 1) // sample_count):
        om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=13, adaptive=True, sample_count=sample_count)
    exp, _ = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                           oracle.params(W, H, SPP, seed=13, adaptive=True))
    nb, msg = compare_stats(pix.pixels, exp, f"adaptive/{sample_count}")
    assert nb == 0, msg
    assert pix.pixels["n"].min() < SPP


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_progressive_calls_equal_single_call(om, pipeline):
    W, H = 40, 24
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, pipeline=pipeline)
    a = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, 8, W, H, a, seed=5, adaptive=False)
    b = om.PixelsBox.new(W * H)
    for _ in range(4):
        om.render(cam, fz, 50, 0.001, 100.0, 8, W, H, b, seed=5, sample_count=2, adaptive=False)
    nb, msg = compare_stats(b.pixels, a.pixels, "progressive")
    assert nb == 0, msg


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_shallow_depth_and_exhaustion(om, oracle, pipeline):
    # max_depth 1 and 0: every hit path ends with -Color::ZERO (render_thread.rs:142)
    W, H = 24, 16
    for depth in (0, 1, 2):
        got, exp, _ = _render_both(om, oracle, om.random_scene(0x5EED), oracle.random_scene(0x5EED),
                                   om.default_camera(W / H), oracle.default_camera(W / H), W, H, 2, "auto",
                                   max_depth=depth, pipeline=pipeline)
        nb, msg = compare_stats(got, exp, f"depth{depth}")
        assert nb == 0, msg


@pytest.mark.parametrize("kernel", [("bvh", "megakernel"), ("sbvh", "megakernel"), ("bvh", "wavefront"),
                                    ("sbvh", "wavefront"), ("bvh2", "wavefront"), ("bvh4", "wavefront")])
def test_ten_k_scene_bvh_bit_exact(om, oracle, kernel):
    W, H, SPP = 32, 18, 2
    got, exp, _ = _render_both(om, oracle, om.random_scene(0x5EED, grid_half=50, extras=False),
                               oracle.random_scene(0x5EED, grid_half=50, extras=False),
                               om.default_camera(W / H), oracle.default_camera(W / H), W, H, SPP, kernel)
    nb, msg = compare_stats(got, exp, "S-10k")
    assert nb == 0, msg


def test_ten_k_half_bvh4_adaptive_and_tail_bit_exact(om, oracle):
    """The half-precision 4-wide tree read through L2 (OM_KERNEL_BVH4 on S-10k): a
    wider frame than test_ten_k_scene_bvh_bit_exact, adaptive sampling, and the persistent tail
    from bounce 2, so most segments run in the tail's traversal."""
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 48, 27, 6
    world = om.random_scene(0x5EED, grid_half=50, extras=False)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, kernel="bvh4", pipeline="wavefront")
    L.check(L.lib.om_set_tail_bounce(fz.ctx, 2), fz.ctx)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=9, adaptive=True)
    p = oracle.params(W, H, SPP, adaptive=True, seed=9)
    exp, _ = oracle.render(oracle.random_scene(0x5EED, grid_half=50, extras=False), oracle.default_camera(W / H), p)
    nb, msg = compare_stats(pix.pixels, exp, "S-10k/bvh4-half")
    assert nb == 0, msg


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_counters_consistent(om, pipeline):
    W, H, SPP = 32, 16, 4
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    for k in KERNELS:
        fz = world.freeze(cam, kernel=k, pipeline=pipeline)
        pix = om.PixelsBox.new(W * H)
        c = om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=2, adaptive=False)
        assert c["samples"] == W * H * SPP
        assert c["segments"] >= c["samples"]
        if k == "brute":
            assert c["prim_tests"] == c["segments"] * 485


@pytest.mark.parametrize("kernel", COMBOS)
def test_counting_build_is_bit_identical(om, kernel):
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 48, 32, 3
    world = om.random_scene(0x5EED, with_torus=True)
    cam = om.default_camera(W / H)
    out = []
    for count in (1, 0):
        fz = world.freeze(cam, kernel=kernel[0], pipeline=kernel[1])
        L.check(L.lib.om_set_counting(fz.ctx, count), fz.ctx)
        pix = om.PixelsBox.new(W * H)
        om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=4, adaptive=False)
        out.append(pix.pixels.copy())
    nb, msg = compare_stats(out[1], out[0], f"count/{kernel}")
    assert nb == 0, msg


@pytest.mark.parametrize("kernel", KERNELS)
def test_pixel_list_shard_equals_full_frame(om, kernel):
    """om_render_device_pixels over rank shards (wavefront) == one full-frame render."""
    import ctypes as C
    import torch
    from raytracingoneweekend_amd import _lib as L
    from raytracingoneweekend_amd import shard
    W, H, SPP = 40, 24, 3
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    full = om.PixelsBox.new(W * H)
    fz = world.freeze(cam, kernel=kernel)
    om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, full, seed=6, adaptive=False)
    shards = []
    p = om.make_params(50, 0.001, 100.0, SPP, W, H, seed=6)
    for r in range(3):
        pix = shard.tile_pixels(W, H, r, 3)
        dpix = torch.from_numpy(pix.view(np.int32)).cuda()
        st = torch.zeros(pix.size * 40, dtype=torch.uint8, device="cuda")
        L.check(L.lib.om_render_device_pixels(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()),
                                              C.c_void_p(dpix.data_ptr()), pix.size, None), fz.ctx)
        torch.cuda.synchronize()
        shards.append(st.cpu().numpy())
    frame = shard.assemble(W, H, shards)
    nb, msg = compare_stats(frame, full.pixels, f"shards/{kernel}")
    assert nb == 0, msg


@pytest.mark.parametrize("tail", [1, 2, 3, 7, 50])
def test_tail_bounce_is_bit_identical(om, oracle, tail):
    """Wavefront scheduling knob: any tail bounce (persistent whole-path launch) == oracle."""
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 48, 30, 4
    world = om.random_scene(0x5EED, with_torus=True)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, kernel="auto", pipeline="wavefront")
    L.check(L.lib.om_set_tail_bounce(fz.ctx, tail), fz.ctx)
    pix = om.PixelsBox.new(W * H)
    c = om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=9, adaptive=False)
    p = oracle.params(W, H, SPP, max_depth=50, seed=9)
    exp, _ = oracle.render(oracle.random_scene(0x5EED, with_torus=True), oracle.default_camera(W / H), p)
    nb, msg = compare_stats(pix.pixels, exp, f"tail{tail}")
    assert nb == 0, msg
    assert c["samples"] == W * H * SPP


def test_auto_pipeline_choice(om, oracle):
    """OM_PIPELINE_AUTO: the wavefront for every world, fixed-spp or adaptive, on one stream or
    two (the faster pipeline on every measured config since r04), observed
    through the per-launch timing classes; bit-exact."""
    import ctypes as C
    from raytracingoneweekend_amd import _lib as L
    W, H = 24, 16
    for world, oworld, adaptive, streams, want in (
            (om.marched_scene(), oracle.marched_scene(), False, 1, "wavefront"),
            (om.marched_scene(), oracle.marched_scene(), False, 2, "wavefront"),
            (om.marched_scene(), oracle.marched_scene(), True, 2, "wavefront"),
            (om.marched_scene(), oracle.marched_scene(), True, 1, "wavefront"),
            (om.random_scene(0x5EED), oracle.random_scene(0x5EED), True, 2, "wavefront"),
            (om.random_scene(0x5EED), oracle.random_scene(0x5EED), False, 1, "wavefront"),
            (om.random_scene(0x5EED), oracle.random_scene(0x5EED), False, 2, "wavefront")):
        cam = om.default_camera(W / H)
        fz = world.freeze(cam)                                    # pipeline="auto" is the default
        L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
        L.check(L.lib.om_set_timing(fz.ctx, 1), fz.ctx)
        pix = om.PixelsBox.new(W * H)
        om.render(cam, fz, 50, 0.001, 100.0, 8, W, H, pix, seed=8, march_steps=256, adaptive=adaptive)
        kt = L.om_kernel_times()
        L.check(L.lib.om_get_kernel_times(fz.ctx, C.byref(kt)), fz.ctx)
        mega = kt.launches[L.KT_CLASSES.index("megakernel")]
        wave = sum(kt.launches[L.KT_CLASSES.index(k)] for k in ("bounce0", "bounce", "tail"))
        assert (mega > 0 and wave == 0) if want == "megakernel" else (mega == 0 and wave > 0), want
        exp, _ = oracle.render(oworld, oracle.default_camera(W / H),
                               oracle.params(W, H, 8, seed=8, march_steps=256, adaptive=adaptive))
        nb, msg = compare_stats(pix.pixels, exp, f"auto/{want}")
        assert nb == 0, msg


def _render_lists(om, world, cam, W, H, spp, lists, seed=12, march_steps=1024):
    from raytracingoneweekend_amd import _lib as L
    fz = world.freeze(cam, pipeline="wavefront")
    L.check(L.lib.om_set_primary_lists(fz.ctx, lists), fz.ctx)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, spp, W, H, pix, seed=seed, march_steps=march_steps, adaptive=False)
    return pix.pixels


@pytest.mark.parametrize("scene", ["traced", "full", "kitchen", "10k", "inside_wide_lens"])
def test_primary_tile_lists_bit_exact(om, oracle, scene):
    """Bounce 0 with per-tile candidate lists (forced on / off / auto) == oracle, incl. a
    wide-aperture camera inside the sphere field (boxes behind the camera, large lens
    parallax) and odd frame sizes (partial tiles)."""
    W, H, SPP = 53, 37, 3
    if scene == "kitchen":
        w, ow, cam, ocam = kitchen_sink(om, oracle)
    else:
        kw = {"traced": {}, "full": {"with_torus": True}, "10k": {"grid_half": 50, "extras": False},
              "inside_wide_lens": {}}[scene]
        w, ow = om.random_scene(0x5EED, **kw), oracle.random_scene(0x5EED, **kw)
        if scene == "inside_wide_lens":
            args = ((0.3, 0.35, 0.2), (5.0, 0.2, 2.0), (0.0, 1.0, 0.0), 70.0, W / H, 1.5, 2.0)
            cam, ocam = om.Camera.new(*args), oracle.camera(*args)
        else:
            cam, ocam = om.default_camera(W / H), oracle.default_camera(W / H)
    exp, _ = oracle.render(ow, ocam, oracle.params(W, H, SPP, seed=12))
    for lists in (2, 0, 1):
        got = _render_lists(om, w, cam, W, H, SPP, lists)
        nb, msg = compare_stats(got, exp, f"lists{lists}/{scene}")
        assert nb == 0, msg


@pytest.mark.parametrize("streams", [1, 2, 3, 4])
def test_concurrent_batches_are_bit_identical(om, oracle, streams):
    """om_set_streams: a fixed-spp call split into batches in flight on
    1-4 streams == the oracle, including a call that starts from a partly rendered frame
    (sample indices from the call-start Stats.n snapshot) and runs past spp_total (the
    excess samples are skipped), under both timing modes."""
    import ctypes as C
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 40, 28, 10
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, kernel="auto", pipeline="wavefront")
    L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
    L.check(L.lib.om_set_timing(fz.ctx, 1 + streams % 2), fz.ctx)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=4, sample_count=3, adaptive=False)
    om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=4, sample_count=9, adaptive=False)   # 7 taken, 2 skipped
    kt = L.om_kernel_times()
    L.check(L.lib.om_get_kernel_times(fz.ctx, C.byref(kt)), fz.ctx)
    L.check(L.lib.om_set_timing(fz.ctx, 0), fz.ctx)
    exp, _ = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                           oracle.params(W, H, SPP, max_depth=50, seed=4))
    nb, msg = compare_stats(pix.pixels, exp, f"streams{streams}")
    assert nb == 0, msg
    span = L.KT_CLASSES.index("bounce_span")
    assert kt.launches[span] > 0 and kt.ms[span] > 0.0
    assert int(pix.pixels["n"].min()) == SPP and int(pix.pixels["n"].max()) == SPP
    assert L.lib.om_set_streams(fz.ctx, 5) == L.OM_ERR_INVALID


@pytest.mark.parametrize("streams", [1, 2, 3, 4])
@pytest.mark.parametrize("sched", [(0, 0), (2, 10), (7, 8)])
def test_concurrent_adaptive_batches_are_bit_identical(om, oracle, streams, sched):
    """Adaptive calls on 1-4 streams: the live pixels dealt to the streams by
    64-entry chunks, each stream's batches planned on the device from its live list (compacted by
    every accumulate), samples past a retirement inside a batch dropped in sample order.  Schedules
    (om_set_adaptive_batches): the default; at most 2 batches per stream per call with 2^10 paths
    targeted (the even share of the call decides); 7 batches at 2^8 paths (every batch of a stream
    sized by its live count).  Calls of 7, 16 and 17 samples and one of 40 == the sequential oracle."""
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 72, 40, 40
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    exp, _ = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                           oracle.params(W, H, SPP, seed=21, adaptive=True))
    for counts in ((7, 16, 17), (40,)):
        fz = world.freeze(cam, kernel="auto", pipeline="wavefront")
        L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
        L.check(L.lib.om_set_adaptive_batches(fz.ctx, *sched), fz.ctx)
        pix = om.PixelsBox.new(W * H)
        for c in counts:
            om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=21, adaptive=True, sample_count=c)
        nb, msg = compare_stats(pix.pixels, exp, f"adaptive streams{streams} sched{sched} calls{counts}")
        assert nb == 0, msg
        assert int(pix.pixels["n"].min()) < SPP
    assert L.lib.om_set_adaptive_batches(fz.ctx, 65, 0) == L.OM_ERR_INVALID
    assert L.lib.om_set_adaptive_batches(fz.ctx, 64, 0) == L.OM_OK
    assert L.lib.om_set_adaptive_batches(fz.ctx, 0, 28) == L.OM_ERR_INVALID


@pytest.mark.parametrize("streams", [1, 2, 3])
def test_concurrent_adaptive_marched_bit_identical(om, oracle, streams):
    """The adaptive schedule on a marched world: camera paths through k_raygen's live
    list, the lane-refilling tail from bounce 1, several batches per stream (2^8 paths targeted),
    calls of 17 and 40 samples == the sequential oracle."""
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 40, 24, 57
    exp, _ = oracle.render(oracle.marched_scene(), oracle.default_camera(W / H),
                           oracle.params(W, H, SPP, seed=23, adaptive=True, march_steps=256))
    cam = om.default_camera(W / H)
    fz = om.marched_scene().freeze(cam, pipeline="wavefront")
    L.check(L.lib.om_set_streams(fz.ctx, streams), fz.ctx)
    L.check(L.lib.om_set_adaptive_batches(fz.ctx, 6, 8), fz.ctx)
    pix = om.PixelsBox.new(W * H)
    for c in (17, 40):
        om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=23, adaptive=True, sample_count=c, march_steps=256)
    nb, msg = compare_stats(pix.pixels, exp, f"adaptive marched streams{streams}")
    assert nb == 0, msg
    assert int(pix.pixels["n"].min()) < SPP


@pytest.mark.parametrize("pipeline", PIPELINES)
@pytest.mark.parametrize("size", [(1, 1), (1, 7), (5, 1), (2, 2), (9, 3), (8, 8), (17, 9)])
def test_degenerate_and_ragged_frames_bit_exact(om, oracle, pipeline, size):
    """Frame edge cases: a 1-pixel-wide or -high frame divides by W-1 = 0 or H-1 = 0
    (render_thread.rs:190-191), so its rays are non-finite and take the reference loop's
    closed-form answer (hits.rs:274-285); partial 8x8 tiles; frames of exactly one tile."""
    W, H = size
    got, exp, _ = _render_both(om, oracle, om.random_scene(0x5EED), oracle.random_scene(0x5EED),
                               om.default_camera(W / H), oracle.default_camera(W / H), W, H, 3, "auto",
                               seed=21, pipeline=pipeline)
    nb, msg = compare_stats(got, exp, f"{W}x{H}/{pipeline}")
    assert nb == 0, msg
    assert (got["n"] == 3).all()


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_sparse_worlds_bit_exact(om, oracle, pipeline):
    """Worlds with a single primitive kind: one infinite plane (accepted by non-finite rays),
    one sphere (the BVH2 holds a single leaf), and only marched objects (no traced list)."""
    W, H, SPP = 24, 16, 3
    cams = (om.default_camera(W / H), oracle.default_camera(W / H))
    mats = (om.Material.new_lambertian((0.4, 0.5, 0.6)), oracle.material("lambertian", (0.4, 0.5, 0.6)))
    builds = []
    w, ow = om.HittableList.new(), oracle.World()
    w += om.InfinitePlane.new((0., 0., 0.), (0., 1., 0.), mats[0]); ow.add_plane((0., 0., 0.), (0., 1., 0.), mats[1])
    builds.append(("plane", w, ow))
    w, ow = om.HittableList.new(), oracle.World()
    w += om.Sphere.new_with_radius((0., 1., 0.), 1., mats[0]); ow.add_sphere_radius((0., 1., 0.), 1., mats[1])
    builds.append(("sphere", w, ow))
    w, ow = om.HittableList.new(), oracle.World()
    w += om.MarchedSphere((0., 1., 0.), 1., mats[0]); ow.add_marched_sphere((0., 1., 0.), 1., mats[1])
    builds.append(("marched", w, ow))
    for name, w, ow in builds:
        got, exp, _ = _render_both(om, oracle, w, ow, cams[0], cams[1], W, H, SPP, "auto", seed=22,
                                   march_steps=256, pipeline=pipeline)
        nb, msg = compare_stats(got, exp, f"{name}/{pipeline}")
        assert nb == 0, msg


def test_zero_samples_and_empty_frames(om):
    """samples_per_pixel = 0 takes no sample (render()'s pass loop never runs) and leaves the
    caller's Stats untouched; a 0-pixel frame is an argument error."""
    from raytracingoneweekend_amd import _lib as L
    W, H = 16, 8
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, 4, W, H, pix, seed=3, sample_count=2, adaptive=False)
    before = pix.pixels.copy()
    om.render(cam, fz, 50, 0.001, 100.0, 0, W, H, pix, seed=3, adaptive=False)
    assert np.array_equal(before.view(np.uint8), pix.pixels.view(np.uint8))
    with pytest.raises(L.OmError, match="width/height"):
        om.render(cam, fz, 50, 0.001, 100.0, 4, 0, H, om.PixelsBox.new(0), seed=3, adaptive=False)


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_async_calls_with_different_seeds_on_one_stream(om, oracle, pipeline):
    """Two om_render_device calls queued back to back on one user stream with different seeds
    and spp_total (so different jitter tables), synchronised once at the end: each frame ==
    the oracle.  Before r02 the second call rewrote the ctx's one jitter table while the first
    call's kernels could still read it."""
    import ctypes as C
    import torch
    from raytracingoneweekend_amd import _lib as L
    W, H = 40, 24
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, pipeline=pipeline)
    s = torch.cuda.Stream()
    cases = [(31, 6), (32, 10), (33, 6)]
    frames = [torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda") for _ in cases]
    torch.cuda.synchronize()
    for (seed, spp), st in zip(cases, frames):
        p = om.make_params(50, 0.001, 100.0, spp, W, H, seed=seed)
        L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()),
                                       C.c_void_p(s.cuda_stream)), fz.ctx)
    s.synchronize()
    for (seed, spp), st in zip(cases, frames):
        exp, _ = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                               oracle.params(W, H, spp, seed=seed))
        got = st.cpu().numpy().view(L.PIXEL_STATS_DTYPE)
        nb, msg = compare_stats(got, exp, f"async seed {seed}/{pipeline}")
        assert nb == 0, msg


def test_python_render_defaults_to_reference_adaptive(om, oracle):
    """api.render() with no `adaptive` argument retires pixels like the reference's
    render threads (ThreadPixels::add_run is unconditional, render_thread.rs:97-101) and
    credits samples_atom with the untaken samples (render_thread.rs:196-198)."""
    W, H, SPP = 32, 24, 24
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    pix = om.PixelsBox.new(W * H)
    atom = [0]
    om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, samples_atom=atom, seed=14)
    exp, ctr = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H),
                             oracle.params(W, H, SPP, seed=14, adaptive=True))
    nb, msg = compare_stats(pix.pixels, exp, "default adaptive")
    assert nb == 0, msg
    assert pix.pixels["n"].min() < SPP
    assert atom[0] == W * H * SPP


@pytest.mark.parametrize("pipeline,adaptive", [("wavefront", False), ("wavefront", True), ("megakernel", False)])
def test_live_progress_word(om, pipeline, adaptive):
    """om_progress: the samples_atom word (render_thread.rs:196-198) advances while a call runs
    (the wavefront adds each accumulated batch) and ends equal to the call's credited count."""
    import ctypes as C
    import torch
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = (1920, 1080, 64) if not adaptive else (640, 360, 96)
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam, pipeline=pipeline)
    prog = L.lib.om_progress(fz.ctx)
    assert prog and prog[0] == 0
    frame = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    L.check(L.lib.om_reset_counters(fz.ctx, C.c_void_p(s.cuda_stream)), fz.ctx)
    p = om.make_params(50, 0.001, 100.0, SPP, W, H, seed=3, adaptive=adaptive)
    L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(frame.data_ptr()),
                                   C.c_void_p(s.cuda_stream)), fz.ctx)
    seen = []
    while not s.query():
        seen.append(int(prog[0]))
    s.synchronize()
    seen.append(int(prog[0]))
    ctr = fz.counters()
    assert all(a <= b for a, b in zip(seen, seen[1:])), "progress went backwards"
    assert seen[-1] == ctr["credited"] == W * H * SPP
    if pipeline == "wavefront":
        assert any(0 < v < seen[-1] for v in seen), "no progress seen inside the call"
    L.check(L.lib.om_reset_progress(fz.ctx), fz.ctx)
    assert prog[0] == 0


@pytest.mark.parametrize("pipeline", PIPELINES)
def test_user_sdf_zoo_bit_exact(om, oracle, pipeline):
    """User marched objects (`HittableList += Arc<dyn Marched>`, hits.rs:96-100) as SDF programs
    (om_world_add_marched_sdf): CSG with every op under non-uniform transforms, visited after the
    typed marched objects in the march loop and unstuck (hits.rs:312-319, 350-356), their normals by
    the trait's central differences (marched.rs:19-44) == the oracle, both pipelines."""
    from scenes_common import user_sdf_zoo
    w, ow, cam, ocam = user_sdf_zoo(om, oracle)
    W, H, SPP = 72, 48, 5
    got, exp, _ = _render_both(om, oracle, w, ow, cam, ocam, W, H, SPP, "auto", march_steps=512, pipeline=pipeline,
                               seed=31)
    nb, msg = compare_stats(got, exp, f"user sdf zoo/{pipeline}")
    assert nb == 0, msg
    for oid in (4, 5, 6):                                  # the three programs (after sphere, box, torus)
        h = np.uint64(oracle.bloom_hash(oid))
        assert int(((got["bloom"] & h) == h).sum()) > 0, f"user object {oid} not seen"


def test_user_sdf_torus_program_equals_marched_torus(om, oracle):
    """The program [torus 0 0 0 R r] is a MarchedTorus (marched.rs:133-151): on the GPU the two worlds
    render identical frames (same object index, so bloom too), equal to the oracle; wavefront with
    the concurrent batches and the adaptive live-list schedule (several batches per stream)."""
    from raytracingoneweekend_amd import _lib as L
    from scenes_common import user_sdf_zoo
    W, H, SPP = 64, 40, 24
    frames = []
    for prog in (False, True):
        w, ow, cam, ocam = user_sdf_zoo(om, oracle, torus_as_program=prog)
        fz = w.freeze(cam, pipeline="wavefront")
        L.check(L.lib.om_set_adaptive_batches(fz.ctx, 5, 8), fz.ctx)
        pix = om.PixelsBox.new(W * H)
        for c in (7, 17):
            om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, pix, seed=33, adaptive=True, sample_count=c, march_steps=256)
        frames.append(pix.pixels.copy())
    assert np.array_equal(frames[0].view(np.uint8), frames[1].view(np.uint8))
    exp, _ = oracle.render(ow, ocam, oracle.params(W, H, SPP, seed=33, adaptive=True, march_steps=256))
    nb, msg = compare_stats(frames[1], exp, "torus program, adaptive")
    assert nb == 0, msg
    assert int(frames[1]["n"].min()) < SPP
