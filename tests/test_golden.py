"""Committed fixtures (tests/golden/golden_v2.npz, made by tests/golden/make_golden.py):
the oracle must keep reproducing them (CPU), and the HIP path must produce the stored
images bit for bit (GPU) — no oracle needed at GPU run time."""
import os

import numpy as np
import pytest

from scenes_common import kitchen_sink

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_v2.npz"))


def test_oracle_reproduces_rng_and_tables(oracle):
    assert np.array_equal(oracle.rng_draws(0, 64), G["rng_seed0"])
    assert np.array_equal(oracle.rng_draws(0x5EED, 64), G["rng_seed5eed"])
    assert np.array_equal(oracle.path_draws(1, 12345, 7, 32), G["path_draws"])
    assert np.array_equal(oracle.jitter_table(1, 16), G["jitter_s1_16"])
    assert np.array_equal(np.array([oracle.bloom_hash(i) for i in range(65)], dtype=np.uint64), G["bloom_1_64"])


def test_oracle_reproduces_scene(oracle):
    ow = oracle.random_scene(0x5EED)
    assert ow.counts()[:8] == list(G["straced_counts"])
    s = np.stack([ow.affine(0, i) for i in range(ow.counts()[0])])
    assert np.array_equal(s.view(np.uint32), G["straced_spheres"].view(np.uint32))


def test_product_scene_matches_golden(om):
    w = om.random_scene(0x5EED)
    s = np.stack([w.export(0, i, 32) for i in range(w.counts()["spheres"])])
    assert np.array_equal(s.view(np.uint32), G["straced_spheres"].view(np.uint32))
    assert np.array_equal(w.export(1, 0, 32).view(np.uint32), G["straced_cube"].view(np.uint32))
    assert np.array_equal(w.export(2, 0, 29).view(np.uint32), G["straced_tri"].view(np.uint32))
    assert np.array_equal(w.export(4, 0, 29).view(np.uint32), G["straced_para"].view(np.uint32))


def test_oracle_reproduces_images(oracle):
    W, H = 40, 24
    st, ctr = oracle.render(oracle.random_scene(0x5EED), oracle.default_camera(W / H), oracle.params(W, H, 8, seed=3),
                            nthreads=3)
    assert np.array_equal(st.view(np.uint8).reshape(-1, 40), G["img_straced_40x24x8_seed3"])
    assert [ctr["samples"], ctr["segments"]] == list(G["img_straced_ctr"])
    st, _ = oracle.render(oracle.marched_scene(), oracle.default_camera(24 / 16),
                          oracle.params(24, 16, 2, seed=2, march_steps=256), nthreads=2)
    assert np.array_equal(st.view(np.uint8).reshape(-1, 40), G["img_marched_24x16x2_seed2"])


def _gpu_render(om, world, cam, W, H, spp, seed, kernel, march_steps=1024):
    fz = world.freeze(cam, kernel=kernel)
    pix = om.PixelsBox.new(W * H)
    om.render(cam, fz, 50, 0.001, 100.0, spp, W, H, pix, seed=seed, march_steps=march_steps, adaptive=False)
    return pix.pixels.view(np.uint8).reshape(-1, 40)


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["brute", "culled", "bvh", "sbvh", "bvh2", "bvh4"])
def test_gpu_matches_golden_images(om, oracle, kernel):
    W, H = 40, 24
    assert np.array_equal(_gpu_render(om, om.random_scene(0x5EED), om.default_camera(W / H), W, H, 8, 3, kernel),
                          G["img_straced_40x24x8_seed3"])
    assert np.array_equal(_gpu_render(om, om.random_scene(0x5EED, with_torus=True), om.default_camera(W / H),
                                      W, H, 2, 4, kernel), G["img_sfull_40x24x2_seed4"])
    w, _, cam, _ = kitchen_sink(om, oracle)
    assert np.array_equal(_gpu_render(om, w, cam, 32, 20, 4, 11, kernel), G["img_kitchen_32x20x4_seed11"])
    assert np.array_equal(_gpu_render(om, om.marched_scene(), om.default_camera(24 / 16), 24, 16, 2, 2, kernel, 256),
                          G["img_marched_24x16x2_seed2"])
