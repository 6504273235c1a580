"""The product's host builders (HittableList -> frozen data) carry exactly the bits the
oracle's restatement computes (Sphere::new / fast_homogenous_inverse / Kahan determinant,
Barycentric::new, MarchedTorus::new, Camera::new)."""
import numpy as np
import pytest

from scenes_common import kitchen_sink


def bits(a):
    return np.asarray(a, dtype=np.float32).view(np.uint32)


@pytest.mark.parametrize("variant", [dict(), dict(with_torus=True), dict(grid_half=50, extras=False)])
def test_random_scene_native_vs_oracle(om, oracle, variant):
    w = om.random_scene(0x5EED, **variant)
    ow = oracle.random_scene(0x5EED, **variant)
    c = w.counts()
    assert list(c.values()) == ow.counts()
    for i in range(c["spheres"]):
        assert np.array_equal(bits(w.export(0, i, 32)), bits(ow.affine(0, i))), i
    for i in range(c["cubes"]):
        assert np.array_equal(bits(w.export(1, i, 32)), bits(ow.affine(1, i)))
    for i in range(c["triangles"]):
        assert np.array_equal(bits(w.export(2, i, 29)), bits(ow.bary(1, i)))
    for i in range(c["parallelograms"]):
        assert np.array_equal(bits(w.export(4, i, 29)), bits(ow.bary(0, i)))
    for i in range(c["marched_torus"]):
        assert np.array_equal(bits(w.export(7, i, 43)), bits(ow.torus(i)))


def test_random_scene_through_python_api_matches_native(om):
    """main.rs:37-100 written against the mirrored API == the native builder, bit for bit."""
    a = om.random_scene_api(0x5EED, with_torus=True)
    b = om.random_scene(0x5EED, with_torus=True)
    assert a.counts() == b.counts()
    for i in range(a.counts()["spheres"]):
        assert np.array_equal(bits(a.export(0, i, 32)), bits(b.export(0, i, 32))), i
    assert np.array_equal(bits(a.export(1, 0, 32)), bits(b.export(1, 0, 32)))
    assert np.array_equal(bits(a.export(7, 0, 43)), bits(b.export(7, 0, 43)))


def test_random_scene_shape(om):
    c = om.random_scene(0x5EED).counts()
    # ground + ~481 of the 484 grid cells (exclusion radius 0.9 around (4,0.2,0)) + cube/tri/para
    assert 470 <= c["spheres"] <= 485 and c["cubes"] == 1 and c["triangles"] == 1 and c["parallelograms"] == 1
    assert c["marched_torus"] == 0
    c10 = om.random_scene(0x5EED, grid_half=50, extras=False).counts()
    assert 9900 <= c10["spheres"] <= 10001 and c10["cubes"] == 0


def test_kitchen_sink_frozen_data(om, oracle):
    w, ow, _, _ = kitchen_sink(om, oracle)
    assert list(w.counts().values()) == ow.counts()
    for i in range(w.counts()["spheres"]):
        assert np.array_equal(bits(w.export(0, i, 32)), bits(ow.affine(0, i)))
    for i in range(w.counts()["cubes"]):
        assert np.array_equal(bits(w.export(1, i, 32)), bits(ow.affine(1, i)))
    assert np.array_equal(bits(w.export(7, 0, 43)), bits(ow.torus(0)))


def test_camera_new_matches_oracle(om, oracle):
    for args in [((13., 2., 3.), (0., 0., 0.), (0., 1., 0.), 20., 1920 / 1080, 0.1, 10.),
                 ((0., 1., 2.), (0., 0.5, -1.), (0., 1., 0.), 60., 1.5, 0.05, 3.)]:
        a = om.Camera.new(*args).raw
        b = oracle.camera(*args)
        for fa, fb in [("origin", "origin"), ("horizontal", "horizontal"), ("vertical", "vertical"),
                       ("lower_left_corner", "llc"), ("u_of_plane", "u"), ("v_of_plane", "v"), ("w_of_plane", "w")]:
            assert np.array_equal(bits(list(getattr(a, fa))), bits(list(getattr(b, fb)))), fa
        assert a.lens_radius == b.lens_radius
