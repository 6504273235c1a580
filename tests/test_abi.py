"""The C-ABI library: loads, exports every symbol include/ottomarcher.h declares,
validates arguments and reports errors without a GPU (no compute calls here)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "ottomarcher.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(om_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree(om):
    from raytracingoneweekend_amd import _lib
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol(om):
    from raytracingoneweekend_amd import _lib
    raw = C.CDLL(_lib.LIB_PATH)
    missing = [n for n in header_functions() if not hasattr(raw, n)]
    assert not missing, missing


def test_library_is_gfx950_code_object(om):
    from raytracingoneweekend_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob and b"render_kernel" in blob


def test_build_id_matches_checked_out_sources(om):
    """Build provenance: the library names the source hash it was built from (baked in at
    link time by csrc/Makefile), which must be the hash of the sources in this tree."""
    from raytracingoneweekend_amd import _lib
    from raytracingoneweekend_amd.build_id import source_hash
    assert re.fullmatch(r"[0-9a-f]{16}", _lib.build_id())
    assert _lib.build_id() == source_hash()
    assert _lib.check_build_provenance() == source_hash()


def test_abi_version_and_struct_sizes(om):
    from raytracingoneweekend_amd import _lib
    assert _lib.lib.om_abi_version() == 2
    assert C.sizeof(_lib.om_material) == 24
    assert C.sizeof(_lib.om_render_params) == 48
    assert _lib.PIXEL_STATS_DTYPE.itemsize == 40


def test_argument_validation(om):
    from raytracingoneweekend_amd import _lib
    L = _lib.lib
    m = L.om_material_lambertian(0.5, 0.5, 0.5)
    assert L.om_world_add_sphere(None, None, C.byref(m)) == _lib.OM_ERR_INVALID
    w = C.c_void_p()
    assert L.om_world_create(C.byref(w)) == 0
    bad = _lib.om_material()
    bad.type = 7
    c = (C.c_float * 3)(0, 0, 0)
    assert L.om_world_add_sphere_radius(w, _lib.fptr(c), 1.0, C.byref(bad)) == _lib.OM_ERR_INVALID
    assert b"invalid material" in L.om_last_error(None)
    assert L.om_world_export(w, 0, 0, _lib.fptr((C.c_float * 32)()), 32) == _lib.OM_ERR_INVALID  # empty world
    assert L.om_world_random_scene(w, 1, 0, -1) == _lib.OM_ERR_INVALID
    assert L.om_set_kernel(None, 0) == _lib.OM_ERR_INVALID
    assert L.om_render(None, None, None, None, None) == _lib.OM_ERR_INVALID
    assert L.om_upload_world(None, w) == _lib.OM_ERR_INVALID
    L.om_world_destroy(w)


def test_create_fails_loudly_without_device(om):
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("a HIP device is present")
    from raytracingoneweekend_amd import _lib
    ctx = C.c_void_p()
    assert _lib.lib.om_create(0, C.byref(ctx)) == _lib.OM_ERR_DEVICE
    with pytest.raises(_lib.OmError):
        om.random_scene().freeze()


def test_mat4_helpers(om):
    F = np.float32
    t = om.m4x4("TR", 1., 2., 3.).to_numpy()
    assert np.array_equal(t, np.array([[1, 0, 0, 1], [0, 1, 0, 2], [0, 0, 1, 3], [0, 0, 0, 1]], F))
    s = om.m4x4("SC", 2., 3., 4.).to_numpy()
    assert np.array_equal(np.diag(s), np.array([2, 3, 4, 1], F))
    r = om.m4x4("RZ", 0.5).to_numpy()
    c, sn = np.cos(F(0.5)), np.sin(F(0.5))
    assert np.allclose(r[:2, :2], [[c, -sn], [sn, c]], atol=1e-7)   # mat4x4.rs:116-123 layout
    m = om.m4x4("TR", 1., 2., 3.) ^ om.m4x4("SC", 2., 4., 8.)
    inv = m.fast_homogenous_inverse().to_numpy()
    assert np.array_equal(inv, np.array([[0.5, 0, 0, -0.5], [0, 0.25, 0, -0.5], [0, 0, 0.125, -0.375], [0, 0, 0, 1]], F))
    assert np.array_equal(om.Mat4x4.identity().to_numpy(), np.eye(4, dtype=F))


def test_world_counts_type_order(om):
    w = om.HittableList.new()
    mat = om.Material.new_lambertian((0.1, 0.2, 0.3))
    w += om.MarchedBox((0, 0, 0), (1, 1, 1), mat)
    w += om.Sphere.new_with_radius((0, 0, 0), 1, mat)
    w += om.InfinitePlane.new((0, 0, 0), (0, 1, 0), mat)
    w += om.Parallelogram.new3points((0, 0, 0), (1, 0, 0), (0, 1, 0), mat)
    c = w.counts()
    assert (c["spheres"], c["infinite_planes"], c["parallelograms"], c["marched_boxes"]) == (1, 1, 1, 1)
    w.clear()
    assert sum(w.counts().values()) == 0
    with pytest.raises(TypeError):
        w += object()


def test_marched_sdf_program_validation(om):
    """om_world_add_marched_sdf (a user `impl Marched`, hits.rs:96-100) accepts well-formed postfix
    programs and refuses malformed ones with OM_ERR_INVALID, on the host, before any device work."""
    from raytracingoneweekend_amd import _lib
    L = _lib.lib
    w = om.HittableList.new()
    mat = om.Material.new_lambertian((0.4, 0.4, 0.4))
    eye = om.Mat4x4.identity()

    def add(ops, n=None):
        arr = _lib.sdf_ops(ops) if ops else np.zeros(1, dtype=_lib.SDF_OP_DTYPE)
        return L.om_world_add_marched_sdf(w.handle, _lib.fptr(eye.m), arr.ctypes.data_as(C.c_void_p),
                                          arr.size if n is None else n, C.byref(mat.raw))
    ok = [[("sphere", 0, 0, 0, 1)],
          [("box", 0, 0, 0, 1, 1, 1), ("round", 0.1)],
          [("sphere", 0, 0, 0, 1), ("torus", 0, 0, 0, 1, 0.2), ("union",)],
          [("sphere", 0, 0, 0, 1)] * 8 + [("union",)] * 7]
    for ops in ok:
        assert add(ops) == 0, L.om_last_error(None)
    bad = [[("union",)],                                           # stack underflow
           [("round", 0.1)],                                       # underflow
           [("sphere", 0, 0, 0, 1), ("sphere", 0, 0, 0, 1)],       # two values left
           [("sphere", 0, 0, 0, 1)] * 9 + [("union",)] * 8,        # deeper than OM_SDF_MAX_STACK
           [(99, 0, 0, 0, 1)],                                     # unknown op
           [("sphere", 0, 0, 0, float("nan"))],                    # non-finite parameter
           [("sphere", 0, 0, 0, 1)] * 65]                          # more than OM_SDF_MAX_OPS
    for ops in bad:
        assert add(ops) == _lib.OM_ERR_INVALID, ops
    assert add([("sphere", 0, 0, 0, 1)], n=0) == _lib.OM_ERR_INVALID
    assert w.counts()["marched_sdf"] == len(ok)
    w += om.MarchedSdf.new(eye, [("sphere", 0, 0, 0, 0.5)], mat)
    assert w.counts()["marched_sdf"] == len(ok) + 1
