"""ctypes binding of libottomarcher.so (the C-ABI declared in include/ottomarcher.h).

The library is the product: every render goes through its HIP kernels.  There is
no CPU fallback — if the shared library is missing, importing this module raises.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# OM_LIB: load another build of the same library (A/B timing of build variants, tools/ablate.sh)
LIB_PATH = os.environ.get("OM_LIB") or os.path.join(_HERE, "libottomarcher.so")

OM_OK = 0
OM_ERR_INVALID, OM_ERR_DEVICE, OM_ERR_STATE, OM_ERR_UNSUPPORTED, OM_ERR_NOMEM = -1, -2, -3, -4, -5
OM_LAMBERTIAN, OM_METAL, OM_DIELECTRIC = 0, 1, 2
OM_KERNEL_AUTO, OM_KERNEL_BRUTE, OM_KERNEL_CULLED, OM_KERNEL_BVH, OM_KERNEL_SBVH, OM_KERNEL_BVH2, OM_KERNEL_BVH4 = \
    0, 1, 2, 3, 4, 5, 6
KERNELS = {"auto": OM_KERNEL_AUTO, "brute": OM_KERNEL_BRUTE, "culled": OM_KERNEL_CULLED, "bvh": OM_KERNEL_BVH,
           "sbvh": OM_KERNEL_SBVH, "bvh2": OM_KERNEL_BVH2, "bvh4": OM_KERNEL_BVH4}
OM_PIPELINE_MEGAKERNEL, OM_PIPELINE_WAVEFRONT, OM_PIPELINE_AUTO = 0, 1, 2
PIPELINES = {"megakernel": OM_PIPELINE_MEGAKERNEL, "wavefront": OM_PIPELINE_WAVEFRONT, "auto": OM_PIPELINE_AUTO}

F3 = C.c_float * 3
F16 = C.c_float * 16


class om_material(C.Structure):
    _fields_ = [("albedo", C.c_float * 3), ("fuzz", C.c_float), ("ior", C.c_float), ("type", C.c_int32)]


class om_camera(C.Structure):
    _fields_ = [(n, C.c_float * 3) for n in ("origin", "horizontal", "vertical", "lower_left_corner",
                                              "u_of_plane", "v_of_plane", "w_of_plane")] + \
               [(n, C.c_float) for n in ("lens_radius", "aspect_ratio", "focus_dist", "viewport_width", "viewport_height")]


class om_render_params(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("width", "height", "spp_total", "sample_begin", "sample_count", "max_depth")] + \
               [("tmin", C.c_float), ("tmax", C.c_float), ("march_steps", C.c_uint32), ("adaptive", C.c_uint32),
                ("seed", C.c_uint64)]


class om_counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("samples", "segments", "prim_tests", "pre_tests", "march_steps", "credited")]


# om_sdf_op (include/ottomarcher.h): one op of a user marched object's SDF program
SDF_OP_DTYPE = np.dtype([("op", "<i4"), ("a", "<f4", 7)])
SDF_OPS = {"sphere": 1, "box": 2, "torus": 3, "union": 4, "intersect": 5, "subtract": 6, "round": 7}


def sdf_ops(ops):
    """[(name or OM_SDF_* code, param, ...), ...] -> a contiguous om_sdf_op array."""
    arr = np.zeros(len(ops), dtype=SDF_OP_DTYPE)
    for i, o in enumerate(ops):
        arr[i]["op"] = SDF_OPS[o[0]] if isinstance(o[0], str) else int(o[0])
        arr[i]["a"][:len(o) - 1] = o[1:]
    return arr


KT_CLASSES = ("bounce0", "bounce", "tail", "accumulate", "megakernel", "bounce_span")   # OM_KT_* order
# draw_to_sdl modes (main.rs:360-367), OM_VIEW_* order
VIEWS = ("normal", "samples", "sample_blur", "depth", "depth_blur", "ids", "id_blur")


class om_kernel_times(C.Structure):
    _fields_ = [("launches", C.c_uint64 * 6), ("ms", C.c_double * 6)]


# numpy view of om_pixel_stats (40 B) — render_thread.rs:9-17
PIXEL_STATS_DTYPE = np.dtype([("bloom", "<u8"), ("sum", "<f4", (3,)), ("n", "<u4"), ("avg_depth", "<f4"),
                              ("bad_avgs", "<u4"), ("color", "u1", (3,)), ("flags", "u1"), ("reserved", "<u4")])
assert PIXEL_STATS_DTYPE.itemsize == 40

# every symbol include/ottomarcher.h declares (tests check the library exports all of them)
EXPORTS = [
    "om_abi_version", "om_build_id", "om_material_lambertian", "om_material_metal", "om_material_metal_fuzz", "om_material_dielectric",
    "om_mat4_identity", "om_mat4_translate", "om_mat4_scale", "om_mat4_rotate", "om_mat4_mul",
    "om_mat4_fast_homogenous_inverse", "om_camera_new", "om_world_create", "om_world_destroy", "om_world_clear",
    "om_world_add_sphere", "om_world_add_sphere_radius", "om_world_add_cube", "om_world_add_cube_length",
    "om_world_add_triangle", "om_world_add_parallelogram", "om_world_add_triangle_basis",
    "om_world_add_parallelogram_basis", "om_world_add_plane", "om_world_add_marched_sphere",
    "om_world_add_marched_box", "om_world_add_marched_torus", "om_world_add_marched_sdf", "om_world_marched_sdf_count", "om_world_counts", "om_world_export",
    "om_world_random_scene", "om_world_basic_scene", "om_world_marched_scene", "om_create", "om_destroy",
    "om_last_error", "om_upload_world", "om_set_kernel", "om_render", "om_render_device",
    "om_render_device_pixels", "om_get_counters", "om_reset_counters", "om_set_counting", "om_set_pipeline",
    "om_set_tail_bounce", "om_set_streams", "om_set_adaptive_batches", "om_set_timing", "om_get_kernel_times", "om_display_device", "om_display",
    "om_write_bmp", "om_write_ppm", "om_set_primary_lists",
    "om_shard_capacity", "om_shard_pixels", "om_shard_assemble_host", "om_comm_unique_id", "om_comm_init_rank",
    "om_comm_destroy", "om_comm_info", "om_render_shard", "om_gather_frame", "om_scatter_frame", "om_multi_create",
    "om_multi_destroy", "om_multi_transport", "om_multi_ctx", "om_multi_upload_world", "om_multi_render",
    "om_multi_last_error", "om_progress", "om_reset_progress", "om_host_register", "om_host_unregister",
    "om_multi_render_host", "om_multi_gather", "om_multi_reset", "om_rccl_library",
]
OM_COMM_ID_BYTES = 128
OM_TRANSPORT_RCCL, OM_TRANSPORT_LOCAL = 0, 1


class OmError(RuntimeError):
    pass


def _share_hip_runtime_with_torch():
    """PyTorch-ROCm ships its own libamdhip64 (same soname).  Loading torch first makes
    libottomarcher.so bind to that one runtime, so torch tensors/streams and this
    library share a single HIP runtime in the process (two runtimes cannot both own
    the device).  torch is optional for the C-ABI itself."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _load():
    _share_hip_runtime_with_torch()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `make -C raytracingoneweekend_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    st = C.c_int32
    vp = C.c_void_p
    fp = C.POINTER(C.c_float)
    mp = C.POINTER(om_material)
    sig = {
        "om_abi_version": (C.c_int32, []),
        "om_build_id": (C.c_char_p, []),
        "om_material_lambertian": (om_material, [C.c_float] * 3),
        "om_material_metal": (om_material, [C.c_float] * 3),
        "om_material_metal_fuzz": (om_material, [C.c_float] * 4),
        "om_material_dielectric": (om_material, [C.c_float]),
        "om_mat4_identity": (st, [fp]),
        "om_mat4_translate": (st, [fp, fp]),
        "om_mat4_scale": (st, [fp, fp]),
        "om_mat4_rotate": (st, [C.c_int32, C.c_float, fp]),
        "om_mat4_mul": (st, [fp, fp, fp]),
        "om_mat4_fast_homogenous_inverse": (st, [fp, fp]),
        "om_camera_new": (st, [fp, fp, fp, C.c_float, C.c_float, C.c_float, C.c_float, C.POINTER(om_camera)]),
        "om_world_create": (st, [C.POINTER(vp)]),
        "om_world_destroy": (None, [vp]),
        "om_world_clear": (st, [vp]),
        "om_world_add_sphere": (st, [vp, fp, mp]),
        "om_world_add_sphere_radius": (st, [vp, fp, C.c_float, mp]),
        "om_world_add_cube": (st, [vp, fp, mp]),
        "om_world_add_cube_length": (st, [vp, fp, C.c_float, mp]),
        "om_world_add_triangle": (st, [vp, fp, fp, fp, mp]),
        "om_world_add_parallelogram": (st, [vp, fp, fp, fp, mp]),
        "om_world_add_triangle_basis": (st, [vp, fp, fp, fp, C.c_float, C.c_float, mp]),
        "om_world_add_parallelogram_basis": (st, [vp, fp, fp, fp, C.c_float, C.c_float, mp]),
        "om_world_add_plane": (st, [vp, fp, fp, mp]),
        "om_world_add_marched_sphere": (st, [vp, fp, C.c_float, mp]),
        "om_world_add_marched_box": (st, [vp, fp, fp, mp]),
        "om_world_add_marched_torus": (st, [vp, fp, fp, mp]),
        "om_world_add_marched_sdf": (st, [vp, fp, vp, C.c_uint32, mp]),
        "om_world_marched_sdf_count": (st, [vp, C.POINTER(C.c_uint32)]),
        "om_world_counts": (st, [vp, C.POINTER(C.c_uint32)]),
        "om_world_export": (st, [vp, C.c_int32, C.c_uint32, fp, C.c_uint32]),
        "om_world_random_scene": (st, [vp, C.c_uint64, C.c_uint32, C.c_int32]),
        "om_world_basic_scene": (st, [vp]),
        "om_world_marched_scene": (st, [vp]),
        "om_create": (st, [C.c_int32, C.POINTER(vp)]),
        "om_destroy": (None, [vp]),
        "om_last_error": (C.c_char_p, [vp]),
        "om_upload_world": (st, [vp, vp]),
        "om_set_kernel": (st, [vp, C.c_int32]),
        "om_render": (st, [vp, C.POINTER(om_camera), C.POINTER(om_render_params), vp, C.POINTER(om_counters)]),
        "om_render_device": (st, [vp, C.POINTER(om_camera), C.POINTER(om_render_params), vp, vp]),
        "om_render_device_pixels": (st, [vp, C.POINTER(om_camera), C.POINTER(om_render_params), vp, vp, C.c_uint32, vp]),
        "om_get_counters": (st, [vp, C.POINTER(om_counters)]),
        "om_reset_counters": (st, [vp, vp]),
        "om_set_counting": (st, [vp, C.c_int32]),
        "om_set_pipeline": (st, [vp, C.c_int32]),
        "om_set_tail_bounce": (st, [vp, C.c_uint32]),
        "om_set_streams": (st, [vp, C.c_uint32]),
        "om_set_adaptive_batches": (st, [vp, C.c_uint32, C.c_uint32]),
        "om_set_timing": (st, [vp, C.c_int32]),
        "om_get_kernel_times": (st, [vp, C.POINTER(om_kernel_times)]),
        "om_display_device": (st, [vp, vp, C.c_uint32, C.c_uint32, C.c_int32, vp, vp]),
        "om_display": (st, [vp, vp, C.c_uint32, C.c_uint32, C.c_int32, vp]),
        "om_write_bmp": (st, [C.c_char_p, vp, C.c_uint32, C.c_uint32]),
        "om_write_ppm": (st, [C.c_char_p, vp, C.c_uint32, C.c_uint32]),
        "om_set_primary_lists": (st, [vp, C.c_int32]),
        "om_shard_capacity": (C.c_uint32, [C.c_uint32, C.c_uint32, C.c_uint32]),
        "om_shard_pixels": (st, [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, C.c_uint32, C.POINTER(C.c_uint32)]),
        "om_shard_assemble_host": (st, [C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(vp), vp]),
        "om_comm_unique_id": (st, [vp]),
        "om_comm_init_rank": (st, [vp, C.c_uint32, C.c_uint32, vp, C.POINTER(vp)]),
        "om_comm_destroy": (None, [vp]),
        "om_render_shard": (st, [vp, C.POINTER(om_camera), C.POINTER(om_render_params), vp, vp]),
        "om_gather_frame": (st, [vp, vp, C.c_uint32, C.c_uint32, vp, vp]),
        "om_scatter_frame": (st, [vp, vp, C.c_uint32, C.c_uint32, vp, vp]),
        "om_multi_create": (st, [C.POINTER(C.c_int32), C.c_uint32, C.POINTER(vp)]),
        "om_multi_destroy": (None, [vp]),
        "om_multi_transport": (C.c_int32, [vp]),
        "om_multi_ctx": (vp, [vp, C.c_uint32]),
        "om_multi_upload_world": (st, [vp, vp]),
        "om_multi_render": (st, [vp, C.POINTER(om_camera), C.POINTER(om_render_params), vp, vp]),
        "om_multi_last_error": (C.c_char_p, [vp]),
        "om_progress": (C.POINTER(C.c_uint64), [vp]),
        "om_reset_progress": (st, [vp]),
        "om_host_register": (st, [vp, C.c_size_t]),
        "om_host_unregister": (st, [vp]),
        "om_multi_render_host": (st, [vp, C.POINTER(om_camera), C.POINTER(om_render_params), vp, C.POINTER(om_counters)]),
        "om_multi_gather": (st, [vp, vp, C.c_uint32, C.c_uint32, vp]),
        "om_multi_reset": (None, [vp]),
        "om_rccl_library": (st, [C.c_char_p, C.c_uint32, C.POINTER(C.c_int32)]),
        "om_comm_info": (st, [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


lib = _load()


def build_id():
    """Source hash the loaded library was built from (om_build_id)."""
    return lib.om_build_id().decode()


def check_build_provenance():
    """Raise if the loaded library was not built from the checked-out sources."""
    from .build_id import source_hash
    want, got = source_hash(), build_id()
    if want != got:
        raise OmError(f"{LIB_PATH} was built from other sources (om_build_id {got}, checked-out sources {want}): "
                      "rebuild with __graft_entry__.build()")
    return got


def check(status, ctx=None):
    """Raise OmError with om_last_error() text when a call fails (reference: panics, hits.rs / traced.rs:193)."""
    if status != OM_OK:
        msg = lib.om_last_error(ctx)
        raise OmError(f"ottomarcher error {status}: {msg.decode() if msg else ''}")
    return status


def f3(v):
    return F3(*[float(x) for x in v])


def fptr(arr):
    return C.cast(arr, C.POINTER(C.c_float))
