"""The Python binding's struct layouts and enum values equal the C header's, field by
field: a C program compiled against include/ottomarcher.h reports offsetof/sizeof and
every enum constant (what a Rust #[repr(C)] mirror must match too)."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRUCTS = {
    "om_material": ["albedo", "fuzz", "ior", "type"],
    "om_camera": ["origin", "horizontal", "vertical", "lower_left_corner", "u_of_plane", "v_of_plane", "w_of_plane",
                  "lens_radius", "aspect_ratio", "focus_dist", "viewport_width", "viewport_height"],
    "om_render_params": ["width", "height", "spp_total", "sample_begin", "sample_count", "max_depth", "tmin", "tmax",
                         "march_steps", "adaptive", "seed"],
    "om_counters": ["samples", "segments", "prim_tests", "pre_tests", "march_steps", "credited"],
    "om_kernel_times": ["launches", "ms"],
    "om_pixel_stats": ["bloom", "sum", "n", "avg_depth", "bad_avgs", "color", "flags", "reserved"],
}
ENUMS = ["OM_LAMBERTIAN", "OM_METAL", "OM_DIELECTRIC", "OM_KERNEL_AUTO", "OM_KERNEL_BRUTE", "OM_KERNEL_CULLED",
         "OM_KERNEL_BVH", "OM_KERNEL_SBVH", "OM_KERNEL_BVH2", "OM_KERNEL_BVH4", "OM_PIPELINE_MEGAKERNEL", "OM_PIPELINE_WAVEFRONT", "OM_PIPELINE_AUTO",
         "OM_KT_BOUNCE0", "OM_KT_BOUNCE", "OM_KT_TAIL", "OM_KT_ACCUMULATE", "OM_KT_MEGAKERNEL", "OM_KT_BOUNCE_SPAN",
         "OM_KT_N",
         "OM_OK", "OM_ERR_INVALID", "OM_ERR_DEVICE", "OM_ERR_STATE", "OM_ERR_UNSUPPORTED", "OM_ERR_NOMEM",
         "OM_ABI_VERSION"]


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    d = tmp_path_factory.mktemp("abi")
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "ottomarcher.h"', "int main(void) {"]
    for s, fields in STRUCTS.items():
        lines.append(f'printf("{s} size %zu\\n", sizeof({s}));')
        for f in fields:
            lines.append(f'printf("{s}.{f} %zu\\n", offsetof({s}, {f}));')
    for e in ENUMS:
        lines.append(f'printf("{e} %d\\n", (int)({e}));')
    lines += ["return 0; }"]
    src = d / "abi.c"
    src.write_text("\n".join(lines))
    exe = d / "abi"
    subprocess.check_call([cc, "-std=c99", "-Wall", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    out = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        k, *rest = line.split()
        out[k if not rest[0].isalpha() else f"{k} {rest[0]}"] = int(rest[-1])
    return out


def test_ctypes_structs_match_header(om, c_layout):
    from raytracingoneweekend_amd import _lib
    for s, fields in STRUCTS.items():
        if s == "om_pixel_stats":
            continue
        cls = getattr(_lib, s)
        assert C.sizeof(cls) == c_layout[f"{s} size"], s
        for f in fields:
            assert getattr(cls, f).offset == c_layout[f"{s}.{f}"], f"{s}.{f}"


def test_pixel_stats_dtype_matches_header(om, c_layout):
    from raytracingoneweekend_amd import _lib
    dt = _lib.PIXEL_STATS_DTYPE
    assert dt.itemsize == c_layout["om_pixel_stats size"]
    for f in STRUCTS["om_pixel_stats"]:
        assert dt.fields[f][1] == c_layout[f"om_pixel_stats.{f}"], f


def test_enum_values_match_binding(om, c_layout):
    from raytracingoneweekend_amd import _lib
    assert c_layout["OM_ABI_VERSION"] == _lib.lib.om_abi_version()
    for i, k in enumerate(_lib.KT_CLASSES):
        assert c_layout[f"OM_KT_{k.upper()}"] == i
    assert c_layout["OM_KT_N"] == len(_lib.KT_CLASSES)
    kernels = {"auto": "OM_KERNEL_AUTO", "brute": "OM_KERNEL_BRUTE", "culled": "OM_KERNEL_CULLED",
               "bvh": "OM_KERNEL_BVH", "sbvh": "OM_KERNEL_SBVH", "bvh2": "OM_KERNEL_BVH2",
               "bvh4": "OM_KERNEL_BVH4"}
    for name, const in kernels.items():
        assert _lib.KERNELS[name] == c_layout[const], name
    assert _lib.PIPELINES["megakernel"] == c_layout["OM_PIPELINE_MEGAKERNEL"]
    assert _lib.PIPELINES["wavefront"] == c_layout["OM_PIPELINE_WAVEFRONT"]
    assert _lib.PIPELINES["auto"] == c_layout["OM_PIPELINE_AUTO"]
    assert np.array_equal([c_layout[k] for k in ("OM_LAMBERTIAN", "OM_METAL", "OM_DIELECTRIC")], [0, 1, 2])
