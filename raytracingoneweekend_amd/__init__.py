"""raytracingoneweekend_amd — MI355X-native drop-in for the per-pixel ray_color hot path
of octaviogarcia/RaytracingOneWeekend ("ottomarcher").

The product is libottomarcher.so (include/ottomarcher.h): host f32 scene builders +
hand-written HIP kernels for gfx950.  This package is the Python mirror of the
reference's Camera / Material / HittableList / render API over that C-ABI.
"""
from . import _lib
from .api import (Camera, Cube, FrozenHittableList, HittableList, InfinitePlane, MarchedBox, MarchedSdf,
                  MarchedSphere, MarchedTorus, Mat4x4, Material, Parallelogram, PixelsBox, Sphere, Triangle, display, m4x4,
                  make_params, render, write_bmp, write_ppm)
from .scenes import basic_scene, default_camera, marched_scene, random_scene, random_scene_api

PIXEL_STATS_DTYPE = _lib.PIXEL_STATS_DTYPE
__version__ = "0.1.0"
