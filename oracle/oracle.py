"""ctypes wrapper of liboro.so — the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker / the timed CPU baseline.  The product
(raytracingoneweekend_amd/) never loads it.  Parity status: "parity unpinned" —
see om_oracle.cpp's header and DESIGN.md §3.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ORO_LIB: another build of the same restatement (liboro_v3.so: the x86-64-v3 CPU baseline)
LIB = os.path.join(HERE, os.environ.get("ORO_LIB", "liboro.so"))

PIXEL_STATS_DTYPE = np.dtype([("bloom", "<u8"), ("sum", "<f4", (3,)), ("n", "<u4"), ("avg_depth", "<f4"),
                              ("bad_avgs", "<u4"), ("color", "u1", (3,)), ("flags", "u1"), ("reserved", "<u4")])


class OroMaterial(C.Structure):
    _fields_ = [("albedo", C.c_float * 3), ("fuzz", C.c_float), ("ior", C.c_float), ("type", C.c_int32)]


class OroCamera(C.Structure):
    _fields_ = [(n, C.c_float * 3) for n in ("origin", "horizontal", "vertical", "llc", "u", "v", "w")] + \
               [(n, C.c_float) for n in ("lens_radius", "aspect", "focus", "vw", "vh")]


class OroParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("width", "height", "spp_total", "sample_begin", "sample_count", "max_depth")] + \
               [("tmin", C.c_float), ("tmax", C.c_float), ("march_steps", C.c_uint32), ("adaptive", C.c_uint32),
                ("seed", C.c_uint64)]


def build():
    """Compile liboro.so (gcc, -ffp-contract=off) if it is missing or stale."""
    src = os.path.join(HERE, "om_oracle.cpp")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-C", HERE, os.path.basename(LIB)], stdout=subprocess.DEVNULL)


def _load():
    build()
    lib = C.CDLL(LIB)
    vp, fp = C.c_void_p, C.POINTER(C.c_float)
    mp = C.POINTER(OroMaterial)
    sig = {
        "oro_world_new": (vp, []), "oro_world_free": (None, [vp]),
        "oro_world_add_sphere": (None, [vp, fp, mp]), "oro_world_add_sphere_radius": (None, [vp, fp, C.c_float, mp]),
        "oro_world_add_cube": (None, [vp, fp, mp]), "oro_world_add_cube_length": (None, [vp, fp, C.c_float, mp]),
        "oro_world_add_bary3": (None, [vp, C.c_int, fp, fp, fp, mp]),
        "oro_world_add_bary": (None, [vp, C.c_int, fp, fp, fp, C.c_float, C.c_float, mp]),
        "oro_world_add_plane": (None, [vp, fp, fp, mp]),
        "oro_world_add_marched_sphere": (None, [vp, fp, C.c_float, mp]),
        "oro_world_add_marched_box": (None, [vp, fp, fp, mp]),
        "oro_world_add_marched_torus": (None, [vp, fp, fp, mp]),
        "oro_world_add_marched_sdf": (None, [vp, fp, vp, C.c_uint32, mp]),
        "oro_world_counts": (None, [vp, C.POINTER(C.c_uint32)]),
        "oro_world_affine": (None, [vp, C.c_int, C.c_uint32, fp]),
        "oro_world_bary": (None, [vp, C.c_int, C.c_uint32, fp]),
        "oro_world_torus": (None, [vp, C.c_uint32, fp]),
        "oro_world_random_scene": (None, [vp, C.c_uint64, C.c_uint32, C.c_int32]),
        "oro_world_marched_scene": (None, [vp]),
        "oro_camera_new": (None, [fp, fp, fp, C.c_float, C.c_float, C.c_float, C.c_float, C.POINTER(OroCamera)]),
        "oro_rng_draws": (None, [C.c_uint64, C.c_uint32, fp]),
        "oro_rng_path_draws": (None, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, fp]),
        "oro_jitter_table": (None, [C.c_uint64, C.c_uint32, fp]),
        "oro_bloom_hash": (C.c_uint64, [C.c_uint64]), "oro_scramble": (C.c_uint64, [C.c_uint64]),
        "oro_display": (None, [vp, C.c_uint32, C.c_uint32, C.c_int32, vp]),
        "oro_hit_world": (C.c_int, [vp, fp, C.c_float, C.c_float, fp, C.POINTER(C.c_uint64)]),
        "oro_scatter": (None, [fp, fp, mp, C.c_uint64, fp, C.POINTER(C.c_uint64)]),
        "oro_get_ray": (None, [C.POINTER(OroCamera), C.c_float, C.c_float, C.c_uint64, fp]),
        "oro_stats_add": (None, [vp, fp, C.c_float, C.c_uint64]),
        "oro_marched_sdf": (C.c_float, [vp, C.c_int, C.c_uint32, fp]),
        "oro_marched_normal": (None, [vp, C.c_int, C.c_uint32, fp, fp]),
        "oro_render": (None, [vp, C.POINTER(OroCamera), C.POINTER(OroParams), vp, C.c_int32, C.POINTER(C.c_uint64)]),
        "oro_render_pixels": (None, [vp, C.POINTER(OroCamera), C.POINTER(OroParams), vp, C.POINTER(C.c_uint32),
                                     C.c_uint32]),
        "oro_render_pixels_mt": (None, [vp, C.POINTER(OroCamera), C.POINTER(OroParams), vp, C.POINTER(C.c_uint32),
                                        C.c_uint32, C.c_int32]),
    }
    for n, (r, a) in sig.items():
        f = getattr(lib, n)
        f.restype = r
        f.argtypes = a
    return lib


lib = _load()


def f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


def fp(a):
    return C.cast(a, C.POINTER(C.c_float))


def material(kind, albedo=(0., 0., 0.), fuzz=0., ior=0.):
    m = OroMaterial()
    m.albedo[:] = [float(x) for x in albedo]
    m.fuzz, m.ior = float(fuzz), float(ior)
    m.type = {"lambertian": 0, "metal": 1, "dielectric": 2}[kind] if isinstance(kind, str) else int(kind)
    return m


SDF_OP_DTYPE = np.dtype([("op", "<i4"), ("a", "<f4", 7)])   # om_sdf_op (include/ottomarcher.h)
SDF_OPS = {"sphere": 1, "box": 2, "torus": 3, "union": 4, "intersect": 5, "subtract": 6, "round": 7}


def sdf_ops(ops):
    """[(name or code, param, ...), ...] -> om_sdf_op records."""
    arr = np.zeros(len(ops), dtype=SDF_OP_DTYPE)
    for i, o in enumerate(ops):
        arr[i]["op"] = SDF_OPS.get(o[0], o[0]) if isinstance(o[0], str) else o[0]
        arr[i]["a"][:len(o) - 1] = o[1:]
    return arr


class World:
    """HittableList restated on the CPU (hits.rs)."""

    def __init__(self):
        self.h = C.c_void_p(lib.oro_world_new())

    def __del__(self):
        if getattr(self, "h", None) and self.h.value:
            lib.oro_world_free(self.h)
            self.h = C.c_void_p()

    def add_sphere(self, l2w, m):
        lib.oro_world_add_sphere(self.h, fp((C.c_float * 16)(*map(float, np.ravel(l2w)))), C.byref(m))

    def add_sphere_radius(self, c, r, m):
        lib.oro_world_add_sphere_radius(self.h, fp(f3(c)), float(r), C.byref(m))

    def add_cube(self, l2w, m):
        lib.oro_world_add_cube(self.h, fp((C.c_float * 16)(*map(float, np.ravel(l2w)))), C.byref(m))

    def add_cube_length(self, c, length, m):
        lib.oro_world_add_cube_length(self.h, fp(f3(c)), float(length), C.byref(m))

    def add_triangle(self, o, up, vp, m):
        lib.oro_world_add_bary3(self.h, 1, fp(f3(o)), fp(f3(up)), fp(f3(vp)), C.byref(m))

    def add_parallelogram(self, o, up, vp, m):
        lib.oro_world_add_bary3(self.h, 0, fp(f3(o)), fp(f3(up)), fp(f3(vp)), C.byref(m))

    def add_plane(self, c, n, m):
        lib.oro_world_add_plane(self.h, fp(f3(c)), fp(f3(n)), C.byref(m))

    def add_marched_sphere(self, c, r, m):
        lib.oro_world_add_marched_sphere(self.h, fp(f3(c)), float(r), C.byref(m))

    def add_marched_box(self, c, s, m):
        lib.oro_world_add_marched_box(self.h, fp(f3(c)), fp(f3(s)), C.byref(m))

    def add_marched_torus(self, l2w, s, m):
        lib.oro_world_add_marched_torus(self.h, fp((C.c_float * 16)(*map(float, np.ravel(l2w)))), fp(f3(s)), C.byref(m))

    def add_marched_sdf(self, l2w, ops, m):
        """A user marched object (Arc<dyn Marched>): `ops` = [(op, params...), ...] as om_sdf_op."""
        arr = sdf_ops(ops)
        lib.oro_world_add_marched_sdf(self.h, fp((C.c_float * 16)(*map(float, np.ravel(l2w)))),
                                      arr.ctypes.data_as(C.c_void_p), arr.size, C.byref(m))
        self.n_sdf = getattr(self, "n_sdf", 0) + 1

    def counts(self):
        """The eight typed counts (hits.rs:370-371), then the user marched objects."""
        out = (C.c_uint32 * 8)()
        lib.oro_world_counts(self.h, out)
        return list(out) + [getattr(self, "n_sdf", 0)]

    def affine(self, kind, i):
        out = (C.c_float * 32)()
        lib.oro_world_affine(self.h, kind, i, fp(out))
        return np.array(list(out), dtype=np.float32)

    def bary(self, kind, i):
        out = (C.c_float * 29)()
        lib.oro_world_bary(self.h, kind, i, fp(out))
        return np.array(list(out), dtype=np.float32)

    def torus(self, i):
        out = (C.c_float * 43)()
        lib.oro_world_torus(self.h, i, fp(out))
        return np.array(list(out), dtype=np.float32)

    def hit(self, orig, direction, tmin=0.001, tmax=100.0):
        ray = (C.c_float * 6)(*map(float, list(orig) + list(direction)))
        out = (C.c_float * 7)()
        oid = C.c_uint64()
        h = lib.oro_hit_world(self.h, fp(ray), float(tmin), float(tmax), fp(out), C.byref(oid))
        return (np.array(list(out), dtype=np.float32), oid.value) if h else None


def random_scene(seed=0x5EED, with_torus=False, grid_half=11, extras=True):
    w = World()
    lib.oro_world_random_scene(w.h, int(seed), (1 if with_torus else 0) | (0 if extras else 2), int(grid_half))
    return w


def marched_scene():
    w = World()
    lib.oro_world_marched_scene(w.h)
    return w


def camera(lookfrom, lookat, vup, vfov, aspect, aperture, focus):
    c = OroCamera()
    lib.oro_camera_new(fp(f3(lookfrom)), fp(f3(lookat)), fp(f3(vup)), float(vfov), float(aspect), float(aperture),
                       float(focus), C.byref(c))
    return c


def default_camera(aspect):
    return camera((13., 2., 3.), (0., 0., 0.), (0., 1., 0.), 20., aspect, 0.1, 10.)


def params(width, height, spp_total, sample_count=None, max_depth=50, tmin=0.001, tmax=100.0, march_steps=1024,
           adaptive=False, seed=1):
    p = OroParams()
    p.width, p.height, p.spp_total = int(width), int(height), int(spp_total)
    p.sample_begin = 0
    p.sample_count = int(spp_total if sample_count is None else sample_count)
    p.max_depth = int(max_depth)
    p.tmin, p.tmax = float(tmin), float(tmax)
    p.march_steps, p.adaptive, p.seed = int(march_steps), 1 if adaptive else 0, int(seed)
    return p


def render(world, cam, p, stats=None, nthreads=0):
    """render_thread::render over all threads (main.rs:170-214); returns (stats, counters)."""
    if stats is None:
        stats = np.zeros(p.width * p.height, dtype=PIXEL_STATS_DTYPE)
    ctr = (C.c_uint64 * 3)()
    lib.oro_render(world.h, C.byref(cam), C.byref(p), stats.ctypes.data_as(C.c_void_p), int(nthreads), ctr)
    return stats, {"samples": ctr[0], "segments": ctr[1], "credited": ctr[2]}


def render_pixels(world, cam, p, pixels, nthreads=1):
    """Render only `pixels` (uint32 row-major indices); returns compact stats[len(pixels)].
    nthreads > 1 (0 = every hardware thread) spreads the pixels over workers: same bits."""
    pixels = np.ascontiguousarray(pixels, dtype=np.uint32)
    stats = np.zeros(pixels.size, dtype=PIXEL_STATS_DTYPE)
    if nthreads == 1:
        lib.oro_render_pixels(world.h, C.byref(cam), C.byref(p), stats.ctypes.data_as(C.c_void_p),
                              pixels.ctypes.data_as(C.POINTER(C.c_uint32)), pixels.size)
    else:
        lib.oro_render_pixels_mt(world.h, C.byref(cam), C.byref(p), stats.ctypes.data_as(C.c_void_p),
                                 pixels.ctypes.data_as(C.POINTER(C.c_uint32)), pixels.size, int(nthreads))
    return stats


def window_pixels(W, H, x0, y0, size):
    """Row-major indices of the size x size window at (x0, y0)."""
    ys, xs = np.meshgrid(np.arange(y0, y0 + size), np.arange(x0, x0 + size), indexing="ij")
    return (ys * W + xs).reshape(-1).astype(np.uint32)


def rng_draws(state, n):
    out = (C.c_float * n)()
    lib.oro_rng_draws(C.c_uint64(state), n, fp(out))
    return np.array(list(out), dtype=np.float32)


def path_draws(seed, pixel, sample, n):
    out = (C.c_float * n)()
    lib.oro_rng_path_draws(C.c_uint64(seed), pixel, sample, n, fp(out))
    return np.array(list(out), dtype=np.float32)


def jitter_table(seed, spp):
    out = (C.c_float * (2 * spp))()
    lib.oro_jitter_table(C.c_uint64(seed), spp, fp(out))
    return np.array(list(out), dtype=np.float32).reshape(spp, 2)


def bloom_hash(i):
    return lib.oro_bloom_hash(C.c_uint64(i))


def scramble(i):
    return lib.oro_scramble(C.c_uint64(i))


def display(stats, W, H, mode, rgb=None):
    """draw_to_sdl view `mode` (main.rs:360-437) of a W*H PIXEL_STATS_DTYPE array -> (H, W, 3) uint8.
    `rgb` (H*W*3 uint8) is updated in place, like the reference's persistent sdlpixels buffer."""
    st = np.ascontiguousarray(stats)
    assert st.dtype == PIXEL_STATS_DTYPE and st.size == W * H
    out = np.zeros(W * H * 3, dtype=np.uint8) if rgb is None else rgb.reshape(-1)
    lib.oro_display(st.ctypes.data, W, H, mode, out.ctypes.data)
    return out.reshape(H, W, 3)
