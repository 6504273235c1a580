"""Python mirror of the reference's scene/render API, driving the HIP hot path.

Names and argument meaning follow the Rust sources so a front-end reads the same:

    world = HittableList.new()
    world += Sphere.new_with_radius((0., -1000., 0.), 1000., Material.new_lambertian((0.5, 0.5, 0.5)))
    m = m4x4("TR", center) ^ m4x4("RX", a) ^ m4x4("SC", 0.2, 0.2, 0.2)       # main.rs:65-68
    world += Sphere.new(m, mat)
    camera = Camera.new(lookfrom, lookat, vup, 20., 3/2, 0.1, 10.)           # camera.rs:38
    frozen = world.freeze(camera)                                             # hits.rs:87-89
    pixels = PixelsBox.new(W * H)                                             # render_thread.rs:53-65
    render(camera, frozen, max_depth, 0.001, 100., spp, W, H, pixels)         # render_thread.rs:145

All arithmetic happens in libottomarcher.so (host f32 builders + HIP kernels);
this module only marshals arguments.
"""
import ctypes as C

import numpy as np

from . import _lib as L
from ._lib import check, f3, fptr, lib

__all__ = [
    "Material", "Mat4x4", "m4x4", "Camera", "Sphere", "Cube", "Triangle", "Parallelogram", "InfinitePlane",
    "MarchedSphere", "MarchedBox", "MarchedTorus", "MarchedSdf", "HittableList", "FrozenHittableList", "PixelsBox", "render",
    "RenderStats",
]


# ---------------------------------------------------------------- materials.rs
class Material:
    """materials.rs:18-38 — tagged union; constructors mirror Material::new_*."""

    def __init__(self, raw):
        self.raw = raw

    @staticmethod
    def new_lambertian(albedo):
        return Material(lib.om_material_lambertian(*[float(x) for x in albedo]))

    @staticmethod
    def new_metal(albedo):
        return Material(lib.om_material_metal(*[float(x) for x in albedo]))

    @staticmethod
    def new_metal_fuzz(albedo, fuzz):
        return Material(lib.om_material_metal_fuzz(*[float(x) for x in albedo], float(fuzz)))

    @staticmethod
    def new_dielectric(index_of_refraction):
        return Material(lib.om_material_dielectric(float(index_of_refraction)))

    @property
    def mat_type(self):
        return self.raw.type

    def __repr__(self):
        r = self.raw
        return f"Material(type={r.type}, albedo={tuple(r.albedo)}, fuzz={r.fuzz}, ior={r.ior})"


# ---------------------------------------------------------------- math/mat4x4.rs
class Mat4x4:
    """Row-major f32 4x4 (mat4x4.rs:8-10); `a ^ b` is dot_mat (mat4x4.rs:167-178)."""

    def __init__(self, values):
        self.m = L.F16(*[float(x) for x in values])

    @staticmethod
    def _out(fn, *args):
        out = L.F16()
        check(fn(*args, fptr(out)))
        return Mat4x4(list(out))

    @classmethod
    def identity(cls):
        return cls._out(lib.om_mat4_identity)

    @classmethod
    def new_translate(cls, v):
        return cls._out(lib.om_mat4_translate, fptr(f3(v)))

    @classmethod
    def new_scale(cls, v):
        return cls._out(lib.om_mat4_scale, fptr(f3(v)))

    @classmethod
    def new_rotate_x(cls, f):
        return cls._out(lib.om_mat4_rotate, 0, float(f))

    @classmethod
    def new_rotate_y(cls, f):
        return cls._out(lib.om_mat4_rotate, 1, float(f))

    @classmethod
    def new_rotate_z(cls, f):
        return cls._out(lib.om_mat4_rotate, 2, float(f))

    def dot_mat(self, other):
        return Mat4x4._out(lib.om_mat4_mul, fptr(self.m), fptr(other.m))

    def __xor__(self, other):
        return self.dot_mat(other)

    def fast_homogenous_inverse(self):
        return Mat4x4._out(lib.om_mat4_fast_homogenous_inverse, fptr(self.m))

    def to_numpy(self):
        return np.array(list(self.m), dtype=np.float32).reshape(4, 4)


def m4x4(kind="ID", *args):
    """The m4x4! macro (mat4x4.rs:181-209): RX/RY/RZ angle, TR x,y,z | TR v, SC x,y,z | SC v, ID."""
    if kind in ("ID", None):
        return Mat4x4.identity()
    if kind in ("RX", "RY", "RZ"):
        return {"RX": Mat4x4.new_rotate_x, "RY": Mat4x4.new_rotate_y, "RZ": Mat4x4.new_rotate_z}[kind](args[0])
    v = args[0] if len(args) == 1 else args
    if kind == "TR":
        return Mat4x4.new_translate(v)
    if kind == "SC":
        return Mat4x4.new_scale(v)
    raise ValueError(f"m4x4!: unknown kind {kind}")


# ---------------------------------------------------------------- camera.rs
class Camera:
    """camera.rs:10-59."""

    def __init__(self, raw):
        self.raw = raw

    @staticmethod
    def new(lookfrom, lookat, vup, vfov_in_degrees, aspect_ratio, aperture, focus_dist):
        raw = L.om_camera()
        check(lib.om_camera_new(fptr(f3(lookfrom)), fptr(f3(lookat)), fptr(f3(vup)), float(vfov_in_degrees),
                                float(aspect_ratio), float(aperture), float(focus_dist), C.byref(raw)))
        return Camera(raw)

    @staticmethod
    def world_camera(vfov_in_degrees, aspect_ratio):                                 # camera.rs:33-35
        return Camera.new((0., 0., 0.), (0., 0., -1.), (0., 1., 0.), vfov_in_degrees, aspect_ratio, 0., 1.)


# ---------------------------------------------------------------- traced.rs / marched.rs
class _Prim:
    def add_to(self, world_ptr):
        raise NotImplementedError


class Sphere(_Prim):
    """traced.rs:13-32 — unit sphere under an affine local_to_world (ellipsoid)."""

    def __init__(self, adder):
        self._adder = adder

    @staticmethod
    def new(m_local_to_world, mat):
        m = m_local_to_world
        return Sphere(lambda w: lib.om_world_add_sphere(w, fptr(m.m), C.byref(mat.raw)))

    @staticmethod
    def new_with_radius(o, r, mat):
        c = f3(o)
        return Sphere(lambda w: lib.om_world_add_sphere_radius(w, fptr(c), float(r), C.byref(mat.raw)))

    def add_to(self, w):
        return self._adder(w)


class Cube(Sphere):
    """traced.rs:229-247 — unit cube (half-extent 0.5) under an affine map."""

    @staticmethod
    def new(m_local_to_world, mat):
        m = m_local_to_world
        return Cube(lambda w: lib.om_world_add_cube(w, fptr(m.m), C.byref(mat.raw)))

    @staticmethod
    def new_with_length(o, length, mat):
        c = f3(o)
        return Cube(lambda w: lib.om_world_add_cube_length(w, fptr(c), float(length), C.byref(mat.raw)))


class Triangle(Sphere):
    """Barycentric<1> (traced.rs:118-226)."""

    _three = "om_world_add_triangle"
    _basis = "om_world_add_triangle_basis"

    @classmethod
    def new3points(cls, origin, upoint, vpoint, mat):
        a, b, c = f3(origin), f3(upoint), f3(vpoint)
        fn = getattr(lib, cls._three)
        return cls(lambda w: fn(w, fptr(a), fptr(b), fptr(c), C.byref(mat.raw)))

    @classmethod
    def new(cls, origin, u, v, u_length, v_length, mat):
        a, b, c = f3(origin), f3(u), f3(v)
        fn = getattr(lib, cls._basis)
        return cls(lambda w: fn(w, fptr(a), fptr(b), fptr(c), float(u_length), float(v_length), C.byref(mat.raw)))


class Parallelogram(Triangle):
    """Barycentric<0> (traced.rs:118-225)."""

    _three = "om_world_add_parallelogram"
    _basis = "om_world_add_parallelogram_basis"


class InfinitePlane(Sphere):
    """traced.rs:77-116."""

    @staticmethod
    def new(center, normal, material):
        a, b = f3(center), f3(normal)
        return InfinitePlane(lambda w: lib.om_world_add_plane(w, fptr(a), fptr(b), C.byref(material.raw)))


class MarchedSphere(Sphere):
    """marched.rs:50-76 (struct literal MarchedSphere{center, radius, material})."""

    def __init__(self, center, radius, material):
        c = f3(center)
        super().__init__(lambda w: lib.om_world_add_marched_sphere(w, fptr(c), float(radius), C.byref(material.raw)))


class MarchedBox(Sphere):
    """marched.rs:79-102 (struct literal MarchedBox{center, sizes, material})."""

    def __init__(self, center, sizes, material):
        c, s = f3(center), f3(sizes)
        super().__init__(lambda w: lib.om_world_add_marched_box(w, fptr(c), fptr(s), C.byref(material.raw)))


class MarchedTorus(Sphere):
    """marched.rs:105-151."""

    @staticmethod
    def new(m_local_to_world, local_sizes, mat):
        m, s = m_local_to_world, f3(local_sizes)
        return MarchedTorus(lambda w: lib.om_world_add_marched_torus(w, fptr(m.m), fptr(s), C.byref(mat.raw)))


class MarchedSdf(Sphere):
    """A user marched object, the device form of `HittableList += Arc<dyn Marched>` (hits.rs:96-100):
    an `impl Marched` whose local_sdf is a postfix program of om_sdf_op (include/ottomarcher.h),
    under MarchedTorus's transform and the trait's default normal (marched.rs:14-44, 139-151).

        MarchedSdf.new(m4x4("TR", 0, 1, 0), [("box", 0, 0, 0, .5, .5, .5), ("sphere", 0, 0, 0, .65),
                                             ("intersect",)], Material.new_metal((.8, .6, .2)))
    """

    @staticmethod
    def new(m_local_to_world, ops, mat):
        m, arr = m_local_to_world, L.sdf_ops(ops)
        return MarchedSdf(lambda w: lib.om_world_add_marched_sdf(w, fptr(m.m), arr.ctypes.data_as(C.c_void_p), arr.size,
                                                                C.byref(mat.raw)))


# ---------------------------------------------------------------- hits.rs
class HittableList:
    """hits.rs:37-110 — host-side list; `world += prim` appends in type order."""

    def __init__(self):
        self._w = C.c_void_p()
        check(lib.om_world_create(C.byref(self._w)))

    @staticmethod
    def new():
        return HittableList()

    def __del__(self):
        if getattr(self, "_w", None) and self._w.value:
            lib.om_world_destroy(self._w)
            self._w = C.c_void_p()

    @property
    def handle(self):
        return self._w

    def __iadd__(self, prim):
        if not isinstance(prim, _Prim):
            # Arc<dyn Traced> user types (hits.rs:91-95) cannot cross the C-ABI; a user marched
            # object is a MarchedSdf (an SDF program)
            raise TypeError("only the reference's primitive types and MarchedSdf can be added to a device world")
        check(prim.add_to(self._w))
        return self

    def clear(self):
        check(lib.om_world_clear(self._w))

    def counts(self):
        out = (C.c_uint32 * 8)()
        check(lib.om_world_counts(self._w, out))
        n = C.c_uint32()
        check(lib.om_world_marched_sdf_count(self._w, C.byref(n)))
        return dict(zip(["spheres", "cubes", "triangles", "infinite_planes", "parallelograms",
                         "marched_spheres", "marched_boxes", "marched_torus", "marched_sdf"], list(out) + [n.value]))

    def export(self, kind, index, n):
        out = (C.c_float * n)()
        check(lib.om_world_export(self._w, int(kind), int(index), fptr(out), n))
        return np.array(list(out), dtype=np.float32)

    def freeze(self, cam=None, device=0, kernel="auto", pipeline="auto"):
        """hits.rs:87-89: snapshot to device memory (the camera is unused: the camera hash is out of scope)."""
        return FrozenHittableList(self, device=device, kernel=kernel, pipeline=pipeline)


class FrozenHittableList:
    """hits.rs:63-69 — a world resident in HBM on one device (om_ctx)."""

    def __init__(self, world, device=0, kernel="auto", pipeline="auto"):
        self._ctx = C.c_void_p()
        check(lib.om_create(int(device), C.byref(self._ctx)))
        check(lib.om_upload_world(self._ctx, world.handle), self._ctx)
        self.set_kernel(kernel)
        self.set_pipeline(pipeline)
        self.device = device

    def set_pipeline(self, pipeline):
        check(lib.om_set_pipeline(self._ctx, L.PIPELINES[pipeline] if isinstance(pipeline, str) else int(pipeline)),
              self._ctx)

    def set_kernel(self, kernel):
        check(lib.om_set_kernel(self._ctx, L.KERNELS[kernel] if isinstance(kernel, str) else int(kernel)), self._ctx)

    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            lib.om_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        self.close()

    @property
    def ctx(self):
        return self._ctx

    def counters(self):
        c = L.om_counters()
        check(lib.om_get_counters(self._ctx, C.byref(c)), self._ctx)
        return {n: getattr(c, n) for n, _ in L.om_counters._fields_}


# ---------------------------------------------------------------- render_thread.rs
class PixelsBox:
    """The caller-owned framebuffer (render_thread.rs:42-65): W*H om_pixel_stats."""

    def __init__(self, image_size):
        self.pixels = np.zeros(int(image_size), dtype=L.PIXEL_STATS_DTYPE)
        self._pinned = None

    @staticmethod
    def new(image_size):
        return PixelsBox(image_size)

    def pin(self):
        """Page-lock the framebuffer (om_host_register) so render()'s copies run as DMA; kept
        until the box dies or `pixels` is replaced.  Best effort, like the C++ render(): a
        refused registration (memlock limit, an already registered buffer) leaves the buffer
        pageable, and the copies still work.  Done by render() on first use (needs a HIP device)."""
        if self._pinned is not None and self._pinned is not self.pixels:
            self.unpin()                                   # `pixels` was replaced: release the old one
        if self._pinned is None and self.pixels.nbytes:
            if lib.om_host_register(self.pixels.ctypes.data, self.pixels.nbytes) == L.OM_OK:
                self._pinned = self.pixels                 # a reference: the array cannot be freed while registered
        return self

    def unpin(self):
        if getattr(self, "_pinned", None) is not None:
            lib.om_host_unregister(self._pinned.ctypes.data)
            self._pinned = None

    def __del__(self):
        self.unpin()


def make_params(max_depth, tmin, tmax, samples_per_pixel, image_width, image_height, sample_count=None,
                seed=1, march_steps=1024, adaptive=False, sample_begin=0):
    p = L.om_render_params()
    p.width, p.height = int(image_width), int(image_height)
    p.spp_total = int(samples_per_pixel)
    p.sample_begin = int(sample_begin)
    p.sample_count = int(samples_per_pixel if sample_count is None else sample_count)
    p.max_depth = int(max_depth)
    p.tmin, p.tmax = float(tmin), float(tmax)
    p.march_steps = int(march_steps)
    p.adaptive = 1 if adaptive else 0
    p.seed = int(seed)
    return p


class RenderStats(dict):
    pass


def render(camera, world, max_depth, tmin, tmax, samples_per_pixel, image_width, image_height, pixels_box,
           tid=0, assigned_thread=None, samples_atom=None, *, seed=1, march_steps=1024, adaptive=True,
           sample_count=None):
    """render_thread::render (render_thread.rs:145-202) for the whole frame.

    `adaptive` defaults to True, as the reference always retires a pixel once bad_avgs
    reaches 5 (ThreadPixels::add_run, render_thread.rs:97-101,195-198) and credits its
    untaken samples to samples_atom; pass adaptive=False for a fixed-spp render (the
    BASELINE metric).

    The reference spawns num_cpus-1 threads with disjoint pixel sets (main.rs:200-214);
    here tid 0 renders every pixel on the device and other tids return at once, so a
    front-end that still spawns threads stays correct.  `samples_atom`, if given, is a
    one-element list incremented by the credited samples (render_thread.rs:196-198).
    """
    if tid != 0:
        return None
    p = make_params(max_depth, tmin, tmax, samples_per_pixel, image_width, image_height,
                    sample_count=sample_count, seed=seed, march_steps=march_steps, adaptive=adaptive)
    buf = pixels_box.pixels if isinstance(pixels_box, PixelsBox) else pixels_box
    if buf.dtype != L.PIXEL_STATS_DTYPE or buf.size != p.width * p.height or not buf.flags["C_CONTIGUOUS"]:
        raise ValueError("pixels must be a contiguous W*H om_pixel_stats array")
    if isinstance(pixels_box, PixelsBox) and p.width * p.height > 0:
        pixels_box.pin()
    ctr = L.om_counters()
    check(lib.om_render(world.ctx, C.byref(camera.raw), C.byref(p), buf.ctypes.data_as(C.c_void_p), C.byref(ctr)),
          world.ctx)
    out = RenderStats({n: getattr(ctr, n) for n, _ in L.om_counters._fields_})
    if samples_atom is not None:
        samples_atom[0] += out["credited"]
    return out


# ---------------------------------------------------------------- main.rs draw_to_sdl
def display(frozen, pixels_box, image_width, image_height, view="normal", rgb=None):
    """One draw_to_sdl view (main.rs:360-437) of the framebuffer, computed on the device
    of `frozen` -> (H, W, 3) uint8 RGB.  `view`: a name of _lib.VIEWS or 0-6 (the
    reference's keypad modes).  Pass the previous `rgb` to keep the reference's
    behaviour for pixels its box filter never visits (W or H == 2)."""
    st = pixels_box.pixels if isinstance(pixels_box, PixelsBox) else pixels_box
    st = np.ascontiguousarray(st)
    W, H = int(image_width), int(image_height)
    if st.dtype != L.PIXEL_STATS_DTYPE or st.size != W * H:
        raise ValueError("display: need W*H om_pixel_stats")
    mode = L.VIEWS.index(view) if isinstance(view, str) else int(view)
    out = np.zeros(W * H * 3, dtype=np.uint8) if rgb is None else np.ascontiguousarray(rgb, dtype=np.uint8).reshape(-1).copy()
    check(lib.om_display(frozen.ctx, st.ctypes.data, W, H, mode, out.ctypes.data), frozen.ctx)
    return out.reshape(H, W, 3)


def write_bmp(path, rgb):
    """24-bit BMP of an (H, W, 3) uint8 image (the F12 save, main.rs:473-476)."""
    a = np.ascontiguousarray(rgb, dtype=np.uint8)
    check(lib.om_write_bmp(str(path).encode(), a.ctypes.data, a.shape[1], a.shape[0]))


def write_ppm(path, rgb):
    """Binary PPM (P6) of an (H, W, 3) uint8 image."""
    a = np.ascontiguousarray(rgb, dtype=np.uint8)
    check(lib.om_write_ppm(str(path).encode(), a.ctypes.data, a.shape[1], a.shape[0]))
