"""Front-end scene builders of main.rs, over the mirrored API.

`random_scene` (main.rs:37-100) has two equivalent builders:
  * random_scene(seed)     -> the native builder om_world_random_scene (fast; 10k variant too)
  * random_scene_api(seed) -> the same scene composed through the Python mirror of the
                              reference API (Material / m4x4 / Sphere.new / `world +=`),
                              exactly as main.rs writes it; tests assert both agree bit for bit.
Both draw from om-rng's SplitMix64 host stream in the reference's draw order.
"""
import numpy as np

from . import _lib as L
from ._lib import check, lib
from .api import (Camera, HittableList, Material, MarchedTorus, Parallelogram, Sphere, Triangle, Cube, m4x4)

F = np.float32
PI = F(3.1415926535897932385)  # utils.rs:29

# scene variants
S_TRACED = 0          # random_scene minus the torus block — configs C0/C1/C4
S_FULL = 1            # random_scene exactly as main.rs:37-100 (torus included)


class SplitMix64:
    """om-rng host stream (SplitMix64) (replaces rand::thread_rng, utils.rs:25)."""

    M = (1 << 64) - 1

    def __init__(self, state):
        self.s = state & self.M

    def next_u64(self):
        self.s = (self.s + 0x9E3779B97F4A7C15) & self.M
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & self.M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & self.M
        return z ^ (z >> 31)

    def rand(self):                                        # f32::rand  utils.rs:25
        return F(self.next_u64() >> 40) * F(5.9604644775390625e-8)

    def rand_range(self, lo, hi):                          # utils.rs:26
        r = self.rand()
        return r * (F(hi) - F(lo)) + F(lo)


def random_scene(seed=0x5EED, with_torus=False, grid_half=11, extras=True):
    """main.rs:37-100 via the native builder.  grid_half=50 gives the ~10k-sphere variant (config C3)."""
    w = HittableList.new()
    flags = (1 if with_torus else 0) | (0 if extras else 2)
    check(lib.om_world_random_scene(w.handle, int(seed), flags, int(grid_half)))
    return w


def basic_scene():
    """main.rs:103-110."""
    w = HittableList.new()
    check(lib.om_world_basic_scene(w.handle))
    return w


def marched_scene():
    """SDF scene of config C2: marched ground, box, sphere and random_scene's torus."""
    w = HittableList.new()
    check(lib.om_world_marched_scene(w.handle))
    return w


def random_scene_api(seed=0x5EED, with_torus=False, grid_half=11, extras=True):
    """main.rs:37-100 written against the mirrored API, statement for statement."""
    g = SplitMix64(seed)
    world = HittableList.new()
    mat_ground = Material.new_lambertian((0.5, 0.5, 0.5))
    world += Sphere.new_with_radius((0., -1000., 0.), 1000.0, mat_ground)
    for a in range(-grid_half, grid_half):
        af = F(a)
        for b in range(-grid_half, grid_half):
            bf = F(b)
            cx = af + F(0.9) * g.rand()
            cz = bf + F(0.9) * g.rand()
            center = (cx, F(0.2), cz)
            d = [center[0] - F(4.), center[1] - F(0.2), center[2] - F(0.)]
            length = np.sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2], dtype=F)
            if length > F(0.9):
                mat_prob = g.rand()
                if mat_prob < F(0.8):
                    c1 = (g.rand(), g.rand(), g.rand())
                    c2 = (g.rand(), g.rand(), g.rand())
                    sphere_mat = Material.new_lambertian(tuple(c1[i] * c2[i] for i in range(3)))
                elif mat_prob < F(0.95):
                    albedo = (g.rand_range(0.5, 1.), g.rand_range(0.5, 1.), g.rand_range(0.5, 1.))
                    fuzz = g.rand_range(0., 0.5)
                    sphere_mat = Material.new_metal_fuzz(albedo, fuzz)
                else:
                    sphere_mat = Material.new_dielectric(1.5)
                m = m4x4("TR", center) \
                    ^ m4x4("RX", g.rand() * F(2.) * PI) ^ m4x4("RY", g.rand() * F(2.) * PI) ^ m4x4("RZ", g.rand() * F(2.) * PI) \
                    ^ m4x4("SC", g.rand() + F(1.), g.rand() + F(1.), g.rand() + F(1.)) \
                    ^ m4x4("SC", 0.2, 0.2, 0.2)
                world += Sphere.new(m, sphere_mat)
    if with_torus:
        mat = Material.new_dielectric(1.5)
        local_to_world = m4x4("TR", 0., 1., 0.) ^ m4x4("RX", 0.6) ^ m4x4("RZ", F(1.33) * F(2.) * PI)
        world += MarchedTorus.new(local_to_world, (0.5, 0.1, 0.1), mat)
    if extras:
        p1 = (F(7.), F(1.), F(0.))
        p2 = (F(6.), F(1.1), F(0.5))
        p3 = (F(6.), F(1.5), F(0.))
        world += Parallelogram.new3points(p1, p2, p3, Material.new_metal((1., 0.5, 1.)))
        world += Triangle.new3points((p1[0] + F(0.), p1[1] + F(0.5), p1[2] + F(0.)), p2, p3,
                                     Material.new_lambertian((1., 1., 0.)))
        mat = Material.new_metal((0.7, 0.6, 0.5))
        m = m4x4("TR", 4., 1., 0.) ^ m4x4("RX", g.rand() * F(2.) * PI) ^ m4x4("RY", g.rand() * F(2.) * PI) \
            ^ m4x4("RZ", g.rand() * F(2.) * PI)
        world += Cube.new(m, mat)
    return world


def default_camera(aspect_ratio):
    """main.rs:136-142: lookfrom (13,2,3), lookat 0, vup +y, vfov 20, aperture 0.1, focus 10."""
    return Camera.new((13., 2., 3.), (0., 0., 0.), (0., 1., 0.), 20., aspect_ratio, 0.1, 10.)
