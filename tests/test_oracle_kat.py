"""Analytic known-answer tests that pin the CPU oracle (the reference ships no tests or
golden vectors, SURVEY.md §4, so closed forms are what anchor the restatement)."""
import ctypes as C
import math

import numpy as np
import pytest

F = np.float32


def test_splitmix64_known_outputs(oracle):
    # SplitMix64 from state 0: the published first outputs 0xe220a8397b1dcdaf, 0x6e789e6aa1b965f4
    d = oracle.rng_draws(0, 2)
    assert d[0] == F((0xE220A8397B1DCDAF >> 40) / 2 ** 24)
    assert d[1] == F((0x6E789E6AA1B965F4 >> 40) / 2 ** 24)


def test_rng_matches_product_python_stream(oracle):
    from raytracingoneweekend_amd.scenes import SplitMix64
    g = SplitMix64(0x5EED)
    assert np.array_equal(oracle.rng_draws(0x5EED, 50), np.array([g.rand() for _ in range(50)], dtype=F))


def _path_draws_py(seed, pixel, sample, n):
    """om-rng v2 path stream restated in Python."""
    M = (1 << 64) - 1

    def mix64(z):
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    skey = mix64((seed + 0x632BE59BD9B4E019) & M)
    return _path_state_draws_py(mix64(((pixel << 32) | sample) ^ skey), n)


def _path_state_draws_py(state, n):
    s, k = state & 0xFFFFFFFF, state >> 32
    out = []
    for _ in range(n):
        s = (s + 0x9E3779B9) & 0xFFFFFFFF
        x = s ^ k
        x ^= x >> 16
        x = (x * 0x21F0AAAD) & 0xFFFFFFFF
        x ^= x >> 15
        x = (x * 0x735A2D97) & 0xFFFFFFFF
        x ^= x >> 15
        out.append((x >> 8) / 2 ** 24)
    return np.array(out, dtype=F)


@pytest.mark.parametrize("seed,pixel,sample", [(1, 0, 0), (1, 12345, 7), (0x5EED, 2073599, 511), (2 ** 63, 7, 2 ** 31)])
def test_path_stream_matches_python_restatement(oracle, seed, pixel, sample):
    assert np.array_equal(oracle.path_draws(seed, pixel, sample, 64), _path_draws_py(seed, pixel, sample, 64))


def test_path_stream_uniformity(oracle):
    d = np.concatenate([oracle.path_draws(1, p, s, 16) for p in range(64) for s in range(16)]).astype(np.float64)
    assert np.all(d * 2 ** 24 == np.floor(d * 2 ** 24)) and (d >= 0).all() and (d < 1).all()
    assert abs(d.mean() - 0.5) < 0.01
    hist, _ = np.histogram(d, bins=16, range=(0, 1))
    assert hist.min() > 0.85 * d.size / 16


def test_draws_on_24bit_grid(oracle):
    d = oracle.rng_draws(12345, 4096).astype(np.float64)
    assert (d >= 0).all() and (d < 1).all()
    assert np.all(d * 2 ** 24 == np.floor(d * 2 ** 24))
    assert abs(d.mean() - 0.5) < 0.02


def test_jitter_table_is_a_permutation_of_strata(oracle):
    # render_thread.rs:164-174: ((s/2)&1, s&1) then shuffled
    jt = oracle.jitter_table(1, 16)
    ref = sorted([(float((s // 2) & 1), float(s & 1)) for s in range(16)])
    assert sorted(map(tuple, jt.tolist())) == ref


def _lam(O, c=(0.5, 0.5, 0.5)):
    return O.material("lambertian", c)


def test_unit_sphere_hit(oracle):
    w = oracle.World()
    w.add_sphere_radius((0., 0., -5.), 1., _lam(oracle))
    out, oid = w.hit((0., 0., 0.), (0., 0., -1.))
    assert out[0] == 4.0                                             # t = |c| - r, exact
    assert tuple(out[1:4]) == (0., 0., -4.)
    assert tuple(out[4:7]) == (0., 0., 1.)
    assert oid == 1
    assert w.hit((0., 0., 0.), (0., 1., 0.)) is None                 # miss
    assert w.hit((0., 0., -5.), (0., 0., -1.), 0.001, 100.)[0][0] == 1.0  # inside: far root


def test_ellipsoid_hit_and_reference_normal(oracle):
    w = oracle.World()
    l2w = np.diag([2., 1., 1., 1.]).astype(F)
    w.add_sphere(l2w, _lam(oracle))
    out, _ = w.hit((-10., 0., 0.), (1., 0., 0.))
    assert out[0] == 8.0
    assert tuple(out[4:7]) == (-1., 0., 0.)


def test_cube_face_normal(oracle):
    w = oracle.World()
    w.add_cube_length((0., 0., -3.), 1., oracle.material("metal", (1, 1, 1)))
    out, _ = w.hit((0., 0., 0.), (0., 0., -1.))
    assert out[0] == 2.5
    assert tuple(out[4:7]) == (0., 0., 1.)
    out, _ = w.hit((5., 0., -3.), (-1., 0., 0.))
    assert out[0] == 4.5 and tuple(out[4:7]) == (1., 0., 0.)


def test_barycentric_inside_outside(oracle):
    w = oracle.World()
    w.add_triangle((0., 0., -2.), (1., 0., -2.), (0., 1., -2.), _lam(oracle))
    out, _ = w.hit((0.25, 0.25, 0.), (0., 0., -1.))
    assert out[0] == 2.0 and tuple(out[4:7]) == (0., 0., 1.)
    assert w.hit((0.75, 0.75, 0.), (0., 0., -1.)) is None           # lambda3 < 0
    p = oracle.World()
    p.add_parallelogram((0., 0., -2.), (1., 0., -2.), (0., 1., -2.), _lam(oracle))
    assert p.hit((0.75, 0.75, 0.), (0., 0., -1.))[0][0] == 2.0
    assert p.hit((1.25, 0.5, 0.), (0., 0., -1.)) is None


def test_plane_hit_normal_against_direction(oracle):
    w = oracle.World()
    w.add_plane((0., -1., 0.), (0., 1., 0.), _lam(oracle))
    out, _ = w.hit((0., 0., 0.), (0., -1., 0.))
    assert out[0] == 1.0 and tuple(out[4:7]) == (0., 1., 0.)
    out, _ = w.hit((0., -2., 0.), (0., 1., 0.))                      # from below: normal flips
    assert out[0] == 1.0 and tuple(out[4:7]) == (0., -1., 0.)
    assert w.hit((0., 0., 0.), (1., 0., 0.)) is None                 # parallel


def test_later_object_wins_ties(oracle):
    # hits.rs:274-285 with traced.rs:51: root == closest is accepted -> later object wins
    w = oracle.World()
    w.add_sphere_radius((0., 0., -5.), 1., _lam(oracle))
    w.add_sphere_radius((0., 0., -5.), 1., _lam(oracle))
    _, oid = w.hit((0., 0., 0.), (0., 0., -1.))
    assert oid == 2


def test_sdf_known_values(oracle):
    w = oracle.World()
    w.add_marched_sphere((0., 0., 0.), 1., _lam(oracle))
    w.add_marched_box((0., 0., 0.), (1., 1., 1.), _lam(oracle))
    w.add_marched_torus(np.eye(4, dtype=F), (1., 0.25, 0.25), _lam(oracle))
    sdf = lambda k, p: oracle.lib.oro_marched_sdf(w.h, k, 0, oracle.fp(oracle.f3(p)))
    assert sdf(0, (2., 0., 0.)) == 1.0
    assert sdf(1, (3., 0., 0.)) == 2.0 and sdf(1, (0., 0., 0.)) == -1.0
    assert sdf(2, (1., 0., 0.)) == F(-0.25) and sdf(2, (0., 0., 0.)) == F(0.75)


def test_user_sdf_program_known_values(oracle):
    """A user marched object's SDF program (om_world_add_marched_sdf) under the identity transform:
    each op against its closed form, including the CSG ops and a deep stack."""
    w = oracle.World()
    eye = np.eye(4, dtype=F)
    progs = [[("sphere", 1., 0., 0., 0.5)],
             [("box", 0., 0., 0., 1., 1., 1.)],
             [("torus", 0., 0., 0., 1., 0.25)],
             [("sphere", 0., 0., 0., 1.), ("sphere", 2., 0., 0., 1.), ("union",)],
             [("sphere", 0., 0., 0., 1.), ("sphere", 2., 0., 0., 1.), ("intersect",)],
             [("sphere", 0., 0., 0., 1.), ("sphere", 2., 0., 0., 1.), ("subtract",)],
             [("box", 0., 0., 0., 1., 1., 1.), ("round", 0.25)],
             [("sphere", 0., 0., 0., 1.), ("sphere", 1., 0., 0., 1.), ("sphere", 2., 0., 0., 1.), ("union",), ("union",)]]
    for ops in progs:
        w.add_marched_sdf(eye, ops, _lam(oracle))
    sdf = lambda i, p: oracle.lib.oro_marched_sdf(w.h, 3, i, oracle.fp(oracle.f3(p)))
    assert sdf(0, (3., 0., 0.)) == 1.5 and sdf(0, (1., 0., 0.)) == -0.5
    assert sdf(1, (3., 0., 0.)) == 2.0 and sdf(1, (0., 0., 0.)) == -1.0
    assert sdf(2, (1., 0., 0.)) == F(-0.25) and sdf(2, (0., 0., 0.)) == F(0.75)
    assert sdf(3, (4., 0., 0.)) == 1.0 and sdf(3, (-2., 0., 0.)) == 1.0       # min(3, 1), min(1, 3)
    assert sdf(4, (1., 0., 0.)) == 0.0 and sdf(4, (4., 0., 0.)) == 3.0        # max(0, 0), max(3, 1)
    assert sdf(5, (-0.5, 0., 0.)) == -0.5 and sdf(5, (1.5, 0., 0.)) == 0.5    # max(-0.5, -1.5), max(0.5, 0.5)
    assert sdf(6, (3., 0., 0.)) == 1.75
    assert sdf(7, (5., 0., 0.)) == 2.0 and sdf(7, (-3., 0., 0.)) == 2.0


def test_user_sdf_torus_program_renders_the_marched_torus(om, oracle):
    """The program [torus 0 0 0 R r] under a MarchedTorus's transform IS that torus (same to_local,
    local_sdf, to_world_f and default normal, marched.rs:14-44, 133-151; same object index): the
    oracle renders the two worlds bit for bit alike, bloom included."""
    from scenes_common import compare_stats, user_sdf_zoo
    W, H, SPP = 24, 16, 2
    _, ow_t, _, ocam = user_sdf_zoo(om, oracle, torus_as_program=False)
    _, ow_p, _, _ = user_sdf_zoo(om, oracle, torus_as_program=True)
    p = oracle.params(W, H, SPP, seed=9, march_steps=256)
    a, _ = oracle.render(ow_t, ocam, p)
    b, _ = oracle.render(ow_p, ocam, p)
    nb, msg = compare_stats(b, a, "torus program vs MarchedTorus")
    assert nb == 0, msg
    assert int(np.count_nonzero(a["bloom"])) > 0


def test_marched_normals(oracle):
    w = oracle.World()
    w.add_marched_box((0., 0., 0.), (1., 1., 1.), _lam(oracle))
    out = (C.c_float * 3)()
    oracle.lib.oro_marched_normal(w.h, 1, 0, oracle.fp(oracle.f3((1.5, 0.2, 0.1))), oracle.fp(out))
    assert tuple(out) == (1., 0., 0.)
    # eps = 1e-7 central differences vanish at |x| = 3 (ulp 2.4e-7): the reference yields a NaN normal
    oracle.lib.oro_marched_normal(w.h, 1, 0, oracle.fp(oracle.f3((3., 0., 0.))), oracle.fp(out))
    assert all(math.isnan(v) for v in out)


def _scatter(O, ray, hit, mat, state):
    out = (C.c_float * 9)()
    st = C.c_uint64()
    O.lib.oro_scatter(O.fp((C.c_float * 6)(*ray)), O.fp((C.c_float * 7)(*hit)), C.byref(mat), C.c_uint64(state),
                      O.fp(out), C.byref(st))
    return np.array(list(out), dtype=F)


def test_dielectric_schlick_normal_incidence(oracle):
    # reflectance(1, 1/1.5) = r0^2 = 0.04: reflect iff 0.04 > u (materials.rs:85, :110-116)
    mat = oracle.material("dielectric", ior=1.5)
    lo = hi = None
    for s in range(2000):
        u = _path_state_draws_py(s, 1)[0]     # oro_scatter draws from om-rng's path stream
        if u < 0.04 and lo is None:
            lo = s
        if u > 0.5 and hi is None:
            hi = s
    r = _scatter(oracle, (0, 0, 1, 0, 0, -1), (1, 0, 0, 0, 0, 0, 1), mat, lo)
    assert tuple(r[6:9]) == (0., 0., 1.) and tuple(r[0:3]) == (1., 1., 1.)
    r = _scatter(oracle, (0, 0, 1, 0, 0, -1), (1, 0, 0, 0, 0, 0, 1), mat, hi)
    assert tuple(r[6:9]) == (0., 0., -1.)


def test_metal_reflection_and_lambertian_hemisphere(oracle):
    s = F(1.0) / np.sqrt(F(2.0))
    r = _scatter(oracle, (0, 1, 0, s, -s, 0), (1, 0, 0, 0, 0, 1, 0), oracle.material("metal", (0.9, 0.8, 0.7)), 3)
    assert np.allclose(r[6:9], [s, s, 0], atol=1e-6) and np.allclose(r[0:3], [0.9, 0.8, 0.7])
    for st in range(50):
        r = _scatter(oracle, (0, 1, 0, 0, -1, 0), (1, 0, 0, 0, 0, 1, 0), _lam(oracle), st)
        assert abs(np.linalg.norm(r[6:9]) - 1) < 1e-5 and r[7] >= -1e-6


def _stats(O):
    return np.zeros(1, dtype=O.PIXEL_STATS_DTYPE)


def test_quantisation_and_bad_run(oracle):
    st = _stats(oracle)
    add = lambda c, d=1.0, i=0: oracle.lib.oro_stats_add(st.ctypes.data_as(C.c_void_p),
                                                         oracle.fp(oracle.f3(c)), F(d), C.c_uint64(i))
    add((0.25, 1.0, 4.0))
    assert tuple(st["color"][0]) == (128, 255, 255)                  # sqrt, clamp 0.999, *256 as u8
    st2 = _stats(oracle)
    oracle.lib.oro_stats_add(st2.ctypes.data_as(C.c_void_p), oracle.fp(oracle.f3((float("nan"), -1.0, 0.0))),
                             F(1.0), C.c_uint64(0))
    assert tuple(st2["color"][0]) == (0, 0, 0)                       # NaN and negatives -> 0
    for _ in range(5):
        add((0.25, 1.0, 4.0))
    assert st["bad_avgs"][0] == 5 and st["flags"][0] & 1 == 1        # Stats::add done rule
    assert st["n"][0] == 6 and st["avg_depth"][0] == 1.0


def test_bloom_and_scramble(oracle):
    assert oracle.bloom_hash(0) == 0 and oracle.scramble(0) == 0
    for i in range(1, 50):
        h = oracle.bloom_hash(i)
        assert 1 <= bin(h).count("1") <= 9


def _render_one(O, world, cam, W=4, H=4, spp=2, depth=50):
    p = O.params(W, H, spp, max_depth=depth, seed=5)
    st, ctr = O.render(world, cam, p, nthreads=2)
    return st, ctr


def test_sky_colour_up_and_down(oracle):
    empty = oracle.World()
    up = oracle.camera((0., 0., 0.), (0., 1., 0.), (1., 0., 0.), 1., 1., 0., 1.)
    st, ctr = _render_one(oracle, empty, up)
    mean = st["sum"] / st["n"][:, None]
    assert np.allclose(mean, [0.5, 0.7, 1.0], atol=1e-4)             # lerp(1, white, sky)
    assert np.isinf(st["avg_depth"]).all() and (st["bloom"] == 0).all()
    down = oracle.camera((0., 0., 0.), (0., -1., 0.), (1., 0., 0.), 1., 1., 0., 1.)
    st, _ = _render_one(oracle, empty, down)
    assert np.allclose(st["sum"] / st["n"][:, None], [1., 1., 1.], atol=1e-4)
    assert ctr["segments"] == ctr["samples"] == 32


def test_depth_exhaustion_returns_black(oracle):
    # camera inside a mirror sphere: every segment hits -> -Color::ZERO (render_thread.rs:142)
    w = oracle.World()
    w.add_sphere_radius((0., 0., 0.), 10., oracle.material("metal", (1., 1., 1.)))
    cam = oracle.camera((0., 0., 0.), (0., 0., -1.), (0., 1., 0.), 40., 1., 0., 1.)
    st, ctr = _render_one(oracle, w, cam, depth=7)
    assert (st["sum"] == 0).all() and (st["n"] == 2).all()
    assert ctr["segments"] == 7 * ctr["samples"]
    assert np.allclose(st["avg_depth"], 10.0, atol=1e-4)


def test_adaptive_credit(oracle):
    empty = oracle.World()
    up = oracle.camera((0., 0., 0.), (0., 1., 0.), (1., 0., 0.), 1., 1., 0., 1.)
    p = oracle.params(2, 2, 20, adaptive=True, seed=1)
    st, ctr = oracle.render(empty, up, p, nthreads=1)
    # constant sky: colour fixed after sample 1 -> 5 bad runs -> retire at n = 6 (render_thread.rs:31-38)
    assert (st["n"] == 6).all()
    assert ctr["credited"] == 4 * 20                                 # skipped samples credited (:196-198)


# ---- reference-semantics traps: each pins one place where the reference
# departs from the textbook integrator, so the oracle cannot silently "fix" it

def test_metal_never_absorbs_below_surface(oracle):
    """materials.rs:62-66: Metal::scatter always returns the fuzzed reflection, even when it
    points into the surface (the textbook version absorbs when scattered . n <= 0)."""
    mat = oracle.material("metal", (0.9, 0.8, 0.7), fuzz=1.0)
    d = np.array([1.0, -0.05, 0.0], dtype=F)
    d = d / np.linalg.norm(d)
    below = 0
    for st in range(200):
        r = _scatter(oracle, (0, 0, 0, *d), (1, 0, 0, 0, 0, 1, 0), mat, st)
        assert np.allclose(r[0:3], [0.9, 0.8, 0.7])                     # attenuation = albedo, always
        assert abs(np.linalg.norm(r[6:9]) - 1) < 1e-5                  # Ray::new normalises (ray.rs:12)
        below += r[7] < 0
    assert below > 0                                                   # some rays go into the surface


def test_ellipsoid_normal_is_l2w_of_local_point(oracle):
    """traced.rs:59: normal = unit(L2W . p_local), not the inverse-transpose (geometric) normal."""
    w = oracle.World()
    w.add_sphere(np.diag([2., 1., 1., 1.]).astype(F), _lam(oracle))
    out, _ = w.hit((-10., 0.5, 0.), (1., 0., 0.))
    lp = np.array([-np.sqrt(F(0.75)), 0.5, 0.0], dtype=F)               # local hit point on the unit sphere
    ref = np.array([2.0, 1.0, 1.0], dtype=F) * lp
    ref = ref / np.linalg.norm(ref)                                    # (-0.961, 0.277, 0)
    geo = lp / np.array([2.0, 1.0, 1.0], dtype=F)
    geo = geo / np.linalg.norm(geo)                                    # (-0.655, 0.756, 0): NOT what the reference does
    assert np.allclose(out[4:7], ref, atol=1e-6)
    assert not np.allclose(out[4:7], geo, atol=1e-2)


def test_cube_normal_is_not_normalised(oracle):
    """traced.rs:296: Cube's normal is L2W . (axis * sign) without .unit()."""
    w = oracle.World()
    w.add_cube(np.diag([1., 3., 1., 1.]).astype(F), _lam(oracle))      # unit cube stretched 3x in y
    out, _ = w.hit((0., 10., 0.), (0., -1., 0.))
    assert out[0] == F(10.0 - 1.5)
    assert tuple(out[4:7]) == (0., 3., 0.)                             # length 3


def test_refract_takes_abs_before_sqrt(oracle):
    """materials.rs:105: r_out_parallel = -sqrt(|1 - |perp|^2|) n.  With the cube's unnormalised
    normal (length 3) |perp|^2 > 1 although cannot_refract is false (cos_theta clamps to 1):
    the abs keeps the refracted direction finite where the textbook form gives NaN."""
    mat = oracle.material("dielectric", ior=1.5)
    s = F(1.0) / np.sqrt(F(2.0))
    st = next(k for k in range(2000) if _path_state_draws_py(k, 1)[0] > 0.04)   # refract, not Schlick-reflect
    r = _scatter(oracle, (0, 0, 0, s, -s, 0), (1, 0, 0, 0, 0, 3, 0), mat, st)
    n = np.array([0, 3, 0], dtype=F)
    uv = np.array([s, -s, 0], dtype=F)
    ratio = F(1.0) / F(1.5)
    perp = ratio * (uv + F(1.0) * n)
    assert float(perp @ perp) > 1.0
    out = perp + (-np.sqrt(np.abs(F(1.0) - perp @ perp))) * n
    assert np.all(np.isfinite(r[6:9]))
    assert np.allclose(r[6:9], out / np.linalg.norm(out), atol=1e-6)


def test_exhausted_depth_colour_is_negative_zero(oracle):
    """render_thread.rs:142: a path that runs out of depth returns -Color::ZERO; Stats::add of
    it onto Color::ZERO gives +0 sums (IEEE: +0 + -0 = +0), so the frame shows black with
    n counted and the first hit's depth, never a NaN (checked bit for bit)."""
    w = oracle.World()
    w.add_sphere_radius((0., 0., 0.), 10., oracle.material("metal", (1., 1., 1.)))
    cam = oracle.camera((0., 0., 0.), (0., 0., -1.), (0., 1., 0.), 40., 1., 0., 1.)
    st, _ = _render_one(oracle, w, cam, depth=3)
    assert (st["sum"].view(np.uint32) == 0).all()                      # +0 bit patterns
    assert (st["color"] == 0).all() and (st["n"] == 2).all()


def test_oracle_tie_scene_later_copy_wins(om, oracle):
    """The oracle itself on the tie scene: a ray at the 10-copy sphere returns the LAST copy, one
    at the shared triangle/parallelogram plane returns the parallelogram (hits.rs:274-285)."""
    from scenes_common import tie_scene
    _, ow = tie_scene(om, oracle)
    c = ow.counts()
    hit = ow.hit((13., 2., 3.), tuple(np.subtract((4., 1., 0.), (13., 2., 3.))))
    assert hit is not None and hit[1] == c[0]              # the last sphere (obj id = gi + 1)
    p1, p2, p3 = (np.array(p) for p in ((-4., 0.3, -1.), (-3.5, 2.2, -1.2), (-2.2, 0.5, 1.)))
    n = np.cross(p2 - p1, p3 - p1)
    n /= np.linalg.norm(n)
    centroid = (p1 + p2 + p3) / 3
    hit = ow.hit(tuple(centroid - 3 * n), tuple(n))      # from the side outside the ellipsoid field
    para0 = c[0] + c[1] + c[2] + c[3]                      # type order: spheres, cubes, triangles, planes, parallelograms
    assert hit is not None and hit[1] == para0 + 1

def test_oracle_tie_scene_duplicates_decide_pixels(om, oracle):
    """The oracle frames of the tie scene with and without the later copies differ in the winning
    ids of many pixels, so the GPU tie tests (test_gpu_edge_cases.py) exercise real ties."""
    from scenes_common import tie_scene
    W, H, SPP = 32, 20, 1
    _, ow = tie_scene(om, oracle)
    _, ow1 = tie_scene(om, oracle, duplicates=False)
    cam = oracle.default_camera(W / H)
    a, _ = oracle.render(ow, cam, oracle.params(W, H, SPP, seed=29))
    b, _ = oracle.render(ow1, cam, oracle.params(W, H, SPP, seed=29))
    assert int((a["bloom"] != b["bloom"]).sum()) > W * H // 20


def test_oracle_nan_normal_scene_reaches_nan(om, oracle):
    """The marched box face at local |x| = 3 gives NaN normals (marched.rs:25-44), which reach
    the pixels' running sums; the GPU test compares against exactly these frames."""
    from scenes_common import nan_normal_world
    W, H, SPP = 32, 20, 1
    _, ow = nan_normal_world(om, oracle)
    st, _ = oracle.render(ow, oracle.default_camera(W / H), oracle.params(W, H, SPP, seed=31, march_steps=256))
    n_nan = int(np.isnan(st["sum"]).any(axis=1).sum())
    assert 0 < n_nan < W * H


def test_threaded_pixel_windows_equal_single_thread_and_full_frame(oracle):
    """oro_render_pixels_mt (the oracle windows of the full-size parity tests and bench.py) ==
    the single-thread pixel-subset form == the same pixels of a whole-frame oro_render."""
    W, H, spp = 40, 24, 5
    w, cam = oracle.random_scene(0x5EED), oracle.default_camera(W / H)
    p = oracle.params(W, H, spp, seed=9, max_depth=20)
    pix = oracle.window_pixels(W, H, 7, 5, 12)
    one = oracle.render_pixels(w, cam, p, pix)
    mt = oracle.render_pixels(w, cam, p, pix, nthreads=3)
    full, _ = oracle.render(w, cam, p)
    assert np.array_equal(one.view(np.uint8), mt.view(np.uint8))
    assert np.array_equal(one.view(np.uint8), full[pix].view(np.uint8))
    assert pix[0] == 5 * W + 7 and pix[-1] == 16 * W + 18
