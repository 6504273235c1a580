"""Shared scene/param helpers for tests: build the SAME world on the product side
(raytracingoneweekend_amd, HIP) and the oracle side (CPU restatement)."""
import numpy as np

F = np.float32


def kitchen_sink(om, O):
    """Every primitive type of hits.rs:370-371, each constructor path used at least once."""
    w = om.HittableList.new()
    ow = O.World()
    lam = lambda c: (om.Material.new_lambertian(c), O.material("lambertian", c))
    met = lambda c, f: (om.Material.new_metal_fuzz(c, f), O.material("metal", c, fuzz=f))
    die = lambda i: (om.Material.new_dielectric(i), O.material("dielectric", ior=i))

    m, om_ = lam((0.5, 0.5, 0.5))
    w += om.InfinitePlane.new((0., -0.5, 0.), (0., 1., 0.05), m); ow.add_plane((0., -0.5, 0.), (0., 1., 0.05), om_)
    m, om_ = lam((0.8, 0.3, 0.3))
    w += om.Sphere.new_with_radius((0., 0.5, -1.), 0.5, m); ow.add_sphere_radius((0., 0.5, -1.), 0.5, om_)
    l2w = om.m4x4("TR", 1.2, 0.4, -1.) ^ om.m4x4("RY", 0.7) ^ om.m4x4("SC", 0.3, 0.6, 0.3)
    m, om_ = met((0.8, 0.8, 0.9), 0.2)
    w += om.Sphere.new(l2w, m); ow.add_sphere(l2w.to_numpy(), om_)
    m, om_ = met((0.9, 0.6, 0.2), 0.0)
    w += om.Cube.new_with_length((-1.3, 0.3, -1.2), 0.6, m); ow.add_cube_length((-1.3, 0.3, -1.2), 0.6, om_)
    l2w = om.m4x4("TR", 0.1, 1.4, -1.8) ^ om.m4x4("RX", 0.4) ^ om.m4x4("RZ", 0.9)
    m, om_ = die(1.5)
    w += om.Cube.new(l2w, m); ow.add_cube(l2w.to_numpy(), om_)
    m, om_ = lam((0.2, 0.9, 0.2))
    w += om.Triangle.new3points((-2., 0., -2.5), (-1., 1.5, -2.5), (-2.5, 1.2, -2.0), m)
    ow.add_triangle((-2., 0., -2.5), (-1., 1.5, -2.5), (-2.5, 1.2, -2.0), om_)
    m, om_ = met((0.7, 0.7, 0.7), 0.05)
    w += om.Parallelogram.new3points((1.5, 0., -2.5), (2.5, 0.2, -2.5), (1.6, 1.4, -2.7), m)
    ow.add_parallelogram((1.5, 0., -2.5), (2.5, 0.2, -2.5), (1.6, 1.4, -2.7), om_)
    m, om_ = lam((0.3, 0.3, 0.9))
    w += om.MarchedSphere((-0.6, 0.25, -0.3), 0.25, m); ow.add_marched_sphere((-0.6, 0.25, -0.3), 0.25, om_)
    m, om_ = met((0.9, 0.9, 0.3), 0.1)
    w += om.MarchedBox((0.6, 0.2, -0.2), (0.15, 0.2, 0.1), m); ow.add_marched_box((0.6, 0.2, -0.2), (0.15, 0.2, 0.1), om_)
    l2w = om.m4x4("TR", 0., 0.9, -0.6) ^ om.m4x4("RX", 0.9) ^ om.m4x4("RZ", 0.3)
    m, om_ = die(1.3)
    w += om.MarchedTorus.new(l2w, (0.35, 0.08, 0.08), m); ow.add_marched_torus(l2w.to_numpy(), (0.35, 0.08, 0.08), om_)
    cam = om.Camera.new((0., 1., 2.), (0., 0.5, -1.), (0., 1., 0.), 60., 1.5, 0.05, 3.)
    ocam = O.camera((0., 1., 2.), (0., 0.5, -1.), (0., 1., 0.), 60., 1.5, 0.05, 3.)
    return w, ow, cam, ocam


def compare_stats(got, exp, label=""):
    """Bitwise comparison of om_pixel_stats arrays; returns (n_bad, message)."""
    g = got.view(np.uint8).reshape(-1, 40)
    e = exp.view(np.uint8).reshape(-1, 40)
    bad = np.any(g != e, axis=1)
    nb = int(bad.sum())
    msg = ""
    if nb:
        idx = np.nonzero(bad)[0][:5]
        rows = []
        for i in idx:
            rows.append(f"px {i}: got sum={got['sum'][i]} n={got['n'][i]} depth={got['avg_depth'][i]} "
                        f"bloom={got['bloom'][i]:x} | exp sum={exp['sum'][i]} n={exp['n'][i]} "
                        f"depth={exp['avg_depth'][i]} bloom={exp['bloom'][i]:x}")
        msg = f"{label}: {nb}/{len(bad)} pixels differ\n" + "\n".join(rows)
    return nb, msg


def compare_stats_nan_payload(got, exp, label=""):
    """compare_stats, except that a NaN in `sum` only has to be a NaN on both sides: the sign
    and mantissa bits of a NaN are not fixed across CPU and GPU (x86's default NaN carries the
    sign bit, gfx950's does not).  Every other byte must match."""
    g = got.copy()
    e = exp.copy()
    gn, en = np.isnan(g["sum"]), np.isnan(e["sum"])
    both = gn & en
    g["sum"][both] = 0.0
    e["sum"][both] = 0.0
    nb, msg = compare_stats(g, e, label)
    mism = int((gn != en).any(axis=1).sum())
    if mism and not nb:
        nb, msg = mism, f"{label}: NaN-ness differs on {mism} pixels"
    return nb, msg


def tie_scene(om, O, duplicates=True):
    """Ground + a 10x10 field of ellipsoids (every 5th followed by an exact duplicate with another
    material: ties inside one BVH leaf) + a unit sphere at (4,1,0) added 10 times with 10
    materials (degenerate centroids: the builder's median split deals the copies over several
    leaves) + a cube twice + a triangle and a parallelogram from the same three points.
    duplicates=False drops every later copy: the frame where the FIRST object would win."""
    w, ow = om.HittableList.new(), O.World()
    rng = np.random.default_rng(20260117)
    palette = [("lambertian", (0.8, 0.3, 0.2), 0.0, 0.0), ("metal", (0.7, 0.8, 0.9), 0.1, 0.0),
               ("dielectric", (0.0, 0.0, 0.0), 0.0, 1.5), ("lambertian", (0.1, 0.6, 0.2), 0.0, 0.0),
               ("metal", (0.9, 0.6, 0.3), 0.4, 0.0)]

    def mat(k):
        kind, alb, fuzz, ior = palette[k % len(palette)]
        if kind == "lambertian":
            return om.Material.new_lambertian(alb), O.material(kind, alb)
        if kind == "metal":
            return om.Material.new_metal_fuzz(alb, fuzz), O.material(kind, alb, fuzz=fuzz)
        return om.Material.new_dielectric(ior), O.material(kind, ior=ior)

    m, m_ = mat(0)
    w += om.Sphere.new_with_radius((0., -1000., 0.), 1000., m); ow.add_sphere_radius((0., -1000., 0.), 1000., m_)
    k = 0
    for a in range(-5, 5):
        for b in range(-5, 5):
            u = rng.random(6, dtype=F)
            l2w = om.m4x4("TR", F(a) + F(0.9) * u[0], F(0.2), F(b) + F(0.9) * u[1]) \
                ^ om.m4x4("RX", u[2] * F(6.2831855)) ^ om.m4x4("RY", u[3] * F(6.2831855)) \
                ^ om.m4x4("SC", F(0.2) * (u[4] + F(1.)), F(0.2), F(0.2) * (u[5] + F(1.)))
            copies = 2 if (duplicates and k % 5 == 0) else 1
            for c in range(copies):
                m, m_ = mat(k + 2 * c)
                w += om.Sphere.new(l2w, m); ow.add_sphere(l2w.to_numpy(), m_)
            k += 1
    for c in range(10 if duplicates else 1):
        m, m_ = mat(c)
        w += om.Sphere.new_with_radius((4., 1., 0.), 1., m); ow.add_sphere_radius((4., 1., 0.), 1., m_)
    l2w = om.m4x4("TR", 0., 1., 0.) ^ om.m4x4("RX", 0.5) ^ om.m4x4("RY", 0.9) ^ om.m4x4("SC", 1.2, 1.2, 1.2)
    for c in range(2 if duplicates else 1):
        m, m_ = mat(3 + c)
        w += om.Cube.new(l2w, m); ow.add_cube(l2w.to_numpy(), m_)
    p1, p2, p3 = (-4., 0.3, -1.), (-3.5, 2.2, -1.2), (-2.2, 0.5, 1.)
    m, m_ = mat(1)
    w += om.Triangle.new3points(p1, p2, p3, m); ow.add_triangle(p1, p2, p3, m_)
    if duplicates:
        m, m_ = mat(0)
        w += om.Parallelogram.new3points(p1, p2, p3, m); ow.add_parallelogram(p1, p2, p3, m_)
    return w, ow


def nan_normal_world(om, O):
    """A marched world whose box face sits at local |x| = 3 (marched.rs:25-44 -> NaN normals
    there), next to a marched sphere and a marched ground (normals well defined)."""
    w, ow = om.HittableList.new(), O.World()
    lam = (om.Material.new_lambertian((0.7, 0.6, 0.5)), O.material("lambertian", (0.7, 0.6, 0.5)))
    met = (om.Material.new_metal_fuzz((0.8, 0.8, 0.8), 0.2), O.material("metal", (0.8, 0.8, 0.8), fuzz=0.2))
    die = (om.Material.new_dielectric(1.5), O.material("dielectric", ior=1.5))
    w += om.MarchedSphere((0., -1000., 0.), 1000., lam[0]); ow.add_marched_sphere((0., -1000., 0.), 1000., lam[1])
    w += om.MarchedBox((0., 0.6, 0.), (3., 0.6, 0.5), met[0]); ow.add_marched_box((0., 0.6, 0.), (3., 0.6, 0.5), met[1])
    w += om.MarchedBox((0., 0.5, 2.2), (3., 0.5, 0.4), lam[0]); ow.add_marched_box((0., 0.5, 2.2), (3., 0.5, 0.4), lam[1])
    w += om.MarchedSphere((4., 1., -1.5), 1., die[0]); ow.add_marched_sphere((4., 1., -1.5), 1., die[1])
    return w, ow


def user_sdf_zoo(om, O, torus_as_program=False):
    """User marched objects (`HittableList += Arc<dyn Marched>`, hits.rs:96-100) as SDF programs
    (om_world_add_marched_sdf) beside typed marched objects: CSG with every op, non-uniform scales,
    a rotated frame.  torus_as_program: the typed torus replaced by the program [torus 0 0 0 R r]
    under the same transform, which must render the same bits (same object index, too)."""
    w, ow = om.HittableList.new(), O.World()
    lam = lambda c: (om.Material.new_lambertian(c), O.material("lambertian", c))
    met = lambda c, f: (om.Material.new_metal_fuzz(c, f), O.material("metal", c, fuzz=f))
    die = lambda i: (om.Material.new_dielectric(i), O.material("dielectric", ior=i))
    m, om_ = lam((0.5, 0.5, 0.5))
    w += om.MarchedSphere((0., -100., 0.), 100., m); ow.add_marched_sphere((0., -100., 0.), 100., om_)
    m, om_ = met((0.7, 0.6, 0.5), 0.1)
    w += om.MarchedBox((1.6, 0.35, -0.4), (0.3, 0.35, 0.2), m); ow.add_marched_box((1.6, 0.35, -0.4), (0.3, 0.35, 0.2), om_)
    tor = om.m4x4("TR", -0.2, 0.7, 0.3) ^ om.m4x4("RX", 0.8) ^ om.m4x4("SC", 1.3, 0.8, 1.1)
    m, om_ = die(1.4)
    if torus_as_program:
        ops = [("torus", 0., 0., 0., 0.45, 0.12)]
        w += om.MarchedSdf.new(tor, ops, m); ow.add_marched_sdf(tor.to_numpy(), ops, om_)
    else:
        w += om.MarchedTorus.new(tor, (0.45, 0.12, 0.12), m); ow.add_marched_torus(tor.to_numpy(), (0.45, 0.12, 0.12), om_)
    progs = [
        # a rounded cube carved by a sphere, scaled non-uniformly
        (om.m4x4("TR", -1.3, 0.55, -0.2) ^ om.m4x4("RY", 0.5) ^ om.m4x4("SC", 0.9, 1.2, 0.8),
         [("box", 0., 0., 0., 0.35, 0.35, 0.35), ("round", 0.05), ("sphere", 0., 0.1, 0., 0.42), ("subtract",)],
         met((0.9, 0.5, 0.3), 0.0)),
        # a sphere intersected with a box, unioned with a torus ring around it
        (om.m4x4("TR", 0.6, 0.45, 0.9) ^ om.m4x4("RZ", 0.3),
         [("sphere", 0., 0., 0., 0.4), ("box", 0., 0., 0., 0.3, 0.3, 0.3), ("intersect",),
          ("torus", 0., 0., 0., 0.45, 0.05), ("union",)],
         lam((0.2, 0.7, 0.9))),
        # three spheres in a row, unioned (deep stack)
        (om.m4x4("TR", 0.2, 0.18, -1.2),
         [("sphere", -0.4, 0., 0., 0.18), ("sphere", 0., 0., 0., 0.18), ("sphere", 0.4, 0., 0., 0.18),
          ("union",), ("union",)],
         die(1.5)),
    ]
    for l2w, ops, (m, om_) in progs:
        w += om.MarchedSdf.new(l2w, ops, m); ow.add_marched_sdf(l2w.to_numpy(), ops, om_)
    cam = om.Camera.new((2.6, 1.4, 3.2), (0., 0.4, -0.2), (0., 1., 0.), 40., 1.5, 0.02, 4.)
    ocam = O.camera((2.6, 1.4, 3.2), (0., 0.4, -0.2), (0., 1., 0.), 40., 1.5, 0.02, 4.)
    return w, ow, cam, ocam
