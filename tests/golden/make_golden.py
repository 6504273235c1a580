"""Generates tests/golden/golden_v2.npz with the CPU oracle (oracle/om_oracle.cpp).

The reference ships no golden vectors and cannot be built here (no Rust toolchain), so
these fixtures pin the oracle against drift and give the GPU tests a stored answer.
Regenerate only on a deliberate contract change:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))


def build(O):
    import raytracingoneweekend_amd as om
    from scenes_common import kitchen_sink
    g = {}
    g["rng_seed0"] = O.rng_draws(0, 64)
    g["rng_seed5eed"] = O.rng_draws(0x5EED, 64)
    g["path_draws"] = O.path_draws(1, 12345, 7, 32)
    g["jitter_s1_16"] = O.jitter_table(1, 16)
    g["bloom_1_64"] = np.array([O.bloom_hash(i) for i in range(65)], dtype=np.uint64)
    ow = O.random_scene(0x5EED)
    n = ow.counts()
    g["straced_counts"] = np.array(n, dtype=np.uint32)
    g["straced_spheres"] = np.stack([ow.affine(0, i) for i in range(n[0])])
    g["straced_cube"] = ow.affine(1, 0)
    g["straced_tri"] = ow.bary(1, 0)
    g["straced_para"] = ow.bary(0, 0)
    # images (om_pixel_stats bytes)
    W, H = 40, 24
    st, ctr = O.render(ow, O.default_camera(W / H), O.params(W, H, 8, seed=3), nthreads=4)
    g["img_straced_40x24x8_seed3"] = st.view(np.uint8).reshape(-1, 40)
    g["img_straced_ctr"] = np.array([ctr["samples"], ctr["segments"]], dtype=np.uint64)
    fw = O.random_scene(0x5EED, with_torus=True)
    st, _ = O.render(fw, O.default_camera(W / H), O.params(W, H, 2, seed=4), nthreads=4)
    g["img_sfull_40x24x2_seed4"] = st.view(np.uint8).reshape(-1, 40)
    _, kw, _, kcam = kitchen_sink(om, O)
    st, _ = O.render(kw, kcam, O.params(32, 20, 4, seed=11), nthreads=4)
    g["img_kitchen_32x20x4_seed11"] = st.view(np.uint8).reshape(-1, 40)
    st, _ = O.render(O.marched_scene(), O.default_camera(24 / 16), O.params(24, 16, 2, seed=2, march_steps=256),
                     nthreads=4)
    g["img_marched_24x16x2_seed2"] = st.view(np.uint8).reshape(-1, 40)
    return g


if __name__ == "__main__":
    from oracle import oracle as O
    g = build(O)
    out = os.path.join(HERE, "golden_v2.npz")
    np.savez_compressed(out, **g)
    print("wrote", out, os.path.getsize(out), "bytes")
