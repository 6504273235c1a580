"""Headless counterpart of the reference front-end (main.rs:123-214 + draw_to_sdl):
compose random_scene through the Camera/Material/HittableList API, render it
progressively on the GPU like the reference's render threads (adaptive retirement
by default, --fixed-spp to take every sample), then save every display view (keys 0-6 of main.rs:360-367) as BMP/PPM —
the F12 save of main.rs:473-476.

    python examples/render_scene.py --width 1000 --height 666 --spp 200 --out out/
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import raytracingoneweekend_amd as om  # noqa: E402
from raytracingoneweekend_amd import _lib as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1000)           # main.rs:125-127
    ap.add_argument("--height", type=int, default=666)
    ap.add_argument("--spp", type=int, default=200)              # main.rs:145
    ap.add_argument("--max-depth", type=int, default=50)         # main.rs:146
    ap.add_argument("--per-call", type=int, default=8, help="samples per render call (progressive passes)")
    ap.add_argument("--fixed-spp", dest="adaptive", action="store_false",
                    help="take every sample of every pixel (default: retire converged pixels like the "
                         "reference's render threads, render_thread.rs:31-38,97-101)")
    ap.add_argument("--torus", action="store_true", help="include the marched torus block of main.rs:73-81")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default="out")
    ap.add_argument("--ppm", action="store_true", help="write PPM instead of BMP")
    args = ap.parse_args()

    W, H = args.width, args.height
    world = om.random_scene_api(0x5EED, with_torus=args.torus)   # main.rs:37-100 through the API
    cam = om.Camera.new((13.0, 2.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, W / H, 0.1, 10.0)  # main.rs:136-142
    frozen = world.freeze(cam)
    pixels = om.PixelsBox.new(W * H)
    t0, credited = time.perf_counter(), 0
    for done in range(0, args.spp, args.per_call):
        c = om.render(cam, frozen, args.max_depth, 0.001, 100.0, args.spp, W, H, pixels, seed=args.seed,
                      adaptive=args.adaptive, sample_count=min(args.per_call, args.spp - done))
        credited += c["credited"]
        print(f"\r{100.0 * credited / (W * H * args.spp):5.1f}%", end="", flush=True)   # main.rs:151-168 log
    dt = time.perf_counter() - t0
    print(f"\n{W}x{H}x{args.spp} in {dt:.3f} s ({W * H * args.spp / dt / 1e6:.0f} Msamples/s credited)")
    os.makedirs(args.out, exist_ok=True)
    for view in L.VIEWS:
        rgb = om.display(frozen, pixels, W, H, view)
        path = os.path.join(args.out, f"{view}.{'ppm' if args.ppm else 'bmp'}")
        (om.write_ppm if args.ppm else om.write_bmp)(path, rgb)
        print("wrote", path)


if __name__ == "__main__":
    main()
