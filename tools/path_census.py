"""Paths alive per bounce (Q_b) on a C1-like frame: segments(max_depth = K) - segments(K-1),
from the counting build's device counters.  Usage: python tools/path_census.py [W H SPP]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import raytracingoneweekend_amd as om  # noqa: E402

W, H, SPP = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (480, 270, 16)
world = om.random_scene(0x5EED)
cam = om.default_camera(W / H)
fz = world.freeze(cam)
prev, out = 0, []
for k in range(1, 51):
    pix = om.PixelsBox.new(W * H)
    c = om.render(cam, fz, k, 0.001, 100.0, SPP, W, H, pix, seed=1, adaptive=False)
    out.append(c["segments"] - prev)
    prev = c["segments"]
n = W * H * SPP
print("samples", n)
print("Q_b / samples:", " ".join(f"{b}:{q / n:.4g}" for b, q in enumerate(out)))
print("segments >= 16:", sum(out[16:]) / n, " >= 8:", sum(out[8:]) / n, " total:", sum(out) / n)
