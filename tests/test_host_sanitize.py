"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only): the product's host
C++ (om_world.cpp scene builders and freeze, om_bvh.cpp BVH/SBVH/BVH2/BVH4 builders,
om_tiles.cpp primary-ray tile lists, om_shard.cpp tile deal) and the CPU oracle, compiled
from their sources into tests/cpp/host_sanitize (make -C tests/cpp sanitize) and driven over
S-traced, S-full, S-10k, S-marched and basic_scene with the default and a wide-lens camera
at 1920x1080 / 53x37 / 1x1 / 8x8.  Any sanitizer report fails the run."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def test_host_code_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", CPP, "sanitize"], stdout=subprocess.DEVNULL)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(CPP, "host_sanitize")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]


def test_packet_traversal_would_visit_more_than_the_busiest_lane():
    """DESIGN.md §8 (VERDICT r05 #1c): on the product's S-traced BVH2, the bounce-1 rays of an 8x8
    tile need more node and leaf visits as a packet (the union) than the busiest lane of the
    shipped per-ray traversal (tests/cpp/packet_union.cpp, host code only)."""
    import re
    subprocess.check_call(["make", "-s", "-C", CPP, "packet_union"])
    out = subprocess.run([os.path.join(CPP, "packet_union")], capture_output=True, text=True, timeout=120, check=True).stdout
    m = re.search(r"per ray ([\d.]+), busiest lane ([\d.]+), packet union ([\d.]+); leaf visits busiest lane ([\d.]+), "
                  r"packet union ([\d.]+)", out)
    per_ray, lane, union, leaf_lane, leaf_union = map(float, m.groups())
    assert union > 1.2 * lane and leaf_union > 1.5 * leaf_lane and lane > per_ray, out
