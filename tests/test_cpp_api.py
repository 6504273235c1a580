"""The C++ mirror API (include/ottomarcher.hpp + examples/random_scene.hpp), exercised by
the compiled driver tests/cpp/test_api.cpp (built by __graft_entry__.build()).

CPU: main.rs's random_scene / basic_scene composed through the C++ API are bit-identical
to the native builders; Camera / Mat4x4 / error behaviour.  GPU: the C++ render() under
main.rs's thread scheme (num_cpus-1 threads, 2730-pixel chunks, tid 0 drives the device),
progressive calls, fixed spp and the reference's adaptive default, compared byte for byte
with the CPU oracle."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "test_api")


@pytest.fixture(scope="module")
def exe(om):
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(EXE)])
    return EXE


def test_cpp_api_scene_composition_and_errors(exe):
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "cpu ok" in r.stdout


@pytest.mark.gpu
def test_cpp_render_threads_match_oracle(exe, oracle, tmp_path):
    fixed, adaptive = tmp_path / "fixed.bin", tmp_path / "adaptive.bin"
    r = subprocess.run([exe, "gpu", str(fixed), str(adaptive)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    W, H = 48, 32
    world, cam = oracle.random_scene(0x5EED), oracle.default_camera(W / H)
    for path, spp, adapt in ((fixed, 8, False), (adaptive, 24, True)):
        got = np.fromfile(path, dtype=np.uint8).reshape(W * H, 40)
        exp, _ = oracle.render(world, cam, oracle.params(W, H, spp, seed=7, adaptive=adapt))
        exp = exp.view(np.uint8).reshape(W * H, 40)
        bad = int(np.any(got != exp, axis=1).sum())
        assert bad == 0, f"{path.name}: {bad}/{W * H} pixels differ from the oracle"


@pytest.mark.gpu
def test_cpp_main_front_end_writes_every_view(exe, tmp_path):
    main = os.path.join(ROOT, "examples", "ottomarcher_main")
    if not os.path.exists(main):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(main)])
    r = subprocess.run([main, "--width", "120", "--spp", "12", "--out", str(tmp_path)], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    W, H = 120, 80                                     # main.rs:124-130: height = width / 1.5
    for view in ("normal", "samples", "samples_blur", "depth", "depth_blur", "ids", "ids_blur"):
        b = (tmp_path / f"{view}.bmp").read_bytes()
        assert b[:2] == b"BM" and int.from_bytes(b[18:22], "little") == W and int.from_bytes(b[22:26], "little") == H
    assert "100.00%" in r.stderr                        # the log thread saw every sample credited
