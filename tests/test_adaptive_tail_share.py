"""The number behind DESIGN.md §5.8's "why the deferred-tail schedule was not built" (VERDICT r05
#3), on the CPU oracle: a deferred tail must leave out of the stream's next adaptive batch every pixel
with a sample still in the tail, because Stats::add takes a pixel's samples in order and retirement
depends on them (render_thread.rs:23-39, 68-102).  A pixel has a path in the tail (bounce >= 8, the
adaptive tail threshold) exactly when rendering its batch at max_depth 8 changes its Stats: a path
cut at depth 8 returns -0 black (render_thread.rs:142) instead of its colour.  With call 1's batches
(~43 samples per live pixel) that is a large share of the non-sky pixels, so the next
batch would run on roughly half the live pixels."""
import numpy as np


def _tail_share(O, batch, n=1500):
    W, H = 1920, 1080
    pix = np.random.default_rng(5).choice(W * H, n, replace=False).astype(np.uint32)
    world, cam = O.random_scene(0x5EED), O.default_camera(W / H)
    cut = O.render_pixels(world, cam, O.params(W, H, batch, max_depth=8, seed=1), pix, nthreads=0)
    full = O.render_pixels(world, cam, O.params(W, H, batch, max_depth=50, seed=1), pix, nthreads=0)
    deep = np.any(cut["sum"] != full["sum"], axis=1) | (cut["bloom"] != full["bloom"])
    sky = full["avg_depth"] == np.inf
    return deep.mean(), deep[~sky].mean()


def test_share_of_pixels_with_a_path_in_the_adaptive_tail(oracle):
    all43, lit43 = _tail_share(oracle, 43)
    all16, lit16 = _tail_share(oracle, 16)
    # r06 (4 000 pixels): 0.348 / 0.450 at 43 samples, 0.201 / 0.259 at 16
    assert 0.25 < all43 < 0.45 and 0.35 < lit43 < 0.55, (all43, lit43)
    assert all16 < all43 and lit16 < lit43
