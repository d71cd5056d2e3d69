"""CPU tests of the oracle's `oceanic_horizon` fragment program (reference
csrc/shaders.cpp:1668-1919 bound by csrc/rasterise_egl.cpp:385).

The reference's arithmetic here is the NVIDIA GLSL compiler's (unpinned).  Pins:
  * ch0 (sky mask) = [ray.y > 0] is geometry only (trace() returns false iff rDirection.y > 0,
    shaders.cpp:1853-1855): exact against a float64 restatement except within 1e-4 of the horizon;
  * ch1 = pow(sundot, 350) on sky pixels: within 1e-3 of float64 (SURVEY §8c tolerance);
  * ch1 on water pixels (20-step ray march, reflection): within 1e-3 of float64 on >= 99% of pixels
    (the march is chaotic at step-halving decisions);
with the harness of tests/optimize_horizon.py:251-268 (full-screen quad, zero background, 960x640,
camera [0,200,0,0,0,0,0,0.9]) and tests/square_test.py:64 (camera [0,150,0,0,0.3,0,0,1.5]).
"""
import numpy as np
import pytest

import oceanic_f64
import scenes
from oracle import oracle

CAMS = {
    "optimize_horizon": [0.0, 200.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.9],
    "square_test": [0.0, 150.0, 0.0, 0.0, 0.3, 0.0, 0.0, 1.5],
    "rolled_moving": [10.0, 120.0, -30.0, 0.05, -0.2, 0.1, 3.0, 1.2],
}


def fullscreen(H, W, C=3, background=None):
    bg = np.zeros((1, H, W, C), np.float32) if background is None else background[None].astype(np.float32)
    v = np.array([[[-1, -1, 0, 1], [-1, 1, 0, 1], [1, 1, 0, 1], [1, -1, 0, 1]]], np.float32)
    f = np.array([[[0, 1, 2], [0, 2, 3]]], np.int32)
    return bg, v, np.ones((1, 4, C), np.float32), f


@pytest.mark.parametrize("name", sorted(CAMS))
def test_oceanic_horizon_against_float64(name):
    cam = CAMS[name]
    H, W = 640, 960
    px, gb, st = oracle.rasterise_fwd(*fullscreen(H, W), shader_id=1, camera_pos=np.array(cam))
    assert st == 0 and (gb[0] >= 0).all()
    ref, rdy = oceanic_f64.render_fullscreen(H, W, cam)
    far = np.abs(rdy) >= 1e-4
    np.testing.assert_array_equal(px[0, ..., 0][far], ref[..., 0][far])
    assert np.all(px[0, ..., 2] == 0.0)
    err = np.abs(px[0, ..., 1].astype(np.float64) - ref[..., 1])
    sky = (ref[..., 0] == 1.0) & far
    water = (ref[..., 0] == 0.0) & far
    assert err[sky].max() <= 1e-3
    assert (err[water] <= 1e-3).mean() >= 0.99 and np.median(err[water]) < 1e-4


def test_oceanic_horizon_background_jitter_and_channels():
    """xy += background.xy / (width, height) (shaders.cpp:1864-1867); C=1 broadcasts the single channel
    (rasterise_egl.cu:39-47); C=4 carries fragColor.w = 1."""
    H, W = 96, 128
    rng = np.random.default_rng(3)
    bg = rng.uniform(-3, 3, size=(H, W, 3)).astype(np.float32)
    cam = CAMS["square_test"]
    px, _, _ = oracle.rasterise_fwd(*fullscreen(H, W, background=bg), shader_id=1, camera_pos=np.array(cam))
    ref, rdy = oceanic_f64.render_fullscreen(H, W, cam, background=bg)
    far = np.abs(rdy) >= 1e-3
    np.testing.assert_array_equal(px[0, ..., 0][far], ref[..., 0][far])
    bg1 = bg[..., :1].copy()
    p1, _, _ = oracle.rasterise_fwd(*fullscreen(H, W, C=1, background=bg1), shader_id=1, camera_pos=np.array(cam))
    ref1, rdy1 = oceanic_f64.render_fullscreen(H, W, cam, background=bg1)
    far1 = np.abs(rdy1) >= 1e-3
    np.testing.assert_array_equal(p1[0, ..., 0][far1], ref1[..., 0][far1])
    bg4 = np.concatenate([bg, bg[..., :1]], -1)
    p4, _, _ = oracle.rasterise_fwd(*fullscreen(H, W, C=4, background=bg4), shader_id=1, camera_pos=np.array(cam))
    np.testing.assert_array_equal(p4[0, ..., :2], px[0, ..., :2])
    assert np.all(p4[0, ..., 2] == 0.0) and np.all(p4[0, ..., 3] == 1.0)


def test_oceanic_horizon_uncovered_pixels_keep_background():
    bg, v, c, f = scenes.random_triangles(F=40, W=64, H=48, radius_px=8.0, seed=5)
    px, gb, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None], shader_id=1,
                                     camera_pos=np.array(CAMS["optimize_horizon"]))
    unc = gb[0] < 0
    assert unc.any() and (~unc).any()
    np.testing.assert_array_equal(px[0][unc], bg[unc])
    assert set(np.unique(px[0][~unc][:, 0])) <= {0.0, 1.0}


FAMILY_CAMS = [[0.0, 150.0, 0.0, 0.0, 0.1, 0.0, 1.0, 0.9, 2.0], [5.0, 120.0, -20.0, 0.02, -0.15, 0.05, 3.0, 1.2, 0.5]]


@pytest.mark.parametrize("sid", [2, 3, 4, 5], ids=["oceanic", "still_cloud", "no_cloud", "simple_proxy"])
def test_oceanic_family_against_float64(sid):
    """The `oceanic` family.  Its noise (hash = fract(cos(n)*41415.9), rand =
    fract(sin(.)*43758.5)) turns any ulp difference into a different random value, so float64 pins
    only what is noise-free: the sky of the cloudless members to 1e-4, and otherwise image statistics
    (mean colour of the water and of the sky within 0.05)."""
    H, W = 48, 72
    for cam in FAMILY_CAMS:
        px, gb, _ = oracle.rasterise_fwd(*fullscreen(H, W), shader_id=sid, camera_pos=np.array(cam))
        ref, rdy = oceanic_f64.render_family_fullscreen(sid, H, W, cam)
        sky = rdy > 1e-4
        water = rdy < -1e-4
        assert np.isfinite(px).all()
        if sid in (4, 5):
            assert np.abs(px[0][sky] - ref[sky]).max() <= 1e-4
        assert np.abs(px[0][sky].mean(0) - ref[sky].mean(0)).max() <= 0.05
        assert np.abs(px[0][water].mean(0) - ref[water].mean(0)).max() <= 0.05
