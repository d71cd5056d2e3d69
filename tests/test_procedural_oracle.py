"""CPU oracle of the last two procedural ops of SURVEY §8f-4 (test infrastructure):
`oceanic_opt_flow` (csrc/shaders.cpp:1178-1398, op csrc/oceanic_opt_flow.cpp) and `hill`
(csrc/shaders.cpp:123-554, op csrc/hill.cpp), pinned by known answers derived from the GLSL and by
float64 restatements (tests/oceanic_f64.py).  The reference ships no rendered outputs for either op, so
beyond these pins their parity is unpinned."""
import numpy as np
import pytest

import oceanic_f64
import scenes
from oracle import oracle

# camera_pos layout of the op (oceanic_opt_flow.cpp:399-414): [0..7] camera, [8] unused, [9] dt,
# [10..12] dx,dy,dz, [13..15] dang1..3
FLOW_CAMS = {
    "static": [0.0, 150.0, 0.0, 0.0, 0.3, 0.0, 0.0, 1.5, 0.0, 0.5, 0, 0, 0, 0, 0, 0],
    "translate": [0.0, 150.0, 0.0, 0.0, 0.3, 0.0, 0.0, 1.5, 0.0, 0.5, 10.0, 0.0, 20.0, 0.0, 0.0, 0.0],
    "rotate": [5.0, 120.0, -20.0, 0.02, 0.15, 0.05, 3.0, 1.2, 0.0, 0.25, 3.0, -1.0, 8.0, 0.01, 0.1, -0.02],
    "look_up": [0.0, 100.0, 0.0, 0.0, -0.2, 0.0, 0.0, 0.9, 0.0, 1.0, 0.0, 0.0, 5.0, 0.0, 0.05, 0.0],
}


def flow_fullscreen(H, W, cam, C=3, background=None):
    v, f = scenes.fullscreen_quad()
    bg = np.zeros((1, H, W, C), np.float32) if background is None else background[None]
    return oracle.rasterise_fwd(bg, v[None], np.ones((1, 4, C), np.float32), f[None], shader_id=6,
                                camera_pos=np.array(cam, np.float32))


def test_opt_flow_static_camera_is_identity():
    """With no camera motion the previous-frame coordinate of every pixel is the pixel itself: the
    program's forward ray, inverse rotation and projection (:1326-1395) cancel analytically."""
    H, W = 96, 128
    px, gb, st = flow_fullscreen(H, W, FLOW_CAMS["static"])
    assert st == 0 and (gb >= 0).all()
    jj, ii = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    np.testing.assert_allclose(px[0, ..., 0], ii + 0.5, atol=2e-3)
    np.testing.assert_allclose(px[0, ..., 1], (H - 1 - jj) + 0.5, atol=2e-3)  # GL window y, rows top first
    assert (px[0, ..., 2] == 0).all()


@pytest.mark.parametrize("name", sorted(FLOW_CAMS))
def test_opt_flow_against_float64(name):
    H, W = 96, 128
    px, _, _ = flow_fullscreen(H, W, FLOW_CAMS[name])
    ref, rdy = oceanic_f64.render_opt_flow_fullscreen(H, W, FLOW_CAMS[name])
    assert np.isfinite(px).all()
    err = np.abs(px[0, ..., :2] - ref)
    tol = 1e-3 + 1e-5 * np.abs(ref)
    assert (err <= tol).mean() >= 0.999 and np.median(err) < 1e-4
    if name == "translate":
        # a translating camera does not move the sky (old_rd = rd and the angles are unchanged, :1349-1351):
        # sky pixels map to themselves, water pixels move
        jj, ii = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
        own = np.stack([ii + 0.5, (H - 1 - jj) + 0.5], -1)
        sky, water = rdy > 1e-3, rdy < -1e-3
        assert sky.any() and water.any()
        np.testing.assert_allclose(px[0, ..., :2][sky], own[sky], atol=2e-3)
        assert np.abs(px[0, ..., :2][water] - own[water]).max() > 1.0


def test_opt_flow_channels_and_uncovered_pixels():
    bg, v, c, f = scenes.random_triangles(F=80, W=96, H=64, C=4, radius_px=14.0, seed=6)
    px, gb, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None], shader_id=6,
                                     camera_pos=np.array(FLOW_CAMS["rotate"], np.float32))
    cov = gb[0] >= 0
    assert 0.1 < cov.mean() < 0.9
    np.testing.assert_array_equal(px[0][~cov], bg[~cov])
    assert (px[0, ..., 2][cov] == 0).all() and (px[0, ..., 3][cov] == 1).all()
    with pytest.raises(ValueError, match="16"):
        oracle.rasterise_fwd(bg[None], v[None], c[None], f[None], shader_id=6, camera_pos=np.zeros(15, np.float32))


HILL_CAMS = {"harness": [0, 0, 3], "high": [1, -2, 6], "low": [2, 5, 2]}


def hill_cam(o):
    cam = np.zeros(12, np.float32)
    cam[:9] = np.arange(9) * 0.1 + 7.0  # r00..r22: shadowed by main()'s constants (shaders.cpp:473-481)
    cam[9:] = o
    return cam


@pytest.mark.parametrize("Ct", [1, 3, 4])
@pytest.mark.parametrize("shape", [(54, 96), (64, 64)], ids=["16x9", "square_letterbox"])
@pytest.mark.parametrize("name", sorted(HILL_CAMS))
def test_hill_against_float64(name, shape, Ct):
    """Sky pixels and the letterbox are noise-free (1e-5 / exact); the grass is driven by hashes that turn
    any rounding difference into a different random value, so terrain pixels are pinned by their mean."""
    H, W = shape
    T = scenes.hill_terrain(H, W, Ct)
    v, f = scenes.fullscreen_quad()
    px, gb, st = oracle.hill_fwd(T[None], v[None], f[None], 4, hill_cam(HILL_CAMS[name]))
    assert st == 0 and (gb >= 0).all()
    ref, hit, box = oceanic_f64.render_hill_fullscreen(T, hill_cam(HILL_CAMS[name]))
    p = px[0]
    assert np.isfinite(p).all()
    assert (p[box] == 0).all()
    sky = ~hit & ~box
    assert 0.1 < sky.mean() and 0.1 < hit.mean()
    assert np.abs(p[sky] - ref[sky]).max() <= 1e-5
    assert np.abs(p[hit].mean(0) - ref[hit].mean(0)).max() <= 0.02
    assert (p[~box][:, 3] == 1).all()
    if shape == (64, 64):
        assert 0.4 < box.mean() < 0.5  # |2 y - 1| >= 0.5625 rows (shaders.cpp:458)


def test_hill_no_depth_test_last_face_wins():
    """hill.cpp:194 leaves GL_DEPTH_TEST off: overlapping faces resolve in draw order (the last one wins),
    unlike Rasterise's depth LESS; pixels no face covers stay 0 (the colour attachment is never cleared
    nor given the background)."""
    H, W = 32, 48
    T = scenes.hill_terrain(H, W, 4)
    near = [[-0.5, -0.5, -0.5, 1], [-0.5, 0.5, -0.5, 1], [0.5, 0.5, -0.5, 1], [0.5, -0.5, -0.5, 1]]
    far = [[-0.8, -0.8, 0.5, 1], [-0.8, 0.8, 0.5, 1], [0.8, 0.8, 0.5, 1], [0.8, -0.8, 0.5, 1]]
    v = np.array(near + far, np.float32)
    f = np.array([[0, 1, 2], [0, 2, 3], [4, 5, 6], [4, 6, 7]], np.int32)
    px, gb, _ = oracle.hill_fwd(T[None], v[None], f[None], 3, hill_cam([0, 0, 3]))
    inner = gb[0, 12:20, 18:30]
    assert ((inner == 2) | (inner == 3)).all()  # the far quad, drawn last
    assert (gb[0, 0, :] == -1).all() and (px[0, 0, :] == 0).all()
    c = np.ones((1, 8, 3), np.float32)
    _, gg, _ = oracle.rasterise_fwd(np.zeros((1, H, W, 3), np.float32), v[None], c, f[None])
    assert ((gg[0, 12:20, 18:30] == 0) | (gg[0, 12:20, 18:30] == 1)).all()  # depth LESS: the near quad


def test_hill_camera_and_channel_checks():
    T = scenes.hill_terrain(8, 8, 4)
    v, f = scenes.fullscreen_quad()
    with pytest.raises(ValueError, match="12"):
        oracle.hill_fwd(T[None], v[None], f[None], 3, np.zeros(11, np.float32))
