"""CPU tests of the oracle (oracle/dirt_oracle.c): known-answer tests derived from the reference, finite
differences of the filter-based gradient, and regression against the committed golden fixtures.

Pins:
  * README square (README.md:27-70): a 16x16 block of 1.0 at rows 56..71, cols 24..39 of 128x128x1.
  * translation KATs (README.md:41): d(sum pixels)/d centre = 0 and d(sum pixels*x)/d centre_x = area.
  * cylinder (tests/rasterise_tests.py:79-132): d/d bgcolor and d/d vertex_color exact (linear).
  * finite differences of pose parameters on pixels away from every face boundary (rasterise_tests.py:91-132
    visualises exactly these Jacobians; here they are asserted).
"""
import glob
import os

import numpy as np
import pytest
import torch

import scenes
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fwd(scene):
    bg, v, c, f = (a[None] for a in scene)
    px, gb, st = oracle.rasterise_fwd(bg, v, c, f)
    assert st == 0
    return px, gb


def test_readme_square_kat():
    px, gb = _fwd(scenes.readme_square())
    expect = np.zeros((128, 128), np.float32)
    expect[56:72, 24:40] = 1.0
    np.testing.assert_array_equal(px[0, :, :, 0], expect)
    assert set(np.unique(gb[0])) == {-1, 0, 1}  # two triangles, background elsewhere


@pytest.mark.parametrize("centre", [(32.0, 64.0), (32.25, 63.5), (100.7, 20.1)])
def test_square_translation_gradient_kats(centre):
    W = H = 128
    bg, v, c, f = (a[None] for a in scenes.readme_square(centre=centre))
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    area = float(px.sum())
    xs = np.broadcast_to(np.arange(W, dtype=np.float32)[None, None, :, None], px.shape).copy()
    rows = np.broadcast_to(np.arange(H, dtype=np.float32)[None, :, None, None], px.shape).copy()
    # d/d centre (pixels) = sum_k dL/dclip_k * 2/W
    gv, _, _ = oracle.rasterise_bwd(v, c, f, px, np.ones_like(px), gb)
    assert abs(gv[0, :, 0].sum() * 2 / W) < 1e-4 and abs(gv[0, :, 1].sum() * 2 / H) < 1e-4
    gv, _, _ = oracle.rasterise_bwd(v, c, f, px, xs, gb)
    assert gv[0, :, 0].sum() * 2 / W == pytest.approx(area, rel=1e-5)
    gv, _, _ = oracle.rasterise_bwd(v, c, f, px, rows, gb)
    assert gv[0, :, 1].sum() * 2 / H == pytest.approx(-area, rel=1e-5)  # rows grow downwards, window y up
    # scaling every w by (1+e) shrinks the square's NDC area by (1+e)^-2
    gv, _, _ = oracle.rasterise_bwd(v, c, f, px, np.ones_like(px), gb)
    assert gv[0, :, 3].sum() == pytest.approx(-2 * area, rel=1e-5)


def test_cylinder_background_and_colour_gradients_exact():
    bg, v, c, f = (a[None] for a in scenes.cylinder_scene())
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    G = np.random.default_rng(0).standard_normal(px.shape).astype(np.float32)
    gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, G, gb)
    covered = gb[0] >= 0
    np.testing.assert_array_equal(gbg[0][~covered], G[0][~covered])
    np.testing.assert_array_equal(gbg[0][covered], 0.0)
    # L = sum G*pixels is linear in the background and in the vertex colours
    d_bgcolor = (G[0][: 18] * (~covered[: 18])[..., None]).sum(axis=(0, 1))  # top half = bgcolor (rasterise_tests.py:88)
    tiled = np.zeros_like(bg)
    tiled[0, :18] = 1.0
    np.testing.assert_allclose((gbg * tiled).sum(axis=(0, 1, 2)), d_bgcolor, rtol=1e-6)
    eps = 1.0
    for ch in range(3):
        c2 = c.copy()
        c2[0, :75, ch] += eps
        px2, _, _ = oracle.rasterise_fwd(bg, v, c2, f)
        fd = float(((px2 - px) * G).sum()) / eps
        assert gc[0, :75, ch].sum() == pytest.approx(fd, rel=1e-4, abs=1e-4)


def _interior_mask(gb, r=2):
    """Pixels whose (2r+1)^2 neighbourhood shows one single face."""
    g = gb[0]
    H, W = g.shape
    m = g >= 0
    for dy in range(-r, r + 1):
        for dx in range(-r, r + 1):
            sh = np.full_like(g, -7)
            sh[max(0, -dy):H - max(0, dy), max(0, -dx):W - max(0, dx)] = g[max(0, dy):H - max(0, -dy) or None,
                                                                             max(0, dx):W - max(0, -dx) or None]
            m &= sh == g
    return m


@pytest.mark.parametrize("param", ["tx", "ty", "tz", "rot"])
def test_cylinder_pose_gradient_matches_finite_differences(param):
    """d(sum G*pixels)/d pose on pixels away from every face boundary (smooth Gouraud interior), chained
    through the differentiable projection of tests/rasterise_tests.py:49-77, against central differences."""
    W, H = 192, 144
    T0 = torch.tensor([0.0, 0.0, -0.25])
    R0 = torch.tensor(0.3)

    def clip_of(T, R):
        cv, cf = scenes.cylinder_clip_vertices(T, R, W, H)
        return cv, cf

    T = T0.clone().requires_grad_(True)
    R = R0.clone().requires_grad_(True)
    cv, cf = clip_of(T, R)
    V = cv.shape[0]
    cols = np.random.default_rng(1).uniform(size=(V, 3)).astype(np.float32)
    bg = np.zeros((H, W, 3), np.float32)
    v_np = cv.detach().numpy().astype(np.float32)
    f_np = cf.numpy().astype(np.int32)
    px, gb, _ = oracle.rasterise_fwd(bg[None], v_np[None], cols[None], f_np[None])
    mask = _interior_mask(gb)
    assert mask.sum() > 200
    G = np.random.default_rng(2).standard_normal(px.shape).astype(np.float32) * mask[None, ..., None]
    gv, _, _ = oracle.rasterise_bwd(v_np[None], cols[None], f_np[None], px, G, gb)
    gT, gR = torch.autograd.grad(cv, [T, R], torch.from_numpy(gv[0]))
    analytic = {"tx": gT[0], "ty": gT[1], "tz": gT[2], "rot": gR}[param].item()

    h = {"tx": 2e-4, "ty": 2e-4, "tz": 2e-4, "rot": 5e-4}[param]

    def loss(delta):
        Tq, Rq = T0.clone(), R0.clone()
        if param == "rot":
            Rq = Rq + delta
        else:
            Tq[{"tx": 0, "ty": 1, "tz": 2}[param]] += delta
        vq, _ = clip_of(Tq, Rq)
        p, g2, _ = oracle.rasterise_fwd(bg[None], vq.detach().numpy().astype(np.float32)[None], cols[None], f_np[None])
        assert np.array_equal(g2[0][mask], gb[0][mask])  # no visibility change on the tested pixels
        return float((p.astype(np.float64) * G).sum())

    fd = (loss(h) - loss(-h)) / (2 * h)
    assert analytic == pytest.approx(fd, rel=5e-2, abs=1e-3 * max(1.0, abs(fd)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_oracle_reproduces_golden_fixture(path):
    z = np.load(path)  # allow_pickle=False (default): data only
    px, gb, st = oracle.rasterise_fwd(z["background"], z["vertices"], z["vertex_colors"], z["faces"])
    assert st == 0
    np.testing.assert_array_equal(px, z["pixels"])
    np.testing.assert_array_equal(gb, z["gbuffer"])
    gv, gc, gbg = oracle.rasterise_bwd(z["vertices"], z["vertex_colors"], z["faces"], px, z["grad_pixels"], gb)
    np.testing.assert_array_equal(gbg, z["grad_background"])
    for a, b in ((gv, z["grad_vertices"]), (gc, z["grad_vertex_colors"])):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6 * max(1.0, float(np.abs(b).max())))


def test_oracle_empty_and_degenerate_inputs():
    bg, v, c, f = scenes.random_triangles(F=20, W=32, H=24, seed=2)
    px, gb, st = oracle.rasterise_fwd(bg[None], v[None], c[None], f[:0][None])
    np.testing.assert_array_equal(px[0], bg)
    assert (gb == -1).all() and st == 0
    f2 = f.copy()
    f2[0] = [0, 0, 0]
    f2[1] = [0, 1, 99999]
    px, gb, st = oracle.rasterise_fwd(bg[None], v[None], c[None], f2[None])
    assert st == 2  # out-of-range index reported, face culled
    assert not np.isin(gb[0] & ((1 << 30) - 1), [0, 1]).any()


@pytest.mark.parametrize("fill", [float("-inf"), float("nan")])
def test_non_finite_background_rule(fill):
    """a background pixel holding a non-finite value (samples/deferred.py:67,81 renders over
    -inf) defines no image difference, so its pixel pairs carry no vertex gradient.  README square over
    -inf with a constant colour: the silhouette pairs are the only ones with a non-zero difference, so the
    vertex gradient is exactly 0 (over a finite background it is the translation / area KAT above)."""
    bg, v, c, f = (a[None] for a in scenes.readme_square())
    bg = np.full_like(bg, fill)
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    assert np.isnan(px[0, 0, 0, 0]) if np.isnan(fill) else px[0, 0, 0, 0] == fill
    gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, np.ones_like(px), gb)
    assert np.all(gv == 0.0)
    # colour and background gradients do not depend on the background's values
    px0, gb0, _ = oracle.rasterise_fwd(np.zeros_like(bg), v, c, f)
    gv0, gc0, gbg0 = oracle.rasterise_bwd(v, c, f, px0, np.ones_like(px0), gb0)
    np.testing.assert_array_equal(gc, gc0)
    np.testing.assert_array_equal(gbg, gbg0)
    # a random scene over a partly non-finite background: every gradient finite
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=300, W=64, H=48, radius_px=8.0, seed=2))
    bg = bg.copy()
    bg[0, ::2, ::3, 0] = fill
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    g = np.random.default_rng(0).standard_normal(px.shape).astype(np.float32)
    gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, g, gb)
    assert np.all(np.isfinite(gv)) and np.all(np.isfinite(gc)) and np.abs(gv).max() > 0


def test_gbuffer_outputs_consistent():
    """oracle.rasterise_fwd_gbuffer (the checker of dirt_rasterise_fwd_gbuffer): depth is the DEPTH24 value
    as float (1.0 uncovered), barycentrics interpolate the Gouraud pixels, face ids name the visible face."""
    bg, v, c, f = scenes.random_triangles(F=400, W=80, H=64, radius_px=9.0, seed=4, perspective=True)
    px, gb, depth, bary, face, st = oracle.rasterise_fwd_gbuffer(bg[None], v[None], c[None], f[None])
    px2, gb2, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
    np.testing.assert_array_equal(px, px2)
    np.testing.assert_array_equal(gb, gb2)
    cov = face[0] >= 0
    assert np.array_equal(cov, gb[0] >= 0)
    assert np.all(depth[0][~cov] == 1.0) and np.all(bary[0][~cov] == 0)
    d24 = np.round(depth[0][cov].astype(np.float64) * (2 ** 24 - 1))
    assert np.abs(d24 - depth[0][cov] * (2 ** 24 - 1)).max() < 2.0  # a 24-bit quantum
    interp = np.einsum("nk,nkc->nc", bary[0][cov], c[f[face[0][cov]]])
    np.testing.assert_allclose(interp, px[0][cov], rtol=1e-5, atol=1e-5)
    # README square: z = 0 -> window depth 0.5, quantised
    _, _, depth, _, face, _ = oracle.rasterise_fwd_gbuffer(*(a[None] for a in scenes.readme_square()))
    assert set(np.unique(face)) == {-1, 0, 1}
    assert np.all(depth[face >= 0] == np.float32(np.float32(8388608) / np.float32(16777215)))


@pytest.mark.parametrize("perspective", [False, True])
@pytest.mark.parametrize("centre_snap", [False, True])
def test_oracle_coverage_matches_exact_integer_rule(centre_snap, perspective):
    """The oracle's visible face on watertight meshes equals the exact-integer statement of R1-R3 in
    tests/exact_cover.py (Python ints, independent of oracle/dirt_oracle.c), and the rule is watertight:
    every pixel centre strictly inside the mesh lies in exactly one triangle, shared edges and vertices on
    pixel centres included."""
    from exact_cover import exact_cover, grid_mesh, snap
    H, W = 80, 96
    v, faces = grid_mesh(7, 6, W, H, seed=11 + 2 * centre_snap + perspective, perspective=perspective,
                         centre_snap=centre_snap)
    count, first = exact_cover(v, faces, W, H)
    X, Y = snap(v, W, H)
    pxc, pyc = np.arange(W) * 256 + 128, (np.arange(H) * 256 + 128)[::-1]
    strict = ((pxc[None, :] > X.min()) & (pxc[None, :] < X.max())) & ((pyc[:, None] > Y.min()) & (pyc[:, None] < Y.max()))
    assert count.max() == 1 and np.all(count[strict] == 1)
    rng = np.random.default_rng(3)
    bg = rng.uniform(0, 1, (1, H, W, 3)).astype(np.float32)
    cols = rng.uniform(0, 1, (1, len(v), 3)).astype(np.float32)
    face = oracle.rasterise_fwd_gbuffer(bg, v[None], cols, faces[None])[4][0]
    np.testing.assert_array_equal(face, first)
