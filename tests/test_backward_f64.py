"""CPU pin of the backward: the oracle (oracle/dirt_oracle.c) against an independent float64 restatement of the
specification (tests/backward_f64.py), DESIGN.md 4 / SURVEY Appendix B.

The reference registers no gradient, so nothing reference-held pins the backward; this is the
second statement of it, written from the spec in float64 (normalised perspective-correct barycentrics, the
clip w of the pair midpoint, the chain rule through the window transform) -- the oracle evaluates the same
quantities in float32 through the cancellation-free identity lambda_k / Wm = a_k / (2D).  Contract:
  * grad_background identical;
  * grad_vertices and grad_vertex_colors within 1e-6 of the gradient's scale (max |float64|), on every golden
    scene, the fuzz scene that exposed the normalised form's cancellation (seed 37851, a 1811-unit sliver) and
    50 clipped-sliver scenes (guard-band and near-plane clipping; the old normalised clipped weight failed 9
    of them, up to 8.6e-6: profiles/r04/f64_pin.txt).
"""
import glob
import os

import numpy as np
import pytest

import backward_f64
import scenes
from oracle import oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PIN = 1e-6


def check_pin(bg, v, c, f, seed):
    gp = np.random.default_rng(seed).standard_normal(bg.shape).astype(np.float32)
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    gv64, gc64, gbg64 = backward_f64.backward_batch(v, f, px, gp, gb)
    gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, gp, gb)
    np.testing.assert_array_equal(gbg, gbg64.astype(np.float32))
    ev, ec = backward_f64.max_rel_err(gv, gv64), backward_f64.max_rel_err(gc, gc64)
    assert ev <= PIN, "grad_vertices: %.3g of the scale vs float64" % ev
    assert ec <= PIN, "grad_vertex_colors: %.3g of the scale vs float64" % ec
    return gb


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_f64_pin_golden_scenes(path):
    z = np.load(path)
    gp = z["grad_pixels"]
    gv64, gc64, gbg64 = backward_f64.backward_batch(z["vertices"], z["faces"], z["pixels"], gp, z["gbuffer"])
    np.testing.assert_array_equal(z["grad_background"], gbg64.astype(np.float32))
    # the committed fixture (oracle output) and a fresh oracle run
    gv, gc, _ = oracle.rasterise_bwd(z["vertices"], z["vertex_colors"], z["faces"], z["pixels"], gp, z["gbuffer"])
    for a, b, name in ((z["grad_vertices"], gv64, "fixture grad_vertices"), (z["grad_vertex_colors"], gc64,
                       "fixture grad_vertex_colors"), (gv, gv64, "grad_vertices"), (gc, gc64, "grad_vertex_colors")):
        e = backward_f64.max_rel_err(a, b)
        assert e <= PIN, "%s: %.3g of the scale vs float64" % (name, e)


def test_f64_pin_fuzz_seed_37851():
    """The round-3 fuzz campaign's sliver, rebuilt from its seed: batch of two 64x48 frames, 5
    channels, with clipped faces."""
    bg, v, c, f = scenes.fuzz_case(37851)
    gb = check_pin(bg, v, c, f, 37851)
    assert ((gb >= 0) & ((gb & (1 << 30)) != 0)).any()  # clipped faces are visible


def test_f64_pin_sub_vertex_beyond_guard_band():
    """Fuzz seed 167059 (batch of two 33x17 frames, 5 channels): clipping faces 71 and 115 of frame 0 leaves a
    sub-vertex at x/w = -4.7e6 (w = 7e-12), far outside the guard band; R5's sub-vertex clamp (twice the band)
    keeps its snapped coordinates, and so every edge coefficient, inside the integer ranges both sides assume."""
    bg, v, c, f = scenes.fuzz_case(167059)
    B, H, W, C = bg.shape
    for fi in (71, 115):
        tris, clipped = backward_f64.setup_face(v[0], f[0][fi], v.shape[1], W, H)
        assert clipped and len(tris) == 3
        assert all(abs(x) < 2 ** 25 for t in tris if t is not None for x in t.A + t.B)
    check_pin(bg, v, c, f, 167059)


def test_f64_pin_clip_vertex_cap():
    """scenes.near_w0_scene seed 41533: a face whose clipped polygon exceeds 8 vertices (rounding near w = 0);
    R5's vertex cap culls it in the oracle and in the float64 statement alike."""
    bg, v, c, f = (a[None] for a in scenes.near_w0_scene(41533, W=33, H=17, C=1))
    before = backward_f64.CAP_CULLS[0]
    for fi in range(f.shape[1]):
        backward_f64.setup_face(v[0], f[0][fi], v.shape[1], 33, 17)
    assert backward_f64.CAP_CULLS[0] > before
    check_pin(bg, v, c, f, 41533)


@pytest.mark.parametrize("block", range(5))
def test_f64_pin_clipped_slivers(block):
    """50 scenes of guard-band and near-plane clipped slivers (10 per case)."""
    for seed in range(10 * block, 10 * block + 10):
        bg, v, c, f = (a[None] for a in scenes.clipped_sliver_scene(seed))
        check_pin(bg, v, c, f, seed)


def test_f64_restatement_readme_square_kats():
    """The float64 statement on its own satisfies the README square's translation KATs (README.md:41):
    d(sum pixels)/d centre_x = 0 and d(sum x pixels)/d centre_x = area (256 px, 16x16 square, C = 1)."""
    bg, v, c, f = scenes.readme_square()
    px, gb, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
    H, W = bg.shape[:2]
    ones = np.ones((1, H, W, 1), np.float32)
    xs = np.broadcast_to(np.arange(W, dtype=np.float32)[None, None, :, None], (1, H, W, 1)).copy()
    for g, expect in ((ones, 0.0), (xs, 256.0)):
        gv, _, _ = backward_f64.backward_batch(v[None], f[None], px, g, gb)
        # centre_x moves every vertex's clip x by the same amount: d/dcentre_x in window px = sum_v dL/dx_v * (2/W)
        d = float(gv[0, :, 0].sum()) * 2.0 / W
        assert abs(d - expect) <= 1e-9 + 0.05 * abs(expect), (d, expect)
