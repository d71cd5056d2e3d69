"""GPU: analytic pins of the HIP path that do not go through the C oracle.

The reference ships no golden vectors and cannot run here, so besides the oracle comparisons these
tests check the HIP kernels against properties that follow from the raster rules or from the
algebra of the backward alone:

* coverage by exact integer arithmetic in Python (R1/R2 snapping in numpy float32, R3 edge functions and the
  top-left rule on Python ints): the face the HIP resolve reports at every pixel is the unique face whose
  snapped triangle contains the pixel centre, on watertight meshes (shared vertices, jittered interior, edges
  through pixel centres, affine and perspective w).  GL requires exactly this watertightness of a shared
  edge (every sample on it belongs to one of its two triangles), which the oracle does not test by itself;
* the backward is linear in grad_pixels (BASELINE config 3 at full size: one frame of 1024x1024x3, 50k tris);
* with grad_pixels = 1 the colour gradient of a channel sums to the number of covered pixels (the
  barycentrics of a pixel sum to 1) and grad_background is exactly the uncovered mask (full size).
"""
import numpy as np
import pytest
import torch

import scenes
from exact_cover import F32, exact_cover, grid_mesh, snap
from test_gpu_parity import RTOL, ATOL_REL, _gpu

pytestmark = pytest.mark.gpu

@pytest.mark.parametrize("perspective", [False, True])
@pytest.mark.parametrize("centre_snap", [False, True])
@pytest.mark.parametrize("shape", [(80, 96, 7, 6), (64, 48, 7, 5)])
def test_watertight_mesh_coverage_exact(shape, centre_snap, perspective):
    import dirt_amd
    H, W, nx, ny = shape
    v, faces = grid_mesh(nx, ny, W, H, seed=H + nx + 2 * centre_snap + perspective, perspective=perspective,
                          centre_snap=centre_snap)
    count, first = exact_cover(v, faces, W, H)
    # the rule itself is watertight: no pixel centre in two triangles of the mesh, none in a hole
    assert count.max() == 1
    X, Y = snap(v, W, H)
    # pixel centres strictly inside the mesh's outer rectangle (its corners are not jittered)
    x0, x1 = X.min(), X.max()
    y0, y1 = Y.min(), Y.max()
    pxc = np.arange(W) * 256 + 128
    pyc = (np.arange(H) * 256 + 128)[::-1]
    strict = ((pxc[None, :] > x0) & (pxc[None, :] < x1)) & ((pyc[:, None] > y0) & (pyc[:, None] < y1))
    assert strict.any() and np.all(count[strict] == 1)
    C = 3
    rng = np.random.default_rng(7)
    bg = rng.uniform(0, 1, (H, W, C)).astype(F32)
    cols = rng.uniform(0, 1, (len(v), C)).astype(F32)
    g = dirt_amd.rasterise_gbuffer(_gpu(bg), _gpu(v), _gpu(cols), _gpu(faces))
    face = g.face_ids.cpu().numpy()
    np.testing.assert_array_equal(face, first)
    # uncovered pixels copy the background; covered ones interpolate (colours in [0, 1])
    px = g.pixels.cpu().numpy()
    np.testing.assert_array_equal(px[first < 0], bg[first < 0])


def _full_c3(seed=0):
    bg, v, c, f = scenes.random_triangles(F=50000, W=1024, H=1024, C=3, radius_px=16.0, seed=seed)
    return _gpu(bg).requires_grad_(True), _gpu(v).requires_grad_(True), _gpu(c).requires_grad_(True), _gpu(f)


def _grads(bg, v, c, f, g):
    import dirt_amd
    px = dirt_amd.rasterise(bg, v, c, f)
    return [t.double().cpu().numpy() for t in torch.autograd.grad(px, [bg, v, c], g)]


def test_backward_linear_in_grad_pixels_full_c3():
    """bwd(g1 + 2 g2) = bwd(g1) + 2 bwd(g2) at BASELINE config 3's full size (the sums are accumulated by
    float atomics in a different order each run, so the test allows the DESIGN.md 5 tolerance)."""
    bg, v, c, f = _full_c3(seed=0)
    gen = torch.Generator(device="cuda").manual_seed(5)
    g1 = torch.randn(bg.shape, device="cuda", generator=gen)
    g2 = torch.randn(bg.shape, device="cuda", generator=gen)
    a = _grads(bg, v, c, f, g1)
    b = _grads(bg, v, c, f, g2)
    ab = _grads(bg, v, c, f, g1 + 2.0 * g2)
    for name, x, y, z in zip(("grad_background", "grad_vertices", "grad_vertex_colors"), a, b, ab):
        want = x + 2.0 * y
        assert np.all(np.isfinite(z)), name
        scale = np.abs(want).max()
        err = np.abs(z - want)
        tol = 4 * RTOL * np.abs(want) + 4 * ATOL_REL * scale
        assert np.all(err <= tol), "%s: max err %g (scale %g)" % (name, err.max(), scale)


def test_colour_gradient_sums_to_coverage_full_c3():
    """grad_pixels = 1: every covered pixel's barycentrics sum to 1, so sum_v dL/dcolour[v, ch] = covered pixel
    count for each channel; grad_background is exactly the uncovered mask (full config 3 frame)."""
    import dirt_amd
    bg, v, c, f = _full_c3(seed=1)
    px, gb = dirt_amd.rasterise_ops._rasterise_batched(bg[None], v[None], c[None], f[None], None, 1024, 1024, 3, 0, 0,
                                                       return_gbuffer=True)
    covered = (gb[0] >= 0).cpu().numpy()
    gbg, gc = torch.autograd.grad(px, [bg, c], torch.ones_like(px))
    gbg, gc = gbg.cpu().numpy(), gc.double().cpu().numpy()
    np.testing.assert_array_equal(gbg, np.broadcast_to((~covered)[..., None], gbg.shape).astype(F32))
    n = covered.sum()
    assert 0.5 * covered.size < n < covered.size
    sums = gc.sum(axis=0)
    np.testing.assert_allclose(sums, np.full(3, float(n)), rtol=1e-4)
