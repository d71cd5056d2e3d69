"""Asserting GPU counterpart of the reference's tests/lighting_tests.py (a visual test there: it shows four renders
with cv2.imshow and checks nothing).  The same scene: the cylinder of tests/rasterise_tests.py (radius 0.2,
height 0.75, end offset 0.1, bevel 0.2, 32 segments), rotation matrix scaled by 0.5 at angle 0, translation
(0, 0, -0.25), perspective_projection(0.1, 20, 0.2, h / w), 256 x 192, and the four renders:
  normals      vertex colours |vertex_normals|                                        (lighting_tests.py:43)
  directional  diffuse_directional(normals, 1, [1, 0, 0], [1, 1, 0], False) + [0, 0, 0.4]   (:47)
  point        diffuse_point(vertices, normals, 1, [0.5, -1, 0.5], [1, 0.5, 0.9], False) + [0, 0, 0.4]  (:48)
  point_split  the same over split vertices with pre-split (face) normals            (:49)

Asserted instead of looked at: every render bit-exact against the oracle given the same vertex colours; the
helpers on the GPU (fused kernels where they apply) against their framework-op statement on the CPU within
float32 rounding; and what the images should show -- the directional light's red and green equal and its
constant blue exact, the point light's colour ratios 1 : 0.5 : 0.9 preserved by the interpolation, and the
split render covering exactly the pixels of the smooth one (same faces, same order) with different shading.
"""
import numpy as np
import pytest
import torch

import dirt_amd
import scenes
from dirt_amd import lighting, matrices
from oracle import oracle

pytestmark = pytest.mark.gpu

W, H = 256, 192
DEV = torch.device("cuda", 0)


def _scene(device):
    v, f = scenes.make_cylinder(0.2, 0.75, 0.1, 0.2, 32)
    v = torch.as_tensor(np.concatenate([v, np.ones([len(v), 1], np.float32)], 1), device=device)
    f = torch.as_tensor(f, device=device)
    r = 0.0
    rot = torch.tensor([[0.5 * np.cos(r), 0.5 * -np.sin(r), 0., 0.], [0.5 * np.sin(r), 0.5 * np.cos(r), 0., 0.],
                        [0., 0., 0.5, 0.], [0., 0., 0., 1.]], dtype=torch.float32, device=device)
    tr = torch.tensor([[1., 0., 0., 0.], [0., 1., 0., 0.], [0., 0., 1., 0.], [0., 0., -0.25, 1.]], device=device)
    tv = v @ rot @ tr
    proj = matrices.perspective_projection(0.1, 20., 0.2, float(H) / W).to(device)
    nrm = lighting.vertex_normals(tv[:, :3], f)
    tvs, fs = lighting.split_vertices_by_face(tv, f)
    nrm_s = lighting.vertex_normals_pre_split(tvs[:, :3], fs)
    ones = torch.ones((tv.shape[0], 3), device=device)
    ones_s = torch.ones((tvs.shape[0], 3), device=device)
    blue = torch.tensor([0., 0., 0.4], device=device)
    cols = {
        "normals": (tv @ proj, torch.abs(nrm), f),
        "directional": (tv @ proj, lighting.diffuse_directional(nrm, ones, [1., 0, 0], [1., 1., 0.], False) + blue, f),
        "point": (tv @ proj, lighting.diffuse_point(tv[:, :3], nrm, ones, [0.5, -1., 0.5], [1., 0.5, 0.9], False) + blue,
                  f),
        "point_split": (tvs @ proj, lighting.diffuse_point(tvs[:, :3], nrm_s, ones_s, [0.5, -1., 0.5], [1., 0.5, 0.9],
                                                           False) + blue, fs),
    }
    return cols


def test_lighting_tests_scene_renders():
    gpu = _scene(DEV)
    cpu = _scene(torch.device("cpu"))
    bg = torch.zeros((H, W, 3), device=DEV)
    images = {}
    for name, (clip, colours, faces) in gpu.items():
        # the helpers on the GPU against their framework-op statement on the CPU
        c_clip, c_col, _ = cpu[name]
        np.testing.assert_allclose(clip.cpu().numpy(), c_clip.numpy(), rtol=0, atol=2e-6)
        np.testing.assert_allclose(colours.cpu().numpy(), c_col.numpy(), rtol=1e-5, atol=2e-6)
        px = dirt_amd.rasterise(bg, clip, colours, faces.int(), height=H, width=W, channels=3)
        # the render against the oracle with the same inputs: bit-exact
        ref, gb, _ = oracle.rasterise_fwd(bg.cpu().numpy()[None], clip.cpu().numpy()[None],
                                          colours.cpu().numpy()[None], faces.int().cpu().numpy()[None])
        np.testing.assert_array_equal(px.cpu().numpy(), ref[0], err_msg=name)
        images[name] = (ref[0], gb[0] >= 0)
    img, cov = images["normals"]
    assert cov.mean() > 0.05 and np.all(img[~cov] == 0) and np.all((img[cov] >= 0) & (img[cov] <= 1 + 1e-6))
    img, cov = images["directional"]
    # light colour [1, 1, 0] on white: red = green = the clamped cosine; blue the constant 0.4
    np.testing.assert_array_equal(img[..., 0], img[..., 1])
    assert np.abs(img[cov][:, 2] - 0.4).max() < 1e-6
    assert img[cov][:, 0].max() > 0.5 and img[cov][:, 0].min() >= 0
    for name in ("point", "point_split"):
        img, cov = images[name]
        lit = img[cov]
        # colours 1 : 0.5 : 0.9 (plus 0.4 blue) at every vertex; Gouraud interpolation keeps the ratios
        np.testing.assert_allclose(lit[:, 1], 0.5 * lit[:, 0], rtol=0, atol=2e-6)
        np.testing.assert_allclose(lit[:, 2] - 0.4, 0.9 * lit[:, 0], rtol=0, atol=4e-6)
        assert lit[:, 0].max() > 0.3
    (a, ca), (b, cb) = images["point"], images["point_split"]
    np.testing.assert_array_equal(ca, cb)  # the same faces in the same order: the same coverage
    d = np.abs(a[ca, 0] - b[cb, 0])
    assert d.max() > 1e-3 and d.mean() < 0.3  # flat vs smooth normals: different (mean 0.14 here), not unrelated
