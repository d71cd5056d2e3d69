"""GPU counterpart of the reference's tests/rasterise_tests.py, with the assertions the reference lacks.

The reference renders the 48x36 split cylinder (rasterise_tests.py:11-77) once with `rasterise` over a
half-bgcolor background (:88) and once as a 2-frame `rasterise_batch` (:89), then builds the full Jacobian
of the pixels w.r.t. translation (3), rotation, bgcolor (3) and vertex_color (3) from one-hot
d_loss/d_pixels, one pixel and channel at a time (:91-132), and only displays it.  Here the same
Jacobians go through the public autograd API on the GPU (dirt_amd.rasterise / rasterise_batch, the HIP
kernels behind the C ABI) and are asserted:
  * bgcolor, vertex_color: the op is linear in them, so every one-hot Jacobian row is exact -- background
    rows are 1 exactly on uncovered pixels of the tinted half, colour rows sum the perspective-correct
    barycentrics of the 75 tinted vertices (1 within rounding on pixels showing only tinted vertices);
  * the batch renders each frame as the single-frame call does (bit-exact) and its Jacobians match;
  * pose: the summed one-hot rows (d sum(G * pixels) / d pose for a mask G of boundary-free pixels)
    against central differences of the GPU forward itself (the oracle's version is tests/test_oracle.py).
"""
import numpy as np
import pytest
import torch

import dirt_amd
import scenes

pytestmark = pytest.mark.gpu

W, H = 48, 36
BGCOLOR = (0.4, 0.2, 0.2)
VCOLOR = (0.7, 0.3, 0.6)


def _inputs(translation=(0., 0., -0.25), rotation=0.0, W=W, H=H):
    dev = torch.device("cuda", 0)
    T = torch.tensor(translation, dtype=torch.float32, requires_grad=True)
    R = torch.tensor(rotation, dtype=torch.float32, requires_grad=True)
    clip, faces = scenes.cylinder_clip_vertices(T, R, W, H)
    V = clip.shape[0]
    bgcolor = torch.tensor(BGCOLOR, device=dev, requires_grad=True)
    vcolor = torch.tensor(VCOLOR, device=dev, requires_grad=True)
    rest = torch.from_numpy(np.random.RandomState(0).uniform(size=[V - 75, 3]).astype(np.float32)).to(dev)
    colors = torch.cat([vcolor[None].expand(75, 3), rest], 0)  # rasterise_tests.py:81-86
    background = torch.cat([bgcolor[None, None].expand(H // 2, W, 3),
                            torch.ones(H - H // 2, W, 3, device=dev)], 0)  # :88
    return T, R, clip.to(dev), faces.to(dev, torch.int32), bgcolor, vcolor, colors, background


def _render_single(W=W, H=H):
    T, R, clip, faces, bgcolor, vcolor, colors, background = _inputs(W=W, H=H)
    pixels = dirt_amd.rasterise(background, clip, colors, faces, height=H, width=W, channels=3)
    return pixels, (T, R, bgcolor, vcolor)


def _render_batch():
    T, R, clip, faces, bgcolor, vcolor, colors, background = _inputs()
    # rasterise_tests.py:89: the same mesh twice, each frame indexing its own vertices
    pixels = dirt_amd.rasterise_batch(torch.stack([background] * 2), torch.stack([clip] * 2),
                                      torch.stack([colors] * 2), torch.stack([faces] * 2),
                                      height=H, width=W, channels=3)
    return pixels, (T, R, bgcolor, vcolor)


def _jacobian_rows(pixels, params, frame=None, pixel_list=None):
    """One-hot d_loss/d_pixels rows (rasterise_tests.py:91-132) for the given (y, x, c) entries."""
    rows = []
    for (y, x, c) in pixel_list:
        g = torch.zeros_like(pixels)
        if frame is None:
            g[y, x, c] = 1.0
        else:
            g[frame, y, x, c] = 1.0
        grads = torch.autograd.grad(pixels, params, g, retain_graph=True, allow_unused=True)
        rows.append(torch.cat([torch.zeros(np.prod(p.shape)) if gr is None else gr.detach().reshape(-1).cpu()
                               for p, gr in zip(params, grads)]))
    return torch.stack(rows).numpy()  # columns: tx ty tz | rot | bgcolor rgb | vertex_color rgb


def _gbuffer_single(W=W, H=H):
    _, _, clip, faces, _, _, colors, background = _inputs(W=W, H=H)
    _, gb = dirt_amd.rasterise_ops._rasterise_batched(background[None].detach(), clip[None].detach(),
                                                     colors[None].detach(), faces[None], None, H, W, 3, 0,
                                                     return_gbuffer=True)
    return gb[0].cpu().numpy()


def test_single_frame_bgcolor_and_vertex_color_jacobians_exact():
    pixels, params = _render_single()
    gb = _gbuffer_single()
    covered = gb >= 0
    # every pixel of the tinted top half and a band of the bottom half, all channels
    entries = [(y, x, c) for y in range(0, H, 2) for x in range(0, W, 3) for c in range(3)]
    J = _jacobian_rows(pixels, params, pixel_list=entries)
    for row, (y, x, c) in zip(J, entries):
        d_bg = row[4:7]
        want = np.zeros(3, np.float32)
        if not covered[y, x] and y < H // 2:
            want[c] = 1.0
        np.testing.assert_array_equal(d_bg, want)
        d_vc = row[7:10]
        assert d_vc[[k for k in range(3) if k != c]].tolist() == [0.0, 0.0]  # channel-diagonal
        if not covered[y, x]:
            assert d_vc[c] == 0.0  # (a background pixel next to an edge still has a pose gradient)
        else:
            assert -1e-6 <= d_vc[c] <= 1.0 + 1e-5  # a sum of barycentrics of tinted vertices
    # the tinted half of the mesh shows up: some covered pixels take all their colour from VCOLOR
    full = [row[7 + c] for row, (y, x, c) in zip(J, entries) if covered[y, x] and abs(row[7 + c] - 1.0) < 1e-5]
    assert len(full) > 10


def test_batch_of_two_frames_matches_single_frame():
    p1, params1 = _render_single()
    p2, params2 = _render_batch()
    assert p2.shape == (2, H, W, 3)
    torch.testing.assert_close(p2[0], p1, rtol=0, atol=0)
    torch.testing.assert_close(p2[1], p1, rtol=0, atol=0)
    entries = [(y, x, c) for y in range(1, H, 5) for x in range(1, W, 5) for c in range(3)]
    J1 = _jacobian_rows(p1, params1, pixel_list=entries)
    for fr in range(2):
        J2 = _jacobian_rows(p2, params2, frame=fr, pixel_list=entries)
        # bgcolor / vertex_color rows exact; pose rows equal up to float atomics order
        np.testing.assert_array_equal(J2[:, 4:], J1[:, 4:])
        np.testing.assert_allclose(J2[:, :4], J1[:, :4], rtol=1e-5, atol=1e-6)


def _interior_mask(gb, r=2):
    H, W = gb.shape
    m = gb >= 0
    for dy in range(-r, r + 1):
        for dx in range(-r, r + 1):
            sh = np.full_like(gb, -7)
            sh[max(0, -dy):H - max(0, dy), max(0, -dx):W - max(0, dx)] = gb[max(0, dy):H - max(0, -dy) or None,
                                                                            max(0, dx):W - max(0, -dx) or None]
            m &= sh == gb
    return m


@pytest.mark.parametrize("param", ["tx", "ty", "tz", "rot"])
def test_pose_jacobian_matches_gpu_finite_differences(param):
    """Summed one-hot pose rows over boundary-free pixels (random weights G) against central differences
    of the GPU forward (fp64 sums of its float32 pixels), at 192x144 so that faces have interiors."""
    W, H = 192, 144
    pixels, params = _render_single(W, H)
    gb = _gbuffer_single(W, H)
    mask = _interior_mask(gb)
    assert mask.sum() > 200
    G = np.random.default_rng(3).standard_normal((H, W, 3)).astype(np.float32) * mask[..., None]
    grads = torch.autograd.grad(pixels, params[:2], torch.from_numpy(G).cuda())
    analytic = {"tx": grads[0][0], "ty": grads[0][1], "tz": grads[0][2], "rot": grads[1]}[param].item()
    h = {"tx": 2e-4, "ty": 2e-4, "tz": 2e-4, "rot": 5e-4}[param]

    def loss(delta):
        t = [0., 0., -0.25]
        rot = 0.0
        if param == "rot":
            rot += delta
        else:
            t[{"tx": 0, "ty": 1, "tz": 2}[param]] += delta
        _, _, clip, faces, _, _, colors, background = _inputs(tuple(t), rot, W, H)
        p, g2 = dirt_amd.rasterise_ops._rasterise_batched(background[None].detach(), clip[None].detach(),
                                                         colors[None].detach(), faces[None], None, H, W, 3, 0,
                                                         return_gbuffer=True)
        assert np.array_equal(g2[0].cpu().numpy()[mask], gb[mask])  # no visibility change on tested pixels
        return float((p[0].double().cpu().numpy() * G).sum())

    fd = (loss(h) - loss(-h)) / (2 * h)
    assert analytic == pytest.approx(fd, rel=5e-2, abs=1e-3 * max(1.0, abs(fd)))
