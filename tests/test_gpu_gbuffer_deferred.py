"""GPU: the deferred-shading G-buffer outputs, non-finite backgrounds and BASELINE config 4's chain.

* dirt_rasterise_fwd_gbuffer's depth / barycentrics / face ids: bit-exact against the oracle
  (oracle.rasterise_fwd_gbuffer), on plain, perspective, clipped, batched and 7-channel scenes.
* backgrounds holding -inf / NaN (reference samples/deferred.py:67,81): forward bit-exact (non-finite
  values in the same places), gradients finite and within tolerance of the oracle (a
  non-finite background pixel carries no vertex gradient across its pixel pairs).
* samples/deferred.py:62-118 end to end (tests/deferred_pipeline.py): three G-buffer renders, dilation,
  per-pixel lighting, backprop into world-space vertex positions through the normals -- the HIP chain
  against the oracle composed with CPU autograd, and against central finite differences of the HIP
  forward chain on interior pixels.
"""
import os

import numpy as np
import pytest
import torch

import deferred_pipeline as dp
from dirt_amd import lighting
import scenes
from oracle import oracle
from test_gpu_parity import assert_close_grad, check_scene, _gpu

pytestmark = pytest.mark.gpu


def _gbuffer_scene(bg, v, c, f):
    import dirt_amd
    if bg.ndim == 3:
        bg, v, c, f = bg[None], v[None], c[None], f[None]
    g = dirt_amd.rasterise_batch_gbuffer(_gpu(bg), _gpu(v), _gpu(c), _gpu(f))
    px, gb, depth, bary, face, _ = oracle.rasterise_fwd_gbuffer(bg, v, c, f)
    np.testing.assert_array_equal(g.pixels.cpu().numpy(), px)
    np.testing.assert_array_equal(g.face_ids.cpu().numpy(), face)
    np.testing.assert_array_equal(g.depth.cpu().numpy(), depth)
    np.testing.assert_array_equal(g.barycentrics.cpu().numpy(), bary)
    return g, (px, gb, depth, bary, face)


@pytest.mark.parametrize("name", ["square", "cube", "random", "perspective", "clipping", "shared", "c4_7ch"])
def test_gbuffer_outputs_bit_exact(name):
    sc = {"square": scenes.readme_square, "cube": scenes.cube_scene,
          "random": lambda: scenes.random_triangles(F=2000, W=160, H=128, radius_px=12.0, seed=3),
          "perspective": lambda: scenes.random_triangles(F=2000, W=160, H=128, radius_px=12.0, seed=4,
                                                         perspective=True),
          "clipping": scenes.clipping_scene, "shared": scenes.shared_mesh_scene,
          "c4_7ch": scenes.deferred_mesh_scene}[name]()
    g, (px, gb, depth, bary, face) = _gbuffer_scene(*sc)
    cov = face >= 0
    assert cov.any()
    # the G-buffer is self-consistent: uncovered = depth 1 / bary 0; covered barycentrics sum to ~1 and the
    # Gouraud pixels are their interpolation of the visible face's colours
    assert np.all(depth[~cov] == 1.0) and np.all(bary[~cov] == 0.0)
    assert np.all((depth[cov] >= 0.0) & (depth[cov] < 1.0))
    assert np.abs(bary[cov].sum(-1) - 1.0).max() < 1e-5


@pytest.mark.parametrize("seed", range(int(os.environ.get("DIRT_GBUF_W0_FIRST", "0")),
                                         int(os.environ.get("DIRT_GBUF_W0_SEEDS", "4"))))
def test_gbuffer_outputs_near_w0_fuzz(seed):
    """The G-buffer outputs (depth, barycentrics of clipped faces' parents, face ids) on the clipping stress
    scenes around w = 0 (scenes.near_w0_scene), bit-exact against the oracle.  DIRT_GBUF_W0_SEEDS=N widens it
    to the seeds below N (default 4), from DIRT_GBUF_W0_FIRST."""
    W, H = [(64, 48), (33, 17), (130, 70), (1024, 8)][seed % 4]
    _gbuffer_scene(*scenes.near_w0_scene(500000 + seed, W=W, H=H, C=(3, 1, 7, 5)[seed % 4]))


@pytest.mark.parametrize("seed", range(int(os.environ.get("DIRT_GBUF_FUZZ_FIRST", "0")),
                                         int(os.environ.get("DIRT_GBUF_FUZZ_SEEDS", "12"))))
def test_gbuffer_outputs_adversarial_fuzz(seed):
    """The G-buffer instantiation of the raster (depth, barycentrics, face ids) on the adversarial fuzz scenes
    of tests/test_gpu_parity.py (pixel-centre vertices, slivers, ties, clipping, w <= 0, guard-band overflow),
    bit-exact against the oracle.  DIRT_GBUF_FUZZ_SEEDS=N widens it to the seeds below N (default 12),
    from DIRT_GBUF_FUZZ_FIRST."""
    W, H = [(64, 48), (33, 17), (130, 70)][seed % 3]
    C = (3, 7, 1, 5)[seed % 4]
    _gbuffer_scene(*scenes.adversarial_scene(100000 + seed, W=W, H=H, C=C))


def test_gbuffer_batch_and_gradient_unchanged():
    """The G-buffer variant's pixels carry the same gradient as rasterise_batch's."""
    import dirt_amd
    bg, v, c, f = scenes.batch_of(scenes.random_triangles, 3, F=600, W=96, H=80, radius_px=10.0, seed=50)
    _gbuffer_scene(bg, v, c, f)
    gp = np.random.default_rng(2).standard_normal(bg.shape).astype(np.float32)
    outs = []
    for fn in (lambda *a: dirt_amd.rasterise_batch_gbuffer(*a).pixels, dirt_amd.rasterise_batch):
        t = [_gpu(a).requires_grad_(True) for a in (bg, v, c)]
        px = fn(t[0], t[1], t[2], _gpu(f))
        outs.append([x.cpu().numpy() for x in torch.autograd.grad(px, t, _gpu(gp))])
    for a, b in zip(*outs):
        assert_close_grad(a, b, "gbuffer-variant grads")


def test_gbuffer_interpolates_vertex_attributes():
    """Barycentrics x the visible face's vertex colours reproduce the Gouraud pixels (within rounding)."""
    bg, v, c, f = scenes.random_triangles(F=1500, W=128, H=96, radius_px=12.0, seed=5, perspective=True)
    g, (px, gb, depth, bary, face) = _gbuffer_scene(bg, v, c, f)
    cov = face[0] >= 0
    tri = f[face[0][cov]]
    interp = np.einsum("nk,nkc->nc", bary[0][cov], c[tri])
    np.testing.assert_allclose(interp, px[0][cov], rtol=1e-5, atol=1e-5)


def test_gbuffer_argument_checks():
    from dirt_amd import _lib
    bg, v, c, f = scenes.random_triangles(F=40, W=32, H=24, C=3, seed=3)
    t = [_gpu(a[None]) for a in (bg, v, c, f)]
    B, H, W, C, V, F = 1, 24, 32, 3, v.shape[0], f.shape[0]
    saved_b, scratch_b = _lib.workspace_sizes(B, H, W, C, V, F)
    saved = torch.empty(saved_b, dtype=torch.uint8, device="cuda")
    scratch = torch.zeros(scratch_b, dtype=torch.uint8, device="cuda")
    px = torch.empty((B, H, W, C), device="cuda")
    gb = torch.empty((B, H, W), dtype=torch.int32, device="cuda")
    depth = torch.empty((B, H, W), device="cuda")
    lib = _lib.load()
    # depth only (the other two NULL)
    _lib.check(lib.dirt_rasterise_fwd_gbuffer(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(),
                                              B, H, W, C, V, F, px.data_ptr(), gb.data_ptr(), saved.data_ptr(), saved_b,
                                              scratch.data_ptr(), scratch_b, 0, 0, None, None, depth.data_ptr(), None,
                                              None, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    _, _, rd, _, _, _ = oracle.rasterise_fwd_gbuffer(bg[None], v[None], c[None], f[None])
    np.testing.assert_array_equal(depth.cpu().numpy(), rd)
    # errors are return codes (never aborts): a null output pointer
    with pytest.raises(ValueError, match="null"):
        _lib.check(lib.dirt_rasterise_fwd_gbuffer(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(),
                                                  t[3].data_ptr(), B, H, W, C, V, F, None, gb.data_ptr(),
                                                  saved.data_ptr(), saved_b, scratch.data_ptr(), scratch_b, 0, 0,
                                                  None, None, depth.data_ptr(), None, None,
                                                  torch.cuda.current_stream().cuda_stream))


@pytest.mark.parametrize("fill", [float("-inf"), float("inf"), float("nan")])
def test_non_finite_background(fill):
    """G-buffers rendered over -inf (samples/deferred.py:67,81): the forward copies the non-finite
    background; the backward's vertex gradient stays finite and matches the oracle."""
    bg, v, c, f = scenes.random_triangles(F=800, W=96, H=80, radius_px=9.0, seed=61)
    bg = bg.copy()
    bg[:] = fill
    g = check_scene(bg, v, c, f, seed=3)
    assert np.all(np.isfinite(g["grad_vertices"])) and np.all(np.isfinite(g["grad_colors"]))
    assert np.abs(g["grad_vertices"]).max() > 0.0  # interior pairs still carry gradient
    # partly non-finite background: only the pixels holding a non-finite value lose their pairs
    bg2 = scenes.random_triangles(F=800, W=96, H=80, radius_px=9.0, seed=61)[0].copy()
    bg2[::3, ::2, 1] = fill
    g2 = check_scene(bg2, v, c, f, seed=4)
    assert np.all(np.isfinite(g2["grad_vertices"]))


def test_non_finite_background_c4_seven_channels():
    bg, v, c, f = scenes.deferred_mesh_scene(W=160, H=128, n=40)
    bg = bg.copy()
    bg[..., :3] = float("-inf")
    g = check_scene(bg, v, c, f, seed=5)
    assert np.all(np.isfinite(g["grad_vertices"]))


def _chain_inputs(n=100, H=512, W=512, seed=0):
    world, faces, albedo = dp.grid_surface(n=n)
    wts = np.random.default_rng(seed).uniform(0.5, 1.5, (H, W, 3)).astype(np.float32)
    return world, faces, albedo, wts


def test_config4_deferred_chain_matches_oracle_autograd():
    """samples/deferred.py:62-118 at C4 size (20k-triangle mesh, 512^2): d loss / d world vertices of the
    HIP chain against the same chain with the oracle's forward/backward under CPU autograd."""
    H = W = 512
    world, faces, albedo, wts = _chain_inputs(H=H, W=W)
    dev = torch.device("cuda", 0)
    Vg = torch.from_numpy(world).to(dev).requires_grad_(True)
    Lg, pxg, validg = dp.chain(dp.hip_render, Vg, torch.from_numpy(faces).to(dev), torch.from_numpy(albedo).to(dev),
                               H, W, torch.from_numpy(wts).to(dev), geometry_on_cpu=True)
    Lg.backward()
    Vc = torch.from_numpy(world).requires_grad_(True)
    Lc, pxc, validc = dp.chain(dp.oracle_render, Vc, torch.from_numpy(faces), torch.from_numpy(albedo), H, W,
                               torch.from_numpy(wts))
    Lc.backward()
    # the three G-buffers are bit-identical (-inf backgrounds included); validity identical; the shading
    # runs in fp32 torch on two devices (pow(., 6) of the specular term differs by a few ulp -> 1e-3)
    with torch.no_grad():
        gh = dp.gbuffers(dp.hip_render, Vg, torch.from_numpy(faces).to(dev), torch.from_numpy(albedo).to(dev), H, W,
                         geometry_on_cpu=True)
        go = dp.gbuffers(dp.oracle_render, Vc, torch.from_numpy(faces), torch.from_numpy(albedo), H, W)
    for a, b in zip(gh[:3], go[:3]):
        np.testing.assert_array_equal(a.cpu().numpy(), b.numpy())
    np.testing.assert_array_equal(validg.cpu().numpy(), validc.numpy())
    assert 0.2 < float(validc.float().mean()) < 0.6
    np.testing.assert_allclose(pxg.detach().cpu().numpy()[validc.expand(-1, -1, 3).numpy()],
                               pxc.detach().numpy()[validc.expand(-1, -1, 3).numpy()], rtol=1e-3, atol=1e-3)
    gg, gc = Vg.grad.cpu().numpy(), Vc.grad.numpy()
    assert np.all(np.isfinite(gg)) and np.all(np.isfinite(gc))
    scale = np.abs(gc).max()
    assert scale > 0
    err = np.abs(gg - gc)
    rel_l2 = float(np.linalg.norm(gg - gc) / np.linalg.norm(gc))
    print("deferred chain: max err %g, scale %g, rel L2 %g" % (err.max(), scale, rel_l2))
    assert rel_l2 < 1e-3
    assert np.all(err <= 1e-2 * np.abs(gc) + 1e-3 * scale), "max err %g of scale %g" % (err.max(), scale)


@pytest.mark.parametrize("seed", [2, 3, 4])
def test_config4_chain_all_on_gpu_against_oracle_chain(seed):
    """The whole chain on the GPU -- clip transform, the fused vertex normals and lighting kernels, the renders
    and their backward -- against the same chain with the oracle's renders and the framework-op lighting under
    CPU autograd (n = 50 mesh, 256^2, the surface's rows jittered per seed).  Both sides see their own float32
    geometry (the clip transform and the normals round differently on the two devices, so a pixel whose centre
    lies on an edge may change sides): loss within 1e-4 relative, d loss / d world vertices within 1e-2 in
    relative L2 norm."""
    H = W = 256
    world, faces, albedo, wts = _chain_inputs(n=50, H=H, W=W, seed=seed)
    world = world + np.random.default_rng(seed).normal(0.0, 0.003, world.shape).astype(np.float32)
    dev = torch.device("cuda", 0)
    Vg = torch.from_numpy(world).to(dev).requires_grad_(True)
    Lg, _, validg = dp.chain(dp.hip_render, Vg, torch.from_numpy(faces).to(dev), torch.from_numpy(albedo).to(dev),
                             H, W, torch.from_numpy(wts).to(dev))
    assert "VertexNormalsFn" in lighting.vertex_normals(Vg, torch.from_numpy(faces).to(dev)).grad_fn.name()
    Lg.backward()
    Vc = torch.from_numpy(world).requires_grad_(True)
    Lc, _, validc = dp.chain(dp.oracle_render, Vc, torch.from_numpy(faces), torch.from_numpy(albedo), H, W,
                             torch.from_numpy(wts))
    Lc.backward()
    assert abs(float(Lg.detach()) - float(Lc.detach())) <= 1e-4 * abs(float(Lc.detach()))
    assert float((validg.cpu() != validc).float().mean()) < 1e-3
    gg, gc = Vg.grad.cpu().numpy(), Vc.grad.numpy()
    assert np.all(np.isfinite(gg)) and np.abs(gc).max() > 0
    rel_l2 = float(np.linalg.norm(gg - gc) / np.linalg.norm(gc))
    assert rel_l2 < 1e-2, rel_l2


def test_config4_deferred_chain_finite_differences():
    """Pins the chain's gradient against central differences of the HIP forward chain on interior
    pixels (every pixel of the loss >= 3 px inside the silhouette, from face_ids): the loss is then
    smooth in the world positions, and the normals' gradient path is exercised."""
    import dirt_amd
    H = W = 256
    world, faces, albedo, wts = _chain_inputs(n=40, H=H, W=W, seed=1)
    dev = torch.device("cuda", 0)
    ft, at, wt = torch.from_numpy(faces).to(dev), torch.from_numpy(albedo).to(dev), torch.from_numpy(wts).to(dev)
    V0 = torch.from_numpy(world).to(dev)
    # interior mask from the G-buffer's face ids
    view, proj = dp.camera(H, W, dev)
    clip = torch.cat([V0, torch.ones_like(V0[:, :1])], 1) @ view @ proj
    gbuf = dirt_amd.rasterise_gbuffer(torch.zeros((H, W, 3), device=dev), clip, at, ft)
    cov = (gbuf.face_ids >= 0).float()[None, None]
    interior = (-torch.nn.functional.max_pool2d(-cov, 7, stride=1, padding=3))[0, 0] > 0.5
    mask = interior[..., None]
    assert interior.float().mean() > 0.1

    def loss(Vw):
        return dp.chain(dp.hip_render, Vw, ft, at, H, W, wt, mask=mask)[0]

    Vg = V0.clone().requires_grad_(True)
    loss(Vg).backward()
    grad = Vg.grad.cpu().numpy().astype(np.float64)
    rng = np.random.default_rng(7)
    # vertices well inside the visible surface (their whole 1-ring projects into the interior)
    ndc = (clip[:, :2] / clip[:, 3:]).cpu().numpy()
    px = np.stack([(ndc[:, 0] + 1) * W / 2, (1 - ndc[:, 1]) * H / 2], 1).astype(int)
    ok = (px[:, 0] > 4) & (px[:, 0] < W - 5) & (px[:, 1] > 4) & (px[:, 1] < H - 5)
    ok[ok] = interior.cpu().numpy()[px[ok, 1], px[ok, 0]]
    cand = np.flatnonzero(ok)
    picks = rng.choice(cand, size=12, replace=False)
    h = 2e-3
    num, ana = [], []
    with torch.no_grad():
        for vi in picks:
            for ax in range(3):
                d = torch.zeros_like(V0)
                d[vi, ax] = h
                fd = (loss(V0 + d).double() - loss(V0 - d).double()).item() / (2 * h)
                num.append(fd)
                ana.append(grad[vi, ax])
    num, ana = np.array(num), np.array(ana)
    scale = np.abs(num).max()
    assert scale > 0
    # filter-based derivative vs the discretised image: agreement to a few % of the gradient scale
    rel = np.abs(num - ana) / scale
    assert np.median(rel) < 0.05 and rel.max() < 0.25, (num, ana)
    assert np.corrcoef(num, ana)[0, 1] > 0.95


def test_config4_batched_gbuffer_renders_match_three_calls():
    """The three G-buffer renders of samples/deferred.py:63-83 as one rasterise_batch call of three frames (the
    geometry shared, tests/deferred_pipeline.py batched=True): bit-identical G-buffers, the same loss and
    gradient to the world vertices as the three separate calls."""
    import deferred_pipeline as dp
    dev = torch.device("cuda", 0)
    world, faces, albedo = dp.grid_surface(n=60)
    H = W = 256
    wts = torch.rand((H, W, 3), device=dev, generator=torch.Generator(device=dev).manual_seed(3))
    ft, at = torch.from_numpy(faces).to(dev), torch.from_numpy(albedo).to(dev)
    Vw = torch.from_numpy(world).to(dev)
    # one set of vertex normals for both (their index_add sums with float atomics: not bit-reproducible)
    nrm = lighting.vertex_normals(Vw, ft.long())
    three = dp.gbuffers(dp.hip_render, Vw, ft, at, H, W, normals=nrm)[:3]
    one = dp.gbuffers(dp.hip_render, Vw, ft, at, H, W, batched=True, normals=nrm)[:3]
    for a, b in zip(three, one):
        assert torch.equal(a, b)  # the same G-buffers (-inf backgrounds included)
    res = []
    for batched in (False, True):
        Vw = torch.from_numpy(world).to(dev).requires_grad_(True)
        L, px, valid = dp.chain(dp.hip_render, Vw, ft, at, H, W, wts, batched=batched)
        g, = torch.autograd.grad(L, [Vw])
        res.append((L.detach(), px.detach(), valid, g))
    (L0, p0, v0, g0), (L1, p1, v1, g1) = res
    assert torch.equal(v0, v1)
    # (the shading around the op is torch's; its kernels may round differently on differently laid out inputs)
    torch.testing.assert_close(L1, L0, rtol=1e-5, atol=0)
    torch.testing.assert_close(g1, g0, rtol=1e-4, atol=1e-5 * float(g0.abs().max()))
