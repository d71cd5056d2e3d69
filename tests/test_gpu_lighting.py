"""Fused lighting kernels (dirt_amd/csrc/lighting_kernels.h) against the framework-op statement of
dirt/lighting.py (dirt_amd/lighting.py `_*_ops`, float32 on the same GPU inputs): forward and backward.

Tolerances (float32): forward 2e-6 abs + 1e-5 rel; backward 1e-4 of the gradient's scale (the kernels sum
in a different order, vertex_normals' scatter uses float atomics).  The fused path must be the one that
runs (grad_fn of the C++ autograd functions); inputs it does not cover fall back to the framework ops.
"""
import numpy as np
import pytest
import torch

from dirt_amd import lighting

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _close_grad(a, b, name):
    scale = float(b.abs().max())
    err = float((a - b).abs().max())
    assert err <= 1e-4 * max(scale, 1e-6), "%s: max err %.3g vs scale %.3g" % (name, err, scale)


def _fused_node(y, cls):
    assert y.grad_fn is not None and cls in y.grad_fn.name(), y.grad_fn.name() if y.grad_fn else None


def _mesh(n=24, seed=0):
    rng = np.random.default_rng(seed)
    u, v = np.meshgrid(np.linspace(-1, 1, n), np.linspace(-1, 1, n))
    world = np.stack([u, 0.2 * np.sin(3 * u) * np.cos(2 * v) + 0.01 * rng.standard_normal(u.shape), v], -1)
    r = (np.arange(n - 1)[:, None] * n + np.arange(n - 1)[None, :]).reshape(-1)
    faces = np.stack([np.stack([r, r + n, r + 1], -1), np.stack([r + 1, r + n, r + n + 1], -1)], 1).reshape(-1, 3)
    return world.reshape(-1, 3).astype(np.float32), faces


@pytest.mark.parametrize("case", ["v3_i64", "v3_i32", "v4_i64", "batched"])
def test_vertex_normals_fused_matches_ops(case):
    world, faces = _mesh()
    V = len(world)
    if case == "v4_i64":
        world = np.concatenate([world, np.ones((V, 1), np.float32)], 1)
    if case == "batched":
        world = np.stack([world, world * np.float32(1.5) + np.float32(0.1)])
    x = torch.from_numpy(world).to(DEV).requires_grad_(True)
    f = torch.from_numpy(faces).to(DEV).to(torch.int32 if case == "v3_i32" else torch.int64)
    y = lighting.vertex_normals(x, f)
    _fused_node(y, "VertexNormalsFn")
    x2 = x.detach().clone().requires_grad_(True)
    y2 = lighting._vertex_normals_ops(x2, f.long())
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=2e-6)
    g = torch.randn_like(y)
    gx, = torch.autograd.grad(y, [x], g)
    gx2, = torch.autograd.grad(y2, [x2], g)
    assert gx.shape == x.shape
    _close_grad(gx, gx2, "d vertices")


@pytest.mark.parametrize("two", [True, False])
def test_diffuse_directional_fused_matches_ops(two):
    gen = torch.Generator(device=DEV).manual_seed(1)
    N = 70001
    n = torch.randn((N, 3), device=DEV, generator=gen)
    n = (n / n.norm(dim=-1, keepdim=True)).requires_grad_(True)
    c = torch.rand((N, 3), device=DEV, generator=gen).requires_grad_(True)
    ld = torch.tensor([1.0, -0.3, -0.5], device=DEV)
    ld = ld / ld.norm()
    lc = torch.tensor([1.0, 0.5, 0.25], device=DEV)
    y = lighting.diffuse_directional(n, c, ld, lc, double_sided=two)
    _fused_node(y, "DiffuseFn")
    n2, c2 = n.detach().clone().requires_grad_(True), c.detach().clone().requires_grad_(True)
    y2 = lighting._diffuse_directional_ops(n2, c2, ld, lc, two)
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=2e-6)
    g = torch.randn((N, 3), device=DEV, generator=gen)
    gn, gc = torch.autograd.grad(y, [n, c], g)
    gn2, gc2 = torch.autograd.grad(y2, [n2, c2], g)
    _close_grad(gn, gn2, "d normals")
    _close_grad(gc, gc2, "d colors")


@pytest.mark.parametrize("two,shininess", [(True, 6.0), (False, 6.0), (False, 1.0), (True, 0.0), (False, 2.5)])
def test_specular_directional_fused_matches_ops(two, shininess):
    gen = torch.Generator(device=DEV).manual_seed(2)
    N = 65537
    p = (torch.rand((N, 3), device=DEV, generator=gen) * 2 - 1).requires_grad_(True)
    n = torch.randn((N, 3), device=DEV, generator=gen)
    n = (n / n.norm(dim=-1, keepdim=True)).requires_grad_(True)
    r = torch.rand((N, 3), device=DEV, generator=gen).requires_grad_(True)
    ld = torch.tensor([1.0, -0.3, -0.5], device=DEV)
    ld = ld / ld.norm()
    lc = torch.tensor([1.0, 1.0, 1.0], device=DEV)
    cam = torch.tensor([0.0, 1.7, 2.2], device=DEV)
    y = lighting.specular_directional(p, n, r, ld, lc, cam, shininess, double_sided=two)
    _fused_node(y, "SpecularFn")
    p2, n2, r2 = (t.detach().clone().requires_grad_(True) for t in (p, n, r))
    y2 = lighting._specular_directional_ops(p2, n2, r2, ld, lc, cam, shininess, two)
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=2e-6)
    g = torch.randn((N, 3), device=DEV, generator=gen)
    grads = torch.autograd.grad(y, [p, n, r], g)
    grads2 = torch.autograd.grad(y2, [p2, n2, r2], g)
    for a, b, name in zip(grads, grads2, ("d positions", "d normals", "d reflectivities")):
        _close_grad(a, b, name)


@pytest.mark.parametrize("two", [True, False])
def test_diffuse_point_fused_matches_ops(two):
    gen = torch.Generator(device=DEV).manual_seed(4)
    N = 50003
    p = (torch.rand((N, 3), device=DEV, generator=gen) * 2 - 1).requires_grad_(True)
    n = torch.randn((N, 3), device=DEV, generator=gen)
    n = (n / n.norm(dim=-1, keepdim=True)).requires_grad_(True)
    c = torch.rand((N, 3), device=DEV, generator=gen).requires_grad_(True)
    lp = torch.tensor([0.5, -1.0, 0.5], device=DEV)
    lc = torch.tensor([1.0, 0.5, 0.9], device=DEV)
    y = lighting.diffuse_point(p, n, c, lp, lc, double_sided=two)
    _fused_node(y, "DiffusePointFn")
    p2, n2, c2 = (t.detach().clone().requires_grad_(True) for t in (p, n, c))
    y2 = lighting._diffuse_point_ops(p2, n2, c2, lp, lc, two)
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=2e-6)
    g = torch.randn((N, 3), device=DEV, generator=gen)
    for a, b, name in zip(torch.autograd.grad(y, [p, n, c], g), torch.autograd.grad(y2, [p2, n2, c2], g),
                          ("d positions", "d normals", "d colors")):
        _close_grad(a, b, name)


def test_light_gradient_falls_back_to_framework_ops():
    """A light direction that needs a gradient is outside the fused kernels: the framework ops run and
    differentiate it."""
    n = torch.nn.functional.normalize(torch.randn((100, 3), device=DEV), dim=-1)
    c = torch.rand((100, 3), device=DEV)
    ld = torch.tensor([0.0, 0.0, -1.0], device=DEV, requires_grad=True)
    y = lighting.diffuse_directional(n, c, ld, torch.ones(3, device=DEV))
    assert "DiffuseFn" not in y.grad_fn.name()
    g, = torch.autograd.grad(y.sum(), [ld])
    assert torch.isfinite(g).all() and float(g.abs().sum()) > 0


def test_fused_backward_refuses_double_backward(monkeypatch):
    """the fused backwards carry no graph, so create_graph=True through them raises instead of
    silently dropping the second-order terms; with DIRT_FUSED_LIGHTING=0 the framework ops run and support it."""
    gen = torch.Generator(device=DEV).manual_seed(5)
    n = torch.nn.functional.normalize(torch.randn((256, 3), device=DEV, generator=gen), dim=-1).requires_grad_(True)
    c = torch.rand((256, 3), device=DEV, generator=gen).requires_grad_(True)
    ld = torch.nn.functional.normalize(torch.tensor([1.0, -0.3, -0.5], device=DEV), dim=0)
    lc = torch.ones(3, device=DEV)
    y = lighting.diffuse_directional(n, c, ld, lc)
    _fused_node(y, "DiffuseFn")
    with pytest.raises(RuntimeError, match="create_graph"):
        torch.autograd.grad(y.square().sum(), [n], create_graph=True)
    world, faces = _mesh(8)
    x = torch.from_numpy(world).to(DEV).requires_grad_(True)
    nv = lighting.vertex_normals(x, torch.from_numpy(faces).to(DEV))
    with pytest.raises(RuntimeError, match="create_graph"):
        torch.autograd.grad(nv.sum(), [x], create_graph=True)
    # first-order gradients are unaffected
    g, = torch.autograd.grad(lighting.diffuse_directional(n, c, ld, lc).sum(), [c])
    assert torch.isfinite(g).all()
    monkeypatch.setattr(lighting, "_FUSED_ENABLED", False)
    y2 = lighting.diffuse_directional(n, c, ld, lc)
    assert "DiffuseFn" not in y2.grad_fn.name()
    gn, = torch.autograd.grad(y2.square().sum(), [n], create_graph=True)
    gg, = torch.autograd.grad(gn.sum(), [c])
    assert torch.isfinite(gg).all()


def test_fused_lighting_captures_into_a_graph():
    """No host-to-device copy inside: the fused calls record into a HIP graph and replay to the eager result."""
    world, faces = _mesh(12)
    x = torch.from_numpy(world).to(DEV)
    f = torch.from_numpy(faces).to(DEV)
    ld = torch.nn.functional.normalize(torch.tensor([1.0, -0.3, -0.5], device=DEV), dim=0)
    lc = torch.ones(3, device=DEV)
    cam = torch.tensor([0.0, 1.0, 2.0], device=DEV)

    def step():
        nrm = lighting.vertex_normals(x, f)
        return (lighting.diffuse_directional(nrm, nrm.abs(), ld, lc) +
                lighting.specular_directional(x, nrm, nrm.abs(), ld, lc, cam, 6.0))

    ref = step()
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream(DEV))
    with torch.cuda.stream(s):
        step()
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        out = step()
    graph.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-6)
