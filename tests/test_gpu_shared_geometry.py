"""GPU: renders that share one geometry (ABI 13 dirt_rasterise_fwd_resolve).

samples/deferred.py:63-83 renders one mesh three times (world positions over -inf, albedo over 0, normals over -inf).
The public op remembers the geometry of its last plain Gouraud forward per (device, stream, capture) and, for a
forward on the same unmodified vertex and face tensors, runs the resolve alone (no setup, bins or visibility pass).
These tests hold such renders to the oracle (pixels bit-exact, gradients in tolerance), count the setup launches to
show which forwards shared, and check that an in-place change of the geometry, a different tensor with equal values,
and HIP-graph replays with the geometry changed in place between them all give the results of the new geometry.
"""
import numpy as np
import pytest
import torch

import scenes
from oracle import oracle
from test_gpu_parity import assert_close_grad, _gpu

pytestmark = pytest.mark.gpu


def _op(impl):
    from dirt_amd import rasterise_ops
    ext = rasterise_ops._torch_ext()
    if impl == "ext":
        assert ext is not None

    def op(bg, v, c, f, H, W, C):
        args = (bg, v, c, f, None, H, W, C, 0, 0, False, False)
        return (ext.rasterise(*args) if impl == "ext" else rasterise_ops._RasteriseFunction.apply(*args))[0]
    return op


def _setup_launches(fn):
    from dirt_amd import _lib
    _lib.profile_enable(True)
    out = fn()
    torch.cuda.synchronize()
    n = _lib.profile_read()["setup_kernel"][0]
    _lib.profile_enable(False)
    return out, n


def _scene():
    """A shared-vertex mesh with three colour sets and backgrounds of the sample's kinds (-inf, 0, -inf)."""
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=3000, W=160, H=128, radius_px=9.0, seed=120))
    rng = np.random.default_rng(121)
    B, H, W, C = bg.shape
    cols = [c, rng.uniform(0, 1, c.shape).astype(np.float32), rng.standard_normal(c.shape).astype(np.float32)]
    bgs = [np.full(bg.shape, -np.inf, np.float32), np.zeros(bg.shape, np.float32), np.full(bg.shape, -np.inf, np.float32)]
    return bgs, v, cols, f, (H, W, C)


@pytest.mark.parametrize("impl", ["ext", "py"])
def test_three_renders_of_one_geometry(impl):
    from dirt_amd import rasterise_ops
    rasterise_ops.workspace_cache_clear(force=True)
    op = _op(impl)
    bgs, v, cols, f, (H, W, C) = _scene()
    vt = _gpu(v).requires_grad_(True)
    ft = _gpu(f)
    cts = [_gpu(c).requires_grad_(True) for c in cols]
    bts = [_gpu(b) for b in bgs]
    gps = [np.random.default_rng(130 + k).standard_normal(bgs[0].shape).astype(np.float32) for k in range(3)]

    def render_all():
        return [op(bts[k], vt, cts[k], ft, H, W, C) for k in range(3)]

    pxs, n_setup = _setup_launches(render_all)
    assert n_setup == 1, "the second and third renders of one geometry should share the first one's setup"
    loss = sum((p * _gpu(g)).sum() for p, g in zip(pxs, gps))
    grads = torch.autograd.grad(loss, [vt] + cts)
    gv_total = np.zeros_like(v)
    for k in range(3):
        px, gb, _ = oracle.rasterise_fwd(bgs[k], v, cols[k], f)
        np.testing.assert_array_equal(pxs[k].detach().cpu().numpy(), px)  # bit-exact, -inf included
        rgv, rgc, _ = oracle.rasterise_bwd(v, cols[k], f, px, gps[k], gb)
        gv_total += rgv
        assert_close_grad(grads[1 + k].cpu().numpy(), rgc, "grad_vertex_colors render %d" % k)
    assert_close_grad(grads[0].cpu().numpy(), gv_total, "grad_vertices (three renders)")


@pytest.mark.parametrize("impl", ["ext", "py"])
def test_shared_geometry_invalidation(impl):
    """An in-place change of the vertices (any in-place op bumps the version counter) or faces makes the next render
    a full one; a different tensor holding equal values is a full render too; every result is the oracle's."""
    from dirt_amd import rasterise_ops
    rasterise_ops.workspace_cache_clear(force=True)
    op = _op(impl)
    bgs, v, cols, f, (H, W, C) = _scene()
    vt, ft = _gpu(v), _gpu(f)
    ct, bt = _gpu(cols[1]), _gpu(bgs[1])

    def check(vv, ff, expect_setups):
        px, n = _setup_launches(lambda: op(bt, vv, ct, ff, H, W, C))
        ref, _, _ = oracle.rasterise_fwd(bgs[1], vv.cpu().numpy(), cols[1], ff.cpu().numpy())
        np.testing.assert_array_equal(px.cpu().numpy(), ref)
        assert n == expect_setups

    check(vt, ft, 1)  # first render: full
    check(vt, ft, 0)  # same tensors: shared
    check(vt[0][None], ft, 0)  # a view of the same elements: shared
    vt.mul_(1.0)  # in place, same values: the version changed, so a full render
    check(vt, ft, 1)
    with torch.no_grad():
        vt[0, ::7, :2] += 0.05  # in place through a view: moves some vertices
    check(vt, ft, 1)
    check(vt, ft, 0)
    ft[0, :5] = ft[0, 5:10].clone()  # faces changed in place
    check(vt, ft, 1)
    check(vt.clone(), ft, 1)  # equal values, another tensor: full
    check(vt, ft.clone(), 1)


@pytest.mark.parametrize("impl", ["ext", "py"])
def test_shared_geometry_in_a_captured_graph(impl):
    """Three renders + backward captured into one HIP graph (the capture's first render is full, the other two share
    it inside the graph); the vertices are changed in place between replays, and every replay gives the oracle's
    pixels and gradients of the current geometry."""
    from dirt_amd import rasterise_ops
    rasterise_ops.workspace_cache_clear(force=True)
    op = _op(impl)
    bgs, v, cols, f, (H, W, C) = _scene()
    vt = _gpu(v).requires_grad_(True)
    ft = _gpu(f)
    cts = [_gpu(c) for c in cols]
    bts = [_gpu(b) for b in bgs]
    g = [_gpu(np.random.default_rng(140 + k).standard_normal(bgs[0].shape).astype(np.float32)) for k in range(3)]
    out = {}

    def step():
        pxs = [op(bts[k], vt, cts[k], ft, H, W, C) for k in range(3)]
        out["px"] = [p.detach() for p in pxs]
        out["gv"] = torch.autograd.grad(sum((p * gk).sum() for p, gk in zip(pxs, g)), [vt])[0]

    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        step()
    torch.cuda.current_stream().wait_stream(s_)
    torch.cuda.synchronize()
    out.clear()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    rng = np.random.default_rng(150)
    for rep in range(3):
        if rep:
            with torch.no_grad():
                vt[0, :, :2] += torch.from_numpy(rng.uniform(-0.01, 0.01, (v.shape[1], 2)).astype(np.float32)).cuda()
        graph.replay()
        torch.cuda.synchronize()
        vn = vt.detach().cpu().numpy()
        gv_total = np.zeros_like(vn)
        for k in range(3):
            px, gb, _ = oracle.rasterise_fwd(bgs[k], vn, cols[k], f)
            np.testing.assert_array_equal(out["px"][k].cpu().numpy(), px)
            rgv, _, _ = oracle.rasterise_bwd(vn, cols[k], f, px, g[k].cpu().numpy(), gb)
            gv_total += rgv
        assert_close_grad(out["gv"].cpu().numpy(), gv_total, "grad_vertices replay %d" % rep)
    del graph
    rasterise_ops.workspace_cache_clear(force=True)


@pytest.mark.parametrize("impl", ["ext", "py"])
def test_geometry_sharing_switch(impl):
    """set_geometry_sharing(False): every render of one geometry is a full one (a training loop's setting, and
    bench.py's api leg); switched back on, the second render shares again; results are the oracle's either way."""
    from dirt_amd import rasterise_ops
    rasterise_ops.workspace_cache_clear(force=True)
    op = _op(impl)
    bgs, v, cols, f, (H, W, C) = _scene()
    vt, ft = _gpu(v), _gpu(f)
    ct, bt = _gpu(cols[1]), _gpu(bgs[1])
    ref, _, _ = oracle.rasterise_fwd(bgs[1], v, cols[1], f)
    prev = rasterise_ops.set_geometry_sharing(False)
    try:
        for _ in range(3):
            px, n = _setup_launches(lambda: op(bt, vt, ct, ft, H, W, C))
            assert n == 1
            np.testing.assert_array_equal(px.cpu().numpy(), ref)
        assert rasterise_ops.set_geometry_sharing(True) is False
        counts = []
        for _ in range(2):
            px, n = _setup_launches(lambda: op(bt, vt, ct, ft, H, W, C))
            counts.append(n)
            np.testing.assert_array_equal(px.cpu().numpy(), ref)
        assert counts == [1, 0]
    finally:
        rasterise_ops.set_geometry_sharing(prev)

