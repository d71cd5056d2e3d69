"""CPU tests of the Python op surface (mirror of the reference dirt/rasterise_ops.py) and helpers."""
import inspect
import math

import numpy as np
import pytest
import torch

import dirt_amd
from dirt_amd import lighting, matrices, rasterise_ops


def test_op_names_and_signatures_match_the_reference():
    # dirt/rasterise_ops.py:10,57,91,110,129,148,167,186 (camera_pos made optional)
    for name in ("rasterise", "rasterise_batch"):
        params = list(inspect.signature(getattr(dirt_amd, name)).parameters)
        # the reference's parameters in its order; `shader` (fork's fragment program) and `check_faces`
        # (opt-in index check) are added keywords after them
        assert params == ["background", "vertices", "vertex_colors", "faces", "camera_pos", "height", "width",
                          "channels", "name", "shader", "check_faces"]
        sig = inspect.signature(getattr(dirt_amd, name))
        assert all(sig.parameters[p].default is None for p in params[4:])
    for name in ("rasterise_grad", "oceanic_no_cloud", "oceanic_simple_proxy", "oceanic_still_cloud",
                 "oceanic_opt_flow", "hill"):
        assert callable(getattr(dirt_amd, name))
    with pytest.raises(ValueError, match="fragment program"):
        rasterise_ops._shader_id("phong")
    assert rasterise_ops._shader_id("oceanic_horizon") == 1 and rasterise_ops._shader_id(None) == 0


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback():
    bg = np.zeros((8, 8, 3), np.float32)
    with pytest.raises(RuntimeError, match="GPU"):
        dirt_amd.rasterise(bg, np.zeros((3, 4), np.float32), np.zeros((3, 3), np.float32), [[0, 1, 2]])


@pytest.mark.parametrize("shapes,msg", [
    (((1, 8, 8, 3), (1, 3, 4), (1, 3, 3), (1, 1, 3)), None),
    (((1, 8, 9, 3), (1, 3, 4), (1, 3, 3), (1, 1, 3)), "background"),
    (((1, 8, 8, 3), (1, 3, 3), (1, 3, 3), (1, 1, 3)), "vertices"),
    (((1, 8, 8, 3), (1, 3, 4), (1, 4, 3), (1, 1, 3)), "vertex_colors"),
    (((1, 8, 8, 3), (1, 3, 4), (1, 3, 3), (1, 1, 2)), "faces"),
    (((2, 8, 8, 3), (1, 3, 4), (1, 3, 3), (1, 1, 3)), "batch"),
])
def test_shape_validation_messages(shapes, msg):
    ts = [torch.zeros(s) for s in shapes]
    if msg is None:
        rasterise_ops._check_shapes(*ts, 8, 8, 3)
    else:
        with pytest.raises(ValueError, match=msg):
            rasterise_ops._check_shapes(*ts, 8, 8, 3)


def test_camera_pos_lengths_per_program():
    # floats each op copies to the host: 8 (rasterise_egl.cpp:323), 9 (oceanic_still_cloud.cpp:323),
    # 16 (oceanic_opt_flow.cpp:323), 12 (hill.cpp:323)
    from dirt_amd import _lib
    cpu = torch.device("cpu")
    for sid, n in ((_lib.SHADER_OCEANIC_HORIZON, 8), (_lib.SHADER_OCEANIC_STILL_CLOUD, 9),
                   (_lib.SHADER_OCEANIC_OPT_FLOW, 16), (_lib.SHADER_HILL, 12)):
        assert rasterise_ops._camera(np.zeros(n), sid, cpu).numel() == n
        with pytest.raises(ValueError):
            rasterise_ops._camera(np.zeros(n - 1), sid, cpu)
    with pytest.raises(ValueError, match="camera_pos"):
        rasterise_ops._camera(None, _lib.SHADER_HILL, cpu)
    assert rasterise_ops._camera(None, _lib.SHADER_GOURAUD, cpu) is None
    assert rasterise_ops._shader_id("oceanic_opt_flow") == 6
    params = list(inspect.signature(dirt_amd.hill).parameters)
    assert params == ["background", "vertices", "vertex_colors", "faces", "camera_pos", "height", "width",
                      "channels", "name"]


def test_matrices_match_reference_formulas():
    P = matrices.perspective_projection(0.1, 20.0, 0.2, 0.75).numpy()
    n, f, r, t = 0.1, 20.0, 0.2, 0.2 * 0.75
    expect = np.array([[n / r, 0, 0, 0], [0, n / t, 0, 0], [0, 0, -(f + n) / (f - n), -2 * f * n / (f - n)],
                       [0, 0, -1, 0]], np.float32).T
    np.testing.assert_allclose(P, expect, rtol=1e-6)
    R = matrices.rodrigues([0.0, 0.5, 0.0]).numpy()
    np.testing.assert_allclose(R[:3, :3] @ R[:3, :3].T, np.eye(3), atol=1e-6)
    c, s = math.cos(0.5), math.sin(0.5)
    # K = [[0,-v2,v1],[v2,0,-v0],[-v1,v0,0]] indexed (in, out): dirt/matrices.py:41-45
    np.testing.assert_allclose(R[:3, :3], [[c, 0, s], [0, 1, 0], [-s, 0, c]], atol=1e-6)
    T = matrices.translation([1.0, 2.0, 3.0]).numpy()
    np.testing.assert_allclose(np.array([0, 0, 0, 1.0]) @ T, [1, 2, 3, 1])
    np.testing.assert_allclose(matrices.compose(T, R).numpy(), T @ R, atol=1e-6)
    assert torch.equal(matrices.compose(), torch.eye(4))


def test_lighting_helpers():
    verts = torch.tensor([[0., 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1]])
    faces = torch.tensor([[0, 1, 2], [0, 1, 3]])
    sv, sf = lighting.split_vertices_by_face(verts, faces)
    assert sv.shape == (6, 3) and sf.tolist() == [[0, 1, 2], [3, 4, 5]]
    n = lighting.vertex_normals_pre_split(sv, sf)
    np.testing.assert_allclose(n[:3].numpy(), [[0, 0, 1]] * 3, atol=1e-6)
    np.testing.assert_allclose(n[3:].numpy(), [[0, -1, 0]] * 3, atol=1e-6)
    vn = lighting.vertex_normals(verts, faces)
    np.testing.assert_allclose(torch.linalg.norm(vn[:2], dim=-1).numpy(), 1.0, atol=1e-6)
    d = lighting.diffuse_directional(n, torch.ones(6, 3), [0., 0., -1.], [1., 0.5, 0.25])
    np.testing.assert_allclose(d[0].numpy(), [1, 0.5, 0.25], atol=1e-6)
    p = lighting.diffuse_point(sv, n, torch.ones(6, 3), [0., 0., 5.], [1., 1., 1.])
    assert p.shape == (6, 3) and float(p.min()) >= 0
    sp = lighting.specular_directional(sv, n, torch.ones(6, 3), [0., 0., -1.], [1., 1., 1.], [0., 0., 3.], 6.0)
    assert sp.shape == (6, 3)


def test_upstream_positional_call_form():
    # upstream DIRT: rasterise_batch(background, vertices, vertex_colors, faces, height, width, channels, name)
    # binds height to the fork's camera_pos slot; an integer there shifts the rest back into place
    up = rasterise_ops._upstream_positional
    assert up(48, 64, 3, None, None) == (None, 48, 64, 3, None)
    assert up(np.int64(48), 64, 3, "nm", None) == (None, 48, 64, 3, "nm")
    cam = [0.0] * 8
    assert up(cam, 48, 64, 3, None) == (cam, 48, 64, 3, None)
    assert up(None, None, None, None, None) == (None, None, None, None, None)
    # mixed positional / keyword forms: keywords stay in their slots
    assert up(48, None, 64, 3, None) == (None, 48, 64, 3, None)      # (.., 48, width=64, channels=3)
    assert up(48, 64, None, 3, None) == (None, 48, 64, 3, None)      # (.., 48, 64, channels=3)
    assert up(48, None, None, 3, "nm") == (None, 48, None, 3, "nm")  # (.., 48, channels=3, name="nm")
    assert up(48, None, None, None, None) == (None, 48, None, None, None)
    if not torch.cuda.is_available():
        # the positional upstream call reaches the device check, not a camera_pos error
        bg = np.zeros((1, 8, 8, 3), np.float32)
        with pytest.raises(RuntimeError, match="GPU"):
            dirt_amd.rasterise_batch(bg, np.zeros((1, 3, 4), np.float32), np.zeros((1, 3, 3), np.float32),
                                     np.zeros((1, 1, 3), np.int32), 8, 8, 3)


def test_tensor_inputs_without_a_gpu_raise_the_same_error():
    """The C++ fast path of the public op (torch tensors in, torch_op.cpp rasterise_checked) fails like the
    Python path when there is no HIP device: no CPU fallback."""
    import torch
    import dirt_amd
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    t = [torch.zeros((1, 8, 8, 3)), torch.zeros((1, 3, 4)), torch.zeros((1, 3, 3)), torch.zeros((1, 1, 3), dtype=torch.int32)]
    with pytest.raises(RuntimeError, match="GPU"):
        dirt_amd.rasterise_batch(*t)


def test_fused_lighting_bindings_check_their_operands():
    """The fused lighting helpers take raw device pointers: their bindings refuse host tensors and shapes
    the kernels do not index by (ValueError), while dirt_amd.lighting runs CPU tensors through the
    framework ops."""
    ext = rasterise_ops._torch_ext()
    if ext is None:
        pytest.skip("the C++ extension is not built")
    z3, p3 = torch.zeros(4, 3), torch.zeros(3)
    with pytest.raises(ValueError, match="GPU"):
        ext.diffuse_directional(z3, z3, p3, p3, True)
    with pytest.raises(ValueError, match="GPU"):
        ext.specular_directional(z3, z3, z3, p3, p3, p3, 6.0, True)
    with pytest.raises(ValueError, match="vertex_normals"):
        ext.vertex_normals(z3, torch.zeros(2, 3, dtype=torch.int32))
    n = torch.nn.functional.normalize(torch.randn(5, 3), dim=-1)
    out = lighting.diffuse_directional(n, torch.ones(5, 3), torch.tensor([0., 0., -1.]), torch.ones(3))
    ref = lighting._diffuse_directional_ops(n, torch.ones(5, 3), torch.tensor([0., 0., -1.]), torch.ones(3), True)
    torch.testing.assert_close(out, ref, rtol=0, atol=0)


def test_shared_geometry_identity_rule():
    """The public op shares a render's setup and visibility with the previous forward only for the same elements of
    the same storage, unmodified (torch version counters): views of them match, in-place edits, clones and other
    layouts do not (rasterise_ops._GeomCache; the C++ op applies the same rule)."""
    ident = rasterise_ops._GeomCache._ident
    v = torch.arange(24, dtype=torch.float32).reshape(1, 6, 4)
    f = torch.arange(6, dtype=torch.int32).reshape(1, 2, 3)
    base = ident(v)
    assert ident(v) == base
    assert ident(v[0][None]) == base  # a view of the same elements (the size-1 dimension's stride is ignored)
    assert ident(v.view(1, 6, 4)) == base
    assert ident(v.clone()) != base  # equal values, another storage
    assert ident(v[:, :5]) != base  # other elements
    assert ident(v.transpose(1, 2).contiguous().transpose(1, 2)) != base  # another layout
    v.mul_(1.0)  # in place, same values: the version counter moved
    assert ident(v) != base
    c = rasterise_ops._GeomCache()
    gb, saved = torch.zeros(1), torch.zeros(2)
    key = ("dev", 0, 0)
    c.store(key, v, f, 8, 8, gb, saved)
    assert c.find(key, v, f, 8, 8) == (gb, saved)
    assert c.find(key, v, f, 8, 9) is None  # other frame size
    assert c.find(("dev", 1, 0), v, f, 8, 8) is None  # other stream / capture
    f[0, 0, 0] = 5  # faces edited in place
    assert c.find(key, v, f, 8, 8) is None
    c.clear()
    assert c.find(key, v, f, 8, 8) is None


def test_geometry_sharing_switch_cpu():
    """set_geometry_sharing returns the previous setting and drives the cache's switch (no extension on CPU)."""
    from dirt_amd import rasterise_ops
    prev = rasterise_ops.set_geometry_sharing(False)
    try:
        assert rasterise_ops._GeomCache.enabled is False
        assert rasterise_ops.set_geometry_sharing(True) is False
        assert rasterise_ops._GeomCache.enabled is True
    finally:
        rasterise_ops.set_geometry_sharing(prev)

