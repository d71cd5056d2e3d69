"""GPU tests of the single-output op and its recompute-mode gradient (C ABI dirt_rasterise_bwd_recompute).

The reference's `Rasterise` op has ONE output (csrc/rasterise_egl.cpp:33-53) and its Python wrapper indexes it
(`_rasterise_module.rasterise(...)[0]`, dirt/rasterise_ops.py:50-54).  dirt_amd.op_library restates that op
over libdirt_mi355x.so with a gradient computed from the op's inputs, output and grad_pixels only, as upstream
DIRT's gradient re-derived its G-buffer (csrc/rasterise_grad_common.h:5-24).  Contract checked here:
  * pixels bit-exact vs the oracle / the golden fixtures, and vs the stateful public op;
  * grad_background bit-identical to the stateful backward and the oracle;
  * grad_vertices / grad_vertex_colors within the suite's tolerance (float-atomic order) of both the stateful
    backward and the oracle -- golden scenes, full-size config 3, an adversarial fuzz batch, clipped faces,
    7 channels, the fused small-scene path and an empty face list.
"""
import glob
import os

import numpy as np
import pytest
import torch

import scenes
from oracle import oracle
from test_gpu_parity import GOLDEN, _gpu, assert_close_grad, run_gpu

pytestmark = pytest.mark.gpu


def run_single_output(bg, v, c, f, gp):
    """Forward through the single-output op module, backward through its registered (recompute) gradient."""
    from dirt_amd import op_library
    mod = op_library.load_op_library()
    bg_t, v_t, c_t = _gpu(bg).requires_grad_(True), _gpu(v).requires_grad_(True), _gpu(c).requires_grad_(True)
    B, H, W, C = bg.shape
    px = mod.rasterise(bg_t, v_t, c_t, _gpu(f), None, H, W, C)
    assert isinstance(px, torch.Tensor) and tuple(px.shape) == (B, H, W, C)  # one output, like REGISTER_OP
    gbg, gv, gc = torch.autograd.grad(px, [bg_t, v_t, c_t], _gpu(gp))
    return {"pixels": px.detach().cpu().numpy(), "grad_background": gbg.cpu().numpy(),
            "grad_vertices": gv.cpu().numpy(), "grad_colors": gc.cpu().numpy()}


def check_both(bg, v, c, f, seed=1, strict=False):
    if bg.ndim == 3:
        bg, v, c, f = bg[None], v[None], c[None], f[None]
    gp = np.random.default_rng(seed).standard_normal(bg.shape).astype(np.float32)
    r = run_single_output(bg, v, c, f, gp)
    s = run_gpu(bg, v, c, f, gp)  # the stateful public op
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    np.testing.assert_array_equal(r["pixels"], px)
    np.testing.assert_array_equal(r["pixels"], s["pixels"])
    gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, gp, gb)
    np.testing.assert_array_equal(r["grad_background"], s["grad_background"])
    np.testing.assert_array_equal(r["grad_background"], gbg)
    for name, key, ref in (("grad_vertex_colors", "grad_colors", gc), ("grad_vertices", "grad_vertices", gv)):
        assert_close_grad(r[key], ref, name + " (recompute vs oracle)", strict)
        assert_close_grad(r[key], s[key], name + " (recompute vs stateful)", strict)
    assert np.all(r["grad_vertices"][..., 2] == 0.0)
    return r


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_recompute_golden_fixtures(path):
    z = np.load(path)
    r = run_single_output(z["background"], z["vertices"], z["vertex_colors"], z["faces"], z["grad_pixels"])
    np.testing.assert_array_equal(r["pixels"], z["pixels"])
    np.testing.assert_array_equal(r["grad_background"], z["grad_background"])
    assert_close_grad(r["grad_colors"], z["grad_vertex_colors"], "grad_vertex_colors", strict=True)
    assert_close_grad(r["grad_vertices"], z["grad_vertices"], "grad_vertices", strict=True)
    s = run_gpu(z["background"], z["vertices"], z["vertex_colors"], z["faces"], z["grad_pixels"])
    np.testing.assert_array_equal(r["grad_background"], s["grad_background"])
    assert_close_grad(r["grad_colors"], s["grad_colors"], "grad_vertex_colors vs stateful")
    assert_close_grad(r["grad_vertices"], s["grad_vertices"], "grad_vertices vs stateful")


def test_recompute_full_size_c3():
    check_both(*scenes.random_triangles(F=50000, W=1024, H=1024, seed=0), strict=True)


def test_recompute_fuzz_batch_clipped_channels_small_and_empty():
    check_both(*scenes.fuzz_case(9003), seed=3)   # a batch of two adversarial 64x48 frames, C = 5
    check_both(*scenes.fuzz_case(37851), seed=4)  # the round-3 sliver scene (clipped faces)
    check_both(*scenes.clipping_scene(C=7), seed=4)
    check_both(*scenes.readme_square(), seed=5)          # fused small-scene forward (F <= 32)
    check_both(*scenes.cube_scene(), seed=6)
    bg, v, c, f = scenes.random_triangles(F=10, W=32, H=32, seed=1)
    r = check_both(bg, v, c, f[:0], seed=7)               # no faces: every pixel is background
    assert np.all(r["grad_vertices"] == 0.0) and np.all(r["grad_colors"] == 0.0)


@pytest.mark.parametrize("seed", range(int(os.environ.get("DIRT_RC_FUZZ_FIRST", "0")),
                                         int(os.environ.get("DIRT_RC_FUZZ_SEEDS", "6"))))
def test_recompute_fuzz_adversarial_scenes(seed):
    """The recompute backward on the adversarial fuzz batches of test_gpu_parity.py (scenes.fuzz_case: clipping,
    w <= 0, slivers, ties, guard-band overflow, channel counts 1..7): the same gradients as the stateful
    backward and the oracle.  DIRT_RC_FUZZ_SEEDS=N widens it (default 6), from DIRT_RC_FUZZ_FIRST."""
    check_both(*scenes.fuzz_case(200000 + seed), seed=seed)


def test_reference_wrapper_body_runs_unchanged():
    """dirt/rasterise_ops.py:39-54 with TF's calls mapped to torch: the op module's single output is indexed
    with [0], exactly as the reference does; the gradient is registered (the fork has none)."""
    from dirt_amd import op_library
    _rasterise_module = op_library.load_op_library(os.path.join("dirt", "librasterise.so"))

    def rasterise(background, vertices, vertex_colors, faces, camera_pos, height=None, width=None, channels=None,
                  name=None):
        background = torch.as_tensor(background, dtype=torch.float32)
        vertices = torch.as_tensor(vertices, dtype=torch.float32)
        vertex_colors = torch.as_tensor(vertex_colors, dtype=torch.float32)
        faces = torch.as_tensor(faces, dtype=torch.int32)
        if height is None:
            height = int(background.shape[0])
        if width is None:
            width = int(background.shape[1])
        if channels is None:
            channels = int(background.shape[2])
        return _rasterise_module.rasterise(
            background[None, ...], vertices[None, ...], vertex_colors[None, ...], faces[None, ...], camera_pos,
            height, width, channels,
            name=name
        )[0]

    bg, v, c, f = scenes.cylinder_scene()
    vt = _gpu(v).requires_grad_(True)
    cam = torch.tensor([0, 150, 0, 0, 0.3, 0, 0, 1.5], dtype=torch.float32, device="cuda")
    px = rasterise(_gpu(bg), vt, _gpu(c), _gpu(f), cam)
    ref, gb, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None])
    assert tuple(px.shape) == bg.shape
    np.testing.assert_array_equal(px.detach().cpu().numpy(), ref[0])
    gp = np.random.default_rng(2).standard_normal(bg.shape).astype(np.float32)
    px.backward(_gpu(gp))
    rgv, _, _ = oracle.rasterise_bwd(v[None], c[None], f[None], ref, gp[None], gb)
    assert_close_grad(vt.grad.cpu().numpy(), rgv[0], "grad_vertices")


def test_recompute_abi_flags_accumulate_and_clean_workspace():
    """Direct C-ABI calls: DIRT_BWD_ACCUMULATE adds into the caller's buffers; a workspace zero-filled once
    and reused with DIRT_BWD_SCRATCH_CLEAN gives the same results call after call."""
    from dirt_amd import _lib
    lib = _lib.load()
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=3000, W=200, H=150, radius_px=12.0, seed=12))
    B, H, W, C = bg.shape
    V, F = v.shape[1], f.shape[1]
    px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
    gp = np.random.default_rng(8).standard_normal(bg.shape).astype(np.float32)
    rgv, rgc, rgbg = oracle.rasterise_bwd(v, c, f, px, gp, gb)
    t = {k: _gpu(a) for k, a in dict(bg=bg, v=v, c=c, f=f, px=px, gp=gp).items()}
    n = _lib.recompute_workspace_size(B, H, W, C, V, F)
    ws = torch.zeros((n,), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream

    def call(gv, gc, gbg, flags):
        _lib.check(lib.dirt_rasterise_bwd_recompute(
            t["bg"].data_ptr(), t["v"].data_ptr(), t["c"].data_ptr(), t["f"].data_ptr(), t["px"].data_ptr(),
            t["gp"].data_ptr(), B, H, W, C, V, F, gv.data_ptr(), gc.data_ptr(), gbg.data_ptr(), ws.data_ptr(), n,
            flags, stream))

    outs = []
    for _ in range(3):
        gv = torch.full((B, V, 4), 7.0, device="cuda")
        gc = torch.full((B, V, C), 7.0, device="cuda")
        gbg = torch.empty((B, H, W, C), device="cuda")
        call(gv, gc, gbg, _lib.BWD_SCRATCH_CLEAN)  # overwrite: the 7s are replaced
        outs.append((gv.cpu().numpy(), gc.cpu().numpy(), gbg.cpu().numpy()))
    for gv, gc, gbg in outs:
        np.testing.assert_array_equal(gbg, rgbg)
        assert_close_grad(gv, rgv, "grad_vertices")
        assert_close_grad(gc, rgc, "grad_vertex_colors")
    # accumulate: a second call adds the same gradient again
    gv = torch.zeros((B, V, 4), device="cuda")
    gc = torch.zeros((B, V, C), device="cuda")
    gbg = torch.empty((B, H, W, C), device="cuda")
    call(gv, gc, gbg, _lib.BWD_SCRATCH_CLEAN | _lib.BWD_ACCUMULATE)
    call(gv, gc, gbg, _lib.BWD_SCRATCH_CLEAN | _lib.BWD_ACCUMULATE)
    assert_close_grad(gv.cpu().numpy(), 2 * rgv, "grad_vertices x2")
    assert_close_grad(gc.cpu().numpy(), 2 * rgc, "grad_vertex_colors x2")
    np.testing.assert_array_equal(gbg.cpu().numpy(), rgbg)
    # a workspace smaller than asked for is refused before any launch
    rc = lib.dirt_rasterise_bwd_recompute(
        t["bg"].data_ptr(), t["v"].data_ptr(), t["c"].data_ptr(), t["f"].data_ptr(), t["px"].data_ptr(),
        t["gp"].data_ptr(), B, H, W, C, V, F, gv.data_ptr(), gc.data_ptr(), gbg.data_ptr(), ws.data_ptr(), n - 1,
        0, stream)
    assert rc == _lib.DIRT_EINVAL and b"workspace" in lib.dirt_last_error()
