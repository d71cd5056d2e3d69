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


def test_gradient_stash_hits_misses_and_stays_exact():
    """VERDICT r4 item 3, ABI v11: dirt_rasterise_fwd_stash leaves the forward's records / g-buffer / coverage bits
    in the recompute workspace with a bitwise record of the geometry; dirt_rasterise_bwd_recompute on the same
    workspace skips its recomputation when vertices and faces are unchanged and recomputes otherwise.  Every
    outcome matches the oracle; the hit / miss itself is read back from the stash header."""
    from dirt_amd import _lib
    lib = _lib.load()
    scenes_ = [tuple(a[None] for a in scenes.random_triangles(F=3000, W=200, H=150, radius_px=12.0, seed=s))
               for s in (21, 22)]
    B, H, W, C = scenes_[0][0].shape
    V, F = scenes_[0][1].shape[1], scenes_[0][3].shape[1]
    n = _lib.recompute_workspace_size(B, H, W, C, V, F)
    ws = torch.zeros((n,), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    gp = np.random.default_rng(9).standard_normal((B, H, W, C)).astype(np.float32)
    refs = []
    for bg, v, c, f in scenes_:
        px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
        refs.append((px,) + tuple(oracle.rasterise_bwd(v, c, f, px, gp, gb)))
    dev = [{k: _gpu(a) for k, a in dict(bg=bg, v=v, c=c, f=f).items()} for bg, v, c, f in scenes_]
    gp_t = _gpu(gp)

    def fwd(k):
        px = torch.empty((B, H, W, C), device="cuda")
        d = dev[k]
        _lib.check(lib.dirt_rasterise_fwd_stash(d["bg"].data_ptr(), d["v"].data_ptr(), d["c"].data_ptr(),
                                                d["f"].data_ptr(), B, H, W, C, V, F, px.data_ptr(), ws.data_ptr(), n,
                                                _lib.FWD_SCRATCH_CLEAN, stream))
        np.testing.assert_array_equal(px.cpu().numpy(), refs[k][0])
        return px

    def bwd(k, px, expect_miss):
        d = dev[k]
        gv, gc = torch.empty((B, V, 4), device="cuda"), torch.empty((B, V, C), device="cuda")
        gbg = torch.empty((B, H, W, C), device="cuda")
        _lib.check(lib.dirt_rasterise_bwd_recompute(
            d["bg"].data_ptr(), d["v"].data_ptr(), d["c"].data_ptr(), d["f"].data_ptr(), px.data_ptr(), gp_t.data_ptr(),
            B, H, W, C, V, F, gv.data_ptr(), gc.data_ptr(), gbg.data_ptr(), ws.data_ptr(), n, _lib.BWD_SCRATCH_CLEAN,
            stream))
        st = _lib.stash_state(B, H, W, C, V, F, ws.data_ptr(), n, stream)
        assert st["last_missed"] == (1 if expect_miss else 0), (k, expect_miss, st)
        _, rgv, rgc, rgbg = refs[k]
        np.testing.assert_array_equal(gbg.cpu().numpy(), rgbg)
        assert_close_grad(gv.cpu().numpy(), rgv, "grad_vertices", strict=True)
        assert_close_grad(gc.cpu().numpy(), rgc, "grad_vertex_colors", strict=True)

    px0 = fwd(0)
    bwd(0, px0, expect_miss=False)   # the forward's own stash
    bwd(0, px0, expect_miss=False)   # again (nothing changed)
    px1 = fwd(1)
    bwd(0, px0, expect_miss=True)    # another geometry in between: recompute (and record scene 0)
    bwd(0, px0, expect_miss=False)   # ... which the next call reuses
    bwd(1, px1, expect_miss=True)
    # one vertex coordinate changed by one ulp in place: a miss, and the gradient of the new geometry
    dev[1]["v"].view(torch.int32)[0, 5, 0] += 1
    v2 = dev[1]["v"].cpu().numpy()
    px2, gb2, _ = oracle.rasterise_fwd(scenes_[1][0], v2, scenes_[1][2], scenes_[1][3])
    refs[1] = (px2,) + tuple(oracle.rasterise_bwd(v2, scenes_[1][2], scenes_[1][3], px2, gp, gb2))
    bwd(1, _gpu(px2), expect_miss=True)
    bwd(1, _gpu(px2), expect_miss=False)
    # faces changed (same vertices): a miss
    dev[1]["f"][0, [0, 1]] = dev[1]["f"][0, [1, 0]]
    f2 = dev[1]["f"].cpu().numpy()
    px3, gb3, _ = oracle.rasterise_fwd(scenes_[1][0], v2, scenes_[1][2], f2)
    refs[1] = (px3,) + tuple(oracle.rasterise_bwd(v2, scenes_[1][2], f2, px3, gp, gb3))
    bwd(1, _gpu(px3), expect_miss=True)


def test_single_output_op_reuses_its_forward_stash():
    """The op module's forward fills the stash its registered gradient then reuses: the gradient equals the
    stateful backward's, and the workspace reports a hit; three renders of one mesh with different colours
    (samples/deferred.py's G-buffer passes) share it."""
    from dirt_amd import _lib, op_library
    mod = op_library.load_op_library()
    op_library._stash_workspaces.clear()
    bg, v, c, f = (a[None] for a in scenes.random_triangles(F=4000, W=256, H=192, radius_px=10.0, seed=31))
    B, H, W, C = bg.shape
    vt = _gpu(v).requires_grad_(True)
    ft = _gpu(f)
    outs = []
    for k in range(3):
        ck = _gpu(np.roll(c, k, axis=-1)).requires_grad_(True)
        outs.append((mod.rasterise(_gpu(bg), vt, ck, ft, None, H, W, C), ck))
    gp = [torch.randn((B, H, W, C), device="cuda") for _ in range(3)]
    loss = sum((px * g).sum() for (px, _), g in zip(outs, gp))
    gv, = torch.autograd.grad(loss, [vt])
    ws = next(iter(op_library._stash_workspaces._d.values()))
    st = _lib.stash_state(B, H, W, C, v.shape[1], f.shape[1], ws.data_ptr(), ws.numel(),
                          torch.cuda.current_stream().cuda_stream)
    assert st["last_missed"] == 0 and st["magic"] != 0, st
    # reference: the stateful public op, same three renders
    import dirt_amd
    vt2 = _gpu(v).requires_grad_(True)
    loss2 = sum((dirt_amd.rasterise_batch(_gpu(bg), vt2, _gpu(np.roll(c, k, axis=-1)), ft) * g).sum()
                for k, g in enumerate(gp))
    gv2, = torch.autograd.grad(loss2, [vt2])
    assert_close_grad(gv.cpu().numpy(), gv2.cpu().numpy(), "grad_vertices (stash vs stateful)")
