"""GPU parity of the `oceanic_horizon` fragment program (shader_id 1): the HIP resolve
against the CPU oracle, bit for bit (both state the GLSL of csrc/shaders.cpp:1668-1919 in float32 with
the same fixed sin/cos/pow algorithms, no contraction, IEEE division and sqrt)."""
import os

import numpy as np
import pytest
import torch

import scenes
from oracle import oracle
from test_oceanic_oracle import CAMS, fullscreen

pytestmark = pytest.mark.gpu


def gpu_fwd(bg, v, c, f, cam):
    from dirt_amd import rasterise_ops
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (bg, v, c, f)]
    B, H, W, C = bg.shape
    px, gb = rasterise_ops._rasterise_batched(*t, torch.tensor(cam, dtype=torch.float32).cuda(), H, W, C, 1,
                                              return_gbuffer=True)
    return px.cpu().numpy(), gb.cpu().numpy()


def check(bg, v, c, f, cam):
    px, gb = gpu_fwd(bg, v, c, f, cam)
    rpx, rgb, _ = oracle.rasterise_fwd(bg, v, c, f, shader_id=1, camera_pos=np.array(cam, np.float32))
    np.testing.assert_array_equal(gb, rgb)
    np.testing.assert_array_equal(px, rpx)
    return px


@pytest.mark.parametrize("name", sorted(CAMS))
def test_fullscreen_harness_960x640(name):
    px = check(*fullscreen(640, 960), CAMS[name])
    assert 0.0 < px[0, ..., 0].mean() < 1.0


def test_background_jitter_and_channel_counts():
    H, W = 96, 128
    bg = np.random.default_rng(3).uniform(-3, 3, size=(H, W, 4)).astype(np.float32)
    for C in (1, 3, 4):
        check(*fullscreen(H, W, C=C, background=bg[..., :C].copy()), CAMS["square_test"])


def test_mesh_with_perspective_and_uncovered_pixels():
    bg, v, c, f = scenes.random_triangles(F=600, W=160, H=120, radius_px=20.0, seed=4, perspective=True)
    check(bg[None], v[None], c[None], f[None], CAMS["rolled_moving"])
    bg, v, c, f = scenes.batch_of(scenes.random_triangles, 3, F=300, W=96, H=64, radius_px=12.0, seed=9)
    check(bg, v, c, f, CAMS["optimize_horizon"])


def test_public_api_and_no_gradient():
    import dirt_amd
    bg, v, c, f = (a[0] for a in fullscreen(64, 96))
    cam = torch.tensor(CAMS["optimize_horizon"]).cuda()
    px = dirt_amd.rasterise(torch.from_numpy(bg).cuda(), torch.from_numpy(v).cuda().requires_grad_(True),
                            torch.from_numpy(c).cuda(), torch.from_numpy(f).cuda(), camera_pos=cam,
                            shader="oceanic_horizon")
    ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None], shader_id=1,
                                     camera_pos=np.array(CAMS["optimize_horizon"], np.float32))
    np.testing.assert_array_equal(px.detach().cpu().numpy(), ref[0])
    with pytest.raises(RuntimeError, match="gradient"):
        px.sum().backward()
    with pytest.raises(ValueError, match="camera_pos"):
        dirt_amd.rasterise(torch.from_numpy(bg).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(c).cuda(),
                           torch.from_numpy(f).cuda(), shader="oceanic_horizon")


def test_session_oceanic_matches_op():
    from dirt_amd.session import RasteriseSession
    bg, v, c, f = fullscreen(128, 192)
    cam = torch.tensor(CAMS["square_test"]).cuda()
    sess = RasteriseSession(1, 128, 192, 3, 4, 2, shader_id=1)
    t = [torch.from_numpy(a).cuda() for a in (bg, v, c, f)]
    for _ in range(2):
        px = sess.forward(*t, camera_pos=cam)
    ref, _, _ = oracle.rasterise_fwd(bg, v, c, f, shader_id=1, camera_pos=np.array(CAMS["square_test"], np.float32))
    np.testing.assert_array_equal(px.cpu().numpy(), ref)


FAMILY_CAMS = [[0.0, 150.0, 0.0, 0.0, 0.1, 0.0, 1.0, 0.9, 2.0], [5.0, 120.0, -20.0, 0.02, -0.15, 0.05, 3.0, 1.2, 0.5]]


@pytest.mark.parametrize("sid", [2, 3, 4, 5], ids=["oceanic", "still_cloud", "no_cloud", "simple_proxy"])
def test_oceanic_family_bit_exact(sid):
    for cam in FAMILY_CAMS:
        px, gb = _family_fwd(sid, *fullscreen(96, 128), cam=cam)
        rpx, rgb, _ = oracle.rasterise_fwd(*fullscreen(96, 128), shader_id=sid, camera_pos=np.array(cam, np.float32))
        np.testing.assert_array_equal(gb, rgb)
        np.testing.assert_array_equal(px, rpx)


def _family_fwd(sid, bg, v, c, f, cam):
    from dirt_amd import rasterise_ops
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (bg, v, c, f)]
    B, H, W, C = bg.shape
    px, gb = rasterise_ops._rasterise_batched(*t, torch.tensor(cam, dtype=torch.float32).cuda(), H, W, C, sid,
                                              return_gbuffer=True)
    return px.cpu().numpy(), gb.cpu().numpy()


def test_procedural_op_names():
    """rasterise_grad (the fork's RasteriseGrad = `oceanic`) and the oceanic_* ops of
    dirt/rasterise_ops.py:91-165 on a mesh with uncovered pixels, bit-exact against the oracle."""
    import dirt_amd
    bg, v, c, f = scenes.random_triangles(F=60, W=80, H=64, radius_px=14.0, seed=2)
    cam = FAMILY_CAMS[1]
    for name, sid in (("rasterise_grad", 2), ("oceanic_still_cloud", 3), ("oceanic_no_cloud", 4),
                      ("oceanic_simple_proxy", 5)):
        px = getattr(dirt_amd, name)(torch.from_numpy(bg).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(c).cuda(),
                                     torch.from_numpy(f).cuda(), torch.tensor(cam).cuda())
        ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None], shader_id=sid,
                                         camera_pos=np.array(cam, np.float32))
        np.testing.assert_array_equal(px.cpu().numpy(), ref[0])


# ---- oceanic_opt_flow (shader id 6) and hill (shader id 7, dirt_hill_fwd) -------------------------------
from test_procedural_oracle import FLOW_CAMS, HILL_CAMS, hill_cam  # noqa: E402


@pytest.mark.parametrize("name", sorted(FLOW_CAMS))
def test_opt_flow_bit_exact(name):
    cam = FLOW_CAMS[name]
    for C in (1, 3, 4):
        px, gb = _family_fwd(6, *fullscreen(96, 128, C=C), cam=cam)
        rpx, rgb, _ = oracle.rasterise_fwd(*fullscreen(96, 128, C=C), shader_id=6, camera_pos=np.array(cam, np.float32))
        np.testing.assert_array_equal(gb, rgb)
        np.testing.assert_array_equal(px, rpx)


def test_opt_flow_mesh_and_public_op():
    import dirt_amd
    bg, v, c, f = scenes.random_triangles(F=300, W=120, H=80, C=3, radius_px=16.0, seed=8, perspective=True)
    cam = FLOW_CAMS["rotate"]
    px = dirt_amd.oceanic_opt_flow(torch.from_numpy(bg).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(c).cuda(),
                                   torch.from_numpy(f).cuda(), torch.tensor(cam).cuda())
    ref, _, _ = oracle.rasterise_fwd(bg[None], v[None], c[None], f[None], shader_id=6,
                                     camera_pos=np.array(cam, np.float32))
    np.testing.assert_array_equal(px.cpu().numpy(), ref[0])
    with pytest.raises(ValueError, match="16"):
        dirt_amd.oceanic_opt_flow(torch.from_numpy(bg).cuda(), torch.from_numpy(v).cuda(), torch.from_numpy(c).cuda(),
                                  torch.from_numpy(f).cuda(), torch.zeros(15).cuda())


def _hill_gpu(T, v, f, C, cam):
    from dirt_amd import _lib
    B, H, W, Ct = T.shape
    V, F = v.shape[1], f.shape[1]
    lib = _lib.load()
    saved_b, scratch_b = _lib.workspace_sizes(B, H, W, C, V, F, 0)
    t, vv, ff, cc = (torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (T, v, f, cam))
    px = torch.empty((B, H, W, C), dtype=torch.float32, device="cuda")
    gb = torch.empty((B, H, W), dtype=torch.int32, device="cuda")
    saved = torch.empty(max(saved_b, 1), dtype=torch.uint8, device="cuda")
    scratch = torch.empty(max(scratch_b, 1), dtype=torch.uint8, device="cuda")
    _lib.check(lib.dirt_hill_fwd(t.data_ptr(), Ct, vv.data_ptr(), ff.data_ptr(), cc.data_ptr(), B, H, W, C, V, F,
                                 px.data_ptr(), gb.data_ptr(), saved.data_ptr(), saved_b, scratch.data_ptr(), scratch_b,
                                 0, torch.cuda.current_stream().cuda_stream))
    return px.cpu().numpy(), gb.cpu().numpy()


@pytest.mark.parametrize("name", sorted(HILL_CAMS))
def test_hill_bit_exact(name):
    v, f = scenes.fullscreen_quad()
    cam = hill_cam(HILL_CAMS[name])
    for (H, W) in ((54, 96), (64, 64), (40, 9), (23, 2)):  # (the last two: one tile column)
        for Ct, C in ((4, 3), (1, 1), (3, 4)):
            T = scenes.hill_terrain(H, W, Ct)[None]
            px, gb = _hill_gpu(T, v[None], f[None], C, cam)
            rpx, rgb, _ = oracle.hill_fwd(T, v[None], f[None], C, cam)
            np.testing.assert_array_equal(gb, rgb)
            np.testing.assert_array_equal(px, rpx)


def test_hill_harness_960x540_and_public_op():
    """tests/square_test.py:14-37: full-screen square, 960x540, channels=3, a 4-channel terrain lookup."""
    import dirt_amd
    v, f = scenes.fullscreen_quad()
    T = scenes.hill_terrain(540, 960, 4)
    cam = hill_cam(HILL_CAMS["harness"])
    px = dirt_amd.hill(torch.from_numpy(T).cuda(), torch.from_numpy(v).cuda(), torch.ones(4, 3).cuda(),
                       torch.from_numpy(f).cuda(), torch.from_numpy(cam).cuda(), height=540, width=960, channels=3)
    ref, _, _ = oracle.hill_fwd(T[None], v[None], f[None], 3, cam)
    np.testing.assert_array_equal(px.cpu().numpy(), ref[0])
    with pytest.raises(ValueError, match="12"):
        dirt_amd.hill(torch.from_numpy(T).cuda(), torch.from_numpy(v).cuda(), torch.ones(4, 3).cuda(),
                      torch.from_numpy(f).cuda(), torch.zeros(11).cuda(), channels=3)
    with pytest.raises(ValueError, match="1, 3 or 4"):
        dirt_amd.hill(torch.zeros(540, 960, 2).cuda(), torch.from_numpy(v).cuda(), torch.ones(4, 3).cuda(),
                      torch.from_numpy(f).cuda(), torch.from_numpy(cam).cuda(), channels=3)


def test_hill_overlap_and_mesh():
    """No depth test (last face wins) and uncovered pixels 0, on overlapping quads and a random mesh."""
    H, W = 32, 48
    T = scenes.hill_terrain(H, W, 4)[None]
    near = [[-0.5, -0.5, -0.5, 1], [-0.5, 0.5, -0.5, 1], [0.5, 0.5, -0.5, 1], [0.5, -0.5, -0.5, 1]]
    far = [[-0.8, -0.8, 0.5, 1], [-0.8, 0.8, 0.5, 1], [0.8, 0.8, 0.5, 1], [0.8, -0.8, 0.5, 1]]
    v = np.array([near + far], np.float32)
    f = np.array([[[0, 1, 2], [0, 2, 3], [4, 5, 6], [4, 6, 7]]], np.int32)
    cam = hill_cam(HILL_CAMS["harness"])
    px, gb = _hill_gpu(T, v, f, 3, cam)
    rpx, rgb, _ = oracle.hill_fwd(T, v, f, 3, cam)
    np.testing.assert_array_equal(gb, rgb)
    np.testing.assert_array_equal(px, rpx)
    _, v, _, f = scenes.random_triangles(F=400, W=96, H=64, C=3, radius_px=18.0, seed=12, perspective=True)
    T = scenes.hill_terrain(64, 96, 4)[None]
    px, gb = _hill_gpu(T, v[None], f[None], 3, cam)
    rpx, rgb, _ = oracle.hill_fwd(T, v[None], f[None], 3, cam)
    np.testing.assert_array_equal(gb, rgb)
    np.testing.assert_array_equal(px, rpx)


@pytest.mark.parametrize("seed", range(int(os.environ.get("DIRT_PROC_FUZZ_FIRST", "0")),
                                         int(os.environ.get("DIRT_PROC_FUZZ_SEEDS", "6"))))
def test_procedural_programs_adversarial_fuzz(seed):
    """The depth-tested procedural programs (oceanic_horizon and the oceanic family, shader ids 1..6 in turn)
    on the adversarial fuzz scenes (pixel-centre vertices, slivers, depth ties, clipping, w <= 0): bit-exact
    g-buffer and pixels.  DIRT_PROC_FUZZ_SEEDS=N widens it to the seeds below N (default 6: each program once),
    from DIRT_PROC_FUZZ_FIRST."""
    W, H = [(64, 48), (33, 17), (130, 70)][seed % 3]
    sid = 1 + seed % 6
    bg, v, c, f = (a[None] for a in scenes.adversarial_scene(300000 + seed, W=W, H=H, C=3))
    cam = np.array(list(CAMS["square_test"]) + [0.3, 0.05, 0.5, 0.0, -0.4, 0.01, 0.0, 0.02], np.float32)
    px, gb = _family_fwd(sid, bg, v, c, f, cam=cam)
    rpx, rgb, _ = oracle.rasterise_fwd(bg, v, c, f, shader_id=sid, camera_pos=cam)
    np.testing.assert_array_equal(gb, rgb)
    np.testing.assert_array_equal(px, rpx)


@pytest.mark.parametrize("seed", range(int(os.environ.get("DIRT_HILL_FUZZ_FIRST", "0")),
                                         int(os.environ.get("DIRT_HILL_FUZZ_SEEDS", "8"))))
def test_hill_adversarial_fuzz(seed):
    """hill (no depth test: the last face in draw order wins) on the adversarial fuzz scenes of
    tests/test_gpu_parity.py -- pixel-centre vertices, slivers, duplicates, clipping, w <= 0 -- bit-exact
    g-buffer and pixels.  DIRT_HILL_FUZZ_SEEDS=N widens it to the seeds below N (default 8),
    from DIRT_HILL_FUZZ_FIRST."""
    W, H = [(64, 48), (33, 17), (130, 70)][seed % 3]
    _, v, _, f = scenes.adversarial_scene(200000 + seed, W=W, H=H, C=3)
    T = scenes.hill_terrain(H, W, 4)[None]
    cam = hill_cam(HILL_CAMS["harness"])
    px, gb = _hill_gpu(T, v[None], f[None], 3, cam)
    rpx, rgb, _ = oracle.hill_fwd(T, v[None], f[None], 3, cam)
    np.testing.assert_array_equal(gb, rgb)
    np.testing.assert_array_equal(px, rpx)


@pytest.mark.parametrize("sid", [1, 2, 3, 4, 5, 6])
def test_programs_on_narrow_and_odd_frames(sid):
    """Every depth-tested fragment program on frames one tile column wide and on odd sizes (the tile-row
    split for a single tile column was wrong until the end of round 2)."""
    from dirt_amd import rasterise_ops
    cam = np.array(list(CAMS["square_test"]) + [0.3, 0.05, 0.5, 0.0, -0.4, 0.01, 0.0, 0.02], np.float32)
    for (H, W) in [(40, 9), (17, 33), (23, 1)]:
        bg, v, c, f = fullscreen(H, W)
        t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (bg, v, c, f)]
        px, gb = rasterise_ops._rasterise_batched(*t, torch.from_numpy(cam).cuda(), H, W, bg.shape[-1], sid,
                                                  return_gbuffer=True)
        rpx, rgb, _ = oracle.rasterise_fwd(bg, v, c, f, shader_id=sid, camera_pos=cam)
        np.testing.assert_array_equal(gb.cpu().numpy(), rgb)
        np.testing.assert_array_equal(px.cpu().numpy(), rpx)
