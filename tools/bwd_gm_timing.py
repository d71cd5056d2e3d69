"""Backward kernel time by requested gradients (dirt_rasterise_bwd with grad_vertex_colors / grad_vertices NULL):
vertices + colours (the full backward), vertices only, colours only -- at configs 3 and 4.

    python tools/bwd_gm_timing.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

dev = torch.device("cuda", 0)
lib = _lib.load()
for name, sc in (("c3", scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)), ("c4", scenes.deferred_mesh_scene())):
    bg, v, c, f = (torch.from_numpy(a[None]).to(dev) for a in sc)
    B, H, W, C = bg.shape
    V, F = v.shape[1], f.shape[1]
    sess = RasteriseSession(B, H, W, C, V, F, device=dev)
    sess.forward(bg, v, c, f)
    g = torch.randn_like(sess.pixels)
    gv = torch.empty((B, V, 4), device=dev)
    gc = torch.empty((B, V, C), device=dev)
    gbg = torch.empty((B, H, W, C), device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    res = {}
    for mode, pv, pc in (("vertices+colours", gv, gc), ("vertices only", gv, None), ("colours only", None, gc)):
        def call():
            _lib.check(lib.dirt_rasterise_bwd(v.data_ptr(), c.data_ptr(), f.data_ptr(), sess.pixels.data_ptr(),
                                              g.data_ptr(), sess.gbuffer.data_ptr(), sess.saved.data_ptr(), B, H, W, C,
                                              V, F, pv.data_ptr() if pv is not None else None,
                                              pc.data_ptr() if pc is not None else None, gbg.data_ptr(),
                                              _lib.BWD_ACCUMULATE, stream))
        for _ in range(10):
            call()
        torch.cuda.synchronize()
        _lib.profile_enable(True)
        for _ in range(100):
            call()
        torch.cuda.synchronize()
        prof = _lib.profile_read()
        _lib.profile_enable(False)
        n, ms = prof["grad_kernel"]
        res[mode] = round(ms / n * 1e3, 2)
    print(name, "grad_kernel us:", res)
