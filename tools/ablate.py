"""Interleaved A/B timing of grad_kernel ablation variants (one process, median of N rounds).

    python tools/ablate.py          # config 3 (50k random triangles, 1024^2 x 3): backward and raster
    python tools/ablate.py c4       # config 4 (20k-tri shared-vertex mesh, 512^2 x 7): backward only
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import scenes  # noqa: E402
from dirt_amd import _lib  # noqa: E402
from dirt_amd.session import RasteriseSession  # noqa: E402

NAMES = {0: "full", 1: "no pairs", 2: "no colour", 3: "no pairs+colour", 4: "no reduction", 5: "no pairs+reduction",
         7: "nothing but staging", 8: "no flush", 16: "no coverage tests", 32: "no DPP scan (all lanes add)",
         64: "no LDS adds", 72: "no LDS adds, no flush", 256: "flush without global atomics"}


def main():
    dev = torch.device("cuda", 0)
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    if which == "c4":
        bg, v, c, f = scenes.deferred_mesh_scene()
    else:
        bg, v, c, f = scenes.random_triangles(F=50000, W=1024, H=1024, seed=0)
    t = [torch.from_numpy(a[None]).to(dev) for a in (bg, v, c, f)]
    B, H, W, C = t[0].shape
    V, F = t[1].shape[1], t[3].shape[1]
    sess = RasteriseSession(B, H, W, C, V, F, device=dev)
    sess.forward(*t)
    g = torch.randn_like(sess.pixels)
    lib = _lib.load()
    fn = lib.dirt_debug_bwd_variant
    P = ctypes.c_void_p
    fn.argtypes = [ctypes.c_int, P, P, P, P] + [ctypes.c_int] * 6 + [P, P, P, P, ctypes.POINTER(ctypes.c_float)]
    fn.restype = ctypes.c_int
    stream = torch.cuda.current_stream().cuda_stream
    res = {k: [] for k in NAMES}
    ms = ctypes.c_float(0)
    for rnd in range(30):
        for k in NAMES:
            _lib.check(fn(k, sess.pixels.data_ptr(), g.data_ptr(), sess.gbuffer.data_ptr(), sess.saved.data_ptr(),
                          B, H, W, C, V, F, sess.grad_vertices.data_ptr(), sess.grad_vertex_colors.data_ptr(),
                          sess.grad_background.data_ptr(), stream, ctypes.byref(ms)))
            if rnd >= 3:
                res[k].append(ms.value * 1e3)
    for k, name in NAMES.items():
        print("grad   %-28s median %8.2f us  min %8.2f" % (name, np.median(res[k]), np.min(res[k])))
    if C != 3:
        return  # the raster variants are instantiated for C = 3 only
    rfn = lib.dirt_debug_raster_variant
    rfn.argtypes = [ctypes.c_int, P, P, P, P] + [ctypes.c_int] * 6 + [P, P, P, P, P, ctypes.POINTER(ctypes.c_float)]
    rfn.restype = ctypes.c_int
    RN = {0: "full", 1: "no pixel loop, no resolve", 2: "bin filter only, no resolve", 4: "no resolve",
          8: "nothing (housekeeping + bg prefetch + gbuffer write)", 32: "no coverage bits",
          64: "no colour loads", 96: "no coverage bits, no colour loads",
          512: "one extra round trip before the slab loads", 1024: "one extra round trip before the colour loads",
          2048: "one extra round trip before the record loads"}
    rres = {k: [] for k in RN}
    for rnd in range(30):
        for k in RN:
            _lib.check(rfn(k, t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), B, H, W, C, V, F,
                           sess.pixels.data_ptr(),
                           sess.gbuffer.data_ptr(), sess.saved.data_ptr(), sess.scratch.data_ptr(), stream,
                           ctypes.byref(ms)))
            if rnd >= 3:
                rres[k].append(ms.value * 1e3)
    for k, name in RN.items():
        print("raster %-28s median %8.2f us  min %8.2f" % (name, np.median(rres[k]), np.min(rres[k])))


if __name__ == "__main__":
    main()
