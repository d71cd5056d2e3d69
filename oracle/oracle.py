"""ctypes wrapper of the CPU oracle (oracle/dirt_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the product
(dirt_amd/) never does.  See the header of dirt_oracle.c for what it restates and its parity status.
"""
import ctypes
import os
import subprocess

import numpy as np

_here = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_here, "libdirt_oracle.so")
_lib = None


def build():
    src = os.path.join(_here, "dirt_oracle.c")
    if not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-C", os.path.dirname(_here), "oracle/libdirt_oracle.so"])


def load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(LIB_PATH)
        P, I = ctypes.c_void_p, ctypes.c_int
        lib.oracle_rasterise_fwd.argtypes = [P, P, P, P, I, I, I, I, I, I, P, P, I]
        lib.oracle_rasterise_fwd.restype = I
        lib.oracle_rasterise_fwd_shader.argtypes = [P, P, P, P, I, I, I, I, I, I, I, P, P, P, I]
        lib.oracle_rasterise_fwd_shader.restype = I
        lib.oracle_oceanic_horizon_pixel.argtypes = [P, I, I, I, ctypes.c_float, ctypes.c_float, P, P]
        lib.oracle_oceanic_horizon_pixel.restype = None
        lib.oracle_oceanic_family_pixel.argtypes = [I, P, I, I, I, ctypes.c_float, ctypes.c_float, P, P]
        lib.oracle_oceanic_family_pixel.restype = None
        lib.oracle_rasterise_bwd.argtypes = [P, P, P, P, P, P, I, I, I, I, I, I, P, P, P, I]
        lib.oracle_rasterise_bwd.restype = I
        lib.oracle_max_threads.argtypes = []
        lib.oracle_max_threads.restype = I
        _lib = lib
    return _lib


def _f32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.float32))


def _i32(x):
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32))


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def rasterise_fwd(background, vertices, vertex_colors, faces, nthreads=0, shader_id=0, camera_pos=None):
    """Batched forward.  background [B,H,W,C], vertices [B,V,4], vertex_colors [B,V,C], faces [B,F,3].
    shader_id 0 = Gouraud, 1 = oceanic_horizon (camera_pos: 8 floats).

    Returns (pixels [B,H,W,C] float32, gbuffer [B,H,W] int32 record index or -1, status)."""
    bg, vs, cs, fs = _f32(background), _f32(vertices), _f32(vertex_colors), _i32(faces)
    B, H, W, C = bg.shape
    V, F = vs.shape[1], fs.shape[1]
    pixels = np.empty((B, H, W, C), np.float32)
    gbuf = np.empty((B, H, W), np.int32)
    cam = np.zeros(16, np.float32)
    if camera_pos is not None:
        c = _f32(camera_pos).reshape(-1)
        cam[:c.size] = c
        if shader_id >= 1 and c.size < (9 if shader_id == 3 else 8):
            raise ValueError("procedural programs need camera_pos (8 floats, 9 for oceanic_still_cloud)")
    st = load().oracle_rasterise_fwd_shader(_ptr(bg), _ptr(vs), _ptr(cs), _ptr(fs), B, H, W, C, V, F, shader_id,
                                            _ptr(cam), _ptr(pixels), _ptr(gbuf), nthreads)
    return pixels, gbuf, st


def oceanic_horizon_pixel(background_frame, tx, ty, camera_pos):
    """The fragment program alone at texCoordV = (tx, ty) of a [H,W,C] background: returns (col.x, col.y)."""
    bg = _f32(background_frame)
    H, W, C = bg.shape
    out = np.zeros(2, np.float32)
    cam = _f32(camera_pos)
    load().oracle_oceanic_horizon_pixel(_ptr(bg), H, W, C, float(tx), float(ty), _ptr(cam), _ptr(out))
    return out


def rasterise_bwd(vertices, vertex_colors, faces, pixels, grad_pixels, gbuffer, nthreads=0):
    """Batched backward: returns (grad_vertices [B,V,4], grad_vertex_colors [B,V,C], grad_background)."""
    vs, cs, fs = _f32(vertices), _f32(vertex_colors), _i32(faces)
    px, gp, gb = _f32(pixels), _f32(grad_pixels), _i32(gbuffer)
    B, H, W, C = px.shape
    V, F = vs.shape[1], fs.shape[1]
    gv = np.empty((B, V, 4), np.float32)
    gc = np.empty((B, V, C), np.float32)
    gbg = np.empty((B, H, W, C), np.float32)
    load().oracle_rasterise_bwd(_ptr(vs), _ptr(cs), _ptr(fs), _ptr(px), _ptr(gp), _ptr(gb), B, H, W, C, V, F,
                                _ptr(gv), _ptr(gc), _ptr(gbg), nthreads)
    return gv, gc, gbg


def rasterise(background, vertices, vertex_colors, faces):
    """Single-frame convenience mirror of dirt.rasterise."""
    p, g, _ = rasterise_fwd(np.asarray(background)[None], np.asarray(vertices)[None],
                            np.asarray(vertex_colors)[None], np.asarray(faces)[None])
    return p[0], g[0]


def max_threads():
    return load().oracle_max_threads()
