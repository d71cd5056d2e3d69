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
        lib.oracle_rasterise_fwd_gbuffer.argtypes = [P, P, P, P, I, I, I, I, I, I, P, P, P, P, P, I]
        lib.oracle_rasterise_fwd_gbuffer.restype = I
        lib.oracle_oceanic_horizon_pixel.argtypes = [P, I, I, I, ctypes.c_float, ctypes.c_float, P, P]
        lib.oracle_oceanic_horizon_pixel.restype = None
        lib.oracle_oceanic_family_pixel.argtypes = [I, P, I, I, I, ctypes.c_float, ctypes.c_float, P, P]
        lib.oracle_oceanic_family_pixel.restype = None
        lib.oracle_opt_flow_pixel.argtypes = [ctypes.c_float, ctypes.c_float, P, ctypes.c_float, ctypes.c_float, P]
        lib.oracle_opt_flow_pixel.restype = None
        lib.oracle_hill_pixel.argtypes = [P, I, I, I, ctypes.c_float, ctypes.c_float, P, P]
        lib.oracle_hill_pixel.restype = None
        lib.oracle_hill_fwd.argtypes = [P, I, P, P, I, I, I, I, I, I, P, P, P, I]
        lib.oracle_hill_fwd.restype = I
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


CAMERA_FLOATS = {3: 9, 6: 16, 7: 12}


def hill_fwd(terrain, vertices, faces, channels, camera_pos, nthreads=0):
    """The Hill op: terrain [B,H,W,Ct] (Ct in 1/3/4), vertices [B,V,4], faces [B,F,3], camera_pos (12
    floats).  Returns (pixels [B,H,W,channels], gbuffer, status)."""
    tr, vs, fs = _f32(terrain), _f32(vertices), _i32(faces)
    B, H, W, Ct = tr.shape
    V, F = vs.shape[1], fs.shape[1]
    pixels = np.empty((B, H, W, channels), np.float32)
    gbuf = np.empty((B, H, W), np.int32)
    cam = np.zeros(16, np.float32)
    c = _f32(camera_pos).reshape(-1)
    if c.size < 12:
        raise ValueError("hill needs camera_pos (12 floats)")
    cam[:min(c.size, 16)] = c[:16]
    st = load().oracle_hill_fwd(_ptr(tr), Ct, _ptr(vs), _ptr(fs), B, H, W, channels, V, F, _ptr(cam), _ptr(pixels),
                                _ptr(gbuf), nthreads)
    return pixels, gbuf, st


def opt_flow_pixel(tx, ty, camera_pos, width, height):
    """oceanic_opt_flow's fragment program alone at texCoordV = (tx, ty): returns new_coord (2 floats)."""
    out = np.zeros(2, np.float32)
    cam = np.zeros(16, np.float32)
    c = _f32(camera_pos).reshape(-1)
    cam[:min(c.size, 16)] = c[:16]
    load().oracle_opt_flow_pixel(float(tx), float(ty), _ptr(cam), float(width), float(height), _ptr(out))
    return out


def hill_pixel(terrain_frame, tx, ty, camera_pos):
    """hill's fragment program alone at texCoordV = (tx, ty) over a [H,W,Ct] terrain: returns fragColor."""
    tr = _f32(terrain_frame)
    H, W, Ct = tr.shape
    out = np.zeros(4, np.float32)
    cam = np.zeros(16, np.float32)
    c = _f32(camera_pos).reshape(-1)
    cam[:min(c.size, 16)] = c[:16]
    load().oracle_hill_pixel(_ptr(tr), H, W, Ct, float(tx), float(ty), _ptr(cam), _ptr(out))
    return out


def rasterise_fwd(background, vertices, vertex_colors, faces, nthreads=0, shader_id=0, camera_pos=None):
    """Batched forward.  background [B,H,W,C], vertices [B,V,4], vertex_colors [B,V,C], faces [B,F,3].
    shader_id 0 = Gouraud, 1 = oceanic_horizon, 2..5 the oceanic family, 6 oceanic_opt_flow (camera_pos:
    8 floats; 9 for oceanic_still_cloud, 16 for oceanic_opt_flow).

    Returns (pixels [B,H,W,C] float32, gbuffer [B,H,W] int32 record index or -1, status)."""
    bg, vs, cs, fs = _f32(background), _f32(vertices), _f32(vertex_colors), _i32(faces)
    B, H, W, C = bg.shape
    V, F = vs.shape[1], fs.shape[1]
    pixels = np.empty((B, H, W, C), np.float32)
    gbuf = np.empty((B, H, W), np.int32)
    cam = np.zeros(16, np.float32)
    if camera_pos is not None:
        c = _f32(camera_pos).reshape(-1)
        cam[:min(c.size, 16)] = c[:16]
        if shader_id >= 1 and c.size < CAMERA_FLOATS.get(shader_id, 8):
            raise ValueError("procedural programs need camera_pos (%d floats)" % CAMERA_FLOATS.get(shader_id, 8))
    st = load().oracle_rasterise_fwd_shader(_ptr(bg), _ptr(vs), _ptr(cs), _ptr(fs), B, H, W, C, V, F, shader_id,
                                            _ptr(cam), _ptr(pixels), _ptr(gbuf), nthreads)
    return pixels, gbuf, st


def rasterise_fwd_gbuffer(background, vertices, vertex_colors, faces, nthreads=0):
    """Gouraud forward plus the deferred-shading G-buffer (dirt_rasterise_fwd_gbuffer).

    Returns (pixels [B,H,W,C], gbuffer [B,H,W], depth [B,H,W] float32, barycentrics [B,H,W,3] float32,
    face_ids [B,H,W] int32, status)."""
    bg, vs, cs, fs = _f32(background), _f32(vertices), _f32(vertex_colors), _i32(faces)
    B, H, W, C = bg.shape
    V, F = vs.shape[1], fs.shape[1]
    pixels = np.empty((B, H, W, C), np.float32)
    gbuf = np.empty((B, H, W), np.int32)
    depth = np.empty((B, H, W), np.float32)
    bary = np.empty((B, H, W, 3), np.float32)
    face = np.empty((B, H, W), np.int32)
    st = load().oracle_rasterise_fwd_gbuffer(_ptr(bg), _ptr(vs), _ptr(cs), _ptr(fs), B, H, W, C, V, F, _ptr(pixels),
                                             _ptr(gbuf), _ptr(depth), _ptr(bary), _ptr(face), nthreads)
    return pixels, gbuf, depth, bary, face, st


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
