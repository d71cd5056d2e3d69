"""ctypes binding of libdirt_mi355x.so (the C ABI in include/dirt_mi355x.h).

This is the Python analogue of `tf.load_op_library(_lib_path + '/librasterise.so')`
(reference dirt/rasterise_ops.py:6-7): the shared library is loaded from the package directory.
There is no fallback: if the library is missing or cannot be loaded the import of the op fails loudly.
"""
import ctypes
import functools
import os

_here = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DIRT_MI355X_LIB", os.path.join(_here, "libdirt_mi355x.so"))

DIRT_OK = 0
DIRT_EINVAL = 1
DIRT_EFACE = 2
DIRT_EHIP = 3

SHADER_GOURAUD = 0
SHADER_OCEANIC_HORIZON = 1
SHADER_OCEANIC = 2
SHADER_OCEANIC_STILL_CLOUD = 3
SHADER_OCEANIC_NO_CLOUD = 4
SHADER_OCEANIC_SIMPLE_PROXY = 5
SHADER_OCEANIC_OPT_FLOW = 6
SHADER_HILL = 7

MAX_CHANNELS = 8
MAX_DIM = 8192
ABI_VERSION = 13

FWD_SCRATCH_CLEAN = 1  # dirt_rasterise_fwd flags
FWD_DEEP_CULL = 2      # dirt_rasterise_fwd: occluder culling for deep scenes (forced; automatic since ABI 12)
FWD_DEEP_CULL_OFF = 8  # dirt_rasterise_fwd: never the occluder culling
BWD_ACCUMULATE = 1     # dirt_rasterise_bwd / dirt_rasterise_bwd_recompute flags
BWD_SCRATCH_CLEAN = 2  # dirt_rasterise_bwd_recompute: the workspace's bin counters are clean

# every symbol include/dirt_mi355x.h declares, with its ctypes signature
_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t
_U = ctypes.c_uint
SIGNATURES = {
    "dirt_abi_version": (_I, []),
    "dirt_workspace_sizes": (_I, [_I, _I, _I, _I, _I, _I, _I64, ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
    "dirt_rasterise_fwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _SZ, _P, _SZ, _I64, _U,
                                _P, _P, _P]),
    "dirt_rasterise_fwd_gbuffer": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _SZ, _P, _SZ, _I64, _U,
                                        _P, _P, _P, _P, _P, _P]),
    "dirt_hill_fwd": (_I, [_P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _SZ, _P, _SZ, _I64, _P]),
    "dirt_rasterise_fwd_resolve": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _SZ, _P, _P, _P, _P, _P]),
    "dirt_rasterise_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _U, _P]),
    "dirt_bwd_recompute_workspace_size": (_I, [_I, _I, _I, _I, _I, _I, ctypes.POINTER(_SZ)]),
    "dirt_rasterise_bwd_recompute": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _SZ, _U,
                                          _P]),
    "dirt_rasterise_fwd_stash": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _SZ, _U, _P]),
    "dirt_scratch_clear": (_I, [_I, _I, _I, _I, _I64, _P, _SZ, _P]),
    "dirt_check_faces": (_I, [_P, _I, _I, _I, _P, _SZ, _P]),
    "dirt_stream_capture_id": (_I, [_P, ctypes.POINTER(ctypes.c_ulonglong)]),
    "dirt_profile_enable": (_I, [_I]),
    "dirt_profile_read": (_I, [_I, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_double)]),
    "dirt_vertex_normals_fwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _P, _P]),
    "dirt_vertex_normals_bwd": (_I, [_P, _I, _P, _I, _I, _I, _I, _P, _P, _P, _P, _I, _P]),
    "dirt_diffuse_directional_fwd": (_I, [_P, _P, _I64, _P, _P, _I, _P, _P]),
    "dirt_diffuse_directional_bwd": (_I, [_P, _P, _I64, _P, _P, _I, _P, _P, _P, _P]),
    "dirt_diffuse_point_fwd": (_I, [_P, _P, _P, _I64, _P, _P, _I, _P, _P]),
    "dirt_diffuse_point_bwd": (_I, [_P, _P, _P, _I64, _P, _P, _I, _P, _P, _P, _P, _P]),
    "dirt_specular_directional_fwd": (_I, [_P, _P, _P, _I64, _P, _P, _P, ctypes.c_float, _I, _P, _P]),
    "dirt_specular_directional_bwd": (_I, [_P, _P, _P, _I64, _P, _P, _P, ctypes.c_float, _I, _P, _P, _P, _P, _P]),
    "dirt_last_error": (ctypes.c_char_p, []),
}

_lib = None


class DirtError(RuntimeError):
    pass


def load():
    """Load (once) and return the library, raising if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libdirt_mi355x.so not found at %s; build it with `make` (or __graft_entry__.build())" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dirt_abi_version() != ABI_VERSION:
        raise ImportError("%s has ABI version %d, this binding expects %d: rebuild with `make`"
                          % (LIB_PATH, lib.dirt_abi_version(), ABI_VERSION))
    _lib = lib
    return lib


def check(rc):
    """Map a C-ABI return code to a Python exception (mirrors OP_REQUIRES -> InvalidArgument)."""
    if rc == DIRT_OK:
        return
    msg = load().dirt_last_error().decode("utf-8", "replace")
    if rc == DIRT_EINVAL:
        raise ValueError(msg)
    if rc == DIRT_EFACE:
        raise IndexError(msg)
    raise DirtError(msg)


@functools.lru_cache(maxsize=256)
def workspace_sizes(B, H, W, C, V, F, bin_capacity=0):
    lib = load()
    saved = ctypes.c_size_t(0)
    scratch = ctypes.c_size_t(0)
    check(lib.dirt_workspace_sizes(B, H, W, C, V, F, bin_capacity, ctypes.byref(saved), ctypes.byref(scratch)))
    return saved.value, scratch.value


@functools.lru_cache(maxsize=256)
def recompute_workspace_size(B, H, W, C, V, F):
    n = ctypes.c_size_t(0)
    check(load().dirt_bwd_recompute_workspace_size(B, H, W, C, V, F, ctypes.byref(n)))
    return n.value


def capture_id(stream):
    """Id of the HIP graph capture `stream` (a hipStream_t handle) is recording, 0 when none."""
    cid = ctypes.c_ulonglong(0)
    check(load().dirt_stream_capture_id(stream, ctypes.byref(cid)))
    return cid.value


def clip_stats(B, H, W, F, bin_capacity, scratch, scratch_bytes, stream, reset=True):
    """Debug (synchronises `stream`): the R5 deviation counters a forward scratch holds, summed since it was last
    cleared -- {"cap_culled": faces culled by the R5 vertex cap, "clamped": clipped faces whose sub-vertices the
    R5 clamp moved}.  `scratch` is a device pointer; reset zeroes the counters afterwards."""
    lib = load()
    fn = lib.dirt_debug_clip_stats
    fn.restype = ctypes.c_int
    fn.argtypes = [_I, _I, _I, _I, _I64, _P, _SZ, _P, _I, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    cap, clamped = ctypes.c_uint32(0), ctypes.c_uint32(0)
    check(fn(B, H, W, F, bin_capacity, scratch, scratch_bytes, stream, 1 if reset else 0, ctypes.byref(cap),
             ctypes.byref(clamped)))
    return {"cap_culled": cap.value, "clamped": clamped.value}


def stash_state(B, H, W, C, V, F, workspace, workspace_bytes, stream):
    """Debug (synchronises `stream`): {"last_missed": 1 if the last dirt_rasterise_bwd_recompute on this workspace
    recomputed, 0 if it reused the gradient stash; "magic": the stash header's magic word (0 = never written)}."""
    lib = load()
    fn = lib.dirt_debug_stash_state
    fn.restype = ctypes.c_int
    fn.argtypes = [_I] * 6 + [_P, _SZ, _P, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    miss, magic = ctypes.c_uint32(0), ctypes.c_uint32(0)
    check(fn(B, H, W, C, V, F, workspace, workspace_bytes, stream, ctypes.byref(miss), ctypes.byref(magic)))
    return {"last_missed": miss.value, "magic": magic.value}


def deep_cull_state():
    """Debug: the automatic deep-scene culling rule of the current device -- {"gen": forwards issued with it,
    "last_deep": generation of the last forward reported deep (0 = none), "next_deep": whether the next forward
    takes the occluder-culling raster}.  Reflects the launches the device has executed so far (no sync)."""
    lib = load()
    fn = lib.dirt_debug_deep_cull_state
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int)]
    gen, last, nxt = ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
    check(fn(ctypes.byref(gen), ctypes.byref(last), ctypes.byref(nxt)))
    return {"gen": gen.value, "last_deep": last.value, "next_deep": bool(nxt.value)}


NUM_KERNELS = 3


def profile_enable(on=True):
    check(load().dirt_profile_enable(1 if on else 0))


def profile_read():
    """{kernel name: (launches, total_ms)} for the launches recorded since profile_enable(True)."""
    lib = load()
    out = {}
    for k in range(NUM_KERNELS):
        name = ctypes.c_char_p()
        n = ctypes.c_int(0)
        ms = ctypes.c_double(0)
        check(lib.dirt_profile_read(k, ctypes.byref(name), ctypes.byref(n), ctypes.byref(ms)))
        out[name.value.decode()] = (n.value, ms.value)
    return out
