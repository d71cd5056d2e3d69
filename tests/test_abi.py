"""CPU tests of the C-ABI boundary: the library loads, exports every symbol include/dirt_mi355x.h declares,
and validates arguments (reference OP_REQUIRES messages, csrc/rasterise_egl.cpp:310-336) before touching
the GPU.  No compute call is made here (there is no GPU in this container)."""
import ctypes
import os
import re

import pytest

from dirt_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dirt_mi355x.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dirt_\w+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for required in ("dirt_rasterise_fwd", "dirt_rasterise_bwd", "dirt_workspace_sizes", "dirt_last_error"):
        assert required in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding knows the signature of each
    assert set(declared_functions()) <= set(_lib.SIGNATURES)


def test_header_flags_match_the_binding():
    """The flag values the header #defines are the ones dirt_amd._lib passes (ABI 12 adds DIRT_FWD_DEEP_CULL_OFF),
    and the forward's flags are distinct bits."""
    text = open(HEADER).read()
    defs = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define\s+(DIRT_(?:FWD|BWD)_\w+)\s+(\d+)u", text)}
    assert defs["DIRT_FWD_SCRATCH_CLEAN"] == _lib.FWD_SCRATCH_CLEAN
    assert defs["DIRT_FWD_DEEP_CULL"] == _lib.FWD_DEEP_CULL
    assert defs["DIRT_FWD_DEEP_CULL_OFF"] == _lib.FWD_DEEP_CULL_OFF
    assert defs["DIRT_BWD_ACCUMULATE"] == _lib.BWD_ACCUMULATE
    assert defs["DIRT_BWD_SCRATCH_CLEAN"] == _lib.BWD_SCRATCH_CLEAN
    fwd = [v for k, v in defs.items() if k.startswith("DIRT_FWD_")]
    assert all(v & (v - 1) == 0 for v in fwd) and len(set(fwd)) == len(fwd)


def test_abi_version_and_workspace_sizes():
    lib = _lib.load()
    assert lib.dirt_abi_version() == _lib.ABI_VERSION == 13
    saved, scratch = _lib.workspace_sizes(1, 1024, 1024, 3, 150000, 50000)
    assert saved >= 50000 * 6 * 128 + 50000 * 32  # 128-B records (6 slots/face) + 32-B face data
    assert scratch > 0
    s2, _ = _lib.workspace_sizes(2, 1024, 1024, 3, 150000, 50000)
    assert s2 >= 2 * saved - 512


@pytest.mark.parametrize("args,msg", [
    ((1, 128, 128, 9, 4, 2), "channels"),
    ((1, 128, 128, 0, 4, 2), "channels"),
    ((1, 0, 128, 3, 4, 2), "height, width"),
    ((1, 128, 9000, 3, 4, 2), "height, width"),
    ((-1, 128, 128, 3, 4, 2), "non-negative"),
    ((1, 128, 128, 3, 4, (1 << 26) + 1), "too large"),
])
def test_invalid_arguments_raise_before_any_gpu_call(args, msg):
    with pytest.raises(ValueError, match=msg):
        _lib.workspace_sizes(*args)
    lib = _lib.load()
    B, H, W, C, V, F = args
    rc = lib.dirt_rasterise_fwd(None, None, None, None, None, B, H, W, C, V, F, 0, None, None, None, 0, None, 0, 0, 0, None, None, None)
    assert rc == _lib.DIRT_EINVAL
    assert msg in lib.dirt_last_error().decode()


def test_null_pointers_and_bad_shader_rejected():
    lib = _lib.load()
    rc = lib.dirt_rasterise_fwd(None, None, None, None, None, 1, 16, 16, 3, 3, 1, 0, None, None, None, 0, None, 0, 0, 0, None, None, None)
    assert rc == _lib.DIRT_EINVAL and "null" in lib.dirt_last_error().decode()
    rc = lib.dirt_rasterise_fwd(None, None, None, None, None, 1, 16, 16, 3, 3, 1, 77, None, None, None, 0, None, 0, 0, 0, None, None, None)
    assert rc == _lib.DIRT_EINVAL and "shader" in lib.dirt_last_error().decode()
    rc = lib.dirt_rasterise_bwd(None, None, None, None, None, None, None, 1, 16, 16, 3, 3, 1, None, None, None, 0, None)
    assert rc == _lib.DIRT_EINVAL


def test_zero_batch_is_a_no_op():
    lib = _lib.load()
    assert lib.dirt_rasterise_fwd(None, None, None, None, None, 0, 16, 16, 3, 3, 1, 0, None, None, None, 0, None, 0, 0,
                                  0, None, None, None) == _lib.DIRT_OK


def test_scratch_clear_validates_without_a_gpu():
    lib = _lib.load()
    # B == 0 is a no-op, a too-small scratch is rejected before any HIP call
    assert lib.dirt_scratch_clear(0, 16, 16, 1, 0, None, 0, None) == _lib.DIRT_OK
    assert lib.dirt_scratch_clear(1, 16, 16, 1, 0, None, 0, None) == _lib.DIRT_EINVAL
    assert "scratch" in lib.dirt_last_error().decode()


def test_cpp_autograd_extension_builds_and_binds():
    """The public op's C++ autograd function (dirt_amd/_dirt_torch) is built in-tree and binds the C ABI
    of the library _lib loads (init dlopens it: no GPU needed)."""
    from dirt_amd import rasterise_ops
    ext = rasterise_ops._torch_ext()
    assert ext is not None
    rasterise_ops.workspace_cache_clear()
    assert ext.scratch_cache_size() == 0


def test_recompute_backward_validates_without_a_gpu():
    """dirt_rasterise_bwd_recompute (the single-output op's gradient, csrc/rasterise_grad_common.h:5-24 shape):
    its workspace size is the forward's saved + scratch + a g-buffer, and bad arguments are refused before any
    HIP call."""
    lib = _lib.load()
    n = _lib.recompute_workspace_size(1, 1024, 1024, 3, 150000, 50000)
    saved, scratch = _lib.workspace_sizes(1, 1024, 1024, 3, 150000, 50000)
    assert n >= saved + scratch + 4 * 1024 * 1024
    with pytest.raises(ValueError, match="channels"):
        _lib.recompute_workspace_size(1, 16, 16, 9, 3, 1)
    args = [None] * 6 + [1, 16, 16, 3, 3, 1] + [None] * 4 + [0, 0, None]
    assert lib.dirt_rasterise_bwd_recompute(*args) == _lib.DIRT_EINVAL
    assert "null" in lib.dirt_last_error().decode()
    args = [None] * 6 + [0, 16, 16, 3, 3, 1] + [None] * 4 + [0, 0, None]
    assert lib.dirt_rasterise_bwd_recompute(*args) == _lib.DIRT_OK  # B == 0: nothing to do


def test_lighting_entry_points_reject_null_pointers_without_a_gpu():
    """The fused lighting entry points validate sizes and pointers before touching the device (CPU-safe)."""
    lib = _lib.load()
    assert lib.dirt_diffuse_directional_fwd(None, None, 5, None, None, 1, None, None) == _lib.DIRT_EINVAL
    assert lib.dirt_diffuse_directional_fwd(None, None, -1, None, None, 1, None, None) == _lib.DIRT_EINVAL
    # (nothing requested: no work and no error; a requested gradient with null inputs: EINVAL before any launch)
    assert lib.dirt_specular_directional_bwd(None, None, None, 4, None, None, None, 6.0, 1, None, None, None, None,
                                             None) == _lib.DIRT_OK
    assert lib.dirt_specular_directional_bwd(None, None, None, 4, None, None, None, 6.0, 1, None, 16, None, None,
                                             None) == _lib.DIRT_EINVAL
    assert lib.dirt_vertex_normals_fwd(None, 2, None, 0, 1, 3, 1, None, None, None) == _lib.DIRT_EINVAL  # stride < 3
    assert lib.dirt_vertex_normals_fwd(None, 3, None, 0, 1, 3, 1, None, None, None) == _lib.DIRT_EINVAL  # null pointers
    assert lib.dirt_diffuse_directional_fwd(None, None, 0, None, None, 1, None, None) == _lib.DIRT_OK  # empty
