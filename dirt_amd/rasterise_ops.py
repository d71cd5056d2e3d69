"""PyTorch mirror of the reference's op surface, dirt/rasterise_ops.py.

Same function names, argument order, defaults and shape inference as the reference
(dirt/rasterise_ops.py:10-203); TensorFlow graph ops become eager PyTorch-ROCm calls into
libdirt_mi355x.so, and the op gets the gradient the reference never registered:
`rasterise` / `rasterise_batch` are differentiable w.r.t. background, vertices and vertex_colors.

Differences from the reference, all deliberate:
  * `camera_pos` is optional (default None): the fork made it a mandatory positional argument of
    `rasterise` (rasterise_ops.py:10) but forgot it in `rasterise_batch` (:84-88), so every
    upstream-style caller raised; here both call forms work, positional ones included: an integer in the
    camera_pos slot is upstream DIRT's `height` (upstream signature `(background, vertices,
    vertex_colors, faces, height=None, width=None, channels=None, name=None)`), so the remaining
    positional arguments shift by one (`_upstream_positional`).
  * channels may be 1..8 (the reference CHECK-aborts unless 1 or 3, csrc/hwc.h:27), so the 7-channel
    deferred G-buffer (BASELINE config 4) is one call instead of three.
  * errors are exceptions, never process aborts (csrc/rasterise_egl.cpp:85-503 LOG(FATAL)).
There is no CPU path: the op requires a HIP device and raises if the native library is missing.
"""
import numpy as np
import torch

from . import _lib

__all__ = [
    "rasterise", "rasterise_batch", "rasterise_grad",
    "oceanic_no_cloud", "oceanic_simple_proxy", "oceanic_still_cloud", "oceanic_opt_flow", "hill",
]


def _device_of(*xs):
    for x in xs:
        if isinstance(x, torch.Tensor) and x.device.type == "cuda":
            return x.device
    if not torch.cuda.is_available():
        raise RuntimeError("dirt_amd.rasterise requires a ROCm/HIP GPU: there is no CPU implementation")
    return torch.device("cuda", torch.cuda.current_device())


def _as_tensor(x, dtype, device):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device)


class _RasteriseFunction(torch.autograd.Function):
    """Rasterise op (csrc/rasterise_egl.cpp:33-53) with its registered gradient."""

    @staticmethod
    def forward(ctx, background, vertices, vertex_colors, faces, camera_pos, height, width, channels, shader_id,
                bin_capacity):
        B, V, F = vertices.shape[0], vertices.shape[1], faces.shape[1]
        H, W, C = height, width, channels
        dev = vertices.device
        lib = _lib.load()
        saved_bytes, scratch_bytes = _lib.workspace_sizes(B, H, W, C, V, F, bin_capacity)
        pixels = torch.empty((B, H, W, C), dtype=torch.float32, device=dev)
        gbuffer = torch.empty((B, H, W), dtype=torch.int32, device=dev)
        saved = torch.empty((max(saved_bytes, 1),), dtype=torch.uint8, device=dev)
        scratch = torch.empty((max(scratch_bytes, 1),), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            cam = camera_pos.data_ptr() if camera_pos is not None else None
            _lib.check(lib.dirt_rasterise_fwd(
                background.data_ptr(), vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(), cam,
                B, H, W, C, V, F, shader_id, pixels.data_ptr(), gbuffer.data_ptr(),
                saved.data_ptr(), saved_bytes, scratch.data_ptr(), scratch_bytes, bin_capacity, 0, None, None,
                stream))
        ctx.save_for_backward(vertices, vertex_colors, faces, pixels, gbuffer, saved)
        ctx.dims = (B, H, W, C, V, F)
        ctx.shader_id = shader_id
        ctx.mark_non_differentiable(gbuffer)
        return pixels, gbuffer

    @staticmethod
    def backward(ctx, grad_pixels, _grad_gbuffer):
        if ctx.shader_id != _lib.SHADER_GOURAUD:
            raise RuntimeError("only the Gouraud fragment program has a gradient (the reference registers none)")
        vertices, vertex_colors, faces, pixels, gbuffer, saved = ctx.saved_tensors
        B, H, W, C, V, F = ctx.dims
        dev = vertices.device
        grad_pixels = grad_pixels.to(dtype=torch.float32).contiguous()
        grad_vertices = torch.empty((B, V, 4), dtype=torch.float32, device=dev)
        grad_colors = torch.empty((B, V, C), dtype=torch.float32, device=dev)
        grad_background = torch.empty((B, H, W, C), dtype=torch.float32, device=dev)
        lib = _lib.load()
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(lib.dirt_rasterise_bwd(
                vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(), pixels.data_ptr(),
                grad_pixels.data_ptr(), gbuffer.data_ptr(), saved.data_ptr(),
                B, H, W, C, V, F, grad_vertices.data_ptr(), grad_colors.data_ptr(), grad_background.data_ptr(),
                0, stream))
        return grad_background, grad_vertices, grad_colors, None, None, None, None, None, None, None


def _check_shapes(background, vertices, vertex_colors, faces, H, W, C):
    # messages follow csrc/rasterise_egl.cpp:310-336
    if background.dim() != 4 or tuple(background.shape[1:]) != (H, W, C):
        raise ValueError("Rasterise expects background_tensor to be 4D, and bgcolor.shape == [None, height, width, channels]")
    if vertices.dim() != 3 or vertices.shape[2] != 4:
        raise ValueError("Rasterise expects vertices to be 3D, and vertices.shape[2] == 4")
    if vertex_colors.dim() != 3 or vertex_colors.shape[1] != vertices.shape[1] or vertex_colors.shape[2] != C:
        raise ValueError("Rasterise expects vertex_colors to be 3D, and vertex_colors.shape == [None, vertices.shape[1], channels]")
    if faces.dim() != 3 or faces.shape[2] != 3:
        raise ValueError("Rasterise expects faces to be 3D, and faces.shape[2] == 3")
    B = vertices.shape[0]
    if background.shape[0] != B or vertex_colors.shape[0] != B or faces.shape[0] != B:
        raise ValueError("Rasterise expects all arguments to have same leading (batch) dimension")
    if not (C >= 1 and C <= _lib.MAX_CHANNELS):
        raise ValueError("Rasterise expects 1 <= channels <= %d" % _lib.MAX_CHANNELS)


# floats of camera_pos each program reads (the op's cudaMemcpy of camera_pos to the host)
_CAMERA_FLOATS = {
    _lib.SHADER_OCEANIC_STILL_CLOUD: (9, "oceanic_still_cloud needs 9 camera_pos floats: cloud_t is [8] "
                                         "(csrc/oceanic_still_cloud.cpp:323,407)"),
    _lib.SHADER_OCEANIC_OPT_FLOW: (16, "oceanic_opt_flow needs 16 camera_pos floats: dt is [9], the camera velocity "
                                       "[10..15] (csrc/oceanic_opt_flow.cpp:323,399-414)"),
    _lib.SHADER_HILL: (12, "hill needs 12 camera_pos floats: the camera origin is [9..11] (csrc/hill.cpp:323,395-407)"),
}


def _upstream_positional(camera_pos, height, width, channels, name):
    """Upstream DIRT has no camera_pos: `rasterise(bg, v, c, f, H, W, C)` binds H to our camera_pos slot.
    An integer there (a camera position is a float tensor / sequence, never a Python int) is that height;
    shift height / width / channels / name back into place."""
    if isinstance(camera_pos, (int, np.integer)) and not isinstance(camera_pos, bool):
        return None, int(camera_pos), height, width, channels
    return camera_pos, height, width, channels, name


def _camera(camera_pos, shader_id, dev):
    if camera_pos is None:
        if shader_id != _lib.SHADER_GOURAUD:
            raise ValueError("procedural fragment programs need camera_pos (8 floats)")
        return None
    camera_pos = _as_tensor(camera_pos, torch.float32, dev).contiguous().reshape(-1)
    if camera_pos.numel() < 8:
        raise ValueError("camera_pos must hold at least 8 floats (csrc/rasterise_egl.cpp:323)")
    need, why = _CAMERA_FLOATS.get(shader_id, (8, ""))
    if camera_pos.numel() < need:
        raise ValueError(why)
    return camera_pos


def _rasterise_batched(background, vertices, vertex_colors, faces, camera_pos, height, width, channels, shader_id,
                       bin_capacity=0, return_gbuffer=False):
    dev = _device_of(background, vertices, vertex_colors, faces, camera_pos)
    background = _as_tensor(background, torch.float32, dev).contiguous()
    vertices = _as_tensor(vertices, torch.float32, dev).contiguous()
    vertex_colors = _as_tensor(vertex_colors, torch.float32, dev).contiguous()
    faces = _as_tensor(faces, torch.int32, dev).contiguous()
    camera_pos = _camera(camera_pos, shader_id, dev)
    _check_shapes(background, vertices, vertex_colors, faces, height, width, channels)
    pixels, gbuffer = _RasteriseFunction.apply(background, vertices, vertex_colors, faces, camera_pos,
                                               int(height), int(width), int(channels), shader_id, int(bin_capacity))
    return (pixels, gbuffer) if return_gbuffer else pixels


_SHADERS = {None: _lib.SHADER_GOURAUD, "gouraud": _lib.SHADER_GOURAUD,
            "oceanic_horizon": _lib.SHADER_OCEANIC_HORIZON, "oceanic": _lib.SHADER_OCEANIC,
            "oceanic_still_cloud": _lib.SHADER_OCEANIC_STILL_CLOUD, "oceanic_no_cloud": _lib.SHADER_OCEANIC_NO_CLOUD,
            "oceanic_simple_proxy": _lib.SHADER_OCEANIC_SIMPLE_PROXY, "oceanic_opt_flow": _lib.SHADER_OCEANIC_OPT_FLOW}


def _shader_id(shader):
    if isinstance(shader, int) and shader in _SHADERS.values():
        return shader
    if shader not in _SHADERS:
        raise ValueError("unknown fragment program %r (expected one of %s)"
                         % (shader, sorted(k for k in _SHADERS if k is not None)))
    return _SHADERS[shader]


def rasterise(background, vertices, vertex_colors, faces, camera_pos=None, height=None, width=None, channels=None,
              name=None, shader=None):
    """Rasterises the given `vertices` and `faces` over `background` (reference dirt/rasterise_ops.py:10-54).

    Args:
        background: float32 [height, width, channels] image to render over (top row first)
        vertices: float32 [vertex count, 4] OpenGL clip-space positions
        vertex_colors: float32 [vertex count, channels]; interpolated perspective-correctly (Gouraud)
        faces: int32 [face count, 3] indices into `vertices`
        camera_pos: float32 [>=8] (cam x, y, z, ang1, ang2, ang3, time, light_z,
            csrc/rasterise_egl.cpp:399-406; 9 floats for oceanic_still_cloud, 16 for oceanic_opt_flow);
            read only by the procedural programs
        height, width, channels: may be None, then inferred from `background`'s shape
        name: ignored (TensorFlow name scope in the reference)
        shader: fragment program. None / 'gouraud': Gouraud colours (upstream DIRT, the default);
            'oceanic_horizon': the program the fork's `Rasterise` op binds (csrc/shaders.cpp:1668-1919,
            rasterise_egl.cpp:385): covered pixels get (sky mask, sun / reflection, 0), jittered by the
            background's first two channels; needs camera_pos and has no gradient (the reference
            registers none).  'oceanic', 'oceanic_still_cloud', 'oceanic_no_cloud',
            'oceanic_simple_proxy', 'oceanic_opt_flow': the programs of the reference's other procedural
            ops (same as calling those ops); forward only

    Returns:
        float32 [height, width, channels] pixels, differentiable w.r.t. background, vertices, vertex_colors.
    """
    camera_pos, height, width, channels, name = _upstream_positional(camera_pos, height, width, channels, name)
    del name
    bshape = tuple(background.shape) if hasattr(background, "shape") else np.shape(background)
    if height is None:
        height = int(bshape[0])
    if width is None:
        width = int(bshape[1])
    if channels is None:
        channels = int(bshape[2])
    dev = _device_of(background, vertices, vertex_colors, faces, camera_pos)
    background = _as_tensor(background, torch.float32, dev)
    vertices = _as_tensor(vertices, torch.float32, dev)
    vertex_colors = _as_tensor(vertex_colors, torch.float32, dev)
    faces = _as_tensor(faces, torch.int32, dev)
    return _rasterise_batched(background[None], vertices[None], vertex_colors[None], faces[None], camera_pos,
                              height, width, channels, _shader_id(shader))[0]


def rasterise_batch(background, vertices, vertex_colors, faces, camera_pos=None, height=None, width=None,
                    channels=None, name=None, shader=None):
    """Rasterises a batch of meshes with equal vertex and face counts (reference dirt/rasterise_ops.py:57-88).

    Conceptually `torch.stack([rasterise(bg_i, v_i, c_i, f_i) for ...])`; every argument carries a leading
    batch dimension and faces index the vertices of their own frame.
    """
    camera_pos, height, width, channels, name = _upstream_positional(camera_pos, height, width, channels, name)
    del name
    bshape = tuple(background.shape) if hasattr(background, "shape") else np.shape(background)
    if height is None:
        height = int(bshape[1])
    if width is None:
        width = int(bshape[2])
    if channels is None:
        channels = int(bshape[3])
    return _rasterise_batched(background, vertices, vertex_colors, faces, camera_pos, height, width, channels,
                              _shader_id(shader))


def _procedural_op(opname, shader, ref):
    def op(background, vertices, vertex_colors, faces, camera_pos, height=None, width=None, channels=None,
           name=None):
        return rasterise(background, vertices, vertex_colors, faces, camera_pos, height, width, channels, name,
                         shader=shader)
    op.__name__ = opname
    op.__doc__ = ("Reference dirt/rasterise_ops.py `%s` (%s): `rasterise` with the `%s` fragment program "
                  "(DESIGN.md 3b); forward only, like the reference." % (opname, ref, shader))
    return op


def hill(background, vertices, vertex_colors, faces, camera_pos, height=None, width=None, channels=None, name=None):
    """Reference dirt/rasterise_ops.py:186-203 `hill` (op csrc/hill.cpp, program csrc/shaders.cpp:123-554).

    `background` is the terrain lookup [height, width, 1|3|4] (x = terrain height, yzw = normal): the op
    checks only its height and width (hill.cpp:310).  `vertex_colors` is shape-checked and not read;
    camera_pos holds 12 floats, of which [9..11] (the camera origin) are read.  There is no depth test:
    where faces overlap the last one in draw order wins (hill.cpp:194); uncovered pixels are 0.
    Forward only, like the reference.  Returns float32 [height, width, channels].
    """
    del name
    bshape = tuple(background.shape) if hasattr(background, "shape") else np.shape(background)
    if height is None:
        height = int(bshape[0])
    if width is None:
        width = int(bshape[1])
    if channels is None:
        channels = int(bshape[2])
    dev = _device_of(background, vertices, vertex_colors, faces, camera_pos)
    terrain = _as_tensor(background, torch.float32, dev).contiguous()[None]
    vertices = _as_tensor(vertices, torch.float32, dev).contiguous()[None]
    vertex_colors = _as_tensor(vertex_colors, torch.float32, dev).contiguous()[None]
    faces = _as_tensor(faces, torch.int32, dev).contiguous()[None]
    camera_pos = _camera(camera_pos, _lib.SHADER_HILL, dev)
    H, W, C = int(height), int(width), int(channels)
    if terrain.dim() != 4 or tuple(terrain.shape[1:3]) != (H, W):
        raise ValueError("Rasterise expects background_tensor to be 4D, and bgcolor.shape == [None, height, width, channels]")
    if terrain.shape[3] not in (1, 3, 4):
        raise ValueError("hill: the terrain lookup (background) must have 1, 3 or 4 channels (csrc/rasterise_egl.cu:33-47)")
    _check_shapes(terrain.new_empty((terrain.shape[0], H, W, C)), vertices, vertex_colors, faces, H, W, C)
    B, V, F = vertices.shape[0], vertices.shape[1], faces.shape[1]
    lib = _lib.load()
    saved_bytes, scratch_bytes = _lib.workspace_sizes(B, H, W, C, V, F, 0)
    pixels = torch.empty((B, H, W, C), dtype=torch.float32, device=dev)
    gbuffer = torch.empty((B, H, W), dtype=torch.int32, device=dev)
    saved = torch.empty((max(saved_bytes, 1),), dtype=torch.uint8, device=dev)
    scratch = torch.empty((max(scratch_bytes, 1),), dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(lib.dirt_hill_fwd(terrain.data_ptr(), int(terrain.shape[3]), vertices.data_ptr(), faces.data_ptr(),
                                     camera_pos.data_ptr(), B, H, W, C, V, F, pixels.data_ptr(), gbuffer.data_ptr(),
                                     saved.data_ptr(), saved_bytes, scratch.data_ptr(), scratch_bytes, 0, stream))
    return pixels[0]


# RasteriseGrad binds the `oceanic` program (csrc/rasterise_grad_egl.cpp:399, SURVEY F4: not a gradient)
rasterise_grad = _procedural_op("rasterise_grad", "oceanic", "rasterise_ops.py:91-108")
oceanic_no_cloud = _procedural_op("oceanic_no_cloud", "oceanic_no_cloud", "rasterise_ops.py:110-127")
oceanic_simple_proxy = _procedural_op("oceanic_simple_proxy", "oceanic_simple_proxy", "rasterise_ops.py:129-146")
oceanic_still_cloud = _procedural_op("oceanic_still_cloud", "oceanic_still_cloud", "rasterise_ops.py:148-165")
oceanic_opt_flow = _procedural_op("oceanic_opt_flow", "oceanic_opt_flow", "rasterise_ops.py:167-184")
