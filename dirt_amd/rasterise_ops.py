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
import collections
import os
import sys
import threading

import numpy as np
import torch

from . import _lib

__all__ = [
    "rasterise", "rasterise_batch", "rasterise_grad", "rasterise_gbuffer", "rasterise_batch_gbuffer", "GBuffer",
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


class _on_device:
    """torch.cuda.device(dev), skipped when dev is already the current device (host overhead per call)."""

    def __init__(self, dev):
        self.ctx = None if dev.index is None or dev.index == torch.cuda.current_device() else torch.cuda.device(dev)

    def __enter__(self):
        if self.ctx is not None:
            self.ctx.__enter__()

    def __exit__(self, *a):
        if self.ctx is not None:
            self.ctx.__exit__(*a)


_DEBUG_SCRATCH = os.environ.get("DIRT_DEBUG_SCRATCH") is not None


class _CaptureKeyedCache:
    """Device buffers per (device, stream, layout), with graph captures kept apart.

    Eager entries: an LRU of `keep` layouts.  An entry made while its stream captures a HIP graph comes from that
    graph's memory pool and is initialised by nodes of that graph, so it is valid only for that graph's replays:
    such entries are keyed by the capture id as well (`dirt_stream_capture_id`), no other capture or eager call
    ever sees one, and they are PINNED -- kept referenced until `clear(force=True)` -- because the graph goes on
    writing them at every replay.  Dropping the reference early would return the block to the pool, and a later
    capture sharing that pool (`torch.cuda.graph(..., pool=...)`, `make_graphed_callables`) could be handed the
    same memory: two graphs writing one buffer.  `make(nbytes, dev, stream)` creates a buffer."""

    def __init__(self, make, keep=4):
        self.keep = keep
        self._make = make
        self._lock = threading.Lock()
        self._d = collections.OrderedDict()
        self._caps = {}  # capture id -> {key: tensor}, pinned

    def get(self, dev, stream, layout, nbytes):
        cid = _lib.capture_id(stream) if torch.cuda.is_current_stream_capturing() else 0
        key = (dev, stream, layout)
        with self._lock:
            if cid:
                t = self._caps.get(cid, {}).get(key)
            else:
                t = self._d.get(key)
                if t is not None:
                    self._d.move_to_end(key)
            if t is not None:
                if _DEBUG_SCRATCH:
                    print("[dirt scratch py] hit stream %x capture %d ptr %x" % (stream, cid, t.data_ptr()), file=sys.stderr)
                return t
        t = self._make(nbytes, dev, stream, layout)
        if _DEBUG_SCRATCH:
            print("[dirt scratch py] new stream %x capture %d ptr %x" % (stream, cid, t.data_ptr()), file=sys.stderr)
        with self._lock:
            if cid:
                self._caps.setdefault(cid, {})[key] = t
            else:
                self._d[key] = t
                while len(self._d) > self.keep:
                    self._d.popitem(last=False)
        return t

    def discard(self, dev, stream, layout):
        """Drop an entry whose call failed after its first launch (its state may no longer be clean).  A capture's
        entry is dropped too: the failed capture is invalid anyway."""
        key = (dev, stream, layout)
        with self._lock:
            self._d.pop(key, None)
            for m in self._caps.values():
                m.pop(key, None)

    def clear(self, force=False):
        """Drop the eager entries; `force` also unpins the graph captures' entries (call it once the graphs that
        were captured through the op are destroyed)."""
        with self._lock:
            self._d.clear()
            if force:
                self._caps = {}

    def __len__(self):
        with self._lock:
            return len(self._d) + sum(len(m) for m in self._caps.values())


def _make_scratch(nbytes, dev, stream, layout):
    # only the bin counters need zeroing (dirt_scratch_clear: a kernel over the counter lines); the slabs are
    # written before they are read.  Under capture the clear is a node of the graph.
    t = torch.empty((max(nbytes, 1),), dtype=torch.uint8, device=dev)
    B, H, W, F, cap = layout
    _lib.check(_lib.load().dirt_scratch_clear(B, H, W, F, cap, t.data_ptr(), nbytes, stream))
    return t


class _Workspace(_CaptureKeyedCache):
    """Per-(device, stream, layout) cache of the forward-only scratch (tile bins, bin counters).

    A scratch zero-filled once stays clean across forwards of the same layout (the bin counters alternate
    between two sets, include/dirt_mi355x.h DIRT_FWD_SCRATCH_CLEAN), so a cached one saves every call the
    counter clear (128 MiB for B = 64 at 8192^2 with one 256-B line per counter) and the allocation.
    Keyed by the stream too: two streams never share a scratch.  Graph captures get scratch of their own,
    pinned for the graphs' lifetime (_CaptureKeyedCache).  An entry whose forward failed after its first launch
    is dropped (`discard`): its alternating bin-count sets may no longer be clean."""

    def __init__(self, keep=4):
        super().__init__(_make_scratch, keep)

    def scratch(self, dev, stream, layout, nbytes):
        return self.get(dev, stream, layout, nbytes)


_workspace = _Workspace()


class _GeomCache:
    """Renders that share their geometry (samples/deferred.py:63-83 renders one mesh three times):
    the Python twin of _dirt_torch's GeomCache.  The last plain Gouraud forward per (device, stream, capture id)
    remembers its geometry -- vertices' and faces' storage, offset, shape, strides and version counters, as detached
    aliases -- with its g-buffer and saved records; a forward on the same, unmodified tensors (or views of the same
    elements) at the same frame size takes dirt_rasterise_fwd_resolve (the resolve alone, pixels bit-identical).
    Writes that bypass the version counter (`.data`, raw pointers) are not seen, like autograd's own saved-tensor
    checks; DIRT_SHARE_GEOMETRY=0 turns it off."""

    enabled = os.environ.get("DIRT_SHARE_GEOMETRY", "1") not in ("", "0")

    def __init__(self):
        self._lock = threading.Lock()
        self._d = collections.OrderedDict()

    @staticmethod
    def _ident(t):
        # (strides of size-1 dimensions do not matter)
        return (t.untyped_storage()._cdata, t.storage_offset(), tuple(t.shape),
                tuple(s if n > 1 else 0 for s, n in zip(t.stride(), t.shape)), t.dtype, t._version)

    def find(self, key, vertices, faces, H, W):
        with self._lock:
            e = self._d.get(key)
        if e is None or e[0] != (self._ident(vertices), self._ident(faces), H, W):
            return None
        return e[2], e[3]

    def store(self, key, vertices, faces, H, W, gbuffer, saved):
        with self._lock:
            # (the detached aliases keep the storages alive, so their addresses identify them)
            self._d[key] = ((self._ident(vertices), self._ident(faces), H, W), (vertices.detach(), faces.detach()),
                            gbuffer, saved)
            self._d.move_to_end(key)
            while len(self._d) > 8:
                self._d.popitem(last=False)

    def clear(self):
        with self._lock:
            self._d.clear()


_geom = _GeomCache()


def set_geometry_sharing(enabled):
    """Turn the shared-geometry cache (renders of one unmodified geometry after the first run the resolve alone) on or
    off for both implementations of the op; returns the previous setting.  Off: every forward is a full one, as in a
    training loop whose optimizer changes the vertices each step (tools and benchmarks that repeat one geometry use
    this to time full steps).  The environment variable DIRT_SHARE_GEOMETRY=0 sets the initial state."""
    prev = _GeomCache.enabled
    _GeomCache.enabled = bool(enabled)
    if not enabled:
        _geom.clear()
    ext = _torch_ext()
    if ext is not None:
        ext.set_geometry_sharing(bool(enabled))
    return prev


def _check_faces_now(faces, B, V, F, stream):
    """Opt-in range check of the face indices (a kernel and a host sync): raises IndexError like the
    SURVEY 8b return code 2.  The reference reads out of bounds (csrc/rasterise_egl.cpp:309-336 checks
    shapes only); the forward itself culls such faces."""
    flag = torch.empty((256,), dtype=torch.uint8, device=faces.device)
    _lib.check(_lib.load().dirt_check_faces(faces.data_ptr(), B, V, F, flag.data_ptr(), 256, stream))


class _RasteriseFunction(torch.autograd.Function):
    """Rasterise op (csrc/rasterise_egl.cpp:33-53) with its registered gradient.

    Outputs: pixels, the int32 record g-buffer and, when `want_gbuf`, depth / barycentrics / face ids
    (non-differentiable).  When a gradient will be needed, the forward zero-fills the vertex and colour
    gradient buffers in passing (filler workgroups of its setup launch) and the backward adds into them
    (DIRT_BWD_ACCUMULATE), so a fwd+bwd costs no separate clearing launch."""

    @staticmethod
    def forward(ctx, background, vertices, vertex_colors, faces, camera_pos, height, width, channels, shader_id,
                bin_capacity, want_gbuf, check_faces):
        B, V, F = vertices.shape[0], vertices.shape[1], faces.shape[1]
        H, W, C = height, width, channels
        dev = vertices.device
        lib = _lib.load()
        saved_bytes, scratch_bytes = _lib.workspace_sizes(B, H, W, C, V, F, bin_capacity)
        pixels = torch.empty((B, H, W, C), dtype=torch.float32, device=dev)
        gbuffer = torch.empty((B, H, W), dtype=torch.int32, device=dev)
        need_grad = shader_id == _lib.SHADER_GOURAUD and any(ctx.needs_input_grad[:3]) and V > 0
        # the accumulators the backward fills (it computes only those; background-only: both)
        want_v, want_c = need_grad and ctx.needs_input_grad[1], need_grad and ctx.needs_input_grad[2]
        if need_grad and not (want_v or want_c):
            want_v = want_c = True
        gv = torch.empty((B, V, 4), dtype=torch.float32, device=dev) if want_v else None
        gc = torch.empty((B, V, C), dtype=torch.float32, device=dev) if want_c else None
        with _on_device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            if check_faces:
                _check_faces_now(faces, B, V, F, stream)
            shareable = (_GeomCache.enabled and shader_id == _lib.SHADER_GOURAUD and not want_gbuf and F > 0 and
                         not (_FWD_FLAGS & (_lib.FWD_DEEP_CULL | _lib.FWD_DEEP_CULL_OFF)))
            gkey = None
            if shareable:
                gkey = (dev, stream, _lib.capture_id(stream) if torch.cuda.is_current_stream_capturing() else 0)
                hit = _geom.find(gkey, vertices, faces, H, W)
                if hit is not None:
                    # a render of the geometry the last forward on this stream rendered: the resolve alone
                    gb_in, saved = hit
                    _lib.check(lib.dirt_rasterise_fwd_resolve(
                        background.data_ptr(), vertex_colors.data_ptr(), B, H, W, C, V, F, gb_in.data_ptr(),
                        saved.data_ptr(), saved.numel(), pixels.data_ptr(), gbuffer.data_ptr(),
                        gv.data_ptr() if want_v else None, gc.data_ptr() if want_c else None, stream))
                    return _RasteriseFunction._finish(ctx, vertices, vertex_colors, faces, pixels, gbuffer, saved, (),
                                                      (B, H, W, C, V, F), shader_id, need_grad, gv, gc, want_v, want_c)
            saved = torch.empty((max(saved_bytes, 1),), dtype=torch.uint8, device=dev)
            layout = (B, H, W, F, bin_capacity)
            scratch = _workspace.scratch(dev, stream, layout, scratch_bytes)
            cam = camera_pos.data_ptr() if camera_pos is not None else None
            zg = (gv.data_ptr() if want_v else None, gc.data_ptr() if want_c else None)
            try:
                extra = _RasteriseFunction._launch(lib, want_gbuf, background, vertices, vertex_colors, faces, cam,
                                                   B, H, W, C, V, F, shader_id, pixels, gbuffer, saved, saved_bytes,
                                                   scratch, scratch_bytes, bin_capacity, zg, stream)
            except Exception:
                _workspace.discard(dev, stream, layout)  # its count sets may be dirty now
                raise
            if shareable:
                _geom.store(gkey, vertices, faces, H, W, gbuffer, saved)
        return _RasteriseFunction._finish(ctx, vertices, vertex_colors, faces, pixels, gbuffer, saved, extra,
                                          (B, H, W, C, V, F), shader_id, need_grad, gv, gc, want_v, want_c)

    @staticmethod
    def _finish(ctx, vertices, vertex_colors, faces, pixels, gbuffer, saved, extra, dims, shader_id, need_grad, gv, gc,
                want_v, want_c):
        ctx.save_for_backward(vertices, vertex_colors, faces, pixels, gbuffer, saved)
        ctx.dims = dims
        ctx.shader_id = shader_id
        ctx.prezeroed = (gv, gc) if need_grad else None
        ctx.want = (want_v, want_c) if need_grad else (True, True)
        ctx.mark_non_differentiable(gbuffer, *extra)
        # only the pixels' gradient is read: no zero gradients filled for the non-differentiable outputs
        ctx.set_materialize_grads(False)
        return (pixels, gbuffer) + extra

    @staticmethod
    def _launch(lib, want_gbuf, background, vertices, vertex_colors, faces, cam, B, H, W, C, V, F, shader_id, pixels,
                gbuffer, saved, saved_bytes, scratch, scratch_bytes, bin_capacity, zg, stream):
        """The forward's C-ABI call; returns the extra G-buffer outputs (empty unless want_gbuf)."""
        if not want_gbuf:
            _lib.check(lib.dirt_rasterise_fwd(
                background.data_ptr(), vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(), cam,
                B, H, W, C, V, F, shader_id, pixels.data_ptr(), gbuffer.data_ptr(),
                saved.data_ptr(), saved_bytes, scratch.data_ptr(), scratch_bytes, bin_capacity,
                _FWD_FLAGS, zg[0], zg[1], stream))
            return ()
        dev = vertices.device
        depth = torch.empty((B, H, W), dtype=torch.float32, device=dev)
        bary = torch.empty((B, H, W, 3), dtype=torch.float32, device=dev)
        face_ids = torch.empty((B, H, W), dtype=torch.int32, device=dev)
        _lib.check(lib.dirt_rasterise_fwd_gbuffer(
            background.data_ptr(), vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(),
            B, H, W, C, V, F, pixels.data_ptr(), gbuffer.data_ptr(), saved.data_ptr(), saved_bytes,
            scratch.data_ptr(), scratch_bytes, bin_capacity, _FWD_FLAGS, zg[0], zg[1],
            depth.data_ptr(), bary.data_ptr(), face_ids.data_ptr(), stream))
        return (depth, bary, face_ids)

    @staticmethod
    def backward(ctx, grad_pixels, _grad_gbuffer, *_grad_extra):
        if ctx.shader_id != _lib.SHADER_GOURAUD:
            raise RuntimeError("only the Gouraud fragment program has a gradient (the reference registers none)")
        vertices, vertex_colors, faces, pixels, gbuffer, saved = ctx.saved_tensors
        B, H, W, C, V, F = ctx.dims
        dev = vertices.device
        if grad_pixels is None:
            grad_pixels = torch.zeros((B, H, W, C), dtype=torch.float32, device=dev)
        grad_pixels = grad_pixels.to(dtype=torch.float32).contiguous()
        # the forward's zero-filled buffers serve one backward (autograd may keep the returned tensors as
        # .grad); a second backward of the same graph (retain_graph) starts from fresh ones
        flags = 0
        if ctx.prezeroed is not None:
            grad_vertices, grad_colors = ctx.prezeroed
            ctx.prezeroed = None
            flags = _lib.BWD_ACCUMULATE
        else:
            want_v, want_c = ctx.want
            grad_vertices = torch.empty((B, V, 4), dtype=torch.float32, device=dev) if want_v else None
            grad_colors = torch.empty((B, V, C), dtype=torch.float32, device=dev) if want_c else None
        # (a background that needs no gradient is not written at all)
        grad_background = (torch.empty((B, H, W, C), dtype=torch.float32, device=dev) if ctx.needs_input_grad[0]
                           else None)
        lib = _lib.load()
        with _on_device(dev):
            stream = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(lib.dirt_rasterise_bwd(
                vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(), pixels.data_ptr(),
                grad_pixels.data_ptr(), gbuffer.data_ptr(), saved.data_ptr(),
                B, H, W, C, V, F, grad_vertices.data_ptr() if grad_vertices is not None else None,
                grad_colors.data_ptr() if grad_colors is not None else None,
                grad_background.data_ptr() if grad_background is not None else None, flags, stream))
        return (grad_background, grad_vertices, grad_colors) + (None,) * 9


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
    An integer there (a camera position is a float tensor / sequence, never a Python int) is that height.

    Upstream slot j (height, width, channels, name) lands in our slot j when passed positionally and in
    our slot j+1 when passed by keyword.  The k positional values fill our first k slots and keyword
    values only upstream slots >= k, i.e. our slots >= k+1, so our slot k is the first empty one: that
    recovers k for fully positional, fully keyword and mixed calls such as
    `rasterise_batch(bg, v, c, f, 48, width=64, channels=3)` or `(bg, v, c, f, 48, 64, channels=3)`."""
    if isinstance(camera_pos, (int, np.integer)) and not isinstance(camera_pos, bool):
        ours = [int(camera_pos), height, width, channels, name]
        k = next((i for i, x in enumerate(ours) if x is None), len(ours))
        up = [ours[j] if j < k else ours[j + 1] for j in range(4)]
        return (None,) + tuple(up)
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


_EXT = None


def _torch_ext():
    """The C++ autograd function (dirt_amd/csrc/torch_op.cpp, module _dirt_torch) bound to the library
    _lib loaded, or None if it is not built or DIRT_TORCH_EXT=0 (then _RasteriseFunction, the same op in
    Python, runs: both call the same HIP kernels through the C ABI; there is no CPU path)."""
    global _EXT
    if _EXT is None:
        _EXT = False
        if os.environ.get("DIRT_TORCH_EXT", "1") != "0":
            try:
                from . import _dirt_torch
            except ImportError:
                _dirt_torch = None
            if _dirt_torch is not None:
                _lib.load()
                _dirt_torch.init(_lib.LIB_PATH)
                _EXT = _dirt_torch
    return _EXT or None


def workspace_cache_clear(force=False):
    """Drop the cached per-layout scratch buffers (both implementations) and the single-output op's workspaces.
    Scratch made inside a graph capture stays pinned (its graph writes it at every replay) unless `force`: call
    `workspace_cache_clear(force=True)` once the graphs captured through the op are destroyed."""
    _workspace.clear(force)
    _geom.clear()
    from . import op_library
    op_library._stash_workspaces.clear(force)
    ext = _torch_ext()
    if ext is not None:
        ext.scratch_cache_clear(bool(force))


def workspace_cache_size():
    ext = _torch_ext()
    return len(_workspace) + (ext.scratch_cache_size() if ext is not None else 0)


# DIRT_CHECK_FACES=1: every call range-checks its face indices (one kernel + a host sync; off by default)
_CHECK_FACES_DEFAULT = os.environ.get("DIRT_CHECK_FACES", "") not in ("", "0")
# Gouraud forwards take the occluder culling of long per-tile lists by the library's automatic rule (ABI 12,
# include/dirt_mi355x.h DIRT_FWD_DEEP_CULL); DIRT_DEEP_CULL=1 forces it, DIRT_DEEP_CULL=0 turns it off (identical
# results either way)
_DEEP_ENV = os.environ.get("DIRT_DEEP_CULL", "")
_FWD_FLAGS = _lib.FWD_SCRATCH_CLEAN | (_lib.FWD_DEEP_CULL if _DEEP_ENV not in ("", "0") else
                                       _lib.FWD_DEEP_CULL_OFF if _DEEP_ENV == "0" else 0)


def _rasterise_batched(background, vertices, vertex_colors, faces, camera_pos, height, width, channels, shader_id,
                       bin_capacity=0, return_gbuffer=False, want_gbuf=False, check_faces=None):
    if check_faces is None:
        check_faces = _CHECK_FACES_DEFAULT
    ext = _torch_ext()
    if (ext is not None and camera_pos is None and shader_id == _lib.SHADER_GOURAUD and type(background) is torch.Tensor
            and type(vertices) is torch.Tensor and type(vertex_colors) is torch.Tensor and type(faces) is torch.Tensor):
        # fast path: dtype / device / contiguity / shape handling in the C++ op (torch_op.cpp rasterise_checked)
        outs = ext.rasterise_checked(background, vertices, vertex_colors, faces, int(height), int(width),
                                     int(channels), int(bin_capacity), bool(want_gbuf), bool(check_faces), _FWD_FLAGS)
        if want_gbuf:
            return outs
        return (outs[0], outs[1]) if return_gbuffer else outs[0]
    dev = _device_of(background, vertices, vertex_colors, faces, camera_pos)
    background = _as_tensor(background, torch.float32, dev).contiguous()
    vertices = _as_tensor(vertices, torch.float32, dev).contiguous()
    vertex_colors = _as_tensor(vertex_colors, torch.float32, dev).contiguous()
    faces = _as_tensor(faces, torch.int32, dev).contiguous()
    camera_pos = _camera(camera_pos, shader_id, dev)
    _check_shapes(background, vertices, vertex_colors, faces, height, width, channels)
    args = (background, vertices, vertex_colors, faces, camera_pos, int(height), int(width), int(channels), shader_id,
            int(bin_capacity), bool(want_gbuf), bool(check_faces))
    outs = ext.rasterise(*args, _FWD_FLAGS) if ext is not None else _RasteriseFunction.apply(*args)
    if want_gbuf:
        return outs
    pixels, gbuffer = outs
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
              name=None, shader=None, check_faces=None):
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
        check_faces: True raises IndexError if a face index lies outside [0, vertex count) (one extra
            kernel and a host sync; default: the DIRT_CHECK_FACES environment variable, else off -- the
            reference does not check and reads out of bounds, this op culls such faces)

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
    # (squeeze, not [0]: the gradient of a select is a zero-filled batch plus a copy, a squeeze's is a view)
    return _rasterise_batched(background[None], vertices[None], vertex_colors[None], faces[None], camera_pos,
                              height, width, channels, _shader_id(shader), check_faces=check_faces).squeeze(0)


def rasterise_batch(background, vertices, vertex_colors, faces, camera_pos=None, height=None, width=None,
                    channels=None, name=None, shader=None, check_faces=None):
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
                              _shader_id(shader), check_faces=check_faces)


GBuffer = collections.namedtuple("GBuffer", ["pixels", "depth", "barycentrics", "face_ids"])


def rasterise_batch_gbuffer(background, vertices, vertex_colors, faces, height=None, width=None, channels=None,
                            name=None, check_faces=None):
    """`rasterise_batch` (Gouraud) that also returns the deferred-shading G-buffer of the same raster pass.

    Returns GBuffer(pixels [B,H,W,C] (differentiable, as rasterise_batch), depth [B,H,W] (the DEPTH24 value
    as float, 1.0 uncovered), barycentrics [B,H,W,3] (perspective-correct, of the visible face's vertices
    faces[b, face_ids]; 0 uncovered), face_ids [B,H,W] int32 (-1 uncovered)).  Upstream DIRT rendered
    these with separate G-buffer programs (csrc/shaders.cpp:2187-2221); here they come from the one
    resolve (include/dirt_mi355x.h dirt_rasterise_fwd_gbuffer)."""
    del name
    bshape = tuple(background.shape) if hasattr(background, "shape") else np.shape(background)
    height = int(bshape[1]) if height is None else height
    width = int(bshape[2]) if width is None else width
    channels = int(bshape[3]) if channels is None else channels
    px, _gb, depth, bary, face = _rasterise_batched(background, vertices, vertex_colors, faces, None, height, width,
                                                    channels, _lib.SHADER_GOURAUD, want_gbuf=True,
                                                    check_faces=check_faces)
    return GBuffer(px, depth, bary, face)


def rasterise_gbuffer(background, vertices, vertex_colors, faces, height=None, width=None, channels=None, name=None,
                      check_faces=None):
    """Single-frame `rasterise_batch_gbuffer` (shapes without the leading batch dimension)."""
    del name
    bshape = tuple(background.shape) if hasattr(background, "shape") else np.shape(background)
    height = int(bshape[0]) if height is None else height
    width = int(bshape[1]) if width is None else width
    channels = int(bshape[2]) if channels is None else channels
    dev = _device_of(background, vertices, vertex_colors, faces)
    g = rasterise_batch_gbuffer(_as_tensor(background, torch.float32, dev)[None],
                                _as_tensor(vertices, torch.float32, dev)[None],
                                _as_tensor(vertex_colors, torch.float32, dev)[None],
                                _as_tensor(faces, torch.int32, dev)[None], height, width, channels,
                                check_faces=check_faces)
    return GBuffer(*(t.squeeze(0) for t in g))


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
