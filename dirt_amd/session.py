"""Preallocated, graph-capturable rasterise forward/backward for fixed shapes.

`rasterise` / `rasterise_batch` allocate their outputs and workspace per call and go through autograd;
that is the drop-in surface.  A serving or training loop that renders the same shapes every step can
instead hold a `RasteriseSession`: buffers are allocated once and each call is a single ctypes call into
the C ABI, so a whole forward+backward step can be captured into a HIP graph (torch.cuda.CUDAGraph) and
replayed without host launch overhead.  Results are identical to the autograd path (same kernels).

The session also removes the per-step housekeeping launches: the scratch is zero-filled once and every
forward leaves it clean (DIRT_FWD_SCRATCH_CLEAN skips the forward's clearing memset), and the forward
zero-fills the gradient accumulators in passing (filler workgroups of its setup launch), so the backward adds into them
(DIRT_BWD_ACCUMULATE) without a clearing kernel of its own.  Hence: the gradients returned by
`backward` stay valid until the next `forward`, and each forward is followed by at most one backward.

Streams: the session's buffers are ordered by the stream each call runs on.  A call on a different stream
than the previous one first makes its stream wait for the previous one (an event, no host sync), so a
session may move between streams -- e.g. a warm-up on the default stream, then a HIP-graph capture on a
side stream -- without racing its own buffers.  (Inside a capture no cross-stream wait is inserted: the
capturing code orders the capture stream itself, as bench.py does with `stream.wait_stream`.)
"""
import torch

from . import _lib


class RasteriseSession:
    def __init__(self, B, H, W, C, V, F, device=None, bin_capacity=0, shader_id=_lib.SHADER_GOURAUD, deep_cull=None):
        """deep_cull: occluder culling for deep scenes of large overlapping triangles -- None: the library's automatic
        rule (the culling raster while one of the device's last 8 forwards was deep), True: always
        (DIRT_FWD_DEEP_CULL), False: never (DIRT_FWD_DEEP_CULL_OFF).  The results are identical in every case."""
        self.dims = (B, H, W, C, V, F)
        self.fwd_flags = _lib.FWD_SCRATCH_CLEAN | {None: 0, True: _lib.FWD_DEEP_CULL, False: _lib.FWD_DEEP_CULL_OFF}[
            None if deep_cull is None else bool(deep_cull)]
        self.shader_id = shader_id
        dev = torch.device(device) if device is not None else torch.device("cuda")
        if dev.type == "cuda" and dev.index is None:  # "cuda" means the current device: compare as cuda:N
            dev = torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.bin_capacity = int(bin_capacity)
        saved_bytes, scratch_bytes = _lib.workspace_sizes(B, H, W, C, V, F, self.bin_capacity)
        self.saved_bytes, self.scratch_bytes = saved_bytes, scratch_bytes
        dev = self.device
        self.pixels = torch.empty((B, H, W, C), dtype=torch.float32, device=dev)
        self.gbuffer = torch.empty((B, H, W), dtype=torch.int32, device=dev)
        self.saved = torch.empty((max(saved_bytes, 1),), dtype=torch.uint8, device=dev)
        self.scratch = torch.empty((max(scratch_bytes, 1),), dtype=torch.uint8, device=dev)
        self.grad_vertices = torch.empty((B, V, 4), dtype=torch.float32, device=dev)
        self.grad_vertex_colors = torch.empty((B, V, C), dtype=torch.float32, device=dev)
        self.grad_background = torch.empty((B, H, W, C), dtype=torch.float32, device=dev)
        self._lib = _lib.load()
        self._inputs = None
        self._last_stream = None
        # clean once (the bin counters; the slabs are written before they are read); every forward leaves
        # it clean
        _lib.check(self._lib.dirt_scratch_clear(B, H, W, F, self.bin_capacity, self.scratch.data_ptr(),
                                                self.scratch_bytes, torch.cuda.current_stream(dev).cuda_stream))
        self._last_stream = torch.cuda.current_stream(dev)

    def clip_stats(self, reset=True):
        """R5 deviation counters of this session's forwards since the last reset (synchronises): faces culled by
        the R5 vertex cap and clipped faces moved by the R5 sub-vertex clamp (0 on ordinary scenes)."""
        B, H, W, C, V, F = self.dims
        return _lib.clip_stats(B, H, W, F, self.bin_capacity, self.scratch.data_ptr(), self.scratch_bytes,
                               self._stream(), reset)

    def _stream(self):
        """The current stream's handle, ordered after the stream of the session's previous call."""
        cur = torch.cuda.current_stream(self.device)
        last = self._last_stream
        if last is not None and last != cur and not torch.cuda.is_current_stream_capturing():
            cur.wait_stream(last)
        self._last_stream = cur
        return cur.cuda_stream

    def _check(self, t, shape, dtype):
        if t.device != self.device or t.dtype != dtype or tuple(t.shape) != shape or not t.is_contiguous():
            raise ValueError("RasteriseSession expects a contiguous %s %s tensor on %s, got %s %s on %s"
                             % (dtype, shape, self.device, t.dtype, tuple(t.shape), t.device))

    def _check_camera(self, camera_pos):
        """camera_pos as rasterise_ops._camera requires it, without copies: a contiguous float32 tensor on
        this device holding at least the floats the fragment program reads (its pointer goes straight to
        the kernel).  Returns the device pointer, or None for Gouraud without a camera."""
        from .rasterise_ops import _CAMERA_FLOATS
        if camera_pos is None:
            if self.shader_id != _lib.SHADER_GOURAUD:
                raise ValueError("procedural fragment programs need camera_pos (8 floats)")
            return None
        need, why = _CAMERA_FLOATS.get(self.shader_id, (8, "camera_pos must hold at least 8 floats "
                                                           "(csrc/rasterise_egl.cpp:323)"))
        if (not isinstance(camera_pos, torch.Tensor) or camera_pos.device != self.device
                or camera_pos.dtype != torch.float32 or not camera_pos.is_contiguous()):
            raise ValueError("RasteriseSession expects camera_pos as a contiguous float32 tensor on %s" % self.device)
        if camera_pos.numel() < need:
            raise ValueError(why or "camera_pos must hold at least %d floats" % need)
        return camera_pos.data_ptr()

    def forward(self, background, vertices, vertex_colors, faces, camera_pos=None):
        B, H, W, C, V, F = self.dims
        self._check(background, (B, H, W, C), torch.float32)
        self._check(vertices, (B, V, 4), torch.float32)
        self._check(vertex_colors, (B, V, C), torch.float32)
        self._check(faces, (B, F, 3), torch.int32)
        cam = self._check_camera(camera_pos)
        self._inputs = (background, vertices, vertex_colors, faces)
        stream = self._stream()
        _lib.check(self._lib.dirt_rasterise_fwd(
            background.data_ptr(), vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(), cam,
            B, H, W, C, V, F, self.shader_id, self.pixels.data_ptr(), self.gbuffer.data_ptr(),
            self.saved.data_ptr(), self.saved_bytes, self.scratch.data_ptr(), self.scratch_bytes,
            self.bin_capacity, self.fwd_flags, self.grad_vertices.data_ptr(),
            self.grad_vertex_colors.data_ptr(), stream))
        return self.pixels

    def backward(self, grad_pixels):
        if self._inputs is None:
            raise RuntimeError("RasteriseSession.backward called before forward")
        if self.shader_id != _lib.SHADER_GOURAUD:
            raise RuntimeError("only the Gouraud fragment program has a gradient (the reference registers none)")
        B, H, W, C, V, F = self.dims
        self._check(grad_pixels, (B, H, W, C), torch.float32)
        _, vertices, vertex_colors, faces = self._inputs
        stream = self._stream()
        _lib.check(self._lib.dirt_rasterise_bwd(
            vertices.data_ptr(), vertex_colors.data_ptr(), faces.data_ptr(), self.pixels.data_ptr(),
            grad_pixels.data_ptr(), self.gbuffer.data_ptr(), self.saved.data_ptr(), B, H, W, C, V, F,
            self.grad_vertices.data_ptr(), self.grad_vertex_colors.data_ptr(), self.grad_background.data_ptr(),
            _lib.BWD_ACCUMULATE, stream))
        return self.grad_background, self.grad_vertices, self.grad_vertex_colors
