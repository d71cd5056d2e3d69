"""Per-vertex / per-pixel lighting helpers -- PyTorch restatement of the reference dirt/lighting.py.

Functions, arguments and formulas follow dirt/lighting.py:34-344.  They generate vertex colours for
Gouraud (direct) shading or shade a G-buffer (deferred shading, samples/deferred.py:93-120) and are
differentiable through torch autograd, so gradients flow from pixels through the rasterise op into
normals and geometry (BASELINE config 4: "gradient through normals").

On the GPU, vertex_normals, diffuse_directional, specular_directional and diffuse_point run as fused HIP
kernels (one launch per forward and per backward, dirt_amd/csrc/lighting_kernels.h, C ABI
dirt_vertex_normals_* / dirt_diffuse_directional_* / dirt_specular_directional_* / dirt_diffuse_point_*) when
their operands are float32 tensors on one GPU, of one [..., 3] shape, with light parameters of shape [3] that need no gradient and a Python-number
shininess; anything else -- CPU tensors, broadcasting, gradients with respect to the light -- runs the
framework-op statement below (`_*_ops`), which is also the fused kernels' fp32 test reference.

The fused backwards are kernels, not differentiable graphs: a second-order gradient through them
(`create_graph=True`) raises RuntimeError rather than silently dropping terms.  DIRT_FUSED_LIGHTING=0 routes every
call to the framework ops (double backward supported).  Out-of-range face indices: the fused vertex_normals skips
such faces; the framework statement's index_select rejects them (on a GPU as a device-side assert).
"""
import os

import torch

__all__ = ["vertex_normals", "vertex_normals_pre_split", "split_vertices_by_face", "diffuse_directional",
           "specular_directional", "diffuse_point"]


def _prepare_vertices_and_faces(vertices, faces):
    vertices = torch.as_tensor(vertices)
    if not vertices.is_floating_point():
        vertices = vertices.float()
    faces = torch.as_tensor(faces, device=vertices.device).long()
    return vertices, faces


def _get_face_normals(vertices, faces):
    # vertices [*, V, 3]; result [*, F, 3] (dirt/lighting.py:23-31).  index_select rather than advanced
    # indexing: its backward is one index_add, where advanced indexing's sorts the indices first
    v = vertices.index_select(-2, faces.reshape(-1)).reshape(vertices.shape[:-2] + (faces.shape[0], 3, vertices.shape[-1]))
    normals = torch.cross(v[..., 1, :] - v[..., 0, :], v[..., 2, :] - v[..., 0, :], dim=-1)
    return normals / (torch.linalg.norm(normals, dim=-1, keepdim=True) + 1.e-12)


_FUSED_ENABLED = os.environ.get("DIRT_FUSED_LIGHTING", "1") != "0"


def _fused():
    """The C++ extension bound to the HIP library (None if not built or DIRT_FUSED_LIGHTING=0: the framework ops
    run)."""
    if not _FUSED_ENABLED:
        return None
    from .rasterise_ops import _torch_ext
    return _torch_ext()


def _gpu_f32(*xs):
    x0 = xs[0]
    return (x0.is_cuda and all(isinstance(x, torch.Tensor) and x.dtype == torch.float32 and x.device == x0.device
                               for x in xs))


def _light_param(x, like):
    """A [3] light parameter usable by the fused kernels (on like's device, float32, no gradient), else None."""
    if not isinstance(x, torch.Tensor) or x.shape != (3,) or x.dtype != torch.float32 or x.device != like.device:
        return None
    if x.requires_grad and torch.is_grad_enabled():
        return None
    return x.contiguous()


def vertex_normals(vertices, faces, name=None):
    """Normalised average of the normals of the faces around each vertex (dirt/lighting.py:34-98)."""
    del name
    vertices = torch.as_tensor(vertices)
    f = torch.as_tensor(faces, device=vertices.device)
    if (_gpu_f32(vertices) and vertices.dim() >= 2 and vertices.shape[-1] >= 3 and f.dim() == 2 and
            f.shape[-1] == 3 and f.dtype in (torch.int32, torch.int64)):
        ext = _fused()
        if ext is not None:
            # (int32 or int64 faces as given; a face with an index outside [0, V) contributes nothing here,
            # where the framework ops raise)
            return ext.vertex_normals(vertices.contiguous(), f.contiguous())
    vertices, faces = _prepare_vertices_and_faces(vertices, faces)
    return _vertex_normals_ops(vertices, faces)


def _vertex_normals_ops(vertices, faces):
    vertices = vertices[..., :3]
    normals_by_face = _get_face_normals(vertices, faces)  # [*, F, 3]
    lead = normals_by_face.shape[:-2]
    summed = torch.zeros(lead + (vertices.shape[-2], 3), dtype=vertices.dtype, device=vertices.device)
    # every face's normal to its three vertices in one index_add (face-major, as faces.reshape(-1))
    summed = summed.index_add(-2, faces.reshape(-1), normals_by_face.repeat_interleave(3, dim=-2))
    return summed / (torch.linalg.norm(summed, dim=-1, keepdim=True) + 1.e-12)


def vertex_normals_pre_split(vertices, faces, name=None, static=False):
    """Face normals written to each face's (unshared) vertices (dirt/lighting.py:101-133)."""
    del name, static
    vertices, faces = _prepare_vertices_and_faces(vertices, faces)
    vertices = vertices[..., :3]
    normals_by_face = _get_face_normals(vertices, faces)  # [*, F, 3]
    out = torch.zeros_like(vertices)
    idx = faces.reshape(-1)
    upd = normals_by_face[..., :, None, :].expand(normals_by_face.shape[:-1] + (3, 3))
    upd = upd.reshape(normals_by_face.shape[:-2] + (idx.numel(), 3))
    out = out.index_copy(-2, idx, upd)
    return out


def split_vertices_by_face(vertices, faces, name=None):
    """Duplicate vertices so each is used by exactly one face (dirt/lighting.py:136-179).

    Returns (new_vertices [*, 3F, D], new_faces [F, 3] = arange(3F))."""
    del name
    vertices, faces = _prepare_vertices_and_faces(vertices, faces)
    F = faces.shape[0]
    new_vertices = vertices[..., faces.reshape(-1), :]
    new_faces = torch.arange(F * 3, dtype=torch.int32, device=vertices.device).reshape(F, 3)
    return new_vertices, new_faces


def diffuse_directional(vertex_normals, vertex_colors, light_direction, light_color, double_sided=True, name=None):
    """Lambertian reflectance under one directional light (dirt/lighting.py:182-225)."""
    del name
    vertex_normals = torch.as_tensor(vertex_normals)
    dev, dt = vertex_normals.device, vertex_normals.dtype
    vertex_colors = torch.as_tensor(vertex_colors, dtype=dt, device=dev)
    if (_gpu_f32(vertex_normals, vertex_colors) and vertex_normals.shape[-1:] == (3,) and
            vertex_colors.shape == vertex_normals.shape):
        ld, lc = _light_param(light_direction, vertex_normals), _light_param(light_color, vertex_normals)
        ext = _fused() if ld is not None and lc is not None else None
        if ext is not None:
            return ext.diffuse_directional(vertex_normals.contiguous(), vertex_colors.contiguous(), ld, lc,
                                           bool(double_sided))
    return _diffuse_directional_ops(vertex_normals, vertex_colors, light_direction, light_color, double_sided)


def _diffuse_directional_ops(vertex_normals, vertex_colors, light_direction, light_color, double_sided):
    dev, dt = vertex_normals.device, vertex_normals.dtype
    light_direction = torch.as_tensor(light_direction, dtype=dt, device=dev)
    light_color = torch.as_tensor(light_color, dtype=dt, device=dev)
    # (an elementwise product and a 3-term sum: a [V, 3] x [3, 1] matmul is a slow GEMM shape)
    cosines = (vertex_normals * -light_direction[..., None, :]).sum(-1, keepdim=True)  # [*, V, 1]
    cosines = cosines.abs() if double_sided else cosines.clamp_min(0.)
    return light_color[..., None, :] * vertex_colors * cosines


def specular_directional(vertex_positions, vertex_normals, vertex_reflectivities, light_direction, light_color,
                         camera_position, shininess, double_sided=True, name=None):
    """Phong reflectance under one directional light (dirt/lighting.py:228-288)."""
    del name
    vertex_positions = torch.as_tensor(vertex_positions)
    dev, dt = vertex_positions.device, vertex_positions.dtype
    as_t = lambda x: torch.as_tensor(x, dtype=dt, device=dev)  # noqa: E731
    vertex_normals, vertex_reflectivities = as_t(vertex_normals), as_t(vertex_reflectivities)
    if (_gpu_f32(vertex_positions, vertex_normals, vertex_reflectivities) and vertex_positions.shape[-1:] == (3,) and
            vertex_normals.shape == vertex_positions.shape and vertex_reflectivities.shape == vertex_positions.shape and
            isinstance(shininess, (int, float))):
        ps = [_light_param(x, vertex_positions) for x in (light_direction, light_color, camera_position)]
        ext = _fused() if all(p is not None for p in ps) else None
        if ext is not None:
            return ext.specular_directional(vertex_positions.contiguous(), vertex_normals.contiguous(),
                                            vertex_reflectivities.contiguous(), ps[0], ps[1], ps[2], float(shininess),
                                            bool(double_sided))
    return _specular_directional_ops(vertex_positions, vertex_normals, vertex_reflectivities, light_direction,
                                     light_color, camera_position, shininess, double_sided)


def _specular_directional_ops(vertex_positions, vertex_normals, vertex_reflectivities, light_direction, light_color,
                              camera_position, shininess, double_sided):
    dev, dt = vertex_positions.device, vertex_positions.dtype
    as_t = lambda x: torch.as_tensor(x, dtype=dt, device=dev)  # noqa: E731
    light_direction, light_color = as_t(light_direction), as_t(light_color)
    camera_position = as_t(camera_position)
    # a Python-number exponent stays a number: no host-to-device copy per call (and the call can be captured
    # into a HIP graph, where such a copy is not permitted)
    shininess = shininess if isinstance(shininess, (int, float)) else as_t(shininess)[..., None, None]
    to_light = -light_direction
    reflected = -to_light + 2. * (vertex_normals * to_light[..., None, :]).sum(-1, keepdim=True) * vertex_normals
    to_camera = camera_position[..., None, :] - vertex_positions
    cosines = ((to_camera / torch.linalg.norm(to_camera, dim=-1, keepdim=True) + 1.e-12) * reflected).sum(-1, keepdim=True)
    cosines = cosines.abs() if double_sided else cosines.clamp_min(0.)
    return light_color[..., None, :] * vertex_reflectivities * torch.pow(cosines, shininess)


def diffuse_point(vertex_positions, vertex_normals, vertex_colors, light_position, light_color, double_sided=True,
                  name=None):
    """Lambertian reflectance under one point light (dirt/lighting.py:291-344)."""
    del name
    vertex_positions = torch.as_tensor(vertex_positions)
    dev, dt = vertex_positions.device, vertex_positions.dtype
    as_t = lambda x: torch.as_tensor(x, dtype=dt, device=dev)  # noqa: E731
    vertex_normals, vertex_colors = as_t(vertex_normals), as_t(vertex_colors)
    if (_gpu_f32(vertex_positions, vertex_normals, vertex_colors) and vertex_positions.shape[-1:] == (3,) and
            vertex_normals.shape == vertex_positions.shape and vertex_colors.shape == vertex_positions.shape):
        lp, lc = _light_param(light_position, vertex_positions), _light_param(light_color, vertex_positions)
        ext = _fused() if lp is not None and lc is not None else None
        if ext is not None:
            return ext.diffuse_point(vertex_positions.contiguous(), vertex_normals.contiguous(),
                                     vertex_colors.contiguous(), lp, lc, bool(double_sided))
    return _diffuse_point_ops(vertex_positions, vertex_normals, vertex_colors, light_position, light_color,
                              double_sided)


def _diffuse_point_ops(vertex_positions, vertex_normals, vertex_colors, light_position, light_color, double_sided):
    dev, dt = vertex_positions.device, vertex_positions.dtype
    as_t = lambda x: torch.as_tensor(x, dtype=dt, device=dev)  # noqa: E731
    light_position, light_color = as_t(light_position), as_t(light_color)
    rel = vertex_positions - light_position[..., None, :]
    incident = rel / (torch.linalg.norm(rel, dim=-1, keepdim=True) + 1.e-12)
    cosines = (vertex_normals * incident).sum(-1)
    cosines = cosines.abs() if double_sided else cosines.clamp_min(0.)
    return light_color[..., None, :] * vertex_colors * cosines[..., None]
