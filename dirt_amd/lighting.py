"""Per-vertex / per-pixel lighting helpers -- PyTorch restatement of the reference dirt/lighting.py.

Functions, arguments and formulas follow dirt/lighting.py:34-344.  They generate vertex colours for
Gouraud (direct) shading or shade a G-buffer (deferred shading, samples/deferred.py:93-120) and are
differentiable through torch autograd, so gradients flow from pixels through the rasterise op into
normals and geometry (BASELINE config 4: "gradient through normals").
"""
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


def vertex_normals(vertices, faces, name=None):
    """Normalised average of the normals of the faces around each vertex (dirt/lighting.py:34-98)."""
    del name
    vertices, faces = _prepare_vertices_and_faces(vertices, faces)
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
    light_position, light_color = as_t(light_position), as_t(light_color)
    rel = vertex_positions - light_position[..., None, :]
    incident = rel / (torch.linalg.norm(rel, dim=-1, keepdim=True) + 1.e-12)
    cosines = (vertex_normals * incident).sum(-1)
    cosines = cosines.abs() if double_sided else cosines.clamp_min(0.)
    return light_color[..., None, :] * vertex_colors * cosines[..., None]
