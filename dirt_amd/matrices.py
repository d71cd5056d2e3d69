"""Homogeneous transform helpers -- PyTorch restatement of the reference dirt/matrices.py.

Same conventions as the reference (dirt/matrices.py:1-8): matrices RIGHT-multiply row vectors, i.e.
they are indexed [*, in, out]; the camera looks along -z in view space (README.md:131-132).
These produce inputs for the rasterise op (clip-space vertices); they run on any torch device and
are differentiable through torch autograd.
"""
import torch

__all__ = ["rodrigues", "translation", "perspective_projection", "pad_3x3_to_4x4", "compose"]


def _t(x, like=None):
    if isinstance(x, torch.Tensor):
        return x if x.is_floating_point() else x.float()
    dev = like.device if isinstance(like, torch.Tensor) else None
    return torch.as_tensor(x, dtype=torch.float32, device=dev)


def rodrigues(vectors, name=None):
    """Batch of angle-axis rotation matrices [*, 4, 4] from rotation vectors [*, 3] (dirt/matrices.py:15-56)."""
    del name
    vectors = _t(vectors) + 1.e-12  # as the reference: derivative is otherwise NaN at exactly zero
    norms = torch.linalg.norm(vectors, dim=-1, keepdim=True)
    vectors = vectors / norms
    norms = norms[..., 0]
    z = torch.zeros_like(vectors[..., 0])
    K = torch.stack([
        torch.stack([z, -vectors[..., 2], vectors[..., 1]], dim=-1),
        torch.stack([vectors[..., 2], z, -vectors[..., 0]], dim=-1),
        torch.stack([-vectors[..., 1], vectors[..., 0], z], dim=-1),
    ], dim=-2)  # indexed by *, x/y/z (in), x/y/z (out)
    c = torch.cos(norms)[..., None, None]
    s = torch.sin(norms)[..., None, None]
    eye = torch.eye(3, dtype=vectors.dtype, device=vectors.device)
    result_3x3 = c * eye + (1 - c) * vectors[..., :, None] * vectors[..., None, :] + s * K
    return pad_3x3_to_4x4(result_3x3)


def translation(x, name=None):
    """Batch of translation matrices [*, 4, 4] from displacements [*, 3] (dirt/matrices.py:59-83)."""
    del name
    x = _t(x)
    zeros = torch.zeros_like(x[..., 0])
    ones = torch.ones_like(zeros)
    return torch.stack([
        torch.stack([ones, zeros, zeros, zeros], dim=-1),
        torch.stack([zeros, ones, zeros, zeros], dim=-1),
        torch.stack([zeros, zeros, ones, zeros], dim=-1),
        torch.stack([x[..., 0], x[..., 1], x[..., 2], ones], dim=-1),
    ], dim=-2)


def perspective_projection(near, far, right, aspect, name=None):
    """OpenGL perspective projection [4, 4] for row vectors (dirt/matrices.py:86-117)."""
    del name
    near, far, right, aspect = (_t(v) for v in (near, far, right, aspect))
    top = right * aspect
    zero = torch.zeros_like(near)
    elements = torch.stack([
        torch.stack([near / right, zero, zero, zero]),
        torch.stack([zero, near / top, zero, zero]),
        torch.stack([zero, zero, -(far + near) / (far - near), -2. * far * near / (far - near)]),
        torch.stack([zero, zero, -torch.ones_like(near), zero]),
    ])  # indexed by x/y/z/w (out), x/y/z/w (in)
    return elements.transpose(0, 1).to(torch.float32)


def pad_3x3_to_4x4(matrix, name=None):
    """Pads [*, 3, 3] transforms to homogeneous [*, 4, 4] (dirt/matrices.py:120-143)."""
    del name
    matrix = _t(matrix)
    top = torch.cat([matrix, torch.zeros_like(matrix[..., :, :1])], dim=-1)
    bottom = torch.cat([torch.zeros_like(matrix[..., :1, :]), torch.ones_like(matrix[..., :1, :1])], dim=-1)
    return torch.cat([top, bottom], dim=-2)


def compose(*matrices):
    """Product of transforms applied first-to-last; identity if empty (dirt/matrices.py:146-171)."""
    if len(matrices) == 0:
        return torch.eye(4)
    if len(matrices) == 1:
        return _t(matrices[0])
    return torch.matmul(_t(matrices[0]), compose(*matrices[1:]))
