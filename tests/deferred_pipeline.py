"""BASELINE config 4: deferred shading with the gradient through normals (reference samples/deferred.py:62-118).

A torch restatement of the sample's chain, parameterised by the renderer so that the same chain runs on
the HIP op and on the CPU oracle (wrapped as an autograd Function, `OracleRasterise`):

  world vertices Vw (the parameter) -> vertex normals (lighting.vertex_normals, :46) and clip-space
  vertices (view + perspective matrices, :50-60) -> three G-buffer renders (:63-83): world positions over
  a -inf background, albedo over 0, normals over -inf -> dilation of positions and normals by a 3x3 max
  pool where the background shows (:85-91) -> per-pixel ambient + diffuse_directional +
  specular_directional (:93-115) -> loss.

Deviation, deliberate: the sample blends `x * (1 - mask) + dilated * mask`, and -inf * 0 is NaN, so in the
reference every background pixel (including the ones the dilation was meant to fill) ends up NaN.  Here
the blend is a select (torch.where), which is what the sample's comment intends ("ensures correct
gradients for pixels just outside the silhouette").  Pixels the dilation does not reach stay
non-finite and are left out of the shading and the loss (selects again, so no NaN reaches a gradient).
The G-buffers' -inf background reaches the rasteriser's backward, whose rule for it is DESIGN.md 4: a
background pixel holding a non-finite value carries no vertex gradient across its pixel pairs.

Test infrastructure only (imported by tests/ and tools/bench_configs.py).
"""
import functools

import numpy as np
import torch
import torch.nn.functional as Fn

from dirt_amd import lighting, matrices


def grid_surface(n=100, seed=0):
    """A rippled n x n grid surface in world space, shared vertices: 2 (n-1)^2 triangles (~20k at n = 100)."""
    rng = np.random.default_rng(seed)
    u, v = np.meshgrid(np.linspace(-1.0, 1.0, n), np.linspace(-1.0, 1.0, n))
    height = 0.15 * np.sin(3.0 * u) * np.cos(2.0 * v) + 0.01 * rng.standard_normal(u.shape)
    world = np.stack([u * 1.4, height, v * 1.4], -1).reshape(-1, 3).astype(np.float32)
    r = np.arange(n - 1)[:, None] * n + np.arange(n - 1)[None, :]
    a = r.reshape(-1)
    faces = np.stack([np.stack([a, a + n, a + 1], -1), np.stack([a + 1, a + n, a + n + 1], -1)], 1).reshape(-1, 3)
    albedo = rng.uniform(0.2, 1.0, size=(len(world), 3)).astype(np.float32)
    return world, faces.astype(np.int32), albedo


@functools.lru_cache(maxsize=16)
def _camera_cpu(H, W):
    view = matrices.compose(matrices.rodrigues([0.9, 0., 0.]), matrices.translation([0., -0.12, -2.3]))
    proj = matrices.perspective_projection(near=0.1, far=20., right=0.1, aspect=float(H) / W)
    return view, proj, torch.linalg.inv(view)[3, :3]


@functools.lru_cache(maxsize=16)
def _camera_on(H, W, device):
    view, proj, pos = _camera_cpu(H, W)
    return view.to(device), proj.to(device), pos.to(device), (view @ proj).to(device)


def camera(H, W, device=None):
    """The sample's camera (samples/deferred.py:50-60, OpenGL perspective); the surface is tilted towards the
    camera (rotation about x) and pushed away along -z.  Built once on the CPU, moved once per device (so a
    step can be captured into a HIP graph: no host-to-device copy inside it)."""
    view, proj = _camera_on(H, W, torch.device(device) if device is not None else torch.device("cpu"))[:2]
    return view, proj


def camera_position(H, W, device=None):
    """The camera's world position, tf.matrix_inverse(view_matrix)[3, :3] (samples/deferred.py:107)."""
    return _camera_on(H, W, torch.device(device) if device is not None else torch.device("cpu"))[2]


@functools.lru_cache(maxsize=16)
def _constants(device):
    return (torch.tensor([0.2, 0.2, 0.2], device=device), unit([1., -0.3, -0.5]).to(device),
            torch.tensor([1., 0., 0.], device=device), torch.tensor([1., 1., 1.], device=device))


def unit(v):
    v = torch.as_tensor(v, dtype=torch.float32)
    return v / torch.linalg.norm(v)


@functools.lru_cache(maxsize=16)
def _backgrounds(H, W, device):
    """The G-buffers' constant backgrounds (-inf for positions and normals, 0 for albedo), made once per device
    rather than filled every step."""
    return torch.full((H, W, 3), float("-inf"), device=device), torch.zeros((H, W, 3), device=device)


def gbuffers(render, Vw, faces, albedo, H, W, geometry_on_cpu=False, batched=False, normals=None):
    """The three G-buffer renders of samples/deferred.py:63-83 ([H,W,3] each) and the clip vertices.

    geometry_on_cpu: compute the clip vertices and normals on the CPU (differentiably) and move them to
    Vw's device, so that two renderers compared on two devices see bit-identical inputs.
    batched: the three renders as one rasterise_batch call of three frames sharing the geometry (the same
    G-buffers and gradients; one op call instead of three).
    normals: precomputed vertex normals (the index_add behind lighting.vertex_normals sums with float atomics on
    the GPU, so two computations may differ in the last bit)."""
    dev = Vw.device
    Vx = Vw.cpu() if geometry_on_cpu else Vw
    # clip = [Vx, 1] @ view @ proj (samples/deferred.py:50-60), as one addmm with the camera's product
    # view @ proj precomputed: the homogeneous 1 picks its last row
    vp = _camera_on(H, W, Vx.device)[3]
    clip = torch.addmm(vp[3], Vx, vp[:3]).to(dev)
    if normals is None:
        normals = lighting.vertex_normals(Vx, faces.to(Vx.device)).to(dev)
    ninf, zero = _backgrounds(H, W, dev)
    if batched:
        import dirt_amd
        bg = torch.stack([ninf, zero, ninf])
        cols = torch.stack([Vw.to(dev), albedo.to(dev), normals])
        f3 = faces.int()[None].expand(3, -1, -1)
        pos, col, nrm = dirt_amd.rasterise_batch(bg, clip[None].expand(3, -1, -1), cols, f3, height=H, width=W,
                                                 channels=3).unbind(0)
        return pos, col, nrm, clip
    pos = render(ninf, clip, Vw, faces, H, W, 3)
    col = render(zero, clip, albedo, faces, H, W, 3)
    nrm = render(ninf, clip, normals, faces, H, W, 3)
    return pos, col, nrm, clip


def shade(pos, col, nrm, H, W):
    """Dilation (:85-91, as a select), per-pixel lighting (:93-115); returns (pixels, valid mask)."""
    dev = pos.device
    bgmask = torch.isinf(pos).any(-1, keepdim=True)

    def dilate(x):
        return Fn.max_pool2d(x.permute(2, 0, 1)[None], 3, stride=1, padding=1)[0].permute(1, 2, 0)

    pos_d = torch.where(bgmask, dilate(pos), pos)
    nrm_d = torch.where(bgmask, dilate(nrm), nrm)
    valid = torch.isfinite(pos_d).all(-1, keepdim=True) & torch.isfinite(nrm_d).all(-1, keepdim=True)
    pos_s, nrm_s, col_s = (torch.where(valid, x, 0.0) for x in (pos_d, nrm_d, col))
    grey, light_direction, red, white = _constants(dev)
    ambient = col_s * grey
    diffuse = lighting.diffuse_directional(nrm_s.reshape(-1, 3), col_s.reshape(-1, 3), light_direction,
                                           light_color=red, double_sided=False)
    specular = lighting.specular_directional(pos_s.reshape(-1, 3), nrm_s.reshape(-1, 3), col_s.reshape(-1, 3),
                                             light_direction, light_color=white,
                                             camera_position=camera_position(H, W, dev), shininess=6.,
                                             double_sided=False)
    pixels = diffuse.reshape(H, W, 3) + specular.reshape(H, W, 3) + ambient
    return pixels, valid


def loss_fn(pixels, valid, weights, mask=None):
    m = valid if mask is None else (valid & mask)
    return torch.where(m, pixels * weights, 0.0).sum()


def chain(render, Vw, faces, albedo, H, W, weights, mask=None, geometry_on_cpu=False, batched=False):
    pos, col, nrm, _ = gbuffers(render, Vw, faces, albedo, H, W, geometry_on_cpu, batched)
    pixels, valid = shade(pos, col, nrm, H, W)
    return loss_fn(pixels, valid, weights, mask), pixels, valid


class OracleRasterise(torch.autograd.Function):
    """The CPU oracle's forward and backward (oracle/dirt_oracle.c) as a torch op, for composing the oracle
    with CPU autograd.  Single frame, shapes as dirt_amd.rasterise."""

    @staticmethod
    def forward(ctx, background, vertices, vertex_colors, faces):
        from oracle import oracle
        bg, v, c, f = (x.detach().cpu().numpy()[None] for x in (background, vertices, vertex_colors, faces))
        px, gb, _ = oracle.rasterise_fwd(bg, v, c, f)
        ctx.save = (v, c, f, px, gb)
        return torch.from_numpy(px[0])

    @staticmethod
    def backward(ctx, grad_pixels):
        from oracle import oracle
        v, c, f, px, gb = ctx.save
        gv, gc, gbg = oracle.rasterise_bwd(v, c, f, px, grad_pixels.detach().cpu().numpy()[None].astype(np.float32), gb)
        return torch.from_numpy(gbg[0]), torch.from_numpy(gv[0]), torch.from_numpy(gc[0]), None


def oracle_render(bg, v, c, f, H, W, C):
    return OracleRasterise.apply(bg, v, c, f.int())


def hip_render(bg, v, c, f, H, W, C):
    import dirt_amd
    return dirt_amd.rasterise(bg, v, c, f.int(), height=H, width=W, channels=C)
