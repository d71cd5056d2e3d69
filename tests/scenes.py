"""Input generators for the parity tests and the bench (BASELINE.json configs).

Each builder returns float32/int32 numpy arrays shaped like the reference op's inputs:
background [H,W,C], vertices [V,4] (clip space), vertex_colors [V,C], faces [F,3].
"""
import math

import numpy as np
import torch

from dirt_amd import lighting, matrices


def readme_square(W=128, H=128, centre=(32.0, 64.0), size=16.0, C=1):
    """README.md:27-70: a square of side `size` pixels centred at `centre` (window coords)."""
    sq = np.array([[0, 0], [0, 1], [1, 1], [1, 0]], np.float32) * size - size / 2.0
    sq = sq + np.array(centre, np.float32)
    sq = sq * 2.0 / np.array([W, H], np.float32) - 1.0
    v = np.concatenate([sq, np.zeros([4, 1], np.float32), np.ones([4, 1], np.float32)], 1).astype(np.float32)
    return (np.zeros([H, W, C], np.float32), v, np.ones([4, C], np.float32), np.array([[0, 1, 2], [0, 2, 3]], np.int32))


def _cube():
    vertices = [[x, y, z] for z in [-1, 1] for y in [-1, 1] for x in [-1, 1]]
    quads = [[0, 1, 3, 2], [4, 5, 7, 6], [1, 5, 4, 0], [2, 6, 7, 3], [4, 6, 2, 0], [3, 7, 5, 1]]
    triangles = sum([[[a, b, c], [c, d, a]] for [a, b, c, d] in quads], [])
    return np.array(vertices, np.float32), np.array(triangles, np.int32)


def cube_scene(W=256, H=256, yaw=0.5):
    """samples/simple.py:37-74 (Gouraud-lit, split-vertex cube; BASELINE config 2 at 256x256)."""
    verts, faces = _cube()
    verts, faces = lighting.split_vertices_by_face(torch.from_numpy(verts), torch.from_numpy(faces))
    colors = torch.ones_like(verts)
    verts_h = torch.cat([verts, torch.ones_like(verts[:, -1:])], 1)
    world = verts_h @ matrices.rodrigues([0., yaw, 0.])
    normals = lighting.vertex_normals_pre_split(world, faces)
    view = matrices.compose(matrices.translation([0., -1.5, -3.5]), matrices.rodrigues([-0.3, 0., 0.]))
    proj = matrices.perspective_projection(near=0.1, far=20., right=0.1, aspect=float(H) / W)
    clip = world @ view @ proj
    lit = lighting.diffuse_directional(normals, colors, light_direction=[1., 0., 0.], light_color=[1., 1., 1.]) * 0.8 \
        + colors * 0.2
    return (np.zeros([H, W, 3], np.float32), clip.numpy().astype(np.float32), lit.numpy().astype(np.float32),
            faces.numpy().astype(np.int32))


def make_cylinder(radius, height, end_offset, bevel, segments):
    """tests/rasterise_tests.py:10-46 (Python-3 restatement)."""
    angles = np.linspace(0., 2 * math.pi, segments, endpoint=False, dtype=np.float32)
    xz = np.stack([np.cos(angles), np.sin(angles)], axis=1) * radius
    top_bevel = np.stack([xz[:, 0] * (1. - bevel), np.ones(segments) * -height / 2. - radius * bevel, xz[:, 1] * (1. - bevel)], 1)
    top = np.stack([xz[:, 0], np.ones(segments) * -height / 2., xz[:, 1]], 1)
    bottom = np.stack([xz[:, 0], np.ones(segments) * height / 2., xz[:, 1]], 1)
    bottom_bevel = np.stack([xz[:, 0] * (1. - bevel), np.ones(segments) * height / 2. + radius * bevel, xz[:, 1] * (1. - bevel)], 1)
    ends = [[0., -height / 2. - end_offset, 0.], [0., height / 2. + end_offset, 0.]]
    all_vertices = np.concatenate([top_bevel, top, bottom, bottom_bevel, ends], 0)
    faces = []

    def make_ring(start):
        for q in range(segments):
            uf, us = start + q, start + (q + 1) % segments
            lf, ls = start + q + segments, start + (q + 1) % segments + segments
            faces.extend([[uf, us, lf], [lf, us, ls]])
    make_ring(0)
    make_ring(segments)
    make_ring(segments * 2)
    for tf_ in range(segments):
        ts = (tf_ + 1) % segments
        bf = tf_ + segments * 3
        bs = (bf + 1) % segments
        faces.extend([[segments * 4, tf_, ts], [segments * 4 + 1, bf, bs]])
    return all_vertices.astype(np.float32), np.array(faces, np.int32)


def cylinder_clip_vertices(translation=(0., 0., -0.25), rotation_xy=0.0, W=48, H=36):
    """Projected split cylinder of tests/rasterise_tests.py:49-77 as a function of the pose (torch, differentiable)."""
    verts, faces = make_cylinder(0.2, 0.75, 0.1, 0., 10)
    verts = np.concatenate([verts, np.ones([len(verts), 1], np.float32)], 1).astype(np.float32)
    r = torch.as_tensor(rotation_xy, dtype=torch.float32)
    t = torch.as_tensor(translation, dtype=torch.float32)
    z, o = torch.zeros(()), torch.ones(())
    view1 = torch.stack([
        torch.stack([0.5 * torch.cos(r), 0.5 * -torch.sin(r), z, z]),
        torch.stack([0.5 * torch.sin(r), 0.5 * torch.cos(r), z, z]),
        torch.stack([z, z, 0.5 * o, z]),
        torch.stack([z, z, z, o]),
    ])
    view2 = torch.stack([
        torch.stack([o, z, z, z]), torch.stack([z, o, z, z]), torch.stack([z, z, o, z]),
        torch.cat([t, o[None]]),
    ])
    sv, sf = lighting.split_vertices_by_face(torch.from_numpy(verts), torch.from_numpy(faces))
    proj = matrices.perspective_projection(0.1, 20., 0.2, float(H) / W)
    return sv @ view1 @ view2 @ proj, sf


def cylinder_scene(W=48, H=36, seed=0, bgcolor=(0.4, 0.2, 0.2), vertex_color=(0.7, 0.3, 0.6)):
    """tests/rasterise_tests.py:79-88: half-bgcolor background, first 75 vertices one colour."""
    clip, faces = cylinder_clip_vertices((0., 0., -0.25), 0.0, W, H)
    V = clip.shape[0]
    rng = np.random.RandomState(seed)
    cols = np.concatenate([np.tile(np.array(vertex_color, np.float32)[None], [75, 1]),
                           rng.uniform(size=[V - 75, 3]).astype(np.float32)], 0)
    bg = np.concatenate([np.tile(np.array(bgcolor, np.float32)[None, None], [H // 2, W, 1]),
                         np.ones([H - H // 2, W, 3], np.float32)], 0)
    return bg.astype(np.float32), clip.detach().numpy().astype(np.float32), cols, faces.numpy().astype(np.int32)


def random_triangles(F=50000, W=1024, H=1024, C=3, radius_px=16.0, seed=0, perspective=False, spread=1.0):
    """SURVEY 8d synthetic distribution (BASELINE config 3): centres U[-1,1]^2, vertex offsets uniform in a
    disk of radius `radius_px` pixels, z ~ U(-0.95,0.95) +-0.01 jitter, w=1 (or w~U(1,3) scaling xyz);
    split vertices (V=3F), colours and background U[0,1].  spread < 1: centres U[-spread, spread]^2 (a
    clustered mesh: spread 0.25 puts every face in the centre 1/16 of the frame)."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(-spread, spread, size=(F, 1, 2))
    ang = rng.uniform(0, 2 * np.pi, size=(F, 3))
    rad = radius_px * np.sqrt(rng.uniform(0, 1, size=(F, 3)))
    off = np.stack([np.cos(ang) * rad * 2.0 / W, np.sin(ang) * rad * 2.0 / H], -1)
    xy = centres + off
    z = rng.uniform(-0.95, 0.95, size=(F, 1)) + rng.uniform(-0.01, 0.01, size=(F, 3))
    v = np.concatenate([xy, z[..., None], np.ones((F, 3, 1))], -1).reshape(F * 3, 4)
    if perspective:
        w = rng.uniform(1, 3, size=(F * 3, 1))
        v = v * w
    faces = np.arange(3 * F, dtype=np.int32).reshape(F, 3)
    cols = rng.uniform(0, 1, size=(3 * F, C))
    bg = rng.uniform(0, 1, size=(H, W, C))
    return bg.astype(np.float32), v.astype(np.float32), cols.astype(np.float32), faces


def clipping_scene(W=96, H=64, C=3, seed=3):
    """Triangles crossing the near plane, behind the camera, and far outside the guard band (R5)."""
    rng = np.random.default_rng(seed)
    tris = []
    for _ in range(40):
        p = rng.uniform(-3, 3, size=(3, 3))
        w = rng.uniform(-0.6, 2.0, size=(3, 1))
        z = rng.uniform(-1.5, 1.5, size=(3, 1)) * np.abs(w)
        tris.append(np.concatenate([p[:, :2], z, w], 1))
    # huge triangle spanning far beyond the guard band, fully in front
    tris.append(np.array([[-5000, -5000, 0.1, 1], [5000, -5000, 0.1, 1], [0, 8000, 0.1, 1]], np.float64))
    # triangle with one vertex behind the eye
    tris.append(np.array([[-0.5, -0.5, 0.2, 1], [0.5, -0.5, 0.2, 1], [0.0, 0.6, -0.5, -0.3]], np.float64))
    v = np.concatenate(tris, 0).astype(np.float32)
    F = len(tris)
    faces = np.arange(3 * F, dtype=np.int32).reshape(F, 3)
    cols = rng.uniform(0, 1, size=(3 * F, C)).astype(np.float32)
    bg = rng.uniform(0, 1, size=(H, W, C)).astype(np.float32)
    return bg, v, cols, faces


def shared_mesh_scene(W=80, H=60, C=3, seed=5, n=12):
    """A jittered grid mesh with SHARED vertices (non-split), partly occluding a second grid."""
    rng = np.random.default_rng(seed)
    verts, faces = [], []
    for layer, z in enumerate([0.2, -0.1]):
        base = len(verts)
        xs = np.linspace(-0.9 + 0.3 * layer, 0.6 + 0.3 * layer, n)
        ys = np.linspace(-0.8, 0.8 - 0.3 * layer, n)
        for yy in ys:
            for xx in xs:
                verts.append([xx + rng.uniform(-0.02, 0.02), yy + rng.uniform(-0.02, 0.02), z + rng.uniform(-0.05, 0.05), 1.0])
        for r in range(n - 1):
            for c in range(n - 1):
                a = base + r * n + c
                faces.append([a, a + 1, a + n])
                faces.append([a + 1, a + n + 1, a + n])
    v = np.array(verts, np.float32)
    f = np.array(faces, np.int32)
    cols = rng.uniform(0, 1, size=(len(v), C)).astype(np.float32)
    bg = rng.uniform(0, 1, size=(H, W, C)).astype(np.float32)
    return bg, v, cols, f


def batch_of(scene_fn, B, **kw):
    """Stack B independent frames of a scene builder (seed offset by frame index)."""
    seed0 = kw.pop("seed", 0)
    takes_seed = "seed" in scene_fn.__code__.co_varnames
    frames = [scene_fn(seed=seed0 + b, **kw) if takes_seed else scene_fn(**kw) for b in range(B)]
    return tuple(np.stack([fr[k] for fr in frames]) for k in range(4))


def deferred_mesh_scene(W=512, H=512, C=7, n=100, seed=0):
    """BASELINE config 4 (samples/deferred.py:63-91 G-buffer): a shared-vertex, subdivided n x n grid surface
    (2 (n-1)^2 ~ 20k triangles at n=100) rippled in depth, seen in perspective, carrying 7 channels per
    vertex (normal xyz, albedo rgb, view depth) -- one 7-channel call instead of the reference's 3+3+1."""
    rng = np.random.default_rng(seed)
    u, v = np.meshgrid(np.linspace(-1.0, 1.0, n), np.linspace(-1.0, 1.0, n))
    height = 0.15 * np.sin(3.0 * u) * np.cos(2.0 * v) + 0.02 * rng.standard_normal(u.shape)
    world = np.stack([u * 1.6, height, v * 1.6 - 0.2], -1).reshape(-1, 3).astype(np.float32)
    faces = []
    for r in range(n - 1):
        for c in range(n - 1):
            a = r * n + c
            faces.append([a, a + 1, a + n])
            faces.append([a + 1, a + n + 1, a + n])
    faces = np.array(faces, np.int32)
    wt = torch.from_numpy(world)
    ft = torch.from_numpy(faces).long()
    normals = lighting.vertex_normals(wt, ft).numpy()
    # tilted-plane perspective built directly in clip space: NDC x, y over [-0.9, 0.9] (plus the ripple),
    # w grows from 1 at the bottom edge to 3 at the top (receding surface)
    w = (2.0 + v).reshape(-1, 1)
    ndc = np.stack([u * 0.9, v * 0.9 + height * 0.5], -1).reshape(-1, 2)
    zc = (0.2 * v + height).reshape(-1, 1)
    clip = np.concatenate([ndc * w, zc * w, w], 1).astype(np.float32)
    albedo = rng.uniform(0.2, 1.0, size=(len(world), 3))
    depth = w
    attrs = np.concatenate([normals, albedo, depth], 1)[:, :C].astype(np.float32)
    bg = np.zeros((H, W, C), np.float32)
    return bg, clip, attrs, faces


def hill_terrain(H, W, C=4):
    """Synthetic terrain lookup for the `hill` program (x = height in [0, 1], yzw = normal * 0.5 + 0.5,
    the layout shaders.cpp:219-237 decodes); rows top first like any background."""
    y, x = np.meshgrid(np.linspace(0, 1, H), np.linspace(0, 1, W), indexing="ij")
    h = 0.5 + 0.25 * np.sin(6.1 * x + 1.3) * np.cos(4.7 * y) + 0.15 * np.sin(13 * x * y + 0.4)
    gy, gx = np.gradient(h)
    n = np.stack([-gx * 40, np.ones_like(h), -gy * 40], -1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    t = np.concatenate([h[..., None], (n + 1) / 2], -1).astype(np.float32)
    return t[..., :C].copy() if C != 4 else t


def fullscreen_quad():
    """The procedural ops' harness geometry (tests/square_test.py:16,31): two faces covering the frame."""
    v = np.array([[-1, -1, 0, 1], [-1, 1, 0, 1], [1, 1, 0, 1], [1, -1, 0, 1]], np.float32)
    f = np.array([[0, 1, 2], [0, 2, 3]], np.int32)
    return v, f


def near_w0_scene(seed, W=64, H=48, C=3, F=160):
    """Clipping stress around w = 0, where R5's plane intersections lose their guard-band guarantee (fuzz seed
    167059): faces with one or two vertices at |w| log-uniform in [1e-14, 1e-2] (either sign) and x, y up to
    1e4 |w| (far outside the guard band) or exactly on a guard plane, near-duplicate copies shifted by a few
    ulps (the seed's two faces), and ordinary faces for the depth test to compete with."""
    rng = np.random.default_rng(seed)
    gx, gy = 32768.0 / W, 32768.0 / H
    tris = []
    for _ in range(F):
        kind = rng.integers(0, 5)
        if kind == 4 and tris:  # near-duplicate of an earlier face: every coordinate nudged by a few ulps
            base = np.array(tris[rng.integers(0, len(tris))], np.float32)
            tris.append((base * (1 + rng.integers(-4, 5, size=base.shape) * np.float32(2 ** -23))).tolist())
            continue
        t = []
        nsmall = rng.integers(1, 3)
        for k in range(3):
            if k < nsmall:
                w = 10.0 ** rng.uniform(-14, -2) * rng.choice([-1.0, 1.0, 1.0])
                if rng.uniform() < 0.3:  # on a guard plane
                    x, y = rng.choice([-gx, gx]) * abs(w), rng.uniform(-gy, gy) * abs(w)
                else:
                    x, y = rng.uniform(-1e4, 1e4, 2) * abs(w)
                z = rng.uniform(-1.5, 1.5) * abs(w)
            else:
                w = rng.uniform(0.3, 2.0)
                x, y = rng.uniform(-1.2, 1.2, 2) * w
                z = rng.uniform(-0.9, 0.9) * w
            t.append([x, y, z, w])
        tris.append([t[i] for i in rng.permutation(3)])
    for _ in range(F // 4):  # ordinary faces
        p = rng.uniform(-1, 1, size=(3, 2))
        z = rng.uniform(-0.9, 0.9)
        tris.append([[p[k, 0], p[k, 1], z, 1.0] for k in range(3)])
    v = np.array(tris, np.float64).reshape(-1, 4).astype(np.float32)
    faces = np.arange(len(v), dtype=np.int32).reshape(-1, 3)
    cols = rng.uniform(0, 1, size=(len(v), C)).astype(np.float32)
    bg = rng.uniform(0, 1, size=(H, W, C)).astype(np.float32)
    return bg, v, cols, faces


def adversarial_scene(seed, W=64, H=48, C=3, F=300):
    """Fuzz scene for the raster rules' edge cases, mixed at random: vertices snapped to pixel centres and
    pixel edges (top-left rule ties), axis-aligned edges, fans sharing edges, slivers, sub-pixel
    triangles, duplicated faces and coplanar overlaps (depth ties: the lower face wins), z beyond the
    near / far planes, w near zero or negative (clipping), coordinates far outside the guard band."""
    rng = np.random.default_rng(seed)
    tris = []

    def ndc_x(px):  # window x (pixels) -> NDC
        return px * 2.0 / W - 1.0

    def ndc_y(py):
        return py * 2.0 / H - 1.0

    for _ in range(F):
        kind = rng.integers(0, 9)
        z = rng.uniform(-0.9, 0.9)
        if kind == 0:    # vertices on pixel centres
            p = rng.integers(0, max(W, H), size=(3, 2)) + 0.5
            t = [[ndc_x(a), ndc_y(b), z, 1.0] for a, b in p]
        elif kind == 1:  # vertices on pixel corners, axis-aligned right triangle
            x0, y0 = rng.integers(0, W), rng.integers(0, H)
            s = rng.integers(1, 12)
            t = [[ndc_x(x0), ndc_y(y0), z, 1.0], [ndc_x(x0 + s), ndc_y(y0), z, 1.0], [ndc_x(x0), ndc_y(y0 + s), z, 1.0]]
        elif kind == 2:  # sliver: nearly collinear
            a = rng.uniform(-1, 1, 2)
            d = rng.uniform(-0.5, 0.5, 2)
            n = np.array([-d[1], d[0]]) * rng.uniform(1e-4, 1e-2)
            t = [[*a, z, 1.0], [*(a + d), z, 1.0], [*(a + 0.5 * d + n), z, 1.0]]
        elif kind == 3:  # sub-pixel triangle
            c = rng.uniform(-1, 1, 2)
            o = rng.uniform(-0.8, 0.8, size=(3, 2)) * np.array([2.0 / W, 2.0 / H])
            t = [[*(c + oo), z, 1.0] for oo in o]
        elif kind == 4 and tris:  # duplicate of an earlier face (exact depth tie)
            t = [list(vv) for vv in tris[rng.integers(0, len(tris))]]
        elif kind == 5 and tris:  # coplanar overlap: an earlier face's plane, shifted in xy
            base = np.array(tris[rng.integers(0, len(tris))], np.float64)
            sh = rng.uniform(-0.05, 0.05, 2)
            t = [[vv[0] + sh[0] * vv[3], vv[1] + sh[1] * vv[3], vv[2], vv[3]] for vv in base]
        elif kind == 6:  # beyond near / far planes or straddling them
            p = rng.uniform(-1, 1, size=(3, 2))
            zz = rng.uniform(-1.6, 1.6, size=3)
            t = [[p[k, 0], p[k, 1], zz[k], 1.0] for k in range(3)]
        elif kind == 7:  # w near zero or negative (perspective clipping)
            p = rng.uniform(-1, 1, size=(3, 2))
            w = rng.choice([rng.uniform(-0.3, 0.3), rng.uniform(0.5, 2.0)], size=3)
            t = [[p[k, 0] * abs(w[k]), p[k, 1] * abs(w[k]), z * abs(w[k]), w[k]] for k in range(3)]
        else:            # fan sharing a centre vertex and edges with the previous fan triangle
            c = rng.uniform(-0.8, 0.8, 2)
            r = rng.uniform(0.02, 0.4)
            a0 = rng.uniform(0, 2 * np.pi)
            for k in range(3):
                a1, a2 = a0 + k * 2.1, a0 + (k + 1) * 2.1
                tris.append([[*c, z, 1.0], [c[0] + r * np.cos(a1), c[1] + r * np.sin(a1), z, 1.0],
                             [c[0] + r * np.cos(a2), c[1] + r * np.sin(a2), z, 1.0]])
            continue
        tris.append(t)
    if rng.uniform() < 0.5:  # one triangle far outside the guard band
        tris.append([[-4000.0, -3000.0, 0.3, 1.0], [5000.0, -2000.0, 0.3, 1.0], [100.0, 6000.0, 0.3, 1.0]])
    v = np.array(tris, np.float64).reshape(-1, 4).astype(np.float32)
    nf = len(tris)
    faces = np.arange(3 * nf, dtype=np.int32).reshape(nf, 3)
    cols = rng.uniform(0, 1, size=(3 * nf, C)).astype(np.float32)
    bg = rng.uniform(0, 1, size=(H, W, C)).astype(np.float32)
    return bg, v, cols, faces


def fuzz_case(seed):
    """The scene of tests/test_gpu_parity.py::test_fuzz_adversarial_scenes for `seed` (a batch of two frames of
    150 faces when seed % 4 == 3, padded to a common F and V, else one frame)."""
    W, H = [(64, 48), (33, 17), (130, 70)][seed % 3]
    C = 3 if seed < 36 else (3, 7, 1, 5)[seed % 4]
    if seed % 4 != 3:
        return tuple(a[None] for a in adversarial_scene(seed, W=W, H=H, C=C))
    frames = [adversarial_scene(seed * 10 + k, W=W, H=H, C=C, F=150) for k in range(2)]
    F = max(fr[3].shape[0] for fr in frames)
    frames = [(bg, v, c, np.concatenate([f, np.zeros((F - f.shape[0], 3), np.int32)])) for bg, v, c, f in frames]
    V = max(fr[1].shape[0] for fr in frames)
    frames = [(bg, np.concatenate([v, np.tile(v[:1], (V - v.shape[0], 1))]),
               np.concatenate([c, np.tile(c[:1], (V - c.shape[0], 1))]), f) for bg, v, c, f in frames]
    return tuple(np.stack([fr[k] for fr in frames]) for k in range(4))


def clipped_sliver_scene(seed, W=48, H=40, C=3, n=10):
    """Faces that take the R5 clipping path and are slivers once clipped -- the case whose normalised pair
    weight (lambda = a / sum a, Wm = sum lambda w) cancels:
      * guard-band slivers: two vertices ~1000x the frame away along a line through it (clipped by the guard
        planes), the third 0.02..3 px off that line;
      * near-plane slivers: one vertex behind the eye (w < 0), the other two a fraction of a pixel apart;
      * a few ordinary faces in front of and behind them (occlusion boundaries), random depths."""
    rng = np.random.default_rng(seed)
    tris = []
    px2ndc = np.array([2.0 / W, 2.0 / H])
    for _ in range(n):
        kind = rng.integers(0, 3)
        z = rng.uniform(-0.8, 0.8)
        if kind == 0:
            p = rng.uniform(-0.8, 0.8, 2)
            a = rng.uniform(0, np.pi)
            d = np.array([np.cos(a), np.sin(a)])
            L = rng.uniform(800.0, 3000.0)
            off = np.array([-d[1], d[0]]) * px2ndc * rng.uniform(0.02, 3.0)
            q = p + rng.uniform(-0.5, 0.5) * d + off
            t = [[*(p - L * d), z, 1.0], [*(p + L * d), z, 1.0], [*q, z, 1.0]]
        elif kind == 1:
            p = rng.uniform(-0.8, 0.8, 2)
            e = rng.uniform(-1, 1, 2)
            e = e / np.linalg.norm(e) * px2ndc * rng.uniform(0.05, 0.8)
            wb = rng.uniform(-1.5, -0.05)
            back = rng.uniform(-1, 1, 2)
            w1, w2 = rng.uniform(0.5, 2.0, 2)
            t = [[back[0] * abs(wb), back[1] * abs(wb), z * abs(wb), wb],
                 [p[0] * w1, p[1] * w1, z * w1, w1], [(p[0] + e[0]) * w2, (p[1] + e[1]) * w2, z * w2, w2]]
        else:
            c = rng.uniform(-0.9, 0.9, 2)
            o = rng.uniform(-0.6, 0.6, size=(3, 2))
            t = [[*(c + oo), z, 1.0] for oo in o]
        tris.append(t)
    v = np.array(tris, np.float64).reshape(-1, 4).astype(np.float32)
    nf = len(tris)
    faces = np.arange(3 * nf, dtype=np.int32).reshape(nf, 3)
    cols = rng.uniform(0, 1, size=(3 * nf, C)).astype(np.float32)
    bg = rng.uniform(0, 1, size=(H, W, C)).astype(np.float32)
    return bg, v, cols, faces
