"""Exact-integer restatement of the coverage rule (R1/R2 snapping in numpy float32, R3 edge functions and the
top-left rule on Python ints) and watertight test meshes.  Test infrastructure: a third, independent
statement of DESIGN.md 3's coverage next to the C oracle and the HIP kernels (used by tests/test_oracle.py
on the CPU and tests/test_gpu_analytic.py on the GPU)."""
import numpy as np

F32 = np.float32


def snap(v, W, H):
    """R1 + R2 (raster_rules.h make_record) in float32: snapped window coordinates in 1/256 px, as Python ints."""
    v = v.astype(F32)
    iw = F32(1.0) / v[:, 3]
    xn, yn = v[:, 0] * iw, v[:, 1] * iw
    hw, hh = F32(0.5) * F32(W), F32(0.5) * F32(H)
    X = np.rint(((xn + F32(1.0)) * hw) * F32(256.0)).astype(np.int64)
    Y = np.rint(((yn + F32(1.0)) * hh) * F32(256.0)).astype(np.int64)
    return X, Y


def exact_cover(v, faces, W, H):
    """[H, W] count of faces whose snapped triangle contains each pixel centre (R3, exact integers, top-left
    rule: E > 0, or E == 0 on a left (A > 0) or top (A == 0, B < 0) edge) and the lowest such face (-1 none).
    Rows top first, as the op's outputs."""
    X, Y = snap(v, W, H)
    px = (np.arange(W, dtype=np.int64) * 256 + 128)[None, :]
    py = (np.arange(H, dtype=np.int64) * 256 + 128)[:, None]
    count = np.zeros((H, W), np.int64)
    first = np.full((H, W), -1, np.int64)
    for f, (a, b, c) in enumerate(faces):
        xs, ys = [int(X[a]), int(X[b]), int(X[c])], [int(Y[a]), int(Y[b]), int(Y[c])]
        A = [ys[(k + 1) % 3] - ys[(k + 2) % 3] for k in range(3)]
        Bc = [xs[(k + 2) % 3] - xs[(k + 1) % 3] for k in range(3)]
        Cc = [xs[(k + 1) % 3] * ys[(k + 2) % 3] - xs[(k + 2) % 3] * ys[(k + 1) % 3] for k in range(3)]
        D = A[0] * xs[0] + Bc[0] * ys[0] + Cc[0]
        if D == 0:
            continue  # degenerate: dropped (R3)
        s = 1 if D > 0 else -1
        inside = np.ones((H, W), bool)
        for k in range(3):
            a_, b_, c_ = s * A[k], s * Bc[k], s * Cc[k]
            E = a_ * px + b_ * py + c_  # int64: |X|, |Y| < 2^18 here, products < 2^37
            owned = a_ > 0 or (a_ == 0 and b_ < 0)
            inside &= (E > 0) | ((E == 0) & owned)
        inside = inside[::-1]  # window j (from the bottom) -> image row
        first[(first < 0) & inside] = f
        count += inside
    return count, first


def grid_mesh(nx, ny, W, H, seed, perspective=False, centre_snap=False):
    """A watertight mesh over [-0.9, 0.9]^2: (nx+1) x (ny+1) shared vertices, interior ones jittered by up to
    0.25 cell (no fold), two triangles per cell with a random diagonal.  centre_snap: interior vertices moved onto pixel
    centres, so that edges run through pixel centres (E == 0 ties decided by the top-left rule)."""
    rng = np.random.default_rng(seed)
    gx, gy = np.meshgrid(np.linspace(-0.9, 0.9, nx + 1), np.linspace(-0.9, 0.9, ny + 1))
    cx, cy = 1.8 / nx, 1.8 / ny
    inner = np.zeros_like(gx, bool)
    inner[1:-1, 1:-1] = True
    gx = gx + inner * rng.uniform(-0.25, 0.25, gx.shape) * cx
    gy = gy + inner * rng.uniform(-0.25, 0.25, gy.shape) * cy
    if centre_snap:
        # NDC of pixel centre i: (i + 0.5) * 2 / W - 1
        ix = np.floor((gx + 1) * W / 2)
        iy = np.floor((gy + 1) * H / 2)
        gx = np.where(inner, (ix + 0.5) * 2.0 / W - 1.0, gx)
        gy = np.where(inner, (iy + 0.5) * 2.0 / H - 1.0, gy)
    n = (nx + 1) * (ny + 1)
    v = np.stack([gx.ravel(), gy.ravel(), np.full(n, 0.25), np.ones(n)], 1)
    if perspective:
        v = v * rng.uniform(1.0, 3.0, size=(n, 1))
    faces = []
    for j in range(ny):
        for i in range(nx):
            p00, p10 = j * (nx + 1) + i, j * (nx + 1) + i + 1
            p01, p11 = p00 + nx + 1, p10 + nx + 1
            if rng.uniform() < 0.5:
                faces += [(p00, p10, p11), (p00, p11, p01)]
            else:
                faces += [(p00, p10, p01), (p10, p11, p01)]
    faces = np.array(faces, np.int32)
    rng.shuffle(faces)  # draw order unrelated to position
    return v.astype(F32), faces
