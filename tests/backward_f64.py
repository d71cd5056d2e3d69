"""Float64 restatement of the registered gradient.  TEST INFRASTRUCTURE ONLY.

An independent statement of the backward next to oracle/dirt_oracle.c (C, float32 contributions summed in
double) and the HIP kernel (float32, atomics): it is written from the specification, in the specification's
own terms, and shares no code or algebra with either --
  * geometry: R1/R2 snapping and R5 clipping (Sutherland-Hodgman against z >= -w and the guard planes, in
    float32, carrying the parent barycentric basis, fan-triangulated) define the rasterised (sub-)triangles,
    whose edge functions are Python integers (R3);
  * pair scalar: s = -0.5 sum_c (G_c(p) + G_c(q)) (I_c(q) - I_c(p)) for horizontally / vertically adjacent
    pixels p < q (window order), in float64; pairs touching a background pixel with a non-finite value carry
    nothing;
  * ownership: the common face; the only face if the other side is background; else the exact coverage tests
    covers(f, q) / covers(g, p) decide whose edge separates the pixels (weight 1), 0.5 / 0.5 when ambiguous;
  * weights: the owner's perspective-correct barycentrics at the pair midpoint M -- screen-space barycentrics
    b_k = E_k(M) / D of the record's snapped vertices, mu_k = (b_k / w_k) / sum_j (b_j / w_j) with the
    record's own clip w, mapped to the parent's vertices through the clip basis (identity for faces that did
    not take the clipping path): lambda_i = sum_k mu_k basis_ki; Wm = sum_k mu_k w_k, the clip w of M on the
    rasterised triangle;
  * chain rule through xw = (x / w + 1) W / 2: dL/dx_i += omega s (W/2) lambda_i / Wm and
    dL/dw_i -= omega s (W/2) lambda_i x_ndc(M) / Wm (x pairs; y pairs with H and y); dL/dz = 0;
  * colours: dL/dc_v += lambda_v(p) G(p) at the pixel centre of every covered pixel; dL/dbackground = G on
    uncovered pixels.
The visible record of each pixel (the forward's g-buffer) is an input: visibility is the forward's output,
pinned separately (tests/exact_cover.py, bit-exact GPU vs oracle).  Pure-Python loops: small frames only.
"""
import numpy as np

F32 = np.float32
GBUF_MULTI = 1 << 30
EXTRA_PER_FACE = 5


def _guard_clamp(xn, g):
    """R5 sub-vertex clamp: x/w of a clipped face's sub-vertex to [-g, g], NaN to g, g = twice the guard band
    (DESIGN.md 3, R5)."""
    return xn if xn <= g and xn >= -g else (-g if xn <= g else g)


def _snap(v4, W, H, clamp=None):
    """R1 + R2 in float32: snapped window coordinates (1/256 px) of one clip-space vertex (clamp: (2 gx, 2 gy)
    for a clipped face's sub-vertex)."""
    x, y, w = F32(v4[0]), F32(v4[1]), F32(v4[3])
    iw = F32(1.0) / w
    hw, hh = F32(0.5) * F32(W), F32(0.5) * F32(H)
    xn, yn = x * iw, y * iw
    if clamp is not None:
        xn, yn = _guard_clamp(xn, clamp[0]), _guard_clamp(yn, clamp[1])
    X = int(np.rint(((xn + F32(1.0)) * hw) * F32(256.0)))
    Y = int(np.rint(((yn + F32(1.0)) * hh) * F32(256.0)))
    return X, Y


class Tri:
    """One rasterised (sub-)triangle: integer edge functions E_k(P) = A_k Px + B_k Py + C_k (interior
    positive, P in 1/256 px), its vertices' clip w and their parent barycentric basis."""

    def __init__(self, verts7, W, H, clamp=None):
        X, Y = zip(*(_snap(p[:4], W, H, clamp) for p in verts7))
        A, B, C = [], [], []
        for k in range(3):
            a, b = (k + 1) % 3, (k + 2) % 3
            A.append(Y[a] - Y[b])
            B.append(X[b] - X[a])
            C.append(X[a] * Y[b] - X[b] * Y[a])
        D = A[0] * X[0] + B[0] * Y[0] + C[0]
        sg = 1 if D > 0 else -1
        self.A, self.B, self.C = [sg * a for a in A], [sg * b for b in B], [sg * c for c in C]
        self.D = sg * D
        self.w = [float(p[3]) for p in verts7]
        self.basis = [[float(p[4 + i]) for i in range(3)] for p in verts7]

    def E(self, px, py):
        return [self.A[k] * px + self.B[k] * py + self.C[k] for k in range(3)]

    def covers(self, i, j):
        """R3 at pixel centre (i, j) (window coordinates): E > 0, or E == 0 on a left / top edge."""
        E = self.E(256 * i + 128, 256 * j + 128)
        for k in range(3):
            if E[k] > 0:
                continue
            if E[k] == 0 and (self.A[k] > 0 or (self.A[k] == 0 and self.B[k] < 0)):
                continue
            return False
        return True

    def weights(self, E2):
        """Parent lambda_i and Wm at the point where the (doubled) edge values are E2 (sum = 2D)."""
        b = [e / (2.0 * self.D) for e in E2]
        q = [b[k] / self.w[k] for k in range(3)]
        sq = q[0] + q[1] + q[2]
        mu = [x / sq for x in q]
        lam = [sum(mu[k] * self.basis[k][i] for k in range(3)) for i in range(3)]
        Wm = sum(mu[k] * self.w[k] for k in range(3))
        return lam, Wm


CAP_CULLS = [0]  # faces culled by R5's vertex cap so far (tests)


def _plane(p, v, gx, gy):
    x, y, z, w = v[0], v[1], v[2], v[3]
    return (z + w, gx * w + x, gx * w - x, gy * w + y, gy * w - y)[p]


def setup_face(verts, face, V, W, H):
    """R5: the rasterised triangles of one face ([] = culled) and whether it took the clipping path."""
    if any(not 0 <= int(k) < V for k in face):
        return [], False
    v = [np.asarray(verts[int(k)], F32) for k in face]
    if not all(np.all(np.isfinite(p)) for p in v):
        return [], False
    gx, gy = F32(32768.0) / F32(W), F32(32768.0) / F32(H)
    if all(p[3] > 0 and abs(p[0]) <= gx * p[3] and abs(p[1]) <= gy * p[3] for p in v):
        poly = [np.concatenate([p, np.eye(3, dtype=F32)[k]]) for k, p in enumerate(v)]
        return [Tri(poly, W, H)], False
    poly = [np.concatenate([p, np.eye(3, dtype=F32)[k]]) for k, p in enumerate(v)]
    for pl in range(5):
        out = []
        n = len(poly)
        for i in range(n):
            a, c = poly[i], poly[(i + 1) % n]
            da, dc = _plane(pl, a, gx, gy), _plane(pl, c, gx, gy)
            if (da >= 0) + ((da >= 0) != (dc >= 0)) > 8 - len(out):  # R5 vertex cap: more than 8 culls the face
                CAP_CULLS[0] += 1
                return [], True
            if da >= 0:
                out.append(a)
            if (da >= 0) != (dc >= 0):
                t = da / (da - dc)
                out.append((a + t * (c - a)).astype(F32))
        poly = out
        if len(poly) < 3:
            return [], True
    if not all(p[3] > 0 for p in poly):
        return [], True
    tris = []
    for s in range(len(poly) - 2):
        t3 = [poly[0], poly[s + 1], poly[s + 2]]
        tri = Tri(t3, W, H, (F32(2.0) * gx, F32(2.0) * gy))
        tris.append(tri if tri.D != 0 else None)
    return tris, True


def _record(tris, F, ri):
    """The (sub-)triangle of record index ri: sub-triangle 0 of face f is record f, sub-triangle s > 0 is
    record F + 5 f + s - 1 (the g-buffer's numbering)."""
    if ri < F:
        return ri, tris[ri][0][0]
    d = ri - F
    f = d // EXTRA_PER_FACE
    return f, tris[f][0][d - f * EXTRA_PER_FACE + 1]


def backward(vertices, faces, pixels, grad_pixels, gbuffer):
    """One frame: vertices [V,4], faces [F,3], pixels / grad_pixels [H,W,C] (rows top first), gbuffer [H,W]
    (visible record, bit 30 = clipped face, -1 background).  Returns float64 (grad_vertices [V,4],
    grad_vertex_colors [V,C], grad_background [H,W,C])."""
    H, W, C = pixels.shape
    V, F = vertices.shape[0], faces.shape[0]
    tris = [setup_face(vertices, faces[f], V, W, H) for f in range(F)]
    I = pixels.astype(np.float64)
    G = grad_pixels.astype(np.float64)
    gv = np.zeros((V, 4))
    gc = np.zeros((V, C))
    gbg = np.zeros((H, W, C))
    rec = np.where(gbuffer < 0, -1, gbuffer & (GBUF_MULTI - 1))

    def at(i, j):  # window (i, j) -> image row
        return H - 1 - j, i

    def face_covers(f, i, j):
        return any(t is not None and t.covers(i, j) for t in tris[f][0])

    for j in range(H):
        for i in range(W):
            r = rec[at(i, j)]
            if r < 0:
                gbg[at(i, j)] = G[at(i, j)]
                continue
            f, t = _record(tris, F, int(r))
            lam, _ = t.weights([2 * e for e in t.E(256 * i + 128, 256 * j + 128)])
            for k in range(3):
                gc[faces[f][k]] += lam[k] * G[at(i, j)]

    def add(ri, i, j, axis, s, omega):
        f, t = _record(tris, F, int(ri))
        if axis == 0:
            E2 = [t.A[k] * (512 * i + 512) + t.B[k] * (512 * j + 256) + 2 * t.C[k] for k in range(3)]
            half, ndc = W / 2.0, (i + 1) / (W / 2.0) - 1.0
        else:
            E2 = [t.A[k] * (512 * i + 256) + t.B[k] * (512 * j + 512) + 2 * t.C[k] for k in range(3)]
            half, ndc = H / 2.0, (j + 1) / (H / 2.0) - 1.0
        lam, Wm = t.weights(E2)
        for k in range(3):
            g = omega * s * half * lam[k] / Wm
            gv[faces[f][k], axis] += g
            gv[faces[f][k], 3] -= g * ndc

    for j in range(H):
        for i in range(W):
            for axis in (0, 1):
                i2, j2 = (i + 1, j) if axis == 0 else (i, j + 1)
                if i2 >= W or j2 >= H:
                    continue
                rp, rq = int(rec[at(i, j)]), int(rec[at(i2, j2)])
                if rp < 0 and rq < 0:
                    continue
                Ip, Iq = I[at(i, j)], I[at(i2, j2)]
                if (rp < 0 and not np.all(np.isfinite(Ip))) or (rq < 0 and not np.all(np.isfinite(Iq))):
                    continue
                s = -0.5 * float(np.sum((G[at(i, j)] + G[at(i2, j2)]) * (Iq - Ip)))
                if s == 0.0:
                    continue
                fp = _record(tris, F, rp)[0] if rp >= 0 else -1
                fq = _record(tris, F, rq)[0] if rq >= 0 else -1
                if fp == fq or fq < 0:
                    add(rp, i, j, axis, s, 1.0)
                elif fp < 0:
                    add(rq, i, j, axis, s, 1.0)
                else:
                    p_covers_q, q_covers_p = face_covers(fp, i2, j2), face_covers(fq, i, j)
                    if not p_covers_q and q_covers_p:
                        add(rp, i, j, axis, s, 1.0)
                    elif p_covers_q and not q_covers_p:
                        add(rq, i, j, axis, s, 1.0)
                    else:
                        add(rp, i, j, axis, s, 0.5)
                        add(rq, i, j, axis, s, 0.5)
    return gv, gc, gbg


def backward_batch(vertices, faces, pixels, grad_pixels, gbuffer):
    outs = [backward(vertices[b], faces[b], pixels[b], grad_pixels[b], gbuffer[b]) for b in range(pixels.shape[0])]
    return tuple(np.stack([o[k] for o in outs]) for k in range(3))


def max_rel_err(approx, exact):
    """max |approx - exact| / max |exact| (the gradient's scale)."""
    scale = float(np.max(np.abs(exact))) if exact.size else 0.0
    if scale == 0.0:
        return float(np.max(np.abs(approx))) if approx.size else 0.0
    return float(np.max(np.abs(approx.astype(np.float64) - exact))) / scale

