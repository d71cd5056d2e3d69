"""float64 numpy restatement of the fork's `oceanic_horizon` fragment program (csrc/shaders.cpp:1668-1919),
vectorised over pixels.  TEST INFRASTRUCTURE: it pins the oracle's fixed float32 sin/cos/pow algorithms
against real math (numpy float64), it is never the thing measured or shipped."""
import numpy as np


def water(px, py, time):
    shift2x = 0.001 * (time * 190.0 * 2.0)
    wave = np.sin(px * 0.021 + shift2x) * 4.5
    wave = wave + np.sin(px * 0.0172 + py * 0.010 + shift2x * 1.121) * 4.0
    wave = wave - np.sin(px * 0.00104 + py * 0.005 + shift2x * 0.121) * 4.0
    wave = wave + np.sin(px * 0.02221 + py * 0.01233 + shift2x * 3.437) * 5.0
    wave = wave + np.sin(px * 0.03112 + py * 0.01122 + shift2x * 4.269) * 2.5
    return 70.0 + wave


def trace(ro, rd, time):
    with np.errstate(divide="ignore", invalid="ignore"):
        t = -ro[1] / rd[1]
    st = np.full_like(t, 0.5)
    old_h = np.zeros_like(t)
    for _ in range(20):
        st = np.where(t > 500.0, 1.0, st)
        st = np.where(t > 800.0, 2.0, st)
        st = np.where(t > 1500.0, 3.0, st)
        p0, p1, p2 = ro[0] + t * rd[0], ro[1] + t * rd[1], ro[2] + t * rd[2]
        h = p1 - water(p0, p2, time)
        t = t + np.maximum(1.0, np.abs(h)) * np.sign(h) * st
        st = np.where(old_h * h < 0.0, st / 2.0, st)
        old_h = h
    return t, ~(rd[1] > 0.0)


def shade(xy_x, xy_y, cam, width, height):
    """(col.x, col.y) for arrays of jittered texCoordV."""
    cam = np.asarray(cam, np.float64)
    light = np.array([0.1, 0.25, cam[7]])
    light = light / np.sqrt(light @ light)
    rdv = np.stack([(xy_x + 1.0) * width / 2.0 - width / 2.0, (xy_y + 1.0) * height / 2.0 - height / 2.0,
                    np.full_like(xy_x, 1.73 * width / 2.0)])
    rdv = rdv / np.sqrt((rdv * rdv).sum(0))
    s1, c1, s2, c2, s3, c3 = np.sin(cam[3]), np.cos(cam[3]), np.sin(cam[4]), np.cos(cam[4]), np.sin(cam[5]), np.cos(cam[5])
    rd = np.stack([c2 * c3 * rdv[0] + (-c1 * s3 + s1 * s2 * c3) * rdv[1] + (s1 * s3 + c1 * s2 * c3) * rdv[2],
                   c2 * s3 * rdv[0] + (c1 * c3 + s1 * s2 * s3) * rdv[1] + (-s1 * c3 + c1 * s2 * s3) * rdv[2],
                   -s2 * rdv[0] + s1 * c2 * rdv[1] + c1 * c2 * rdv[2]])
    ro = cam[:3].reshape(3, 1) * np.ones_like(rd)
    time = cam[6]
    sundot = np.clip((rd * light[:, None]).sum(0), 0.0, 1.0)
    dist, hit = trace(ro, rd, time)
    col0 = np.where(hit, 0.0, 1.0)
    sky = np.power(sundot, 350.0)
    wx, wz = ro[0] + dist * rd[0], ro[2] + dist * rd[2]
    d = 0.4
    n = np.stack([water(wx - d, wz, time) - water(wx + d, wz, time), np.ones_like(wx),
                  water(wx, wz - d, time) - water(wx, wz + d, time)])
    n = n / np.sqrt((n * n).sum(0))
    rr = rd - 2.0 * (n * rd).sum(0) * n
    sd = np.clip((rr * light[:, None]).sum(0), 0.0, 1.0)
    refl = 0.5 * sd ** 10.0 + 0.25 * sd ** 3.5 + 0.75 * sd ** 300.0
    return col0, np.where(hit, refl, sky), rd


def render_fullscreen(H, W, cam, background=None):
    """The harness of tests/optimize_horizon.py:251-268: full-screen quad, w = 1, so texCoordV is the
    pixel centre in NDC; returns [H, W, 2] (rows top first) and the ray y component."""
    j = np.arange(H, dtype=np.float64)[:, None] * np.ones((1, W))
    i = np.arange(W, dtype=np.float64)[None, :] * np.ones((H, 1))
    tx = (i + 0.5) / W * 2.0 - 1.0
    ty = (j + 0.5) / H * 2.0 - 1.0
    if background is not None:
        bg = np.asarray(background, np.float64)[::-1]  # window rows bottom first
        tx = tx + bg[..., 0] / W
        ty = ty + (bg[..., 1] if bg.shape[-1] > 1 else bg[..., 0]) / H
    c0, c1, rd = shade(tx.ravel(), ty.ravel(), cam, float(W), float(H))
    out = np.stack([c0.reshape(H, W), c1.reshape(H, W)], -1)[::-1]
    return out, rd[1].reshape(H, W)[::-1]


# ---- the oceanic family (shaders.cpp:556-1176, 1402-1666, 1921-2185), float64 -------------------------
FAMILY = {
    2: dict(wavegain=1.0, large=1.0, small=1.0, fog=(0.5, 0.7, 1.1), skybottom=(0.6, 0.8, 1.2), skytop=(0.05, 0.2, 0.5),
            reflsky=(0.025, 0.10, 0.20), water=(0.2, 0.25, 0.3), s1=(160.0, 120.0), s2=(190.0, 130.0), cos=False,
            iters=7, steps=20, clouds=1),
    3: dict(wavegain=1.0, large=1.0, small=1.0, fog=(0.5, 0.7, 1.1), skybottom=(0.6, 0.8, 1.2), skytop=(0.05, 0.2, 0.5),
            reflsky=(0.025, 0.10, 0.20), water=(0.2, 0.25, 0.3), s1=(160.0, 120.0), s2=(190.0, 130.0), cos=False,
            iters=7, steps=20, clouds=2),
    4: dict(wavegain=1.0, large=1.0, small=1.0, fog=(0.5, 0.7, 1.1), skybottom=(0.6, 0.8, 1.2), skytop=(0.05, 0.2, 0.5),
            reflsky=(0.025, 0.10, 0.20), water=(0.2, 0.25, 0.3), s1=(160.0, 120.0), s2=(190.0, 130.0), cos=False,
            iters=7, steps=20, clouds=0),
    5: dict(wavegain=0.75, large=0.75, small=1.5, fog=(0.4, 0.4, 1.2), skybottom=(0.5, 0.5, 1.3), skytop=(0.15, 0.1, 0.7),
            reflsky=(0.1, 0.1, 0.15), water=(0.1, 0.2, 0.5), s1=(260.0, 100.0), s2=(150.0, 230.0), cos=True,
            iters=3, steps=10, clouds=0),
}


def _fract(x):
    return x - np.floor(x)


def _mix(a, b, t):
    return a * (1.0 - t) + b * t


def _smooth(e0, e1, x):
    t = np.clip((x - e0) / (e1 - e0), 0.0, 1.0)
    return t * t * (3.0 - 2.0 * t)


def _hash(n):
    return _fract(np.cos(n) * 41415.92653)


def _rand2(x, y):
    return _fract(np.sin(x * 12.9898 + y * 4.1414) * 43758.5453)


def _noise2(x, y):
    ix, iy = np.floor(x), np.floor(y)
    ux, uy = _fract(x), _fract(y)
    ux, uy = ux * ux * (3 - 2 * ux), uy * uy * (3 - 2 * uy)
    return _mix(_mix(_rand2(ix, iy), _rand2(ix + 1, iy), ux), _mix(_rand2(ix, iy + 1), _rand2(ix + 1, iy + 1), ux), uy)


def _noise3(x, y, z):
    px, py, pz = np.floor(x), np.floor(y), np.floor(z)
    fx, fy, fz = _smooth(0, 1, _fract(x)), _smooth(0, 1, _fract(y)), _smooth(0, 1, _fract(z))
    n = px + py * 57.0 + 113.0 * pz
    return _mix(_mix(_mix(_hash(n), _hash(n + 1), fx), _mix(_hash(n + 57), _hash(n + 58), fx), fy),
                _mix(_mix(_hash(n + 113), _hash(n + 114), fx), _mix(_hash(n + 170), _hash(n + 171), fx), fy), fz)


def _fbm3(x, y, z):
    def m(x, y, z):
        return -1.6 * y - 1.2 * z, 1.6 * x + 0.72 * y - 0.96 * z, 1.2 * x - 0.96 * y + 1.28 * z
    f = 0.5 * _noise3(x, y, z)
    x, y, z = (v * 1.1 for v in m(x, y, z))
    f = f + 0.25 * _noise3(x, y, z)
    x, y, z = (v * 1.2 for v in m(x, y, z))
    f = f + 0.1666 * _noise3(x, y, z)
    x, y, z = m(x, y, z)
    return f + 0.0834 * _noise3(x, y, z)


def _fbm2(x, y):
    f = 0.5 * _noise2(x, y)
    for c in (0.25, 0.1666, 0.0834):
        x, y = 1.6 * x + 1.2 * y, -1.2 * x + 1.6 * y
        f = f + c * _noise2(x, y)
    return f


def _water_family(P, px, py, time):
    s1x, s1y = 0.001 * time * P["s1"][0] * 2.0, 0.001 * time * P["s1"][1] * 2.0
    s2x, s2y = 0.001 * time * P["s2"][0] * 2.0, -0.001 * time * P["s2"][1] * 2.0
    fn = np.cos if P["cos"] else np.sin
    wave = fn(px * 0.021 + s2x) * 4.5 + fn(px * 0.0172 + py * 0.010 + s2x * 1.121) * 4.0
    wave = wave - fn(px * 0.00104 + py * 0.005 + s2x * 0.121) * 4.0
    wave = wave + fn(px * 0.02221 + py * 0.01233 + s2x * 3.437) * 5.0 + fn(px * 0.03112 + py * 0.01122 + s2x * 4.269) * 2.5
    wave = wave * P["large"] - _fbm2(px * 0.004 - s2x * 0.5, py * 0.004 - s2y * 0.5) * P["small"] * 24.0
    amp = 6.0 * P["small"]
    s1x, s1y = s1x * 0.3, s1y * 0.3
    for _ in range(P["iters"]):
        wave = wave - np.abs(np.sin((_noise2(px * 0.01 + s1x, py * 0.01 + s1y) - 0.5) * 3.14)) * amp
        amp *= 0.51
        s1x, s1y = s1x * 1.841, s1y * 1.841
        px, py = px * 1.6 * 0.9331 - py * 1.2 * 0.9331, px * 1.2 * 0.9331 + py * 1.6 * 0.9331
    return 70.0 + wave


def _cloud_pos(P, ro, c, rd, q3, shx, shy):
    if P["clouds"] == 1:
        base = [ro[k] + c * rd[k] for k in range(3)]
    else:
        base = [c * rd[k] for k in range(3)]
    return base[0] + 831.0, base[1] + 321.0 + q3 - shx * 0.2, base[2] + 1330.0 + shy * 3.0


def shade_family(sid, xy_x, xy_y, cam, width, height):
    P = FAMILY[sid]
    cam = np.asarray(cam, np.float64)
    light = np.array([0.1, 0.25, cam[7]])
    light = light / np.sqrt(light @ light)
    rdv = np.stack([(xy_x + 1.0) * width / 2.0 - width / 2.0, (xy_y + 1.0) * height / 2.0 - height / 2.0,
                    np.full_like(xy_x, 1.73 * width / 2.0)])
    rdv = rdv / np.sqrt((rdv * rdv).sum(0))
    s1, c1, s2, c2, s3, c3 = np.sin(cam[3]), np.cos(cam[3]), np.sin(cam[4]), np.cos(cam[4]), np.sin(cam[5]), np.cos(cam[5])
    rd = np.stack([c2 * c3 * rdv[0] + (-c1 * s3 + s1 * s2 * c3) * rdv[1] + (s1 * s3 + c1 * s2 * c3) * rdv[2],
                   c2 * s3 * rdv[0] + (c1 * c3 + s1 * s2 * s3) * rdv[1] + (-s1 * c3 + c1 * s2 * s3) * rdv[2],
                   -s2 * rdv[0] + s1 * c2 * rdv[1] + c1 * c2 * rdv[2]])
    ro = cam[:3]
    time = cam[6]
    ct = cam[8] if P["clouds"] == 2 else time
    shx, shy = ct * 80.0, ct * 60.0
    sundot = np.clip((rd * light[:, None]).sum(0), 0.0, 1.0)
    out = np.zeros((3, rd.shape[1]))
    sky = rd[1] > 0
    with np.errstate(all="ignore"):
        # sky
        t = (1.0 - 0.7 * rd[1]) ** 15.0
        col = [0.8 * (P["skybottom"][k] * t + P["skytop"][k] * (1 - t)) + 0.47 * (1.6, 1.4, 1.0)[k] * sundot ** 350.0
               + 0.4 * (0.8, 0.9, 1.0)[k] * sundot ** 2.0 for k in range(3)]
        if P["clouds"]:
            sm = np.zeros((4, rd.shape[1]))
            active = sky.copy()
            for q in range(100):
                base = 350.0 + q * 12.0
                c = ((base - cam[1]) if P["clouds"] == 1 else base) / rd[1]
                cx, cy, cz = _cloud_pos(P, ro, c, rd, q * 0.15, shx, shy)
                alpha = _smooth(0.5, 1.0, _fbm3(cx * 0.0015, cy * 0.0015, cz * 0.0015)) * 0.9
                lc = [_mix((1.1, 1.05, 1.0)[k], 0.7 * (0.4, 0.4, 0.3)[k], alpha) for k in range(3)]
                alpha = np.where(active, (1.0 - sm[3]) * alpha, 0.0)
                for k in range(3):
                    sm[k] += lc[k] * alpha
                sm[3] += alpha
                active &= ~(sm[3] > 0.98)
            a = _smooth(0.7, 1.0, sm[3])
            for k in range(3):
                v = sm[k] / (sm[3] + 0.0001) - 0.6 * (0.8, 0.75, 0.7)[k] * sundot ** 13.0 * a \
                    + 0.2 * (1.3, 1.2, 1.0)[k] * sundot ** 5.0 * (1.0 - a)
                col[k] = _mix(col[k], v, sm[3] * (1.0 - t))
        for k in range(3):
            out[k] = np.where(sky, col[k], 0.0)
        # water
        t = -ro[1] / rd[1]
        st = np.full_like(t, 0.5)
        old = np.zeros_like(t)
        for _ in range(P["steps"]):
            st = np.where(t > 500, 1.0, st)
            st = np.where(t > 800, 2.0, st)
            st = np.where(t > 1500, 3.0, st)
            h = ro[1] + t * rd[1] - _water_family(P, ro[0] + t * rd[0], ro[2] + t * rd[2], time)
            t = t + np.maximum(1.0, np.abs(h)) * np.sign(h) * st
            st = np.where(old * h < 0, st / 2.0, st)
            old = h
        dist = t
        w = [ro[k] + dist * rd[k] for k in range(3)]
        d = 0.1 * P["wavegain"] * 4.0
        n = np.stack([_water_family(P, w[0] - d, w[2], time) - _water_family(P, w[0] + d, w[2], time), np.ones_like(dist),
                      _water_family(P, w[0], w[2] - d, time) - _water_family(P, w[0], w[2] + d, time)])
        n = n / np.sqrt((n * n).sum(0))
        rr = rd - 2.0 * (n * rd).sum(0) * n
        refl = 1.0 - np.clip(rr[1], 0.0, 1.0)
        if P["clouds"]:
            fro = [w[k] + 20.0 * rr[k] for k in range(3)]
            s = np.zeros_like(dist)
            active = ~sky
            for q in range(10):
                base = 350.0 + q * 120.0
                c = ((base - fro[1]) if P["clouds"] == 1 else base) / rr[1]
                cx, cy, cz = _cloud_pos(P, fro, c, rr, q * 0.15, shx, shy)
                alpha = _smooth(0.5, 1.0, _fbm3(cx * 0.0015, cy * 0.0015, cz * 0.0015))
                s = np.where(active, s + (1.0 - s) * alpha, s)
                active &= ~(s > 0.98)
            fogv = np.clip(1.0 - s, 0.0, 1.0)
        else:
            fogv = np.ones_like(dist)
        sh = _smooth(0.2, 1.0, fogv) * 0.7 + 0.3
        wsky, wwat = refl * sh, (1.0 - refl) * sh
        sd = np.clip((rr * light[:, None]).sum(0), 0.0, 1.0)
        wsun = wsky * (0.5 * sd ** 10.0 + 0.25 * sd ** 3.5 + 0.75 * sd ** 300.0)
        fo = 1.0 - np.exp(-np.maximum(0.0003 * dist, 0.0) ** 1.5)
        for k in range(3):
            cw = wsky * P["reflsky"][k] + wwat * P["water"][k] + (0.003, 0.005, 0.005)[k] * (w[1] - 70.0 + 30.0) \
                + (1.5, 1.3, 1.0)[k] * wsun
            out[k] = np.where(sky, out[k], _mix(cw, P["fog"][k] + 0.6 * (0.6, 0.5, 0.4)[k] * sd ** 4.0, fo))
    return out, rd


def render_family_fullscreen(sid, H, W, cam):
    j = np.arange(H, dtype=np.float64)[:, None] * np.ones((1, W))
    i = np.arange(W, dtype=np.float64)[None, :] * np.ones((H, 1))
    tx = (i + 0.5) / W * 2.0 - 1.0
    ty = (j + 0.5) / H * 2.0 - 1.0
    out, rd = shade_family(sid, tx.ravel(), ty.ravel(), cam, float(W), float(H))
    return np.moveaxis(out.reshape(3, H, W), 0, -1)[::-1], rd[1].reshape(H, W)[::-1]


# ---- oceanic_opt_flow (shaders.cpp:1178-1398), float64 --------------------------------------------------
def _rot(cam3, cam4, cam5):
    s1, c1, s2, c2, s3, c3 = np.sin(cam3), np.cos(cam3), np.sin(cam4), np.cos(cam4), np.sin(cam5), np.cos(cam5)
    # rows: ray_dir_p = R @ ray_dir (shaders.cpp:1330-1333)
    return np.array([[c2 * c3, -c1 * s3 + s1 * s2 * c3, s1 * s3 + c1 * s2 * c3],
                     [c2 * s3, c1 * c3 + s1 * s2 * s3, -s1 * c3 + c1 * s2 * s3],
                     [-s2, s1 * c2, c1 * c2]])


def opt_flow(tx, ty, cam, width, height):
    """new_coord for arrays of texCoordV (no jitter); cam: 16 floats (oceanic_opt_flow.cpp:399-414)."""
    cam = np.asarray(cam, np.float64)
    dt = cam[9]
    rdv = np.stack([(tx + 1.0) * width / 2.0 - width / 2.0, (ty + 1.0) * height / 2.0 - height / 2.0,
                    np.full_like(tx, 1.73 * width / 2.0)])
    rdv = rdv / np.sqrt((rdv * rdv).sum(0))
    rd = _rot(cam[3], cam[4], cam[5]) @ rdv
    with np.errstate(divide="ignore", invalid="ignore"):
        t = -cam[1] / rd[1]
    st = np.full_like(t, 0.5)
    old_h = np.zeros_like(t)
    for _ in range(20):
        st = np.where(t > 500.0, 1.0, st)
        st = np.where(t > 800.0, 2.0, st)
        st = np.where(t > 1500.0, 3.0, st)
        h = cam[1] + t * rd[1] - 58.0
        t = t + np.maximum(1.0, np.abs(h)) * np.sign(h) * st
        st = np.where(old_h * h < 0.0, st / 2.0, st)
        old_h = h
    wpos = cam[:3, None] + t * rd
    old_rd = np.where(rd[1] > 0.0, rd, wpos - (cam[:3] - cam[10:13] * dt)[:, None])
    o = _rot(cam[3] - cam[13] * dt, cam[4] - cam[14] * dt, cam[5] - cam[15] * dt).T @ old_rd
    o = o / o[2] * (1.73 * width / 2.0)
    return o[0] + width / 2.0, o[1] + height / 2.0, rd


def render_opt_flow_fullscreen(H, W, cam):
    j = np.arange(H, dtype=np.float64)[:, None] * np.ones((1, W))
    i = np.arange(W, dtype=np.float64)[None, :] * np.ones((H, 1))
    tx = (i + 0.5) / W * 2.0 - 1.0
    ty = (j + 0.5) / H * 2.0 - 1.0
    x, y, rd = opt_flow(tx.ravel(), ty.ravel(), cam, float(W), float(H))
    return np.stack([x.reshape(H, W), y.reshape(H, W)], -1)[::-1], rd[1].reshape(H, W)[::-1]


# ---- hill (shaders.cpp:123-554), float64 ---------------------------------------------------------------
def _hill_sample(T, u, v, ch):
    """GL_LINEAR / CLAMP_TO_EDGE lookup of channel(s) ch of a [H, W, 4] texel array (GL rows bottom first)."""
    H, W = T.shape[:2]
    x, y = u * W - 0.5, v * H - 0.5
    fx, fy = np.floor(x), np.floor(y)
    a, b = (x - fx)[..., None], (y - fy)[..., None]
    i0, j0 = fx.astype(np.int64), fy.astype(np.int64)

    def tx(i, j):
        return T[np.clip(j, 0, H - 1), np.clip(i, 0, W - 1)][..., ch]
    r0 = tx(i0, j0) * (1 - a) + tx(i0 + 1, j0) * a
    r1 = tx(i0, j0 + 1) * (1 - a) + tx(i0 + 1, j0 + 1) * a
    return r0 * (1 - b) + r1 * b


def _hill_uv(px, pz):
    return np.clip((pz - 5.0) / 20.0, 0, 1), np.clip((px + 14.0) / 28.0, 0, 1)


def _hill_terrain(T, px, pz):
    u, v = _hill_uv(px, pz)
    return _hill_sample(T, u, v, [0])[..., 0] * 10.3 - 6.1


def _hill_hash1(p):
    x, y = _fract(p / 3.07965), _fract(p / 7.4235)
    d = y * (x + 19.19) + x * (y + 19.19)
    return _fract((x + d) * (y + d))


def _hill_hash2(px, py):
    x, y = _fract(px / 3.07965), _fract(py / 7.4235)
    d = x * (y + 19.19) + y * (x + 19.19)
    return _fract((x + d) * (y + d))


def _hill_noise(x, y):
    px, py = np.floor(x), np.floor(y)
    fx, fy = _fract(x), _fract(y)
    fx, fy = fx * fx * (3 - 2 * fx), fy * fy * (3 - 2 * fy)
    n = px + py * 57.0
    return _mix(_mix(_hill_hash1(n), _hill_hash1(n + 1), fx), _mix(_hill_hash1(n + 57), _hill_hash1(n + 58), fx), fy)


def _hill_voronoi(x, y):
    px, py = np.floor(x), np.floor(y)
    fx, fy = _fract(x), _fract(y)
    res, idv = np.full_like(x, 100.0), np.zeros_like(x)
    for j in (-1, 0, 1):
        for i in (-1, 0, 1):
            h = _hill_hash2(px + i, py + j)
            d = (i - fx + h) ** 2 + (j - fy + h) ** 2
            better = d < res
            res, idv = np.where(better, d, res), np.where(better, h, idv)
    return np.maximum(0.4 - np.sqrt(res), 0.0), idv


def _hill_de(T, px, py, pz):
    base = _hill_terrain(T, px, pz) - 1.3
    qx, qz = px * 4.0, pz * 4.0
    height = _hill_noise(qx * 2, qz * 2) * 0.75 + _hill_noise(qx, qz) * 0.35 + _hill_noise(qx * 0.5, qz * 0.5) * 0.2
    y = (py - base - height) ** 2
    ax = qx * 2.5 + np.sin(y * 4.0 + qz * 12.3) * 0.12 + np.sin(1.5 * qz) * y * 0.5
    ay = qz * 2.5 + np.sin(y * 4.0 + qx * 12.3) * 0.12 + np.sin(1.5 * qx) * y * 0.5
    vx, vid = _hill_voronoi(ax, ay)
    f = vx * 0.6 + y * 0.58
    return y - f * 1.4, np.clip(f * 1.5, 0, 1), vid


def _hill_sky(rd, sun):
    amt = np.maximum((rd * sun[:, None]).sum(0), 0.0)
    v = (1.0 - np.maximum(rd[1], 0.0)) ** 6.0
    sunc = np.array([1.0, 0.75, 0.6])[:, None]
    sky = _mix(np.array([0.1, 0.2, 0.3])[:, None], 0.32, v) + sunc * amt * amt * 0.25
    sky = sky + sunc * np.minimum(amt ** 800.0 * 1.5, 0.3)
    return np.clip(sky, 0, 1)


def hill(tex, tx, ty, cam):
    """fragColor [4, n] for arrays of texCoordV over a terrain lookup [H, W, Ct] (rows top first)."""
    with np.errstate(all="ignore"):  # far grass samples overflow (y*y), as in float32
        return _hill(tex, tx, ty, cam)


def _hill(tex, tx, ty, cam):
    tex = np.asarray(tex, np.float64)
    H, W, Ct = tex.shape
    T = np.ones((H, W, 4))
    if Ct == 1:
        T[..., :3] = tex[..., :1]
    else:
        T[..., :Ct] = tex
    T = T[::-1]  # GL rows bottom first
    width, height = float(W), float(H)
    cam = np.asarray(cam, np.float64)
    xyx, xyy = (tx + 1) / 2, (-ty + 1) / 2
    box = np.abs(xyy * height - height / 2) / (width / 2) >= 0.5625
    sun = np.array([0.35, 0.2, 0.3])
    sun = sun / np.sqrt(sun @ sun)
    rv = np.stack([xyx * width - width / 2, xyy * height - height / 2, np.full_like(xyx, 0.85 * width)])
    rv = rv / np.sqrt((rv * rv).sum(0))
    R = np.array([[0.999999573, -0.0000933038802, 0.000919791287], [0.000918443273, -0.0135434586, -0.999907861],
                  [0.000105752439, 0.999908279, -0.0135433672]])  # [r_row][col]
    d = np.stack([-(R[0, 0] * rv[0] + R[1, 0] * rv[1] + R[2, 0] * rv[2]),
                  R[0, 2] * rv[0] + R[1, 2] * rv[1] + R[2, 2] * rv[2],
                  R[0, 1] * rv[0] + R[1, 1] * rv[1] + R[2, 1] * rv[2]])
    ro = np.array([-cam[9], cam[11], cam[10]])
    with np.errstate(divide="ignore", invalid="ignore"):
        t = -(ro[1] + 1.0) / d[1]
    t = np.where(d[1] > -0.015, 80.0, t)
    t_inc, st, old_h, h = np.zeros_like(t), np.ones_like(t), np.zeros_like(t), np.zeros_like(t)
    for _ in range(100):
        t = t + t_inc
        p = ro[:, None] + t * d
        h = p[1] - _hill_terrain(T, p[0], p[2])
        t_inc = np.maximum(1.0, np.abs(h)) * np.sign(h) * st
        st = np.where(h * old_h < 0, st / 2, st)
        old_h = h
    hit = np.abs(h) < 0.05
    dist = t
    sky = _hill_sky(d, sun)
    pos = ro[:, None] + dist * d
    u, v = _hill_uv(pos[0], pos[2])
    nor = (_hill_sample(T, u, v, [1, 2, 3]) * 2 - 1).T
    nz = _hill_noise(pos[0] * 0.025, pos[2] * 0.025)
    mat = _mix(np.array([0.0, 0.3, 0.0])[:, None], np.array([0.2, 0.3, 0.0])[:, None], nz)
    fn, w, nx, ny = 0.0, 0.7, pos[0] * 0.1, pos[2] * 0.1
    for _ in range(3):
        fn, w, nx, ny = fn + _hill_noise(nx, ny) * w, w * 0.6, 2 * nx, 2 * ny
    rcoc = np.maximum(dist * 0.3 * 0.04, (2.0 / height) * (1.0 + dist * 0.3))
    cw = np.concatenate([mat * 0.15, np.zeros_like(mat[:1])])
    dd = np.zeros_like(dist)
    live = np.ones_like(dist, bool)
    for _ in range(15):
        live = live & ~(cw[3] > 0.99)
        rx, ry, rz = _hill_de(T, pos[0] + d[0] * dd, pos[1] + d[1] * dd, pos[2] + d[2] * dd)
        rx = rx + 0.5 * rcoc
        take = live & (rx < rcoc)
        alpha = (1 - cw[1]) * np.clip((-rx + rcoc) / (2 * rcoc), 0, 1)
        tip = np.stack([np.full_like(rz, 0.35), np.full_like(rz, 0.35), np.minimum(rz ** 4 * 35, 0.35)])
        gra = _mix(mat, tip, ry ** 9.0 * 0.7) * ry
        cw = np.where(take, cw + np.concatenate([gra * alpha, alpha[None]]), cw)
        dd = np.where(live, dd + np.maximum(rx * 0.7, 0.1), dd)
    cw[:3] = np.where(cw[3] < 0.2, np.array([0.1, 0.15, 0.05])[:, None], cw[:3])
    mat = cw[:3] * (fn + 0.5)
    hl = ((sun[:, None] * nor).sum(0)) ** 2 * 4
    mat = mat * np.array([1.0, 0.75, 0.6])[:, None] * hl
    fog = np.clip(dist * dist * 0.0000012, 0, 1)
    col = np.where(hit, _mix(mat, sky, fog), sky)
    rgb = np.maximum(col, 0) ** 0.45 * 1.3
    lum = 0.2125 * rgb[0] + 0.7154 * rgb[1] + 0.0721 * rgb[2]
    vig = 0.4 + 0.5 * np.maximum(40 * xyx * xyy * (1 - xyx) * (1 - xyy), 0) ** 0.2
    out = _mix(0.5, _mix(lum, rgb, 1.3), 1.1) * vig
    out = np.concatenate([out, np.ones_like(out[:1])])
    return np.where(box, 0.0, out), hit & ~box, box


def render_hill_fullscreen(tex, cam):
    H, W = np.asarray(tex).shape[:2]
    j = np.arange(H, dtype=np.float64)[:, None] * np.ones((1, W))
    i = np.arange(W, dtype=np.float64)[None, :] * np.ones((H, 1))
    tx = (i + 0.5) / W * 2.0 - 1.0
    ty = (j + 0.5) / H * 2.0 - 1.0
    out, hit, box = hill(tex, tx.ravel(), ty.ravel(), cam)
    return (np.moveaxis(out.reshape(4, H, W), 0, -1)[::-1], hit.reshape(H, W)[::-1], box.reshape(H, W)[::-1])
