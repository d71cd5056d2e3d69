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
