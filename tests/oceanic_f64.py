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
